#!/usr/bin/env python3
"""Median per-dispatch PMC value per kernel from rocprofv3 --pmc CSV output
directories: pmc_kernels.py DIR [DIR ...] (one counter per directory)."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    vals = collections.defaultdict(list)
    for p in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            vals[(r["Counter_Name"], r["Kernel_Name"][:80])].append(float(r["Counter_Value"]))
    for (c, k), v in sorted(vals.items()):
        if "rsamd" in k:
            print(f"{d.split('/')[-1]:28s} {c:11s} n={len(v):2d} median_kib={sorted(v)[len(v) // 2]:.0f} {k}")
