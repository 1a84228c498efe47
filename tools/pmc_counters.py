#!/usr/bin/env python3
"""Median per-dispatch value of every counter in one rocprofv3 --pmc output
directory, for the dispatches whose kernel name contains KERNEL_SUBSTRING.
  python tools/pmc_counters.py DIR KERNEL_SUBSTRING  -> one JSON line
"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d, sub = sys.argv[1], sys.argv[2]
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if sub in row.get("Kernel_Name", ""):
                    vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    if not vals:
        sys.exit(f"no counter rows for {sub!r} under {d}")
    print(json.dumps({c: {"median": statistics.median(v), "dispatches": len(v)} for c, v in sorted(vals.items())}))


if __name__ == "__main__":
    main()
