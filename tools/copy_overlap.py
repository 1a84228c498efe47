#!/usr/bin/env python3
"""Summarise a rocprofv3 memory_copy_trace.csv: per direction busy time and
how much of the H2D and D2H intervals overlap."""
import csv
import glob
import sys


def merge(iv):
    iv.sort()
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def inter(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        tot += max(0, e - s)
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


for path in glob.glob(sys.argv[1] + "/**/*memory_copy_trace.csv", recursive=True):
    rows = list(csv.DictReader(open(path)))
    d = {}
    for r in rows:
        d.setdefault(r["Direction"], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    m = {k: merge(v) for k, v in d.items()}
    for k, v in m.items():
        print(k, "copies", len(d[k]), "busy_ms", round(sum(e - s for s, e in v) / 1e6, 2),
              "bytes_per_copy", rows[0].get("Size"))
    keys = list(m)
    if len(keys) >= 2:
        print("overlap_ms", round(inter(m[keys[0]], m[keys[1]]) / 1e6, 2))
    t0 = min(s for v in d.values() for s, _ in v)
    for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
        print(r["Direction"], (int(r["Start_Timestamp"]) - t0) // 1000, (int(r["End_Timestamp"]) - t0) // 1000,
              r.get("Size"), r.get("Queue_Id", r.get("Stream_Id", "")))
