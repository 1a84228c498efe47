#!/usr/bin/env python3
"""Per-call breakdown of small host calls from a rocprofv3 trace of
`small_latency lib200` (--kernel-trace --hip-runtime-trace --output-format csv):
for each library call, the host time before the launch (checks, plan lookup,
copy-in), the launch call, launch -> kernel start, the kernel, and kernel end
-> the call's next runtime call (the spin's exit and copy-out are host work
after the kernel).  Prints medians per call kind.
  python tools/small_breakdown.py gpurun_out/r6d/prof/lib200"""
import csv
import statistics as st
import sys

pre = sys.argv[1]
api = list(csv.DictReader(open(pre + "_hip_api_trace.csv")))
ker = {int(k["Correlation_Id"]): k for k in csv.DictReader(open(pre + "_kernel_trace.csv"))}
launches = [a for a in api if a["Function"] == "hipLaunchKernel" and int(a["Correlation_Id"]) in ker]
# consecutive launches: the gap to the next call's first runtime call bounds the
# host time after the kernel (spin exit + copy-out + the next call's prologue)
rows = []
for i, a in enumerate(launches[:-1]):
    k = ker[int(a["Correlation_Id"])]
    name = k["Kernel_Name"].split("<")[0].split("::")[-1]
    ls, le = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
    ks, ke = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
    nxt = int(launches[i + 1]["Start_Timestamp"])
    rows.append((name, k["Grid_Size_X"], (le - ls) / 1e3, (ks - le) / 1e3, (ke - ks) / 1e3, (nxt - ke) / 1e3,
                 (nxt - ls) / 1e3))
groups = {}
for r in rows:
    groups.setdefault((r[0], r[1]), []).append(r)
print("kernel grid calls | launch call | launch->start | kernel | end->next launch | launch->next launch (us, medians)")
for key, rs in groups.items():
    med = [st.median(x[i] for x in rs) for i in range(2, 7)]
    print(key[0], key[1], len(rs), "|", " | ".join(f"{m:.2f}" for m in med))
