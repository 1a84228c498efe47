#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs into HBM bytes per kernel launch.

Reads the counter_collection CSVs of separate FETCH_SIZE and WRITE_SIZE passes
(gfx950 cannot fit both in one TCC pass) and applies the corrections of
/opt/skills/guides/MI355X_MICROARCH.md section "HBM":
  * FETCH_SIZE and WRITE_SIZE are in KiB;
  * on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide (16 B per
    lane) coalesced streaming read, so it is doubled;
  * WRITE_SIZE is exact for 16-B-per-lane streaming stores.
Writes/updates profiles/pmc_traffic.json:
  {"<key>": {"kernel": ..., "fetch_kib_raw": ..., "write_kib_raw": ...,
             "hbm_bytes_per_launch": ..., "alg_bytes_per_launch": ..., "ratio": ...}}

Usage: pmc_summary.py KEY KERNEL_SUBSTRING ALG_BYTES FETCH_DIR WRITE_DIR [OUT_JSON]
"""
import csv
import glob
import json
import os
import statistics
import sys


def counter_values(d, counter, kernel_sub):
    vals = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                if kernel_sub not in row.get("Kernel_Name", ""):
                    continue
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    key, kernel_sub, alg = sys.argv[1], sys.argv[2], int(sys.argv[3])
    fdir, wdir = sys.argv[4], sys.argv[5]
    out = sys.argv[6] if len(sys.argv) > 6 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_traffic.json")
    fetch = counter_values(fdir, "FETCH_SIZE", kernel_sub)
    write = counter_values(wdir, "WRITE_SIZE", kernel_sub)
    if not fetch or not write:
        sys.exit(f"no counter rows for {kernel_sub!r}: fetch={len(fetch)} write={len(write)}")
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    hbm = int(round((2 * f_kib + w_kib) * 1024))
    rec = {"kernel": kernel_sub, "launches": [len(fetch), len(write)], "fetch_kib_raw": f_kib, "write_kib_raw": w_kib,
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 wide-read FETCH_SIZE is half)",
           "hbm_bytes_per_launch": hbm, "alg_bytes_per_launch": alg, "ratio": round(hbm / alg, 4)}
    data = {}
    if os.path.exists(out):
        data = json.load(open(out))
    data[key] = rec
    with open(out, "w") as f:
        json.dump(data, f, indent=1)
    print(key, json.dumps(rec))


if __name__ == "__main__":
    main()
