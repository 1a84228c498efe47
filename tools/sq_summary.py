#!/usr/bin/env python3
"""Summarise SQ/GRBM counter passes (tools/gpu_sq.sh) per workload.

For each WORKLOAD:DIR argument, reads the workload's JSON line from DIR.log
(kernel name, algorithmic bytes) and the counter_collection CSVs under DIR,
keeps the dispatches of that kernel and takes the median per counter.  Derived
(MI355X_MICROARCH.md: SQ_*_CYCLES / WAIT / ACTIVE count quad-cycles,
WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES; kernel cycles ~
GRBM_GUI_ACTIVE / 8 XCDs; a wave64 VALU instruction occupies a SIMD-32 for 2
cycles):
  valu_per_wave        SQ_INSTS_VALU / SQ_WAVES
  valu_pipe_util       SQ_INSTS_VALU * 2 / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
  active/wait fractions of SQ_WAVE_CYCLES
  clock_GHz            GRBM_GUI_ACTIVE / 8 / kernel duration (when DIR has a kernel trace; else null)
Usage: sq_summary.py OUT_JSON WORKLOAD:DIR [WORKLOAD:DIR ...]
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def meta_of(d):
    try:
        for line in open(d + ".log"):
            if line.startswith("{"):
                return json.loads(line)
    except OSError:
        pass
    return {}


def counters(d, kernel_sub):
    vals = collections.defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if kernel_sub and kernel_sub not in row.get("Kernel_Name", ""):
                    continue
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {c: statistics.median(v) for c, v in vals.items()}, {c: len(v) for c, v in vals.items()}


def main():
    out, args = sys.argv[1], sys.argv[2:]
    res = collections.defaultdict(dict)
    for a in args:
        w, d = a.split(":", 1)
        meta = meta_of(d)
        kern = meta.get("kernel", "")
        c, n = counters(d, kern)
        res[w].setdefault("kernel", kern)
        res[w].setdefault("alg_bytes_per_launch", meta.get("alg_bytes_per_launch"))
        res[w].setdefault("counters", {}).update(c)
        res[w].setdefault("dispatches", {}).update(n)
    for w, r in res.items():
        c = r["counters"]
        der = {}
        if c.get("SQ_WAVES"):
            der["valu_per_wave"] = round(c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"], 1)
            if "SQ_INSTS_SALU" in c:
                der["salu_per_wave"] = round(c["SQ_INSTS_SALU"] / c["SQ_WAVES"], 1)
            if "SQ_INSTS_SMEM" in c:
                der["smem_per_wave"] = round(c["SQ_INSTS_SMEM"] / c["SQ_WAVES"], 1)
        if c.get("GRBM_GUI_ACTIVE") and "SQ_INSTS_VALU" in c:
            cyc = c["GRBM_GUI_ACTIVE"] / 8
            der["kernel_cycles"] = round(cyc)
            der["valu_pipe_util"] = round(c["SQ_INSTS_VALU"] * 2 / (1024 * cyc), 4)
            if r.get("alg_bytes_per_launch"):
                der["alg_bytes_per_cycle"] = round(r["alg_bytes_per_launch"] / cyc, 1)
        if c.get("SQ_WAVE_CYCLES"):
            wc = c["SQ_WAVE_CYCLES"]
            for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if k in c:
                    der[k.lower() + "_frac"] = round(c[k] / wc, 4)
            if c.get("SQ_WAVES"):
                der["wave_cycles_per_wave"] = round(wc / c["SQ_WAVES"], 1)
        if c.get("TCC_BUSY") and c.get("GRBM_GUI_ACTIVE"):
            # summed over the TCC channels (16 per XCD, 128 in all) and the 8 XCDs' GUI_ACTIVE
            cyc = c["GRBM_GUI_ACTIVE"] / 8
            for k in ("TCC_EA0_RDREQ_DRAM_CREDIT_STALL", "TCC_EA0_WRREQ_DRAM_CREDIT_STALL", "TCC_EA0_WRREQ_STALL",
                      "TCC_BUSY"):
                if k in c:
                    der[k.lower() + "_per_channel_cycle"] = round(c[k] / (128 * cyc), 4)
        if c.get("SQ_BUSY_CYCLES") and c.get("GRBM_GUI_ACTIVE"):
            der["sq_busy_frac"] = round(c["SQ_BUSY_CYCLES"] / c["GRBM_GUI_ACTIVE"], 4)
        r["derived"] = der
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for w, r in res.items():
        print(w, r["kernel"], json.dumps(r["derived"]))


if __name__ == "__main__":
    main()
