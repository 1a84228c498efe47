#!/usr/bin/env python3
"""Host API per-call times by shard size, pageable and pinned caller arrays,
with the direct path from every size (RSAMD_DIRECT_MIN=0) or only where the
pipeline would run (RSAMD_DIRECT_MIN=huge): where should a pageable call be
page-locked and coded in place instead of copied through the zero-copy
staging buffer?  TUNING builds read the knob per call.
  python tools/direct_small_probe.py --lib build/ab/tuning/librsamd.so"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--sizes", default="4096,65536,262144,1048576,4194304,16777216")
    a = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    from rsamd import _lib
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    import rsamd
    k, m = 4, 2
    rs = rsamd.ReedSolomon.create(k, m)
    for S in [int(x) for x in a.sizes.split(",")]:
        rng = np.random.default_rng(S)
        page = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        pin = [torch.empty(S, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(k + m)]
        for x, y in zip(pin, page):
            x[:] = y
        reps = max(10, min(300, (64 << 20) // S))
        for mode, dmin in (("staged", str(1 << 40)), ("direct", "0")):
            os.environ["RSAMD_DIRECT_MIN"] = dmin
            row = {"S": S, "mode": mode}
            for name, sh in (("pageable", page), ("pinned", pin)):
                for _ in range(3):
                    rs.encodeParity(sh, 0, S)
                ts = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    rs.encodeParity(sh, 0, S)
                    ts.append((time.perf_counter() - t0) * 1e6)
                ts.sort()
                row[f"{name}_us"] = round(ts[len(ts) // 2], 1)
                row[f"{name}_GiBps"] = round(k * S / (ts[len(ts) // 2] * 1e-6) / 2**30, 2)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
