#!/usr/bin/env python3
"""Per-call times of the host-buffer encodeParity (4+2 x 64 MiB), pageable
and pinned caller arrays alternated call by call, to see whether the pageable
leg's lower mean in some bench runs is every call (the per-call page
registration) or a few slow calls.
  python tools/host_calls.py [--calls N]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    import rsamd
    k, m, n = 4, 2, 64 << 20
    rng = np.random.default_rng(5)
    page = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] + [np.zeros(n, np.uint8) for _ in range(m)]
    pin = [torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(k + m)]
    for x, y in zip(pin, page):
        x[:] = y
    rs = rsamd.ReedSolomon.create(k, m)
    for _ in range(3):
        rs.encodeParity(page, 0, n)
        rs.encodeParity(pin, 0, n)
    res = {"pageable": [], "pinned": []}
    for _ in range(a.calls):
        for name, sh in (("pageable", page), ("pinned", pin)):
            t0 = time.perf_counter()
            rs.encodeParity(sh, 0, n)
            res[name].append(round((time.perf_counter() - t0) * 1e3, 3))
    for name, v in res.items():
        s = sorted(v)
        print(json.dumps({"leg": name, "mean_ms": round(sum(v) / len(v), 3), "median_ms": s[len(s) // 2],
                          "min_ms": s[0], "max_ms": s[-1], "GiBps_mean": round(k * n / (sum(v) / len(v) * 1e-3) / 2**30, 2),
                          "calls_ms": v}), flush=True)


if __name__ == "__main__":
    main()
