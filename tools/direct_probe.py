#!/usr/bin/env python3
"""Host API direct path (capi.cpp run_direct): per-call times of a 4+2 x 64 MiB
encodeParity on caller arrays of different backing -- torch pinned
(hipHostMalloc), numpy (pageable, registered per call), anonymous mmap with
MADV_HUGEPAGE and with MADV_NOHUGEPAGE -- over direct-kernel block counts
(RSAMD_DIRECT_BLOCKS, TUNING builds read it per call).
  python tools/direct_probe.py --lib build/ab/tuning/librsamd.so [--calls N]"""
import argparse
import json
import mmap
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--calls", type=int, default=6)
    ap.add_argument("--blocks", default="64,128,256,512,1024")
    a = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    from rsamd import _lib
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    import rsamd
    k, m, n = 4, 2, 64 << 20
    rng = np.random.default_rng(5)
    src = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] + [np.zeros(n, np.uint8) for _ in range(m)]
    maps = []

    def mm(advice):
        b = mmap.mmap(-1, n)
        b.madvise(advice)
        maps.append(b)
        return np.frombuffer(b, np.uint8)

    kinds = {
        "pinned": [torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(k + m)],
        "numpy": [x.copy() for x in src],
        "mmap_huge": [mm(mmap.MADV_HUGEPAGE) for _ in range(k + m)],
        "mmap_nohuge": [mm(mmap.MADV_NOHUGEPAGE) for _ in range(k + m)],
    }
    for sh in kinds.values():
        for x, y in zip(sh, src):
            x[:] = y
    rs = rsamd.ReedSolomon.create(k, m)
    ref = None
    for blocks in [int(b) for b in a.blocks.split(",")]:
        os.environ["RSAMD_DIRECT_BLOCKS"] = str(blocks)
        for name, sh in kinds.items():
            for _ in range(2):
                rs.encodeParity(sh, 0, n)
            ts = []
            for _ in range(a.calls):
                t0 = time.perf_counter()
                rs.encodeParity(sh, 0, n)
                ts.append((time.perf_counter() - t0) * 1e3)
            if ref is None:
                ref = [x.copy() for x in sh[k:]]
            ok = all(np.array_equal(x, y) for x, y in zip(sh[k:], ref))
            ts.sort()
            print(json.dumps({"blocks": blocks, "mem": name, "median_ms": round(ts[len(ts) // 2], 3),
                              "min_ms": round(ts[0], 3), "GiBps": round(k * n / (ts[len(ts) // 2] * 1e-3) / 2**30, 2),
                              "parity_equal": ok}), flush=True)


if __name__ == "__main__":
    main()
