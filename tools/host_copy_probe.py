#!/usr/bin/env python3
"""encodeParity on 4+2 x 64 MiB pinned host shards, a few calls (for
rocprofv3 --memory-copy-trace --kernel-trace: do the two streams' copies
overlap?)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import numpy as np
    import torch
    import rsamd
    n = 64 << 20
    pinned = os.environ.get("PROBE_PAGEABLE") is None
    sh = [torch.empty(n, dtype=torch.uint8, pin_memory=pinned).numpy() for _ in range(6)]
    for a in sh[:4]:
        a[:] = np.random.default_rng(1).integers(0, 256, n, dtype=np.uint8)
    rs = rsamd.ReedSolomon.create(4, 2)
    rs.encodeParity(sh, 0, n)
    t0 = time.perf_counter()
    for _ in range(3):
        rs.encodeParity(sh, 0, n)
    print("GiB/s", 4 * n * 3 / (time.perf_counter() - t0) / 2**30, "pinned" if pinned else "pageable")


if __name__ == "__main__":
    main()
