#!/usr/bin/env python3
"""The host-inclusive encodeParity path under a trace: 4+2 x 64 MiB host
shards per call (pinned, then pageable), N calls each, wall time per call
printed.  Run under rocprofv3 --kernel-trace --memory-copy-trace to see the
chunk pipeline (host.cpp run_chunks): the gaps between H2D copies, kernels
and D2H copies.
  python tools/host_trace.py [--calls N] [--mib M]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "java-reed-solomon-distributed-file-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=6)
    ap.add_argument("--mib", type=int, default=64)
    a = ap.parse_args()
    import torch
    import rsamd
    k, m, n = 4, 2, a.mib << 20
    rs = rsamd.ReedSolomon.create(k, m)
    rng = np.random.default_rng(5)
    pin = [torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(k + m)]
    for x in pin[:k]:
        x[:] = rng.integers(0, 256, n, dtype=np.uint8)
    page = [x.copy() for x in pin]
    for name, sh in (("pinned", pin), ("pageable", page)):
        ts = []
        for _ in range(a.calls):
            t0 = time.perf_counter()
            rs.encodeParity(sh, 0, n)
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"buffers": name, "ms": [round(t * 1e3, 3) for t in ts],
                          "GiBps": [round(k * n / t / 2**30, 2) for t in ts]}), flush=True)


if __name__ == "__main__":
    main()
