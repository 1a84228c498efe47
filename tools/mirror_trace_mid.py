#!/usr/bin/env python3
"""Per-chunk timelines (RSAMD_TRACE, TUNING build) of mid-size pageable
4+2 encodeParity calls -- 1, 2 and 4 MiB per shard through the mirrored
pipeline -- bound to the GPU's NUMA node; 20 warm calls each, the last 5
traced.  Summarise with tools/mirror_trace.py.
  python tools/mirror_trace_mid.py OUT.jsonl"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import numpy as np
    import torch
    from rsamd import _lib
    _lib.LIB_PATH = os.path.join(ROOT, "build", "ab", "tuning", "librsamd.so")
    import rsamd
    from rsamd import parallel
    import bench
    torch.cuda.init()
    out = os.path.abspath(sys.argv[1])
    rs = rsamd.ReedSolomon.create(4, 2)
    with bench.gpu_numa_bound(torch, parallel, {}):
        for S in (1 << 20, 2 << 20, 4 << 20):
            rng = np.random.default_rng(S)
            sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(4)] + [np.zeros(S, np.uint8) for _ in range(2)]
            for _ in range(20):
                rs.encodeParity(sh, 0, S)
            os.environ["RSAMD_TRACE"] = out
            for _ in range(5):
                rs.encodeParity(sh, 0, S)
            os.environ.pop("RSAMD_TRACE")


if __name__ == "__main__":
    main()
