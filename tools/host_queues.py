#!/usr/bin/env python3
"""Does the host pipeline's rate depend on how many HIP streams the process
created before it?  (HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues
round robin; if the pipeline's H2D and D2H streams land on one queue, their
copies serialize.)  Creates N torch streams (each used once), then times
encodeParity on pinned 4+2 x 64 MiB host shards.
  python tools/host_queues.py N [LIB]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "java-reed-solomon-distributed-file-system_amd"))


def main():
    n_extra = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    import torch
    if len(sys.argv) > 2:  # a variant librsamd.so
        from rsamd import _lib
        _lib.LIB_PATH = os.path.abspath(sys.argv[2])
    import rsamd
    streams = [torch.cuda.Stream() for _ in range(n_extra)]
    x = torch.zeros(1024, device="cuda")
    for s in streams:
        with torch.cuda.stream(s):
            x.add_(1)
    torch.cuda.synchronize()
    k, m, n = 4, 2, 64 << 20
    rs = rsamd.ReedSolomon.create(k, m)
    pin = [torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(k + m)]
    rng = np.random.default_rng(1)
    for a in pin[:k]:
        a[:] = rng.integers(0, 256, n, dtype=np.uint8)
    rs.encodeParity(pin, 0, n)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        rs.encodeParity(pin, 0, n)
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"extra_streams": n_extra, "lib": sys.argv[2] if len(sys.argv) > 2 else "in-tree", "GiBps": [round(k * n / t / 2**30, 2) for t in ts]}), flush=True)


if __name__ == "__main__":
    main()
