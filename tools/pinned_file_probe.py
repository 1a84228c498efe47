#!/usr/bin/env python3
"""The pinned file encode's two sides (capi.cpp file_encode_direct): a 256 MiB
file and its 4+2 shards in rs_host_alloc buffers, encoded N times; prints the
mean call time.  Under `rocprofv3 --kernel-trace --stats` (gpu_run.sh kprobe)
the kernel's own mean duration says whether the kernel or the host split
bounds the call.
  python tools/pinned_file_probe.py [--calls 10]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--block", type=int, default=1000)
    a = ap.parse_args()
    import numpy as np
    from rsamd import _lib
    if os.environ.get("RSAMD_TEST_LIB"):
        _lib.LIB_PATH = os.path.abspath(os.environ["RSAMD_TEST_LIB"])
    import rsamd
    from rsamd.device import HostBuffer
    from rsamd.layout import file_encode_into, file_layout
    k, m, n = 4, 2, 256 << 20
    rs = rsamd.ReedSolomon.create(k, m)
    f = HostBuffer(n)
    f.array[:] = np.random.default_rng(1).integers(0, 256, n, dtype=np.uint8)
    _, S = file_layout(rs, n, a.block)
    sh = [HostBuffer(S) for _ in range(k + m)]
    views = [b.array for b in sh]
    for _ in range(3):
        file_encode_into(rs, f.array, views, a.block)
    t0 = time.perf_counter()
    for _ in range(a.calls):
        file_encode_into(rs, f.array, views, a.block)
    t = (time.perf_counter() - t0) / a.calls
    print(json.dumps({"env": {x: os.environ[x] for x in os.environ if x.startswith("RSAMD_")}, "file_MiB": n >> 20, "block": a.block, "calls": a.calls, "ms_per_call": round(t * 1e3, 3),
                      "GiBps": round(n / t / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
