#!/usr/bin/env python3
"""hipHostRegister probe: cost of registering pageable host buffers, and the
host-API encode rate when the caller's pageable shards are registered around
each call (the library then sees page-locked memory and DMAs directly)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import numpy as np
    import torch
    torch.cuda.init()
    import rsamd
    hip = ctypes.CDLL("libamdhip64.so")
    for mb in (4, 64, 256):
        n = mb << 20
        a = np.ones(n + 4096, np.uint8)
        res = []
        for off in (0, 123):
            t0 = time.perf_counter()
            rc = hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data + off), ctypes.c_size_t(n), ctypes.c_uint(0))
            t1 = time.perf_counter()
            rc2 = hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data + off))
            res.append((off, rc, rc2, round((t1 - t0) * 1e3, 3)))
        print(mb, "MiB (offset, rc, rc_unreg, register ms):", res, flush=True)
    # overlapping ranges in one allocation
    big = np.ones(8 << 20, np.uint8)
    r1 = hip.hipHostRegister(ctypes.c_void_p(big.ctypes.data), ctypes.c_size_t(4 << 20), 0)
    r2 = hip.hipHostRegister(ctypes.c_void_p(big.ctypes.data + (2 << 20)), ctypes.c_size_t(4 << 20), 0)
    print("overlap register rcs", r1, r2, flush=True)
    hip.hipHostUnregister(ctypes.c_void_p(big.ctypes.data))
    if r2 == 0:
        hip.hipHostUnregister(ctypes.c_void_p(big.ctypes.data + (2 << 20)))

    k, m, n = 4, 2, 64 << 20
    rng = np.random.default_rng(1)
    sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] + [np.zeros(n, np.uint8) for _ in range(m)]
    rs = rsamd.ReedSolomon.create(k, m)

    def plain():
        rs.encodeParity(sh, 0, n)

    def registered():
        for a in sh:
            assert hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(n), 0) == 0
        rs.encodeParity(sh, 0, n)
        for a in sh:
            hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data))

    for name, fn in (("pageable", plain), ("registered per call", registered), ("pageable", plain),
                     ("registered per call", registered)):
        fn()
        t0 = time.perf_counter()
        for _ in range(4):
            fn()
        print(name, "GiB/s", round(4 * k * n / (time.perf_counter() - t0) / 2**30, 2), flush=True)


if __name__ == "__main__":
    main()
