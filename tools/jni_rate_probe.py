#!/usr/bin/env python3
"""encodeParity through the JNI shim's marshalling (jni/rs_jni_core.c over
the mock JNI of tests/jni_mock, critical-region pinning in 32 MiB slices)
against the same call straight into librsamd, 4+2 pageable shards of 16 and
64 MiB, bound to the GPU's NUMA node like the bench's host legs.
  python tools/jni_rate_probe.py"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import numpy as np
    import torch
    import rsamd
    from rsamd import parallel
    import bench
    from test_jni_core import Jvm, build_mock
    torch.cuda.init()
    lib = build_mock()
    jvm = Jvm(lib)
    rs = rsamd.ReedSolomon.create(4, 2)
    extra = {}
    with bench.gpu_numa_bound(torch, parallel, extra):
        for n in (16 << 20, 64 << 20):
            rng = np.random.default_rng(n)
            sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(4)] + [np.zeros(n, np.uint8) for _ in range(2)]
            arrs = [jvm.bytes(a) for a in sh]
            outer = jvm.objects(arrs)
            h = C.c_void_p(rs.handle) if not isinstance(rs.handle, C.c_void_p) else rs.handle
            res = {}
            for name, fn in (("shim", lambda: lib.mock_encode_parity(1, h, outer, 0, n)),
                             ("direct", lambda: rs.encodeParity(sh, 0, n))):
                for _ in range(3):
                    fn()
                reps = 10
                t0 = time.perf_counter()
                for _ in range(reps):
                    fn()
                res[name] = round(4 * n / ((time.perf_counter() - t0) / reps) / 2**30, 2)
            assert jvm.exception() == ("", "")
            print(json.dumps({"shard_MiB": n >> 20, **res}), flush=True)


if __name__ == "__main__":
    main()
