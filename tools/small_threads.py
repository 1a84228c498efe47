#!/usr/bin/env python3
"""Concurrent small calls: T threads, each with its own arrays, each making
`reps` 4+2 x 1000-B decodeMissing {0} calls from C (tests/jni_mock's timing
loop; ctypes drops the GIL for the call), against the wall clock: aggregate
calls per second and each thread's median per call, for T = 1, 2, 4, 8, 16.
Every thread's output is checked against the oracle afterwards.  Prints one
JSON line.  (A chunkserver serving many clients makes such calls at once;
each calling thread has its own stream and staging buffer, host.hpp
ThreadCtx.)"""
import ctypes as C
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import numpy as np
    import torch
    import rsamd
    from rsamd import _lib, parallel
    import bench
    from oracle import c_ref
    torch.cuda.init()
    mj = bench._mockjni()
    k, m, S, reps = 4, 2, 1000, 2000
    T = k + m
    rs = rsamd.ReedSolomon.create(k, m)
    oc = c_ref.Codec(k, m)
    out, extra = {}, {}
    with bench.gpu_numa_bound(torch, parallel, extra):
        for nt in (1, 2, 4, 8, 16):
            jobs = []
            for t in range(nt):
                rng = np.random.default_rng(100 + t)
                want = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + \
                       [np.zeros(S, np.uint8) for _ in range(m)]
                oc.encode_parity(want, 0, S)
                sh = [a.copy() for a in want]
                sh[0][:] = 0x3C
                ptrs = (_lib.u8p * T)(*[a.ctypes.data_as(_lib.u8p) for a in sh])
                lens = (C.c_int64 * T)(*[S] * T)
                pres = np.array([0] + [1] * (T - 1), np.uint8)
                jobs.append({"want": want, "sh": sh, "ptrs": ptrs, "lens": lens, "pres": pres, "us": None})

            bar = threading.Barrier(nt)

            def run(j):
                # warm-up: the thread's first call creates its context (stream, staging buffer)
                mj.mock_time_capi(1, rs.handle, j["ptrs"], T, j["lens"], j["pres"].ctypes.data_as(_lib.u8p), S, 50)
                bar.wait()
                j["t0"] = time.perf_counter()
                j["us"] = mj.mock_time_capi(1, rs.handle, j["ptrs"], T, j["lens"],
                                            j["pres"].ctypes.data_as(_lib.u8p), S, reps)
                j["t1"] = time.perf_counter()

            ths = [threading.Thread(target=run, args=(j,)) for j in jobs]
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            wall = max(j["t1"] for j in jobs) - min(j["t0"] for j in jobs)
            ok = all(j["us"] > 0 and all(np.array_equal(a, b) for a, b in zip(j["sh"], j["want"])) for j in jobs)
            out[f"t{nt}"] = {"calls_per_s": round(nt * (reps + 20) / wall), "median_us": [round(j["us"], 2) for j in jobs],
                             "bit_exact": bool(ok)}
    out["note"] = (f"{k}+{m} x {S}-B decodeMissing {{0}}, {reps} timed calls (+20 warm-up) per thread from C, "
                   f"threads released together after a warm-up; calls_per_s = all threads' timed calls / wall time")
    out["numa"] = extra.get("host_legs_numa")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
