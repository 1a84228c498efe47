#!/usr/bin/env python3
"""Concurrency stress of the host paths (the process-wide copy pool with its
polling threads, the mirrored pipeline's shared slot sets, the zero-copy
path, and with --pinned P a share P of the calls on the library's pinned
buffers: the in-place direct kernels, the pinned file decode's file tee): T
threads at once, each making random calls -- encodeParity / decodeMissing at
random sizes (4 KiB .. 24 MiB per shard) and offsets, and file encode / decode
at random sizes and blocks (4 KiB of sentinel past the decoded file) -- for a
fixed time, every result checked against the oracle.  Prints one JSON line
per thread and a summary; exits 1 on any mismatch.
  python tools/host_stress.py [--threads 8] [--seconds 60] [--pinned 0.3]"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def worker(tid, seconds, oracle, res, pinned_share=0.0):
    import numpy as np
    import rsamd
    from rsamd.device import HostBuffer
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    rng = np.random.default_rng(1000 + tid)
    calls = bad = npinned = 0
    t_end = time.time() + seconds
    while time.time() < t_end:
        pinned = rng.random() < pinned_share
        held = []

        def buf(size, fill=None):  # a pageable array, or one on rs_host_alloc memory
            if pinned:
                held.append(HostBuffer(size))
                a = held[-1].array
                if fill is not None:
                    a[:] = fill
                return a
            return np.zeros(size, np.uint8) if fill is None else np.full(size, fill, np.uint8)

        def rand(size):
            a = buf(size)
            a[:] = rng.integers(0, 256, size, dtype=np.uint8)
            return a

        k = int(rng.choice([4, 4, 10, 3, 6]))
        m = int(rng.choice([2, 2, 4, 1, 3]))
        rs = rsamd.ReedSolomon.create(k, m)
        oc = oracle.Codec(k, m)
        if rng.random() < 0.6:
            n = int(rng.choice([4 << 10, 64 << 10, 300 << 10, 1 << 20, 3 << 20, 24 << 20]))
            n += int(rng.integers(0, 4096))
            off = int(rng.integers(0, 64))
            cnt = n - off - int(rng.integers(0, 64))
            sh = [rand(n) for _ in range(k)] + [buf(n, 0) for _ in range(m)]
            ref = [a.copy() for a in sh]
            oc.encode_parity(ref, off, cnt)
            rs.encodeParity(sh, off, cnt)
            ok = all(np.array_equal(a, b) for a, b in zip(sh, ref))
            e = int(rng.integers(1, m + 1))
            miss = sorted(int(x) for x in rng.choice(k + m, e, replace=False))
            for j in miss:
                sh[j][off:off + cnt] = 0
            rs.decodeMissing(sh, [i not in miss for i in range(k + m)], off, cnt)
            ok = ok and all(np.array_equal(a, b) for a, b in zip(sh, ref))
        else:
            block = int(rng.choice([1000, 1000, 4096, 520, 8]))
            n = int(rng.choice([90_999, 1 << 20, 5 << 20, 20 << 20])) + int(rng.integers(0, 5000))
            data = rand(n)
            _, S = file_layout(rs, n, block)
            sh = [buf(S, 0xEE) for _ in range(k + m)]
            file_encode_into(rs, data, sh, block)
            ref = oc.file_encode(data.tobytes(), block)
            ok = all(np.array_equal(a, b) for a, b in zip(sh, ref))
            e = int(rng.integers(1, m + 1))
            miss = sorted(int(x) for x in rng.choice(k + m, e, replace=False))
            for j in miss:
                sh[j][:] = 0
            out = buf(n + 4096, 0x33)
            file_decode_into(rs, sh, [i not in miss for i in range(k + m)], S, out[:n], block)
            ok = ok and np.array_equal(out[:n], data) and bool((out[n:] == 0x33).all()) and \
                all(np.array_equal(a, b) for a, b in zip(sh, ref))
        calls += 1
        npinned += int(pinned)
        bad += 0 if ok else 1
        for h in held:
            h.free()
    res[tid] = {"thread": tid, "calls": calls, "pinned_calls": npinned, "bad": bad}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=60)
    ap.add_argument("--pinned", type=float, default=0.0, help="share of calls on rs_host_alloc buffers")
    a = ap.parse_args()
    from rsamd import _lib
    if os.environ.get("RSAMD_TEST_LIB"):  # e.g. the bounds-checking build
        _lib.LIB_PATH = os.path.abspath(os.environ["RSAMD_TEST_LIB"])
    import torch
    torch.cuda.init()
    from oracle import c_ref
    res = {}
    ts = [threading.Thread(target=worker, args=(t, a.seconds, c_ref, res, a.pinned)) for t in range(a.threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for t in sorted(res):
        print(json.dumps(res[t]), flush=True)
    total = sum(r["calls"] for r in res.values())
    bad = sum(r["bad"] for r in res.values())
    oob = None
    lib = _lib.load()
    if hasattr(lib, "rs_bounds_report"):  # the bounds build: kernel accesses outside their declared buffers
        import ctypes as C
        n, addr, ln, where = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint32()
        lib.rs_bounds_report(C.byref(n), C.byref(addr), C.byref(ln), C.byref(where))
        oob = n.value
    print(json.dumps({"threads": a.threads, "seconds": a.seconds, "calls": total, "bad": bad,
                      "all_threads_finished": len(res) == a.threads, "bounds_violations": oob}), flush=True)
    return 1 if bad or oob or len(res) != a.threads else 0


if __name__ == "__main__":
    sys.exit(main())
