#!/usr/bin/env python3
"""Line-owner kernel A/B: the master's 4 M chunk groups
of 4+2 x 1000 B packed back to back, a random presence bitmask per group
(<= 2 erasures), decoded by two librsamd builds taking turns on ONE pool:
the product (a run's ragged first and last line written whole, the foreign
bytes loaded and written back) and RSAMD_GROUP_FOREIGN=0 (the ragged ends as
8-byte stores, partial lines to HBM).  Also the uniform {0,1} decode and the
encode.  Both builds' outputs are checked equal (verify after each decode).
Fractions of 8 TB/s of the algorithmic bytes.
  python tools/cg_foreign_ab.py LIB_A LIB_B [--reps N]"""
import argparse
import ctypes as C
import itertools
import json
import time

import numpy as np

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--groups", type=int, default=4 << 20)
    a = ap.parse_args()
    import torch
    libs = []
    for path in a.libs:
        lib = C.CDLL(path, mode=C.RTLD_LOCAL)
        h = C.c_void_p()
        assert lib.rs_codec_create(4, 2, C.byref(h)) == 0
        libs.append((path, lib, h))
    k, m, S, T, B = 4, 2, 1000, 6, a.groups
    buf = torch.empty(B * T * S, dtype=torch.uint8, device="cuda:0")
    base = C.c_void_p(buf.data_ptr())
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    sz = C.c_size_t
    lib0 = libs[0][1]
    lib0.rs_fill_synthetic_dev.argtypes = [C.c_void_p, C.c_int, sz, sz, sz, sz, C.c_uint64, C.c_uint64, C.c_void_p]
    assert lib0.rs_fill_synthetic_dev(base, k, B, S, S, T * S, 7, 0, st) == 0
    for _, lib, _h in libs:
        lib.rs_encode_batch_dev.argtypes = [C.c_void_p, C.c_void_p, sz, sz, sz, sz, C.c_void_p]
        lib.rs_decode_batch_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, sz, sz, sz, sz, C.c_void_p]
        lib.rs_decode_batch_masked_bits_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, sz, sz, sz, sz,
                                                        C.c_void_p, C.c_void_p]
        lib.rs_verify_batch_dev.argtypes = [C.c_void_p, C.c_void_p, sz, sz, sz, sz, C.c_void_p, C.c_void_p]
    assert lib0.rs_encode_batch_dev(libs[0][2], base, B, S, S, T * S, st) == 0
    pats = np.array([[i not in mi for i in range(T)] for e in range(3) for mi in itertools.combinations(range(T), e)],
                    dtype=bool)
    pres = pats[np.random.default_rng(0).integers(0, len(pats), B)]
    bits = (pres.astype(np.uint32) << np.arange(T, dtype=np.uint32)).sum(axis=1, dtype=np.uint32)
    dbits = torch.from_numpy(bits.view(np.int32)).to("cuda:0")
    alg_masked = (k * int((~pres).any(axis=1).sum()) + int((~pres).sum())) * S
    present01 = (C.c_uint8 * T)(0, 0, 1, 1, 1, 1)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")

    def timed(fn, iters=10):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            fn()
            torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters * 1e-3

    for r in range(a.reps):
        row = {"rep": r}
        for path, lib, h in libs:
            tag = "foreign0" if "foreign0" in path else "product"
            t = timed(lambda: lib.rs_encode_batch_dev(h, base, B, S, S, T * S, st))
            row[tag + "_encode"] = round(T * S * B / t / 1e9 / PEAK, 4)
            t = timed(lambda: lib.rs_decode_batch_dev(h, base, present01, B, S, S, T * S, st))
            row[tag + "_decode_0_1"] = round(T * S * B / t / 1e9 / PEAK, 4)
            t = timed(lambda: lib.rs_decode_batch_masked_bits_dev(h, base, C.c_void_p(dbits.data_ptr()), B, S, S,
                                                                  T * S, None, st))
            row[tag + "_masked_bits"] = round(alg_masked / t / 1e9 / PEAK, 4)
            # correctness: clobber every absent chunk, decode, verify
            v = buf.view(B, T, S)
            v[torch.from_numpy(~pres).to("cuda:0")] = 0x3C
            lib.rs_decode_batch_masked_bits_dev(h, base, C.c_void_p(dbits.data_ptr()), B, S, S, T * S, None, st)
            flag.zero_()
            lib.rs_verify_batch_dev(h, base, B, S, S, T * S, C.c_void_p(flag.data_ptr()), st)
            torch.cuda.synchronize()
            row[tag + "_verified"] = int(flag.item()) == 0
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
