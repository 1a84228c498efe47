#!/usr/bin/env python3
"""Same-pool A/B of the per-stripe-pattern (masked bits) decode between
librsamd builds, packed and granule layouts.  One pool per
shape (contiguous, from the first library), the builds take turns on it.
  python tools/masked_ab.py LIB [LIB ...] [--reps N]
Legs per shape:
  packed      rs_decode_batch_masked_bits_dev, one bitmask per stripe;
  view_rep    granule batch through its packed view, each stripe's bitmask
              repeated per granule row (only when shard_len >= G);
  granule     rs_decode_granule_masked_bits_dev, one bitmask per stripe
              (libraries that export it).
Prints one JSON line per (shape, repetition): fraction of 8 TB/s of the
algorithmic bytes (k survivors read + absent shards written per stripe that
has an erasure)."""
import ctypes as C
import itertools
import json
import sys

import numpy as np

SHAPES = [("10p4_4MiB_x128", 10, 4, 4 << 20, 128, 32 << 10, "rand4"),
          ("4p2_4KiB_x1M", 4, 2, 4 << 10, 1 << 20, 64 << 10, "le2"),
          ("4p2_1MiB_x4096", 4, 2, 1 << 20, 4096, 64 << 10, "le2")]


def bind(path):
    lib = C.CDLL(path)
    P, Z = C.c_void_p, C.c_size_t
    lib.rs_codec_create.argtypes = [C.c_int, C.c_int, C.POINTER(P)]
    lib.rs_encode_batch_dev.argtypes = [P, P, Z, Z, Z, Z, P]
    lib.rs_decode_batch_masked_bits_dev.argtypes = [P, P, P, Z, Z, Z, Z, P, P]
    lib.rs_fill_synthetic_dev.argtypes = [P, C.c_int, Z, Z, Z, Z, C.c_uint64, C.c_uint64, P]
    lib.rs_dev_alloc.argtypes = [C.POINTER(P), Z, C.c_int, C.POINTER(C.c_int)]
    lib.rs_dev_free.argtypes = [P]
    lib.has_granule = hasattr(lib, "rs_decode_granule_masked_bits_dev")
    if lib.has_granule:
        lib.rs_decode_granule_masked_bits_dev.argtypes = [P, P, P, Z, Z, Z, P, P]
    return lib


def patterns(kind, k, m, B):
    T = k + m
    rng = np.random.default_rng(0)
    if kind == "rand4":
        pres = np.ones((B, T), dtype=bool)
        for t in range(B):
            pres[t, rng.choice(T, 4, replace=False)] = False
        return pres
    pats = np.array([[i not in mi for i in range(T)] for e in range(3) for mi in itertools.combinations(range(T), e)],
                    dtype=bool)
    return pats[rng.integers(0, len(pats), B)]


def main():
    args = sys.argv[1:]
    reps = 3
    if "--reps" in args:
        i = args.index("--reps")
        reps = int(args[i + 1])
        del args[i:i + 2]
    import torch
    libs = [bind(p) for p in args]
    names = [f"{i}:" + "/".join(p.split("/")[-2:]).replace(".so", "") for i, p in enumerate(args)]
    st = torch.cuda.current_stream()
    sp = C.c_void_p(st.cuda_stream)
    for name, k, m, S, B, G, kind in SHAPES:
        T = k + m
        nbytes = B * T * S
        pool, got = C.c_void_p(), C.c_int(0)
        assert libs[0].rs_dev_alloc(C.byref(pool), nbytes, 1, C.byref(got)) == 0
        pres = patterns(kind, k, m, B)
        bits = (pres.astype(np.uint32) << np.arange(T, dtype=np.uint32)).sum(axis=1, dtype=np.uint32)
        alg = (k * int((~pres).any(axis=1).sum()) + int((~pres).sum())) * S
        dbits = torch.from_numpy(bits.view(np.int32)).to("cuda:0")
        rep_bits = torch.from_numpy(np.repeat(bits, S // G).view(np.int32)).to("cuda:0") if S >= G else None
        hs = []
        for lib in libs:
            h = C.c_void_p()
            assert lib.rs_codec_create(k, m, C.byref(h)) == 0
            hs.append(h)
        rows = B * S // G

        def legs(j):
            lib, h = libs[j], hs[j]
            out = [("packed", lambda: lib.rs_decode_batch_masked_bits_dev(h, pool, C.c_void_p(dbits.data_ptr()), B, S,
                                                                          S, T * S, None, sp))]
            if rep_bits is not None:
                out.append(("view_rep", lambda: lib.rs_decode_batch_masked_bits_dev(
                    h, pool, C.c_void_p(rep_bits.data_ptr()), rows, G, G, T * G, None, sp)))
            if lib.has_granule:
                out.append(("granule", lambda: lib.rs_decode_granule_masked_bits_dev(
                    h, pool, C.c_void_p(dbits.data_ptr()), B, S, G, None, sp)))
            return out

        assert libs[0].rs_fill_synthetic_dev(pool, k, B, S, S, T * S, 0x5EED, 0, sp) == 0
        assert libs[0].rs_encode_batch_dev(hs[0], pool, B, S, S, T * S, sp) == 0
        for rep in range(reps):
            out = {"shape": name, "G": G, "rep": rep, "contiguous": bool(got.value)}
            for j in range(len(libs)):
                for leg, call in legs(j):
                    for _ in range(5):
                        assert call() == 0
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(10):
                        assert call() == 0
                    e1.record(st)
                    torch.cuda.synchronize()
                    out[f"{names[j]}:{leg}"] = round(alg / (e0.elapsed_time(e1) / 10 * 1e-3) / 8e12, 4)
            print(json.dumps(out), flush=True)
        torch.cuda.synchronize()
        del dbits, rep_bits
        libs[0].rs_dev_free(pool)


if __name__ == "__main__":
    main()
