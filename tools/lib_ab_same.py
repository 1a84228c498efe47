#!/usr/bin/env python3
"""A/B of librsamd.so builds in ONE process on ONE pool per shape, so the
allocation's placement (bimodal per allocation) is common to
every build: each library is loaded with its own handle (ctypes, RTLD_LOCAL),
the pool comes from the first one's rs_dev_alloc (contiguous), and the
builds take turns on it.  Prints one JSON line per repetition with the
fraction of 8 TB/s per (shape, build).
  python tools/lib_ab_same.py LIB [LIB ...] [--reps N] [--set single]
Shapes: 4+2 x 1 MiB x 4096 encode (the headline) and decode {0}, 10+4 x 4 MiB x 128 encode
and decode {0,1,2,3} and verify, 10+4 x 4 MiB x 1024 encode.  --set single: decodes
of one and two shards, packed and in the granule layout's view (4+2: 64 KiB
granules, 10+4: 32 KiB), with the encodes for reference."""
import ctypes as C
import json
import sys

SHAPES = [("4p2_1MiB_x4096_enc", 4, 2, 1 << 20, 4096, None),
          ("4p2_1MiB_x4096_dec0", 4, 2, 1 << 20, 4096, (0,)),
          ("10p4_4MiB_x128_enc", 10, 4, 4 << 20, 128, None),
          ("10p4_4MiB_x128_dec0123", 10, 4, 4 << 20, 128, (0, 1, 2, 3)),
          ("10p4_4MiB_x128_verify", 10, 4, 4 << 20, 128, "verify"),
          ("10p4_4MiB_x1024_enc", 10, 4, 4 << 20, 1024, None)]
# (name, k, m, S, B, miss, granule)
SINGLE = [("4p2g_enc", 4, 2, 1 << 20, 4096, None, 64 << 10),
          ("4p2g_dec0", 4, 2, 1 << 20, 4096, (0,), 64 << 10),
          ("10p4g_enc", 10, 4, 4 << 20, 128, None, 32 << 10),
          ("10p4g_dec0", 10, 4, 4 << 20, 128, (0,), 32 << 10),
          ("10p4g_dec01", 10, 4, 4 << 20, 128, (0, 1), 32 << 10),
          ("10p4g_dec012", 10, 4, 4 << 20, 128, (0, 1, 2), 32 << 10),
          ("10p4_dec0", 10, 4, 4 << 20, 128, (0,), 0),
          ("10p4_dec01", 10, 4, 4 << 20, 128, (0, 1), 0)]
# --set occ: the shapes of an occupancy sweep (granule and packed, encode and decodes)
OCC = [("4p2g_enc", 4, 2, 1 << 20, 4096, None, 64 << 10),
       ("4p2g_dec0", 4, 2, 1 << 20, 4096, (0,), 64 << 10),
       ("4p2g_dec01", 4, 2, 1 << 20, 4096, (0, 1), 64 << 10),
       ("4p2g_dec05", 4, 2, 1 << 20, 4096, (0, 5), 64 << 10),
       ("4p2_enc", 4, 2, 1 << 20, 4096, None, 0),
       ("4p2g4k_enc", 4, 2, 4096, 1 << 20, None, 64 << 10),
       ("10p4g_enc", 10, 4, 4 << 20, 128, None, 32 << 10),
       ("10p4g_dec0123", 10, 4, 4 << 20, 128, (0, 1, 2, 3), 32 << 10),
       ("10p4g_dec0", 10, 4, 4 << 20, 128, (0,), 32 << 10),
       ("10p4_enc", 10, 4, 4 << 20, 128, None, 0),
       ("10p4_dec0123", 10, 4, 4 << 20, 128, (0, 1, 2, 3), 0)]


def bind(path):
    lib = C.CDLL(path)
    P = C.c_void_p
    lib.rs_codec_create.argtypes = [C.c_int, C.c_int, C.POINTER(P)]
    lib.rs_encode_batch_dev.argtypes = [P, P, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, P]
    lib.rs_decode_batch_dev.argtypes = [P, P, C.c_char_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, P]
    lib.rs_fill_synthetic_dev.argtypes = [P, C.c_int, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_uint64,
                                          C.c_uint64, P]
    lib.rs_dev_alloc.argtypes = [C.POINTER(P), C.c_size_t, C.c_int, C.POINTER(C.c_int)]
    lib.rs_dev_free.argtypes = [P]
    lib.rs_verify_batch_dev.argtypes = [P, P, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, P, P]
    return lib


def main():
    args = sys.argv[1:]
    reps = 3
    if "--reps" in args:
        i = args.index("--reps")
        reps = int(args[i + 1])
        del args[i:i + 2]
    shapes = [sh + (0,) for sh in SHAPES]
    if "--set" in args:
        i = args.index("--set")
        if args[i + 1] == "single":
            shapes = SINGLE
        elif args[i + 1] == "occ":
            shapes = OCC
        del args[i:i + 2]
    import torch
    libs = [bind(p) for p in args]
    st = torch.cuda.current_stream()
    sp = C.c_void_p(st.cuda_stream)
    for name, k, m, S, B, miss, G in shapes:
        if G:  # the granule layout through its packed view: B*S/G stripes of G-byte shards
            S, B = G, B * S // G
        stride = S
        nbytes = B * (k + m) * stride
        pool, got = C.c_void_p(), C.c_int(0)
        assert libs[0].rs_dev_alloc(C.byref(pool), nbytes, 1, C.byref(got)) == 0
        assert libs[0].rs_fill_synthetic_dev(pool, k, B, S, stride, stride * (k + m), 0x5EED, 0, sp) == 0
        hs = []
        for lib in libs:
            h = C.c_void_p()
            assert lib.rs_codec_create(k, m, C.byref(h)) == 0
            hs.append(h)
        verify = miss == "verify"
        miss = None if verify else miss
        present = bytes(0 if (miss and i in miss) else 1 for i in range(k + m))
        alg = (k + (len(miss) if miss else m)) * S * B
        if verify:
            flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
            assert libs[0].rs_encode_batch_dev(hs[0], pool, B, S, stride, stride * (k + m), sp) == 0

        def call(j):
            if verify:
                assert libs[j].rs_verify_batch_dev(hs[j], pool, B, S, stride, stride * (k + m),
                                                   C.c_void_p(flag.data_ptr()), sp) == 0
            elif miss:
                assert libs[j].rs_decode_batch_dev(hs[j], pool, present, B, S, stride, stride * (k + m), sp) == 0
            else:
                assert libs[j].rs_encode_batch_dev(hs[j], pool, B, S, stride, stride * (k + m), sp) == 0
        for rep in range(reps):
            out = {"shape": name, "rep": rep, "contiguous": bool(got.value)}
            for j, path in enumerate(args):
                for _ in range(5):
                    call(j)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(10):
                    call(j)
                e1.record(st)
                torch.cuda.synchronize()
                out[path.split("/")[-2]] = round(alg / (e0.elapsed_time(e1) / 10 * 1e-3) / 8e12, 4)
            print(json.dumps(out), flush=True)
        torch.cuda.synchronize()
        if verify:
            assert int(flag.item()) == 0, "verify flagged a clean batch"
        libs[0].rs_dev_free(pool)


if __name__ == "__main__":
    main()
