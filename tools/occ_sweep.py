#!/usr/bin/env python3
"""Occupancy sweep of the vector kernels on one pool per shape: a TUNING build
(make TUNING=1) reads RSAMD_VEC_LDS_PAD at every launch, so this process sets
it between legs and times the same batch at each cap (dynamic LDS per
one-wave workgroup: 160 KiB / pad waves per CU).  Pads alternate within a
repetition, so placement and clock drift are common to all of them.
Prints one JSON line per (shape, repetition): fraction of 8 TB/s per pad.
  python tools/occ_sweep.py [--lib build/ab/tuning/librsamd.so] [--reps N]
                            [--pads 0,10240,...] [--shapes name,...] [--env VAR]
                            [--cross RSAMD_BLOCK_XCD=0,1 ...]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))

# (name, k, m, S, B, miss, granule); miss None = encode, "verify" = verify
SHAPES = [("4p2g_enc", 4, 2, 1 << 20, 4096, None, 64 << 10),
          ("4p2g_dec0", 4, 2, 1 << 20, 4096, (0,), 64 << 10),
          ("4p2g_dec01", 4, 2, 1 << 20, 4096, (0, 1), 64 << 10),
          ("4p2g_dec05", 4, 2, 1 << 20, 4096, (0, 5), 64 << 10),
          ("4p2g_verify", 4, 2, 1 << 20, 4096, "verify", 64 << 10),
          ("4p2_enc", 4, 2, 1 << 20, 4096, None, 0),
          ("4p2_dec01", 4, 2, 1 << 20, 4096, (0, 1), 0),
          ("4p2g4k_enc", 4, 2, 4096, 1 << 20, None, 64 << 10),
          ("4p2_4k_enc", 4, 2, 4096, 1 << 20, None, 0),
          ("10p4g_enc", 10, 4, 4 << 20, 128, None, 32 << 10),
          ("10p4g_dec0123", 10, 4, 4 << 20, 128, (0, 1, 2, 3), 32 << 10),
          ("10p4g_dec01", 10, 4, 4 << 20, 128, (0, 1), 32 << 10),
          ("10p4g_dec012", 10, 4, 4 << 20, 128, (0, 1, 2), 32 << 10),
          ("10p4g_dec0", 10, 4, 4 << 20, 128, (0,), 32 << 10),
          ("10p4g_verify", 10, 4, 4 << 20, 128, "verify", 32 << 10),
          ("10p4_enc", 10, 4, 4 << 20, 128, None, 0),
          ("10p4_dec0123", 10, 4, 4 << 20, 128, (0, 1, 2, 3), 0),
          ("10p4x1024_enc", 10, 4, 4 << 20, 1024, None, 0),
          # other codes (runtime-k kernel), granule layout at rs_granule_recommended
          ("17p3g_enc", 17, 3, 1 << 20, 512, None, 16 << 10),
          ("17p3g_dec012", 17, 3, 1 << 20, 512, (0, 1, 2), 16 << 10),
          ("8p4g_enc", 8, 4, 1 << 20, 1024, None, 32 << 10),
          ("8p4g_dec0", 8, 4, 1 << 20, 1024, (0,), 32 << 10),
          ("6p3g_enc", 6, 3, 1 << 20, 2048, None, 32 << 10),
          ("6p3g_dec01", 6, 3, 1 << 20, 2048, (0, 1), 32 << 10),
          # other granules, for the layout x occupancy cross-check
          ("4p2g32_enc", 4, 2, 1 << 20, 4096, None, 32 << 10),
          ("4p2g128_enc", 4, 2, 1 << 20, 4096, None, 128 << 10),
          ("4p2g32_dec0", 4, 2, 1 << 20, 4096, (0,), 32 << 10),
          ("4p2g128_dec0", 4, 2, 1 << 20, 4096, (0,), 128 << 10),
          ("4p2g128_dec05", 4, 2, 1 << 20, 4096, (0, 5), 128 << 10),
          ("10p4g16_enc", 10, 4, 4 << 20, 128, None, 16 << 10),
          ("10p4g64_enc", 10, 4, 4 << 20, 128, None, 64 << 10),
          ("10p4g64_dec0123", 10, 4, 4 << 20, 128, (0, 1, 2, 3), 64 << 10),
          # one stripe of 4 GB shards: the master's chunk groups shard-major (4 M x 1000 B)
          ("4p2_1x4G_enc", 4, 2, 4096000000, 1, None, 0),
          ("4p2_1x4G_dec0", 4, 2, 4096000000, 1, (0,), 0),
          ("4p2_1x4G_dec01", 4, 2, 4096000000, 1, (0, 1), 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "build/ab/tuning/librsamd.so"))
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--pads", default="0,10240,11520,12544,13568,14848,16384,20480,27136")
    ap.add_argument("--shapes", default="")
    ap.add_argument("--env", default="RSAMD_VEC_LDS_PAD")
    ap.add_argument("--cross", action="append", default=[],
                    help="VAR=v1,v2,...: an outer knob; 'unset' leaves VAR unset (repeatable: all combinations)")
    a = ap.parse_args()
    import itertools
    cross = []
    for c in a.cross:
        var, _, vals = c.partition("=")
        cross.append([(var, v) for v in vals.split(",")])
    combos = list(itertools.product(*cross)) if cross else [()]
    import ctypes as C
    import torch
    from lib_ab_same import bind
    lib = bind(a.lib)
    pads = [int(x) for x in a.pads.split(",")]
    want = set(a.shapes.split(",")) if a.shapes else None
    st = torch.cuda.current_stream()
    sp = C.c_void_p(st.cuda_stream)
    for name, k, m, S, B, miss, G in SHAPES:
        if want and name not in want:
            continue
        if G:
            S, B = G, B * S // G
        stride = S
        nbytes = B * (k + m) * stride
        pool, got = C.c_void_p(), C.c_int(0)
        assert lib.rs_dev_alloc(C.byref(pool), nbytes, 1, C.byref(got)) == 0
        assert lib.rs_fill_synthetic_dev(pool, k, B, S, stride, stride * (k + m), 0x5EED, 0, sp) == 0
        h = C.c_void_p()
        assert lib.rs_codec_create(k, m, C.byref(h)) == 0
        assert lib.rs_encode_batch_dev(h, pool, B, S, stride, stride * (k + m), sp) == 0
        verify = miss == "verify"
        flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
        present = bytes(0 if (miss and not verify and i in miss) else 1 for i in range(k + m))
        alg = (k + (m if (miss is None or verify) else len(miss))) * S * B

        def call():
            if verify:
                assert lib.rs_verify_batch_dev(h, pool, B, S, stride, stride * (k + m), C.c_void_p(flag.data_ptr()),
                                               sp) == 0
            elif miss:
                assert lib.rs_decode_batch_dev(h, pool, present, B, S, stride, stride * (k + m), sp) == 0
            else:
                assert lib.rs_encode_batch_dev(h, pool, B, S, stride, stride * (k + m), sp) == 0
        for rep in range(a.reps):
            out = {"shape": name, "rep": rep}
            for combo, pad in itertools.product(combos, pads):
                for var, v in combo:
                    if v == "unset":
                        os.environ.pop(var, None)
                    else:
                        os.environ[var] = v
                os.environ[a.env] = str(pad)
                for _ in range(6):
                    call()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(10):
                    call()
                e1.record(st)
                torch.cuda.synchronize()
                key = "/".join([f"{var}={v}" for var, v in combo] + [str(pad)])
                out[key] = round(alg / (e0.elapsed_time(e1) / 10 * 1e-3) / 8e12, 4)
            print(json.dumps(out), flush=True)
        os.environ.pop(a.env, None)
        for c in cross:
            os.environ.pop(c[0][0], None)
        torch.cuda.synchronize()
        assert int(flag.item()) == 0, name
        lib.rs_dev_free(pool)


if __name__ == "__main__":
    main()
