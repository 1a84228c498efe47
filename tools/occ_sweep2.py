#!/usr/bin/env python3
"""Occupancy sweep of the other kernel families, as tools/occ_sweep.py does
for the vector kernels: a TUNING build reads the knob at every launch, this
process changes it between legs (pads alternate within a repetition).
  --family masked: per-stripe patterns (RSAMD_MASKED_LDS_PAD): config[4] in
      the granule layout, random <= 2 erasures per stripe; 10+4 x 4 MiB x 128
      granule, 4 random erasures per stripe; 4+2 x 1 MiB x 4096 granule, random
  --family file: the fused file kernels (RSAMD_FILE_LDS_PAD for the untiled
      encode, RSAMD_FILE_TILE_LDS_PAD extra bytes per tiled-decode workgroup)
  --family copy: the copy kernel (RSAMD_COPY_LDS_PAD), 2 x 8 GiB
  --family group: the master's chunk groups, XCD remap (1) or plain order (0)
      of the line-owner kernel (RSAMD_GROUP_XCD); the file family also
      sweeps RSAMD_FILE_XCD
Prints one JSON line per (leg, repetition): fraction of 8 TB/s per pad.
  python tools/occ_sweep2.py --family masked|file|copy [--pads ...] [--reps N]"""
import argparse
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def sweep(torch, st, name, env, pads, fn, alg, reps):
    for rep in range(reps):
        out = {"leg": name, "rep": rep, "env": env}
        for pad in pads:
            os.environ[env] = str(pad)
            for _ in range(4):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(8):
                fn()
            e1.record(st)
            torch.cuda.synchronize()
            out[str(pad)] = round(alg / (e0.elapsed_time(e1) / 8 * 1e-3) / 8e12, 4)
        os.environ.pop(env, None)
        print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", required=True, choices=["masked", "file", "copy", "group", "slots"])
    ap.add_argument("--lib", default=os.path.join(ROOT, "build/ab/tuning/librsamd.so"))
    ap.add_argument("--pads", default="0,10240,11520,12544,13568,14848,16384,20480")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--shapes", default="", help="masked family: comma-separated shape names")
    a = ap.parse_args()
    import numpy as np
    import torch
    from rsamd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    import rsamd
    from rsamd import device as rdev
    pads = [int(x) for x in a.pads.split(",")]
    st = torch.cuda.current_stream()
    if a.family == "masked":
        shapes = [("cfg4_granule_random", 4, 2, 4096, 1 << 20, None),
                  ("10p4_granule_4random", 10, 4, 4 << 20, 128, 4),
                  ("4p2_1MiB_granule_random", 4, 2, 1 << 20, 4096, None),
                  # other codes (the runtime-k masked kernel)
                  ("6p3_granule_3random", 6, 3, 1 << 20, 2048, 3),
                  ("8p4_granule_2random", 8, 4, 1 << 20, 1024, 2),
                  ("17p3_granule_3random", 17, 3, 1 << 20, 512, 3)]
        want = set(a.shapes.split(",")) if a.shapes else None
        for name, k, m, S, B, nerase in shapes:
            if want and name not in want:
                continue
            T = k + m
            rs = rsamd.ReedSolomon.create(k, m)
            lay = rdev.GranuleLayout.make(B, T, S)
            pool = rdev.DeviceBuffer(lay.nbytes, contiguous=True)
            base = pool.data_ptr()
            rdev.fill_synthetic(base, k, lay, 0x5EED, 0, st)
            rdev.encode(rs, base, lay, st)
            rng = np.random.default_rng(0)
            if nerase:
                pres = np.ones((B, T), dtype=bool)
                for t in range(B):
                    pres[t, rng.choice(T, nerase, replace=False)] = False
            else:
                pats = np.array([[i not in mi for i in range(T)] for e in range(3)
                                 for mi in itertools.combinations(range(T), e)], dtype=bool)
                pres = pats[rng.integers(0, len(pats), B)]
            alg = (k * int((~pres).any(axis=1).sum()) + int((~pres).sum())) * S
            bits = torch.from_numpy(rdev.presence_bits(pres).view(np.int32)).to("cuda:0")
            sweep(torch, st, name, "RSAMD_MASKED_LDS_PAD", pads,
                  lambda: rdev.decode_masked_bits(rs, base, bits.data_ptr(), lay, 0, st), alg, a.reps)
            flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
            rdev.verify(rs, base, lay, flag.data_ptr(), st)
            torch.cuda.synchronize()
            assert int(flag.item()) == 0, name
            pool.free()
    elif a.family == "file":
        from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
        rs = rsamd.ReedSolomon.create(4, 2)
        n = 4 << 30
        _, S = file_layout(rs, n)
        stride = (S + 255) // 256 * 256
        f = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        from rsamd.device import StripeLayout
        rdev.fill_synthetic(f.data_ptr(), 1, StripeLayout(1, n, n, n), 0x5EED, 0, st)
        sh = torch.empty(6 * stride, dtype=torch.uint8, device="cuda:0")
        sweep(torch, st, "file_encode_4GiB", "RSAMD_FILE_LDS_PAD", pads,
              lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, stream=st), n + 6 * S, a.reps)
        g = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        present = [False, True, True, True, True, False]
        tile_pads = [0, 8192, 16384, 24576, 32768, 49152]
        sweep(torch, st, "file_decode_0_5_4GiB_tiled", "RSAMD_FILE_TILE_LDS_PAD", tile_pads,
              lambda: decode_file_dev(rs, sh.data_ptr(), S, stride, present, g.data_ptr(), n, stream=st),
              4 * S + n, a.reps)
        sweep(torch, st, "file_encode_4GiB_order", "RSAMD_FILE_XCD", [1, 0],
              lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, stream=st), n + 6 * S, a.reps)
        sweep(torch, st, "file_decode_0_5_4GiB_order", "RSAMD_FILE_XCD", [1, 0],
              lambda: decode_file_dev(rs, sh.data_ptr(), S, stride, present, g.data_ptr(), n, stream=st),
              4 * S + n, a.reps)
        # the tiled encode (RSAMD_FILE_ENCODE=1) at extra LDS per workgroup, against the default
        os.environ["RSAMD_FILE_ENCODE"] = "1"
        sweep(torch, st, "file_encode_4GiB_tiled", "RSAMD_FILE_TILE_LDS_PAD", tile_pads,
              lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, stream=st), n + 6 * S, a.reps)
        os.environ.pop("RSAMD_FILE_ENCODE")
        torch.cuda.synchronize()
        assert torch.equal(f, g)
    elif a.family == "slots":
        # the master's chunk groups in 1 KiB slots (shard stride 1024, 1000-B shards: the
        # 8-byte kernels gf_vec8_kernel / gf_masked8_kernel)
        from rsamd.device import StripeLayout
        k, m, S, B = 4, 2, 1000, 4 << 20
        rs = rsamd.ReedSolomon.create(k, m)
        lay = StripeLayout(B, S, 1024, 6 * 1024)
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, 0x5EED, 0, st)
        rdev.encode(rs, buf.data_ptr(), lay, st)
        sweep(torch, st, "slots_encode", "RSAMD_VEC8_LDS_PAD", pads, lambda: rdev.encode(rs, buf.data_ptr(), lay, st),
              6 * S * B, a.reps)
        pats = np.array([[i not in mi for i in range(6)] for e in range(3)
                         for mi in itertools.combinations(range(6), e)], dtype=bool)
        pres = pats[np.random.default_rng(0).integers(0, len(pats), B)]
        alg = (k * int((~pres).any(axis=1).sum()) + int((~pres).sum())) * S
        bits = torch.from_numpy(rdev.presence_bits(pres).view(np.int32)).to("cuda:0")
        sweep(torch, st, "slots_masked_bits", "RSAMD_MASKED8_LDS_PAD", pads,
              lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, st), alg, a.reps)
    elif a.family == "group":
        # the master's chunk groups (line-owner kernel): the knob is RSAMD_GROUP_XCD (0 plain, 1 remap)
        from rsamd.device import StripeLayout
        k, m, S, B = 4, 2, 1000, 4 << 20
        rs = rsamd.ReedSolomon.create(k, m)
        lay = StripeLayout(B, S, S, 6 * S)
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, 0x5EED, 0, st)
        rdev.encode(rs, buf.data_ptr(), lay, st)
        sweep(torch, st, "cg_encode", "RSAMD_GROUP_XCD", [1, 0], lambda: rdev.encode(rs, buf.data_ptr(), lay, st),
              6 * S * B, a.reps)
        for xcd in ("1", "0"):  # extra LDS per wave (fewer waves per CU) in either order
            os.environ["RSAMD_GROUP_XCD"] = xcd
            sweep(torch, st, f"cg_encode_xcd{xcd}", "RSAMD_GROUP_LDS_PAD_ENV", [0, 1280, 2560, 5120, 8192],
                  lambda: rdev.encode(rs, buf.data_ptr(), lay, st), 6 * S * B, a.reps)
        os.environ.pop("RSAMD_GROUP_XCD")
        pres01 = [False, False, True, True, True, True]
        sweep(torch, st, "cg_decode01", "RSAMD_GROUP_XCD", [1, 0],
              lambda: rdev.decode(rs, buf.data_ptr(), pres01, lay, st), 6 * S * B, a.reps)
        pats = np.array([[i not in mi for i in range(6)] for e in range(3)
                         for mi in itertools.combinations(range(6), e)], dtype=bool)
        pres = pats[np.random.default_rng(0).integers(0, len(pats), B)]
        alg = (k * int((~pres).any(axis=1).sum()) + int((~pres).sum())) * S
        bits = torch.from_numpy(rdev.presence_bits(pres).view(np.int32)).to("cuda:0")
        sweep(torch, st, "cg_masked_bits", "RSAMD_GROUP_XCD", [1, 0],
              lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, st), alg, a.reps)
        for xcd in ("1", "0"):
            os.environ["RSAMD_GROUP_XCD"] = xcd
            sweep(torch, st, f"cg_masked_bits_xcd{xcd}", "RSAMD_GROUP_LDS_PAD_ENV", [0, 1280, 2560, 5120, 8192],
                  lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, st), alg, a.reps)
        os.environ.pop("RSAMD_GROUP_XCD")
    else:
        n = 8 << 30
        buf = torch.empty(2 * n, dtype=torch.uint8, device="cuda:0")
        sweep(torch, st, "copy_8GiB", "RSAMD_COPY_LDS_PAD", pads,
              lambda: rdev.copy(buf.data_ptr() + n, buf.data_ptr(), n, st), 2 * n, a.reps)


if __name__ == "__main__":
    main()
