#!/usr/bin/env python3
"""One device workload per process, for rocprofv3 --pmc passes: prepares the
data (fill + encode), then launches the measured kernel 3 times and prints
{"workload", "kernel", "alg_bytes_per_launch"} as JSON.  tools/gpu_pmc_all.sh
runs every workload under FETCH_SIZE and WRITE_SIZE and turns the median
dispatch into HBM bytes per launch (tools/pmc_summary.py).

Workloads (bench.py's configs):
  enc42g     4+2 x 1 MiB x 4096, encode, granule layout (the headline)  alg (4+2) S B
  enc42      the same, packed shards
  dec42_01   4+2 x 1 MiB x 4096, decode {0,1}          alg (4+2) S B
  enc104p / dec104p   enc104 / dec104 with a 4 KiB pad between shards
  enc104     10+4 x 4 MiB x 128, encode                 alg 14 S B
  enc104k / enc104kg  10+4 x 4 MiB x 1024 encode, packed / granule layout (32 KiB)  alg 14 S B
  enc104kc   enc104k on a pool from rs_dev_alloc (physically contiguous, as bench.py allocates)
  dec104     10+4 x 4 MiB x 128, decode {0,1,2,3}       alg 14 S B
  enc42_4k   4+2 x 4 KiB x 1 M, encode                  alg 6 S B
  maskbits   4+2 x 4 KiB x 1 M, per-stripe bitmasks      alg (4 * stripes with a loss + erased shards) S
  gmaskbits  the same in the granule layout (64 KiB rows of 16 stripes)
  cgmaskbits / cgmaskbits1k   4+2 x 1000 B x 4 M chunk groups, stride 1000 / 1024, bitmasks
  cgenc / cgdec01             the same groups at stride 1000: encode / uniform {0,1} decode (line-owner kernel)
  cgdec05 / cgdec15           ... uniform {0,5} / {1,5} decodes
  cgsmenc / cgsmdec01 / cgsmdec05  the same 4 M groups shard-major ([server][group*1000], one
                                   array per server): encode, decodes via rs_decode_groups_shard_major_dev
  cgsmh2odd  ... {0,3} lost from group 2 M + 1 on only (one run 112 B past a line; the head
             peel of a TUNING build is RSAMD_LINE_PEEL)    alg 6 S (B - 2 M - 1)
  enc42off   4+2 x 1 MiB x 1024 packed, 16 B past a line, encode (with a TUNING build:
             RSAMD_LINE_PEEL=0 codes it unpeeled, unset peels to 1 KiB)  alg 6 S B
  fenc       4 GiB file -> 4+2 shards (fused)            alg file + 6 S
  fdec_05    4+2 shards {0,5} -> 4 GiB file (tiled)      alg 4 S + file
"""
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))

SEED = 0x5EED


def main():
    name = sys.argv[1]
    import numpy as np
    import torch
    if len(sys.argv) > 2:  # a variant librsamd.so (A/B builds)
        from rsamd import _lib
        _lib.LIB_PATH = os.path.abspath(sys.argv[2])
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    st = torch.cuda.current_stream()

    def stripes(k, m, S, B, pad=0):
        rs = rsamd.ReedSolomon.create(k, m)
        lay = StripeLayout.packed(B, k + m, S, pad=pad)
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, st)
        rdev.encode(rs, buf.data_ptr(), lay, st)
        return rs, lay, buf

    if name == "enc42g":
        k, m, S, B = 4, 2, 1 << 20, 4096
        rs = rsamd.ReedSolomon.create(k, m)
        lay = rdev.GranuleLayout.make(B, k + m, S)
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, st)
        fn = lambda: rdev.encode(rs, buf.data_ptr(), lay, st)  # noqa: E731
        alg = (k + m) * S * B
        kernel = f"gf_vec_kernel<{k}, {m}, false>"
    elif name in ("dec42_01", "dec104", "enc104", "enc42_4k", "enc42", "enc104p", "dec104p"):
        k, m, S, B = {"dec42_01": (4, 2, 1 << 20, 4096), "dec104": (10, 4, 4 << 20, 128),
                      "enc104": (10, 4, 4 << 20, 128), "enc42_4k": (4, 2, 4096, 1 << 20),
                      "enc42": (4, 2, 1 << 20, 4096), "enc104p": (10, 4, 4 << 20, 128),
                      "dec104p": (10, 4, 4 << 20, 128)}[name]
        rs, lay, buf = stripes(k, m, S, B, 4096 if name.endswith("p") else 0)
        if name.startswith("dec"):
            miss = (0, 1) if k == 4 else (0, 1, 2, 3)
            present = [i not in miss for i in range(k + m)]
            fn = lambda: rdev.decode(rs, buf.data_ptr(), present, lay, st)  # noqa: E731
            alg = (k + len(miss)) * S * B
            kernel = f"gf_vec_kernel<{k}, {len(miss)}, false>"
        else:
            fn = lambda: rdev.encode(rs, buf.data_ptr(), lay, st)  # noqa: E731
            alg = (k + m) * S * B
            kernel = f"gf_vec_kernel<{k}, {m}, false>"
    elif name in ("enc104k", "enc104kg", "enc104kc"):
        k, m, S, B = 10, 4, 4 << 20, 1024
        rs = rsamd.ReedSolomon.create(k, m)
        lay = rdev.GranuleLayout.make(B, k + m, S) if name == "enc104kg" else StripeLayout.packed(B, k + m, S)
        # enc104kc: the pool as bench.py allocates it (rs_dev_alloc, one physically contiguous range)
        buf = (rdev.DeviceBuffer(lay.nbytes, contiguous=True) if name == "enc104kc"
               else torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0"))
        rdev.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, st)
        fn = lambda: rdev.encode(rs, buf.data_ptr(), lay, st)  # noqa: E731
        alg = (k + m) * S * B
        kernel = f"gf_vec_kernel<{k}, {m}, false>"
    elif name == "enc42off":
        k, m, S, B = 4, 2, 1 << 20, 1024
        rs = rsamd.ReedSolomon.create(k, m)
        lay = StripeLayout.packed(B, k + m, S)
        pool = torch.empty(lay.nbytes + 4096, dtype=torch.uint8, device="cuda:0")
        b = pool.data_ptr() + 16
        rdev.fill_synthetic(b, k, lay, SEED, 0, st)
        fn = lambda: rdev.encode(rs, b, lay, st)  # noqa: E731
        alg = (k + m) * S * B
        kernel = f"gf_vec_kernel<{k}, {m}, false>"
    elif name == "maskbits":
        k, m, S, B = 4, 2, 4096, 1 << 20
        rs, lay, buf = stripes(k, m, S, B)
        pats = np.array([[i not in miss for i in range(6)] for e in range(3)
                         for miss in itertools.combinations(range(6), e)], dtype=bool)
        present = pats[np.random.default_rng(0).integers(0, len(pats), B)]
        bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).to("cuda:0")
        fn = lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, st)  # noqa: E731
        alg = (4 * int((~present).any(axis=1).sum()) + int((~present).sum())) * S
        kernel = "gf_masked_kernel<4, 2>"
    elif name == "gmaskbits":
        # config[4] in the granule layout, a random pattern per stripe (<= 2 erasures)
        k, m, S, B = 4, 2, 4096, 1 << 20
        rs = rsamd.ReedSolomon.create(k, m)
        lay = rdev.GranuleLayout.make(B, k + m, S)
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, st)
        rdev.encode(rs, buf.data_ptr(), lay, st)
        pats = np.array([[i not in miss for i in range(6)] for e in range(3)
                         for miss in itertools.combinations(range(6), e)], dtype=bool)
        present = pats[np.random.default_rng(0).integers(0, len(pats), B)]
        bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).to("cuda:0")
        fn = lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, st)  # noqa: E731
        alg = (4 * int((~present).any(axis=1).sum()) + int((~present).sum())) * S
        kernel = "gf_masked_kernel<4, 2, true>"
    elif name in ("cgmaskbits", "cgmaskbits1k"):
        # the master's chunk groups: 4+2 x 1000 B x 4 M, stride 1000 (8-byte kernel) or 1024
        k, m, S, B = 4, 2, 1000, 4 << 20
        stride = 1000 if name == "cgmaskbits" else 1024
        rs = rsamd.ReedSolomon.create(k, m)
        lay = StripeLayout(B, S, stride, 6 * stride)
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, st)
        rdev.encode(rs, buf.data_ptr(), lay, st)
        pats = np.array([[i not in miss for i in range(6)] for e in range(3)
                         for miss in itertools.combinations(range(6), e)], dtype=bool)
        present = pats[np.random.default_rng(0).integers(0, len(pats), B)]
        bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).to("cuda:0")
        fn = lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, st)  # noqa: E731
        alg = (4 * int((~present).any(axis=1).sum()) + int((~present).sum())) * S
        kernel = "gf_group8_kernel<4, 2, true>" if stride == 1000 else "gf_masked8_kernel<4, 2>"
    elif name in ("cgenc", "cgdec01", "cgdec05", "cgdec15"):
        # the master's chunk groups packed back to back (stride 1000): the
        # line-owner kernel, encode or the uniform {0,1} decode
        k, m, S, B = 4, 2, 1000, 4 << 20
        rs = rsamd.ReedSolomon.create(k, m)
        lay = StripeLayout(B, S, S, 6 * S)
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, st)
        rdev.encode(rs, buf.data_ptr(), lay, st)
        if name == "cgenc":
            fn = lambda: rdev.encode(rs, buf.data_ptr(), lay, st)  # noqa: E731
        else:
            miss = {"cgdec01": (0, 1), "cgdec05": (0, 5), "cgdec15": (1, 5)}[name]
            pres = [i not in miss for i in range(6)]
            fn = lambda: rdev.decode(rs, buf.data_ptr(), pres, lay, st)  # noqa: E731
        alg = 6 * S * B
        kernel = "gf_group8_kernel<4, 2, false>"
    elif name in ("cgsmenc", "cgsmdec01", "cgsmdec05", "cgsmh2odd"):
        # the master's chunk groups in its own layout: one array per server
        from rsamd.recovery import recover_groups_shard_major_dev
        k, m, S, B = 4, 2, 1000, 4 << 20
        rs = rsamd.ReedSolomon.create(k, m)
        lay = StripeLayout.recommended(1, 6, S * B)
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, st)
        rdev.encode(rs, buf.data_ptr(), lay, st)
        alg = 6 * S * B
        if name == "cgsmenc":
            fn = lambda: rdev.encode(rs, buf.data_ptr(), lay, st)  # noqa: E731
            kernel = "gf_vec_kernel<4, 2, false>"
        elif name == "cgsmh2odd":
            g0 = B // 2 + 1
            pres = np.ones((B, 6), bool)
            pres[g0:, [0, 3]] = False
            fn = lambda: recover_groups_shard_major_dev(buf.data_ptr(), lay.shard_stride, pres, S, st)  # noqa: E731
            kernel = "gf_vec_kernel<4, 2, false>"
            alg = 6 * S * (B - g0)
        else:
            miss = (0, 1) if name == "cgsmdec01" else (0, 5)
            pres = np.tile(np.array([i not in miss for i in range(6)]), (B, 1))
            fn = lambda: recover_groups_shard_major_dev(buf.data_ptr(), lay.shard_stride, pres, S, st)  # noqa: E731
            kernel = "gf_vec_kernel<4, 2, false>"
    elif name == "ver104":
        k, m, S, B = 10, 4, 4 << 20, 128
        rs, lay, buf = stripes(k, m, S, B)
        flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
        fn = lambda: rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)  # noqa: E731
        alg = (k + m) * S * B  # read-only
        kernel = "gf_vec_kernel<10, 4, true>"
    elif name == "maskbits104":
        k, m, S, B = 10, 4, 4 << 20, 128
        rs, lay, buf = stripes(k, m, S, B)
        rng = np.random.default_rng(0)
        present = np.ones((B, k + m), dtype=bool)
        for t in range(B):
            present[t, rng.choice(k + m, 4, replace=False)] = False
        bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).to("cuda:0")
        fn = lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, st)  # noqa: E731
        alg = (k * B + int((~present).sum())) * S
        kernel = "gf_masked_kernel<10, 4>"
    elif name in ("fenc", "fdec_05"):
        rs = rsamd.ReedSolomon.create(4, 2)
        n = (4 << 30) // 4000 * 4000
        _, S = file_layout(rs, n, 1000)
        stride = (S + 255) // 256 * 256
        f = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        rdev.fill_synthetic(f.data_ptr(), 1, StripeLayout(1, n, n, n), SEED, 0, st)
        sh = torch.empty(6 * stride, dtype=torch.uint8, device="cuda:0")
        enc = lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, 1000, stream=st)  # noqa: E731
        enc()
        if name == "fenc":
            fn, alg, kernel = enc, n + 6 * S, "file_encode_kernel<4, 2"
        else:
            g = torch.empty(n, dtype=torch.uint8, device="cuda:0")
            present = [0, 1, 1, 1, 1, 0]
            fn = lambda: decode_file_dev(rs, sh.data_ptr(), S, stride, present, g.data_ptr(), n, 1000, stream=st)  # noqa: E731
            alg, kernel = 4 * S + n, "file_decode_tiled_kernel<4, 1"
    else:
        raise SystemExit(f"unknown workload {name}")
    fn()  # (warm: plans uploaded)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(3):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 3 * 1e-3
    print(json.dumps({"workload": name, "kernel": kernel, "alg_bytes_per_launch": alg,
                      "frac_of_8TBps": round(alg / t / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
