#!/usr/bin/env python3
"""Fused file layout kernels (row f1) by tile shape, on a TUNING=1 build.

A 4 GiB file, 4+2, block 1000 (the DFS's), as bench.py's layout legs.  A tile
of R block rows spans R * 1000 columns of each shard; R = 8 (the default
shapes) puts every other tile 64 B past a 128-B line on the shard side, R = 16
keeps every tile and every wave's 1 KiB on whole lines.  Variants alternate
over --rounds rounds; each one's output is checked against the first.
  python tools/file_tile_probe.py --lib build/ab/tuning/librsamd.so [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "java-reed-solomon-distributed-file-system_amd"))
PEAK = 8000.0
ENC = [("untiled", {}),
       ("tiled_256x2_R8", {"RSAMD_FILE_ENCODE": "1", "RSAMD_ENC_TILE": "256,2"}),
       ("tiled_512x2_R16", {"RSAMD_FILE_ENCODE": "1", "RSAMD_ENC_TILE": "512,2"}),
       ("tiled_512x1_R8", {"RSAMD_FILE_ENCODE": "1", "RSAMD_ENC_TILE": "512,1"}),
       ("tiled_512x1_R8_lds48K", {"RSAMD_FILE_ENCODE": "1", "RSAMD_ENC_TILE": "512,1", "RSAMD_FILE_TILE_LDS_PAD": "16000"}),
       ("tiled_512x1_R8_lds64K", {"RSAMD_FILE_ENCODE": "1", "RSAMD_ENC_TILE": "512,1", "RSAMD_FILE_TILE_LDS_PAD": "32000"}),
       ("tiled_1024x1_R16", {"RSAMD_FILE_ENCODE": "1", "RSAMD_ENC_TILE": "1024,1"})]
DEC = [("tiled_512x1_R8", {"RSAMD_DEC_TILE": "512,1"}),
       ("tiled_512x2_R16", {"RSAMD_DEC_TILE": "512,2"}),
       ("tiled_256x2_R8", {"RSAMD_DEC_TILE": "256,2"}),
       ("tiled_256x1_R4", {"RSAMD_DEC_TILE": "256,1"}),
       ("tiled_512x1_R8_lds48K", {"RSAMD_DEC_TILE": "512,1", "RSAMD_FILE_TILE_LDS_PAD": "16000"}),
       ("tiled_1024x1_R16", {"RSAMD_DEC_TILE": "1024,1"})]
KNOBS = ("RSAMD_FILE_ENCODE", "RSAMD_ENC_TILE", "RSAMD_DEC_TILE", "RSAMD_FILE_TILE_LDS_PAD")


def timed(torch, st, fn, iters=5, warm_s=0.4):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(st)
    for _ in range(iters):
        fn()
    e.record(st)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def setenv(kv):
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(kv)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--gib", type=int, default=4)
    a = ap.parse_args()
    from rsamd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    st = torch.cuda.current_stream()
    rs = rsamd.ReedSolomon.create(4, 2)
    n = a.gib << 30
    _, S = file_layout(rs, n)
    stride = (S + 255) // 256 * 256
    f = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    rdev.fill_synthetic(f.data_ptr(), 1, StripeLayout(1, n, n, n), 11, 0, st)
    sh = torch.empty(6 * stride, dtype=torch.uint8, device="cuda:0")
    g = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    present = [False, True, True, True, True, False]
    setenv({})
    encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, stream=st)
    ref = sh.view(6, stride)[:, :S].clone()
    res = {("enc", v): [] for v, _ in ENC}
    res.update({("dec", v): [] for v, _ in DEC})
    ok = {}
    for _ in range(a.rounds):
        for v, kv in ENC:
            setenv(kv)
            sh.fill_(0)
            t = timed(torch, st, lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, stream=st))
            res[("enc", v)].append((n + 6 * S) / t / 1e9 / PEAK)
            ok[("enc", v)] = ok.get(("enc", v), True) and bool(torch.equal(sh.view(6, stride)[:, :S], ref))
        setenv({})
        encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, stream=st)
        for v, kv in DEC:
            setenv(kv)
            g.fill_(0)
            t = timed(torch, st, lambda: decode_file_dev(rs, sh.data_ptr(), S, stride, present, g.data_ptr(), n,
                                                         stream=st))
            res[("dec", v)].append((4 * S + n) / t / 1e9 / PEAK)
            ok[("dec", v)] = ok.get(("dec", v), True) and bool(torch.equal(f, g))
    setenv({})
    for (kind, v), fr in res.items():
        print(json.dumps({"leg": "file_" + kind, "variant": v, "frac": [round(x, 4) for x in fr],
                          "verified": ok[(kind, v)]}), flush=True)


if __name__ == "__main__":
    main()
