#!/usr/bin/env python3
"""Decode patterns of the bench headline's granule batch (4+2 x 1 MiB x 4096,
G = 64 KiB, one contiguous pool): encode and decodes {0}, {5}, {0,5}, {0,1},
legs alternated, each warmed up 0.6 s, fractions of 8 TB/s of the
algorithmic bytes ((k + outputs) * S * B).  --lib runs a variant build.
  python tools/dec_probe.py [--rounds R] [--lib LIB]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "java-reed-solomon-distributed-file-system_amd"))


def timed(torch, st, fn, iters=10, warm_s=0.6):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(st)
    for _ in range(iters):
        fn()
    e.record(st)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--granule", type=int, default=64)
    ap.add_argument("--row-pad", type=int, default=0, help="KiB between granule rows (the packed view's stripe stride grows)")
    a = ap.parse_args()
    import torch
    if a.lib:
        from rsamd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    import rsamd
    from rsamd import device as rdev
    k, m, S, B = 4, 2, 1 << 20, 4096
    rs = rsamd.ReedSolomon.create(k, m)
    lay = rdev.GranuleLayout.make(B, k + m, S, a.granule << 10)
    if a.row_pad:
        G = a.granule << 10
        lay = rdev.StripeLayout(lay.rows, G, G, (k + m) * G + (a.row_pad << 10))
    pool = rdev.DeviceBuffer(lay.nbytes, contiguous=True)
    base, st = pool.data_ptr(), torch.cuda.current_stream()
    rdev.fill_synthetic(base, k, lay, 0x5EED, 0, st)
    rdev.encode(rs, base, lay, st)
    legs = [("enc", None), ("dec0", (0,)), ("dec5", (5,)), ("dec05", (0, 5)), ("dec01", (0, 1))]
    for r in range(a.rounds):
        out = {"round": r, "lib": a.lib or "in-tree", "G_KiB": a.granule, "row_pad_KiB": a.row_pad}
        for name, miss in legs:
            if miss is None:
                t = timed(torch, st, lambda: rdev.encode(rs, base, lay, st))
                out[name] = round((k + m) * S * B / t / 8e12, 4)
            else:
                pres = [i not in miss for i in range(k + m)]
                t = timed(torch, st, lambda: rdev.decode(rs, base, pres, lay, st))
                out[name] = round((k + len(miss)) * S * B / t / 8e12, 4)
        print(json.dumps(out), flush=True)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    rdev.verify(rs, base, lay, flag.data_ptr(), st)
    torch.cuda.synchronize()
    assert int(flag.item()) == 0
    pool.free()


if __name__ == "__main__":
    main()
