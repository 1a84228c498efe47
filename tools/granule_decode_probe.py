#!/usr/bin/env python3
"""Single-output decodes on the granule layout: the
headline batch (4+2 x 1 MiB x 4096) on ONE contiguous pool, viewed with
granules G = 16 KiB .. 256 KiB, timed for encode and decodes {0}, {5}, {0,5},
{0,1}, {2,3}, with the block-order table and with plain / XCD-contiguous order
(rs_debug_block_order).  Legs alternated, each warmed up 0.6 s.  Fractions
of 8 TB/s of the algorithmic bytes ((k + outputs) * S * B).
Usage: python tools/granule_decode_probe.py [ROUNDS] [GRANULES_KIB] [ORDERS]
  GRANULES_KIB: comma list (default 16,32,64,128,256)
  ORDERS: name:rot:xcd;... (default table:-1:-1;plain:0:0;xcd:0:1)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def timed(torch, st, fn, iters=8, warm_s=0.6):
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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    granules = [int(x) << 10 for x in (sys.argv[2] if len(sys.argv) > 2 else "16,32,64,128,256").split(",")]
    spec = sys.argv[3] if len(sys.argv) > 3 else "table:-1:-1;plain:0:0;xcd:0:1"
    orders = [(n, int(r), int(x)) for n, r, x in (o.split(":") for o in spec.split(";"))]
    import torch
    import rsamd
    from rsamd import _lib
    from rsamd import device as rdev
    k, m, S, B = 4, 2, 1 << 20, 4096
    rs = rsamd.ReedSolomon.create(k, m)
    st = torch.cuda.current_stream()
    pool = rdev.DeviceBuffer(B * (k + m) * S, contiguous=True)
    base = pool.data_ptr()
    lib = _lib.load()
    legs = [("enc", None), ("dec0", (0,)), ("dec5", (5,)), ("dec05", (0, 5)), ("dec01", (0, 1)), ("dec23", (2, 3))]
    for r in range(rounds):
        for G in granules:
            lay = rdev.GranuleLayout.make(B, k + m, S, G)
            rdev.fill_synthetic(base, k, lay, 0x5EED, 0, st)
            rdev.encode(rs, base, lay, st)
            for oname, rot, xcd in orders:
                lib.rs_debug_block_order(rot, xcd)
                out = {"round": r, "G_KiB": G >> 10, "order": oname}
                for name, miss in legs:
                    if miss is None:
                        fn = lambda: rdev.encode(rs, base, lay, st)  # noqa: E731
                        nout = m
                    else:
                        present = [i not in miss for i in range(k + m)]
                        fn = lambda p=present: rdev.decode(rs, base, p, lay, st)  # noqa: E731
                        nout = len(miss)
                    t = timed(torch, st, fn)
                    out[name] = round((k + nout) * S * B / t / 8e12, 4)
                print(json.dumps(out), flush=True)
            lib.rs_debug_block_order(-1, -1)
    pool.free()


if __name__ == "__main__":
    main()
