#!/usr/bin/env python3
"""Granule rows padded and shifted so that reads and writes fall in separate
128 KiB-aligned blocks (HBM serves a block that mixes
them 4-5 points slower).

Each variant is G:ROW:SHIFT in KiB -- granule G, granule-row stride ROW
(>= (k+m)*G; the pad sits after the last shard), batch base moved SHIFT KiB
from a 2 MiB-aligned pool -- coded through the packed view (rows stripes of
G-byte shards, shard stride G, stripe stride ROW), legs alternated across
variants: encode, decode of the first m data shards, decode of shard 0,
verify.  Fractions of 8 TB/s of the algorithmic bytes.
  python tools/row_stride_probe.py [--k 10 --m 4 --S-MiB 4 --B 128] V [V ...]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "java-reed-solomon-distributed-file-system_amd"))


def timed(torch, st, fn, iters=10, warm_s=0.3):
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
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--S-MiB", type=int, default=4)
    ap.add_argument("--B", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch
    import rsamd
    from rsamd import device as rdev
    k, m, S, B = a.k, a.m, a.S_MiB << 20, a.B
    T = k + m
    rs = rsamd.ReedSolomon.create(k, m)
    st = torch.cuda.current_stream()
    pools = []
    for v in a.variants:
        G, row, shift = (int(x) << 10 for x in v.split(":"))
        assert row >= T * G and (S * B) % G == 0
        lay = rdev.StripeLayout(S * B // G, G, G, row)
        pool = rdev.DeviceBuffer(lay.nbytes + shift, contiguous=True)
        base = pool.data_ptr() + shift
        rdev.fill_synthetic(base, k, lay, 0x5EED, 0, st)
        rdev.encode(rs, base, lay, st)
        pools.append((v, lay, pool, base))
    dec = [i not in range(m) for i in range(T)]
    dec0 = [i != 0 for i in range(T)]
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    for r in range(a.rounds):
        for v, lay, pool, base in pools:
            out = {"round": r, "variant": v, "mem_x": round(lay.nbytes / (T * S * B), 4)}
            t = timed(torch, st, lambda: rdev.encode(rs, base, lay, st))
            out["enc"] = round(T * S * B / t / 8e12, 4)
            t = timed(torch, st, lambda: rdev.decode(rs, base, dec, lay, st))
            out["dec_first_m"] = round((k + m) * S * B / t / 8e12, 4)
            t = timed(torch, st, lambda: rdev.decode(rs, base, dec0, lay, st))
            out["dec0"] = round((k + 1) * S * B / t / 8e12, 4)
            t = timed(torch, st, lambda: rdev.verify(rs, base, lay, flag.data_ptr(), st), 5)
            out["verify"] = round(T * S * B / t / 8e12, 4)
            print(json.dumps(out), flush=True)
    for v, lay, pool, base in pools:
        flag.zero_()
        rdev.verify(rs, base, lay, flag.data_ptr(), st)
        torch.cuda.synchronize()
        assert int(flag.item()) == 0, v
        pool.free()


if __name__ == "__main__":
    main()
