#!/usr/bin/env python3
"""Product kernels on the granule-interleaved stripe layout.

A batch of B stripes of k+m shards of S bytes stored as [stripe][granule]
[shard][G] (granule g of every shard stored together) is, byte for byte, a
packed batch of B*S/G stripes of G-byte shards: shard stride G, stripe stride
(k+m)*G.  Coding is per column, so the existing entry points code it
unchanged.  This probe times encode / decode / verify of the BASELINE shapes
in the packed layout and in the granule layout for a few G, on ONE contiguous
pool per shape, legs alternated over rounds, each leg warmed up 0.6 s, with
the table's block order and with the plain order (rs_debug_block_order).
Usage: python tools/granule_probe.py [ROUNDS]"""
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
    import torch
    import rsamd
    from rsamd import _lib
    from rsamd import device as rdev
    from rsamd.device import DeviceBuffer, StripeLayout
    st = torch.cuda.current_stream()
    lib = _lib.load()
    shapes = [("4p2_1MiB_x4096", 4, 2, 1 << 20, 4096, [(0,), (0, 1)]),
              ("10p4_4MiB_x128", 10, 4, 4 << 20, 128, [(0, 1, 2, 3)]),
              ("10p4_4MiB_x1024", 10, 4, 4 << 20, 1024, [])]
    for name, k, m, S, B, decs in shapes:
        rs = rsamd.ReedSolomon.create(k, m)
        pool = DeviceBuffer(B * (k + m) * S, contiguous=True)
        base = pool.data_ptr()
        flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
        res = {}
        for r in range(rounds):
            for G in (None, 32768, 65536, 131072):
                lay = (StripeLayout(B, S, S, (k + m) * S) if G is None else
                       StripeLayout(B * S // G, G, G, (k + m) * G))
                rdev.fill_synthetic(base, k, lay, 0x5EED, 0, st)
                for order in ("table", "plain"):
                    lib.rs_debug_block_order(-1 if order == "table" else 0, -1 if order == "table" else 0)
                    tag = f"{'packed' if G is None else 'G' + str(G // 1024) + 'K'} {order}"
                    t = timed(torch, st, lambda: rdev.encode(rs, base, lay, st))
                    res.setdefault(f"encode {tag}", []).append(round((k + m) * S * B / t / 8e12, 4))
                    for miss in decs:
                        present = [i not in miss for i in range(k + m)]
                        t = timed(torch, st, lambda: rdev.decode(rs, base, present, lay, st))
                        res.setdefault(f"decode {''.join(map(str, miss))} {tag}", []).append(
                            round((k + len(miss)) * S * B / t / 8e12, 4))
                    if r == 0:
                        flag.zero_()
                        rdev.verify(rs, base, lay, flag.data_ptr(), st)
                        torch.cuda.synchronize()
                        assert int(flag.item()) == 0, f"{name} {tag}: verify flagged the batch"
            lib.rs_debug_block_order(-1, -1)
            print(f"{name} round {r} done", file=sys.stderr, flush=True)
        for key, v in res.items():
            print(json.dumps({"shape": name, "leg": key, "fracs": v, "median": sorted(v)[len(v) // 2]}), flush=True)
        pool.free()
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
