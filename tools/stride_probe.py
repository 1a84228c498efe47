#!/usr/bin/env python3
"""Packed [stripe][shard][stride] batches at padded shard strides: which
stride should rs_shard_stride_recommended return?

For each shape K:M:S_KiB:B and each pad P (bytes after the 256-rounded
shard), the batch is one rs_dev_alloc pool, encoded and decoded (the first m
data shards) in alternation over --rounds rounds; fractions of 8 TB/s of
(k+m)*S*B and (k+e)*S*B.
  python tools/stride_probe.py --shapes 10:4:4096:1024 4:2:1024:4096 --pads 0 256 1024 4096 8192
--offsets O ...: one pool per shape (allocated once, --extra-MiB larger), the
batch placed O KiB past its start, so the only thing that changes between
variants is the batch's address; the pool's base address is printed.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "java-reed-solomon-distributed-file-system_amd"))
PEAK = 8000.0


def timed(torch, st, fn, iters=8, warm_s=0.4):
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
    ap.add_argument("--shapes", nargs="+", default=["10:4:4096:1024"])
    ap.add_argument("--pads", nargs="+", type=int, default=[0, 4096])
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--offsets", nargs="*", type=int, default=None, help="KiB offsets of the batch in one pool")
    ap.add_argument("--extra-MiB", type=int, default=512)
    a = ap.parse_args()
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import DeviceBuffer, StripeLayout
    st = torch.cuda.current_stream()
    for shape in a.shapes:
        k, m, skib, B = map(int, shape.split(":"))
        S = skib << 10
        rs = rsamd.ReedSolomon.create(k, m)
        present = [i >= m for i in range(k + m)]  # the first m data shards rebuilt
        if a.offsets is not None:
            lay = StripeLayout.packed(B, k + m, S, pad=a.pads[0])
            pool = DeviceBuffer(lay.nbytes + (a.extra_MiB << 20))
            res = {o: {"enc": [], "dec": []} for o in a.offsets}
            for r in range(a.rounds):
                for o in a.offsets:
                    base = pool.data_ptr() + (o << 10)
                    device.fill_synthetic(base, k, lay, 7, 0, st)
                    te = timed(torch, st, lambda: device.encode(rs, base, lay, st))
                    td = timed(torch, st, lambda: device.decode(rs, base, present, lay, st))
                    res[o]["enc"].append((k + m) * S * B / te / 1e9 / PEAK)
                    res[o]["dec"].append((k + m) * S * B / td / 1e9 / PEAK)
            for o in a.offsets:
                print(json.dumps({"shape": shape, "pad": a.pads[0], "pool_base": hex(pool.data_ptr()),
                                  "contiguous": pool.contiguous, "offset_KiB": o,
                                  "encode": [round(x, 4) for x in res[o]["enc"]],
                                  "decode_first_m": [round(x, 4) for x in res[o]["dec"]]}), flush=True)
            pool.free()
            torch.cuda.empty_cache()
            continue
        res = {p: {"enc": [], "dec": []} for p in a.pads}
        for r in range(a.rounds):
            for p in a.pads:
                lay = StripeLayout.packed(B, k + m, S, pad=p)
                buf = DeviceBuffer(lay.nbytes)
                device.fill_synthetic(buf.data_ptr(), k, lay, 7, 0, st)
                te = timed(torch, st, lambda: device.encode(rs, buf.data_ptr(), lay, st))
                td = timed(torch, st, lambda: device.decode(rs, buf.data_ptr(), present, lay, st))
                res[p]["enc"].append((k + m) * S * B / te / 1e9 / PEAK)
                res[p]["dec"].append((k + m) * S * B / td / 1e9 / PEAK)
                buf.free()
                del buf
                torch.cuda.empty_cache()
        for p in a.pads:
            print(json.dumps({"shape": shape, "pad": p, "stride": (S + 255) // 256 * 256 + p,
                              "encode": [round(x, 4) for x in res[p]["enc"]],
                              "decode_first_m": [round(x, 4) for x in res[p]["dec"]]}), flush=True)


if __name__ == "__main__":
    main()
