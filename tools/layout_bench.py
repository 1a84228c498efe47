#!/usr/bin/env python3
"""Time the row-f1/f2 device paths in one process (file I/O variant from
RSAMD_LAYOUT_IO, read once per process): fused file encode / decode of a 4 GiB
file, and the per-stripe-pattern masked decode on 1 M x 4 KiB stripes."""
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))
sys.path.insert(0, ROOT)


def timed(torch, st, fn, iters=5):
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
    import numpy as np
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    st = torch.cuda.current_stream()
    out = {"io": os.environ.get("RSAMD_LAYOUT_IO", "default")}
    rs = rsamd.ReedSolomon.create(4, 2)
    n = 4 << 30
    blk = int(os.environ.get("RSAMD_BENCH_BLOCK", "1000"))
    out["block"] = blk
    n = n // (4 * blk) * (4 * blk)
    _, S = file_layout(rs, n, blk)
    pad = int(os.environ.get("RSAMD_BENCH_PAD", "0"))
    out["pad"] = pad
    stride = (S + 255) // 256 * 256 + pad
    f = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    rdev.fill_synthetic(f.data_ptr(), 1, StripeLayout(1, n, n, n), 0x5EED, 0, st)
    sh = torch.empty(6 * stride, dtype=torch.uint8, device="cuda:0")
    t = timed(torch, st, lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, blk, stream=st))
    out["file_encode_hbm_frac"] = round((n + 6 * S) / t / 8e12, 4)
    g = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    for present in ([1] * 6, [0, 1, 1, 1, 1, 0], [0, 0, 1, 1, 1, 1]):
        t = timed(torch, st, lambda: decode_file_dev(rs, sh.data_ptr(), S, stride, present, g.data_ptr(), n,
                                                     blk, stream=st))
        key = "file_decode_" + "".join(map(str, present))
        out[key + "_hbm_frac"] = round((4 * S + n) / t / 8e12, 4)
        out[key + "_ok"] = bool(torch.equal(f, g))
    del f, g, sh
    torch.cuda.empty_cache()
    if os.environ.get("RSAMD_BENCH_SKIP_MASKED"):
        print(json.dumps(out), flush=True)
        return
    B, S = 1 << 20, 4096
    lay = StripeLayout.packed(B, 6, S)
    buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    rdev.fill_synthetic(buf.data_ptr(), 4, lay, 0x5EED, 0, st)
    rdev.encode(rs, buf.data_ptr(), lay, st)
    pats = np.array([[i not in miss for i in range(6)] for e in range(3)
                     for miss in itertools.combinations(range(6), e)], dtype=bool)
    present = pats[np.random.default_rng(0).integers(0, len(pats), B)]
    alg = (4 * int((~present).any(axis=1).sum()) + int((~present).sum())) * S
    t = timed(torch, st, lambda: rdev.decode_masked(rs, buf.data_ptr(), present, lay, st))
    out["masked_decode_1Mx4KiB_GiBps"] = round(4 * S * B / t / 2**30, 1)
    out["masked_decode_hbm_frac"] = round(alg / t / 8e12, 4)
    bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).to("cuda:0")
    t = timed(torch, st, lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, st))
    out["masked_bits_decode_hbm_frac"] = round(alg / t / 8e12, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
