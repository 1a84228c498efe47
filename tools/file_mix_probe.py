#!/usr/bin/env python3
"""The fused file kernels in HBM (row f1, bench.py layout_legs) by block size:
a 4 GiB file encoded into 4+2 shards and decoded back with {0,5} erased, at
1000-byte blocks (the DFS's) and at blocks long enough that every run is a
plain stream.  If the long blocks read no higher, the 1000-byte kernels are at
the ceiling of their read/write mix (encode: 4 parts read, 6 written), not
held back by the interleave.  Fractions of 8 TB/s, HIP events, 5 calls.
  python tools/file_mix_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import torch
    import rsamd
    import bench
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    rs = rsamd.ReedSolomon.create(4, 2)
    n = 4 << 30
    f = torch.empty(n, dtype=torch.uint8, device=dev)
    rdev.fill_synthetic(f.data_ptr(), 1, StripeLayout(1, n, n, n), 0x5EED, 0, st)
    g = torch.empty(n, dtype=torch.uint8, device=dev)
    for block in (1000, 1024, 4096, 65536, 1 << 20):
        _, S = file_layout(rs, n, block)
        stride = (S + 255) // 256 * 256
        sh = torch.empty(6 * stride, dtype=torch.uint8, device=dev)
        te = bench.timed(torch, st, lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, block, st), 5)
        present = [False, True, True, True, True, False]
        td = bench.timed(torch, st, lambda: decode_file_dev(rs, sh.data_ptr(), S, stride, present, g.data_ptr(), n,
                                                            block, False, st), 5)
        ok = bool(torch.equal(f, g))
        print(json.dumps({"block": block, "encode_frac": round((n + 6 * S) / te / 8e12, 4),
                          "decode_0_5_frac": round((4 * S + n) / td / 8e12, 4), "round_trip_ok": ok}), flush=True)
        del sh
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
