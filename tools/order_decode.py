#!/usr/bin/env python3
"""Fraction of HBM peak of the 4+2 x 1 MiB x 4096 encode and decodes
({0}, {0,1}, {0,5}) in one process, for block-order A/B runs
(RSAMD_BLOCK_ROT / RSAMD_BLOCK_XCD are read once per process)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench  # noqa: F401  (puts the package on sys.path)
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    k, m, S, B = 4, 2, 1 << 20, 4096
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream()
    rdev.fill_synthetic(buf.data_ptr(), k, lay, 0x5EED, 0, st)
    out = {"rot": os.environ.get("RSAMD_BLOCK_ROT", "table"), "xcd": os.environ.get("RSAMD_BLOCK_XCD", "table")}
    t = bench.timed(torch, st, lambda: rdev.encode(rs, buf.data_ptr(), lay, st), 20)
    out["encode"] = round(6 * S * B / t / 8e12, 4)
    for miss in ((0,), (0, 1), (0, 5)):
        present = [i not in miss for i in range(6)]
        t = bench.timed(torch, st, lambda: rdev.decode(rs, buf.data_ptr(), present, lay, st), 20)
        out["decode_" + "_".join(map(str, miss))] = round((4 + len(miss)) * S * B / t / 8e12, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
