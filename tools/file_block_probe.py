#!/usr/bin/env python3
"""Row f1: is the fused file encode's gap to its XOR reference (0.825 warm,
tools/file_granule_mem.hip, 1 KiB blocks, 16-B file loads) the DFS's 1000-B
block?  Times the product file encode / {0,5} decode of a 4 GiB file at
block 1000 (the DFS's, ConfigVariables.java:4-9: 16-B column vectors straddle
blocks, so the file side moves in 8-B halves) and block 1024 (every vector
inside one block), legs alternated over rounds, each warmed up 0.6 s.  The
file-side I/O mode is RSAMD_LAYOUT_IO (read once per process: run once per
mode).  Usage: RSAMD_LAYOUT_IO=n python tools/file_block_probe.py [ROUNDS]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from granule_probe import timed  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    st = torch.cuda.current_stream()
    rs = rsamd.ReedSolomon.create(4, 2)
    n0 = 4 << 30
    f = torch.empty(n0, dtype=torch.uint8, device="cuda:0")
    rdev.fill_synthetic(f.data_ptr(), 1, StripeLayout(1, n0, n0, n0), 0x5EED, 0, st)
    g = torch.empty(n0, dtype=torch.uint8, device="cuda:0")
    sh = torch.empty(6 * (n0 // 4 + (1 << 20)), dtype=torch.uint8, device="cuda:0")
    present = [False, True, True, True, True, False]
    res = {}
    for r in range(rounds):
        for blk in (1000, 1024):
            n = n0 // (4 * blk) * (4 * blk)
            _, S = file_layout(rs, n, blk)
            stride = (S + 255) // 256 * 256
            t = timed(torch, st, lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, blk, stream=st))
            res.setdefault(f"encode block {blk}", []).append(round((n + 6 * S) / t / 8e12, 4))
            t = timed(torch, st, lambda: decode_file_dev(rs, sh.data_ptr(), S, stride, present, g.data_ptr(), n, blk,
                                                         stream=st))
            res.setdefault(f"decode block {blk}", []).append(round((n + 4 * S) / t / 8e12, 4))
            if r == 0:
                assert torch.equal(f[:n], g[:n]), f"round trip failed at block {blk}"
    io = os.environ.get("RSAMD_LAYOUT_IO", "default (1)")
    for k, v in res.items():
        print(json.dumps({"io": io, "leg": k, "fracs": v, "median": sorted(v)[len(v) // 2]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
