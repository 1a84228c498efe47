#!/usr/bin/env python3
"""A/B of the two kernel families in one process on one GPU: table kernels
(rs_debug_xornet(0)) against the run-time compiled XOR-network kernels
(rs_debug_xornet(1)), alternating, on the bench shapes; fraction of the 8 TB/s
HBM peak per leg (HIP events, bench.py's warm-up rule).
Usage: python tools/xornet_ab.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))

import bench  # noqa: E402  (timed(), SEED)

SHAPES = [  # name, k, m, S, B, erasures for the decode leg
    ("4p2_1MiB_x4096", 4, 2, 1 << 20, 4096, (0, 1)),
    ("10p4_4MiB_x128", 10, 4, 4 << 20, 128, (0, 1, 2, 3)),
    ("10p4_4MiB_x1024", 10, 4, 4 << 20, 1024, (0, 1, 2, 3)),
    ("4p2_4KiB_x1M", 4, 2, 4096, 1 << 20, (0, 1)),
]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    import torch

    import rsamd
    from rsamd import _lib
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    lib = _lib.load()
    st = torch.cuda.current_stream()
    for name, k, m, S, B, miss in SHAPES:
        rs = rsamd.ReedSolomon.create(k, m)
        lay = StripeLayout.packed(B, k + m, S)
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, bench.SEED, 0, st)
        present = [i not in miss for i in range(k + m)]
        res = {"shape": name}
        for rep in range(reps):
            for mode in (0, 1):
                lib.rs_debug_xornet(mode)
                t = bench.timed(torch, st, lambda: rdev.encode(rs, buf.data_ptr(), lay, st), 10)
                res.setdefault(f"enc_x{mode}", []).append(round((k + m) * S * B / t / 8e12, 4))
                t = bench.timed(torch, st, lambda: rdev.decode(rs, buf.data_ptr(), present, lay, st), 10)
                res.setdefault(f"dec_x{mode}", []).append(round((k + len(miss)) * S * B / t / 8e12, 4))
        lib.rs_debug_xornet(-1)
        flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
        rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
        res["verified"] = int(flag.item()) == 0
        print(json.dumps(res), flush=True)
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
