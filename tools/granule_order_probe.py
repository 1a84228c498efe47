#!/usr/bin/env python3
"""Block order for the granule layout's small sub-stripes: the product encode
(and a decode) of the BASELINE shapes in the granule layout for several G,
under plain order, the XCD-contiguous remap and two chunk rotations, on ONE
contiguous pool per shape, alternated over rounds, each leg warmed up 0.6 s.
Usage: python tools/granule_order_probe.py [ROUNDS]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from granule_probe import timed  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    import torch
    import rsamd
    from rsamd import _lib
    from rsamd import device as rdev
    from rsamd.device import DeviceBuffer, StripeLayout
    st = torch.cuda.current_stream()
    lib = _lib.load()
    shapes = [("4p2_1MiB_x4096", 4, 2, 1 << 20, 4096, (0, 1), (8192, 16384, 32768, 65536, 131072)),
              ("10p4_4MiB_x128", 10, 4, 4 << 20, 128, (0, 1, 2, 3), (8192, 16384, 32768, 65536)),
              ("10p4_4MiB_x1024", 10, 4, 4 << 20, 1024, None, (16384, 32768, 65536))]
    for name, k, m, S, B, miss, grans in shapes:
        rs = rsamd.ReedSolomon.create(k, m)
        pool = DeviceBuffer(B * (k + m) * S, contiguous=True)
        base = pool.data_ptr()
        res = {}
        for r in range(rounds):
            for G in grans:
                lay = StripeLayout(B * S // G, G, G, (k + m) * G)
                rdev.fill_synthetic(base, k, lay, 0x5EED, 0, st)
                chunks = G // 1024
                orders = [("plain", 0, 0), ("xcd", 0, 1), ("rot3/8", max(1, 3 * chunks // 8 - 1), 0),
                          ("rot3/8+xcd", max(1, 3 * chunks // 8 - 1), 1), ("table", -1, -1)]
                for oname, rot, xcd in orders:
                    lib.rs_debug_block_order(rot, xcd)
                    t = timed(torch, st, lambda: rdev.encode(rs, base, lay, st))
                    res.setdefault(f"G{G // 1024}K encode {oname}", []).append(round((k + m) * S * B / t / 8e12, 4))
                    if miss:
                        present = [i not in miss for i in range(k + m)]
                        t = timed(torch, st, lambda: rdev.decode(rs, base, present, lay, st))
                        res.setdefault(f"G{G // 1024}K decode {oname}", []).append(
                            round((k + len(miss)) * S * B / t / 8e12, 4))
            lib.rs_debug_block_order(-1, -1)
            print(f"{name} round {r} done", file=sys.stderr, flush=True)
        for key, v in res.items():
            print(json.dumps({"shape": name, "leg": key, "fracs": v, "median": sorted(v)[len(v) // 2]}), flush=True)
        pool.free()
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
