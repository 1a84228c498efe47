#!/usr/bin/env python3
"""10+4 x 4 MiB x B, 4 random erasures per stripe (device bitmasks, row f2)
next to the uniform {0,1,2,3} decode, under each block order
(rs_debug_block_order), in one process on one pool; fraction of 8 TB/s.
Usage: [SORTED=1] python tools/masked_order_probe.py [stripes] [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))

import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    import numpy as np
    import torch

    import rsamd
    from rsamd import _lib
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    lib = _lib.load()
    st = torch.cuda.current_stream()
    k, m, S = 10, 4, 4 << 20
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    pool = rdev.DeviceBuffer(lay.nbytes, contiguous=True)
    rdev.fill_synthetic(pool.data_ptr(), k, lay, bench.SEED, 0, st)
    rdev.encode(rs, pool.data_ptr(), lay, st)
    rng = np.random.default_rng(0)
    present = np.ones((B, k + m), dtype=bool)
    for t in range(B):
        present[t, rng.choice(k + m, 4, replace=False)] = False
    if os.environ.get("SORTED"):  # stripes in bitmask order: neighbours share erasures
        present = present[np.argsort(rdev.presence_bits(present), kind="stable")]
    bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).to("cuda:0")
    alg = (k * B + int((~present).sum())) * S
    uni = [i >= 4 for i in range(k + m)]
    chunks = S // 1024
    for rep in range(reps):
        for order, (rot, xcd) in (("table", (-1, -1)), ("plain", (0, 0)), ("xcd", (0, 1)),
                                  ("rot3/8", (3 * chunks // 8 - 1, 0)), ("rot1/4", (chunks // 4 - 1, 0))):
            lib.rs_debug_block_order(rot, xcd)
            tm = bench.timed(torch, st, lambda: rdev.decode_masked_bits(rs, pool.data_ptr(), bits.data_ptr(), lay, 0,
                                                                        st), 8)
            tu = bench.timed(torch, st, lambda: rdev.decode(rs, pool.data_ptr(), uni, lay, st), 8)
            print(json.dumps({"rep": rep, "order": order, "masked": round(alg / tm / 8e12, 4),
                              "uniform": round(14 * S * B / tu / 8e12, 4)}), flush=True)
    lib.rs_debug_block_order(-1, -1)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    rdev.verify(rs, pool.data_ptr(), lay, flag.data_ptr(), st)
    assert int(flag.item()) == 0
    pool.free()


if __name__ == "__main__":
    main()
