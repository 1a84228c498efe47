#!/usr/bin/env python3
"""10+4 x 4 MiB (BASELINE configs[3]) through the product kernels over shard
pads, block orders and the two kernel families, in one process: fraction of
the 8 TB/s HBM peak for encode and the {0,1,2,3} decode.
  family: table (rs_debug_xornet(0)) / xornet (rs_debug_xornet(1))
  order:  plain (stripe-major), xcd (XCD-contiguous remap), rot (3/8-stripe
          chunk rotation per stripe), via rs_debug_block_order
Usage: [ALLOC=contiguous PADS=0,8192 ORDERS=xcd,rot FAMILIES=table] python tools/order_pad_sweep.py [stripes ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))

import bench  # noqa: E402


PADS = [int(x) for x in os.environ.get("PADS", "0,4096,8192").split(",")]
ORDERS = os.environ.get("ORDERS", "plain,xcd,rot").split(",")
FAMILIES = [f for f in (("table", 1024), ("xornet", 2048)) if f[0] in os.environ.get("FAMILIES", "table,xornet")]


def main():
    counts = [int(a) for a in sys.argv[1:]] or [128, 1024]
    import torch

    import rsamd
    from rsamd import _lib
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    lib = _lib.load()
    st = torch.cuda.current_stream()
    k, m, S = 10, 4, 4 << 20
    rs = rsamd.ReedSolomon.create(k, m)
    present = [i >= 4 for i in range(k + m)]
    for B in counts:
        for pad in PADS:
            lay = StripeLayout.packed(B, k + m, S, pad=pad)
            if os.environ.get("ALLOC") == "contiguous":
                buf = rdev.DeviceBuffer(lay.nbytes, contiguous=True)
            else:
                buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
            rdev.fill_synthetic(buf.data_ptr(), k, lay, bench.SEED, 0, st)
            for fam, chunk in FAMILIES:
                lib.rs_debug_xornet(0 if fam == "table" else 1)
                chunks = S // chunk
                orders = {"plain": (0, 0), "xcd": (0, 1), "rot": (3 * chunks // 8 - 1, 0)}
                for order in ORDERS:
                    rot, xcd = orders[order]
                    lib.rs_debug_block_order(rot, xcd)
                    te = bench.timed(torch, st, lambda: rdev.encode(rs, buf.data_ptr(), lay, st), 8)
                    td = bench.timed(torch, st, lambda: rdev.decode(rs, buf.data_ptr(), present, lay, st), 8)
                    print(json.dumps({"stripes": B, "pad": pad, "family": fam, "order": order,
                                      "alloc": os.environ.get("ALLOC", "hipmalloc"),
                                      "enc": round(14 * S * B / te / 8e12, 4),
                                      "dec": round(14 * S * B / td / 8e12, 4)}), flush=True)
            lib.rs_debug_block_order(-1, -1)
            lib.rs_debug_xornet(-1)
            flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
            rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
            assert int(flag.item()) == 0
            if isinstance(buf, rdev.DeviceBuffer):
                buf.free()
            del buf
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
