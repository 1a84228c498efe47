#!/usr/bin/env python3
"""Does the best block order depend on where the pool lands?  One process:
ALLOCS pools in turn (freed and allocated again; contiguous rs_dev_alloc or
torch), and on each the 4+2 x 1 MiB x 4096 encode under several block orders
(rs_debug_block_order).  Prints one JSON line per allocation."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))

ORDERS = [("table", -1, -1), ("rot383", 383, 0), ("rot127", 127, 0), ("rot7", 7, 0), ("xcd", 0, 1),
          ("stripe_major", 0, 0)]


def main():
    import torch
    import rsamd
    from rsamd import _lib
    from rsamd import device as rdev
    from rsamd.device import DeviceBuffer, StripeLayout
    k, m = 4, 2
    S = int(os.environ.get("SHARD", str(1 << 20)))
    B = (24 << 30) // ((k + m) * S)
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    st = torch.cuda.current_stream()
    lib = _lib.load()
    for mode in os.environ.get("ALLOCS", "contiguous,contiguous,contiguous,torch,torch,torch").split(","):
        buf = DeviceBuffer(lay.nbytes, True) if mode == "contiguous" else torch.empty(lay.nbytes, dtype=torch.uint8,
                                                                                    device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, 0x5EED, 0, st)
        out = {"alloc": mode, "shard": S}
        for name, rot, xcd in ORDERS:
            lib.rs_debug_block_order(rot, xcd)
            for _ in range(3):
                rdev.encode(rs, buf.data_ptr(), lay, st)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(st)
            for _ in range(15):
                rdev.encode(rs, buf.data_ptr(), lay, st)
            e.record(st)
            torch.cuda.synchronize()
            out[name] = round((k + m) * S * B / (s.elapsed_time(e) / 15 * 1e-3) / 8e12, 4)
        lib.rs_debug_block_order(-1, -1)
        print(json.dumps(out), flush=True)
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
