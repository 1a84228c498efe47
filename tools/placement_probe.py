#!/usr/bin/env python3
"""Does the best block order depend on where the pool lands?  One process:
ALLOCS pools in turn (freed and allocated again; contiguous rs_dev_alloc or
torch), each after a contiguous spacer of SPACERS[i] GiB (shifts where the
pool lands; default none), and on each the K+M x SHARD x STRIPES encode
(default the 4+2 x 1 MiB x 4096 headline) under several block orders
(rs_debug_block_order; ORDERS=name,... selects).  Prints one JSON line per
allocation."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))

ORDERS = [("table", -1, -1), ("rot383", 383, 0), ("rot127", 127, 0), ("rot7", 7, 0), ("xcd", 0, 1),
          ("stripe_major", 0, 0), ("rot1535", 1535, 0), ("xcd_rot1535", 1535, 1), ("xcd_rot383", 383, 1)]
if os.environ.get("ORDERS"):
    ORDERS = [o for o in ORDERS if o[0] in os.environ["ORDERS"].split(",")]


def main():
    import torch
    import rsamd
    from rsamd import _lib
    from rsamd import device as rdev
    from rsamd.device import DeviceBuffer, StripeLayout
    k, m = int(os.environ.get("K", "4")), int(os.environ.get("M", "2"))
    S = int(os.environ.get("SHARD", str(1 << 20)))
    B = int(os.environ.get("STRIPES", "0")) or (24 << 30) // ((k + m) * S)
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    st = torch.cuda.current_stream()
    lib = _lib.load()
    modes = os.environ.get("ALLOCS", "contiguous,contiguous,contiguous,torch,torch,torch").split(",")
    spacers = [float(x) for x in os.environ.get("SPACERS", ",".join("0" * len(modes))).split(",")]
    for mode, sp in zip(modes, spacers):
        spacer = DeviceBuffer(int(sp * (1 << 30)), True) if sp > 0 else None
        buf = DeviceBuffer(lay.nbytes, True) if mode == "contiguous" else torch.empty(lay.nbytes, dtype=torch.uint8,
                                                                                    device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, 0x5EED, 0, st)
        va = buf.data_ptr()
        out = {"alloc": mode, "k": k, "m": m, "shard": S, "stripes": B, "spacer_GiB": sp, "va": hex(va),
               "va_align_log2": (va & -va).bit_length() - 1}
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
        if spacer is not None:
            spacer.free()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
