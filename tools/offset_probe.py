#!/usr/bin/env python3
"""Rate vs where the stripe batch starts inside ONE physically contiguous
range (rs_dev_alloc): allocates the batch plus SLACK_GIB, then for each base
offset in OFFSETS_MIB (default 0, STEP_MIB, ... < SLACK_GIB) fills and encodes
the K+M x SHARD x STRIPES batch at base + offset (the product encode, block
order from the table unless ROT/XCD are set) and prints one JSON line:
{"offset_mib", "frac"}.  Separates "the batch's physical alignment" from
"which pool the allocator returned" (tools/placement_probe.py)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import torch
    import rsamd
    from rsamd import _lib
    from rsamd import device as rdev
    from rsamd.device import DeviceBuffer, StripeLayout
    k, m = int(os.environ.get("K", "4")), int(os.environ.get("M", "2"))
    S = int(os.environ.get("SHARD", str(1 << 20)))
    B = int(os.environ.get("STRIPES", "4096"))
    slack = int(float(os.environ.get("SLACK_GIB", "16")) * (1 << 30))
    step = int(float(os.environ.get("STEP_MIB", "256")) * (1 << 20))
    offs = ([int(float(x) * (1 << 20)) for x in os.environ["OFFSETS_MIB"].split(",")] if os.environ.get("OFFSETS_MIB")
            else list(range(0, slack, step)))
    assert max(offs) <= slack
    reps = int(os.environ.get("REPS", "10"))
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    st = torch.cuda.current_stream()
    lib = _lib.load()
    if os.environ.get("ROT") or os.environ.get("XCD"):
        lib.rs_debug_block_order(int(os.environ.get("ROT", "0")), int(os.environ.get("XCD", "0")))
    pool = DeviceBuffer(lay.nbytes + slack, True)
    assert pool.contiguous, "no contiguous range on this device"
    alg = (k + m) * S * B
    for off in offs:
        base = pool.data_ptr() + off
        rdev.fill_synthetic(base, k, lay, 0x5EED, 0, st)
        for _ in range(3):
            rdev.encode(rs, base, lay, st)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st)
        for _ in range(reps):
            rdev.encode(rs, base, lay, st)
        e.record(st)
        torch.cuda.synchronize()
        frac = alg / (s.elapsed_time(e) / reps * 1e-3) / 8e12
        print(json.dumps({"k": k, "m": m, "shard": S, "stripes": B, "offset_mib": off / (1 << 20),
                          "frac": round(frac, 4)}), flush=True)
    pool.free()


if __name__ == "__main__":
    main()
