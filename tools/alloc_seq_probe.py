#!/usr/bin/env python3
"""Encode rate of one stripe geometry over a sequence of allocations in ONE
process (free, then allocate again): does the rate follow the allocation
mode or where the allocator happens to place the pool?  Usage:
alloc_seq_probe.py K M SHARD_BYTES STRIPES MODE[,MODE...]  (MODE: torch |
contiguous | big_torch = 24 GiB torch block allocated and freed first)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    k, m, S, B = map(int, sys.argv[1:5])
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import DeviceBuffer, StripeLayout
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    st = torch.cuda.current_stream()
    for mode in sys.argv[5].split(","):
        if mode == "big_torch":
            t = torch.empty(24 << 30, dtype=torch.uint8, device="cuda:0")
            del t
            torch.cuda.empty_cache()
            continue
        buf = DeviceBuffer(lay.nbytes, True) if mode == "contiguous" else torch.empty(lay.nbytes, dtype=torch.uint8,
                                                                                    device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), k, lay, 0x5EED, 0, st)
        for _ in range(3):
            rdev.encode(rs, buf.data_ptr(), lay, st)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st)
        for _ in range(20):
            rdev.encode(rs, buf.data_ptr(), lay, st)
        e.record(st)
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 20
        print(json.dumps({"mode": mode, "frac": round((k + m) * S * B / (ms * 1e-3) / 8e12, 4),
                          "base": hex(buf.data_ptr())}), flush=True)
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
