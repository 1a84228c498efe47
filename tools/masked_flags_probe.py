#!/usr/bin/env python3
"""Per-stripe presence patterns from host flags against device bitmasks: is the
gap between the two legs kernel time or time between kernels?

config[4] (4+2 x 4 KiB x 1 M) in the granule layout and the 4 M chunk groups
(4+2 x 1000 B, stride 1000), a random pattern per stripe (<= 2 erasures).
Each leg runs back to back; run it under rocprofv3 --kernel-trace --stats to
compare the kernels' own durations with the per-call times printed here.
  python tools/masked_flags_probe.py [--iters 20]
"""
import argparse
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "java-reed-solomon-distributed-file-system_amd"))


def per_call_ms(torch, st, fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record(st)
    for _ in range(iters):
        fn()
    e.record(st)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters, t_host * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout, presence_bits
    st = torch.cuda.current_stream()
    rs = rsamd.ReedSolomon.create(4, 2)
    allp = np.array([[i not in miss for i in range(6)] for e in range(3)
                     for miss in itertools.combinations(range(6), e)], dtype=bool)
    for name, B, S, lay in [("cfg4_granule", 1 << 20, 4096, rdev.GranuleLayout.make(1 << 20, 6, 4096)),
                            ("chunk_groups_stride1000", 4 << 20, 1000, StripeLayout(4 << 20, 1000, 1000, 6000))]:
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        rdev.fill_synthetic(buf.data_ptr(), 4, lay, 7, 0, st)
        rdev.encode(rs, buf.data_ptr(), lay, st)
        pats = allp[np.random.default_rng(1).integers(0, len(allp), B)]
        bits = torch.from_numpy(presence_bits(pats).view(np.int32)).to("cuda:0")
        flags = np.ascontiguousarray(pats)
        gpu_f, host_f = per_call_ms(torch, st, lambda: rdev.decode_masked(rs, buf.data_ptr(), flags, lay, st), a.iters)
        gpu_b, host_b = per_call_ms(torch, st, lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(),
                                                                               lay, 0, st), a.iters)
        print(json.dumps({"batch": name, "flags_ms_per_call": round(gpu_f, 4), "flags_host_enqueue_ms": round(host_f, 4),
                          "bits_ms_per_call": round(gpu_b, 4), "bits_host_enqueue_ms": round(host_b, 4)}), flush=True)
        del buf, bits
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
