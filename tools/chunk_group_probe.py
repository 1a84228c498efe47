#!/usr/bin/env python3
"""Row f2 at the DFS's own shard size: the master's recovery of 6 x 1000-B
chunk groups (ChunkserverDiskRecoveryMachine.java:34-48, MasterImpl.java:794-839),
batched: B groups of 4+2 x 1000 B, a random presence pattern per group
(<= 2 erasures), device bitmasks, one call.  Strides 1000 (groups packed back
to back, the natural layout), 1008 and 1024.  Also the uniform {0,1} decode
and the encode of the same batch.  Fractions of 8 TB/s of the algorithmic
bytes (k survivors read + absent shards written per group with an erasure).
  python tools/chunk_group_probe.py [--groups N] [--reps R]"""
import argparse
import itertools
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "java-reed-solomon-distributed-file-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=4 << 20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--strides", default="1000,1008,1024")
    ap.add_argument("--lib", default=None, help="a variant librsamd.so (A/B builds)")
    a = ap.parse_args()
    import torch
    import rsamd
    if a.lib:
        from rsamd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    k, m, S, B = 4, 2, 1000, a.groups
    T = k + m
    rs = rsamd.ReedSolomon.create(k, m)
    st = torch.cuda.current_stream()
    pats = np.array([[i not in mi for i in range(T)] for e in range(3) for mi in itertools.combinations(range(T), e)],
                    dtype=bool)
    pres = pats[np.random.default_rng(0).integers(0, len(pats), B)]
    alg_m = (k * int((~pres).any(axis=1).sum()) + int((~pres).sum())) * S
    bits = torch.from_numpy(rdev.presence_bits(pres).view(np.int32)).to("cuda:0")

    def timed(fn, n=10):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(n):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n * 1e-3

    for stride in [int(x) for x in a.strides.split(",")]:
        lay = StripeLayout(B, S, stride, stride * T)
        pool = rdev.DeviceBuffer(lay.nbytes, contiguous=True)
        base = pool.data_ptr()
        rdev.fill_synthetic(base, k, lay, 0x5EED, 0, st)
        rdev.encode(rs, base, lay, st)
        for rep in range(a.reps):
            out = {"groups": B, "S": S, "stride": stride, "rep": rep, "lib": a.lib or "in-tree"}
            t = timed(lambda: rdev.encode(rs, base, lay, st))
            out["encode"] = round(T * S * B / t / 8e12, 4)
            t = timed(lambda: rdev.decode(rs, base, [False, False, True, True, True, True], lay, st))
            out["decode_0_1"] = round(T * S * B / t / 8e12, 4)
            t = timed(lambda: rdev.decode_masked_bits(rs, base, bits.data_ptr(), lay, 0, st))
            out["masked_bits"] = round(alg_m / t / 8e12, 4)
            out["masked_bits_ms"] = round(t * 1e3, 3)
            print(json.dumps(out), flush=True)
        flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
        rdev.verify(rs, base, lay, flag.data_ptr(), st)
        torch.cuda.synchronize()
        assert int(flag.item()) == 0
        pool.free()


if __name__ == "__main__":
    main()
