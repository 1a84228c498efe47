#!/usr/bin/env python3
"""BASELINE configs[3] packed (10+4 x 4 MiB x 1024, 56 GiB) on the two kinds of
pool a caller can have, in one process, alternating (the
packed batch read 0.73 or 0.78 by allocation): a physically contiguous range
from rs_dev_alloc (what bench.py allocates) and plain hipMalloc memory (torch),
each at the packed stride and at rs_shard_stride_recommended (+4 KiB), plus the
granule layout.  Fractions of 8 TB/s from HIP events, 3 rounds.
  python tools/pool_state_probe.py [--rounds 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    k, m, S, B = 10, 4, 4 << 20, 1024
    rs = rsamd.ReedSolomon.create(k, m)
    lays = {"packed": StripeLayout.packed(B, k + m, S), "stride_rec": StripeLayout.recommended(B, k + m, S),
            "granule": rdev.GranuleLayout.make(B, k + m, S)}
    nbytes = max(l.nbytes for l in lays.values())
    contig = rdev.DeviceBuffer(nbytes, contiguous=True)
    plain = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    pools = {"contiguous" if contig.contiguous else "contiguous_fallback": contig.data_ptr(), "hipmalloc": plain.data_ptr()}
    st = torch.cuda.current_stream()
    alg = (k + m) * S * B
    res = {}
    for rnd in range(a.rounds):
        for pname, base in pools.items():
            for lname, lay in lays.items():
                rdev.fill_synthetic(base, k, lay, 0x5EED, 0, st)
                rdev.encode(rs, base, lay, st)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(5):
                    rdev.encode(rs, base, lay, st)
                e1.record(st)
                torch.cuda.synchronize()
                frac = alg / (e0.elapsed_time(e1) / 5 * 1e-3) / 8e12
                res.setdefault(f"{pname}/{lname}", []).append(round(frac, 4))
        print(json.dumps({"round": rnd, **{key: v[-1] for key, v in res.items()}}), flush=True)
    print(json.dumps({"summary": {key: {"min": min(v), "max": max(v)} for key, v in res.items()},
                      "pool_addresses_mod_1G": {p: b % (1 << 30) for p, b in pools.items()}}), flush=True)
    contig.free()


if __name__ == "__main__":
    main()
