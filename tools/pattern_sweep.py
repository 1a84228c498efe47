#!/usr/bin/env python3
"""Every erasure pattern of 4+2 as a uniform decode over a granule batch, and
the random per-stripe mix as one bitmask launch (--config chunk/chunk1024: the
master's packed 6 x 1000-B chunk groups instead).

For each of the 21 non-empty patterns (6 single, 15 double erasures) the whole
batch is decoded with that pattern (rs_decode_batch_dev on the granule view)
and timed; the fraction of 8 TB/s counts the algorithmic bytes
((k + erased) * S per stripe).  The random mix of bench.py's config[4] leg
(the 22 patterns of <= 2 erasures, uniform, seed 0) is then decoded in one
bitmask launch (rs_decode_granule_masked_bits_dev), and its time is compared
with the time the same stripes would take at their patterns' uniform rates:
    predicted = sum over stripes of t_uniform(pattern) / B.
  python tools/pattern_sweep.py [--config headline|cfg4] [--shift KiB] [--no-mix]"""
import argparse
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "java-reed-solomon-distributed-file-system_amd"))


def timed(torch, st, fn, iters=10, warm_s=0.3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(st)
    for _ in range(iters):
        fn()
    e.record(st)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4", choices=["headline", "cfg4", "chunk", "chunk1024"])
    ap.add_argument("--shift", type=int, default=0, help="KiB added to the batch's base address")
    ap.add_argument("--no-mix", action="store_true")
    ap.add_argument("--lib", default=None, help="a variant librsamd.so (A/B runs)")
    ap.add_argument("--granule", type=int, default=0, help="granule KiB (default: rs_granule_recommended)")
    a = ap.parse_args()
    import numpy as np
    import torch
    if a.lib:
        from rsamd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    import rsamd
    from rsamd import device as rdev
    k, m = 4, 2
    rs = rsamd.ReedSolomon.create(k, m)
    if a.config.startswith("chunk"):  # the master's chunk groups, packed (bench.py chunk_group_leg)
        S, B = 1000, 4 << 20
        stride = 1024 if a.config == "chunk1024" else 1000
        lay = rdev.StripeLayout(B, S, stride, (k + m) * stride)
    else:
        S, B = (1 << 20, 4096) if a.config == "headline" else (4096, 1 << 20)
        lay = rdev.GranuleLayout.make(B, k + m, S, a.granule << 10)
    pool = rdev.DeviceBuffer(lay.nbytes + (a.shift << 10), contiguous=True)
    base, st = pool.data_ptr() + (a.shift << 10), torch.cuda.current_stream()
    rdev.fill_synthetic(base, k, lay, 0x5EED, 0, st)
    rdev.encode(rs, base, lay, st)
    t_enc = timed(torch, st, lambda: rdev.encode(rs, base, lay, st))
    print(json.dumps({"config": a.config, "S": S, "B": B, "granule": getattr(lay, "granule", 0), "shift_KiB": a.shift, "lib": a.lib or "in-tree",
                      "encode": round((k + m) * S * B / t_enc / 8e12, 4)}), flush=True)
    t_pat = {}
    for e in (1, 2):
        for miss in itertools.combinations(range(k + m), e):
            pres = [i not in miss for i in range(k + m)]
            t = timed(torch, st, lambda: rdev.decode(rs, base, pres, lay, st))
            t_pat[miss] = t
            print(json.dumps({"miss": list(miss), "frac": round((k + e) * S * B / t / 8e12, 4),
                              "ms": round(t * 1e3, 4)}), flush=True)
    fr = [(k + len(mi)) * S * B / t / 8e12 for mi, t in t_pat.items()]
    print(json.dumps({"uniform_min": round(min(fr), 4), "uniform_max": round(max(fr), 4),
                      "uniform_mean": round(sum(fr) / len(fr), 4)}), flush=True)
    if a.no_mix:
        pool.free()
        return
    # bench.py's config[4] mix: the 22 patterns of <= 2 erasures, uniform per stripe
    pats = [tuple(mi) for e in range(3) for mi in itertools.combinations(range(k + m), e)]
    pick = np.random.default_rng(0).integers(0, len(pats), B)
    pres = np.array([[i not in pats[p] for i in range(k + m)] for p in range(len(pats))], dtype=bool)[pick]
    counts = np.bincount(pick, minlength=len(pats))
    predicted = sum(int(c) * t_pat[pats[p]] / B for p, c in enumerate(counts) if pats[p])
    alg = (k * int((~pres).any(axis=1).sum()) + int((~pres).sum())) * S
    bits = torch.from_numpy(rdev.presence_bits(pres).view(np.int32)).to("cuda:0")
    t = timed(torch, st, lambda: rdev.decode_masked_bits(rs, base, bits.data_ptr(), lay, 0, st))
    print(json.dumps({"mix": "22 patterns of <= 2 erasures, seed 0", "masked_bits_frac": round(alg / t / 8e12, 4),
                      "masked_ms": round(t * 1e3, 4), "predicted_from_uniform_ms": round(predicted * 1e3, 4),
                      "predicted_frac": round(alg / predicted / 8e12, 4),
                      "masked_over_predicted_time": round(t / predicted, 4)}), flush=True)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    rdev.verify(rs, base, lay, flag.data_ptr(), st)
    torch.cuda.synchronize()
    assert int(flag.item()) == 0
    pool.free()


if __name__ == "__main__":
    main()
