#!/usr/bin/env python3
"""Shard-major chunk-group recovery, run by run: why does an offline set that
grows mid-loop (two runs) read below either run alone?

4+2 x 1000 B x B groups in the master's layout [server][group * 1000]
(rs_decode_groups_shard_major_dev).  Each case is a list of (g0, g1, missing)
runs; fractions of 8 TB/s of (k * B + erased chunks) * 1000 B.  Run it under
rocprofv3 --kernel-trace --stats to see each run's kernels.
--lib LIB --peels A ...: a TUNING=1 build, each case at RSAMD_LINE_PEEL=A (the
head-peel alignment of launch_gf_tables, 0 = none); --batch also codes
4+2 x 1 MiB x 1024 stripe batches placed O bytes past a line (--offsets).
  python tools/shard_major_probe.py [--groups 4194304] [--rounds 2]
      [--lib build/ab/tuning/librsamd.so --peels 0 128 256 1024] [--batch --offsets 0 16 112 1008]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "java-reed-solomon-distributed-file-system_amd"))
PEAK = 8000.0


def timed(torch, st, fn, iters=8, warm_s=0.4):
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
    ap.add_argument("--groups", type=int, default=4 << 20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--peels", nargs="*", default=[None])
    ap.add_argument("--batch", action="store_true")
    ap.add_argument("--offsets", nargs="*", type=int, default=[0, 16, 112, 1008])
    a = ap.parse_args()
    import numpy as np
    if a.lib:
        from rsamd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import DeviceBuffer, StripeLayout
    from rsamd.recovery import recover_groups_shard_major_dev
    k, m, S, T, B = 4, 2, 1000, 6, a.groups
    h = B // 2
    cases = {
        "full_0": [(0, B, (0,))],
        "full_03": [(0, B, (0, 3))],
        "h1odd_0": [(0, h + 1, (0,))],
        "h1even_0": [(0, h, (0,))],
        "h2odd_03": [(h + 1, B, (0, 3))],
        "h2even_03": [(h, B, (0, 3))],
        "h2odd_0": [(h + 1, B, (0,))],
        "grows_odd": [(0, h + 1, (0,)), (h + 1, B, (0, 3))],
        "grows_even": [(0, h, (0,)), (h, B, (0, 3))],
        "split_same_odd": [(0, h + 1, (0, 3)), (h + 1, B, (0, 5))],
    }
    st = torch.cuda.current_stream()
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.recommended(1, T, S * B)
    pool = DeviceBuffer(lay.nbytes)
    base = pool.data_ptr()
    device.fill_synthetic(base, k, lay, 7, 0, st)
    device.encode(rs, base, lay, st)
    def set_peel(v):
        if v is None:
            os.environ.pop("RSAMD_LINE_PEEL", None)
        else:
            os.environ["RSAMD_LINE_PEEL"] = str(v)

    # a random pattern per group (<= 2 erasures): past 64 runs the call takes
    # the per-stripe pattern kernels over the same layout
    import itertools
    allp = np.array([[i not in miss for i in range(T)] for e in range(3)
                     for miss in itertools.combinations(range(T), e)], dtype=bool)
    rnd = allp[np.random.default_rng(5).integers(0, len(allp), B)]
    cases["random_per_group"] = "random"
    res = {(c, v): [] for c in cases for v in a.peels}
    for _ in range(a.rounds):
        for name, runs in cases.items():
            pres = np.ones((B, T), bool)
            alg = 0
            if runs == "random":
                pres = rnd
                e = (~rnd).sum(axis=1)
                alg = int(((k + e) * (e > 0)).sum()) * S
                runs = []
            for g0, g1, miss in runs:
                pres[g0:g1, list(miss)] = False
                alg += (g1 - g0) * (k + len(miss)) * S
            for v in a.peels:
                set_peel(v)
                t = timed(torch, st, lambda: recover_groups_shard_major_dev(base, lay.shard_stride, pres, S, st))
                res[(name, v)].append((alg / t / 1e9 / PEAK, t * 1e3))
    for name in cases:
        for v in a.peels:
            print(json.dumps({"case": name, "line_peel": v,
                              "runs": "random" if cases[name] == "random" else
                              [[g0, g1, list(mi)] for g0, g1, mi in cases[name]],
                              "frac": [round(f, 4) for f, _ in res[(name, v)]],
                              "ms": [round(t, 3) for _, t in res[(name, v)]]}), flush=True)
    pool.free()
    del pool
    torch.cuda.empty_cache()
    if a.batch:
        # 4+2 x 1 MiB x 1024 packed stripes O bytes past a line: encode, decode {0,1}
        blay = StripeLayout.packed(1024, T, 1 << 20)
        bpool = DeviceBuffer(blay.nbytes + 4096)
        bres = {(o, v): [] for o in a.offsets for v in a.peels}
        for _ in range(a.rounds):
            for o in a.offsets:
                b = bpool.data_ptr() + o
                device.fill_synthetic(b, k, blay, 7, 0, st)
                for v in a.peels:
                    set_peel(v)
                    te = timed(torch, st, lambda: device.encode(rs, b, blay, st))
                    td = timed(torch, st, lambda: device.decode(rs, b, [False, False, True, True, True, True], blay, st))
                    n = T * (1 << 20) * 1024
                    bres[(o, v)].append((n / te / 1e9 / PEAK, n / td / 1e9 / PEAK))
        for o in a.offsets:
            for v in a.peels:
                print(json.dumps({"batch": "4+2 x 1 MiB x 1024", "offset": o, "line_peel": v,
                                  "encode": [round(x, 4) for x, _ in bres[(o, v)]],
                                  "decode_0_1": [round(y, 4) for _, y in bres[(o, v)]]}), flush=True)
        bpool.free()


if __name__ == "__main__":
    main()
