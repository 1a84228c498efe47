#!/usr/bin/env python3
"""The fused file encode (row f1, bench.py layout_legs: a 4 GiB file, 4+2,
1000-byte blocks) by the way it reads the file, on a TUNING=1 build, in one
process on one set of buffers: RSAMD_LAYOUT_IO 1 (two plain 8-byte loads per
lane, the default), 2 (one plain 16-byte load when the lane's 16 bytes lie in
one block row), and 3 (the same, non-temporal: measured in round 5,
profiles/r5/file_io_ab_r6i.txt, and deleted; it now runs as 2), each at occupancy caps
(RSAMD_FILE_LDS_PAD) 11520 (the default) and 14848.  Variants alternate over
--rounds rounds; every variant's shards are checked against the first's.
  python tools/file_io_ab.py --lib build/ab/tuning/librsamd.so [--rounds 4]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "java-reed-solomon-distributed-file-system_amd"))
VARIANTS = [("plain8", {"RSAMD_LAYOUT_IO": "1"}),
            ("pair16", {"RSAMD_LAYOUT_IO": "2"}),
            ("pair16_nt", {"RSAMD_LAYOUT_IO": "3"}),
            ("plain8_lds14848", {"RSAMD_LAYOUT_IO": "1", "RSAMD_FILE_LDS_PAD": "14848"}),
            ("pair16_lds14848", {"RSAMD_LAYOUT_IO": "2", "RSAMD_FILE_LDS_PAD": "14848"}),
            ("pair16_nt_lds14848", {"RSAMD_LAYOUT_IO": "3", "RSAMD_FILE_LDS_PAD": "14848"})]
KNOBS = ("RSAMD_LAYOUT_IO", "RSAMD_FILE_LDS_PAD")


def timed(torch, st, fn, iters=5, warm_s=0.3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
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
    ap.add_argument("--lib", required=True)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--gib", type=int, default=4)
    a = ap.parse_args()
    from rsamd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    from rsamd.layout import encode_file_dev, file_layout
    st = torch.cuda.current_stream()
    rs = rsamd.ReedSolomon.create(4, 2)
    n = a.gib << 30
    _, S = file_layout(rs, n)
    stride = (S + 255) // 256 * 256
    f = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    rdev.fill_synthetic(f.data_ptr(), 1, StripeLayout(1, n, n, n), 11, 0, st)
    sh = torch.empty(6 * stride, dtype=torch.uint8, device="cuda:0")
    ref = None
    res = {name: [] for name, _ in VARIANTS}
    for r in range(a.rounds):
        for name, env in VARIANTS:
            for kk in KNOBS:
                os.environ.pop(kk, None)
            os.environ.update(env)
            sh.fill_(0)
            t = timed(torch, st, lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, stream=st))
            if ref is None:
                ref = sh.clone()
            ok = bool(torch.equal(sh, ref))
            frac = round((n + 6 * S) / t / 8e12, 4)
            res[name].append(frac)
            print(json.dumps({"round": r, "variant": name, "encode_frac": frac, "same_shards": ok}), flush=True)
            if not ok:
                sys.exit(1)
    print(json.dumps({"median": {k: sorted(v)[len(v) // 2] for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
