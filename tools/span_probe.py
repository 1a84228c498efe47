#!/usr/bin/env python3
"""The master's chunk groups packed back to back (4+2 x 1000 B x 4 M groups,
group-major): the line-owner kernel against the span-owner kernel
(RSAMD_GROUP_SPAN, TUNING build), alternating in one process, each output
compared byte for byte with the other's.  Fractions of 8 TB/s of the
algorithmic bytes (encode 6 x 1000 B per group, decode {0,1} / {0,5} the
same), HIP events over 10 calls.
  python tools/span_probe.py [--lib build/ab/tuning/librsamd.so] [--rounds 2]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "build/ab/tuning/librsamd.so"))
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    from rsamd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    import torch
    import rsamd
    import bench
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    k, m, S, B = 4, 2, 1000, 4 << 20
    st = torch.cuda.current_stream()
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout(B, S, S, 6 * S)
    src = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    rdev.fill_synthetic(src.data_ptr(), k, lay, 0x5EED, 0, st)
    bufs = {"line": src.clone(), "span": src.clone()}
    alg = 6 * S * B
    legs = {"encode": None, "dec01": (0, 1), "dec05": (0, 5)}
    for rnd in range(a.rounds):
        for leg, miss in legs.items():
            res = {}
            for name, buf in bufs.items():
                os.environ["RSAMD_GROUP_SPAN"] = "49152" if name == "span" else "0"
                if miss is None:
                    fn = lambda: rdev.encode(rs, buf.data_ptr(), lay, st)  # noqa: E731
                else:
                    pres = [i not in miss for i in range(6)]
                    fn = lambda: rdev.decode(rs, buf.data_ptr(), pres, lay, st)  # noqa: E731
                t = bench.timed(torch, st, fn, 10)
                res[name] = round(alg / t / 8e12, 4)
            same = bool(torch.equal(bufs["line"], bufs["span"]))
            print(json.dumps({"round": rnd, "leg": leg, **res, "same_bytes": same}), flush=True)
    os.environ.pop("RSAMD_GROUP_SPAN", None)


if __name__ == "__main__":
    main()
