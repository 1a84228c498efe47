#!/usr/bin/env python3
"""Host file encode with page-locking opted in (capi.cpp file_encode_interior:
the block rows inside whole pages coded in place, the rows either side
staged) over many placements of the file and shards within their pages:
every mismatch against the oracle is printed with each array's address
modulo 4096 and the bad byte ranges.
  python tools/file_interior_probe.py [--k 3 --m 2 --block 520 --n 2614744 --trials 40]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--m", type=int, default=2)
    ap.add_argument("--block", type=int, default=520)
    ap.add_argument("--n", type=int, default=2614744)
    ap.add_argument("--trials", type=int, default=40)
    ap.add_argument("--register", type=int, default=1)
    a = ap.parse_args()
    import torch  # noqa: F401
    import rsamd
    from rsamd import _lib
    from rsamd.layout import file_encode_into, file_layout
    from oracle import c_ref
    c_ref.build()
    _lib.load().rs_set_host_register(a.register)
    k, m, blk, n = a.k, a.m, a.block, a.n
    rs = rsamd.ReedSolomon.create(k, m)
    oc = c_ref.Codec(k, m)
    _, S = file_layout(rs, n, blk)
    rng = np.random.default_rng(1)
    bad_trials = 0
    for t in range(a.trials):
        def view(size):
            raw = np.empty(size + 8192, np.uint8)
            o = (-raw.ctypes.data) % 4096 + int(rng.integers(0, 512)) * 8
            return raw[o:o + size]
        f = view(n)
        f[:] = rng.integers(0, 256, n, dtype=np.uint8)
        sh = [view(S) for _ in range(k + m)]
        for x in sh:
            x[:] = 0xEE
        file_encode_into(rs, f, sh, blk)
        ref = oc.file_encode(f.tobytes(), blk)
        rec = {"trial": t, "file_mod": f.ctypes.data % 4096, "shard_mod": [x.ctypes.data % 4096 for x in sh]}
        bad = []
        for i in range(k + m):
            d = np.flatnonzero(sh[i] != ref[i])
            if len(d):
                bad.append({"shard": i, "count": int(len(d)), "first": int(d[0]), "last": int(d[-1]),
                            "first_row": int(d[0]) // blk, "last_row": int(d[-1]) // blk,
                            "got": int(sh[i][d[0]]), "want": int(ref[i][d[0]])})
        if bad:
            bad_trials += 1
            rec["bad"] = bad
            print(json.dumps(rec), flush=True)
    print(json.dumps({"trials": a.trials, "bad_trials": bad_trials, "S": S, "rows": S // blk}))
    _lib.load().rs_set_host_register(0)


if __name__ == "__main__":
    main()
