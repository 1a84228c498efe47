#!/usr/bin/env python3
"""Pageable host calls by size: 4+2 encodeParity per call at 16 KiB .. 64 MiB
per shard, and the client's file calls (encode, decode {0,5}) on 1 .. 64 MiB
files (the DFS client's files are split into shards of a quarter of the
file, so mid sizes are the common case), GiB/s of data shards and us per
call, bound to the GPU's NUMA node as bench.py binds its host legs.  One child
process per TUNING variant; each prints one JSON line.
  python tools/host_sizes.py [--lib build/ab/tuning/librsamd.so] [--var RSAMD_MIRROR_MIN=1048576 ...]
  (HS_CODE=10,4 in the environment: another code than 4+2)"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILE_SIZES = [90_999, 256 << 10, 1 << 20, 3 << 20, 4 << 20, 16 << 20, 64 << 20]
SIZES = [16 << 10, 32 << 10, 64 << 10, 128 << 10, 192 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20, 16 << 20, 64 << 20]


def child():
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))
    from rsamd import _lib
    if os.environ.get("RSAMD_TEST_LIB"):
        _lib.LIB_PATH = os.path.abspath(os.environ["RSAMD_TEST_LIB"])
    import rsamd
    from rsamd import parallel
    import bench
    from oracle import c_ref
    torch.cuda.init()
    k, m = (int(x) for x in os.environ.get("HS_CODE", "4,2").split(","))
    rs = rsamd.ReedSolomon.create(k, m)
    out, extra = {}, {}
    with bench.gpu_numa_bound(torch, parallel, extra):
        for S in SIZES:
            rng = np.random.default_rng(S)
            sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
            reps = max(5, min(200, (256 << 20) // (k * S)))
            for _ in range(3):
                rs.encodeParity(sh, 0, S)
            t0 = time.perf_counter()
            for _ in range(reps):
                rs.encodeParity(sh, 0, S)
            t = (time.perf_counter() - t0) / reps
            ref = [a.copy() for a in sh[:k]] + [np.zeros(S, np.uint8) for _ in range(m)]
            c_ref.Codec(k, m).encode_parity(ref, 0, S)
            assert all(np.array_equal(a, b) for a, b in zip(sh, ref)), S
            out[f"{S >> 10}K"] = {"us": round(t * 1e6, 1), "GiBps": round(k * S / t / 2**30, 2)}
        # the client's file calls (1000-byte blocks): encode, then decode {0, 5}
        from rsamd.layout import file_decode_into, file_encode_into, file_layout
        for F in FILE_SIZES:
            rng = np.random.default_rng(F)
            data = rng.integers(0, 256, F, dtype=np.uint8)
            _, S = file_layout(rs, F)
            fsh = [np.zeros(S, np.uint8) for _ in range(k + m)]
            fout = np.zeros(F, np.uint8)
            reps = max(5, min(100, (256 << 20) // F))
            pres = [i not in (0, 5) for i in range(k + m)]
            row = {}
            for name, fn in (("enc", lambda: file_encode_into(rs, data, fsh)),
                             ("dec05", lambda: file_decode_into(rs, fsh, pres, S, fout))):
                for _ in range(3):
                    fn()
                t0 = time.perf_counter()
                for _ in range(reps):
                    fn()
                t = (time.perf_counter() - t0) / reps
                row[name] = {"us": round(t * 1e6, 1), "GiBps": round(F / t / 2**30, 2)}
            ref = c_ref.Codec(k, m).file_encode(data.tobytes(), 1000)
            assert np.array_equal(np.stack(fsh), ref) and np.array_equal(fout, data), F
            out[f"file_{F >> 10}K"] = row
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "build/ab/tuning/librsamd.so"))
    ap.add_argument("--var", nargs="*", default=[""])
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child()
    for var in a.var:
        env = dict(os.environ, RSAMD_TEST_LIB=a.lib)
        for kv in filter(None, var.split(",")):
            key, val = kv.split("=", 1)
            env[key] = val
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                           text=True, timeout=400)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        res = json.loads(line[-1]) if line else {"error": r.stderr[-600:]}
        print(json.dumps({"var": var, **res}), flush=True)
        if r.returncode:
            return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
