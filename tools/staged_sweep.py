#!/usr/bin/env python3
"""The staged host pipeline on pageable arrays (host.cpp run_chunks with a
pinned mirror; the default for pageable callers since page-locking them is
opt-in): 4+2 x 64 MiB encodeParity and decodeMissing {0,1} per call, one child
process per setting of the TUNING build's knobs (RSAMD_CHUNKS chunks per call,
RSAMD_MIRROR_BYTES pinned mirror per buffer, RSAMD_COPY_THREADS copy-pool
threads), each printing one JSON line.
  python tools/staged_sweep.py [--lib build/ab/tuning/librsamd.so]
                               [--chunks 8 16] [--mirror-mib 24 48] [--threads 8 15]"""
import argparse
import itertools
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    import numpy as np
    import torch  # noqa: F401 -- one HIP runtime (rsamd/_lib.py)
    sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))
    from rsamd import _lib
    _lib.LIB_PATH = os.environ["RSAMD_TEST_LIB"]
    import rsamd
    k, m, n = 4, 2, 64 << 20
    rs = rsamd.ReedSolomon.create(k, m)
    rng = np.random.default_rng(5)
    sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] + [np.zeros(n, np.uint8) for _ in range(m)]
    out = {}
    for name, fn in (("encode", lambda: rs.encodeParity(sh, 0, n)),
                     ("decode01", lambda: rs.decodeMissing(sh, [False, False] + [True] * (k + m - 2), 0, n))):
        for _ in range(3):
            fn()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        out[name + "_GiBps"] = round(k * n / ((time.perf_counter() - t0) / 10) / 2**30, 2)
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "build/ab/tuning/librsamd.so"))
    ap.add_argument("--chunks", nargs="+", type=int, default=[8])
    ap.add_argument("--mirror-mib", nargs="+", type=int, default=[24])
    ap.add_argument("--threads", nargs="+", type=int, default=[15])
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child()
    for c, mm, t in itertools.product(a.chunks, a.mirror_mib, a.threads):
        env = dict(os.environ, RSAMD_TEST_LIB=a.lib, RSAMD_CHUNKS=str(c), RSAMD_MIRROR_BYTES=str(mm << 20),
                   RSAMD_COPY_THREADS=str(t))
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                           text=True, timeout=300)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        res = json.loads(line[-1]) if line else {"error": r.stderr[-400:]}
        print(json.dumps({"chunks": c, "mirror_MiB": mm, "threads": t, **res}), flush=True)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
