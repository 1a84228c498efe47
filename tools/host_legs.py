#!/usr/bin/env python3
"""The bench's host-inclusive legs (bench.py host_inclusive: 4+2 x 64 MiB
encodeParity / decodeMissing {0,1} per call, a 256 MiB file through
ReedSolomonEncoder / ReedSolomonDecoder {0,5}, pageable and pinned) next to
the link bound measured in the same process, bound to the GPU's NUMA node as
the bench binds them.  One child process per variant of the TUNING build's
knobs; each prints one JSON line.  The pageable encode is checked against the
oracle.  --trace writes the mirrored pipeline's per-chunk timeline
(RSAMD_TRACE, TUNING build) of the pageable encode calls to the given file.
  python tools/host_legs.py [--lib build/ab/tuning/librsamd.so]
                            [--var RSAMD_MIRROR_BYTES=16777216,RSAMD_COPY_NT=0 ...] [--trace FILE] [--small]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(trace):
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
    extra = {}
    out = {}
    with bench.gpu_numa_bound(torch, parallel, extra):
        link = bench.host_link(torch)
        out.update(bench.host_inclusive(rsamd, 4, 2, link))
        if os.environ.get("HOST_LEGS_SMALL"):  # the bench's next legs: small calls after the large ones
            out.update(bench.config0_single_stripe(rsamd, 4, 2))
            out.update(bench.host_by_size(rsamd, 4, 2))
        # the pageable encode against the oracle (and, traced, a timeline of it)
        k, m, n = 4, 2, 64 << 20
        rng = np.random.default_rng(9)
        sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] + [np.zeros(n, np.uint8) for _ in range(m)]
        rs = rsamd.ReedSolomon.create(k, m)
        if trace:
            os.environ["RSAMD_TRACE"] = trace
        for _ in range(3):
            rs.encodeParity(sh, 0, n)
        from rsamd.layout import file_encode_into, file_layout
        data = rng.integers(0, 256, k * n, dtype=np.uint8)
        _, S = file_layout(rs, len(data))
        fsh = [np.zeros(S, np.uint8) for _ in range(k + m)]
        for _ in range(2):
            file_encode_into(rs, data, fsh)
        os.environ.pop("RSAMD_TRACE", None)
        fref = c_ref.Codec(k, m).file_encode(data.tobytes(), 1000)
        out["pageable_file_encode_vs_oracle"] = bool(np.array_equal(np.stack(fsh), fref))
        ref = [a.copy() for a in sh[:k]] + [np.zeros(n, np.uint8) for _ in range(m)]
        c_ref.Codec(k, m).encode_parity(ref, 0, n)
        out["pageable_encode_vs_oracle"] = (all(np.array_equal(a, b) for a, b in zip(sh, ref))
                                            if not os.environ.get("RSAMD_MIRROR_NOCOPY") else "skipped (NOCOPY)")
    out["numa"] = extra.get("host_legs_numa")
    out["link"] = link
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "build/ab/tuning/librsamd.so"))
    ap.add_argument("--var", nargs="*", default=[""], help="comma-separated NAME=VALUE settings, one child each")
    ap.add_argument("--trace", default="")
    ap.add_argument("--small", action="store_true", help="then the bench's small-call legs (configs[0], by size)")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a.trace)
    for var in a.var:
        env = dict(os.environ, RSAMD_TEST_LIB=a.lib)
        if a.small:
            env["HOST_LEGS_SMALL"] = "1"
        for kv in filter(None, var.split(",")):
            key, val = kv.split("=", 1)
            env[key] = val
        cmd = [sys.executable, os.path.abspath(__file__), "--child"] + (["--trace", a.trace] if a.trace else [])
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        res = json.loads(line[-1]) if line else {"error": r.stderr[-600:]}
        print(json.dumps({"var": var, "lib": os.path.relpath(a.lib, ROOT), **res}), flush=True)
        if r.returncode:
            return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
