#!/usr/bin/env python3
"""Host file API (rs_file_encode / rs_file_decode) per-call rates on a 256 MiB
file, 4+2, pageable numpy and pinned buffers, over direct-kernel block counts
(RSAMD_DIRECT_BLOCKS; TUNING builds read it per call).  Run under
rocprofv3 --kernel-trace to see which kernels served the calls.
  python tools/direct_file_probe.py [--lib L] [--blocks 128,256] [--calls N]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--blocks", default="256")
    ap.add_argument("--rows", default="1", help="RSAMD_DEC_TILED values (direct file decode: 1 LDS-tiled, 0 untiled)")
    a = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    from rsamd import _lib
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    import rsamd
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    k, m = 4, 2
    rs = rsamd.ReedSolomon.create(k, m)
    n = 256 << 20
    _, S = file_layout(rs, n)
    rng = np.random.default_rng(3)
    src = rng.integers(0, 256, n, dtype=np.uint8)
    kinds = {}
    for name, alloc in (("numpy", lambda nb: np.empty(nb, np.uint8)),
                        ("pinned", lambda nb: torch.empty(nb, dtype=torch.uint8, pin_memory=True).numpy())):
        f = alloc(n)
        f[:] = src
        kinds[name] = (f, [alloc(S) for _ in range(k + m)], alloc(n))
    present = [False] + [True] * (k + m - 2) + [False]
    import itertools
    for blocks, rows in itertools.product([int(b) for b in a.blocks.split(",")], a.rows.split(",")):
        os.environ["RSAMD_DIRECT_BLOCKS"] = str(blocks)
        os.environ["RSAMD_DEC_TILED"] = rows
        for name, (f, sh, out) in kinds.items():
            for leg in ("encode", "decode_0_5"):
                def call():
                    if leg == "encode":
                        file_encode_into(rs, f, sh)
                    else:
                        file_decode_into(rs, sh, present, S, out)
                call()
                ts = []
                for _ in range(a.calls):
                    t0 = time.perf_counter()
                    call()
                    ts.append((time.perf_counter() - t0) * 1e3)
                ts.sort()
                ok = bool(np.array_equal(out, f)) if leg != "encode" else True
                print(json.dumps({"blocks": blocks, "rows": rows, "mem": name, "leg": leg, "median_ms": round(ts[len(ts) // 2], 3),
                                  "GiBps": round(n / (ts[len(ts) // 2] * 1e-3) / 2**30, 2), "file_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
