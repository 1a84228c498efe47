#!/usr/bin/env python3
"""The CPU side of BASELINE.md's table: the oracle's scalar restatement of the
reference's default coding loop (InputOutputByteTableCodingLoop, -O2
-fno-tree-vectorize; decode = the reference's decodeMissing, two
codeSomeShards passes) timed per config on this host, 1 thread and 16
threads, each on a bounded sample of host-resident stripes (SECONDS per mode).
Prints one JSON line per config."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEED = 0x5EED
CONFIGS = [  # name, k, m, S, erasures (None = encode)
    ("C2 encode", 4, 2, 1 << 20, None),
    ("C3 decode {0}", 4, 2, 1 << 20, (0,)),
    ("C3 decode {0,1}", 4, 2, 1 << 20, (0, 1)),
    ("C3 decode {0,5}", 4, 2, 1 << 20, (0, 5)),
    ("C4 10+4 encode", 10, 4, 4 << 20, None),
    ("C4 10+4 decode {0,1,2,3}", 10, 4, 4 << 20, (0, 1, 2, 3)),
    ("C5 4 KiB encode", 4, 2, 4096, None),
    ("C5 4 KiB decode {0,1}", 4, 2, 4096, (0, 1)),
]


def main():
    import numpy as np
    from oracle import c_ref
    c_ref.build()
    budget = float(os.environ.get("SECONDS", "3"))
    threads = min(16, os.cpu_count() or 1)
    for name, k, m, S, miss in CONFIGS:
        codec = c_ref.Codec(k, m)
        present = None if miss is None else [i not in miss for i in range(k + m)]
        out = {"config": name, "k": k, "m": m, "shard_bytes": S}
        for nthr in (1, threads):
            n = max(nthr * 4, (64 << 20) // ((k + m) * S))  # stripes per call: >= 64 MiB, >= 4 per thread
            host = np.zeros(n * (k + m) * S, dtype=np.uint8)
            for t in range(n):
                host[t * (k + m) * S: t * (k + m) * S + k * S] = c_ref.fill_synthetic(k * S, SEED, t)
            if present is not None:
                codec.code_stripes(host, n, S, S, (k + m) * S, None, nthr)  # parity first, then decode
            done, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < budget:
                codec.code_stripes(host, n, S, S, (k + m) * S, present, nthr)
                done += n
            el = time.perf_counter() - t0
            out[f"GiBps_{nthr}thr"] = round(k * S * done / el / 2**30, 3)
        out["threads"] = threads
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
