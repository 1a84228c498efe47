#!/usr/bin/env python3
"""Per-call latency of the JNI-facing host API for small stripes
(encodeParity / decodeMissing of one 4+2 stripe from host buffers), the
regime of the master's 6 x 1000-B recovery calls and small files.  Prints one
JSON line; RSAMD_ZC_BYTES=0 disables the zero-copy small-call path (A/B)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch  # noqa: F401  (HIP runtime first, as rsamd._lib does)
    import rsamd
    from oracle import c_ref
    k, m = 4, 2
    rs = rsamd.ReedSolomon.create(k, m)
    oc = c_ref.Codec(k, m)
    out = {"zc_bytes": os.environ.get("RSAMD_ZC_BYTES", "default")}
    sizes = [int(x) for x in os.environ.get("SIZES", "1000 4096 65536 174080 1048576").split()]
    for S in sizes:
        rng = np.random.default_rng(S)
        sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        ref = [a.copy() for a in sh]
        oc.encode_parity(ref, 0, S)
        reps = 300 if S <= 65536 else 60

        def t_us(fn):
            fn()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            return round((time.perf_counter() - t0) / reps * 1e6, 1)

        out[f"encode_{S}_us"] = t_us(lambda: rs.encodeParity(sh, 0, S))
        assert all(np.array_equal(a, b) for a, b in zip(sh, ref)), S
        present = [True] * (k + m)
        present[0] = present[5] = False

        def dec():
            sh[0][:] = 0
            sh[5][:] = 0
            rs.decodeMissing(sh, present, 0, S)

        out[f"decode_0_5_{S}_us"] = t_us(dec)
        assert all(np.array_equal(a, b) for a, b in zip(sh, ref)), S
        out[f"cpu_port_encode_{S}_us"] = t_us(lambda: oc.encode_parity(ref, 0, S))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
