#!/usr/bin/env python3
"""Host-inclusive rate of the JNI marshalling (jni/rs_jni_core.c over
librsamd, through the mock JNI of tests/test_jni_core.py) against a direct
rs_encode_parity call on the same host arrays: 4+2, n MiB per shard.
Usage: python tools/jni_rate_probe.py [MiB ...]"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import numpy as np
    from test_jni_core import Jvm, build_mock

    import rsamd
    from rsamd import _lib
    native = _lib.load()
    jvm = Jvm(build_mock())
    h = C.c_void_p()
    assert native.rs_codec_create(4, 2, C.byref(h)) == 0
    rs = rsamd.ReedSolomon.create(4, 2)
    for mib in [int(a) for a in sys.argv[1:]] or [1, 4, 16, 64]:
        n = mib << 20
        rng = np.random.default_rng(mib)
        data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(4)] + [np.zeros(n, np.uint8)] * 2
        arrs = jvm.objects([jvm.bytes(d) for d in data])
        sh = [d.copy() for d in data]

        def rate(fn, reps=4):
            fn()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            return round(4 * n / ((time.perf_counter() - t0) / reps) / 2**30, 2)
        out = {"MiB_per_shard": mib,
               "jni_core_GiBps": rate(lambda: jvm.lib.mock_encode_parity(1, h, arrs, 0, n)),
               "direct_GiBps": rate(lambda: rs.encodeParity(sh, 0, n))}
        assert jvm.exception() == ("", ""), jvm.exception()
        print(json.dumps(out), flush=True)
    native.rs_codec_destroy(h)


if __name__ == "__main__":
    main()
