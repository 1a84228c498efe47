#!/usr/bin/env python3
"""rs_file_encode / rs_file_decode on a 256 MiB pageable host file, a few
calls (for rocprofv3 --memory-copy-trace --kernel-trace: how busy are the two
copy directions?)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import numpy as np
    import torch  # noqa: F401
    import rsamd
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    rs = rsamd.ReedSolomon.create(4, 2)
    data = np.random.default_rng(1).integers(0, 256, 256 << 20, dtype=np.uint8)
    _, S = file_layout(rs, len(data))
    sh = [np.zeros(S, np.uint8) for _ in range(6)]
    out = np.empty(len(data), np.uint8)
    present = [False, True, True, True, True, False]
    for name, fn in (("file_encode", lambda: file_encode_into(rs, data, sh)),
                     ("file_decode_0_5", lambda: file_decode_into(rs, sh, present, S, out))):
        fn()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        print(name, "GiB/s", round(3 * len(data) / (time.perf_counter() - t0) / 2**30, 2), flush=True)
    assert np.array_equal(out, data)


if __name__ == "__main__":
    main()
