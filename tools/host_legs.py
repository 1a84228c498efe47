#!/usr/bin/env python3
"""bench.py's host-inclusive legs alone (4+2, 64 MiB shards; 256 MiB file),
as one JSON line -- for A/B runs of the host pipeline's knobs
(RSAMD_PIPE_STREAMS, RSAMD_CHUNKS, RSAMD_HOST_REGISTER) or of a variant build
(--lib path/to/librsamd.so)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench  # puts the package on sys.path
    import torch
    torch.cuda.init()
    lib = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else None
    if lib:
        from rsamd import _lib
        _lib.LIB_PATH = os.path.abspath(lib)
    import rsamd
    out = bench.host_inclusive(rsamd, 4, 2)
    out.pop("host_inclusive_note", None)
    out = {k.replace("host_inclusive_", ""): v for k, v in out.items() if k.endswith("GiBps")}
    print(json.dumps({"lib": lib or "in-tree", **out}), flush=True)


if __name__ == "__main__":
    main()
