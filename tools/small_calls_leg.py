#!/usr/bin/env python3
"""bench.py's small-call leg alone (host_small_calls: 1000-B decode, 4 KiB
encode, the 90,999-B fixture file's encode / decode {0,5}, from C through the
mock JNIEnv's timing loops), bound to the GPU's NUMA node as the bench binds
it; prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import torch
    import rsamd
    from rsamd import parallel
    import bench
    torch.cuda.init()
    extra = {}
    with bench.gpu_numa_bound(torch, parallel, extra):
        out = bench.host_small_calls(rsamd, 4, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
