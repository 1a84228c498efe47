#!/usr/bin/env python3
"""The round-6 host legs alone (bench.py's host_small_calls, host_groups_leg,
host_jni_legs), bound to the GPU's NUMA node after measuring the link, one
JSON line: a quick check of those legs without the whole bench."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import torch
    import bench
    import rsamd
    from rsamd import parallel
    torch.cuda.init()
    extra = {}
    with bench.gpu_numa_bound(torch, parallel, extra):
        link = bench.host_link(torch)
        extra.update(bench.host_small_calls(rsamd, 4, 2))
        extra.update(bench.host_groups_leg(rsamd, 4, 2, link))
        extra.update(bench.host_jni_legs(rsamd, 4, 2, link))
        small = bench.host_jni_legs(rsamd, 4, 2, link, huge=0)  # the same on 4 KiB pages
        extra.update({k.replace("host_jni_", "host_jni4k_"): v for k, v in small.items()})
        if "--inclusive" in sys.argv:
            extra.update(bench.host_inclusive(rsamd, 4, 2, link))
    extra["host_link"] = link
    print(json.dumps(extra), flush=True)


if __name__ == "__main__":
    main()
