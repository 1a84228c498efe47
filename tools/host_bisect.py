#!/usr/bin/env python3
"""Why the bench's host-inclusive legs read 34 GiB/s while tools/host_trace.py
reads 44 on the same box: bench.py's host legs (host_link + host_inclusive)
in a fresh process, then after the CPU baseline, then after cpu_configs, with
the CPU the main thread runs on and the GPU's NUMA node printed each time.
  python tools/host_bisect.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def where():
    f = open("/proc/self/stat").read().rsplit(")", 1)[1].split()
    return int(f[36])  # field 39: the CPU last run on


def numa_of_cpu(cpu):
    base = "/sys/devices/system/node"
    for d in os.listdir(base):
        if d.startswith("node") and os.path.exists(f"{base}/{d}/cpu{cpu}"):
            return int(d[4:])
    return None


def main():
    import torch
    import bench
    import rsamd
    torch.cuda.init()
    pci = bench.pci_address(torch)
    gnode = None
    for d in os.listdir("/sys/bus/pci/devices"):
        if pci and d.startswith(pci):
            try:
                gnode = int(open(f"/sys/bus/pci/devices/{d}/numa_node").read())
            except OSError:
                pass
    print(json.dumps({"gpu_pci": pci, "gpu_numa_node": gnode, "affinity": sorted(os.sched_getaffinity(0))}),
          flush=True)

    def host(tag):
        cpu = where()
        link = bench.host_link(torch)
        out = bench.host_inclusive(rsamd, 4, 2, link)
        print(json.dumps({"stage": tag, "cpu": cpu, "cpu_node": numa_of_cpu(cpu), "link": link,
                          **{k: v for k, v in out.items() if "frac" in k or k.endswith("GiBps")}}), flush=True)

    host("fresh")
    host("fresh again")
    bench.cpu_baseline(4, 2, 1 << 20, 8.0)
    host("after cpu_baseline")
    bench.cpu_configs()
    host("after cpu_configs")


if __name__ == "__main__":
    main()
