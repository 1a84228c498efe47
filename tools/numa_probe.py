#!/usr/bin/env python3
"""Where the process runs against where the GPU's PCIe root is: the GPU's
NUMA node (sysfs of its PCI address), the CPUs this process may use, and the
host-inclusive legs (bench.host_inclusive) with the process left where the
scheduler put it, then bound to the GPU's node (its CPUs that the process may
use; host arrays are allocated after the bind, so first touch places them there).
  python tools/numa_probe.py [--bind]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpulist(text):
    out = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bind", action="store_true")
    a = ap.parse_args()
    import bench  # puts the package on sys.path
    import torch
    torch.cuda.init()
    import rsamd
    from rsamd import parallel
    ident = parallel.device_identity(torch)
    info = {"pci": ident["pci"], "allowed_cpus": len(os.sched_getaffinity(0))}
    node = None
    if ident["pci"]:
        dom, bus, dev = ident["pci"].split(":")
        for fn in range(8):
            p = f"/sys/bus/pci/devices/{dom}:{bus}:{dev}.{fn}/numa_node"
            if os.path.exists(p):
                node = int(open(p).read())
                break
    info["gpu_numa_node"] = node
    nodes = {}
    for d in sorted(os.listdir("/sys/devices/system/node")) if os.path.isdir("/sys/devices/system/node") else []:
        if d.startswith("node"):
            nodes[int(d[4:])] = cpulist(open(f"/sys/devices/system/node/{d}/cpulist").read())
    allowed = os.sched_getaffinity(0)
    info["allowed_by_node"] = {n: len(c & allowed) for n, c in nodes.items()}
    info["running_on_cpu"] = os.sched_getcpu() if hasattr(os, "sched_getcpu") else None
    if a.bind and node is not None and node >= 0 and nodes.get(node, set()) & allowed:
        os.sched_setaffinity(0, nodes[node] & allowed)
        info["bound_to_node"] = node
        info["bound_cpus"] = len(nodes[node] & allowed)
    out = bench.host_inclusive(rsamd, 4, 2)
    out.pop("host_inclusive_note", None)
    info.update({k.replace("host_inclusive_", ""): v for k, v in out.items() if k.endswith("GiBps")})
    print(json.dumps(info), flush=True)


if __name__ == "__main__":
    main()
