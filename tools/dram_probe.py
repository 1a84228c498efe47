#!/usr/bin/env python3
"""Runs build/probes/dram_probe (tools/dram_probe.cpp, CPU only) bound to 16
CPUs of each NUMA node in turn (the job's CPU quota on the GPU box is 16) --
the node's first 16, then 16 spread over its CCDs --
first-touching its buffers there, and prints one JSON line per node plus the
node's memory description from sysfs.  Host DRAM bandwidth under the pageable
host calls' copies (the 8-GPU host-inclusive bound)."""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "probes", "dram_probe")


def cpus(text):
    out = []
    for part in text.strip().split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def main():
    nodes = sorted(glob.glob("/sys/devices/system/node/node[0-9]*"))
    allowed = os.sched_getaffinity(0)
    for nd, spread in [(nd, sp) for nd in nodes for sp in (False, True)]:
        node_cpus = [c for c in cpus(open(os.path.join(nd, "cpulist")).read()) if c in allowed]
        # the node's first 16 CPUs (two 8-core CCDs: each CCD's link to the I/O die
        # caps its bandwidth), or 16 spread over its CCDs (every 4th of its first 64)
        cl = node_cpus[0:64:4][:16] if spread else node_cpus[:16]
        if not cl:
            continue
        spec = ",".join(str(c) for c in cl)
        p = subprocess.run([BIN, spec], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
        line = json.loads(p.stdout.strip().splitlines()[-1])
        try:
            mem = open(os.path.join(nd, "meminfo")).read().split("\n")[0]
        except OSError:
            mem = ""
        line.update(node=os.path.basename(nd), spread_over_ccds=spread, node_meminfo=mem.strip())
        print(json.dumps(line), flush=True)
    # As the bench runs its host legs: bound to ALL of the node's CPUs (the
    # scheduler places the threads within the 16-CPU quota).  (Round 6 also
    # timed a build that pinned the pool's workers round-robin to the node's
    # CCDs: no faster here, and slower host legs; deleted.  profiles/r6/
    # dram_probe_spread_ab_r6j.json, host_legs_pool_spread_ab_r6j.txt.)
    for nd in nodes[-1:]:
        node_cpus = [c for c in cpus(open(os.path.join(nd, "cpulist")).read()) if c in allowed]
        spec = ",".join(str(c) for c in node_cpus)
        p = subprocess.run([BIN, spec, "pool"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=300)
        line = json.loads(p.stdout.strip().splitlines()[-1])
        line.update(node=os.path.basename(nd), all_node_cpus=len(node_cpus))
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    sys.exit(main())
