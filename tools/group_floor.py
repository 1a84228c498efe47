#!/usr/bin/env python3
"""The traffic floor of the master's chunk groups in their group-major layout
([group][6][1000], stride 1000: ChunkserverDiskRecoveryMachine.java:22-48)
when HBM is read and written in whole 128-byte lines.

Every byte of a group is an input (one of the first k present shards), an
output (an absent shard) or unused (a present shard beyond the first k).  A
line must be READ when it holds an input byte, or output bytes next to bytes
that must survive the whole-line write; a line is WRITTEN when it holds an
output byte.  A line holding both an input and an output byte therefore
costs two line transfers for one line of content: at 1000-byte shards every
run of inputs or outputs starts and ends mid-line.  The floor below assumes
the best possible ownership (a neighbouring group's bytes in a shared line
cost nothing extra), so no whole-line kernel can move fewer bytes; only
partial-line writes can, and HBM serves those as read-modify-writes (DESIGN.md
3.4: 2.7-3 % fewer bytes, 1-5 points slower).

Workloads as tools/pmc_workloads.py builds them (4 M groups; 64 000 sampled,
the ratio is per group): encode, uniform decodes, and the per-group bitmask
leg (one of the 22 patterns of <= 2 erasures per group, numpy seed 0).
  python tools/group_floor.py
"""
import itertools

import numpy as np

S, T, LINE = 1000, 6, 128


def floor_traffic(patterns):
    """(algorithmic bytes, whole-line read bytes, whole-line write bytes) of
    groups packed back to back from a 128-byte-aligned base."""
    n = len(patterns)
    role = np.zeros(n * T * S, np.int8)  # 0 unused, 1 input, 2 output
    alg = 0
    for g, p in enumerate(patterns):
        miss = [i for i in range(T) if not p[i]]
        if not miss:
            continue
        for i in [i for i in range(T) if p[i]][:4]:
            role[(g * T + i) * S:(g * T + i + 1) * S] = 1
        for i in miss:
            role[(g * T + i) * S:(g * T + i + 1) * S] = 2
        alg += (4 + len(miss)) * S
    r = role.reshape(-1, LINE)
    has_in, has_out, keep = (r == 1).any(1), (r == 2).any(1), (r != 2).any(1)
    return alg, int((has_in | (has_out & keep)).sum()) * LINE, int(has_out.sum()) * LINE


def main():
    g = 64000
    pats = np.array([[i not in miss for i in range(T)] for e in range(3)
                     for miss in itertools.combinations(range(T), e)], bool)
    cases = [("encode", np.tile([1, 1, 1, 1, 0, 0], (g, 1))), ("decode {0,1}", np.tile([0, 0, 1, 1, 1, 1], (g, 1))),
             ("decode {0,5}", np.tile([0, 1, 1, 1, 1, 0], (g, 1))), ("decode {0}", np.tile([0, 1, 1, 1, 1, 1], (g, 1))),
             ("per-group bitmasks", pats[np.random.default_rng(0).integers(0, len(pats), g)])]
    for name, p in cases:
        alg, rd, wr = floor_traffic(p.astype(bool))
        print(f"{name:20s} algorithmic {alg / g:7.1f} B/group  whole-line floor: read {rd / g:7.1f} "
              f"write {wr / g:7.1f}  ratio {(rd + wr) / alg:.4f}")


if __name__ == "__main__":
    main()
