#!/usr/bin/env python3
"""Randomized parity fuzz of the two stripe layouts beside the packed batch,
against the oracle, for a fixed time:
  granule   -- rs_granule_copy_shard in, rs_encode_batch_dev over the granule
               view, per-stripe bitmask decodes (rs_decode_granule_masked_bits_dev,
               some stripes undecodable), rs_granule_copy_shard out; random
               k (1..12), m (1..4), granules of 16 B .. 64 KiB dividing or
               divided by the shard length;
  shard     -- the master's layout ([server][group * chunk], random server
               pads): rs_decode_groups_shard_major_dev with offline sets that
               grow mid-loop, clean runs and random per-group patterns; random
               k / m, chunks of 8 B .. 4 KiB (odd ones too), 1 .. 30,000 groups.
Every result byte for byte against the oracle, pads and canaries included.
Progress every 30 s; one JSON summary; exits 1 on any mismatch.  RSAMD_TEST_LIB
selects another build (the bounds build's report is read at the end).
  python tools/layout_fuzz.py [--seconds 180] [--seed 1]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def granule_case(rng, np, torch, rsamd, rdev, c_ref, st):
    k = int(rng.integers(1, 13))
    m = int(rng.integers(1, 5))
    T = k + m
    G = int(rng.choice([16, 64, 256, 1024, 4096, 16384, 65536]))
    if rng.random() < 0.5:
        S = G * int(rng.integers(1, 9))          # a stripe spans several rows
        n = int(rng.integers(1, 40))
    else:
        S = max(16, G // int(rng.choice([1, 2, 4, 8, 16])))  # a row holds several stripes
        S = S if G % S == 0 else G
        per = G // S
        n = per * int(rng.integers(1, 40))
    while n * T * S > (48 << 20) and n > 1:
        n = max(1, n // 2)
        if G > S:
            n = max(G // S, n // (G // S) * (G // S))
    lay = rdev.GranuleLayout.make(n, T, S, G)
    rs = rsamd.ReedSolomon.create(k, m)
    oc = c_ref.Codec(k, m)
    pool = torch.from_numpy(rng.integers(0, 256, lay.nbytes, dtype=np.uint8)).to("cuda:0")
    data = rng.integers(0, 256, (n, T, S), dtype=np.uint8)
    for t in range(n):
        for s in range(k):
            rdev.copy_shard(lay, pool.data_ptr(), t, s, data[t, s].ctypes.data, True, st)
    torch.cuda.synchronize()
    rdev.encode(rs, pool.data_ptr(), lay, st)
    want = data.copy()
    oc.code_stripes(want.reshape(-1), n, S, S, T * S)  # packed host copy: [stripe][shard][S]
    pres = np.ones((n, T), dtype=bool)
    undec = 0
    for t in range(n):
        e = int(rng.integers(0, m + 2))
        miss = rng.choice(T, min(e, T), replace=False)
        pres[t, miss] = False
        undec += int((~pres[t]).sum() > m)
    # erase through the layout: zero buffers copied over the absent shards
    zero = np.full(S, 0x66, np.uint8)
    for t in range(n):
        for s in np.nonzero(~pres[t])[0]:
            rdev.copy_shard(lay, pool.data_ptr(), t, int(s), zero.ctypes.data, True, st)
    bits = torch.from_numpy(rdev.presence_bits(pres).view(np.int32)).to("cuda:0")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    rdev.decode_masked_bits(rs, pool.data_ptr(), bits.data_ptr(), lay, bad.data_ptr(), st)
    torch.cuda.synchronize()
    ok = int(bad.item()) == undec
    out = np.empty(S, np.uint8)
    for t in range(n):
        dec = (~pres[t]).sum() <= m
        for s in range(T):
            rdev.copy_shard(lay, pool.data_ptr(), t, s, out.ctypes.data, False, st)
            torch.cuda.synchronize()
            exp = want[t, s] if (dec or pres[t, s]) else zero
            if not np.array_equal(out, exp):
                ok = False
    return ok, {"k": k, "m": m, "G": G, "S": S, "n": n}


def shard_case(rng, np, torch, rsamd, recovery, c_ref, st):
    k, m = [(4, 2), (4, 2), (10, 4), (3, 3), (6, 1), (2, 2)][int(rng.integers(0, 6))]
    T = k + m
    L = int(rng.choice([1000, 1000, 8, 24, 999, 1024, 4096, int(rng.integers(1, 4097))]))
    n = int(rng.integers(1, 30001))
    while n * L * T > (96 << 20):
        n //= 2
    pad = int(rng.choice([0, 0, 8, 4096, int(rng.integers(0, 300))]))
    stride = n * L + pad
    oc = c_ref.Codec(k, m)
    data = np.zeros((T, stride), np.uint8)
    data[:, n * L:] = 0xC5  # pads
    rows = [rng.integers(0, 256, n * L, dtype=np.uint8) for _ in range(k)] + [np.zeros(n * L, np.uint8) for _ in range(m)]
    oc.encode_parity(rows, 0, n * L)
    for i in range(T):
        data[i, :n * L] = rows[i]
    want = data.copy()
    kind = int(rng.integers(0, 3))
    pres = np.ones((n, T), dtype=bool)
    if kind == 0:  # one offline set, grown at a random group
        off0 = rng.choice(T, int(rng.integers(1, m + 1)), replace=False)
        pres[:, off0] = False
        if (~pres[0]).sum() < m and n > 1:
            g = int(rng.integers(1, n))
            more = [s for s in range(T) if pres[0, s]]
            pres[g:, int(rng.choice(more))] = False
    elif kind == 1:  # clean, then a failure
        g = int(rng.integers(0, n))
        pres[g:, rng.choice(T, int(rng.integers(1, m + 1)), replace=False)] = False
    else:  # a random pattern per group (<= m absent)
        for g in range(n):
            e = int(rng.integers(0, m + 1))
            if e:
                pres[g, rng.choice(T, e, replace=False)] = False
    erased = want.copy()
    for s in range(T):
        for g in np.nonzero(~pres[:, s])[0]:
            erased[s, g * L:(g + 1) * L] = 0x3A
    dev = torch.from_numpy(erased.reshape(-1).copy()).to("cuda:0")
    recovery.recover_groups_shard_major_dev(dev.data_ptr(), stride, pres, L, st, data_shards=k, parity_shards=m)
    torch.cuda.synchronize()
    ok = np.array_equal(dev.cpu().numpy().reshape(T, stride), want)
    return ok, {"k": k, "m": m, "L": L, "n": n, "pad": pad, "kind": kind}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    from rsamd import _lib
    if os.environ.get("RSAMD_TEST_LIB"):
        _lib.LIB_PATH = os.path.abspath(os.environ["RSAMD_TEST_LIB"])
    import numpy as np
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd import recovery
    from oracle import c_ref
    rng = np.random.default_rng(a.seed)
    st = torch.cuda.current_stream()
    counts = {"granule": [0, 0], "shard": [0, 0]}
    first_bad = None
    t_end, t_note = time.time() + a.seconds, time.time() + 30
    while time.time() < t_end:
        if time.time() > t_note:
            print(json.dumps({"progress": counts}), flush=True)
            t_note = time.time() + 30
        if rng.random() < 0.5:
            name, (ok, desc) = "granule", granule_case(rng, np, torch, rsamd, rdev, c_ref, st)
        else:
            name, (ok, desc) = "shard", shard_case(rng, np, torch, rsamd, recovery, c_ref, st)
        counts[name][0] += 1
        if not ok:
            counts[name][1] += 1
            if first_bad is None:
                first_bad = {"layout": name, **desc}
    oob = None
    lib = _lib.load()
    if hasattr(lib, "rs_bounds_report"):
        import ctypes as C
        nn, addr, ln, where = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint32()
        lib.rs_bounds_report(C.byref(nn), C.byref(addr), C.byref(ln), C.byref(where))
        oob = nn.value
    bad = counts["granule"][1] + counts["shard"][1]
    print(json.dumps({"seconds": a.seconds, "seed": a.seed, "cases": counts, "bad": bad, "first_bad": first_bad,
                      "bounds_violations": oob}), flush=True)
    return 1 if bad or oob else 0


if __name__ == "__main__":
    sys.exit(main())
