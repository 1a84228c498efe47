#!/usr/bin/env python3
"""Randomized parity fuzz of the device batch API (rs_encode_batch_dev,
rs_verify_batch_dev, rs_decode_batch_dev, rs_decode_batch_masked_bits_dev)
against the oracle, for a fixed time: random k (1..16) and m (1..4), shard
lengths from 1 byte to 200 KB (multiples of 8, 16, 1000 and odd ones), 1..64
stripes, random pads between shards and stripes, random base offsets (0..255
bytes past an aligned start).  Every byte of the allocation is compared after
each call, so a write into a pad or past the batch is a mismatch too.  Prints
one JSON summary; exits 1 on any mismatch.  Works with the bounds build too
(RSAMD_TEST_LIB; its report is read at the end).
  python tools/device_fuzz.py [--seconds 300] [--seed 1]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    from rsamd import _lib
    if os.environ.get("RSAMD_TEST_LIB"):
        _lib.LIB_PATH = os.path.abspath(os.environ["RSAMD_TEST_LIB"])
    import numpy as np
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    from oracle import c_ref
    rng = np.random.default_rng(a.seed)
    st = torch.cuda.current_stream()
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    bad_count = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    cases = bad = 0
    first_bad = None
    t_end = time.time() + a.seconds
    t_note = time.time() + 30
    while time.time() < t_end:
        if time.time() > t_note:  # a progress line every 30 s (a silent GPU run reads as hung)
            print(json.dumps({"progress_cases": cases, "bad": bad}), flush=True)
            t_note = time.time() + 30
        k = int(rng.integers(1, 17))
        m = int(rng.integers(1, 5))
        T = k + m
        kind = rng.integers(0, 5)
        S = int([rng.integers(1, 4097), rng.integers(1, 25001) * 8, rng.integers(1, 12501) * 16,
                 rng.integers(1, 201) * 1000, rng.integers(1, 200001)][kind])
        B = int(rng.integers(1, 65))
        while B > 1 and B * T * S > (64 << 20):
            B //= 2
        pad = int(rng.choice([0, 0, 8, 16, 256, int(rng.integers(0, 300))]))
        spad = int(rng.choice([0, 0, 8, 4096, int(rng.integers(0, 500))]))
        lay = StripeLayout(B, S, S + pad, T * (S + pad) + spad)
        off = int(rng.choice([0, 0, 8, 16, int(rng.integers(0, 256))]))
        total = off + lay.nbytes + 512
        host = rng.integers(0, 256, total, dtype=np.uint8)
        dev = torch.from_numpy(host).to("cuda:0")
        base = dev.data_ptr() + off
        rs = rsamd.ReedSolomon.create(k, m)
        oc = c_ref.Codec(k, m)
        # encode
        want = host.copy()
        oc.code_stripes(want[off:], B, S, lay.shard_stride, lay.stripe_stride)
        rdev.encode(rs, base, lay, st)
        got = dev.cpu().numpy()
        ok = np.array_equal(got, want)
        # verify: clean, then one flipped parity byte
        flag.zero_()
        rdev.verify(rs, base, lay, flag.data_ptr(), st)
        torch.cuda.synchronize()
        ok = ok and int(flag.item()) == 0
        t = int(rng.integers(0, B))
        p = int(rng.integers(k, T))
        c = int(rng.integers(0, S))
        pos = off + t * lay.stripe_stride + p * lay.shard_stride + c
        dev[pos] ^= 0x21
        flag.zero_()
        rdev.verify(rs, base, lay, flag.data_ptr(), st)
        torch.cuda.synchronize()
        ok = ok and int(flag.item()) != 0
        dev[pos] ^= 0x21
        # uniform decode: erase up to m shards in every stripe, rebuild
        e = int(rng.integers(1, m + 1))
        miss = sorted(int(x) for x in rng.choice(T, e, replace=False))
        erased = want.copy()
        for tt in range(B):
            for j in miss:
                s0 = off + tt * lay.stripe_stride + j * lay.shard_stride
                erased[s0:s0 + S] = 0x5A
        dev.copy_(torch.from_numpy(erased))
        rdev.decode(rs, base, [i not in miss for i in range(T)], lay, st)
        ok = ok and np.array_equal(dev.cpu().numpy(), want)
        # per-stripe bitmasks: a random pattern per stripe, some undecodable
        pres = np.ones((B, T), dtype=bool)
        n_undec = 0
        erased = want.copy()
        for tt in range(B):
            e = int(rng.integers(0, m + 2))  # m + 1: undecodable
            ms = rng.choice(T, min(e, T), replace=False)
            pres[tt, ms] = False
            if (~pres[tt]).sum() > m:
                n_undec += 1
            for j in ms:
                s0 = off + tt * lay.stripe_stride + int(j) * lay.shard_stride
                erased[s0:s0 + S] = 0xA7
        expect = erased.copy()
        for tt in range(B):
            if (~pres[tt]).sum() <= m:  # decodable: back to the encoded bytes
                s0 = off + tt * lay.stripe_stride
                for j in range(T):
                    expect[s0 + j * lay.shard_stride:s0 + j * lay.shard_stride + S] = \
                        want[s0 + j * lay.shard_stride:s0 + j * lay.shard_stride + S]
        dev.copy_(torch.from_numpy(erased))
        bits = torch.from_numpy(rdev.presence_bits(pres).view(np.int32)).to("cuda:0")
        bad_count.zero_()
        rdev.decode_masked_bits(rs, base, bits.data_ptr(), lay, bad_count.data_ptr(), st)
        torch.cuda.synchronize()
        ok = ok and np.array_equal(dev.cpu().numpy(), expect) and int(bad_count.item()) == n_undec
        cases += 1
        if not ok:
            bad += 1
            if first_bad is None:
                first_bad = {"k": k, "m": m, "S": S, "B": B, "pad": pad, "spad": spad, "off": off}
    oob = None
    lib = _lib.load()
    if hasattr(lib, "rs_bounds_report"):
        import ctypes as C
        n, addr, ln, where = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint32()
        lib.rs_bounds_report(C.byref(n), C.byref(addr), C.byref(ln), C.byref(where))
        oob = n.value
    print(json.dumps({"seconds": a.seconds, "seed": a.seed, "cases": cases, "bad": bad, "first_bad": first_bad,
                      "bounds_violations": oob}), flush=True)
    return 1 if bad or oob else 0


if __name__ == "__main__":
    sys.exit(main())
