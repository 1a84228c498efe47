#!/usr/bin/env python3
"""Randomized parity fuzz of the device file calls (rs_file_encode_dev /
rs_file_decode_dev: the fused k = 4 kernels and the generic split / merge
paths) against the oracle, for a fixed time: random k (1..10), m (0..4),
blocks (1 B to 8 KiB, the DFS's 1000 often), files from 1 byte to 6 MB,
shard strides with random pads, random file offsets, random erasures
(write_missing on and off).  Every byte of the shard and file allocations is
compared, pads included.  Progress every 30 s; one JSON summary; exits 1 on
any mismatch.  RSAMD_TEST_LIB selects another build (the bounds build's
report is read at the end).
  python tools/file_fuzz.py [--seconds 180] [--seed 1]"""
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
    ap.add_argument("--seconds", type=float, default=180)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    from rsamd import _lib
    if os.environ.get("RSAMD_TEST_LIB"):
        _lib.LIB_PATH = os.path.abspath(os.environ["RSAMD_TEST_LIB"])
    import numpy as np
    import torch
    import rsamd
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    from oracle import c_ref
    rng = np.random.default_rng(a.seed)
    st = torch.cuda.current_stream()
    cases = bad = 0
    first_bad = None
    t_end, t_note = time.time() + a.seconds, time.time() + 30
    while time.time() < t_end:
        if time.time() > t_note:
            print(json.dumps({"progress_cases": cases, "bad": bad}), flush=True)
            t_note = time.time() + 30
        k = int(rng.choice([4, 4, 4, int(rng.integers(1, 11))]))
        m = int(rng.integers(0, 5))
        T = k + m
        block = int(rng.choice([1000, 1000, 8, 16, 520, 4096, 8192, 1, 7, 999, int(rng.integers(1, 3000))]))
        n = int(rng.choice([1, block, k * block, k * block + 1, int(rng.integers(1, 200_000)),
                            int(rng.integers(1, 6_000_000))]))
        rs = rsamd.ReedSolomon.create(k, m)
        oc = c_ref.Codec(k, m)
        _, S = file_layout(rs, n, block)
        stride = int(S + rng.choice([0, 0, 8, 256 - S % 256 if S % 256 else 0, int(rng.integers(0, 300))]))
        foff = int(rng.choice([0, 0, 8, int(rng.integers(0, 64))]))
        data = rng.integers(0, 256, n, dtype=np.uint8)
        fdev = torch.empty(foff + n + 64, dtype=torch.uint8, device="cuda:0")
        fdev[:] = torch.from_numpy(rng.integers(0, 256, foff + n + 64, dtype=np.uint8))
        fdev[foff:foff + n] = torch.from_numpy(data)
        fsnap = fdev.cpu().numpy()
        sh0 = rng.integers(0, 256, T * stride + 64, dtype=np.uint8)
        sdev = torch.from_numpy(sh0).to("cuda:0")
        encode_file_dev(rs, fdev.data_ptr() + foff, n, sdev.data_ptr(), stride, block, st)
        ref = oc.file_encode(data.tobytes(), block)
        want = sh0.copy()
        for i in range(T):
            want[i * stride:i * stride + S] = ref[i]
        got = sdev.cpu().numpy()
        ok = np.array_equal(got, want) and np.array_equal(fdev.cpu().numpy(), fsnap)
        e = int(rng.integers(0, m + 1))
        miss = sorted(int(x) for x in rng.choice(T, e, replace=False)) if e else []
        present = [i not in miss for i in range(T)]
        erased = want.copy()
        for j in miss:
            erased[j * stride:j * stride + S] = 0x3C
        sdev.copy_(torch.from_numpy(erased))
        wm = bool(rng.integers(0, 2))
        ooff = int(rng.choice([0, 8, int(rng.integers(0, 64))]))
        out0 = rng.integers(0, 256, ooff + n + 64, dtype=np.uint8)
        odev = torch.from_numpy(out0).to("cuda:0")
        decode_file_dev(rs, sdev.data_ptr(), S, stride, present, odev.data_ptr() + ooff, n, block, wm, st)
        owant = out0.copy()
        owant[ooff:ooff + n] = data
        ok = ok and np.array_equal(odev.cpu().numpy(), owant)
        sgot = sdev.cpu().numpy()
        if wm:
            ok = ok and np.array_equal(sgot, want)
        else:  # survivors untouched; absent shards scratch, pads untouched
            for i in range(T):
                if present[i]:
                    ok = ok and np.array_equal(sgot[i * stride:i * stride + S], want[i * stride:i * stride + S])
                ok = ok and np.array_equal(sgot[i * stride + S:(i + 1) * stride], want[i * stride + S:(i + 1) * stride])
        cases += 1
        if not ok:
            bad += 1
            if first_bad is None:
                first_bad = {"k": k, "m": m, "block": block, "n": n, "S": S, "stride": stride, "foff": foff,
                             "miss": miss, "write_missing": wm}
    oob = None
    lib = _lib.load()
    if hasattr(lib, "rs_bounds_report"):
        import ctypes as C
        nn, addr, ln, where = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint32()
        lib.rs_bounds_report(C.byref(nn), C.byref(addr), C.byref(ln), C.byref(where))
        oob = nn.value
    print(json.dumps({"seconds": a.seconds, "seed": a.seed, "cases": cases, "bad": bad, "first_bad": first_bad,
                      "bounds_violations": oob}), flush=True)
    return 1 if bad or oob else 0


if __name__ == "__main__":
    sys.exit(main())
