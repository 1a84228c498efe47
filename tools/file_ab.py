#!/usr/bin/env python3
"""Row f1 on one box, in one process: the fused file encode (untiled default,
tiled opt-in RSAMD_FILE_ENCODE=1) and the tiled {0,5} decode of a 4 GiB file,
for a few shard-stride pads, legs alternated over ROUNDS rounds so that the
memory system's slow drift and per-box state hit every leg alike.  Each leg
warms up for 0.6 s of back-to-back calls (bench.py's leg warm-up).
Usage: python tools/file_ab.py [ROUNDS]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))
PADS = (0, 4096, 65536 + 4096, 1 << 20)


def timed(torch, st, fn, iters=5, warm_s=0.6):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(st)
    for _ in range(iters):
        fn()
    e.record(st)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    st = torch.cuda.current_stream()
    rs = rsamd.ReedSolomon.create(4, 2)
    n = 4 << 30
    _, S = file_layout(rs, n)
    base = (S + 255) // 256 * 256
    f = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    rdev.fill_synthetic(f.data_ptr(), 1, StripeLayout(1, n, n, n), 0x5EED, 0, st)
    sh = torch.empty(6 * (base + max(PADS)), dtype=torch.uint8, device="cuda:0")
    g = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    present = [False, True, True, True, True, False]
    res = {}
    for r in range(rounds):
        for pad in PADS:
            stride = base + pad
            for tiled in (0, 1):
                os.environ["RSAMD_FILE_ENCODE"] = str(tiled)
                t = timed(torch, st, lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, stream=st))
                res.setdefault(f"encode pad {pad:>8} {'tiled' if tiled else 'untiled'}", []).append(
                    round((n + 6 * S) / t / 8e12, 4))
            os.environ["RSAMD_FILE_ENCODE"] = "0"
            t = timed(torch, st, lambda: decode_file_dev(rs, sh.data_ptr(), S, stride, present, g.data_ptr(), n,
                                                         stream=st))
            res.setdefault(f"decode pad {pad:>8} tiled {{0,5}}", []).append(round((4 * S + n) / t / 8e12, 4))
            if r == 0 and not torch.equal(f, g):
                print(json.dumps({"error": f"round trip failed at pad {pad}"}), flush=True)
                return 1
        print(f"round {r} done", file=sys.stderr, flush=True)
    for k, v in res.items():
        print(f"{k:<36} " + " ".join(f"{x:.4f}" for x in v) + f"   median {sorted(v)[len(v) // 2]:.4f}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
