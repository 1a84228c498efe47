#!/usr/bin/env python3
"""Fused file encode / decode {0,5} of a 4 GiB file (bench.py's layout legs)
over alternating pool allocations in one process: torch (hipMalloc) against
rs_dev_alloc contiguous pools, for file and shards alike."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import DeviceBuffer, StripeLayout
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    rs = rsamd.ReedSolomon.create(4, 2)
    n = (4 << 30) // 4000 * 4000
    _, S = file_layout(rs, n)
    stride = (S + 255) // 256 * 256
    st = torch.cuda.current_stream()

    def timed(fn, it=5):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st)
        for _ in range(it):
            fn()
        e.record(st)
        torch.cuda.synchronize()
        return s.elapsed_time(e) / it * 1e-3

    for mode in (sys.argv[1] if len(sys.argv) > 1 else "torch,contiguous,torch,contiguous,torch,contiguous").split(","):
        mk = (lambda nb: DeviceBuffer(nb, True)) if mode == "contiguous" else (
            lambda nb: torch.empty(nb, dtype=torch.uint8, device="cuda:0"))
        f, sh, g = mk(n), mk(6 * stride), mk(n)
        rdev.fill_synthetic(f.data_ptr(), 1, StripeLayout(1, n, n, n), 0x5EED, 0, st)
        t_enc = timed(lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, stream=st))
        present = [False, True, True, True, True, False]
        t_dec = timed(lambda: decode_file_dev(rs, sh.data_ptr(), S, stride, present, g.data_ptr(), n, stream=st))
        print(json.dumps({"mode": mode, "file_encode": round((n + 6 * S) / t_enc / 8e12, 4),
                          "file_decode_0_5": round((4 * S + n) / t_dec / 8e12, 4)}), flush=True)
        del f, sh, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
