#!/usr/bin/env python3
"""Is the headline encode's run-to-run spread (0.785 vs 0.815 of peak, whole
runs slow or fast) a property of the 24 GiB allocation?  One process: the
BASELINE config-2 batch allocated by torch (caching allocator -> hipMalloc),
by hipMalloc directly, or by hipExtMallocWithFlags(hipDeviceMallocContiguous);
fill, 5 warm-up and 30 timed encodes; prints the fraction of 8 TB/s.
Usage: alloc_probe.py torch|hipmalloc|contiguous"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def main():
    mode = sys.argv[1]
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    k, m, S, B = 4, 2, 1 << 20, 4096
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    st = torch.cuda.current_stream()
    hip = None
    if mode == "torch":
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        base = buf.data_ptr()
    else:
        hip = ctypes.CDLL("libamdhip64.so")
        p = ctypes.c_void_p()
        if mode == "hipmalloc":
            rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(lay.nbytes))
        else:
            rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(lay.nbytes), ctypes.c_uint(0x4))
        if rc != 0:
            print(json.dumps({"mode": mode, "alloc_rc": rc}), flush=True)
            return
        base = p.value
    rdev.fill_synthetic(base, k, lay, 0x5EED, 0, st)
    for _ in range(5):
        rdev.encode(rs, base, lay, st)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(30)]
    for s, e in evs:
        s.record(st)
        rdev.encode(rs, base, lay, st)
        e.record(st)
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(e) for s, e in evs)
    avg = sum(ms) / len(ms)
    print(json.dumps({"mode": mode, "frac": round(6 * S * B / (avg * 1e-3) / 8e12, 4), "avg_ms": round(avg, 4),
                      "min_ms": round(ms[0], 4), "max_ms": round(ms[-1], 4), "base": hex(base)}), flush=True)
    if hip is not None:
        hip.hipFree(ctypes.c_void_p(base))


if __name__ == "__main__":
    main()
