#!/usr/bin/env python3
"""Cost of page-locking a pageable 64 MiB caller array per call, the way the
host API does it (host.cpp HostRegistration): hipHostRegister (default or
mapped flag), hipHostGetDevicePointer, hipHostUnregister -- first call on a
range and repeated calls.
  python tools/reg_cost.py"""
import ctypes
import json
import time

import numpy as np


def main():
    import torch
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    n = 64 << 20
    arrs = [np.ones(n, np.uint8) for _ in range(6)]
    for flag_name, flag in (("default", 0), ("mapped", 2)):
        for rep in range(4):
            t0 = time.perf_counter()
            for a in arrs:
                rc = hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(n), ctypes.c_uint(flag))
                assert rc == 0, rc
            t1 = time.perf_counter()
            ok = 0
            for a in arrs:
                d = ctypes.c_void_p()
                rc = hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(a.ctypes.data + 4096 + 3), 0)
                ok += rc == 0
                dev_same = d.value == a.ctypes.data + 4096 + 3
            t2 = time.perf_counter()
            for a in arrs:
                assert hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data)) == 0
            t3 = time.perf_counter()
            print(json.dumps({"flag": flag_name, "rep": rep, "register_ms_6x64MiB": round((t1 - t0) * 1e3, 3),
                              "devptr_ok": ok, "devptr_equals_host_va": dev_same,
                              "getdevptr_ms": round((t2 - t1) * 1e3, 3),
                              "unregister_ms": round((t3 - t2) * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
