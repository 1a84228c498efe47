#!/usr/bin/env python3
"""Host<->device copy rates on this box (pinned / pageable, one direction or
both at once on two streams) -- the ceiling of the host-inclusive legs."""
import json
import os
import time

import torch


def main():
    n = 256 << 20
    dev = torch.empty(2 * n, dtype=torch.uint8, device="cuda:0")
    out = {}
    for kind in ("pinned", "pageable"):
        a = torch.empty(n, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        b = torch.empty(n, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        a.fill_(1)
        b.fill_(2)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

        def run(h2d, d2h, reps=5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                if h2d:
                    with torch.cuda.stream(s1):
                        dev[:n].copy_(a, non_blocking=True)
                if d2h:
                    with torch.cuda.stream(s2):
                        b.copy_(dev[n:], non_blocking=True)
            torch.cuda.synchronize()
            return (h2d + d2h) * n * reps / (time.perf_counter() - t0) / 1e9

        run(True, True, 1)
        out[kind + "_h2d_GBps"] = round(run(True, False), 1)
        out[kind + "_d2h_GBps"] = round(run(False, True), 1)
        out[kind + "_both_GBps"] = round(run(True, True), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__" and not os.environ.get("PROBE_THREADS"):
    main()


def threads_probe():
    """Pageable H2D and D2H issued from two host threads at once (hipMemcpy via
    ctypes releases the GIL): does the runtime overlap the directions?"""
    import ctypes
    import glob
    import os
    import threading
    lib = [p for p in glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so*"))]
    hip = ctypes.CDLL(lib[0])
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    n = 256 << 20
    dev = torch.empty(2 * n, dtype=torch.uint8, device="cuda:0")
    out = {}
    for kind in ("pageable", "pinned"):
        a = torch.empty(n, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        b = torch.empty(n, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        a.fill_(1)
        b.fill_(2)
        torch.cuda.synchronize()

        def h2d(reps):
            for _ in range(reps):
                assert hip.hipMemcpy(dev.data_ptr(), a.data_ptr(), n, 1) == 0

        def d2h(reps):
            for _ in range(reps):
                assert hip.hipMemcpy(b.data_ptr(), dev.data_ptr() + n, n, 2) == 0

        h2d(1)
        d2h(1)
        t0 = time.perf_counter()
        th = [threading.Thread(target=h2d, args=(4,)), threading.Thread(target=d2h, args=(4,))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        out[kind + "_two_threads_both_GBps"] = round(2 * 4 * n / (time.perf_counter() - t0) / 1e9, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__" and os.environ.get("PROBE_THREADS"):
    threads_probe()
