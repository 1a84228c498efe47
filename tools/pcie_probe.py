#!/usr/bin/env python3
"""Host<->device copy rates on this box (pinned / pageable, one direction or
both at once on two streams) -- the ceiling of the host-inclusive legs."""
import json
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


if __name__ == "__main__":
    main()
