#!/usr/bin/env python3
"""Is the 4+2 headline's two-level rate (0.80 / 0.83 of peak) a clock state?
Runs the headline encode back to back for SECONDS on one contiguous pool and,
per window of ~0.25 s, prints the window's rate next to every pp_dpm_* clock
level the driver marks active (*) and gpu_busy_percent, read from sysfs."""
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))


def clocks():
    out = {}
    for f in sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_*")):
        card = f.split("/")[4]
        try:
            lines = open(f).read().splitlines()
        except OSError:
            continue
        act = [ln.split(":", 1)[1].strip().rstrip("*").strip() for ln in lines if ln.strip().endswith("*")]
        out[f"{card}.{os.path.basename(f)[7:]}"] = act[0] if act else None
    return out


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    import torch
    import rsamd
    from rsamd import device as rdev
    from rsamd.device import DeviceBuffer, StripeLayout
    k, m, S, B = 4, 2, 1 << 20, 4096
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    st = torch.cuda.current_stream()
    pool = DeviceBuffer(lay.nbytes, True)
    rdev.fill_synthetic(pool.data_ptr(), k, lay, 0x5EED, 0, st)
    print(json.dumps({"sysfs": sorted(clocks())}), flush=True)
    t_end = time.time() + secs
    while time.time() < t_end:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(60):
            rdev.encode(rs, pool.data_ptr(), lay, st)
        e1.record(st)
        c = clocks()  # sampled while the launches run
        torch.cuda.synchronize()
        frac = (k + m) * S * B / (e0.elapsed_time(e1) / 60 * 1e-3) / 8e12
        row = {"t": round(time.time() % 1000, 2), "frac": round(frac, 4)}
        row.update({k2: v for k2, v in c.items() if k2.startswith("card") and v})
        print(json.dumps(row), flush=True)
    pool.free()


if __name__ == "__main__":
    main()
