#!/usr/bin/env python3
"""Benchmark: device-resident Reed-Solomon encode on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 4 data + 2 parity shards, 1 MiB per shard,
4096 stripes per GPU, all resident in HBM ([stripe][shard][1 MiB], 24 GiB per
GPU) before timing starts.  One step = one rs_encode_batch_dev call over the
whole batch (one kernel launch).  N GPUs = N independent processes, each
encoding its own 4096 stripes (stripes are independent: no collective on the
data path; torch.distributed is used only for the timing barrier and the max
over ranks).  value = user data protected per second over all GPUs =
N * k * S * B * steps / t  (GiB/s).

Also reported (rank 0): decode rates for 1 and 2 erasures, the device copy
kernel rate, the roofline of the encode kernel (HIP events on the launch
stream), and the CPU baseline -- the oracle's scalar restatement of the
reference loop (InputOutputByteTableCodingLoop.java:12-44) timed on a bounded
sample on this host.

Run:  python bench.py [--gpus N --steps K --warmup W]
      (N > 1 is launched by torch.distributed.run, one rank per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd")
sys.path.insert(0, PKG_DIR)
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
SEED = 0x5EED
METRIC = "RS encode/decode GiB/s device-resident, 4+2×1 MiB stripes, at 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--m", type=int, default=2)
    ap.add_argument("--shard-bytes", type=int, default=1 << 20)
    ap.add_argument("--stripes", type=int, default=4096, help="stripes per GPU")
    ap.add_argument("--pad", type=int, default=0, help="bytes of padding between shards (layout A/B only)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    ap.add_argument("--no-extras", action="store_true", help="skip decode/copy/host-inclusive/CPU legs")
    ap.add_argument("--alloc", choices=["contiguous", "hipmalloc"], default="contiguous",
                    help="HBM for the headline stripe batch: rs_dev_alloc contiguous range (default) or torch/hipMalloc "
                         "(the other configs' pools stay hipMalloc: contiguous measured no better there)")
    return ap.parse_args()


def main():
    args = parse()
    import torch

    import rsamd
    from rsamd import parallel
    r = parallel.init_from_env(use_gpu=True)
    world, rank = r.world, r.rank
    dev = torch.device("cuda", torch.cuda.current_device())

    from rsamd import device as rdev
    from rsamd.device import StripeLayout

    k, m, S, B = args.k, args.m, args.shard_bytes, args.stripes
    # Weak scaling: every rank owns B stripes of a global batch of B * world.
    stripe0, count = parallel.stripe_partition(B * world, world, rank)
    assert count == B
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S, pad=args.pad)
    buf = stripe_pool(torch, rdev, lay.nbytes, dev, args.alloc)
    stream = torch.cuda.current_stream()
    rdev.fill_synthetic(buf.data_ptr(), k, lay, SEED, stripe0=stripe0, stream=stream)
    torch.cuda.synchronize()

    def barrier():
        parallel.barrier(r)

    def step():
        rdev.encode(rs, buf.data_ptr(), lay, stream)

    for _ in range(args.warmup):
        step()
    barrier()
    # Per-launch HIP events on the launch stream (the kernel's own duration).
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s, e in evs:
        s.record(stream)
        step()
        e.record(stream)
    barrier()
    elapsed = parallel.max_over_ranks(r, time.perf_counter() - t0)
    launch_times = sorted(s.elapsed_time(e) for s, e in evs)
    launch_ms = sum(launch_times) / len(launch_times)
    median_ms = launch_times[len(launch_times) // 2]

    # Verify the timed result before reporting (a wrong fast kernel is not done).
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream)
    ok = parallel.all_ranks_true(r, int(flag.item()) == 0)

    buf_alloc = buf.contiguous if isinstance(buf, rdev.DeviceBuffer) else None
    user_bytes = k * S * B  # per GPU per step
    value = world * user_bytes * args.steps / elapsed / 2**30
    alg_bytes = (k + m) * S * B  # per launch: each data byte read once, each parity byte written once
    achieved = alg_bytes / (launch_ms * 1e-3) / 1e9

    extra = {}
    cpu = None
    if rank == 0 and not args.no_extras:
        extra = device_extras(torch, rs, rdev, buf, lay, stream, k, m, S, B)
        del buf
        torch.cuda.empty_cache()
        if world == 1:  # multi-GPU runs report the scaling line only (the other ranks wait)
            extra.update(other_configs(torch, rsamd, rdev, dev, stream))
            extra.update(layout_legs(torch, rsamd, dev, stream))
            cpu = cpu_baseline(k, m, S, args.cpu_seconds)
            extra.update(host_inclusive(rsamd, k, m))
            extra.update(config0_single_stripe(rsamd, k, m))
    if world > 1 and not args.no_extras:
        # every rank at once: the node's aggregate host <-> device rate
        extra.update(host_inclusive_all_ranks(rsamd, parallel, r, k, m))
    traffic = pmc_traffic(k, m, S, B)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 bytes generated in HBM)",
            "config": {
                "workload": f"encode {k}+{m} x {S // 1024} KiB shards x {B} stripes per GPU (BASELINE configs[1])",
                "k": k, "m": m, "shard_bytes": S, "stripes_per_gpu": B, "global_stripes": B * world,
                "parallelism": f"stripe-partitioned x{world} (no collective; {r.backend} only for timing)",
                "hbm_alloc": alloc_note(buf_alloc),
            },
            "verified": ok,
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "kernel": f"gf_vec_kernel<{k},{m},false> (rs_encode_batch_dev)",
                "alg_bytes_per_launch": alg_bytes,
                "avg_launch_ms": round(launch_ms, 4),
                "median_launch_ms": round(median_ms, 4),  # SURVEY 8(d) asks for the median too
                # also as a fraction of the measured device copy kernel
                "frac_of_copy_kernel": (round(achieved / extra["copy_kernel_GBps"], 4)
                                        if extra.get("copy_kernel_GBps") else None),
            },
            "cpu_baseline": cpu,
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    parallel.shutdown(r)


def stripe_pool(torch, rdev, nbytes, dev, mode):
    """HBM for a stripe batch: one physically contiguous range from
    rs_dev_alloc (what a service keeping its stripes resident allocates once;
    +1.2-1.5 points of the 8 TB/s peak on the headline encode over hipMalloc
    memory, tools/alloc_probe.py) or a torch (hipMalloc) tensor."""
    if mode == "contiguous":
        return rdev.DeviceBuffer(nbytes, contiguous=True)
    return torch.empty(nbytes, dtype=torch.uint8, device=dev)


def alloc_note(contiguous):
    if contiguous is None:
        return "hipMalloc (torch)"
    return "rs_dev_alloc: physically contiguous" if contiguous else "rs_dev_alloc: hipMalloc (no contiguous range)"


def timed(torch, stream, fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # Untimed calls: the first builds any host-side plans; after that host work
    # the GPU has idled and needs some tens of ms of load before it runs at its
    # steady rate (a 10+4 masked leg read 0.64-0.68 of peak over its first ~8
    # calls, then 0.71-0.75 per call: profiles/r1/masked/masked_per_call.txt).
    # So warm up for at least 3 calls AND 50 ms.
    fn()
    torch.cuda.synchronize()
    t0, n = time.perf_counter(), 0
    while n < 2 or time.perf_counter() - t0 < 0.05:
        fn()
        torch.cuda.synchronize()
        n += 1
    s.record(stream)
    for _ in range(iters):
        fn()
    e.record(stream)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def device_extras(torch, rs, rdev, buf, lay, stream, k, m, S, B):
    out = {}
    for miss in [(0,), (0, 1), (0, 5)]:
        present = [i not in miss for i in range(k + m)]
        t = timed(torch, stream, lambda: rdev.decode(rs, buf.data_ptr(), present, lay, stream), 5)
        e = len(miss)
        key = "decode_" + "_".join(map(str, miss))
        out[key + "_GiBps"] = round(k * S * B / t / 2**30, 2)
        out[key + "_hbm_frac"] = round((k + e) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
    # row f3: isParityCorrect over the batch (reads k+m shards, writes nothing)
    flag = torch.zeros(1, dtype=torch.int32, device=buf.device)
    t = timed(torch, stream, lambda: rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream), 5)
    out["verify_GiBps"] = round(k * S * B / t / 2**30, 2)
    out["verify_hbm_frac"] = round((k + m) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
    out["verify_clean"] = int(flag.item()) == 0
    n = min(buf.numel() // 2, 8 << 30)
    t = timed(torch, stream, lambda: rdev.copy(buf.data_ptr() + n, buf.data_ptr(), n, stream), 5)
    out["copy_kernel_GBps"] = round(2 * n / t / 1e9, 1)
    out["copy_kernel_hbm_frac"] = round(2 * n / t / 1e9 / HBM_PEAK_GBPS, 4)
    return out


def other_configs(torch, rsamd, rdev, dev, stream, alloc="hipmalloc"):
    """BASELINE configs[3] (10+4 x 4 MiB; the per-GPU share of 1024 stripes over
    8 GPUs) and configs[4] (4+2 x 4 KiB x 1 M stripes), encode and decode."""
    from rsamd.device import StripeLayout
    out = {}
    for name, k, m, S, B, miss, pad in [("cfg3_10p4_4MiB_x128", 10, 4, 4 << 20, 128, (0, 1, 2, 3), 0),
                                        ("cfg3_10p4_4MiB_x128_pad4K", 10, 4, 4 << 20, 128, (0, 1, 2, 3), 4096),
                                        ("cfg4_4p2_4KiB_x1M", 4, 2, 4096, 1 << 20, (0, 1), 0)]:
        rs = rsamd.ReedSolomon.create(k, m)
        lay = StripeLayout.packed(B, k + m, S, pad=pad)
        buf = stripe_pool(torch, rdev, lay.nbytes, dev, alloc)
        rdev.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, stream)
        t = timed(torch, stream, lambda: rdev.encode(rs, buf.data_ptr(), lay, stream), 10)
        out[name + "_encode_GiBps"] = round(k * S * B / t / 2**30, 2)
        out[name + "_encode_hbm_frac"] = round((k + m) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
        present = [i not in miss for i in range(k + m)]
        t = timed(torch, stream, lambda: rdev.decode(rs, buf.data_ptr(), present, lay, stream), 10)
        out[name + "_decode_" + "_".join(map(str, miss)) + "_GiBps"] = round(k * S * B / t / 2**30, 2)
        out[name + "_decode_hbm_frac"] = round((k + len(miss)) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream)
        out[name + "_verified"] = int(flag.item()) == 0
        # row f3 (isParityCorrect) on the same batch: (k+m)*S*B bytes read
        t = timed(torch, stream, lambda: rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream), 5)
        out[name + "_verify_hbm_frac"] = round((k + m) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
        if name == "cfg3_10p4_4MiB_x128":
            # row f2 for the wide code: 4 random erasures per stripe, device bitmasks, one launch
            import numpy as np
            rng = np.random.default_rng(0)
            present = np.ones((B, k + m), dtype=bool)
            for t_ in range(B):
                present[t_, rng.choice(k + m, 4, replace=False)] = False
            bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).to(dev)
            alg = (k * B + int((~present).sum())) * S
            t = timed(torch, stream, lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0,
                                                                     stream), 5)
            out[name + "_decode_masked_bits_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)
            rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream)
            out[name + "_decode_masked_bits_verified"] = int(flag.item()) == 0
        if name.startswith("cfg4"):
            # row f2: a random presence pattern per stripe (<= 2 erasures), one launch
            import itertools
            import numpy as np
            pats = np.array([[i not in miss for i in range(k + m)] for e in range(3)
                             for miss in itertools.combinations(range(k + m), e)], dtype=bool)
            present = pats[np.random.default_rng(0).integers(0, len(pats), B)]
            # algorithmic bytes: k survivors read + the absent shards written, for
            # every stripe with an erasure (complete stripes are not touched)
            alg = (k * int((~present).any(axis=1).sum()) + int((~present).sum())) * S
            # 10 calls: the first call's host-side prep is not overlapped with a previous call
            t = timed(torch, stream, lambda: rdev.decode_masked(rs, buf.data_ptr(), present, lay, stream), 10)
            out[name + "_decode_masked_GiBps"] = round(k * S * B / t / 2**30, 2)
            out[name + "_decode_masked_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)
            rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream)
            out[name + "_decode_masked_verified"] = int(flag.item()) == 0
            # the same patterns as device-resident bitmasks (no host work per call)
            bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).to(dev)
            t = timed(torch, stream, lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0,
                                                                     stream), 5)
            out[name + "_decode_masked_bits_GiBps"] = round(k * S * B / t / 2**30, 2)
            out[name + "_decode_masked_bits_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)
            rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream)
            out[name + "_decode_masked_bits_verified"] = int(flag.item()) == 0
        del buf
        torch.cuda.empty_cache()
    return out


def layout_legs(torch, rsamd, dev, stream):
    """Row f1: the client layout fused into the kernels -- a 4 GiB file encoded
    straight into 4+2 shards, and decoded back with 2 erasures."""
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    rs = rsamd.ReedSolomon.create(4, 2)
    n = 4 << 30
    _, S = file_layout(rs, n)
    stride = (S + 255) // 256 * 256
    f = torch.empty(n, dtype=torch.uint8, device=dev)
    from rsamd import device as rdev
    from rsamd.device import StripeLayout
    rdev.fill_synthetic(f.data_ptr(), 1, StripeLayout(1, n, n, n), SEED, 0, stream)
    sh = torch.empty(6 * stride, dtype=torch.uint8, device=dev)
    out = {}
    t = timed(torch, stream, lambda: encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, stream=stream), 5)
    out["file_encode_4GiB_GiBps"] = round(n / t / 2**30, 2)
    out["file_encode_hbm_frac"] = round((n + 6 * S) / t / 1e9 / HBM_PEAK_GBPS, 4)
    g = torch.empty(n, dtype=torch.uint8, device=dev)
    present = [False, True, True, True, True, False]
    t = timed(torch, stream, lambda: decode_file_dev(rs, sh.data_ptr(), S, stride, present, g.data_ptr(), n,
                                                     stream=stream), 5)
    out["file_decode_0_5_4GiB_GiBps"] = round(n / t / 2**30, 2)
    out["file_decode_hbm_frac"] = round((4 * S + n) / t / 1e9 / HBM_PEAK_GBPS, 4)
    out["file_round_trip_ok"] = bool(torch.equal(f, g))
    del f, g, sh
    torch.cuda.empty_cache()
    return out


def cpu_baseline(k, m, S, budget_s):
    """The oracle's scalar InputOutputByteTable loop (the reference's default
    coding loop, -O2 -fno-tree-vectorize) on host-resident stripes."""
    import numpy as np
    from oracle import c_ref
    c_ref.build()
    codec = c_ref.Codec(k, m)
    n = 8
    stride = S
    host = np.zeros(n * (k + m) * stride, dtype=np.uint8)
    for t in range(n):
        host[t * (k + m) * S: t * (k + m) * S + k * S] = c_ref.fill_synthetic(k * S, SEED, t)
    done, t0 = 0, time.perf_counter()
    while True:
        codec.code_stripes(host, n, S, stride, (k + m) * stride, None, 1)
        done += n
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    rate = k * S * done / el / 2**30
    threads = min(16, os.cpu_count() or 1)
    done_mt, t1 = 0, time.perf_counter()
    nm = threads * 2
    host_mt = np.zeros(nm * (k + m) * S, dtype=np.uint8)
    while time.perf_counter() - t1 < budget_s / 2:
        codec.code_stripes(host_mt, nm, S, S, (k + m) * S, None, threads)
        done_mt += nm
    rate_mt = k * S * done_mt / (time.perf_counter() - t1) / 2**30
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(rate, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{done} stripes of {k}+{m} x {S // 1024} KiB encoded by the scalar restatement of "
                      f"InputOutputByteTableCodingLoop (oracle/rs_oracle.c, -O2 -fno-tree-vectorize), "
                      f"{el:.1f} s, host-resident",
            "multi_thread": {"value": round(rate_mt, 4), "threads": threads, "stripes": done_mt},
            "cpu_model": model}


def host_inclusive(rsamd, k, m):
    """Rates of the JNI-facing host-buffer API: H2D + kernel + D2H on pageable
    buffers, chunked and overlapped on three streams (host.cpp run_chunks)."""
    import numpy as np
    from rsamd.layout import file_encode_into, file_layout
    n = 64 << 20
    rng = np.random.default_rng(5)
    sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] + [np.zeros(n, np.uint8) for _ in range(m)]
    rs = rsamd.ReedSolomon.create(k, m)
    out = {}

    def rate(fn, user_bytes, reps=3):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return round(user_bytes / ((time.perf_counter() - t0) / reps) / 2**30, 3)

    out["host_inclusive_encode_GiBps"] = rate(lambda: rs.encodeParity(sh, 0, n), k * n)
    present = [False, False] + [True] * (k + m - 2)
    out["host_inclusive_decode_0_1_GiBps"] = rate(lambda: rs.decodeMissing(sh, present, 0, n), k * n)
    data = rng.integers(0, 256, k * n, dtype=np.uint8)
    _, S = file_layout(rs, len(data))
    fsh = [np.zeros(S, np.uint8) for _ in range(k + m)]
    out["host_inclusive_file_encode_GiBps"] = rate(lambda: file_encode_into(rs, data, fsh), len(data))
    from rsamd.layout import file_decode_into
    fpresent = [False] + [True] * (k + m - 2) + [False]
    fout = np.empty(len(data), np.uint8)
    out["host_inclusive_file_decode_0_%d_GiBps" % (k + m - 1)] = rate(
        lambda: file_decode_into(rs, fsh, fpresent, S, fout), len(data))
    # the same calls on pinned (page-locked) host buffers, where
    # the two streams' H2D and D2H overlap as DMA
    import torch
    pin = [torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(k + m)]
    for a, b in zip(pin, sh):
        a[:] = b
    out["host_inclusive_pinned_encode_GiBps"] = rate(lambda: rs.encodeParity(pin, 0, n), k * n)
    out["host_inclusive_pinned_decode_0_1_GiBps"] = rate(lambda: rs.decodeMissing(pin, present, 0, n), k * n)
    del pin
    out["host_inclusive_note"] = (f"{k}+{m}, {n >> 20} MiB host shards per call, pageable unless 'pinned' "
                                  f"(file legs: a {len(data) >> 20} MiB file); PCIe-bound, never the bench value")
    return out


def config0_single_stripe(rsamd, k, m, S=64 << 10, reps=200):
    """BASELINE configs[0]: one 4+2 stripe of 64 KiB shards, encode then a
    1-erasure decode, through the JNI-facing host API (H2D + kernel + D2H per
    call) -- a latency, not a throughput -- next to the oracle's scalar port of
    the reference loop on the same host buffers."""
    import numpy as np
    from oracle import c_ref
    rng = np.random.default_rng(0)
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    sh = [a.copy() for a in data] + [np.zeros(S, np.uint8) for _ in range(m)]
    rs = rsamd.ReedSolomon.create(k, m)
    oc = c_ref.Codec(k, m)
    ref = [a.copy() for a in data] + [np.zeros(S, np.uint8) for _ in range(m)]
    present = [False] + [True] * (k + m - 1)

    def per_call_us(fn):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return round((time.perf_counter() - t0) / reps * 1e6, 1)

    out = {"cfg0_gpu_host_api_encode_us": per_call_us(lambda: rs.encodeParity(sh, 0, S)),
           "cfg0_cpu_port_encode_us": per_call_us(lambda: oc.encode_parity(ref, 0, S))}
    ok = all(np.array_equal(a, b) for a, b in zip(sh, ref))

    def gpu_decode():
        sh[0][:] = 0
        rs.decodeMissing(sh, present, 0, S)

    def cpu_decode():
        ref[0][:] = 0
        oc.decode_missing(ref, present, 0, S)

    out["cfg0_gpu_host_api_decode_0_us"] = per_call_us(gpu_decode)
    out["cfg0_cpu_port_decode_0_us"] = per_call_us(cpu_decode)
    out["cfg0_bit_exact"] = ok and all(np.array_equal(a, b) for a, b in zip(sh, ref)) and \
        np.array_equal(sh[0], data[0])
    out["cfg0_note"] = (f"one {k}+{m} stripe of {S >> 10} KiB shards per call, host buffers; GPU = host API "
                        f"(H2D + kernel + D2H), CPU = oracle scalar port, 1 thread")
    return out


def host_inclusive_all_ranks(rsamd, parallel, r, k, m, n=64 << 20, reps=4):
    """SURVEY 8(d) host-inclusive rate at N GPUs: every rank calls the
    JNI-facing encodeParity on its own host shards at the same time (pinned,
    then pageable), bracketed by barriers; aggregate user bytes over the
    slowest rank's time.  Bound by the node's PCIe / host memory, not HBM."""
    import numpy as np
    import torch
    rng = np.random.default_rng(100 + r.rank)
    rs = rsamd.ReedSolomon.create(k, m)
    pin = [torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(k + m)]
    for a in pin[:k]:
        a[:] = rng.integers(0, 256, n, dtype=np.uint8)
    pageable = [a.copy() for a in pin]
    out = {}
    for name, sh in (("pinned", pin), ("pageable", pageable)):
        rs.encodeParity(sh, 0, n)  # warm-up (staging buffers, pinned mirrors)
        parallel.barrier(r)
        t0 = time.perf_counter()
        for _ in range(reps):
            rs.encodeParity(sh, 0, n)
        el = parallel.max_over_ranks(r, time.perf_counter() - t0)
        out[f"host_inclusive_{name}_encode_all_ranks_GiBps"] = round(r.world * reps * k * n / el / 2**30, 2)
    out["host_inclusive_all_ranks_note"] = (f"{r.world} ranks at once, {k}+{m} x {n >> 20} MiB host shards per "
                                            f"call, {reps} calls per rank")
    del pin, pageable
    return out


def pmc_traffic(k, m, S, B):
    """HBM bytes per launch from the committed rocprofv3 PMC summary for this
    exact workload (profiles/pmc_traffic.json), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        key = f"encode_{k}_{m}_{S}_{B}"
        return d[key]["hbm_bytes_per_launch"] if key in d else None
    except (OSError, ValueError, KeyError):
        return None


if __name__ == "__main__":
    main()
