#!/usr/bin/env python3
"""Benchmark: device-resident Reed-Solomon encode on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 4 data + 2 parity shards, 1 MiB per shard,
4096 stripes per GPU, all resident in HBM ([stripe][shard][1 MiB], 24 GiB per
GPU) before timing starts.  One step = one rs_encode_batch_dev call over the
whole batch (one kernel launch).  N GPUs = N processes, one per GPU, each
encoding its own 4096 stripes (stripes are independent, ReedSolomon.java:90-104:
no collective on the data path; torch.distributed only lines the ranks up for
timing and reduces a few scalars).  value = user data protected per second over
all GPUs = N * k * S * B * steps / t  (GiB/s), t = the slowest rank's time.

Legs every rank runs at every N (whole-job aggregates, slowest rank's time):
  * 4+2 decode {0,1} on the same batch (BASELINE configs[2], weak scaling);
  * BASELINE configs[3] strong-scaled: 10+4 x 4 MiB, 1024 stripes in all, split
    by stripe index (128 per GPU at N=8), encode and {0,1,2,3} decode;
  * a sustained >= 5 s back-to-back encode with the GPU clocks sampled;
  * at N>1: the host-inclusive rate with every rank calling the JNI-facing
    host API at once.
At N=1 rank 0 also reports the per-GPU legs (more erasure patterns, verify,
copy kernel, configs[4], the fused file layout, host-inclusive rates,
configs[0]) and the CPU baseline -- the oracle's scalar restatement of the
reference loop (InputOutputByteTableCodingLoop.java:12-44) timed on bounded
samples on this host, 1 thread and the host's CPU share.  Before any of that
(N=1, default config) two rocprofv3 --pmc child runs measure the headline
kernel's HBM bytes per launch for roofline.traffic (--no-live-pmc skips them).

Run:  python bench.py [--gpus N --steps K --warmup W]
      --gpus N > 1 without WORLD_SIZE in the environment: this process starts
      torch.distributed.run with N ranks (before anything touches the GPU) and
      exits with its status; under a launcher WORLD_SIZE must equal N.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import math
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd")
sys.path.insert(0, PKG_DIR)
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
SEED = 0x5EED
METRIC = "RS encode/decode GiB/s device-resident, 4+2×1 MiB stripes, at 1/2/4/8 GPU"
CFG3_STRIPES = 1024  # BASELINE configs[3]: 10+4 x 4 MiB, 1024 stripes over the GPUs


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--m", type=int, default=2)
    ap.add_argument("--shard-bytes", type=int, default=1 << 20)
    ap.add_argument("--stripes", type=int, default=4096, help="stripes per GPU")
    ap.add_argument("--pad", type=int, default=0, help="bytes of padding between shards (layout A/B only)")
    ap.add_argument("--layout", choices=["packed", "granule"], default="granule",
                    help="HBM layout of the headline batch: the granule layout (default; include/rs_amd.h, "
                         "64 KiB granules: the same stripes and bytes, placement-robust, DESIGN.md 3.6) or "
                         "packed shards (also timed in extra.packed_4p2_1MiB_x4096_*)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline sample budget (headline config)")
    ap.add_argument("--sustained-seconds", type=float, default=5.0, help="back-to-back encode leg length")
    ap.add_argument("--cfg3-stripes", type=int, default=CFG3_STRIPES,
                    help="global stripe count of the strong-scaled 10+4 x 4 MiB leg")
    ap.add_argument("--leg-warm-s", type=float, default=LEG_WARM_S,
                    help="seconds of back-to-back untimed calls before each extra leg's timed region")
    ap.add_argument("--no-extras", action="store_true", help="headline only")
    ap.add_argument("--launch-probe", action="store_true",
                    help="launcher self-test: ranks join the process group on CPU (gloo) and report, no GPU work")
    ap.add_argument("--alloc", choices=["contiguous", "hipmalloc"], default="contiguous",
                    help="HBM for the headline stripe batch: rs_dev_alloc contiguous range (default) or torch/hipMalloc")
    ap.add_argument("--no-live-pmc", action="store_true",
                    help="skip the rocprofv3 --pmc child runs that measure the headline kernel's HBM bytes in this run "
                         "(roofline.traffic then comes from profiles/pmc_traffic.json)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# Rank launcher
# ---------------------------------------------------------------------------
def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_command(n: int, argv, port: int):
    """torch.distributed.run command that re-runs this script with the same
    arguments as n ranks on this node (rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(args, argv) -> int:
    """Start the N ranks as a child launcher and return its exit status.
    Called before this process touches the GPU (no torch.cuda call here): the
    ranks are children, never an exec of this process."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(launch_command(args.gpus, argv, free_port()), env=env).returncode


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    global LEG_WARM_S
    LEG_WARM_S = args.leg_warm_s
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args, argv)
    if int(env_world or 1) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}: refusing to report a mislabelled line",
              file=sys.stderr)
        return 2
    if args.launch_probe:
        return launch_probe(args)
    live = None
    # The live passes profile one process on cuda:0, so they run at N = 1 only:
    # at N > 1 every rank would start its own pair at once, all on GPU 0 (the
    # line then cites the committed summary of the same kernel and batch).
    if (not (args.no_extras or args.no_live_pmc) and args.gpus == 1 and args.pad == 0
            and (args.k, args.m, args.shard_bytes, args.stripes) == (4, 2, 1 << 20, 4096)):
        # before this process touches the GPU: the passes are children
        live = live_pmc_traffic("enc42" if args.layout == "packed" else "enc42g")
    return run(args, live)


def launch_probe(args) -> int:
    from rsamd import parallel
    r = parallel.init_from_env(use_gpu=False)
    total = parallel.sum_over_ranks(r, 1.0)
    start, count = parallel.stripe_partition(args.cfg3_stripes, r.world, r.rank)
    covered = parallel.sum_over_ranks(r, float(count))
    # the headline's per-rank record exchange (device identities), here with
    # host identities since the probe touches no GPU
    recs = parallel.gather_objects(r, {"rank": r.rank, "pid": os.getpid(), "stripe0": start, "stripes": count})
    if r.rank == 0:
        print(json.dumps({"probe": True, "n_gpus": r.world, "ranks_seen": int(total), "backend": r.backend,
                          "cfg3_stripes_covered": int(covered), "records": recs}), flush=True)
    parallel.shutdown(r)
    return 0


# ---------------------------------------------------------------------------
# Timing helpers
# ---------------------------------------------------------------------------
LEG_WARM_S = 0.6  # --leg-warm-s


def warm(torch, fn):
    """Untimed calls before a leg's timed region: at least 3, and back to back
    (synchronised every 4 calls) for at least LEG_WARM_S seconds."""
    fn()
    torch.cuda.synchronize()
    t0, n = time.perf_counter(), 0
    while n < 2 or time.perf_counter() - t0 < LEG_WARM_S:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
        n += 4


def timed(torch, stream, fn, iters):
    """Average seconds per call of fn on this GPU alone (HIP events)."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # Untimed calls: the first builds any host-side plans; after that host work
    # the GPU has idled and needs some tens of ms of load before it runs at its
    # steady rate (a 10+4 masked leg read 0.64-0.68 of peak over its first ~8
    # calls, then 0.71-0.75 per call: profiles/r1/masked/masked_per_call.txt).
    # From idle the memory system itself ramps too: the headline encode reads
    # 0.76, 0.805, then a steady 0.826-0.829 of peak over its first ~0.5 s of
    # load at constant clocks (profiles/r2/ab/clock_state_r2aj.txt).  So warm
    # up for at least 3 calls AND LEG_WARM_S seconds of back-to-back calls.
    warm(torch, fn)
    s.record(stream)
    for _ in range(iters):
        fn()
    e.record(stream)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def timed_all_ranks(torch, parallel, r, fn, iters):
    """Seconds per call with every rank calling fn at once: warm-up as in
    timed(), then barrier + synchronize on both sides of `iters` calls; the
    slowest rank's time."""
    warm(torch, fn)
    parallel.barrier(r)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    parallel.barrier(r)
    return parallel.max_over_ranks(r, time.perf_counter() - t0) / iters


# ---------------------------------------------------------------------------
# The run
# ---------------------------------------------------------------------------
def run(args, live_traffic=None):
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
    lay = (StripeLayout.packed(B, k + m, S, pad=args.pad) if args.layout == "packed"
           else rdev.GranuleLayout.make(B, k + m, S))
    buf = stripe_pool(torch, rdev, lay.nbytes, dev, args.alloc)
    stream = torch.cuda.current_stream()
    rdev.fill_synthetic(buf.data_ptr(), k, lay, SEED, stripe0=stripe0, stream=stream)
    torch.cuda.synchronize()

    def step():
        rdev.encode(rs, buf.data_ptr(), lay, stream)

    for _ in range(args.warmup):
        step()
    parallel.barrier(r)
    # Per-launch HIP events on the launch stream (the kernel's own duration).
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s, e in evs:
        s.record(stream)
        step()
        e.record(stream)
    parallel.barrier(r)
    local_elapsed = time.perf_counter() - t0
    elapsed = parallel.max_over_ranks(r, local_elapsed)
    launch_times = sorted(s.elapsed_time(e) for s, e in evs)
    launch_ms = sum(launch_times) / len(launch_times)
    median_ms = launch_times[len(launch_times) // 2]

    # Verify the timed result before reporting (a wrong fast kernel is not done):
    # the GPU's own parity check over every stripe, and sampled stripes
    # gathered to the host and compared with the oracle (the checker only).
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream)
    ok = parallel.all_ranks_true(r, int(flag.item()) == 0)
    oracle_check = check_vs_oracle(torch, rdev, buf, lay, k, m, S, B, stripe0, stream)
    oracle_ok = parallel.all_ranks_true(r, oracle_check["ok"])

    # Which GPU each rank ran on, and its own launch times: the line must show
    # that N GPUs did the work (distinct devices), not N ranks on one.
    me = dict(parallel.device_identity(torch), rank=rank, avg_launch_ms=round(launch_ms, 4),
              median_launch_ms=round(median_ms, 4), stripe0=stripe0, stripes=count,
              timed_region_s=round(local_elapsed, 4))
    ranks = parallel.gather_objects(r, me)
    distinct = parallel.distinct_devices(ranks)
    refusal = device_refusal(r.backend, world, ranks)
    if refusal:
        if rank == 0:
            print(f"bench.py: {refusal}: refusing to report", file=sys.stderr, flush=True)
        parallel.shutdown(r)
        return 3
    slow_ms = max(d["avg_launch_ms"] for d in ranks)
    fast_ms = min(d["avg_launch_ms"] for d in ranks)

    buf_alloc = buf.contiguous if isinstance(buf, rdev.DeviceBuffer) else None
    user_bytes = k * S * B  # per GPU per step
    value = world * user_bytes * args.steps / elapsed / 2**30
    alg_bytes = (k + m) * S * B  # per launch: each data byte read once, each parity byte written once
    # Per-GPU roofline of the slowest rank's kernel (at N = 1: this GPU's).
    achieved = alg_bytes / (slow_ms * 1e-3) / 1e9

    extra, cpu, link = {}, None, None
    if not args.no_extras:
        extra.update(decode_all_ranks(torch, parallel, r, rs, rdev, buf, lay, stream, k, m, S, B, args.steps))
        extra.update(sustained(torch, parallel, r, rs, rdev, buf, lay, stream, k, m, S, B, args.sustained_seconds))
        if world == 1:
            extra.update(device_extras(torch, rs, rdev, buf, lay, stream, k, m, S, B))
        if isinstance(buf, rdev.DeviceBuffer):
            buf.free()
        del buf
        torch.cuda.empty_cache()
        extra.update(cfg3_strong(torch, rsamd, parallel, r, rdev, dev, stream, args.cfg3_stripes, args.steps))
        if world == 1:
            extra.update(other_configs(torch, rsamd, rdev, dev, stream))
            extra.update(granule_legs(torch, rsamd, rdev, dev, stream, headline_layout=args.layout))
            extra.update(chunk_group_legs(torch, rsamd, rdev, dev, stream))
            extra.update(layout_legs(torch, rsamd, dev, stream))
            # The host legs before the CPU baseline, small calls first: run
            # after the baseline's 16 busy threads and the large host calls, the
            # configs[0] and 64 KiB calls took 44-52 us against 37 in a process
            # of their own (profiles/r5/bench_r6q.json, bench_r6x.json,
            # host_sizes_slots_r6t.txt).
            with gpu_numa_bound(torch, parallel, extra):
                link = host_link(torch)
                extra.update(config0_single_stripe(rsamd, k, m))
                extra.update(host_small_calls(rsamd, k, m))
                extra.update(host_by_size(rsamd, k, m))
                extra.update(host_inclusive(rsamd, k, m, link))
                extra.update(host_jni_legs(rsamd, k, m, link))
                extra.update(host_groups_leg(rsamd, k, m, link))
            cpu = cpu_baseline(k, m, S, args.cpu_seconds)
            extra["cpu_configs"] = cpu_configs()
        else:
            # every rank at once: the node's aggregate host <-> device rate
            with gpu_numa_bound(torch, parallel, extra):
                link = host_link(torch)
                extra.update(host_inclusive_all_ranks(rsamd, parallel, r, k, m, link))
            # The CPU baseline at N > 1: rank 0 alone, after every GPU leg,
            # 1 thread (the reference's single-threaded client loop).
            parallel.barrier(r)
            if rank == 0:
                cpu = cpu_baseline(k, m, S, args.cpu_seconds, multi=False)
            parallel.barrier(r, sync_gpu=False)
    traffic = pmc_traffic(k, m, S, B, 0 if args.layout == "packed" else lay.granule)
    traffic_source = "profiles/pmc_traffic.json (committed rocprofv3 --pmc summary)"
    if live_traffic and live_traffic.get("hbm_bytes_per_launch"):
        traffic, traffic_source = live_traffic["hbm_bytes_per_launch"], "rocprofv3 --pmc passes in this run"

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
                "hbm_layout": ("packed shards" if args.layout == "packed"
                               else f"granule layout, {lay.granule // 1024} KiB granules"),
            },
            "verified": ok,
            "verified_vs_oracle": oracle_ok,
            "oracle_check": oracle_check["note"],
            "devices": ranks,
            "distinct_gpus": distinct,
            "backend": r.backend,
            "rank_avg_launch_ms_min": fast_ms,
            "rank_avg_launch_ms_max": slow_ms,
            "host_link": link,
            "roofline": roofline_object(world, achieved, traffic, traffic_source, live_traffic, k, m, alg_bytes,
                                        slow_ms, fast_ms, launch_ms, median_ms, extra),
            "cpu_baseline": cpu,
            "extra": extra,
        }
        # configs[3]'s legs last in `extra`: the driver's record keeps the tail
        # of stdout, and this is the one config without a driver-kept key otherwise
        extra_sorted = {k: v for k, v in extra.items() if not k.startswith("cfg3_strong")}
        extra_sorted.update({k: v for k, v in extra.items() if k.startswith("cfg3_strong")})
        line["extra"] = extra_sorted
        print(json.dumps(line), flush=True)
    parallel.shutdown(r)
    return 0


# The driver keeps the first 23 keys of `roofline` (BENCH_r05): the contract's
# six first, then the legs' fractions that matter most at this N, the rest
# after them, the bookkeeping last.
FIRST_N1 = ["c2_dec2_frac", "c3_enc_frac", "c3_enc_granule_frac", "c4_enc_frac", "c4_enc_granule_frac",
            "file_enc_frac", "file_dec_frac", "shard_major_dec01_frac", "group_major_bits_frac", "host_enc_link_frac",
            "host_file_enc_link_frac", "host_groups_link_frac", "host_jni_enc_link_frac",
            "host_jni_file_enc_link_frac", "host_dec_1000B_us", "host_enc_4K_us", "verify_frac"]
FIRST_NN = ["c2_dec2_frac", "c3_enc_frac", "c3_enc_granule_frac", "c3_dec4_frac", "c3_dec4_granule_frac",
            "sustained_frac", "host_pinned_all_ranks_frac_of_N_links", "host_pageable_all_ranks_frac_of_N_links",
            "host_pageable_all_ranks_GiBps", "host_pinned_all_ranks_GiBps"]


def roofline_object(world, achieved, traffic, traffic_source, live_traffic, k, m, alg_bytes, slow_ms, fast_ms,
                    launch_ms, median_ms, extra):
    head = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic}
    summary = decode_summary(extra)
    first = FIRST_N1 if world == 1 else FIRST_NN
    obj = dict(head)
    obj.update({key: summary.get(key) for key in first})
    obj.update({key: v for key, v in summary.items() if key not in obj})
    obj.update({
        "kernel": f"gf_vec_kernel<{k},{m},false> (rs_encode_batch_dev)",
        "alg_bytes_per_launch": alg_bytes,
        "avg_launch_ms": round(launch_ms, 4),
        # also as a fraction of the measured device copy kernel
        "frac_of_copy_kernel": (round(achieved / extra["copy_kernel_GBps"], 4)
                                if extra.get("copy_kernel_GBps") else None),
        "traffic_live": live_traffic,
        "traffic_source": traffic_source,
        "achieved_basis": ("the slowest rank's mean HIP-event launch time; per GPU" if world > 1
                           else "mean HIP-event launch time"),
        "frac_per_gpu_min": round(alg_bytes / (slow_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        "frac_per_gpu_max": round(alg_bytes / (fast_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        "aggregate_achieved": round(world * alg_bytes / (slow_ms * 1e-3) / 1e9, 1),
        "aggregate_peak": world * HBM_PEAK_GBPS,
        "median_launch_ms": round(median_ms, 4),  # SURVEY 8(d) asks for the median too
    })
    return obj


def decode_summary(extra):
    """Short roofline keys for every leg: fractions of 8 TB/s for the device
    legs, of the measured link bound for the host legs, microseconds for the
    small calls (None where the leg did not run, e.g. at N > 1)."""
    g = extra.get
    d01 = g("decode_0_1_hbm_frac") or g("decode_0_1_all_ranks_hbm_frac_per_gpu")
    return {
        "c2_dec1_frac": g("decode_0_hbm_frac"), "c2_dec2_frac": d01,
        "decode_0_5_frac": g("decode_0_5_hbm_frac"),
        "decode_patterns_min": g("decode_patterns_min"),
        "decode_2_erasures_target_0_50_met": (d01 >= 0.50 and (g("decode_0_5_hbm_frac") or 1) >= 0.50)
        if d01 is not None else None,
        # configs[2]-[4] (BASELINE.json), the master's recovery (f2), the fused
        # file layout (f1), verify (f3), and the host-inclusive legs against the
        # link bound
        "c3_enc_frac": g("cfg3_strong_encode_hbm_frac_per_gpu"),
        "c3_dec4_frac": g("cfg3_strong_decode_hbm_frac_per_gpu"),
        "c3_enc_pad_frac": g("cfg3_strong_stride_rec_encode_hbm_frac_per_gpu"),
        "c3_dec4_pad_frac": g("cfg3_strong_stride_rec_decode_hbm_frac_per_gpu"),
        "c3_enc_granule_frac": g("cfg3_strong_granule32K_encode_hbm_frac_per_gpu"),
        "c3_dec4_granule_frac": g("cfg3_strong_granule32K_decode_hbm_frac_per_gpu"),
        "c3_x128_enc_frac": g("cfg3_10p4_4MiB_x128_encode_hbm_frac"),
        "c4_enc_frac": g("cfg4_4p2_4KiB_x1M_encode_hbm_frac"), "c4_dec2_frac": g("cfg4_4p2_4KiB_x1M_decode_hbm_frac"),
        "c4_enc_granule_frac": g("granule_4p2_4KiB_x1M_encode_hbm_frac"),
        "c4_dec2_granule_frac": g("granule_4p2_4KiB_x1M_decode_hbm_frac"),
        "c4_patterns_bits_granule_frac": g("granule_4p2_4KiB_x1M_decode_masked_bits_hbm_frac"),
        "packed_enc_frac": g("packed_4p2_1MiB_x4096_encode_hbm_frac"),
        "verify_frac": g("verify_hbm_frac"),
        "sustained_frac": g("sustained_hbm_frac"),
        "shard_major_enc_frac": g("chunk_groups_4p2_1000B_x4M_shard_major_encode_hbm_frac"),
        "shard_major_dec0_frac": g("chunk_groups_4p2_1000B_x4M_shard_major_decode_0_hbm_frac"),
        "shard_major_dec01_frac": g("chunk_groups_4p2_1000B_x4M_shard_major_decode_0_1_hbm_frac"),
        "shard_major_dec05_frac": g("chunk_groups_4p2_1000B_x4M_shard_major_decode_0_5_hbm_frac"),
        "shard_major_grows_frac": g("chunk_groups_4p2_1000B_x4M_shard_major_decode_grows_hbm_frac"),
        "group_major_enc_frac": g("chunk_groups_4p2_1000B_x4M_encode_hbm_frac"),
        "group_major_dec01_frac": g("chunk_groups_4p2_1000B_x4M_decode_0_1_hbm_frac"),
        "group_major_bits_frac": g("chunk_groups_4p2_1000B_x4M_decode_masked_bits_hbm_frac"),
        "file_enc_frac": g("file_encode_hbm_frac"), "file_dec_frac": g("file_decode_hbm_frac"),
        "host_enc_GiBps": g("host_inclusive_encode_GiBps"),
        "host_enc_link_frac": g("host_inclusive_encode_frac_of_link_bound"),
        "host_dec01_link_frac": g("host_inclusive_decode_0_1_frac_of_link_bound"),
        "host_file_enc_GiBps": g("host_inclusive_file_encode_GiBps"),
        "host_file_enc_link_frac": g("host_inclusive_file_encode_frac_of_link_bound"),
        "host_file_dec_link_frac": g("host_inclusive_file_decode_0_5_frac_of_link_bound"),
        "host_file_enc_all_gpu_link_frac": g("host_inclusive_file_encode_frac_of_all_gpu_link_bound"),
        "host_file_dec_all_gpu_link_frac": g("host_inclusive_file_decode_0_5_frac_of_all_gpu_link_bound"),
        "host_pinned_enc_link_frac": g("host_inclusive_pinned_encode_frac_of_link_bound"),
        "host_pinned_file_enc_link_frac": g("host_inclusive_pinned_file_encode_frac_of_link_bound"),
        "host_pinned_file_dec_link_frac": g("host_inclusive_pinned_file_decode_0_5_frac_of_link_bound"),
        # the master's recovery on its host arrays (NativeReedSolomon.recoverGroupsShardMajor)
        "host_groups_GiBps": g("host_groups_dec0_GiBps"),
        "host_groups_link_frac": g("host_groups_dec0_frac_of_link_bound"),
        "host_groups_grows_link_frac": g("host_groups_grows_frac_of_link_bound"),
        # a JVM caller: the JNI core over the mock JNIEnv
        "host_jni_enc_link_frac": g("host_jni_encode_frac_of_link_bound"),
        "host_jni_dec01_link_frac": g("host_jni_decode_0_1_frac_of_link_bound"),
        "host_jni_file_enc_link_frac": g("host_jni_file_encode_frac_of_link_bound"),
        "host_jni_file_dec_link_frac": g("host_jni_file_decode_0_5_frac_of_link_bound"),
        # small calls, microseconds per call from C
        "host_dec_1000B_us": g("host_dec_1000B_us"), "host_enc_4K_us": g("host_enc_4K_us"),
        "host_jni_dec_1000B_us": g("host_jni_dec_1000B_us"), "host_jni_enc_4K_us": g("host_jni_enc_4K_us"),
        "cpu_port_dec_1000B_us": g("cpu_port_dec_1000B_us"),
        "host_file_enc_88K_us": g("host_file_enc_88K_us"), "host_file_dec05_88K_us": g("host_file_dec05_88K_us"),
        "host_enc_64K_us": g("host_enc_64K_us"), "host_enc_256K_us": g("host_enc_256K_us"),
        "host_enc_1M_us": g("host_enc_1024K_us"),
        "host_enc_4M_us": g("host_enc_4096K_us"),
        "host_file_enc_1M_us": g("host_file_enc_1M_us"), "host_file_dec05_1M_us": g("host_file_dec05_1M_us"),
        # N > 1: every rank calling the host API at once
        "host_pinned_all_ranks_GiBps": g("host_inclusive_pinned_encode_all_ranks_GiBps"),
        "host_pageable_all_ranks_GiBps": g("host_inclusive_pageable_encode_all_ranks_GiBps"),
        "host_pinned_all_ranks_frac_of_N_links": g("host_inclusive_pinned_encode_all_ranks_frac_of_N_links"),
        "host_pageable_all_ranks_frac_of_N_links": g("host_inclusive_pageable_encode_all_ranks_frac_of_N_links"),
    }


def device_refusal(backend, world, ranks):
    """Why a line of `world` ranks with these device identities must not be
    reported, or None.  Under RCCL ("nccl") every rank owns a GPU, so N ranks
    must sit on N distinct GPUs; gloo is how ranks share one GPU on purpose
    (rehearsals) and the line then says distinct_gpus < n_gpus."""
    from rsamd import parallel
    if len(ranks) != world:
        return f"{len(ranks)} device records for {world} ranks"
    distinct = parallel.distinct_devices(ranks)
    if backend == "nccl" and distinct != world:
        return f"{world} nccl ranks ran on {distinct} distinct GPU(s) ({[d.get('pci') for d in ranks]})"
    return None


def check_vs_oracle(torch, rdev, buf, lay, k, m, S, B, stripe0, stream):
    """The timed batch against the oracle: stripes {0, 1, B/2, B-1} of this
    rank are gathered to the host (rs_granule_copy_shard for the granule
    layout, a slice copy for packed shards) and compared, data and parity
    bytes, with the oracle's restatement of encodeParity
    (ReedSolomon.java:90-104) on the same synthetic bytes.  The oracle is the
    checker here: nothing it computes feeds the timed path."""
    import numpy as np
    from oracle import c_ref
    oc = c_ref.Codec(k, m)  # (builds the oracle only if it is missing; the build is atomic)
    picks = sorted({0, min(1, B - 1), B // 2, B - 1})
    ok = True
    for t in picks:
        got = [np.empty(S, np.uint8) for _ in range(k + m)]
        for s_ in range(k + m):
            if isinstance(lay, rdev.GranuleLayout):
                rdev.copy_shard(lay, buf.data_ptr(), t, s_, got[s_].ctypes.data, False, stream)
            else:
                tv = buf.tensor() if isinstance(buf, rdev.DeviceBuffer) else buf
                off = t * lay.stripe_stride + s_ * lay.shard_stride
                got[s_][:] = tv[off: off + S].cpu().numpy()
        torch.cuda.synchronize()
        data = c_ref.synthetic_shards(k, S, SEED, stripe0 + t,
                                      lay.granule if isinstance(lay, rdev.GranuleLayout) else 0)
        ref = [data[i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        oc.encode_parity(ref, 0, S)
        ok = ok and all(np.array_equal(a, b) for a, b in zip(got, ref))
    return {"ok": bool(ok), "note": f"stripes {picks} of each rank's batch, all {k + m} shards gathered from HBM "
                                    f"after the timed region, equal to oracle/rs_oracle.c encodeParity: {bool(ok)}"}


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


def decode_all_ranks(torch, parallel, r, rs, rdev, buf, lay, stream, k, m, S, B, iters):
    """BASELINE configs[2] at N GPUs: every rank decodes erasures {0,1} of its
    own B stripes at once.  Afterwards shards 0 and 1 are overwritten with
    other bytes, decoded once more and the batch verified, so a decode that
    wrote nothing cannot pass."""
    present = [i not in (0, 1) for i in range(k + m)]
    t = timed_all_ranks(torch, parallel, r, lambda: rdev.decode(rs, buf.data_ptr(), present, lay, stream), iters)
    rdev.fill_synthetic(buf.data_ptr(), 2, lay, SEED ^ 0xBAD, 0, stream)  # clobber shards 0 and 1
    rdev.decode(rs, buf.data_ptr(), present, lay, stream)
    flag = torch.zeros(1, dtype=torch.int32, device=buf.device)
    rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream)
    ok = parallel.all_ranks_true(r, int(flag.item()) == 0)
    return {"decode_0_1_all_ranks_GiBps": round(r.world * k * S * B / t / 2**30, 2),
            "decode_0_1_all_ranks_hbm_frac_per_gpu": round((k + 2) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4),
            "decode_0_1_all_ranks_verified": ok}


def sustained(torch, parallel, r, rs, rdev, buf, lay, stream, k, m, S, B, seconds):
    """>= `seconds` of back-to-back headline encodes on every rank (so the
    rate is seen at thermal steady state, not over an 80 ms burst), with the
    GPU clocks sampled from sysfs meanwhile."""
    sampler = ClockSampler(pci=pci_address(torch))
    rdev.encode(rs, buf.data_ptr(), lay, stream)
    parallel.barrier(r)
    sampler.start()
    t0, n = time.perf_counter(), 0
    while True:
        for _ in range(32):
            rdev.encode(rs, buf.data_ptr(), lay, stream)
        n += 32
        torch.cuda.synchronize()
        if time.perf_counter() - t0 >= seconds:
            break
    el = time.perf_counter() - t0
    clocks = sampler.stop()
    parallel.barrier(r)
    el_max = parallel.max_over_ranks(r, el)
    n_all = parallel.sum_over_ranks(r, float(n))
    out = {"sustained_seconds": round(el_max, 2), "sustained_launches_all_ranks": int(n_all),
           "sustained_GiBps": round(k * S * B * n_all / el_max / 2**30, 2),
           "sustained_hbm_frac": round((k + m) * S * B * n / el / 1e9 / HBM_PEAK_GBPS, 4),
           "sustained_clocks": clocks}
    return out


def pci_address(torch):
    """PCI address prefix ("dddd:bb:dd.") of this rank's GPU, or None."""
    try:
        p = torch.cuda.get_device_properties(torch.cuda.current_device())
        return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}."
    except (AttributeError, RuntimeError):
        return None


class ClockSampler:
    """Samples busy %, SCLK and MCLK every 0.25 s on a thread.  With pci (this
    rank's GPU, pci_address()) only the DRM card at that PCI address is read
    -- the node's other GPUs may be busy with other jobs; without it, or when
    no card matches, stop() reports the busiest card's samples."""

    def __init__(self, period=0.25, pci=None, root="/sys/class/drm"):
        import glob
        self.cards = sorted(d for d in glob.glob(root + "/card*/device") if os.path.exists(d + "/pp_dpm_sclk"))
        mine = [d for d in self.cards if pci and os.path.basename(os.path.realpath(d)).startswith(pci)]
        self.matched = bool(mine)
        if mine:
            self.cards = mine[:1]
        self.period, self.samples, self._stop = period, {c: [] for c in self.cards}, threading.Event()
        self._t = threading.Thread(target=self._loop, daemon=True)

    @staticmethod
    def _read(path):
        try:
            with open(path) as f:
                return f.read()
        except OSError:
            return None

    @staticmethod
    def _current_mhz(text):
        for line in (text or "").splitlines():
            if line.rstrip().endswith("*"):
                for tok in line.split():
                    if tok.lower().endswith("mhz"):
                        try:
                            return float(tok[:-3])
                        except ValueError:
                            return None
        return None

    def _loop(self):
        while not self._stop.wait(self.period):
            for c in self.cards:
                busy = self._read(c + "/gpu_busy_percent")
                self.samples[c].append((float(busy) if busy and busy.strip().isdigit() else None,
                                        self._current_mhz(self._read(c + "/pp_dpm_sclk")),
                                        self._current_mhz(self._read(c + "/pp_dpm_mclk"))))

    def start(self):
        self._t.start()

    def stop(self):
        self._stop.set()
        self._t.join(timeout=2)
        if not self.cards:
            return {"source": "sysfs pp_dpm_sclk", "note": "no card exposes pp_dpm_sclk here"}

        def score(c):
            return sum(b or 0 for b, _, _ in self.samples[c])
        c = max(self.cards, key=score)
        s = self.samples[c]

        def med(vals):
            vals = sorted(v for v in vals if v is not None)
            return vals[len(vals) // 2] if vals else None
        return {"source": "sysfs pp_dpm_sclk / pp_dpm_mclk / gpu_busy_percent", "card": c.split("/")[-2],
                "card_pci": os.path.basename(os.path.realpath(c)),
                "card_choice": "this GPU's PCI address" if self.matched else "busiest card (no PCI match)",
                "samples": len(s), "busy_pct_max": max((b for b, _, _ in s if b is not None), default=None),
                "busy_pct_median": med(b for b, _, _ in s), "sclk_mhz_median": med(x for _, x, _ in s),
                "sclk_mhz_min": min((x for _, x, _ in s if x is not None), default=None),
                "mclk_mhz_median": med(x for _, _, x in s)}


def device_extras(torch, rs, rdev, buf, lay, stream, k, m, S, B):
    out = {}
    for miss in [(0,), (0, 1), (0, 5)]:
        present = [i not in miss for i in range(k + m)]
        t = timed(torch, stream, lambda: rdev.decode(rs, buf.data_ptr(), present, lay, stream), 5)
        e = len(miss)
        key = "decode_" + "_".join(map(str, miss))
        out[key + "_GiBps"] = round(k * S * B / t / 2**30, 2)
        out[key + "_hbm_frac"] = round((k + e) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
    out.update(decode_patterns(torch, rs, rdev, buf.data_ptr(), lay, stream, k, m, S, B)[0])
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


def decode_patterns(torch, rs, rdev, base, lay, stream, k, m, S, B, prefix="decode_patterns"):
    """Every erasure pattern of 1..m shards decoded uniformly over the batch
    (after one warm-up, back to back: 2 untimed and 5 timed calls each),
    fractions of 8 TB/s of (k + e) * S * B.  On the granule layout the
    patterns whose rebuilt shards fill whole 128 KiB-aligned blocks run with
    the encode and the rest 4-5 points lower."""
    import itertools
    pats = [mi for e in range(1, m + 1) for mi in itertools.combinations(range(k + m), e)]
    warm(torch, lambda: rdev.decode(rs, base, [i not in pats[0] for i in range(k + m)], lay, stream))
    fr, secs = {}, {}
    for mi in pats:
        present = [i not in mi for i in range(k + m)]
        for _ in range(2):
            rdev.decode(rs, base, present, lay, stream)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(5):
            rdev.decode(rs, base, present, lay, stream)
        e.record(stream)
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / 5 * 1e-3
        secs[mi] = t
        fr["_".join(map(str, mi))] = round((k + len(mi)) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
    v = list(fr.values())
    return {prefix + "_hbm_frac": fr, prefix + "_min": min(v), prefix + "_max": max(v),
            prefix + "_mean": round(sum(v) / len(v), 4)}, secs


def cfg3_strong(torch, rsamd, parallel, r, rdev, dev, stream, total, iters):
    """BASELINE configs[3]: 10+4 x 4 MiB, `total` stripes split across the
    ranks by stripe index (strong scaling), encode then a {0,1,2,3} decode,
    every rank at once.  GiB/s = all data bytes / the slowest rank's time.
    The pool is one contiguous range, as the headline's."""
    from rsamd.device import StripeLayout
    k, m, S = 10, 4, 4 << 20
    start, count = parallel.stripe_partition(total, r.world, r.rank)
    most = parallel.stripe_partition(total, r.world, 0)[1]  # rank 0 holds the largest share
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(count, k + m, S)
    rlay = StripeLayout.recommended(count, k + m, S)  # rs_shard_stride_recommended (include/rs_amd.h)
    pool = rdev.DeviceBuffer(max(lay.nbytes, rlay.nbytes), contiguous=True)
    base = pool.data_ptr()
    rdev.fill_synthetic(base, k, lay, SEED, start, stream)
    n = max(3, iters // 2)
    out = {"cfg3_strong_note": f"10+4 x 4 MiB, {total} stripes split over {r.world} GPU(s) "
                               f"({most} on the busiest), every rank at once, {alloc_note(pool.contiguous)}"}
    t = timed_all_ranks(torch, parallel, r, lambda: rdev.encode(rs, base, lay, stream), n)
    out["cfg3_strong_encode_GiBps"] = round(k * S * total / t / 2**30, 2)
    out["cfg3_strong_encode_hbm_frac_per_gpu"] = round((k + m) * S * most / t / 1e9 / HBM_PEAK_GBPS, 4)
    miss = (0, 1, 2, 3)
    present = [i not in miss for i in range(k + m)]
    t = timed_all_ranks(torch, parallel, r, lambda: rdev.decode(rs, base, present, lay, stream), n)
    out["cfg3_strong_decode_0_1_2_3_GiBps"] = round(k * S * total / t / 2**30, 2)
    out["cfg3_strong_decode_hbm_frac_per_gpu"] = round((k + len(miss)) * S * most / t / 1e9 / HBM_PEAK_GBPS, 4)
    rdev.fill_synthetic(base, len(miss), lay, SEED ^ 0xBAD, 0, stream)  # the decode must rewrite shards 0-3
    rdev.decode(rs, base, present, lay, stream)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    rdev.verify(rs, base, lay, flag.data_ptr(), stream)
    out["cfg3_strong_verified"] = parallel.all_ranks_true(r, int(flag.item()) == 0)
    # the same [stripe][shard][stride] layout at the recommended shard stride
    if rlay.shard_stride != lay.shard_stride:
        rdev.fill_synthetic(base, k, rlay, SEED, start, stream)
        out["cfg3_strong_stride_rec"] = rlay.shard_stride
        t = timed_all_ranks(torch, parallel, r, lambda: rdev.encode(rs, base, rlay, stream), n)
        out["cfg3_strong_stride_rec_encode_hbm_frac_per_gpu"] = round((k + m) * S * most / t / 1e9 / HBM_PEAK_GBPS, 4)
        t = timed_all_ranks(torch, parallel, r, lambda: rdev.decode(rs, base, present, rlay, stream), n)
        out["cfg3_strong_stride_rec_decode_hbm_frac_per_gpu"] = round((k + len(miss)) * S * most / t / 1e9 /
                                                                      HBM_PEAK_GBPS, 4)
        rdev.fill_synthetic(base, len(miss), rlay, SEED ^ 0xBAD, 0, stream)
        rdev.decode(rs, base, present, rlay, stream)
        flag.zero_()
        rdev.verify(rs, base, rlay, flag.data_ptr(), stream)
        out["cfg3_strong_stride_rec_verified"] = parallel.all_ranks_true(r, int(flag.item()) == 0)
    # the same stripes in the granule layout, on the same pool
    glay = rdev.GranuleLayout.make(count, k + m, S)
    rdev.fill_synthetic(base, k, glay, SEED, start, stream)
    tag = f"cfg3_strong_granule{glay.granule // 1024}K"
    t = timed_all_ranks(torch, parallel, r, lambda: rdev.encode(rs, base, glay, stream), n)
    out[tag + "_encode_GiBps"] = round(k * S * total / t / 2**30, 2)
    out[tag + "_encode_hbm_frac_per_gpu"] = round((k + m) * S * most / t / 1e9 / HBM_PEAK_GBPS, 4)
    t = timed_all_ranks(torch, parallel, r, lambda: rdev.decode(rs, base, present, glay, stream), n)
    out[tag + "_decode_0_1_2_3_GiBps"] = round(k * S * total / t / 2**30, 2)
    out[tag + "_decode_hbm_frac_per_gpu"] = round((k + len(miss)) * S * most / t / 1e9 / HBM_PEAK_GBPS, 4)
    rdev.fill_synthetic(base, len(miss), glay, SEED ^ 0xBAD, 0, stream)
    rdev.decode(rs, base, present, glay, stream)
    flag.zero_()
    rdev.verify(rs, base, glay, flag.data_ptr(), stream)
    out[tag + "_verified"] = parallel.all_ranks_true(r, int(flag.item()) == 0)
    pool.free()
    torch.cuda.empty_cache()
    return out


def granule_legs(torch, rsamd, rdev, dev, stream, headline_layout="granule"):
    """The same stripes in the granule layout (include/rs_amd.h, DESIGN.md
    3.6): the headline batch (4+2 x 1 MiB x 4096, 64 KiB granules),
    config[3]'s per-GPU share (10+4 x 4 MiB x 128, 32 KiB granules) and
    config[4] (4+2 x 4 KiB x 1 M, 16 stripes per 64 KiB granule row), each on
    a contiguous pool: encode, decode, verify; then the erased shards are
    overwritten, decoded and the batch verified."""
    out = packed_headline_leg(torch, rsamd, rdev, dev, stream) if headline_layout == "granule" else {}
    for name, k, m, S, B, miss in [("granule_4p2_1MiB_x4096", 4, 2, 1 << 20, 4096, (0, 1)),
                                   ("granule_10p4_4MiB_x128", 10, 4, 4 << 20, 128, (0, 1, 2, 3)),
                                   ("granule_4p2_4KiB_x1M", 4, 2, 4096, 1 << 20, (0, 1))]:
        if name == "granule_4p2_1MiB_x4096" and headline_layout == "granule":
            continue  # the headline itself
        rs = rsamd.ReedSolomon.create(k, m)
        lay = rdev.GranuleLayout.make(B, k + m, S)
        pool = rdev.DeviceBuffer(lay.nbytes, contiguous=True)
        base = pool.data_ptr()
        rdev.fill_synthetic(base, k, lay, SEED, 0, stream)
        out[name + "_granule_bytes"] = lay.granule
        t = timed(torch, stream, lambda: rdev.encode(rs, base, lay, stream), 10)
        out[name + "_encode_GiBps"] = round(k * S * B / t / 2**30, 2)
        out[name + "_encode_hbm_frac"] = round((k + m) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
        present = [i not in miss for i in range(k + m)]
        t = timed(torch, stream, lambda: rdev.decode(rs, base, present, lay, stream), 10)
        out[name + "_decode_" + "_".join(map(str, miss)) + "_GiBps"] = round(k * S * B / t / 2**30, 2)
        out[name + "_decode_hbm_frac"] = round((k + len(miss)) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        t = timed(torch, stream, lambda: rdev.verify(rs, base, lay, flag.data_ptr(), stream), 5)
        out[name + "_verify_hbm_frac"] = round((k + m) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
        rdev.fill_synthetic(base, len(miss), lay, SEED ^ 0xBAD, 0, stream)  # overwrite the erased shards
        rdev.decode(rs, base, present, lay, stream)
        flag.zero_()
        rdev.verify(rs, base, lay, flag.data_ptr(), stream)
        out[name + "_verified"] = int(flag.item()) == 0
        if k == 10:
            # row f2 in the granule layout: 4 random erasures per stripe (the packed leg's
            # patterns), one bitmask per stripe in HBM, one launch
            import numpy as np
            rng = np.random.default_rng(0)
            pres = np.ones((B, k + m), dtype=bool)
            for t_ in range(B):
                pres[t_, rng.choice(k + m, 4, replace=False)] = False
            bits = torch.from_numpy(rdev.presence_bits(pres).view(np.int32)).to(dev)
            alg = (k * B + int((~pres).sum())) * S
            t = timed(torch, stream, lambda: rdev.decode_masked_bits(rs, base, bits.data_ptr(), lay, 0, stream), 5)
            out[name + "_decode_masked_bits_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)
            rdev.fill_synthetic(base, k, lay, SEED, 0, stream)
            rdev.encode(rs, base, lay, stream)
            granule_clobber(torch, pool.tensor(), lay, pres, dev)
            rdev.decode_masked_bits(rs, base, bits.data_ptr(), lay, 0, stream)
            flag.zero_()
            rdev.verify(rs, base, lay, flag.data_ptr(), stream)
            out[name + "_decode_masked_bits_verified"] = int(flag.item()) == 0
        if S < lay.granule:
            # row f2 for config[4] in the granule layout: the packed leg's random
            # pattern per stripe (<= 2 erasures), 16 stripes of different patterns
            # per granule row, as host flags and as device bitmasks
            import itertools
            import numpy as np
            pats = np.array([[i not in mi for i in range(k + m)] for e in range(3)
                             for mi in itertools.combinations(range(k + m), e)], dtype=bool)
            pres = pats[np.random.default_rng(0).integers(0, len(pats), B)]
            alg = (k * int((~pres).any(axis=1).sum()) + int((~pres).sum())) * S
            t = timed(torch, stream, lambda: rdev.decode_masked(rs, base, pres, lay, stream), 10)
            out[name + "_decode_masked_GiBps"] = round(k * S * B / t / 2**30, 2)
            out[name + "_decode_masked_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)
            bits = torch.from_numpy(rdev.presence_bits(pres).view(np.int32)).to(dev)
            t = timed(torch, stream, lambda: rdev.decode_masked_bits(rs, base, bits.data_ptr(), lay, 0, stream), 5)
            out[name + "_decode_masked_bits_GiBps"] = round(k * S * B / t / 2**30, 2)
            out[name + "_decode_masked_bits_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)
            # the same stripes at their patterns' uniform rates: the time the mix
            # would take if each stripe ran as fast as a batch of its own pattern
            pat_out, secs = decode_patterns(torch, rs, rdev, base, lay, stream, k, m, S, B,
                                            prefix=name + "_decode_patterns")
            out.update(pat_out)
            counts = np.bincount(rdev.presence_bits(pres), minlength=1 << (k + m))
            pred = sum(int(c) * secs[tuple(i for i in range(k + m) if not (w >> i) & 1)] / B
                       for w, c in enumerate(counts) if c and w != (1 << (k + m)) - 1)
            out[name + "_decode_masked_bits_uniform_prediction_hbm_frac"] = round(alg / pred / 1e9 / HBM_PEAK_GBPS, 4)
            out[name + "_decode_masked_bits_time_over_prediction"] = round(t / pred, 4)
            for tag, call in (("_decode_masked", lambda: rdev.decode_masked(rs, base, pres, lay, stream)),
                              ("_decode_masked_bits",
                               lambda: rdev.decode_masked_bits(rs, base, bits.data_ptr(), lay, 0, stream))):
                rdev.fill_synthetic(base, k, lay, SEED, 0, stream)
                rdev.encode(rs, base, lay, stream)
                granule_clobber(torch, pool.tensor(), lay, pres, dev)
                call()
                flag.zero_()
                rdev.verify(rs, base, lay, flag.data_ptr(), stream)
                out[name + tag + "_verified"] = int(flag.item()) == 0
        pool.free()
        torch.cuda.empty_cache()
    return out


def packed_headline_leg(torch, rsamd, rdev, dev, stream):
    """The headline's stripes (4+2 x 1 MiB x 4096) in the packed layout
    (shard s of stripe t at t*6 MiB + s MiB, the shards as contiguous byte
    ranges), on a contiguous pool: encode, decode {0,1} and verify, then
    shards 0-1 overwritten, decoded and verified.  Then the headline's
    granule layout on plain hipMalloc memory: encode and verify."""
    from rsamd.device import StripeLayout
    k, m, S, B = 4, 2, 1 << 20, 4096
    name = "packed_4p2_1MiB_x4096"
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    pool = rdev.DeviceBuffer(lay.nbytes, contiguous=True)
    base = pool.data_ptr()
    rdev.fill_synthetic(base, k, lay, SEED, 0, stream)
    out = {name + "_alloc": alloc_note(pool.contiguous)}
    t = timed(torch, stream, lambda: rdev.encode(rs, base, lay, stream), 20)
    out[name + "_encode_GiBps"] = round(k * S * B / t / 2**30, 2)
    out[name + "_encode_hbm_frac"] = round((k + m) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
    present = [False, False, True, True, True, True]
    t = timed(torch, stream, lambda: rdev.decode(rs, base, present, lay, stream), 10)
    out[name + "_decode_0_1_hbm_frac"] = round((k + 2) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    t = timed(torch, stream, lambda: rdev.verify(rs, base, lay, flag.data_ptr(), stream), 5)
    out[name + "_verify_hbm_frac"] = round((k + m) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
    rdev.fill_synthetic(base, 2, lay, SEED ^ 0xBAD, 0, stream)  # overwrite shards 0 and 1
    rdev.decode(rs, base, present, lay, stream)
    flag.zero_()
    rdev.verify(rs, base, lay, flag.data_ptr(), stream)
    out[name + "_verified"] = int(flag.item()) == 0
    pool.free()
    torch.cuda.empty_cache()
    # The headline's own layout on plain hipMalloc memory (a torch tensor), for
    # callers without rs_dev_alloc's contiguous pools.
    glay = rdev.GranuleLayout.make(B, k + m, S)
    buf = torch.empty(glay.nbytes, dtype=torch.uint8, device=dev)
    rdev.fill_synthetic(buf.data_ptr(), k, glay, SEED, 0, stream)
    t = timed(torch, stream, lambda: rdev.encode(rs, buf.data_ptr(), glay, stream), 20)
    gname = "granule_4p2_1MiB_x4096_hipmalloc"
    out[gname + "_encode_GiBps"] = round(k * S * B / t / 2**30, 2)
    out[gname + "_encode_hbm_frac"] = round((k + m) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
    flag.zero_()
    rdev.verify(rs, buf.data_ptr(), glay, flag.data_ptr(), stream)
    out[gname + "_verified"] = int(flag.item()) == 0
    del buf
    torch.cuda.empty_cache()
    return out


def chunk_group_legs(torch, rsamd, rdev, dev, stream, B=4 << 20):
    out = chunk_group_leg(torch, rsamd, rdev, dev, stream, B, 1000)
    out.update(chunk_group_leg(torch, rsamd, rdev, dev, stream, B, 1024))
    out.update(chunk_group_shard_major_leg(torch, rsamd, rdev, dev, stream, B))
    return out


def chunk_group_shard_major_leg(torch, rsamd, rdev, dev, stream, B):
    """Row f2 in the layout the master's loop implies (MasterImpl.java:733-743,
    794-839): it reads group g's chunk from every present server, and the
    offline set is the same for every group (it only grows when a read fails
    mid-loop), so a batching master holds one array per server with the B
    groups' 1000-byte chunks back to back, [server][group * 1000].  A run of
    groups with one pattern is then ONE stripe of B * 1000-byte shards
    (rs_decode_groups_shard_major_dev).  Encode, decodes {0}, {0,1}, {0,5} with
    the per-group flags passed as the master would (B x 6 host flags, run
    detection inside the timed calls), and a set that grows at group B/2 + 1
    (two runs, the second 8 bytes off a 16-byte boundary).  Each decode is
    verified after the absent chunks were overwritten."""
    import numpy as np
    from rsamd.device import StripeLayout
    from rsamd.recovery import recover_groups_shard_major_dev
    k, m, S, T = 4, 2, 1000, 6
    name = "chunk_groups_4p2_1000B_x4M_shard_major"
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.recommended(1, T, S * B)  # one stripe: server stride = the recommended shard stride
    pool = rdev.DeviceBuffer(lay.nbytes, contiguous=True)
    buf, base = pool.tensor(), pool.data_ptr()
    out = {name + "_layout": f"[server][group * 1000], server stride {lay.shard_stride}"}
    rdev.fill_synthetic(base, k, lay, SEED, 0, stream)
    t = timed(torch, stream, lambda: rdev.encode(rs, base, lay, stream), 10)
    out[name + "_encode_GiBps"] = round(k * S * B / t / 2**30, 2)
    out[name + "_encode_hbm_frac"] = round(T * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    view = buf[: T * lay.shard_stride].view(T, lay.shard_stride)
    cases = {"0": [(0, B, (0,))], "0_1": [(0, B, (0, 1))], "0_5": [(0, B, (0, 5))],
             "grows": [(0, B // 2 + 1, (0,)), (B // 2 + 1, B, (0, 3))]}
    for tag, runs in cases.items():
        pres = np.ones((B, T), bool)
        erased = 0
        for g0, g1, miss in runs:
            pres[g0:g1, list(miss)] = False
            erased += (g1 - g0) * len(miss)
        alg = (k * B + erased) * S
        t = timed(torch, stream, lambda: recover_groups_shard_major_dev(base, lay.shard_stride, pres, S, stream), 10)
        out[name + f"_decode_{tag}_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)
        for g0, g1, miss in runs:
            for j in miss:
                view[j, g0 * S: g1 * S].fill_(0x3C)
        recover_groups_shard_major_dev(base, lay.shard_stride, pres, S, stream)
        flag.zero_()
        rdev.verify(rs, base, lay, flag.data_ptr(), stream)
        out[name + f"_decode_{tag}_verified"] = int(flag.item()) == 0
    del buf, view
    pool.free()
    torch.cuda.empty_cache()
    return out


def chunk_group_leg(torch, rsamd, rdev, dev, stream, B, stride):
    """Row f2 at the DFS's own shard size: the master's recovery decodes one
    6 x 1000-B chunk group at a time (ChunkserverDiskRecoveryMachine.java:34-48,
    MasterImpl.java:794-839).  B = 4 M groups of 4+2 x 1000 B packed back to
    back (stride 1000, 24 GB: the 8-byte-aligned kernels, kernels.hip) or
    with each shard padded to 1 KiB (stride 1024).
    Encode and uniform {0,1} decode, then a random pattern per group
    (<= 2 erasures) as device bitmasks and as host flags; each decode is
    verified after the absent shards were overwritten."""
    import itertools
    import numpy as np
    from rsamd.device import StripeLayout
    k, m, S, T = 4, 2, 1000, 6
    name = "chunk_groups_4p2_1000B_x4M" + ("" if stride == S else f"_stride{stride}")
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout(B, S, stride, T * stride)
    pool = rdev.DeviceBuffer(lay.nbytes, contiguous=True)
    buf, base = pool.tensor(), pool.data_ptr()
    out = {name + "_layout": f"shard stride {stride}, group stride {T * stride}"}
    rdev.fill_synthetic(base, k, lay, SEED, 0, stream)
    t = timed(torch, stream, lambda: rdev.encode(rs, base, lay, stream), 10)
    out[name + "_encode_GiBps"] = round(k * S * B / t / 2**30, 2)
    out[name + "_encode_hbm_frac"] = round(T * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
    present = [False, False, True, True, True, True]
    t = timed(torch, stream, lambda: rdev.decode(rs, base, present, lay, stream), 10)
    out[name + "_decode_0_1_hbm_frac"] = round(T * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    clobber(torch, buf, lay, T, np.tile(np.array(present), (B, 1)), dev)
    rdev.decode(rs, base, present, lay, stream)
    rdev.verify(rs, base, lay, flag.data_ptr(), stream)
    out[name + "_decode_verified"] = int(flag.item()) == 0
    pats = np.array([[i not in mi for i in range(T)] for e in range(3) for mi in itertools.combinations(range(T), e)],
                    dtype=bool)
    pres = pats[np.random.default_rng(0).integers(0, len(pats), B)]
    alg = (k * int((~pres).any(axis=1).sum()) + int((~pres).sum())) * S
    bits = torch.from_numpy(rdev.presence_bits(pres).view(np.int32)).to(dev)
    t = timed(torch, stream, lambda: rdev.decode_masked_bits(rs, base, bits.data_ptr(), lay, 0, stream), 10)
    out[name + "_decode_masked_bits_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)
    out[name + "_decode_masked_bits_groups_per_s"] = round(B / t, 0)
    t = timed(torch, stream, lambda: rdev.decode_masked(rs, base, pres, lay, stream), 10)
    out[name + "_decode_masked_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)
    for tag, call in (("_decode_masked_bits", lambda: rdev.decode_masked_bits(rs, base, bits.data_ptr(), lay, 0,
                                                                              stream)),
                      ("_decode_masked", lambda: rdev.decode_masked(rs, base, pres, lay, stream))):
        clobber(torch, buf, lay, T, pres, dev)
        call()
        flag.zero_()
        rdev.verify(rs, base, lay, flag.data_ptr(), stream)
        out[name + tag + "_verified"] = int(flag.item()) == 0
    del buf, bits
    pool.free()
    torch.cuda.empty_cache()
    return out


def granule_clobber(torch, buf, lay, present, dev):
    """clobber() for a GranuleLayout batch: 0x5A over every absent shard."""
    T, G, S = lay.total_shards, lay.granule, lay.shard_len
    mask = torch.from_numpy(~present).to(dev)
    if S >= G:  # (stripe, granule row of the stripe, shard, G) -> index by (stripe, shard)
        buf.view(lay.n_stripes, S // G, T, G).permute(0, 2, 1, 3)[mask] = 0x5A
    else:  # (granule row, shard, stripe of the row, S) -> index by (row, stripe of the row, shard)
        per = G // S
        buf.view(lay.rows, T, per, S).permute(0, 2, 1, 3)[mask.view(lay.rows, per, T)] = 0x5A


def clobber(torch, buf, lay, total_shards, present, dev):
    """Overwrite every absent shard of a (n_stripes, total_shards) presence
    pattern with 0x5A, so a decode that skips a stripe fails the verify after it."""
    v = buf.view(lay.n_stripes, lay.stripe_stride)[:, : total_shards * lay.shard_stride]
    v = v.view(lay.n_stripes, total_shards, lay.shard_stride)
    mask = torch.from_numpy(~present).to(dev)
    v[mask] = 0x5A


def other_configs(torch, rsamd, rdev, dev, stream, alloc="contiguous"):
    """BASELINE configs[3] per-GPU share at N=8 (10+4 x 4 MiB x 128, packed and
    4 KiB-padded) and configs[4] (4+2 x 4 KiB x 1 M stripes), encode, decode,
    verify, and per-stripe erasure patterns (row f2)."""
    import numpy as np
    from rsamd.device import StripeLayout
    out = {}
    for name, k, m, S, B, miss, pad in [("cfg3_10p4_4MiB_x128", 10, 4, 4 << 20, 128, (0, 1, 2, 3), 0),
                                        ("cfg3_10p4_4MiB_x128_pad4K", 10, 4, 4 << 20, 128, (0, 1, 2, 3), 4096),
                                        ("cfg4_4p2_4KiB_x1M", 4, 2, 4096, 1 << 20, (0, 1), 0)]:
        rs = rsamd.ReedSolomon.create(k, m)
        lay = StripeLayout.packed(B, k + m, S, pad=pad)
        pool = stripe_pool(torch, rdev, lay.nbytes, dev, alloc)
        buf = pool.tensor() if isinstance(pool, rdev.DeviceBuffer) else pool
        rdev.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, stream)
        t = timed(torch, stream, lambda: rdev.encode(rs, buf.data_ptr(), lay, stream), 10)
        out[name + "_encode_GiBps"] = round(k * S * B / t / 2**30, 2)
        out[name + "_encode_hbm_frac"] = round((k + m) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
        present = [i not in miss for i in range(k + m)]
        t = timed(torch, stream, lambda: rdev.decode(rs, buf.data_ptr(), present, lay, stream), 10)
        out[name + "_decode_" + "_".join(map(str, miss)) + "_GiBps"] = round(k * S * B / t / 2**30, 2)
        out[name + "_decode_hbm_frac"] = round((k + len(miss)) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        clobber(torch, buf, lay, k + m, np.tile(np.array(present), (B, 1)), dev)
        rdev.decode(rs, buf.data_ptr(), present, lay, stream)
        rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream)
        out[name + "_verified"] = int(flag.item()) == 0
        # row f3 (isParityCorrect) on the same batch: (k+m)*S*B bytes read
        t = timed(torch, stream, lambda: rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream), 5)
        out[name + "_verify_hbm_frac"] = round((k + m) * S * B / t / 1e9 / HBM_PEAK_GBPS, 4)
        if name == "cfg3_10p4_4MiB_x128":
            # row f2 for the wide code: 4 random erasures per stripe, device bitmasks, one launch
            rng = np.random.default_rng(0)
            present = np.ones((B, k + m), dtype=bool)
            for t_ in range(B):
                present[t_, rng.choice(k + m, 4, replace=False)] = False
            bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).to(dev)
            alg = (k * B + int((~present).sum())) * S
            t = timed(torch, stream, lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0,
                                                                     stream), 5)
            out[name + "_decode_masked_bits_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)
            clobber(torch, buf, lay, k + m, present, dev)
            rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, stream)
            rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream)
            out[name + "_decode_masked_bits_verified"] = int(flag.item()) == 0
        if name.startswith("cfg4"):
            # row f2: a random presence pattern per stripe (<= 2 erasures), one launch
            import itertools
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
            clobber(torch, buf, lay, k + m, present, dev)
            rdev.decode_masked(rs, buf.data_ptr(), present, lay, stream)
            rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream)
            out[name + "_decode_masked_verified"] = int(flag.item()) == 0
            # the same patterns as device-resident bitmasks (no host work per call)
            bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).to(dev)
            t = timed(torch, stream, lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0,
                                                                     stream), 5)
            out[name + "_decode_masked_bits_GiBps"] = round(k * S * B / t / 2**30, 2)
            out[name + "_decode_masked_bits_hbm_frac"] = round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)
            clobber(torch, buf, lay, k + m, present, dev)
            rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, stream)
            rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), stream)
            out[name + "_decode_masked_bits_verified"] = int(flag.item()) == 0
        del buf
        if isinstance(pool, rdev.DeviceBuffer):
            pool.free()
        del pool
        torch.cuda.empty_cache()
    out["other_configs_alloc"] = alloc_note(True) if alloc == "contiguous" else alloc_note(None)
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


# ---------------------------------------------------------------------------
# CPU baseline (the oracle's scalar restatement of the reference loop)
# ---------------------------------------------------------------------------
def host_cpu_share():
    """(threads to use, description): the CPUs this process may run on
    (sched_getaffinity), capped by a cgroup v2 CPU quota when one is set --
    the host's CPU share for this job, which on the GPU box is smaller than
    os.cpu_count()."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, math.floor(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    threads = min(aff, quota) if quota else aff
    model, sockets = "", set()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name") and not model:
                model = line.split(":", 1)[1].strip()
            if line.startswith("physical id"):
                sockets.add(line.split(":", 1)[1].strip())
    except OSError:
        pass
    return threads, {"threads": threads, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                     "os_cpu_count": os.cpu_count(), "sockets": len(sockets) or None, "cpu_model": model}


def cpu_rate(codec, k, m, S, present, threads, budget_s, min_stripes):
    """GiB/s of user data (k*S per stripe) the oracle codes on `threads`
    pthreads, stripes split across them, over >= budget_s."""
    import numpy as np
    from oracle import c_ref
    n = max(min_stripes, threads * 2)
    n = min(n, max(threads, (8 << 30) // ((k + m) * S)))  # <= 8 GiB of host stripes unless a thread has none
    host = np.zeros(n * (k + m) * S, dtype=np.uint8)
    for t in range(n):
        host[t * (k + m) * S: t * (k + m) * S + k * S] = c_ref.fill_synthetic(k * S, SEED, t)
    if present is not None:
        codec.code_stripes(host, n, S, S, (k + m) * S, None, threads)  # parity first, then decode
    done, t0 = 0, time.perf_counter()
    while True:
        codec.code_stripes(host, n, S, S, (k + m) * S, present, threads)
        done += n
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return k * S * done / el / 2**30, done, el


def cpu_baseline(k, m, S, budget_s, multi=True):
    """The oracle's scalar InputOutputByteTable loop (the reference's default
    coding loop, -O2 -fno-tree-vectorize) on host-resident stripes: 1 thread,
    then (multi) the host's CPU share."""
    from oracle import c_ref
    c_ref.build()
    codec = c_ref.Codec(k, m)
    rate, done, el = cpu_rate(codec, k, m, S, None, 1, budget_s, 8)
    threads, share = host_cpu_share()
    if not multi:
        return {"value": round(rate, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
                "sample": f"{done} stripes of {k}+{m} x {S // 1024} KiB encoded by the scalar restatement of "
                          f"InputOutputByteTableCodingLoop (oracle/rs_oracle.c, -O2 -fno-tree-vectorize), "
                          f"{el:.1f} s, host-resident, rank 0 after every GPU leg",
                "cpu_model": share["cpu_model"]}
    rate_mt, done_mt, _ = cpu_rate(codec, k, m, S, None, threads, budget_s / 2, 8)
    # The same at os.cpu_count() threads (the plan's `nproc`):
    # on the GPU box they time-share the job's CPU quota, so this is a check
    # that oversubscribing the share gains nothing, not a larger baseline.
    ncpu = os.cpu_count() or 1
    at_ncpu = None
    if ncpu > threads:
        r_n, d_n, e_n = cpu_rate(codec, k, m, S, None, ncpu, max(1.0, budget_s / 4), 8)
        at_ncpu = {"threads": ncpu, "value": round(r_n, 4), "stripes": d_n, "seconds": round(e_n, 2)}
    return {"value": round(rate, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{done} stripes of {k}+{m} x {S // 1024} KiB encoded by the scalar restatement of "
                      f"InputOutputByteTableCodingLoop (oracle/rs_oracle.c, -O2 -fno-tree-vectorize), "
                      f"{el:.1f} s, host-resident",
            "multi_thread": {"value": round(rate_mt, 4), "stripes": done_mt, **share,
                             "at_os_cpu_count": at_ncpu},
            "cpu_model": share["cpu_model"]}


CPU_CONFIGS = [  # name, k, m, S, erasures (None = encode); BASELINE configs[2..4]
    ("C3_decode_0", 4, 2, 1 << 20, (0,)),
    ("C3_decode_0_1", 4, 2, 1 << 20, (0, 1)),
    ("C4_10p4_4MiB_encode", 10, 4, 4 << 20, None),
    ("C4_10p4_4MiB_decode_0_1_2_3", 10, 4, 4 << 20, (0, 1, 2, 3)),
    ("C5_4KiB_encode", 4, 2, 4096, None),
    ("C5_4KiB_decode_0_1", 4, 2, 4096, (0, 1)),
]


def cpu_configs(budget_s=1.0):
    """The CPU side of BASELINE configs[2..4]: the oracle's decodeMissing /
    encodeParity restatement (two codeSomeShards passes for a decode, as
    ReedSolomon.java:175-272) on 1 thread and on the host's CPU share, each a
    bounded sample of >= budget_s."""
    from oracle import c_ref
    threads, _ = host_cpu_share()
    out = {}
    for name, k, m, S, miss in CPU_CONFIGS:
        codec = c_ref.Codec(k, m)
        present = None if miss is None else [i not in miss for i in range(k + m)]
        min_stripes = max(1, (32 << 20) // ((k + m) * S))
        r1, n1, _ = cpu_rate(codec, k, m, S, present, 1, budget_s, min(min_stripes, 64))
        rn, nn, _ = cpu_rate(codec, k, m, S, present, threads, budget_s, min_stripes)
        out[name] = {"GiBps_1thr": round(r1, 3), f"GiBps_{threads}thr": round(rn, 3), "stripes_1thr": n1,
                     "stripes_mt": nn}
    out["note"] = f"oracle scalar port, host-resident, >= {budget_s} s per sample; GiB/s of k*S user bytes"
    return out


# ---------------------------------------------------------------------------
# Host-resident legs (PCIe-inclusive; never the bench value)
# ---------------------------------------------------------------------------
@contextlib.contextmanager
def gpu_numa_bound(torch, parallel, extra):
    """The host legs run on the CPUs of this GPU's NUMA node, as a deployment
    places one client process per GPU: the legs' host arrays are allocated
    inside, so first touch puts them on that node.  Unbound, the pageable
    direct-path legs read 49.8-52.6 GiB/s by where the scheduler put the
    process; bound 51.5-52.7 (tools/numa_probe.py, profiles/r3/numa_r3s2n.txt).
    The affinity is restored afterwards (the CPU baseline runs unbound)."""
    ident = parallel.device_identity(torch)
    node, cpus = parallel.gpu_numa_cpus(ident.get("pci"))
    saved = os.sched_getaffinity(0)
    bound = bool(cpus)
    if bound:
        os.sched_setaffinity(0, cpus)
    extra["host_legs_numa"] = {"gpu_numa_node": node, "bound_cpus": len(cpus) if bound else 0,
                               "note": "host legs bound to the GPU's NUMA node" if bound
                               else "GPU NUMA node unknown: host legs unbound"}
    try:
        yield
    finally:
        if bound:
            os.sched_setaffinity(0, saved)


def _host_dev_ptr(ptr):
    """Device address of page-locked host memory (hipHostGetDevicePointer)."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    d = C.c_void_p()
    if hip.hipHostGetDevicePointer(C.byref(d), C.c_void_p(ptr), C.c_uint(0)) != 0 or not d.value:
        return None
    return d.value


def host_link(torch, n=64 << 20, reps=8):
    """The host <-> device link measured in this run: pinned n-byte copies
    H2D alone, D2H alone, and both at once on two streams (each direction
    timed by events on its own stream), GB/s -- by the copy engines (torch
    copy_), and by a copy kernel loading or storing the pinned buffer through
    its device mapping (rs_copy_dev), the way the direct host path moves its
    bytes.  The host-inclusive legs are quoted against the larger of the two
    bounds these give (link_bound_GiBps)."""
    from rsamd import device as rdev
    a = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    b = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    pa, pb = _host_dev_ptr(a.data_ptr()), _host_dev_ptr(b.data_ptr())
    kernel_mode = [False]

    def up_fn():
        if kernel_mode[0]:
            rdev.copy(d1.data_ptr(), pa, n, torch.cuda.current_stream())
        else:
            d1.copy_(a, non_blocking=True)

    def down_fn():
        if kernel_mode[0]:
            rdev.copy(pb, d2.data_ptr(), n, torch.cuda.current_stream())
        else:
            b.copy_(d2, non_blocking=True)

    def run(up, down):
        s1, s2 = streams
        ev = {}
        for name, on, st, fn in (("h2d", up, s1, up_fn), ("d2h", down, s2, down_fn)):
            if not on:
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                e0.record(st)
                for _ in range(reps):
                    fn()
                e1.record(st)
            ev[name] = (e0, e1)
        torch.cuda.synchronize()
        return {k: n * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9 for k, (e0, e1) in ev.items()}

    # Warm-up: a fresh process's first ~2 s of two-way copies run the D2H side
    # at 28-33 GB/s instead of 48 (profiles/r3/link_probe_r3zq.txt).
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.5:
        run(True, True)
    h2d, d2h = run(True, False)["h2d"], run(False, True)["d2h"]
    # Both at once: the best of 3 stream pairs.  Streams map onto the
    # process's few hardware queues by creation order, and a pair that lands
    # on one queue serialises the directions (D2H read 28 GB/s instead of 48
    # in one run, bench_r3zp.json): that is the pair, not the link.
    both = None
    for _ in range(3):
        streams[:] = [torch.cuda.Stream(), torch.cuda.Stream()]
        got = run(True, True)
        if both is None or got["h2d"] + got["d2h"] > both["h2d"] + both["d2h"]:
            both = got
    out = {"h2d_GBps": round(h2d, 2), "d2h_GBps": round(d2h, 2),
           "both_h2d_GBps": round(both["h2d"], 2), "both_d2h_GBps": round(both["d2h"], 2),
           "both_GBps": round(both["h2d"] + both["d2h"], 2),
           "note": f"pinned {n >> 20} MiB copies, {reps} per direction, torch copy_ on dedicated streams, "
                   f"each direction timed by HIP events on its own stream, alone and with the other running "
                   f"(best of 3 stream pairs); kernel_*: the same by a copy kernel through the buffers' "
                   f"device mapping"}
    if pa and pb:
        kernel_mode[0] = True
        run(True, True)
        kh, kd = run(True, False)["h2d"], run(False, True)["d2h"]
        kb = run(True, True)
        out["kernel"] = {"h2d_GBps": round(kh, 2), "d2h_GBps": round(kd, 2), "both_h2d_GBps": round(kb["h2d"], 2),
                         "both_d2h_GBps": round(kb["d2h"], 2), "both_GBps": round(kb["h2d"] + kb["d2h"], 2)}
    del a, b, d1, d2
    return out


def link_bound_GiBps(link, up, down):
    """User GiB/s the measured link allows for a call that moves `up` bytes
    H2D and `down` bytes D2H per user byte, with both directions overlapped
    as far as the data allows: while both run, each moves at its rate with
    the other running (both_*); the remainder of the larger direction at its
    rate alone.  With a kernel-driven measurement in `link` as well, the
    larger of the two bounds."""
    if not link:
        return None
    if link.get("kernel"):
        return max(link_bound_GiBps({k: v for k, v in link.items() if k != "kernel"}, up, down),
                   link_bound_GiBps(link["kernel"], up, down))
    h, d = link["h2d_GBps"] * 1e9, link["d2h_GBps"] * 1e9
    hb, db = link.get("both_h2d_GBps", h / 1e9) * 1e9, link.get("both_d2h_GBps", d / 1e9) * 1e9
    tc = min(up / hb, down / db) if down else 0.0  # both directions busy
    t = tc + (up - hb * tc) / h + ((down - db * tc) / d if down else 0.0)
    return round(1 / t / 2**30, 2)


def host_inclusive(rsamd, k, m, link=None):
    """Rates of the JNI-facing host-buffer API on pageable buffers (the
    mirrored pipeline, host.cpp run_mirrored) and on the library's own pinned
    buffers (rs_host_alloc, what NativeReedSolomon.allocatePinned hands a JVM:
    coded in place across the link), each next to the bound of the link
    measured in this run (host_link)."""
    import numpy as np
    from rsamd.layout import file_encode_into, file_layout
    n = 64 << 20
    rng = np.random.default_rng(5)
    sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] + [np.zeros(n, np.uint8) for _ in range(m)]
    rs = rsamd.ReedSolomon.create(k, m)
    out = {}

    def rate(fn, user_bytes, reps=24):
        # 3 untimed calls: the first allocates the staging buffers, and the
        # second of a fresh process still runs at a third of the rate (14.6 ms
        # against 5.6 ms for a 4+2 x 64 MiB encode, tools/host_trace.py).
        # 24 timed calls: a single slow call moved a 5-call mean by 5%
        # (profiles/r3/host_calls_r3zf.txt: pageable calls 5.56-5.65 ms), and
        # the 12-call pinned encode read 0.917 of the link bound in one run
        # against 1.00-1.01 in every other (profiles/r5/bench_r6q.json)
        for _ in range(3):
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
    # the same calls on pinned (page-locked) host buffers from the
    # library's allocator (rsamd.device.HostBuffer = rs_host_alloc)
    from rsamd.device import HostBuffer
    held = []

    def pinned(nbytes):
        held.append(HostBuffer(nbytes))
        return held[-1].array

    pin = [pinned(n) for _ in range(k + m)]
    for a, b in zip(pin, sh):
        a[:] = b
    out["host_inclusive_pinned_encode_GiBps"] = rate(lambda: rs.encodeParity(pin, 0, n), k * n)
    out["host_inclusive_pinned_decode_0_1_GiBps"] = rate(lambda: rs.decodeMissing(pin, present, 0, n), k * n)
    # the file calls on pinned buffers (the direct kernels plus the split / merge on the host)
    pfile = pinned(len(data))
    pfile[:] = data
    pfsh = [pinned(S) for _ in range(k + m)]
    pfout = pinned(len(data))
    out["host_inclusive_pinned_file_encode_GiBps"] = rate(lambda: file_encode_into(rs, pfile, pfsh), len(data))
    out["host_inclusive_pinned_file_decode_0_%d_GiBps" % (k + m - 1)] = rate(
        lambda: file_decode_into(rs, pfsh, fpresent, S, pfout), len(data))
    pinned_file_ok = np.array_equal(pfout, data) and all(np.array_equal(a, b) for a, b in zip(pfsh, fsh))
    out["host_inclusive_file_legs_bit_exact"] = bool(pinned_file_ok and np.array_equal(fout, data))
    del pin, pfile, pfsh, pfout
    for b in held:
        b.free()
    out["host_inclusive_note"] = (f"{k}+{m}, {n >> 20} MiB host shards per call, pageable unless 'pinned' (rs_host_alloc) "
                                  f"(file legs: a {len(data) >> 20} MiB file); PCIe-bound, never the bench value; "
                                  f"pinned calls of >= 64 KiB per shard are coded in place across the link by one "
                                  f"kernel (the direct path, no copies); pageable ones go through the "
                                  f"mirrored pipeline (copied chunk by chunk into the library's device-mapped "
                                  f"pinned slots, overlapped with the link; the library never page-locks caller "
                                  f"memory, DESIGN.md 5.3); pageable file calls keep the split / merge on the "
                                  f"CPU, so only coded bytes cross the link")
    # Each leg against the link bound of the bytes it must move (up / down per
    # user byte): encode k up, m down per k user bytes; decode {0,1} k up, 2
    # down.  The pageable file calls keep the layout on the CPU (capi.cpp
    # file_encode_mirrored / file_decode_mirrored), so only coded bytes cross:
    # file encode 1 up (the data), m/k down (parity); file decode {0,k+m-1} 1 up
    # (the k survivors), 2/k down (the rebuilt shards).  Their *_all_gpu_* keys
    # keep round 4's bound, where the GPU also did the layout and moved every
    # shard (file encode (k+m)/k down; file decode 1 + 2/k down: the file too).
    fdec = "host_inclusive_file_decode_0_%d_GiBps" % (k + m - 1)
    legs = {"host_inclusive_encode_GiBps": (1.0, m / k), "host_inclusive_pinned_encode_GiBps": (1.0, m / k),
            "host_inclusive_decode_0_1_GiBps": (1.0, 2 / k), "host_inclusive_pinned_decode_0_1_GiBps": (1.0, 2 / k),
            "host_inclusive_file_encode_GiBps": (1.0, m / k), fdec: (1.0, 2.0 / k),
            "host_inclusive_pinned_file_encode_GiBps": (1.0, m / k),
            "host_inclusive_pinned_" + fdec[len("host_inclusive_"):]: (1.0, 2.0 / k)}
    for key, (up, down) in legs.items():
        bound = link_bound_GiBps(link, up, down)
        if bound and key in out:
            out[key.replace("_GiBps", "_link_bound_GiBps")] = bound
            out[key.replace("_GiBps", "_frac_of_link_bound")] = round(out[key] / bound, 4)
    for key, (up, down) in (("host_inclusive_file_encode_GiBps", (1.0, (k + m) / k)), (fdec, (1.0, 1.0 + 2.0 / k))):
        bound = link_bound_GiBps(link, up, down)
        if bound and key in out:
            out[key.replace("_GiBps", "_frac_of_all_gpu_link_bound")] = round(out[key] / bound, 4)
    return out


def _mockjni():
    """The mock JNIEnv over librsamd (tests/jni_mock, built by build()): a C
    caller for the small-call and JNI legs."""
    d = os.path.join(ROOT, "tests", "jni_mock")
    if d not in sys.path:
        sys.path.insert(0, d)
    import mockjni
    return mockjni.load()


def _mock_array(mj, a):
    """A mock Java byte[] holding a copy of NumPy array a."""
    import ctypes as C
    o = mj.mock_new_bytes(len(a))
    if len(a):
        C.memmove(mj.mock_data(o), a.ctypes.data, len(a))
    return o


def _mock_view(mj, o, n):
    import ctypes as C
    import numpy as np
    return np.ctypeslib.as_array(C.cast(mj.mock_data(o), C.POINTER(C.c_uint8)), shape=(n,))


def _mock_objects(mj, arrs):
    objs = mj.mock_new_objects(len(arrs))
    for i, o in enumerate(arrs):
        mj.mock_set(objs, i, o)
    return objs


def host_small_calls(rsamd, k, m, reps=2000):
    """Small host calls per call, median microseconds of `reps` calls from a C
    caller (no Python per call; tests/jni_mock's timing loops): 4+2 x 1000-B
    decodeMissing {0} -- the recovery machine's call per chunk group
    (ChunkserverDiskRecoveryMachine.java:44) -- and 4+2 x 4 KiB encodeParity
    (configs[4]'s stripe), through the C-ABI and through the JNI core over the
    mock JNIEnv (the path a JVM caller takes, minus the JVM's own JNI cost);
    every output checked against the oracle afterwards.  Beside them the
    scalar port's time for the same decode (1 thread, a bounded batch)."""
    import ctypes as C
    import numpy as np
    from rsamd import _lib
    from oracle import c_ref
    mj = _mockjni()
    rs = rsamd.ReedSolomon.create(k, m)
    oc = c_ref.Codec(k, m)
    out, ok = {}, True
    T = k + m
    for S, kind, key in ((1000, 1, "dec_1000B"), (4096, 0, "enc_4K")):
        rng = np.random.default_rng(S)
        want = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        oc.encode_parity(want, 0, S)
        sh = [a.copy() for a in want]
        if kind == 1:
            sh[0][:] = 0x3C
        else:
            for p in range(k, T):
                sh[p][:] = 0
        present = np.array([0] + [1] * (T - 1), np.uint8)
        ptrs = (_lib.u8p * T)(*[a.ctypes.data_as(_lib.u8p) for a in sh])
        lens = (C.c_int64 * T)(*[S] * T)
        us = mj.mock_time_capi(kind, rs.handle, ptrs, T, lens, present.ctypes.data_as(_lib.u8p), S, reps)
        ok = ok and us > 0 and all(np.array_equal(a, b) for a, b in zip(sh, want))
        mj.mock_reset()
        arrs = [_mock_array(mj, a) for a in sh]
        if kind == 1:
            _mock_view(mj, arrs[0], S)[:] = 0x3C
        else:
            for p in range(k, T):
                _mock_view(mj, arrs[p], S)[:] = 0
        pres = mj.mock_new_bools(T)
        C.memmove(mj.mock_data(pres), present.ctypes.data, T)
        usj = mj.mock_time_jni(kind, rs.handle, _mock_objects(mj, arrs), pres, S, reps)
        ok = ok and usj > 0 and all(np.array_equal(_mock_view(mj, o, S), b) for o, b in zip(arrs, want))
        out[f"host_{key}_us"] = round(us, 2)
        out[f"host_jni_{key}_us"] = round(usj, 2)
    # the client's file calls on the reference's own fixture file (90,999 B,
    # tests/golden/reference_test.txt; ClientCLI.java:177 -> ReedSolomonEncoder
    # / ReedSolomonDecoder), 1000-B blocks: encode, and decode with {0,5} absent
    blk = 1000
    with open(os.path.join(ROOT, "tests", "golden", "reference_test.txt"), "rb") as f:
        fdata = np.frombuffer(f.read(), np.uint8).copy()
    fref = oc.file_encode(fdata.tobytes(), blk)
    S = fref.shape[1]
    fsh = [np.zeros(S, np.uint8) for _ in range(T)]
    fptrs = (_lib.u8p * T)(*[a.ctypes.data_as(_lib.u8p) for a in fsh])
    flens = (C.c_int64 * T)(*[S] * T)
    fout = np.zeros(len(fdata), np.uint8)
    src = fdata.ctypes.data_as(_lib.u8p)
    us = mj.mock_time_capi_file(0, rs.handle, src, len(fdata), blk, fptrs, T, flens, None, None, reps)
    ok = ok and us > 0 and np.array_equal(np.stack(fsh), fref)
    out["host_file_enc_88K_us"] = round(us, 2)
    fpres = np.array([0] + [1] * (T - 2) + [0], np.uint8)
    fsh[0][:] = 0x3C
    fsh[T - 1][:] = 0x3C
    us = mj.mock_time_capi_file(1, rs.handle, src, len(fdata), blk, fptrs, T, flens,
                                fpres.ctypes.data_as(_lib.u8p), fout.ctypes.data_as(_lib.u8p), reps)
    ok = ok and us > 0 and np.array_equal(fout, fdata) and np.array_equal(np.stack(fsh), fref)
    out["host_file_dec05_88K_us"] = round(us, 2)
    rate, n, el = cpu_rate(oc, k, m, 1000, [False] + [True] * (T - 1), 1, 1.0, 100_000)
    out["cpu_port_dec_1000B_us"] = round(k * 1000 / (rate * 2**30) * 1e6, 3)
    out["host_small_calls_bit_exact"] = bool(ok)
    out["host_small_calls_note"] = (
        f"{k}+{m}, one stripe per call, pageable host arrays; median of {reps} calls from C "
        f"(tests/jni_mock timing loops): host_* through the C-ABI, host_jni_* through jni/rs_jni_core.c over the "
        f"mock JNIEnv; the small-call pass is one signalled direct-kernel launch (DESIGN.md 5.2); "
        f"host_file_*_88K_us: rs_file_encode / rs_file_decode {{0,5}} of the reference's 90,999-B fixture file, "
        f"1000-B blocks; "
        f"cpu_port_dec_1000B_us: the oracle's scalar decodeMissing per 1000-B group, 1 thread, {n} groups in "
        f"{el:.1f} s")
    return out


def host_groups_leg(rsamd, k, m, link=None, N=1 << 20, chunk=1000, reps=5):
    """The master's recovery loop on its pageable host arrays
    (rs_decode_groups_shard_major = NativeReedSolomon.recoverGroupsShardMajor;
    MasterImpl.java:733-743, 794-839 with ChunkserverDiskRecoveryMachine.java:
    34-48 per group): k+m arrays of N 1000-B chunks, one per server; offline
    {0} for every group (one run), then a set that grows to {0, k+m-1} at group
    N/2 + 1 (two runs).  GiB/s of user data (k chunks per group) against the
    link bound of the bytes each call moves (the k survivors up, the rebuilt
    chunks down); the rebuilt chunks checked against the oracle on sampled
    groups.  Beside it: the same groups through one decodeMissing per group
    (host_dec_1000B_us) and the scalar port."""
    import numpy as np
    from oracle import c_ref
    from rsamd.recovery import recover_groups_shard_major
    T, L = k + m, N * chunk
    rng = np.random.default_rng(11)
    blk = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
    servers = []
    for i in range(T):
        a = np.empty(L, np.uint8)
        if i < k:
            for o in range(0, L, len(blk)):
                n = min(len(blk), L - o)
                a[o:o + n] = np.roll(blk, 4099 * i)[:n]
        servers.append(a)
    rs = rsamd.ReedSolomon.create(k, m)
    rs.encodeParity(servers, 0, L)
    sample = rng.choice(N, 64, replace=False)
    oc = c_ref.Codec(k, m)
    ok = True
    for g in sample:  # the encode itself, per group, against the oracle
        grp = [s[g * chunk:(g + 1) * chunk].copy() for s in servers]
        ref = [x.copy() for x in grp[:k]] + [np.zeros(chunk, np.uint8) for _ in range(m)]
        oc.encode_parity(ref, 0, chunk)
        ok = ok and all(np.array_equal(x, y) for x, y in zip(grp, ref))
    saved = {s: servers[s].copy() for s in (0, T - 1)}
    out = {}
    j = N // 2 + 1
    for name, down in (("dec0", 1.0 / k), ("grows", (1.0 + (N - j) / N) / k)):
        present = np.ones((N, T), bool)
        present[:, 0] = False
        if name == "grows":
            present[j:, T - 1] = False
        servers[0][:] = 0x3C
        if name == "grows":
            servers[T - 1][j * chunk:] = 0x3C
        for _ in range(2):
            recover_groups_shard_major(servers, present, chunk, k, m)
        t0 = time.perf_counter()
        for _ in range(reps):
            recover_groups_shard_major(servers, present, chunk, k, m)
        t = (time.perf_counter() - t0) / reps
        ok = ok and all(np.array_equal(servers[s], saved[s]) for s in saved)
        key = f"host_groups_{name}_GiBps"
        out[key] = round(k * L / t / 2**30, 3)
        bound = link_bound_GiBps(link, 1.0, down)
        if bound:
            out[key.replace("_GiBps", "_link_bound_GiBps")] = bound
            out[key.replace("_GiBps", "_frac_of_link_bound")] = round(out[key] / bound, 4)
    out["host_groups_bit_exact"] = bool(ok)
    out["host_groups_note"] = (f"{k}+{m} x {chunk}-B chunk groups x {N}, one pageable array per server "
                               f"({L / 1e9:.2f} GB each); one call = every group (runs of one offline set, each "
                               f"one decodeMissing of run-long shards through the mirrored pipeline); {reps} calls "
                               f"timed per leg; dec0: offline {{0}}; grows: {{0}} then {{0,{T - 1}}} from group "
                               f"{j}; GiB/s of k chunks per group")
    del servers, saved
    return out


def host_jni_legs(rsamd, k, m, link=None, n=64 << 20, fbytes=256 << 20, reps=24, huge=1):
    """What a JVM caller gets: the JNI core (jni/rs_jni_core.c, the marshalling
    NativeReedSolomon's natives run) over the mock JNIEnv and librsamd, Java
    byte[] arrays in and out -- one library call per Java call with the arrays
    pinned only around the library's copy batches.  encodeParity and
    decodeMissing {0,1} of 4+2 x 64 MiB, encodeFile / decodeFile {0,5} of a
    256 MiB file, against the link bound of the bytes each moves; outputs
    checked against the numpy-array calls' (themselves oracle-checked)."""
    import numpy as np
    mj = _mockjni()
    mj.mock_reset()
    mj.mock_hugepages(huge)
    rs = rsamd.ReedSolomon.create(k, m)
    T = k + m
    rng = np.random.default_rng(17)
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    ref = data + [np.zeros(n, np.uint8) for _ in range(m)]
    rs.encodeParity(ref, 0, n)
    arrs = [_mock_array(mj, a) for a in ref[:k]] + [mj.mock_new_bytes(n) for _ in range(m)]
    objs = _mock_objects(mj, arrs)
    out = {}

    def rate(fn, user_bytes):
        for _ in range(3):
            fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return round(user_bytes / ((time.perf_counter() - t0) / reps) / 2**30, 3)

    out["host_jni_encode_GiBps"] = rate(lambda: mj.mock_encode_parity(1, rs.handle, objs, 0, n), k * n)
    ok = all(np.array_equal(_mock_view(mj, o, n), r) for o, r in zip(arrs, ref))
    present = mj.mock_new_bools(T)
    _mock_view(mj, present, T)[:] = [0, 0] + [1] * (T - 2)
    _mock_view(mj, arrs[0], n)[:] = 0
    _mock_view(mj, arrs[1], n)[:] = 0
    out["host_jni_decode_0_1_GiBps"] = rate(lambda: mj.mock_decode_missing(1, rs.handle, objs, present, 0, n), k * n)
    ok = ok and all(np.array_equal(_mock_view(mj, o, n), r) for o, r in zip(arrs, ref))
    from rsamd.layout import file_encode_into, file_layout
    fdata = rng.integers(0, 256, fbytes, dtype=np.uint8)
    _, S = file_layout(rs, fbytes)
    fref = [np.zeros(S, np.uint8) for _ in range(T)]
    file_encode_into(rs, fdata, fref)
    farr = _mock_array(mj, fdata)
    fsh = [mj.mock_new_bytes(S) for _ in range(T)]
    fobjs = _mock_objects(mj, fsh)
    out["host_jni_file_encode_GiBps"] = rate(lambda: mj.mock_file_encode(1, rs.handle, farr, 1000, fobjs), fbytes)
    ok = ok and all(np.array_equal(_mock_view(mj, o, S), r) for o, r in zip(fsh, fref))
    fpres = mj.mock_new_bools(T)
    _mock_view(mj, fpres, T)[:] = [0] + [1] * (T - 2) + [0]
    fout = mj.mock_new_bytes(fbytes)
    out["host_jni_file_decode_0_%d_GiBps" % (T - 1)] = rate(
        lambda: mj.mock_file_decode(1, rs.handle, fobjs, fpres, S, 1000, fout, fbytes), fbytes)
    ok = ok and np.array_equal(_mock_view(mj, fout, fbytes), fdata)
    ok = ok and all(np.array_equal(_mock_view(mj, o, S), r) for o, r in zip(fsh, fref))
    exc = mj.mock_exc_class().decode()
    out["host_jni_bit_exact"] = bool(ok and not exc)
    legs = {"host_jni_encode_GiBps": (1.0, m / k), "host_jni_decode_0_1_GiBps": (1.0, 2 / k),
            "host_jni_file_encode_GiBps": (1.0, m / k), "host_jni_file_decode_0_%d_GiBps" % (T - 1): (1.0, 2.0 / k)}
    for key, (up, down) in legs.items():
        bound = link_bound_GiBps(link, up, down)
        if bound:
            out[key.replace("_GiBps", "_frac_of_link_bound")] = round(out[key] / bound, 4)
    out["host_jni_note"] = (f"jni/rs_jni_core.c over the mock JNIEnv (tests/jni_mock) and librsamd: Java byte[] "
                            f"arrays ({k}+{m} x {n >> 20} MiB; a {fbytes >> 20} MiB file, 1000-B blocks) on "
                            f"{'transparent huge pages (a JVM run with -XX:+UseTransparentHugePages, INTEGRATION.md)' if huge else '4 KiB pages'}, "
                            f"one library call per Java call with the arrays movable (pinned only around the "
                            f"library's copy batches, rs_set_relocator); {reps} calls timed per leg")
    mj.mock_hugepages(0)
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
        for _ in range(20):  # steady state: the first calls of a process pay its staging setup
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
    ok = ok and all(np.array_equal(a, b) for a, b in zip(sh, ref)) and np.array_equal(sh[0], data[0])
    # the same two calls from C (tests/jni_mock timing loops: median of 2000,
    # no Python per call), the latency a JNI or C caller sees
    import ctypes as C
    from rsamd import _lib
    mj = _mockjni()
    T = k + m
    ptrs = (_lib.u8p * T)(*[a.ctypes.data_as(_lib.u8p) for a in sh])
    lens = (C.c_int64 * T)(*[S] * T)
    pres = np.array([0] + [1] * (T - 1), np.uint8)
    out["cfg0_gpu_capi_encode_us"] = round(mj.mock_time_capi(0, rs.handle, ptrs, T, lens, None, S, 2000), 2)
    sh[0][:] = 0
    out["cfg0_gpu_capi_decode_0_us"] = round(
        mj.mock_time_capi(1, rs.handle, ptrs, T, lens, pres.ctypes.data_as(_lib.u8p), S, 2000), 2)
    out["cfg0_bit_exact"] = bool(ok and out["cfg0_gpu_capi_encode_us"] > 0 and out["cfg0_gpu_capi_decode_0_us"] > 0
                                 and all(np.array_equal(a, b) for a, b in zip(sh, ref)))
    out["cfg0_note"] = (f"one {k}+{m} stripe of {S >> 10} KiB shards per call, host buffers; GPU = host API "
                        f"(H2D + kernel + D2H) through the Python binding (cfg0_gpu_host_api_*) and from C "
                        f"(cfg0_gpu_capi_*: median of 2000 calls), CPU = oracle scalar port, 1 thread")
    return out


def host_by_size(rsamd, k, m, sizes=(64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20)):
    """Pageable encodeParity per call by shard size (the mid sizes a DFS
    client's files give: the shards are a quarter of the file), microseconds
    per call, each result checked against the oracle (tools/host_sizes.py is
    the full sweep)."""
    import numpy as np
    from oracle import c_ref
    rs = rsamd.ReedSolomon.create(k, m)
    out, ok = {}, True
    for S in sizes:
        rng = np.random.default_rng(S)
        sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        reps = max(5, min(100, (128 << 20) // (k * S)))
        for _ in range(3):
            rs.encodeParity(sh, 0, S)
        t0 = time.perf_counter()
        for _ in range(reps):
            rs.encodeParity(sh, 0, S)
        out[f"host_enc_{S >> 10}K_us"] = round((time.perf_counter() - t0) / reps * 1e6, 1)
        ref = [a.copy() for a in sh[:k]] + [np.zeros(S, np.uint8) for _ in range(m)]
        c_ref.Codec(k, m).encode_parity(ref, 0, S)
        ok = ok and all(np.array_equal(a, b) for a, b in zip(sh, ref))
    # the client's 1 MiB file (1000-byte blocks): encodeFile, then decodeFile with {0, k+m-1} absent
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    F = 1 << 20
    data = np.random.default_rng(F).integers(0, 256, F, dtype=np.uint8)
    _, S = file_layout(rs, F)
    fsh = [np.zeros(S, np.uint8) for _ in range(k + m)]
    fout = np.zeros(F, np.uint8)
    pres = [i not in (0, k + m - 1) for i in range(k + m)]
    for name, fn in (("host_file_enc_1M_us", lambda: file_encode_into(rs, data, fsh)),
                     ("host_file_dec05_1M_us", lambda: file_decode_into(rs, fsh, pres, S, fout))):
        for _ in range(3):
            fn()
        t0 = time.perf_counter()
        for _ in range(50):
            fn()
        out[name] = round((time.perf_counter() - t0) / 50 * 1e6, 1)
    ref = c_ref.Codec(k, m).file_encode(data.tobytes(), 1000)
    ok = ok and np.array_equal(np.stack(fsh), ref) and np.array_equal(fout, data)
    out["host_by_size_bit_exact"] = bool(ok)
    return out


def host_inclusive_all_ranks(rsamd, parallel, r, k, m, link=None, n=64 << 20, reps=4):
    """SURVEY 8(d) host-inclusive rate at N GPUs: every rank calls the
    JNI-facing encodeParity on its own host shards at the same time (pinned,
    then pageable), bracketed by barriers; aggregate user bytes over the
    slowest rank's time.  Bound by the node's PCIe / host memory, not HBM."""
    import numpy as np
    from rsamd.device import HostBuffer
    rng = np.random.default_rng(100 + r.rank)
    rs = rsamd.ReedSolomon.create(k, m)
    held = [HostBuffer(n) for _ in range(k + m)]  # rs_host_alloc: the library's pinned buffers
    pin = [b.array for b in held]
    for a in pin[:k]:
        a[:] = rng.integers(0, 256, n, dtype=np.uint8)
    pageable = [a.copy() for a in pin]
    out = {}
    for name, sh in (("pinned", pin), ("pageable", pageable)):
        for _ in range(3):  # warm-up (staging buffers, pinned mirrors; a fresh process's second call is slow)
            rs.encodeParity(sh, 0, n)
        parallel.barrier(r)
        t0 = time.perf_counter()
        for _ in range(reps):
            rs.encodeParity(sh, 0, n)
        el = parallel.max_over_ranks(r, time.perf_counter() - t0)
        out[f"host_inclusive_{name}_encode_all_ranks_GiBps"] = round(r.world * reps * k * n / el / 2**30, 2)
    out["host_inclusive_all_ranks_note"] = (f"{r.world} ranks at once, {k}+{m} x {n >> 20} MiB host shards per "
                                            f"call, {reps} calls per rank")
    bound = link_bound_GiBps(link, 1.0, m / k)  # rank 0's own link, measured alone
    if bound:
        out["host_inclusive_rank0_link_bound_GiBps"] = bound
        for name in ("pinned", "pageable"):
            out[f"host_inclusive_{name}_encode_all_ranks_frac_of_N_links"] = round(
                out[f"host_inclusive_{name}_encode_all_ranks_GiBps"] / (r.world * bound), 4)
    del pin, pageable
    for b in held:
        b.free()
    return out


def profiled() -> bool:
    """True when this process already runs under rocprofv3 (its tool library is
    preloaded): a nested profiler would fight it, so no live passes then."""
    env = os.environ
    return any("rocprof" in env.get(v, "") for v in ("LD_PRELOAD", "ROCP_TOOL_LIBRARIES", "HSA_TOOLS_LIB")) or \
        any(v.startswith("ROCPROF") for v in env)


def live_pmc_traffic(workload="enc42g", seconds=90):
    """HBM bytes per launch of the headline kernel, measured now: two
    rocprofv3 --pmc children (FETCH_SIZE, then WRITE_SIZE: they do not fit one
    gfx950 TCC pass) over tools/pmc_workloads.py `workload` (enc42g: the
    granule layout, enc42: packed), which fills and encodes the headline
    batch and launches gf_vec_kernel<4,2,false> 3 times.  Bytes =
    (2 * FETCH_SIZE + WRITE_SIZE) KiB, MI355X_MICROARCH.md's gfx950 wide-read
    correction (tools/pmc_summary.py does the same for the committed summary).
    Median over the launches.  Returns None when rocprofv3 is missing, this
    process is itself profiled, or a pass fails or outlives its limit."""
    import csv
    import glob
    import shutil
    import statistics
    import tempfile
    rocprof = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3")
                                            else None)
    if rocprof is None or profiled():
        return None
    kernel = "gf_vec_kernel<4, 2, false>"
    alg = 6 * (1 << 20) * 4096
    vals = {}
    t0 = time.perf_counter()
    env = dict(os.environ, TMPDIR="/tmp")
    with tempfile.TemporaryDirectory(prefix="rsamd_pmc_", dir="/tmp") as tmp:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = ["timeout", "-s", "KILL", str(seconds), rocprof, "--pmc", counter, "--output-format", "csv",
                   "-d", d, "-o", "run", "--", sys.executable, os.path.join(ROOT, "tools", "pmc_workloads.py"),
                   workload]
            try:
                p = subprocess.run(cmd, cwd=tmp, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                   timeout=seconds + 30)
            except (OSError, subprocess.TimeoutExpired):
                return None
            if p.returncode != 0:
                print(f"bench.py: live {counter} pass failed ({p.returncode}); using the committed summary",
                      file=sys.stderr)
                return None
            got = []
            for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
                with open(path) as f:
                    got += [float(row["Counter_Value"]) for row in csv.DictReader(f)
                            if row.get("Counter_Name") == counter and kernel in row.get("Kernel_Name", "")]
            if not got:
                return None
            vals[counter] = (statistics.median(got), len(got))
    (f_kib, nf), (w_kib, nw) = vals["FETCH_SIZE"], vals["WRITE_SIZE"]
    hbm = int(round((2 * f_kib + w_kib) * 1024))
    return {"kernel": kernel, "launches": [nf, nw], "fetch_kib_raw": f_kib, "write_kib_raw": w_kib,
            "hbm_bytes_per_launch": hbm, "alg_bytes_per_launch": alg, "ratio": round(hbm / alg, 4),
            "seconds": round(time.perf_counter() - t0, 1)}


def pmc_traffic(k, m, S, B, granule=0):
    """HBM bytes per launch from the committed rocprofv3 PMC summary for this
    exact workload and layout (profiles/pmc_traffic.json), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        key = f"encode_{k}_{m}_{S}_{B}" + (f"_granule{granule}" if granule else "")
        return d[key]["hbm_bytes_per_launch"] if key in d else None
    except (OSError, ValueError, KeyError):
        return None


if __name__ == "__main__":
    sys.exit(main())
