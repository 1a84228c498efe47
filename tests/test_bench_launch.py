"""CPU tests of bench.py's rank launcher (the driver's `bench.py --gpus N`).

`bench.py --gpus N` with no WORLD_SIZE in the environment must start N ranks
itself (torch.distributed.run as a child process) and relay rank 0's line; under
a launcher, WORLD_SIZE must equal --gpus or the run refuses to report.  The
--launch-probe mode makes the ranks join the process group on CPU (gloo) and
report, so the whole launch path runs here without a GPU.
"""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(kw)
    return env


def test_launch_command_shape():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launch_command(4, ["--gpus", "4", "--steps", "3"], 12345)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=12345" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert os.path.samefile(cmd[-5], BENCH)


def test_self_launch_two_ranks():
    """`bench.py --gpus 2` (no launcher) runs 2 ranks that see each other."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-probe", "--cfg3-stripes", "1024"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    # stdout is the one JSON line and nothing else (gloo's connect messages
    # are kept on stderr: parallel.init_from_env)
    assert len(p.stdout.strip().splitlines()) == 1, p.stdout
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    got = lines[0]
    assert got["n_gpus"] == 2 and got["ranks_seen"] == 2 and got["backend"] == "gloo"
    assert got["cfg3_stripes_covered"] == 1024
    recs = got["records"]  # gathered in rank order, one per process
    assert [d["rank"] for d in recs] == [0, 1] and len({d["pid"] for d in recs}) == 2
    assert [(d["stripe0"], d["stripes"]) for d in recs] == [(0, 512), (512, 512)]


def test_world_size_mismatch_refused():
    """Under a launcher that started a different number of ranks, refuse."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--launch-probe"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE=1" in p.stderr and not p.stdout.strip()


def test_gpus_must_be_positive():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "0"], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 2


FAKE_ROCPROF = r'''#!/bin/bash
# stand-in for rocprofv3 --pmc C --output-format csv -d DIR -o run -- prog...: writes the
# counter CSV layout rocprofv3 writes, 4 launches of the headline kernel plus the fill kernel
while [ "$1" != "--" ]; do case "$1" in --pmc) C=$2; shift;; -d) D=$2; shift;; esac; shift; done
mkdir -p "$D/host/123"
F="$D/host/123/run_counter_collection.csv"
echo 'Kernel_Name,Counter_Name,Counter_Value' > "$F"
echo '"fill_kernel",'$C',999' >> "$F"
for v in 8388600 8388608 8388610 8388700; do
  echo '"void gf_vec_kernel<4, 2, false>(GfArgs)",'$C','$v >> "$F"
done
'''


def test_live_pmc_traffic_parses_and_corrects(tmp_path, monkeypatch):
    """bench.live_pmc_traffic: two child passes, median over the headline
    kernel's launches, FETCH_SIZE doubled (gfx950 wide reads), KiB -> bytes;
    skipped under a profiler."""
    sys.path.insert(0, ROOT)
    import bench
    fake = tmp_path / "rocprofv3"
    fake.write_text(FAKE_ROCPROF)
    fake.chmod(0o755)
    monkeypatch.setenv("PATH", f"{tmp_path}:{os.environ['PATH']}")
    for v in ("LD_PRELOAD", "ROCP_TOOL_LIBRARIES", "HSA_TOOLS_LIB"):
        monkeypatch.delenv(v, raising=False)
    got = bench.live_pmc_traffic(seconds=30)
    assert got["launches"] == [4, 4]
    # medians (8388608 + 8388610) / 2 KiB raw for both; reads 16 GiB, FETCH_SIZE shows half, writes 8 GiB
    assert got["hbm_bytes_per_launch"] == int(round((2 * 8388609 + 8388609) * 1024))
    assert got["alg_bytes_per_launch"] == 6 * (1 << 20) * 4096
    assert abs(got["ratio"] - 1.0) < 1e-4
    monkeypatch.setenv("LD_PRELOAD", "/opt/rocm/lib/librocprofiler-sdk-tool.so")
    assert bench.live_pmc_traffic(seconds=30) is None


def test_clock_sampler_reads_this_gpus_card(tmp_path):
    """The sustained leg's clock samples come from the DRM card at this GPU's
    PCI address, not from the busiest card (a node's other GPUs may run other
    jobs at 100%)."""
    sys.path.insert(0, ROOT)
    import time
    import bench
    for card, bdf, busy, sclk in (("card0", "0000:05:00.0", 100, 2400), ("card8", "0000:75:00.0", 40, 2100)):
        dev = tmp_path / "pci" / bdf
        dev.mkdir(parents=True)
        (dev / "gpu_busy_percent").write_text(f"{busy}\n")
        (dev / "pp_dpm_sclk").write_text(f"0: 500Mhz\n1: {sclk}Mhz *\n")
        (dev / "pp_dpm_mclk").write_text("0: 900Mhz\n1: 2000Mhz *\n")
        (tmp_path / card).mkdir()
        os.symlink(dev, tmp_path / card / "device")
    s = bench.ClockSampler(period=0.01, pci="0000:75:00.", root=str(tmp_path))
    s.start()
    time.sleep(0.1)
    r = s.stop()
    assert r["card"] == "card8" and r["card_pci"] == "0000:75:00.0" and r["sclk_mhz_median"] == 2100
    assert r["card_choice"].startswith("this GPU")
    s = bench.ClockSampler(period=0.01, pci=None, root=str(tmp_path))
    s.start()
    time.sleep(0.1)
    r = s.stop()
    assert r["card"] == "card0" and r["card_choice"].startswith("busiest")


def test_live_pmc_only_at_one_gpu(monkeypatch):
    """The live PMC passes profile cuda:0 from child processes, so a rank of an
    N > 1 run (WORLD_SIZE set by the driver's launcher) must not start them --
    every rank would profile GPU 0 at once.  At N = 1 they run, before run()."""
    sys.path.insert(0, ROOT)
    import bench
    calls = []
    monkeypatch.setattr(bench, "live_pmc_traffic", lambda w: calls.append(("pmc", w)) or {"hbm_bytes_per_launch": 1})
    monkeypatch.setattr(bench, "run", lambda args, live=None: calls.append(("run", args.gpus, live)) or 0)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    assert bench.main(["--gpus", "1"]) == 0  # the headline's default layout: granule
    assert calls == [("pmc", "enc42g"), ("run", 1, {"hbm_bytes_per_launch": 1})]
    calls.clear()
    assert bench.main(["--gpus", "1", "--layout", "packed"]) == 0
    assert calls == [("pmc", "enc42"), ("run", 1, {"hbm_bytes_per_launch": 1})]
    calls.clear()
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    assert bench.main(["--gpus", "2"]) == 0
    assert calls == [("run", 2, None)]


def test_device_refusal_under_nccl():
    """N nccl ranks must sit on N distinct GPUs; gloo rehearsals may share one."""
    sys.path.insert(0, ROOT)
    import bench
    a = {"index": 0, "pci": "0000:05:00", "uuid": "u0"}
    b = {"index": 1, "pci": "0000:15:00", "uuid": "u1"}
    same = dict(a, index=1)
    assert bench.device_refusal("nccl", 2, [a, b]) is None
    msg = bench.device_refusal("nccl", 2, [a, same])
    assert msg and "1 distinct GPU" in msg
    assert bench.device_refusal("gloo", 2, [a, same]) is None
    assert bench.device_refusal("nccl", 2, [a]) is not None  # a missing record
    # no PCI address: the UUID tells the devices apart
    assert bench.device_refusal("nccl", 2, [dict(a, pci=None), dict(b, pci=None)]) is None


def test_link_bound():
    """link_bound_GiBps: both directions overlapped while both have bytes to
    move (at their rates with the other running), then the rest alone."""
    sys.path.insert(0, ROOT)
    import bench
    link = {"h2d_GBps": 50.0, "d2h_GBps": 50.0, "both_h2d_GBps": 40.0, "both_d2h_GBps": 40.0}
    # 1 byte up, 0.5 down per user byte: 12.5 ps both (0.5 up, 0.5 down), then 0.5 up alone in 10 ps
    assert abs(bench.link_bound_GiBps(link, 1.0, 0.5) - 1 / 22.5e-12 / 2**30) < 0.01
    # only uploads: the H2D rate alone
    assert abs(bench.link_bound_GiBps(link, 1.0, 0.0) - 50e9 / 2**30) < 0.01
    # 1 up, 1 down: all of it at the both-ways rates
    assert abs(bench.link_bound_GiBps(link, 1.0, 1.0) - 40e9 / 2**30) < 0.01
    assert bench.link_bound_GiBps(None, 1.0, 0.5) is None
    # a kernel-driven measurement too: the larger of the two bounds
    link2 = dict(link, kernel={"h2d_GBps": 60.0, "d2h_GBps": 45.0, "both_h2d_GBps": 44.0, "both_d2h_GBps": 44.0})
    assert abs(bench.link_bound_GiBps(link2, 1.0, 0.0) - 60e9 / 2**30) < 0.01
    assert abs(bench.link_bound_GiBps(link2, 1.0, 1.0) - 44e9 / 2**30) < 0.01
    link3 = dict(link, kernel={"h2d_GBps": 30.0, "d2h_GBps": 30.0, "both_h2d_GBps": 20.0, "both_d2h_GBps": 20.0})
    assert bench.link_bound_GiBps(link3, 1.0, 0.5) == bench.link_bound_GiBps(link, 1.0, 0.5)


def test_decode_summary_keys():
    """roofline's short decode / config keys, all scalars (what a record that
    keeps only the parsed line's scalar keys shows): taken from the extra legs at N = 1, the all-ranks
    {0,1} leg at N > 1, None where a leg did not run."""
    sys.path.insert(0, ROOT)
    import bench
    ex = {"decode_0_hbm_frac": 0.87, "decode_0_1_hbm_frac": 0.86, "decode_0_5_hbm_frac": 0.85,
          "decode_patterns_min": 0.84, "cfg3_strong_encode_hbm_frac_per_gpu": 0.77,
          "granule_4p2_4KiB_x1M_encode_hbm_frac": 0.87}
    s = bench.decode_summary(ex)
    assert (s["c2_dec1_frac"], s["c2_dec2_frac"], s["decode_0_5_frac"], s["decode_patterns_min"]) == \
        (0.87, 0.86, 0.85, 0.84)
    assert s["decode_2_erasures_target_0_50_met"] is True
    assert s["c3_enc_frac"] == 0.77 and s["c4_enc_granule_frac"] == 0.87
    assert s["c3_enc_pad_frac"] is None
    # every key is a scalar: a record that drops nested objects keeps them all
    assert all(not isinstance(v, (dict, list)) for v in s.values())
    n8 = bench.decode_summary({"decode_0_1_all_ranks_hbm_frac_per_gpu": 0.45})
    assert n8["c2_dec2_frac"] == 0.45 and n8["c2_dec1_frac"] is None
    assert n8["decode_2_erasures_target_0_50_met"] is False
    assert bench.decode_summary({})["decode_2_erasures_target_0_50_met"] is None


def test_roofline_first_keys():
    """The driver keeps the first 23 keys of `roofline`: the contract's six,
    then configs[2]-[4], f1, f2 and the host legs at N = 1 (the multi-GPU legs
    at N > 1); the bookkeeping keys come last."""
    sys.path.insert(0, ROOT)
    import bench
    for world, first in ((1, bench.FIRST_N1), (8, bench.FIRST_NN)):
        obj = bench.roofline_object(world, 6900.0, 1.0, "src", None, 4, 2, 100, 3.7, 3.6, 3.7, 3.7, {})
        keys = list(obj)
        assert keys[:6] == ["bound", "achieved", "peak", "unit", "frac", "traffic"]
        assert keys[6:6 + len(first)] == first and 6 + len(first) <= 23
        assert keys[-1] == "median_launch_ms" and "traffic_source" not in keys[:23]
        assert all(not isinstance(obj[key], (dict, list)) for key in keys[:23])
    for key in ("c3_enc_frac", "c3_enc_granule_frac", "c4_enc_frac", "c4_enc_granule_frac", "file_enc_frac",
                "file_dec_frac", "shard_major_dec01_frac", "group_major_bits_frac", "host_enc_link_frac",
                "host_file_enc_link_frac", "host_groups_link_frac", "host_jni_enc_link_frac",
                "host_jni_file_enc_link_frac", "host_dec_1000B_us", "host_enc_4K_us"):
        assert key in bench.FIRST_N1
    assert "host_pageable_all_ranks_frac_of_N_links" in bench.FIRST_NN
