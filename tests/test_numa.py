"""CPU tests of the NUMA placement of the host legs: rsamd.parallel.gpu_numa_cpus
reads the GPU's node and that node's CPUs from sysfs, and bench.gpu_numa_bound
binds the process there for the legs and restores its affinity afterwards."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd"))
sys.path.insert(0, ROOT)


def _sysfs(tmp_path, pci, node, cpulist):
    dev = tmp_path / "bus/pci/devices" / f"{pci}.0"
    dev.mkdir(parents=True)
    (dev / "numa_node").write_text(f"{node}\n")
    if node >= 0:
        nd = tmp_path / "devices/system/node" / f"node{node}"
        nd.mkdir(parents=True)
        nd.joinpath("cpulist").write_text(cpulist + "\n")
    return str(tmp_path)


def test_cpulist():
    from rsamd.parallel import _cpulist
    assert _cpulist("0-3,8,10-11") == {0, 1, 2, 3, 8, 10, 11}
    assert _cpulist("5") == {5} and _cpulist("") == set()


def test_gpu_numa_cpus(tmp_path):
    from rsamd.parallel import gpu_numa_cpus
    allowed = os.sched_getaffinity(0)
    lo = min(allowed)
    root = _sysfs(tmp_path, "0000:75:00", 1, f"{lo}-{lo + 1},100000")
    node, cpus = gpu_numa_cpus("0000:75:00", sysfs=root)
    assert node == 1 and cpus == {lo, lo + 1} & allowed  # only CPUs this process may use
    assert gpu_numa_cpus(None, sysfs=root) == (None, set())
    assert gpu_numa_cpus("0000:99:00", sysfs=root) == (None, set())  # no such device


def test_gpu_numa_cpus_unknown_node(tmp_path):
    from rsamd.parallel import gpu_numa_cpus
    root = _sysfs(tmp_path, "0000:75:00", -1, "")
    assert gpu_numa_cpus("0000:75:00", sysfs=root) == (None, set())


def test_bench_binds_and_restores(monkeypatch):
    import bench
    from rsamd import parallel
    before = os.sched_getaffinity(0)
    target = {min(before)}
    seen = {}
    monkeypatch.setattr(parallel, "device_identity", lambda torch: {"pci": "x"})
    monkeypatch.setattr(parallel, "gpu_numa_cpus", lambda pci: (3, target))
    extra = {}
    with bench.gpu_numa_bound(None, parallel, extra):
        seen["inside"] = os.sched_getaffinity(0)
    assert seen["inside"] == target
    assert os.sched_getaffinity(0) == before
    assert extra["host_legs_numa"]["gpu_numa_node"] == 3 and extra["host_legs_numa"]["bound_cpus"] == 1
    monkeypatch.setattr(parallel, "gpu_numa_cpus", lambda pci: (None, set()))
    extra = {}
    with bench.gpu_numa_bound(None, parallel, extra):
        assert os.sched_getaffinity(0) == before
    assert extra["host_legs_numa"]["bound_cpus"] == 0
