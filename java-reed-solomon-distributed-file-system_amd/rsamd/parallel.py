"""Stripe partitioning across GPUs (one process per GPU).

Stripes are independent: GPU g owns a contiguous range
of stripe indices and codes it with no data-path collective.  torch.distributed
is used only to line ranks up for timing and to reduce a few scalars (elapsed
time, verification flags, device identities).  The backend is RCCL ("nccl")
when every rank of this node has a GPU of its own (LOCAL_WORLD_SIZE <= visible
devices, so a multi-node job keeps RCCL); gloo when ranks share a GPU or run on
CPU.  RSAMD_DIST_BACKEND=gloo|nccl overrides the choice.
"""
from __future__ import annotations

import contextlib
import os
import sys
from dataclasses import dataclass


@dataclass(frozen=True)
class Rank:
    rank: int
    world: int
    local: int
    backend: str

    @property
    def distributed(self) -> bool:
        return self.world > 1


def stripe_partition(total_stripes: int, world: int, rank: int):
    """Contiguous [start, start+count) share of `total_stripes` for `rank`;
    shares differ by at most one stripe and cover every stripe exactly once."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    base, extra = divmod(total_stripes, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def init_from_env(use_gpu: bool = True) -> Rank:
    """Read RANK / WORLD_SIZE / LOCAL_RANK (torch.distributed.run), select the
    local GPU and initialise the process group when world > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("RSAMD_DIST_BACKEND")
    import torch
    if backend is None:
        # RCCL needs a device of its own per rank; ranks that share a GPU (more
        # ranks on this node than devices, e.g. a rehearsal on a one-GPU box)
        # line up over gloo.  Per node: LOCAL_WORLD_SIZE, not WORLD_SIZE.
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        backend = "nccl" if use_gpu and torch.cuda.device_count() >= local_world else "gloo"
    if use_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            kw = {}
            if backend == "nccl":
                kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
            # gloo prints "Rank r is connected to ..." on stdout while it
            # connects; the bench's stdout must carry its JSON line only.
            with _stdout_to_stderr():
                dist.init_process_group(backend, **kw)
                dist.barrier()
    return Rank(rank, world, local, backend)


@contextlib.contextmanager
def _stdout_to_stderr():
    """File descriptor 1 points at stderr inside the block (native code
    writing to stdout included)."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def _reduce(r: Rank, value: float, op: str, dtype=None) -> float:
    if not r.distributed:
        return value
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if r.backend == "nccl" else torch.device("cpu")
    t = torch.tensor([value], dtype=dtype or torch.float64, device=dev)
    dist.all_reduce(t, op=getattr(dist.ReduceOp, op))
    return float(t.item())


def max_over_ranks(r: Rank, value: float) -> float:
    return _reduce(r, value, "MAX")


def sum_over_ranks(r: Rank, value: float) -> float:
    return _reduce(r, value, "SUM")


def all_ranks_true(r: Rank, flag: bool) -> bool:
    return _reduce(r, 0.0 if flag else 1.0, "MAX") == 0.0


def barrier(r: Rank, sync_gpu: bool = True) -> None:
    if sync_gpu:
        import torch
        torch.cuda.synchronize()
    if r.distributed:
        import torch.distributed as dist
        dist.barrier()


def shutdown(r: Rank) -> None:
    if r.distributed:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def gather_objects(r: Rank, obj) -> list:
    """obj from every rank, in rank order (a one-element list at world 1)."""
    if not r.distributed:
        return [obj]
    import torch.distributed as dist
    out = [None] * r.world
    dist.all_gather_object(out, obj)
    return out


def device_identity(torch) -> dict:
    """This rank's GPU: torch index, PCI address (domain:bus:device) and UUID
    as the runtime reports them (None where the runtime has no field)."""
    idx = torch.cuda.current_device()
    p = torch.cuda.get_device_properties(idx)
    pci = None
    if all(hasattr(p, a) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id")):
        pci = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    uuid = getattr(p, "uuid", None)
    return {"index": idx, "pci": pci, "uuid": str(uuid) if uuid is not None else None, "name": p.name,
            "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
            or os.environ.get("CUDA_VISIBLE_DEVICES")}


def distinct_devices(identities) -> int:
    """Distinct physical GPUs among rank identities (by PCI address, else
    UUID, else torch index)."""
    keys = set()
    for d in identities:
        keys.add(d.get("pci") or d.get("uuid") or f"index{d.get('index')}")
    return len(keys)


def _cpulist(text: str) -> set:
    """CPU ids of a sysfs cpulist ("0-3,8,10-11")."""
    out = set()
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
    return out


def gpu_numa_cpus(pci, sysfs="/sys"):
    """(NUMA node of the GPU at PCI address `pci` (domain:bus:device), the
    CPUs of that node this process may run on) from sysfs, or (None, set())
    when either is unknown.  A host process that feeds one GPU from its own
    memory runs best there: first touch then places its buffers on the node
    of the GPU's PCIe root (numa_r3s2n.txt)."""
    if not pci:
        return None, set()
    node = None
    for fn in range(8):
        path = os.path.join(sysfs, "bus/pci/devices", f"{pci}.{fn}", "numa_node")
        if os.path.exists(path):
            with open(path) as f:
                node = int(f.read())
            break
    if node is None or node < 0:
        return None, set()
    path = os.path.join(sysfs, "devices/system/node", f"node{node}", "cpulist")
    if not os.path.exists(path):
        return node, set()
    with open(path) as f:
        return node, _cpulist(f.read()) & os.sched_getaffinity(0)
