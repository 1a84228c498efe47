"""Multi-process (world_size 2, gloo, CPU) tests of the stripe-partitioned path.

The GPU path shards stripes across ranks with no data-path collective
(rsamd.parallel).  Here each rank codes its own stripe range with
the CPU oracle (the checker, standing in for the GPU so the test runs on CPU),
and rank 0 checks that the union of the ranks' results equals a single-process
run, and that the timing reductions behave.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    import sys
    for p in (ROOT, PKG_DIR):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), RSAMD_DIST_BACKEND="gloo")
    import torch.distributed as dist
    from oracle import c_ref
    from rsamd import parallel
    try:
        r = parallel.init_from_env(use_gpu=False)
        start, count = parallel.stripe_partition(total, r.world, r.rank)
        k, m, S = 4, 2, 4096
        codec = c_ref.Codec(k, m)
        digests = {}
        for t in range(start, start + count):
            sh = [a for a in c_ref.fill_synthetic(k * S, 0x5EED, t).reshape(k, S)] + \
                 [np.zeros(S, np.uint8) for _ in range(m)]
            sh = [np.ascontiguousarray(a) for a in sh]
            codec.encode_parity(sh, 0, S)
            digests[t] = hashlib.sha256(b"".join(a.tobytes() for a in sh[k:])).hexdigest()
        gathered = [None] * r.world
        dist.all_gather_object(gathered, digests)
        mx = parallel.max_over_ranks(r, float(r.rank + 1))
        sm = parallel.sum_over_ranks(r, float(count))
        ok = parallel.all_ranks_true(r, True)
        bad = parallel.all_ranks_true(r, r.rank == 0)
        parallel.barrier(r, sync_gpu=False)
        if r.rank == 0:
            q.put((gathered, mx, sm, ok, bad))
        parallel.shutdown(r)
    except Exception as e:  # noqa: BLE001
        q.put(("error", repr(e)))
        raise


@pytest.mark.parametrize("total", [8, 7])
def test_two_rank_partition_matches_single_process(oracle_lib, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert res[0] != "error", res
    gathered, mx, sm, ok, bad = res
    merged = {}
    for d in gathered:
        assert not (set(d) & set(merged)), "stripe coded twice"
        merged.update(d)
    assert sorted(merged) == list(range(total))
    assert mx == 2.0 and sm == total and ok is True and bad is False
    # single-process reference
    codec = oracle_lib.Codec(4, 2)
    for t in range(total):
        sh = [np.ascontiguousarray(a) for a in oracle_lib.fill_synthetic(4 * 4096, 0x5EED, t).reshape(4, 4096)]
        sh += [np.zeros(4096, np.uint8) for _ in range(2)]
        codec.encode_parity(sh, 0, 4096)
        assert merged[t] == hashlib.sha256(b"".join(a.tobytes() for a in sh[4:])).hexdigest()


def test_stripe_partition_properties():
    from rsamd.parallel import stripe_partition
    for total in (0, 1, 7, 8, 4096, 4097):
        for world in (1, 2, 3, 8):
            ranges = [stripe_partition(total, world, r) for r in range(world)]
            covered = [t for s, c in ranges for t in range(s, s + c)]
            assert covered == list(range(total))
            assert max(c for _, c in ranges) - min(c for _, c in ranges) <= 1
    with pytest.raises(ValueError):
        stripe_partition(8, 2, 2)
