"""World-2 run of the stripe-partitioned product path on the GPU.

Two spawned ranks share cuda:0 (gloo lines them up: RCCL needs a device per
rank) and each codes ITS stripe_partition share of a global batch through
librsamd -- encode, then a {0,5} decode after the erased shards were
overwritten (the erasure pattern of ReedSolomonTest.java:77-93).  The parent
checks the union of the ranks' bytes against the oracle, stripe by stripe, and
that the shares cover the batch exactly once (independence of stripes:
ReedSolomon.java:90-104; partition: SURVEY.md 8e).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT

pytestmark = pytest.mark.gpu

SEED = 0x5EED
CASES = [(4, 2, 65536, 7, (0, 5)), (10, 4, 12304, 5, (0, 1, 2, 13))]  # k, m, S, global stripes, erasures


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import sys
    for p in (ROOT, PKG_DIR):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import torch
        import torch.distributed as dist

        import rsamd
        from rsamd import device, parallel
        from rsamd.device import StripeLayout
        r = parallel.init_from_env(use_gpu=True)
        assert r.backend == "gloo", r.backend  # two ranks on one device
        st = torch.cuda.current_stream()
        results = []
        for k, m, S, total, miss in CASES:
            start, count = parallel.stripe_partition(total, r.world, r.rank)
            shares = [None] * r.world
            dist.all_gather_object(shares, (start, count))
            rs = rsamd.ReedSolomon.create(k, m)
            lay = StripeLayout.packed(count, k + m, S)
            buf = torch.zeros(lay.nbytes, dtype=torch.uint8, device="cuda")
            device.fill_synthetic(buf.data_ptr(), k, lay, SEED, start, st)
            device.encode(rs, buf.data_ptr(), lay, st)
            encoded = device.view_shards(buf.cpu().numpy(), lay, k + m).copy()
            v = buf.view(count, lay.stripe_stride)[:, : (k + m) * lay.shard_stride].view(count, k + m,
                                                                                        lay.shard_stride)
            for i in miss:
                v[:, i].fill_(0x5A)
            present = [i not in miss for i in range(k + m)]
            device.decode(rs, buf.data_ptr(), present, lay, st)
            decoded = device.view_shards(buf.cpu().numpy(), lay, k + m).copy()
            flag = torch.zeros(1, dtype=torch.int32, device="cuda")
            device.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
            ok = parallel.all_ranks_true(r, int(flag.item()) == 0)
            results.append((start, count, shares, encoded, decoded, ok))
        parallel.barrier(r)
        q.put((rank, results))
        parallel.shutdown(r)
    except Exception as e:  # noqa: BLE001
        q.put((rank, "error: " + repr(e)))
        raise


def test_two_ranks_share_one_gpu_and_match_oracle(gpu, oracle_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(got[r], str), got[r]
    for ci, (k, m, S, total, miss) in enumerate(CASES):
        shares = got[0][ci][2]
        assert shares == got[1][ci][2]
        covered = sorted(t for s, c in shares for t in range(s, s + c))
        assert covered == list(range(total)), shares
        codec = oracle_lib.Codec(k, m)
        for r in (0, 1):
            start, count, _, encoded, decoded, ok = got[r][ci]
            assert ok, f"rank {r} verify flagged a mismatch ({k}+{m})"
            for j in range(count):
                t = start + j
                ref = [np.ascontiguousarray(a) for a in oracle_lib.fill_synthetic(k * S, SEED, t).reshape(k, S)]
                ref += [np.zeros(S, np.uint8) for _ in range(m)]
                codec.encode_parity(ref, 0, S)
                ref = np.stack(ref)
                assert np.array_equal(encoded[j], ref), f"rank {r} stripe {t}: encode differs from the oracle"
                assert np.array_equal(decoded[j], ref), f"rank {r} stripe {t}: decode {miss} differs"
