"""GPU tests: the device-resident calls are capturable in a HIP graph.

rs_encode_batch_dev, rs_verify_batch_dev, rs_decode_batch_dev and
rs_decode_batch_masked_bits_dev only enqueue kernels on the caller's stream
once the codec's device tables exist (the first call per device uploads them),
so a service can capture its per-batch sequence once and replay it, paying
one graph launch instead of one launch per call.  Captured through
torch.cuda.graph on a side stream, replayed over fresh data, and checked
against the oracle, the saved shards and the verify flag.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED


def test_graph_replay_encode_verify_decode(gpu, oracle_lib):
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    k, m, S, B = 4, 2, 4096 + 8, 64  # 16-byte vectors plus an 8-byte tail: both kernels in the graph
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    buf = torch.zeros(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.current_stream()
    miss = [1, 4]
    present = [i not in miss for i in range(k + m)]
    # warm-up outside capture: uploads the encode / verify / decode tables
    device.encode(rs, buf.data_ptr(), lay, st)
    device.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
    device.decode(rs, buf.data_ptr(), present, lay, st)
    torch.cuda.synchronize()

    g_enc, g_dec = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_enc):
        cs = torch.cuda.current_stream()
        flag.zero_()
        device.encode(rs, buf.data_ptr(), lay, cs)
        device.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), cs)
    with torch.cuda.graph(g_dec):
        device.decode(rs, buf.data_ptr(), present, lay, torch.cuda.current_stream())

    v = buf.view(B, k + m, lay.shard_stride)[:, :, :S]
    c = oracle_lib.Codec(k, m)
    for rep in range(3):
        device.fill_synthetic(buf.data_ptr(), k, lay, SEED, 1000 * rep, st)
        v[:, k:, :] = 0
        g_enc.replay()
        torch.cuda.synchronize()
        assert int(flag.item()) == 0, rep
        for t in (0, B // 2, B - 1):
            sh = [x.copy() for x in v[t].cpu().numpy()]
            assert np.array_equal(np.concatenate(sh[:k]), oracle_lib.fill_synthetic(k * S, SEED, 1000 * rep + t))
            ref = [x.copy() for x in sh]
            for p in range(m):
                ref[k + p][:] = 0
            c.encode_parity(ref, 0, S)
            assert all(np.array_equal(a, b) for a, b in zip(sh, ref)), (rep, t)
        saved = v.clone()
        v[:, miss, :] = 0x5A
        g_dec.replay()
        torch.cuda.synchronize()
        assert torch.equal(v, saved), rep


def test_graph_replay_masked_bits(gpu):
    import itertools
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    k, m, S, B = 4, 2, 4096, 4096
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream()
    pats = np.array([[i not in miss for i in range(k + m)] for e in range(3)
                     for miss in itertools.combinations(range(k + m), e)], dtype=bool)
    present = pats[np.random.default_rng(7).integers(0, len(pats), B)]
    bits = torch.from_numpy(device.presence_bits(present).view(np.int32)).to("cuda:0")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, st)
    device.encode(rs, buf.data_ptr(), lay, st)
    device.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, bad.data_ptr(), st)  # warm-up
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        device.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, bad.data_ptr(), torch.cuda.current_stream())
    v = buf.view(B, k + m, S)
    erased = torch.from_numpy(~present).to("cuda:0")
    for rep in range(2):
        device.fill_synthetic(buf.data_ptr(), k, lay, SEED, 77 * (rep + 1), st)
        device.encode(rs, buf.data_ptr(), lay, st)
        saved = v.clone()
        v[erased] = 0xA5
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(v, saved), rep
    assert int(bad.item()) == 0
