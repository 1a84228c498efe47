"""GPU tests at the launch-size limit: a dispatch's grid holds at most
2^32 - 1 work-items, i.e. 2^26 - 1 one-wave blocks (kernels.hip
kMaxGridBlocks), so batches with more stripe columns than that are cut into
several launches.  4+2 stripes of one 16-byte vector per shard make one block
per stripe: 2^26 + 1000 stripes (6.4 GB) cross the cut.  Encode, verify,
decode and the per-stripe-bitmask decode are checked on both sides of it
against the oracle and the saved shards.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED
MAX_BLOCKS = (2**32 - 1) // 64  # kernels.hip kMaxGridBlocks


def test_batch_beyond_one_grid(gpu, oracle_lib):
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    k, m, S = 4, 2, 16
    B = MAX_BLOCKS + 1000
    lay = StripeLayout.packed(B, k + m, S, align=16)
    buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream()
    device.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, st)
    v = buf.view(B, k + m, S)
    v[:, k:, :] = 0
    rs = rsamd.ReedSolomon.create(k, m)
    device.encode(rs, buf.data_ptr(), lay, st)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
    assert int(flag.item()) == 0
    c = oracle_lib.Codec(k, m)
    sample = [0, 1, MAX_BLOCKS - 1, MAX_BLOCKS, MAX_BLOCKS + 1, B - 1]
    for t in sample:
        sh = [x.copy() for x in v[t].cpu().numpy()]
        assert np.array_equal(np.concatenate(sh[:k]), oracle_lib.fill_synthetic(k * S, SEED, t)), t
        ref = [x.copy() for x in sh]
        for p in range(m):
            ref[k + p][:] = 0
        c.encode_parity(ref, 0, S)
        assert all(np.array_equal(a, b) for a, b in zip(sh, ref)), t
    # a corrupted byte past the cut is seen
    v[B - 2, 5, 3] ^= 1
    device.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
    assert int(flag.item()) != 0
    v[B - 2, 5, 3] ^= 1
    # erase {0, 5}, decode, compare
    saved = v[:, [0, 5], :].clone()
    v[:, [0, 5], :] = 0
    device.decode(rs, buf.data_ptr(), [False, True, True, True, True, False], lay, st)
    assert torch.equal(v[:, [0, 5], :], saved)
    # per-stripe bitmasks already in HBM: {1, 2} missing everywhere
    saved = v[:, [1, 2], :].clone()
    v[:, [1, 2], :] = 0
    bits = torch.full((B,), 0b111001, dtype=torch.int32, device="cuda:0")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, bad.data_ptr(), st)
    assert int(bad.item()) == 0
    assert torch.equal(v[:, [1, 2], :], saved)
    del buf, v, saved, bits
    torch.cuda.empty_cache()
