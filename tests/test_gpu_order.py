"""GPU tests of the kernels' block order (kernels.hip block_item / block_order).

The one-shot grids map block b to a (stripe, column chunk) pair through a
per-geometry table: an XCD-contiguous remap (groups of 8 * span blocks, a
trailing partial group left in place) or a per-stripe chunk rotation
(DESIGN.md 3.3).  Both must be bijections: every column of every stripe coded
exactly once.  These geometries hit each branch -- rotation (1 MiB shards,
narrow and wide stripes), the remap with and without a partial trailing group,
and tiny grids where the remap degenerates -- and compare every parity byte,
and every rebuilt byte of a per-stripe-pattern decode, with the oracle.
"""
import itertools

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _encode_and_check(oracle_lib, k, m, S, B):
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    rng = np.random.default_rng(k * 1000 + S + B)
    host = np.zeros((B, k + m, lay.shard_stride), np.uint8)
    host[:, :k, :S] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    host[:, k:, :] = 0x77  # stale parity: every byte must be rewritten
    dev = torch.from_numpy(host.reshape(-1).copy()).to("cuda:0")
    device.encode(rs, dev.data_ptr(), lay)
    torch.cuda.synchronize()
    out = dev.cpu().numpy().reshape(B, k + m, lay.shard_stride)[:, :, :S]
    oc = oracle_lib.Codec(k, m)
    for t in range(B):
        ref = [host[t, i, :S].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        oc.encode_parity(ref, 0, S)
        for p in range(m):
            assert np.array_equal(out[t, k + p], ref[k + p]), (k, m, S, B, t, p)
    return rs, lay, dev, out


@pytest.mark.parametrize("k,m,S,B", [
    (4, 2, 1 << 20, 3),       # 1024 chunks: rotation
    (4, 2, 512 << 10, 5),     # 512 chunks: quarter-stripe rotation
    (10, 4, 1 << 20, 2),      # wide stripe, 1 MiB: rotation
    (10, 4, 4 << 20, 1),      # wide stripe, 4 MiB: rotation, a single stripe
    (4, 2, 4096, 13),         # XCD remap, 52 blocks: one group of 48 + 4 in place
    (4, 2, 64 << 10, 5),      # XCD remap, 320 blocks, no remainder
    (4, 2, 2 << 20, 1),       # XCD remap over one stripe
    (4, 2, 1024, 7),          # one chunk per stripe, 7 blocks: remap degenerates to identity
    (4, 2, (1 << 20) + 4096, 2),  # 1028 chunks: not the rotation size
])
def test_encode_every_column_once(gpu, oracle_lib, k, m, S, B):
    _encode_and_check(oracle_lib, k, m, S, B)


def test_masked_decode_under_remap(gpu, oracle_lib):
    """Per-stripe presence patterns with the XCD remap and a partial group."""
    import torch
    from rsamd import device
    k, m, S, B = 4, 2, 4096, 29
    rs, lay, dev, clean = _encode_and_check(oracle_lib, k, m, S, B)
    pats = [p for e in range(3) for p in itertools.combinations(range(k + m), e)]
    present = np.array([[i not in pats[t % len(pats)] for i in range(k + m)] for t in range(B)], bool)
    v = dev.view(B, k + m, lay.shard_stride)
    for t in range(B):
        for j in range(k + m):
            if not present[t, j]:
                v[t, j, :S] = 0xC3
    device.decode_masked(rs, dev.data_ptr(), present, lay)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy().reshape(B, k + m, lay.shard_stride)[:, :, :S], clean)
