"""Seeded random cases of the master's recovery loop in its own layout
(rs_decode_groups_shard_major_dev; MasterImpl.java:733-743, 794-839) against
the oracle, bit-exact: codes 4+2, 10+4, 3+3 and 6+1; chunk lengths that are
and are not multiples of 8 or 16; server strides with pads of 0 to 4 KiB + 1;
one to five runs of groups, each with its own offline set (empty sets too, so
runs need nothing, and sets that shrink as well as grow); random bytes in
every chunk, so the survivors are checked on the reference's exact choice
(the first k present, ReedSolomon.java:210-222).  Every byte of the pool,
pads included, must come back as the oracle encoded it.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CODES = [(4, 2), (10, 4), (3, 3), (6, 1)]
CHUNKS = [1000, 1024, 8, 13, 4096, 999, 1000, 2000]
PADS = [0, 8, 256, 4096, 1, 0, 24, 4097]


@pytest.mark.parametrize("case", range(24))
def test_shard_major_random(gpu, oracle_lib, case):
    import torch
    from rsamd.recovery import recover_groups_shard_major_dev
    rng = np.random.default_rng(7000 + case)
    k, m = CODES[case % len(CODES)]
    T = k + m
    chunk = CHUNKS[case % len(CHUNKS)]
    pad = PADS[(case // 2) % len(PADS)]
    N = int(rng.integers(1, 3001))
    L = N * chunk
    stride = L + pad
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(T)]
    oracle_lib.Codec(k, m).encode_parity(rows, 0, L)  # parity of every group at once (per column)
    want = rng.integers(0, 256, T * stride, dtype=np.uint8)  # pads: random bytes that must survive
    for s in range(T):
        want[s * stride: s * stride + L] = rows[s]
    cuts = sorted(set(int(x) for x in rng.integers(1, N, int(rng.integers(0, 5))))) if N > 1 else []
    bounds = [0] + cuts + [N]
    present = np.ones((N, T), bool)
    host = want.copy()
    for g0, g1 in zip(bounds[:-1], bounds[1:]):
        e = int(rng.integers(0, m + 1))
        miss = [int(x) for x in rng.choice(T, e, replace=False)] if e else []
        present[g0:g1, miss] = False
        for s in miss:
            host[s * stride + g0 * chunk: s * stride + g1 * chunk] = 0x3C
    dev = torch.from_numpy(host).to("cuda:0")
    recover_groups_shard_major_dev(dev.data_ptr(), stride, present, chunk, torch.cuda.current_stream(),
                                   data_shards=k, parity_shards=m)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    if not np.array_equal(got, want):
        i = int(np.flatnonzero(got != want)[0])
        s, off = divmod(i, stride)
        raise AssertionError(f"k={k} m={m} chunk={chunk} pad={pad} N={N} runs={bounds}: first wrong byte "
                             f"server {s} offset {off} (group {off // chunk})")


@pytest.mark.parametrize("chunk,pad", [(1000, 0), (13, 8), (4096, 256)])
def test_shard_major_many_runs(gpu, oracle_lib, chunk, pad):
    """Flags that change every group or few groups (more than the 64 runs the
    call codes one by one) go to the per-stripe pattern kernels in one launch:
    same results, against the oracle, with random bytes in every chunk."""
    import torch
    from rsamd.recovery import recover_groups_shard_major_dev
    rng = np.random.default_rng(chunk + pad)
    k, m = 4, 2
    T = k + m
    N = 3001
    L = N * chunk
    stride = L + pad
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(T)]
    oracle_lib.Codec(k, m).encode_parity(rows, 0, L)
    want = rng.integers(0, 256, T * stride, dtype=np.uint8)
    for s in range(T):
        want[s * stride: s * stride + L] = rows[s]
    present = np.ones((N, T), bool)
    host = want.copy()
    g = 0
    while g < N:
        n = int(rng.integers(1, 4))
        e = int(rng.integers(0, m + 1))
        miss = [int(x) for x in rng.choice(T, e, replace=False)] if e else []
        present[g: g + n, miss] = False
        for s in miss:
            host[s * stride + g * chunk: s * stride + min(N, g + n) * chunk] = 0x3C
        g += n
    dev = torch.from_numpy(host).to("cuda:0")
    recover_groups_shard_major_dev(dev.data_ptr(), stride, present, chunk, torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    assert np.array_equal(got, want), int(np.flatnonzero(got != want)[0])
