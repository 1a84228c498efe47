"""GPU tests of batched recovery with a presence pattern per stripe
(ChunkserverDiskRecoveryMachine.java:14-57 driven per
chunk group by MasterImpl.java:794-839).  Bit-exact against the golden
fixtures and the oracle."""
import itertools
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _golden(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)["shards"]


def _run_masked(rs, batch, present, stride=None):
    import torch
    from rsamd import device
    from rsamd.device import StripeLayout
    B, T, S = batch.shape
    stride = stride or S
    host = np.zeros((B, T, stride), np.uint8)
    host[:, :, :S] = batch
    for t in range(B):
        for j in range(T):
            if not present[t][j]:
                host[t, j, :S] = 0x3C  # garbage the decode must overwrite
    dev = torch.from_numpy(host.reshape(-1).copy()).to("cuda:0")
    device.decode_masked(rs, dev.data_ptr(), present, StripeLayout(B, S, stride, stride * T),
                         torch.cuda.current_stream())
    torch.cuda.synchronize()
    return dev.cpu().numpy().reshape(B, T, stride)[:, :, :S]


def test_masked_4_2_every_pattern_mixed(gpu, golden_dir):
    import rsamd
    g = _golden(golden_dir, "rs_4_2_s4096_b8.npz")
    pats = [tuple(i not in miss for i in range(6))
            for e in range(3) for miss in itertools.combinations(range(6), e)]  # 22 patterns
    batch = np.concatenate([g] * 3)[: len(pats)]
    rs = rsamd.ReedSolomon.create(4, 2)
    out = _run_masked(rs, batch, pats)
    assert np.array_equal(out, batch)


@pytest.mark.parametrize("n", [1, 2, 22])
def test_masked_flag_bytes_any_nonzero(gpu, golden_dir, n):
    """Host flags are bytes, nonzero = present (capi.cpp presence_bits reads a
    row of up to 8 flags as one word; the last rows, whose word would run past
    the array, take the per-byte loop): 1 and 2 stripes stay inside one word,
    22 stripes cover every 4+2 pattern."""
    import rsamd
    g = _golden(golden_dir, "rs_4_2_s4096_b8.npz")
    pats = [tuple(i not in miss for i in range(6))
            for e in range(3) for miss in itertools.combinations(range(6), e)][-n:]
    vals = np.array([1, 2, 0x7F, 0x80, 0xFF, 0x41], np.uint8)
    flags = np.where(np.array(pats, bool), np.resize(vals, (n, 6)), 0).astype(np.uint8)
    batch = np.concatenate([g] * 3)[:n]
    rs = rsamd.ReedSolomon.create(4, 2)
    assert np.array_equal(_run_masked(rs, batch, flags), batch)
    flags[-1] = [0x80, 0, 0, 0, 0, 0xFF]  # two present: refused before any launch
    with pytest.raises(rsamd.IllegalArgumentException, match="^Not enough shards present$"):
        _run_masked(rs, batch, flags)


def test_masked_10_4_and_generic_17_3(gpu, golden_dir):
    import rsamd
    g = _golden(golden_dir, "rs_10_4_s1024_b4.npz")
    pats = [[i not in miss for i in range(14)] for miss in [(0, 1, 2, 3), (), (13,), (2, 7, 11)]]
    assert np.array_equal(_run_masked(rsamd.ReedSolomon.create(10, 4), g, pats), g)
    g = _golden(golden_dir, "rs_17_3_s512_b2.npz")
    pats = [[i not in miss for i in range(20)] for miss in [(0, 5, 19), (17, 18)]]
    assert np.array_equal(_run_masked(rsamd.ReedSolomon.create(17, 3), g, pats), g)


@pytest.mark.parametrize("k,m", [(10, 4), (3, 3), (6, 3)])
def test_masked8_runtime_k_chunk_groups(gpu, oracle_lib, k, m):
    """The 8-byte kernel's runtime-k build (k != 4) on 1000-byte shards packed
    back to back: random patterns of up to m erasures, host flags and device
    bitmasks, against the oracle."""
    import rsamd
    from rsamd.device import presence_bits
    S, B, T = 1000, 300, k + m
    rng = np.random.default_rng(k * 31 + m)
    batch = np.zeros((B, T, S), np.uint8)
    batch[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    c = oracle_lib.Codec(k, m)
    for t in range(B):
        c.encode_parity([batch[t, i] for i in range(T)], 0, S)
    pats = []
    for t in range(B):
        miss = rng.choice(T, int(rng.integers(0, m + 1)), replace=False)
        pats.append([i not in miss for i in range(T)])
    rs = rsamd.ReedSolomon.create(k, m)
    assert np.array_equal(_run_masked(rs, batch, pats, S), batch)
    out, bad, _ = _run_bits(rs, batch, presence_bits(pats), S)
    assert bad == 0 and np.array_equal(out, batch)


def test_masked_more_than_four_outputs(gpu, oracle_lib):
    """m = 6: patterns with 5-6 erasures need two output groups."""
    import rsamd
    k, m, S, B = 4, 6, 256, 6
    rng = np.random.default_rng(6)
    batch = np.zeros((B, k + m, S), np.uint8)
    c = oracle_lib.Codec(k, m)
    for t in range(B):
        batch[t, :k] = rng.integers(0, 256, (k, S), dtype=np.uint8)
        c.encode_parity([batch[t, i] for i in range(k + m)], 0, S)
    misses = [(0, 1, 2, 3, 4, 5), (1,), (4, 5, 6, 7, 8), (), (0, 9), (3, 4, 5, 6, 7, 8)]
    pats = [[i not in mi for i in range(k + m)] for mi in misses]
    assert np.array_equal(_run_masked(rsamd.ReedSolomon.create(k, m), batch, pats), batch)


@pytest.mark.parametrize("S,stride", [(1000, 1000), (1000, 1008), (4096, 4099), (1004, 1016), (1000, 1024)])
def test_masked_chunk_groups_like_the_master(gpu, oracle_lib, S, stride):
    """The DFS recovers 6 x 1000-byte chunk groups: packed back to back
    (stride 1000) they take the 8-byte kernel (gf_masked8_kernel, 125 vectors
    per shard); stride 1008 the 16-byte kernel plus an 8-byte tail; 1004/1016
    the 8-byte kernel plus a 4-byte tail; odd strides the byte kernel."""
    import rsamd
    rng = np.random.default_rng(S + stride)
    B = 500
    batch = np.zeros((B, 6, S), np.uint8)
    batch[:, :4] = rng.integers(0, 256, (B, 4, S), dtype=np.uint8)
    c = oracle_lib.Codec(4, 2)
    for t in range(B):
        c.encode_parity([batch[t, i] for i in range(6)], 0, S)
    allp = [tuple(i not in miss for i in range(6)) for e in range(3) for miss in itertools.combinations(range(6), e)]
    pats = [allp[int(x)] for x in rng.integers(0, len(allp), B)]
    assert np.array_equal(_run_masked(rsamd.ReedSolomon.create(4, 2), batch, pats, stride), batch)


def test_masked_not_enough_fails_before_launch(gpu):
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    rs = rsamd.ReedSolomon.create(4, 2)
    buf = torch.full((2 * 6 * 64,), 7, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(rsamd.IllegalArgumentException, match="^Not enough shards present$"):
        device.decode_masked(rs, buf.data_ptr(), [[1] * 6, [1, 1, 1, 0, 0, 0]], StripeLayout(2, 64, 64, 384))
    assert int((buf != 7).sum().item()) == 0


def test_masked_full_size_small_objects(gpu):
    """BASELINE configs[4] shape: 1 M stripes of 4 KiB, a random pattern per stripe."""
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    rs = rsamd.ReedSolomon.create(4, 2)
    B, S = 1 << 20, 4096
    lay = StripeLayout.packed(B, 6, S)
    buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream()
    device.fill_synthetic(buf.data_ptr(), 4, lay, 0x5EED, 0, st)
    device.encode(rs, buf.data_ptr(), lay, st)
    ref = buf.clone()
    rng = np.random.default_rng(1)
    allp = np.array([[i not in miss for i in range(6)] for e in range(3)
                     for miss in itertools.combinations(range(6), e)], dtype=bool)
    pats = allp[rng.integers(0, len(allp), B)]
    v = buf.view(B, 6, S)
    mask = torch.from_numpy(~pats).to("cuda:0")
    v.masked_fill_(mask[:, :, None], 0)
    device.decode_masked(rs, buf.data_ptr(), pats, lay, st)
    assert torch.equal(buf, ref)
    del buf, ref, v
    torch.cuda.empty_cache()


def test_recovery_machine_mirror(gpu, oracle_lib):
    from rsamd.recovery import ChunkserverDiskRecoveryMachine
    rng = np.random.default_rng(9)
    S = 1000
    shards = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(4)] + [np.zeros(S, np.uint8)] * 2
    shards = [s.copy() for s in shards]
    oracle_lib.Codec(4, 2).encode_parity(shards, 0, S)
    for miss in [(0,), (0, 5), (2, 3), (4,)]:
        mach = ChunkserverDiskRecoveryMachine()
        for i in range(6):
            if i not in miss:
                mach.addChunkserverDisksData(i, shards[i].tobytes())
        for j in miss:
            assert mach.retrieveRecoveredDiskData(j) == shards[j].tobytes()


def _run_bits(rs, batch, words, stride=None):
    """Device-resident presence bitmasks (rs_decode_batch_masked_bits_dev);
    returns (shards, bad count)."""
    import torch
    from rsamd import device
    from rsamd.device import StripeLayout
    B, T, S = batch.shape
    stride = stride or S
    host = np.zeros((B, T, stride), np.uint8)
    host[:, :, :S] = batch
    for t in range(B):
        for j in range(T):
            if not (int(words[t]) >> j) & 1:
                host[t, j, :S] = 0x3C
    dev = torch.from_numpy(host.reshape(-1).copy()).to("cuda:0")
    bits = torch.from_numpy(np.asarray(words, dtype=np.uint32).view(np.int32)).to("cuda:0")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.decode_masked_bits(rs, dev.data_ptr(), bits.data_ptr(), StripeLayout(B, S, stride, stride * T),
                              bad.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    return dev.cpu().numpy().reshape(B, T, stride)[:, :, :S], int(bad.item()), host[:, :, :S]


@pytest.mark.parametrize("S,stride", [(4096, 4096), (1000, 1008), (999, 1001), (1000, 1000), (1004, 1016)])
def test_bits_every_bitmask_4_2(gpu, oracle_lib, S, stride):
    """All 64 bitmasks of 4+2 plus out-of-range words: decodable stripes are
    rebuilt bit-exact, the rest are left untouched and counted."""
    import rsamd
    words = list(range(64)) + [64, 0xFFFFFFFF, 1 << 31]
    B = len(words)
    rng = np.random.default_rng(S)
    batch = np.zeros((B, 6, S), np.uint8)
    batch[:, :4] = rng.integers(0, 256, (B, 4, S), dtype=np.uint8)
    c = oracle_lib.Codec(4, 2)
    for t in range(B):
        c.encode_parity([batch[t, i] for i in range(6)], 0, S)
    out, bad, before = _run_bits(rsamd.ReedSolomon.create(4, 2), batch, words, stride)
    ok = np.array([w < 64 and bin(w).count("1") >= 4 for w in words])
    assert bad == int((~ok).sum())
    assert np.array_equal(out[ok], batch[ok])
    assert np.array_equal(out[~ok], before[~ok])


def test_bits_10_4_and_17_3(gpu, golden_dir):
    import rsamd
    from rsamd.device import presence_bits
    g = _golden(golden_dir, "rs_10_4_s1024_b4.npz")
    pats = [[i not in miss for i in range(14)] for miss in [(0, 1, 2, 3), (), (13,), (2, 7, 11)]]
    out, bad, _ = _run_bits(rsamd.ReedSolomon.create(10, 4), g, presence_bits(pats))
    assert bad == 0 and np.array_equal(out, g)
    g = _golden(golden_dir, "rs_17_3_s512_b2.npz")
    pats = [[i not in miss for i in range(20)] for miss in [(0, 5, 19), (17, 18)]]
    out, bad, _ = _run_bits(rsamd.ReedSolomon.create(17, 3), g, presence_bits(pats))
    assert bad == 0 and np.array_equal(out, g)


@pytest.mark.parametrize("k,m", [(12, 9), (10, 10)])
def test_bits_rejects_wide_codes_host_path_still_decodes(gpu, oracle_lib, k, m):
    """k+m > 20 or > 65536 decodable patterns: the bitmask call refuses before
    any launch; the host-flag call falls back to per-call records."""
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    rs = rsamd.ReedSolomon.create(k, m)
    S, B, T = 64, 3, k + m
    buf = torch.zeros(B * T * S, dtype=torch.uint8, device="cuda:0")
    bits = torch.zeros(B, dtype=torch.int32, device="cuda:0")
    with pytest.raises(rsamd.IllegalArgumentException):
        device.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), StripeLayout(B, S, S, S * T))
    rng = np.random.default_rng(k)
    batch = np.zeros((B, T, S), np.uint8)
    batch[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    c = oracle_lib.Codec(k, m)
    for t in range(B):
        c.encode_parity([batch[t, i] for i in range(T)], 0, S)
    pats = [[i not in miss for i in range(T)] for miss in [tuple(range(m)), (), (k - 1, k + m - 1)]]
    assert np.array_equal(_run_masked(rs, batch, pats), batch)


def test_bits_full_size_small_objects(gpu):
    """1 M stripes of 4 KiB with device-resident bitmasks, against the host-flag call."""
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout, presence_bits
    rs = rsamd.ReedSolomon.create(4, 2)
    B, S = 1 << 20, 4096
    lay = StripeLayout.packed(B, 6, S)
    buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream()
    device.fill_synthetic(buf.data_ptr(), 4, lay, 0x5EED, 0, st)
    device.encode(rs, buf.data_ptr(), lay, st)
    ref = buf.clone()
    rng = np.random.default_rng(2)
    allp = np.array([[i not in miss for i in range(6)] for e in range(3)
                     for miss in itertools.combinations(range(6), e)], dtype=bool)
    pats = allp[rng.integers(0, len(allp), B)]
    mask = torch.from_numpy(~pats).to("cuda:0")
    buf.view(B, 6, S).masked_fill_(mask[:, :, None], 0)
    bits = torch.from_numpy(presence_bits(pats).view(np.int32)).to("cuda:0")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, bad.data_ptr(), st)
    assert torch.equal(buf, ref) and int(bad.item()) == 0
    del buf, ref, mask
    torch.cuda.empty_cache()


@pytest.mark.parametrize("pad", [0, 8, 256])
def test_shard_major_groups_like_the_master(gpu, oracle_lib, pad):
    """The master's recovery loop batched in its own layout
    (MasterImpl.java:733-743, 794-839): one array per server, 1000-byte chunk
    groups back to back (rs_decode_groups_shard_major_dev).  Offline sets {0}
    and {0,5} for every group, a set that grows mid-loop (a read fails at an
    odd group, so the second run starts 8 bytes off a 16-byte boundary), and
    groups that need nothing before the failure.  Parity from the oracle on the
    long stripe (a run of groups is one stripe of N*1000-byte shards); every
    byte, server pads included, must come back as encoded."""
    import torch
    from rsamd.recovery import recover_groups_shard_major_dev
    k, m, chunk, N = 4, 2, 1000, 2049
    T = k + m
    L = N * chunk
    stride = L + pad
    rng = np.random.default_rng(pad + 1)
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)] + [np.zeros(L, np.uint8) for _ in range(m)]
    oracle_lib.Codec(k, m).encode_parity(rows, 0, L)
    want = np.full(T * stride, 0x77, np.uint8)
    for s in range(T):
        want[s * stride: s * stride + L] = rows[s]
    j = 1001
    cases = {
        "offline_0": [(0, N, (0,))],
        "offline_0_5": [(0, N, (0, 5))],
        "grows_mid_loop": [(0, j, (0,)), (j, N, (0, 3))],
        "fails_after_clean_run": [(0, j, ()), (j, N, (2,))],
    }
    st = torch.cuda.current_stream()
    for name, runs in cases.items():
        host = want.copy()
        present = np.ones((N, T), bool)
        for g0, g1, miss in runs:
            for s in miss:
                present[g0:g1, s] = False
                host[s * stride + g0 * chunk: s * stride + g1 * chunk] = 0x3C
        dev = torch.from_numpy(host).to("cuda:0")
        recover_groups_shard_major_dev(dev.data_ptr(), stride, present, chunk, st)
        torch.cuda.synchronize()
        got = dev.cpu().numpy()
        assert np.array_equal(got, want), (name, int(np.flatnonzero(got != want)[0]))


def test_shard_major_not_enough_touches_nothing(gpu):
    import torch
    from rsamd.codec import IllegalArgumentException
    from rsamd.recovery import recover_groups_shard_major_dev
    N, T = 64, 6
    host = np.arange(N * 1000 * T, dtype=np.uint64).astype(np.uint8)
    dev = torch.from_numpy(host).to("cuda:0")
    present = np.ones((N, T), bool)
    present[:10, 1] = False
    present[40, :3] = False  # undecodable
    with pytest.raises(IllegalArgumentException):
        recover_groups_shard_major_dev(dev.data_ptr(), N * 1000, present)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), host)


def test_shard_major_any_nonzero_flag(gpu, oracle_lib):
    """The C entry point reads a flag as present when nonzero, as the Java
    boolean[] is read (rows with different nonzero bytes but the same pattern
    are one run): random nonzero values in every present flag, two runs."""
    import ctypes as C
    import torch
    import rsamd
    from rsamd import _lib
    k, m, chunk, N = 4, 2, 1000, 1026
    T, L = k + m, N * chunk
    rng = np.random.default_rng(9)
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)] + [np.zeros(L, np.uint8) for _ in range(m)]
    oracle_lib.Codec(k, m).encode_parity(rows, 0, L)
    want = np.concatenate(rows)
    flags = rng.integers(1, 256, (N, T), dtype=np.uint8)
    flags[:500, 0] = 0
    flags[500:, 2] = 0
    flags[500:, 5] = 0
    host = want.copy()
    host[0: 500 * chunk] = 0x3C
    for s in (2, 5):
        host[s * L + 500 * chunk: (s + 1) * L] = 0x3C
    dev = torch.from_numpy(host).to("cuda:0")
    rs = rsamd.ReedSolomon.create(k, m)
    rc = _lib.load().rs_decode_groups_shard_major_dev(rs.handle, C.c_void_p(dev.data_ptr()), L, chunk, N,
                                                      flags.ctypes.data_as(_lib.u8p), None)
    assert rc == 0, _lib.last_error()
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), want)
