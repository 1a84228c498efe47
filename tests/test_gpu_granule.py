"""GPU parity tests of the granule layout (include/rs_amd.h)
through the C-ABI, against the oracle.  Bit-exact.

  * host shards scattered into a granule batch with rs_granule_copy_shard,
    encoded through the layout's view, parity gathered back and compared with
    the oracle's encodeParity (ReedSolomon.java:90-104) -- 4+2, 10+4, 17+3;
  * uniform-pattern decode (ReedSolomon.java:175-272): the reference test's
    {0,5} (ReedSolomonTest.java:77-93) and 10+4 {0,1,2,3};
  * per-stripe patterns (decode_masked, one pattern per stripe; formerly repeated over
    its sub-stripes), and device bitmasks, one per stripe;
  * verify flags a single flipped byte and passes a clean batch;
  * BASELINE config[3] at full size in the granule layout (10+4 x 4 MiB x 128,
    G = 32 KiB): encode -> verify clean -> erase 4 -> decode -> verify clean,
    plus sampled stripes gathered and checked against the oracle.
"""

import numpy as np
import pytest

from oracle import c_ref

pytestmark = pytest.mark.gpu


def _upload(torch, lay, shards):
    """Scatter (n, total, S) host shards into a new granule batch."""
    from rsamd import device
    dev = torch.zeros(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream()
    n, total, _ = shards.shape
    for t in range(n):
        for s in range(total):
            device.copy_shard(lay, dev.data_ptr(), t, s, shards[t, s].ctypes.data, True, st)
    torch.cuda.synchronize()
    return dev


def _download(torch, lay, dev, n, total):
    """Gather every shard back into (n, total, S) host arrays."""
    from rsamd import device
    out = np.zeros((n, total, lay.shard_len), dtype=np.uint8)
    st = torch.cuda.current_stream()
    for t in range(n):
        for s in range(total):
            device.copy_shard(lay, dev.data_ptr(), t, s, out[t, s].ctypes.data, False, st)
    torch.cuda.synchronize()
    return out


def _oracle_encode(k, m, shards):
    codec = c_ref.Codec(k, m)
    want = shards.copy()
    for t in range(want.shape[0]):
        codec.encode_parity([want[t, i] for i in range(k + m)], 0, want.shape[2])
    return want


@pytest.mark.parametrize("k,m,S,G,n", [(4, 2, 256 << 10, 64 << 10, 6), (10, 4, 128 << 10, 32 << 10, 4),
                                       (17, 3, 64 << 10, 16 << 10, 3), (4, 2, 48 << 10, 16 << 10, 5),
                                       (4, 2, 4 << 10, 64 << 10, 32), (10, 4, 8 << 10, 32 << 10, 8)])
def test_granule_encode_matches_oracle(gpu, k, m, S, G, n):
    import torch
    import rsamd
    from rsamd import device
    lay = device.GranuleLayout.make(n, k + m, S, G)
    rng = np.random.default_rng(k * 1000 + G)
    shards = rng.integers(0, 256, (n, k + m, S), dtype=np.uint8)
    shards[:, k:, :] = 0x5A  # parity buffers hold garbage before the encode
    dev = _upload(torch, lay, shards)
    rs = rsamd.ReedSolomon.create(k, m)
    device.encode(rs, dev.data_ptr(), lay, torch.cuda.current_stream())
    got = _download(torch, lay, dev, n, k + m)
    np.testing.assert_array_equal(got, _oracle_encode(k, m, shards))
    # the layout's bytes are the formula's (rs_amd.h): the last stripe's last byte column
    flat = dev.cpu().numpy()
    t, c = n - 1, S - 1
    x = t * S + c
    for s in range(k + m):
        assert flat[(x // G) * (k + m) * G + s * G + x % G] == got[t, s, c]


@pytest.mark.parametrize("k,m,miss", [(4, 2, (0, 5)), (4, 2, (2, 3)), (10, 4, (0, 1, 2, 3)), (10, 4, (3, 7, 10, 13))])
def test_granule_uniform_decode(gpu, k, m, miss):
    import torch
    import rsamd
    from rsamd import device
    S, G, n = 128 << 10, device.recommended_granule(k + m), 4
    lay = device.GranuleLayout.make(n, k + m, S, G)
    rng = np.random.default_rng(len(miss) * 7 + k)
    shards = rng.integers(0, 256, (n, k + m, S), dtype=np.uint8)
    want = _oracle_encode(k, m, shards)
    clobbered = want.copy()
    clobbered[:, list(miss), :] = 0xA5
    dev = _upload(torch, lay, clobbered)
    rs = rsamd.ReedSolomon.create(k, m)
    present = [i not in miss for i in range(k + m)]
    device.decode(rs, dev.data_ptr(), present, lay, torch.cuda.current_stream())
    np.testing.assert_array_equal(_download(torch, lay, dev, n, k + m), want)


def test_granule_per_stripe_patterns(gpu):
    """decode_masked on a granule batch: every stripe its own erasures, one
    pattern per stripe (rs_decode_granule_masked_dev finds a block's stripe
    from its batch column); then the same patterns as device bitmasks, one
    word per stripe, with an undecodable stripe left alone and counted once
    although it spans 4 granule rows."""
    import torch
    import rsamd
    from rsamd import device
    k, m, S, G, n = 4, 2, 64 << 10, 16 << 10, 15
    lay = device.GranuleLayout.make(n, k + m, S, G)
    import itertools
    pats = [[i not in mi for i in range(k + m)] for e in range(3) for mi in itertools.combinations(range(k + m), e)]
    present = np.array(pats[:n], dtype=bool)
    rng = np.random.default_rng(11)
    want = _oracle_encode(k, m, rng.integers(0, 256, (n, k + m, S), dtype=np.uint8))
    clobbered = want.copy()
    clobbered[~present] = 0x33
    rs = rsamd.ReedSolomon.create(k, m)
    dev = _upload(torch, lay, clobbered)
    device.decode_masked(rs, dev.data_ptr(), present, lay, torch.cuda.current_stream())
    np.testing.assert_array_equal(_download(torch, lay, dev, n, k + m), want)
    dev = _upload(torch, lay, clobbered)
    bits = device.presence_bits(present)
    bits[4] = 0b000111  # 3 of 6 present: undecodable, left as it is
    dbits = torch.from_numpy(bits.view(np.int32)).to("cuda:0")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.decode_masked_bits(rs, dev.data_ptr(), dbits.data_ptr(), lay, bad.data_ptr(), torch.cuda.current_stream())
    got = _download(torch, lay, dev, n, k + m)
    assert int(bad.item()) == 1
    np.testing.assert_array_equal(got[4], clobbered[4])
    keep = np.arange(n) != 4
    np.testing.assert_array_equal(got[keep], want[keep])


@pytest.mark.parametrize("S,G", [(4 << 10, 64 << 10), (1 << 10, 8 << 10), (2064, 8256), (4160, 1040)])
def test_granule_small_shards_patterns_per_stripe(gpu, S, G):
    """Several stripes per granule row (config[4]'s 4 KiB shards in 64 KiB
    rows, 16 stripes each), each stripe its OWN pattern -- every 4+2 pattern
    with at most 2 erasures, cycled; as host flags and as device bitmasks.
    The 2064/8256 and 4160/1040 shapes (not whole 1 KiB chunks) take the
    byte-granular kernel."""
    import itertools
    import torch
    import rsamd
    from rsamd import device
    k, m = 4, 2
    n = max(64, 2 * G // S)
    lay = device.GranuleLayout.make(n, k + m, S, G)
    pats = [[i not in mi for i in range(k + m)] for e in range(3) for mi in itertools.combinations(range(k + m), e)]
    present = np.array([pats[(7 * t) % len(pats)] for t in range(n)], dtype=bool)
    want = _oracle_encode(k, m, np.random.default_rng(9).integers(0, 256, (n, k + m, S), dtype=np.uint8))
    rs = rsamd.ReedSolomon.create(k, m)
    clobbered = want.copy()
    clobbered[~present] = 0x11
    dev = _upload(torch, lay, clobbered)
    device.decode_masked(rs, dev.data_ptr(), present, lay, torch.cuda.current_stream())
    np.testing.assert_array_equal(_download(torch, lay, dev, n, k + m), want)
    dev = _upload(torch, lay, clobbered)
    bits = device.presence_bits(present)
    bits[1] = 0b110001  # undecodable: untouched, counted once
    dbits = torch.from_numpy(bits.view(np.int32)).to("cuda:0")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.decode_masked_bits(rs, dev.data_ptr(), dbits.data_ptr(), lay, bad.data_ptr(), torch.cuda.current_stream())
    got = _download(torch, lay, dev, n, k + m)
    assert int(bad.item()) == 1
    np.testing.assert_array_equal(got[1], clobbered[1])
    keep = np.arange(n) != 1
    np.testing.assert_array_equal(got[keep], want[keep])


def test_granule_small_shards_decode(gpu):
    """config[4]-style 4 KiB shards, 16 stripes per 64 KiB granule row: {0,1}
    decode with one pattern for the batch."""
    import torch
    import rsamd
    from rsamd import device
    k, m, S, n = 4, 2, 4 << 10, 64
    lay = device.GranuleLayout.make(n, k + m, S)
    assert lay.granule == 64 << 10 and lay.rows == 4
    want = _oracle_encode(k, m, np.random.default_rng(9).integers(0, 256, (n, k + m, S), dtype=np.uint8))
    rs = rsamd.ReedSolomon.create(k, m)
    clobbered = want.copy()
    clobbered[:, [0, 1], :] = 0x77
    dev = _upload(torch, lay, clobbered)
    device.decode(rs, dev.data_ptr(), [False, False, True, True, True, True], lay, torch.cuda.current_stream())
    np.testing.assert_array_equal(_download(torch, lay, dev, n, k + m), want)


def test_granule_verify_flags_one_byte(gpu):
    import torch
    import rsamd
    from rsamd import device
    k, m, S, G, n = 10, 4, 64 << 10, 32 << 10, 3
    lay = device.GranuleLayout.make(n, k + m, S, G)
    want = _oracle_encode(k, m, np.random.default_rng(5).integers(0, 256, (n, k + m, S), dtype=np.uint8))
    rs = rsamd.ReedSolomon.create(k, m)
    dev = _upload(torch, lay, want)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.verify(rs, dev.data_ptr(), lay, flag.data_ptr(), torch.cuda.current_stream())
    assert int(flag.item()) == 0
    bad = want.copy()
    bad[2, 12, S - 1] ^= 1  # last byte of the last parity granule of the last stripe
    dev = _upload(torch, lay, bad)
    device.verify(rs, dev.data_ptr(), lay, flag.data_ptr(), torch.cuda.current_stream())
    assert int(flag.item()) == 1


def test_granule_config3_full_size_round_trip(gpu):
    """config[3]'s per-GPU share at N = 8 in the granule layout: 10+4 x 4 MiB x
    128 stripes, G = 32 KiB, on a contiguous pool."""
    import torch
    import rsamd
    from rsamd import device
    k, m, S, n = 10, 4, 4 << 20, 128
    lay = device.GranuleLayout.make(n, k + m, S)
    assert lay.granule == 32 << 10
    pool = device.DeviceBuffer(lay.nbytes, contiguous=True)
    st = torch.cuda.current_stream()
    base = pool.data_ptr()
    device.fill_synthetic(base, k, lay, 0x5EED, 0, st)
    rs = rsamd.ReedSolomon.create(k, m)
    device.encode(rs, base, lay, st)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.verify(rs, base, lay, flag.data_ptr(), st)
    assert int(flag.item()) == 0
    # sampled stripes against the oracle (gathered through rs_granule_copy_shard)
    for t in (0, 77, n - 1):
        got = np.zeros((k + m, S), dtype=np.uint8)
        for s in range(k + m):
            device.copy_shard(lay, base, t, s, got[s].ctypes.data, False, st)
        torch.cuda.synchronize()
        want = got.copy()
        want[k:] = 0
        c_ref.Codec(k, m).encode_parity([want[i] for i in range(k + m)], 0, S)
        np.testing.assert_array_equal(got, want)
    snap = pool.tensor().clone()
    miss = (0, 1, 2, 3)
    present = [i not in miss for i in range(k + m)]
    zero = np.zeros(S, dtype=np.uint8)
    for t in range(0, n, 9):  # erase shards 0-3 of every 9th stripe from a zero host buffer
        for s in miss:
            device.copy_shard(lay, base, t, s, zero.ctypes.data, True, st)
    device.decode(rs, base, present, lay, st)
    torch.cuda.synchronize()
    assert torch.equal(pool.tensor(), snap)
    pool.free()


def test_granule_headline_full_size_round_trip(gpu):
    """The bench headline's own batch at full size: 4+2 x 1 MiB x 4096
    stripes in the granule layout, G = 64 KiB, on a contiguous pool
    (BASELINE configs[1]).  Encode, verify clean, stripes {0, 1, 2048, 4095}
    gathered and compared with the oracle (data from the synthetic fill,
    parity from encodeParity, ReedSolomon.java:90-104); then shards 0 and 5 of
    EVERY stripe overwritten -- the erasure pattern of ReedSolomonTest.java:77-93
    -- decoded, and the whole 24 GiB batch compared byte for byte with the
    encoded one."""
    import torch
    import rsamd
    from rsamd import device
    k, m, S, n = 4, 2, 1 << 20, 4096
    lay = device.GranuleLayout.make(n, k + m, S)
    assert lay.granule == 64 << 10
    pool = device.DeviceBuffer(lay.nbytes, contiguous=True)
    st = torch.cuda.current_stream()
    base = pool.data_ptr()
    device.fill_synthetic(base, k, lay, 0x5EED, 0, st)
    rs = rsamd.ReedSolomon.create(k, m)
    device.encode(rs, base, lay, st)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.verify(rs, base, lay, flag.data_ptr(), st)
    assert int(flag.item()) == 0
    oc = c_ref.Codec(k, m)
    for t in (0, 1, n // 2, n - 1):
        got = np.zeros((k + m, S), dtype=np.uint8)
        for s in range(k + m):
            device.copy_shard(lay, base, t, s, got[s].ctypes.data, False, st)
        torch.cuda.synchronize()
        want = np.zeros_like(got)
        want[:k] = c_ref.synthetic_shards(k, S, 0x5EED, t, lay.granule)
        oc.encode_parity([want[i] for i in range(k + m)], 0, S)
        np.testing.assert_array_equal(got, want)
    snap = pool.tensor().clone()
    rows = pool.tensor().view(lay.rows, k + m, lay.granule)
    rows[:, 0] = 0x5A  # shard 0 (DataDiskOne) of every stripe
    rows[:, 5] = 0xA5  # shard 5 (ParityDiskTwo)
    device.decode(rs, base, [False, True, True, True, True, False], lay, st)
    torch.cuda.synchronize()
    assert torch.equal(pool.tensor(), snap)
    del snap, rows
    pool.free()
    torch.cuda.empty_cache()


def test_granule_per_stripe_patterns_wide_code(gpu):
    """k+m = 21 > 20: no pattern table, so rs_decode_granule_masked_dev builds
    per-call records for the distinct patterns; up to 9 erasures per stripe
    take three output groups.  Each stripe spans 2 granule rows; against the
    oracle's encodeParity."""
    import torch
    import rsamd
    from rsamd import device
    k, m, S, n = 12, 9, 32 << 10, 6
    lay = device.GranuleLayout.make(n, k + m, S)
    assert lay.granule == 16 << 10
    rng = np.random.default_rng(21)
    want = _oracle_encode(k, m, rng.integers(0, 256, (n, k + m, S), dtype=np.uint8))
    present = np.ones((n, k + m), dtype=bool)
    for t, e in enumerate([9, 0, 1, 5, 9, 3]):
        present[t, rng.choice(k + m, e, replace=False)] = False
    clobbered = want.copy()
    clobbered[~present] = 0x6B
    rs = rsamd.ReedSolomon.create(k, m)
    dev = _upload(torch, lay, clobbered)
    device.decode_masked(rs, dev.data_ptr(), present, lay, torch.cuda.current_stream())
    np.testing.assert_array_equal(_download(torch, lay, dev, n, k + m), want)
    # device bitmasks need the pattern table (k+m <= 20): refused before any launch
    bits = torch.zeros(n, dtype=torch.int32, device="cuda:0")
    with pytest.raises(rsamd.IllegalArgumentException):
        device.decode_masked_bits(rs, dev.data_ptr(), bits.data_ptr(), lay)
