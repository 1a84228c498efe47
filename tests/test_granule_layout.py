"""CPU tests of the granule layout (include/rs_amd.h).

The layout stores granule g of every shard of a stripe together.  The batch
entry points code it through its `view`, the packed batch of granule-byte
sub-stripes with the same bytes.  These tests check, without a GPU:
  * the view's addresses are exactly the layout's formula;
  * coding per sub-stripe of the view equals coding the logical stripes (the
    oracle on both sides; ReedSolomon.java:90-104 codes each byte column
    independently, so this is exact for encode and decode);
  * view_shards gathers the logical shards back;
  * rs_granule_recommended and rs_granule_copy_shard's argument checks.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import c_ref


def _layout(n, total, S, G):
    from rsamd.device import GranuleLayout
    return GranuleLayout.make(n, total, S, G)


def _to_granules(shards: np.ndarray, G: int) -> np.ndarray:
    """(n, total, S) logical shards -> flat bytes of the granule layout, by the
    header's formula: byte c of shard s of stripe t, x = t*S + c, at
    (x // G)*total*G + s*G + x % G."""
    n, total, S = shards.shape
    out = np.zeros(n * total * S, dtype=np.uint8)
    t, s, c = np.meshgrid(np.arange(n), np.arange(total), np.arange(S), indexing="ij")
    x = t * S + c  # the batch column
    addr = (x // G) * total * G + s * G + x % G
    out[addr.reshape(-1)] = shards.reshape(-1)
    return out


def test_recommended_granule():
    from rsamd.device import recommended_granule
    assert recommended_granule(6) == 64 << 10      # 4+2
    assert recommended_granule(14) == 32 << 10     # 10+4
    assert recommended_granule(20) == 16 << 10     # 17+3
    assert recommended_granule(3) == 128 << 10
    assert recommended_granule(1) == 512 << 10
    assert recommended_granule(256) == 4 << 10     # clamped at 4 KiB
    assert recommended_granule(0) == 0


def test_view_addresses_match_the_formula():
    from rsamd.device import view_shards
    rng = np.random.default_rng(3)
    n, total, S, G = 3, 6, 4096, 1024
    lay = _layout(n, total, S, G)
    shards = rng.integers(0, 256, (n, total, S), dtype=np.uint8)
    flat = _to_granules(shards, G)
    # the view's sub-stripes: sub-stripe u = t*(S/G) + g holds granule g of every shard of stripe t
    v = lay.view
    assert (v.n_stripes, v.shard_len, v.shard_stride, v.stripe_stride) == (n * S // G, G, G, total * G)
    sub = view_shards(flat, v, total)
    for t in range(n):
        for g in range(S // G):
            np.testing.assert_array_equal(sub[t * (S // G) + g], shards[t, :, g * G:(g + 1) * G])
    np.testing.assert_array_equal(view_shards(flat, lay, total), shards)
    assert lay.nbytes == flat.size


def test_small_shards_share_a_granule_row():
    """shard_len < granule: a row holds granule/shard_len whole stripes (config[4]'s 4 KiB shards)."""
    from rsamd.device import view_shards
    rng = np.random.default_rng(4)
    n, total, S, G = 8, 6, 1024, 4096
    lay = _layout(n, total, S, G)
    shards = rng.integers(0, 256, (n, total, S), dtype=np.uint8)
    flat = _to_granules(shards, G)
    v = lay.view
    assert (v.n_stripes, v.shard_len, v.shard_stride, v.stripe_stride) == (n * S // G, G, G, total * G)
    sub = view_shards(flat, v, total)
    for t in range(n):  # stripe t is columns [(t % 4)*S, +S) of row t // 4
        np.testing.assert_array_equal(sub[t // 4, :, (t % 4) * S:(t % 4 + 1) * S], shards[t])
    np.testing.assert_array_equal(view_shards(flat, lay, total), shards)
    with pytest.raises(ValueError):
        lay.subs_per_stripe


@pytest.mark.parametrize("k,m,S,G", [(4, 2, 8192, 2048), (10, 4, 4096, 1024), (3, 2, 3072, 1024),
                                     (4, 2, 1024, 4096), (10, 4, 512, 2048)])
def test_coding_the_view_equals_coding_the_stripes(k, m, S, G):
    """Encode and decode per sub-stripe of the view == the oracle on the
    logical stripes (every byte column is coded on its own)."""
    from rsamd.device import view_shards
    rng = np.random.default_rng(k * 100 + m)
    total = k + m
    n = max(2, 2 * G // S)
    lay = _layout(n, total, S, G)
    codec = c_ref.Codec(k, m)
    logical = rng.integers(0, 256, (n, total, S), dtype=np.uint8)
    logical[:, k:, :] = 0
    want = logical.copy()
    for t in range(n):
        sh = [want[t, i] for i in range(total)]
        codec.encode_parity(sh, 0, S)
    flat = _to_granules(logical, G)
    sub = view_shards(flat, lay.view, total).copy()
    for u in range(sub.shape[0]):
        sh = [sub[u, i] for i in range(total)]
        codec.encode_parity(sh, 0, G)
    got_flat = np.zeros_like(flat)
    # scatter the coded sub-stripes back through the view's packed addressing
    got_flat.reshape(sub.shape[0], total, G)[:] = sub
    np.testing.assert_array_equal(view_shards(got_flat, lay, total), want)
    # decode: erase data shard 0 and the last parity shard, per sub-stripe
    present = [i not in (0, total - 1) for i in range(total)]
    for u in range(sub.shape[0]):
        sub[u, 0] = 0
        sub[u, total - 1] = 0
        sh = [sub[u, i] for i in range(total)]
        codec.decode_missing(sh, present, 0, G)
    got_flat.reshape(sub.shape[0], total, G)[:] = sub
    np.testing.assert_array_equal(view_shards(got_flat, lay, total), want)


def test_make_rejects_bad_granules():
    from rsamd.device import GranuleLayout
    with pytest.raises(ValueError):
        GranuleLayout.make(1, 6, 4096, 3000)
    with pytest.raises(ValueError):
        GranuleLayout.make(1, 6, 4096, 8)
    with pytest.raises(ValueError):
        GranuleLayout.make(3, 6, 1024, 4096)  # 3 stripes of 1 KiB do not fill whole 4 KiB rows
    assert GranuleLayout.make(1, 14, 1 << 20).granule == 32 << 10
    assert GranuleLayout.make(16, 6, 4096).rows == 1  # 16 x 4 KiB stripes in one 64 KiB row


def test_copy_shard_argument_checks(native):
    """RS_E_INVALID before any HIP call (so these run without a GPU)."""
    RS_E_INVALID = -10
    buf = (C.c_uint8 * 64)()
    base = C.c_void_p(C.addressof(buf))
    f = native.rs_granule_copy_shard
    assert f(None, 6, 4, 4096, 1024, 0, 0, base, 1, None) == RS_E_INVALID       # NULL base
    assert f(base, 6, 4, 4096, 1024, 0, 0, None, 1, None) == RS_E_INVALID       # NULL buf
    assert f(base, 6, 4, 4096, 1024, 0, 6, base, 1, None) == RS_E_INVALID       # shard out of range
    assert f(base, 6, 4, 4096, 1024, 0, -1, base, 1, None) == RS_E_INVALID
    assert f(base, 6, 4, 4096, 1024, 4, 0, base, 1, None) == RS_E_INVALID       # stripe out of range
    assert b"stripe 4 outside [0, 4)" in native.rs_last_error_message()
    assert f(base, 6, 0, 4096, 1024, 0, 0, base, 0, None) == RS_E_INVALID       # empty batch
    assert f(base, 6, 4, 4096, 3000, 0, 0, base, 1, None) == RS_E_INVALID       # neither divides the other
    assert b"must divide one another" in native.rs_last_error_message()
    assert f(base, 6, 4, 4096, 0, 0, 0, base, 1, None) == RS_E_INVALID          # granule 0
    assert f(base, 6, 4, 0, 1024, 0, 0, base, 1, None) == RS_E_INVALID          # shard_len 0


def test_copy_shard_python_checks():
    """device.copy_shard refuses a stripe or shard outside the batch before
    calling the library (no GPU needed)."""
    from rsamd import device
    from rsamd.device import GranuleLayout
    lay = GranuleLayout.make(4, 6, 4096, 1024)
    for stripe, shard in ((4, 0), (-1, 0), (0, 6), (0, -1)):
        with pytest.raises(ValueError):
            device.copy_shard(lay, 1 << 20, stripe, shard, 1 << 21, True)


def test_granule_masked_argument_checks(native):
    """rs_decode_granule_masked[_bits]_dev: shape errors are RS_E_INVALID
    before any HIP call; an empty batch is RS_OK (runs without a GPU)."""
    import rsamd
    RS_E_INVALID = -10
    rs = rsamd.ReedSolomon.create(4, 2)
    buf = (C.c_uint8 * 64)()
    base = C.c_void_p(C.addressof(buf))
    present = np.ones(6 * 4, dtype=np.uint8)
    pp = present.ctypes.data_as(C.POINTER(C.c_uint8))
    f, fb = native.rs_decode_granule_masked_dev, native.rs_decode_granule_masked_bits_dev
    assert f(rs.handle, base, pp, 4, 4096, 3000, None) == RS_E_INVALID      # neither divides the other
    assert b"must divide one another" in native.rs_last_error_message()
    assert f(rs.handle, base, pp, 1, 4096, 8192, None) == RS_E_INVALID      # G does not divide n * S
    assert b"does not divide" in native.rs_last_error_message()
    assert f(rs.handle, base, pp, 4, 4096, 0, None) == RS_E_INVALID         # granule 0
    assert f(rs.handle, base, None, 4, 4096, 1024, None) == RS_E_INVALID    # NULL present
    assert f(rs.handle, None, pp, 4, 4096, 1024, None) == RS_E_INVALID      # NULL base
    assert f(None, base, pp, 4, 4096, 1024, None) == RS_E_INVALID           # NULL codec
    assert f(rs.handle, base, pp, 0, 4096, 1024, None) == 0                 # nothing to do
    assert fb(rs.handle, base, base, 4, 4096, 3000, None, None) == RS_E_INVALID
    assert fb(rs.handle, base, None, 4, 4096, 1024, None, None) == RS_E_INVALID
    assert fb(rs.handle, base, base, 0, 4096, 1024, None, None) == 0
