"""Seeded random cases through the C-ABI against the oracle, bit-exact, on
inputs that are NOT codewords: random bytes in every shard, parity included,
so a decode is compared on its exact semantics (survivors = the first k
present shards, ReedSolomon.java:210-222; missing parity recomputed from the
data, :259-271) rather than on a round trip that any survivor choice passes.

  * host API (ReedSolomon.encodeParity / decodeMissing / isParityCorrect,
    ReedSolomon.java:90-272): k in 1..20, m in 0..8, shard lengths 1..70000,
    random offset and byteCount, random erasure sets of 0..m shards;
  * device batches (rs_encode_batch_dev / rs_decode_batch_dev /
    rs_decode_batch_masked_dev): 4+2, 10+4 and generic shapes, padded shard
    and stripe strides, 8-aligned and odd base addresses, a uniform erasure
    set and one random set per stripe.
Every byte outside the coded range and every present shard must be unchanged.
"""
import numpy as np
import pytest
from bytes_report import describe


def assert_equal_bytes(got, want, msg):
    d = describe(got, want)
    assert d is None, f"{msg}: {d}"


pytestmark = pytest.mark.gpu


def _random_present(rng, k, m):
    e = int(rng.integers(0, m + 1))
    miss = rng.choice(k + m, e, replace=False) if e else []
    return [i not in set(int(x) for x in miss) for i in range(k + m)]


@pytest.mark.parametrize("case", range(48))
def test_host_api_random(gpu, oracle_lib, case):
    import rsamd
    rng = np.random.default_rng(1000 + case)
    k = int(rng.integers(1, 21))
    m = int(rng.integers(0, 9))
    n = int(rng.choice([1, 7, 16, 1000, 4096, 4097, int(rng.integers(1, 70001))]))
    off = int(rng.integers(0, n))
    cnt = int(rng.integers(0, n - off + 1))
    shards = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k + m)]
    rs = rsamd.ReedSolomon.create(k, m)
    oc = oracle_lib.Codec(k, m)

    got = [s.copy() for s in shards]
    ref = [s.copy() for s in shards]
    rs.encodeParity(got, off, cnt)
    oc.encode_parity(ref, off, cnt)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert_equal_bytes(a, b, f"encode k={k} m={m} n={n} off={off} cnt={cnt} shard {i}")
    assert rs.isParityCorrect(got, off, cnt) == oc.is_parity_correct(ref, off, cnt) == True  # noqa: E712
    if m and cnt:
        bad = [s.copy() for s in got]
        j = int(rng.integers(off, off + cnt))
        bad[k + int(rng.integers(0, m))][j] ^= 1 + int(rng.integers(0, 255))
        assert not rs.isParityCorrect(bad, off, cnt)

    present = _random_present(rng, k, m)
    got = [s.copy() for s in shards]
    ref = [s.copy() for s in shards]
    rs.decodeMissing(got, present, off, cnt)
    oc.decode_missing(ref, present, off, cnt)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert_equal_bytes(a, b, f"decode k={k} m={m} n={n} off={off} cnt={cnt} "
                                                    f"present={present} shard {i}")


def _oracle_batch(oc, batch, fn):
    """Apply an oracle call per stripe of a (B, T, S) array, in place."""
    for t in range(batch.shape[0]):
        fn(t, [batch[t, i] for i in range(batch.shape[1])])


@pytest.mark.parametrize("case", range(24))
def test_device_batch_random(gpu, oracle_lib, case):
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    rng = np.random.default_rng(5000 + case)
    k, m = [(4, 2), (10, 4), (4, 2), (10, 4), (3, 3), (6, 1), (12, 4), (2, 5)][case % 8]
    T = k + m
    S = int(rng.choice([16, 256, 1000, 1024, 4096, 5000, 65536, int(rng.integers(1, 20000))]))
    B = int(rng.integers(1, 40))
    shard_pad = int(rng.choice([0, 0, 8, 16, 3]))
    stripe_pad = int(rng.choice([0, 0, 16, 8, 5]))
    base_off = int(rng.choice([0, 0, 8, 1]))
    shard_stride = S + shard_pad
    stripe_stride = T * shard_stride + stripe_pad
    lay = StripeLayout(B, S, shard_stride, stripe_stride)
    nbytes = base_off + B * stripe_stride + 64
    host = rng.integers(0, 256, nbytes, dtype=np.uint8)

    def view(buf):
        return np.lib.stride_tricks.as_strided(buf[base_off:], (B, T, S), (stripe_stride, shard_stride, 1))

    rs = rsamd.ReedSolomon.create(k, m)
    oc = oracle_lib.Codec(k, m)
    st = torch.cuda.current_stream()
    desc = f"k={k} m={m} S={S} B={B} shard_pad={shard_pad} stripe_pad={stripe_pad} base_off={base_off}"

    def run(call, expect_fn):
        dev = torch.from_numpy(host.copy()).to("cuda:0")
        call(dev.data_ptr() + base_off)
        torch.cuda.synchronize()
        want = host.copy()
        expect_fn(view(want))
        np.testing.assert_array_equal(dev.cpu().numpy(), want, err_msg=desc)

    run(lambda p: device.encode(rs, p, lay, st),
        lambda v: _oracle_batch(oc, v, lambda t, sh: oc.encode_parity(sh, 0, S)))
    present = _random_present(rng, k, m)
    run(lambda p: device.decode(rs, p, present, lay, st),
        lambda v: _oracle_batch(oc, v, lambda t, sh: oc.decode_missing(sh, present, 0, S)))
    pres = np.array([_random_present(rng, k, m) for _ in range(B)], dtype=bool)
    run(lambda p: device.decode_masked(rs, p, pres, lay, st),
        lambda v: _oracle_batch(oc, v, lambda t, sh: oc.decode_missing(sh, list(pres[t]), 0, S)))


@pytest.mark.parametrize("case", range(16))
def test_host_api_random_large(gpu, oracle_lib, case):
    """The same host calls at sizes that take the direct path (capi.cpp
    run_direct / run_direct_interior): shards of 256 KiB to 3 MiB, pageable
    NumPy arrays (pages inside the range locked and coded in place, the ends
    staged) or page-locked ones, each shard a view at a random offset of its
    own buffer (common residues modulo 16 or 8, and none: the staged
    pipeline), k up to 20 and m up to 8 (several launch groups)."""
    import torch
    import rsamd
    rng = np.random.default_rng(3000 + case)
    k = int(rng.integers(1, 21))
    m = int(rng.integers(0, 9))
    n = int(rng.integers(256 << 10, 3 << 20))
    off = int(rng.integers(0, 5000))
    cnt = int(rng.integers(n // 2, n - off + 1))
    pinned = case % 4 == 3
    residue = [16, 8, 1][case % 3]  # shard start offsets are multiples of this

    def buf(nbytes):
        if pinned:
            return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).numpy()
        return np.empty(nbytes, np.uint8)

    def shard_views():
        out = []
        for _ in range(k + m):
            o = int(rng.integers(0, 4096 // residue)) * residue
            b = buf(n + o)
            out.append(b[o:o + n])
        return out

    src = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k + m)]
    rs = rsamd.ReedSolomon.create(k, m)
    oc = oracle_lib.Codec(k, m)
    desc = f"k={k} m={m} n={n} off={off} cnt={cnt} pinned={pinned} residue={residue}"

    got = shard_views()
    for g, s in zip(got, src):
        g[:] = s
    ref = [s.copy() for s in src]
    rs.encodeParity(got, off, cnt)
    oc.encode_parity(ref, off, cnt)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert_equal_bytes(a, b, f"encode {desc} shard {i}")
    assert rs.isParityCorrect(got, off, cnt)
    if m:
        j = int(rng.choice([off, off + cnt - 1, int(rng.integers(off, off + cnt))]))
        s = k + int(rng.integers(0, m))
        got[s][j] ^= 0x41
        assert not rs.isParityCorrect(got, off, cnt), desc
        got[s][j] ^= 0x41

    present = _random_present(rng, k, m)
    got2 = shard_views()
    for g, s in zip(got2, src):
        g[:] = s
    ref = [s.copy() for s in src]
    rs.decodeMissing(got2, present, off, cnt)
    oc.decode_missing(ref, present, off, cnt)
    for i, (a, b) in enumerate(zip(got2, ref)):
        assert_equal_bytes(a, b, f"decode {desc} present={present} shard {i}")
