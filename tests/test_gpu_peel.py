"""The head peel of launch_gf_tables (kernels.hip): a batch of >= 256 MiB of
columns whose base is not on a 1 KiB / 128 B boundary codes its first columns
on the byte kernel and the rest on the 16-byte kernels from the boundary.
Results must not depend on where the batch sits: every byte at every offset
equals the line-aligned batch, which is checked against the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

K, M, S, B = 4, 2, 1 << 20, 256  # 256 MiB of columns: the peel's threshold
T = K + M


def _oracle_stripe(oracle_lib, host, lay, t, K=K, M=M):
    rows = [host[t * lay.stripe_stride + i * lay.shard_stride:][:S].copy() for i in range(K)]
    rows += [np.zeros(S, np.uint8) for _ in range(M)]
    oracle_lib.Codec(K, M).encode_parity(rows, 0, S)
    return rows[K:]


# (k, m, shard-stride pad, offsets): 1 KiB-multiple strides peel to 1 KiB; a
# 128-B pad leaves line-multiple strides only, so those batches peel to 128 B
@pytest.mark.parametrize("K,M,pad,offsets", [(4, 2, 0, (8, 16, 112, 1008, 2056)), (4, 2, 128, (48, 8)),
                                             (10, 4, 0, (16, 1000))], ids=["4p2", "4p2_pad128", "10p4"])
def test_misaligned_batches_equal_the_aligned_batch(gpu, oracle_lib, K, M, pad, offsets):
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    T = K + M
    rs = rsamd.ReedSolomon.create(K, M)
    lay = StripeLayout.packed(B, T, S, pad=pad)
    st = torch.cuda.current_stream()
    pool = torch.full((lay.nbytes + 4096,), 0x5A, dtype=torch.uint8, device="cuda:0")  # pads keep 0x5A
    base0 = pool.data_ptr()
    assert base0 % 4096 == 0
    device.fill_synthetic(base0, K, lay, 0xD15C, 0, st)
    device.encode(rs, base0, lay, st)
    want = pool[: lay.nbytes].clone()
    host = want.cpu().numpy()
    for t in (0, 1, B - 1):
        for p, par in enumerate(_oracle_stripe(oracle_lib, host, lay, t, K, M)):
            off = t * lay.stripe_stride + (K + p) * lay.shard_stride
            assert np.array_equal(host[off: off + S], par), (t, p)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    view = lambda o: pool[o: o + lay.nbytes].view(B, T, lay.shard_stride)  # noqa: E731
    present = [i >= 2 for i in range(T)]
    for o in offsets:
        b = base0 + o
        v = view(o)
        pool.fill_(0x5A)
        device.fill_synthetic(b, K, lay, 0xD15C, 0, st)
        device.encode(rs, b, lay, st)
        assert torch.equal(pool[o: o + lay.nbytes], want), ("encode", o)
        # decode {0,1}: the peeled head columns come back too
        v[:, 0:2, :S].fill_(0x3C)
        device.decode(rs, b, present, lay, st)
        assert torch.equal(pool[o: o + lay.nbytes], want), ("decode", o)
        # verify passes, then sees one wrong byte inside the peeled head
        flag.zero_()
        device.verify(rs, b, lay, flag.data_ptr(), st)
        assert int(flag.item()) == 0, o
        v[7, K + 1, 3] ^= 1
        device.verify(rs, b, lay, flag.data_ptr(), st)
        assert int(flag.item()) != 0, o
        v[7, K + 1, 3] ^= 1
        # nothing outside the batch was written
        assert int((pool[:o] != 0x5A).sum()) == 0 and int((pool[o + lay.nbytes:] != 0x5A).sum()) == 0
    del pool, want
    torch.cuda.empty_cache()


@pytest.mark.parametrize("pad", [0, 4096 + 8])
def test_shard_major_run_past_a_line_at_scale(gpu, oracle_lib, pad):
    """The master's offline set grows at odd group 300 033 of 600 064 (the
    second run, 300 MB per server, starts 1000 B past a 1 KiB boundary):
    every chunk comes back, and the groups around the failure match the
    oracle's parity.  With a pad after each server's array, its sentinel
    bytes (and every byte at the runs' group boundaries) come back unchanged."""
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    from rsamd.recovery import recover_groups_shard_major_dev
    chunk, N, j = 1000, 600_064, 300_033
    rs = rsamd.ReedSolomon.create(K, M)
    stride = N * chunk + pad
    lay = StripeLayout(1, N * chunk, stride, T * stride)
    st = torch.cuda.current_stream()
    buf = torch.full((lay.nbytes,), 0xA5, dtype=torch.uint8, device="cuda:0")
    device.fill_synthetic(buf.data_ptr(), K, lay, 0x6A57E2, 0, st)
    device.encode(rs, buf.data_ptr(), lay, st)
    want = buf.clone()
    v = buf.view(T, stride)
    present = np.ones((N, T), bool)
    for g0, g1, miss in [(0, j, (0,)), (j, N, (0, 3))]:
        present[g0:g1, list(miss)] = False
        for s in miss:
            v[s, g0 * chunk: g1 * chunk].fill_(0x3C)
    recover_groups_shard_major_dev(buf.data_ptr(), stride, present, chunk, st)
    assert torch.equal(buf, want)
    if pad:
        assert int((buf.view(T, stride)[:, N * chunk:] != 0xA5).sum()) == 0
    w = want.view(T, stride)[:, : N * chunk].reshape(T, N, chunk)[:, j - 2: j + 3].cpu().numpy()
    for g in range(5):
        rows = [w[i, g].copy() for i in range(K)] + [np.zeros(chunk, np.uint8) for _ in range(M)]
        oracle_lib.Codec(K, M).encode_parity(rows, 0, chunk)
        for p in range(M):
            assert np.array_equal(w[K + p, g], rows[K + p]), (g, p)
    del buf, want, v
    torch.cuda.empty_cache()


@pytest.mark.parametrize("o", [8, 112])
def test_masked_patterns_on_a_misaligned_batch(gpu, o):
    """Per-stripe presence patterns (host flags and device bitmasks) on a
    batch o bytes past a line: the masked launches peel their head too."""
    import itertools
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout, presence_bits
    rs = rsamd.ReedSolomon.create(K, M)
    lay = StripeLayout.packed(B, T, S)
    st = torch.cuda.current_stream()
    pool = torch.full((lay.nbytes + 4096,), 0x5A, dtype=torch.uint8, device="cuda:0")
    b = pool.data_ptr() + o
    device.fill_synthetic(b, K, lay, 0xBEEF, 0, st)
    device.encode(rs, b, lay, st)
    want = pool.clone()
    allp = np.array([[i not in miss for i in range(T)] for e in range(M + 1)
                     for miss in itertools.combinations(range(T), e)], dtype=bool)
    pats = allp[np.random.default_rng(o).integers(0, len(allp), B)]
    v = pool[o: o + lay.nbytes].view(B, T, lay.shard_stride)
    mask = torch.from_numpy(~pats).to("cuda:0")
    for bits in (False, True):
        v.masked_fill_(mask[:, :, None], 0x3C)
        if bits:
            words = torch.from_numpy(presence_bits(pats).view(np.int32)).to("cuda:0")
            bad = torch.zeros(1, dtype=torch.int32, device="cuda:0")
            device.decode_masked_bits(rs, b, words.data_ptr(), lay, bad.data_ptr(), st)
            assert int(bad.item()) == 0
        else:
            device.decode_masked(rs, b, pats, lay, st)
        assert torch.equal(pool, want), bits
    # Undecodable stripes (fewer than k shards present) through the peeled
    # launch: each is counted exactly once and left untouched; the rest decode.
    rng = np.random.default_rng(o + 1)
    undec = np.sort(rng.choice(B, 7, replace=False))
    pats2 = pats.copy()
    pats2[undec] = np.array([i < K - 1 for i in range(T)])  # k - 1 present
    v.masked_fill_(mask[:, :, None], 0x3C)
    before = pool.clone()
    words = torch.from_numpy(presence_bits(pats2).view(np.int32)).to("cuda:0")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.decode_masked_bits(rs, b, words.data_ptr(), lay, bad.data_ptr(), st)
    assert int(bad.item()) == len(undec), (int(bad.item()), len(undec))
    got = pool[o: o + lay.nbytes].view(B, T * lay.shard_stride)
    ok = np.setdiff1d(np.arange(B), undec)
    ref = want[o: o + lay.nbytes].view(B, T * lay.shard_stride)
    old = before[o: o + lay.nbytes].view(B, T * lay.shard_stride)
    idx = torch.from_numpy(ok).to("cuda:0")
    assert torch.equal(got[idx], ref[idx])
    idx = torch.from_numpy(undec).to("cuda:0")
    assert torch.equal(got[idx], old[idx])
    del pool, want, v, mask, before, got, ref, old
    torch.cuda.empty_cache()
