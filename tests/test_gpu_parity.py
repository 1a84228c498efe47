"""GPU parity tests: the HIP engine (through the C-ABI) against the oracle and
the committed golden fixtures.  Bit-exact everywhere (integer GF(2^8) work).

Coverage mirrors the reference's tests and edge cases:
  * encode parity of golden batches for 4+2, 10+4 and 17+3 (specialised and
    generic kernels);
  * decode of every erasure subset up to m (4+2), the reference test's {0, 5}
    pattern (ReedSolomonTest.java:77-93), and 10+4 {0,1,2,3};
  * parity verification (isParityCorrect) and single-byte corruption;
  * the Java host API with offsets / byte counts / ragged lengths, untouched
    bytes outside the range, and CodingLoop-level calls with random rows;
  * misaligned layouts (byte kernel) and <16-byte tails;
  * BASELINE full-size shapes through size-independent properties
    (encode -> erase -> decode round trip, verify == clean, sampled stripes
    against the oracle).
"""
import itertools
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED


def _torch():
    import torch
    return torch


def upload(batch: np.ndarray, shard_stride: int = None, extra: int = 0):
    """(B, T, S) host batch -> device buffer [stripe][shard][shard_stride]."""
    torch = _torch()
    B, T, S = batch.shape
    stride = shard_stride or S
    host = np.zeros((B, T, stride), dtype=np.uint8)
    host[:, :, :S] = batch
    flat = np.zeros(B * T * stride + extra, dtype=np.uint8)
    flat[: B * T * stride] = host.reshape(-1)
    dev = torch.from_numpy(flat).to("cuda:0")
    return dev, stride


def download(dev, B, T, S, stride):
    h = dev.cpu().numpy()[: B * T * stride].reshape(B, T, stride)
    return h[:, :, :S]


def layout(B, T, S, stride):
    from rsamd.device import StripeLayout
    return StripeLayout(B, S, stride, stride * T)


def run_encode(codec, batch, stride=None, base_off=0):
    torch = _torch()
    from rsamd import device
    B, T, S = batch.shape
    k = codec.getDataShardCount()
    work = batch.copy()
    work[:, k:, :] = 0
    dev, stride = upload(work, stride, extra=base_off)
    if base_off:  # shift the whole batch by base_off bytes (misaligned base)
        dev2 = torch.zeros_like(dev)
        dev2[base_off:] = dev[: dev.numel() - base_off]
        dev = dev2
    device.encode(codec, dev.data_ptr() + base_off, layout(B, T, S, stride), torch.cuda.current_stream())
    torch.cuda.synchronize()
    host = dev.cpu().numpy()[base_off: base_off + B * T * stride].reshape(B, T, stride)[:, :, :S]
    return host


def golden(golden_dir, name):
    d = np.load(os.path.join(golden_dir, name), allow_pickle=False)
    return d["shards"], d["matrix"]


@pytest.mark.parametrize("name,k,m", [("rs_4_2_s4096_b8.npz", 4, 2), ("rs_10_4_s1024_b4.npz", 10, 4),
                                      ("rs_17_3_s512_b2.npz", 17, 3)])
def test_encode_golden(gpu, golden_dir, name, k, m):
    import rsamd
    shards, matrix = golden(golden_dir, name)
    rs = rsamd.ReedSolomon.create(k, m)
    assert np.array_equal(rs.matrix(), matrix)
    out = run_encode(rs, shards)
    assert np.array_equal(out, shards)


def test_decode_every_erasure_subset_4_2(gpu, golden_dir):
    torch = _torch()
    import rsamd
    from rsamd import device
    shards, _ = golden(golden_dir, "rs_4_2_s4096_b8.npz")
    B, T, S = shards.shape
    rs = rsamd.ReedSolomon.create(4, 2)
    for e in (1, 2):
        for miss in itertools.combinations(range(6), e):
            work = shards.copy()
            work[:, list(miss), :] = 0xA5  # garbage in the erased buffers must be overwritten
            dev, stride = upload(work)
            present = [i not in miss for i in range(6)]
            device.decode(rs, dev.data_ptr(), present, layout(B, T, S, stride), torch.cuda.current_stream())
            torch.cuda.synchronize()
            assert np.array_equal(download(dev, B, T, S, stride), shards), miss


@pytest.mark.parametrize("miss", [(0, 1, 2, 3), (0,), (10, 11, 12, 13), (3, 9, 12), (1, 5, 10, 13)])
def test_decode_10_4(gpu, golden_dir, miss):
    torch = _torch()
    import rsamd
    from rsamd import device
    shards, _ = golden(golden_dir, "rs_10_4_s1024_b4.npz")
    B, T, S = shards.shape
    rs = rsamd.ReedSolomon.create(10, 4)
    work = shards.copy()
    work[:, list(miss), :] = 0
    dev, stride = upload(work)
    device.decode(rs, dev.data_ptr(), [i not in miss for i in range(T)], layout(B, T, S, stride),
                  torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert np.array_equal(download(dev, B, T, S, stride), shards)


def test_decode_generic_17_3(gpu, golden_dir):
    torch = _torch()
    import rsamd
    from rsamd import device
    shards, _ = golden(golden_dir, "rs_17_3_s512_b2.npz")
    B, T, S = shards.shape
    rs = rsamd.ReedSolomon.create(17, 3)
    for miss in [(0,), (2, 18), (0, 8, 16), (17, 18, 19)]:
        work = shards.copy()
        work[:, list(miss), :] = 0
        dev, stride = upload(work)
        device.decode(rs, dev.data_ptr(), [i not in miss for i in range(T)], layout(B, T, S, stride),
                      torch.cuda.current_stream())
        torch.cuda.synchronize()
        assert np.array_equal(download(dev, B, T, S, stride), shards), miss


@pytest.mark.parametrize("name,k,m", [("rs_4_2_s4096_b8.npz", 4, 2), ("rs_10_4_s1024_b4.npz", 10, 4)])
def test_verify_flags_every_position(gpu, golden_dir, name, k, m):
    """isParityCorrect (ReedSolomon.java:115-164) on the vector kernels: a single flipped bit in
    any parity shard, data shard, first/middle/last vector or stripe is caught, and the clean
    golden batch passes.  Covers every output slot of gf_vec_kernel<K,M,true> (10+4 included,
    whose accumulators are pinned before the compares)."""
    torch = _torch()
    import rsamd
    from rsamd import device
    shards, _ = golden(golden_dir, name)
    B, T, S = shards.shape
    rs = rsamd.ReedSolomon.create(k, m)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.current_stream()
    dev, stride = upload(shards)
    device.verify(rs, dev.data_ptr(), layout(B, T, S, stride), flag.data_ptr(), st)
    assert int(flag.item()) == 0
    for t, shard, col, bit in [(0, k, 0, 0), (B - 1, k + m - 1, S - 1, 7), (B // 2, k + 1, S // 2, 3),
                               (1, 0, 17, 5), (B - 1, k - 1, S - 16, 1)] + [(2 % B, k + p, 16 * p + 5, p) for p in range(m)]:
        bad = shards.copy()
        bad[t, shard, col] ^= 1 << bit
        dev, stride = upload(bad)
        flag.zero_()
        device.verify(rs, dev.data_ptr(), layout(B, T, S, stride), flag.data_ptr(), st)
        assert int(flag.item()) == 1, (t, shard, col, bit)


def test_verify_batch(gpu, golden_dir):
    torch = _torch()
    import rsamd
    from rsamd import device
    shards, _ = golden(golden_dir, "rs_4_2_s4096_b8.npz")
    B, T, S = shards.shape
    rs = rsamd.ReedSolomon.create(4, 2)
    dev, stride = upload(shards)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.verify(rs, dev.data_ptr(), layout(B, T, S, stride), flag.data_ptr(), torch.cuda.current_stream())
    assert int(flag.item()) == 0
    bad = shards.copy()
    bad[5, 5, 4095] ^= 0x10
    dev, stride = upload(bad)
    device.verify(rs, dev.data_ptr(), layout(B, T, S, stride), flag.data_ptr(), torch.cuda.current_stream())
    assert int(flag.item()) == 1


@pytest.mark.parametrize("stride_pad,base_off", [(3, 0), (0, 5), (13, 1)])
def test_misaligned_layouts_use_byte_path(gpu, golden_dir, stride_pad, base_off):
    import rsamd
    shards, _ = golden(golden_dir, "rs_4_2_s4096_b8.npz")
    rs = rsamd.ReedSolomon.create(4, 2)
    out = run_encode(rs, shards[:3], stride=4096 + stride_pad, base_off=base_off)
    assert np.array_equal(out, shards[:3])


# small ragged batches (<= 16 KiB of columns) take the byte kernel alone; larger
# ones the vector kernel plus a tail launch
@pytest.mark.parametrize("S", [1, 3, 15, 16, 17, 31, 1000, 4097, 5467, 20003, 70001])
def test_tails_and_ragged_lengths(gpu, oracle_lib, S):
    import rsamd
    rng = np.random.default_rng(S)
    B = 3
    batch = np.zeros((B, 6, S), np.uint8)
    batch[:, :4] = rng.integers(0, 256, (B, 4, S), dtype=np.uint8)
    c = oracle_lib.Codec(4, 2)
    for t in range(B):
        c.encode_parity([batch[t, i] for i in range(6)], 0, S)
    rs = rsamd.ReedSolomon.create(4, 2)
    stride = (S + 15) // 16 * 16  # aligned strides, len not a multiple of 16 -> tail kernel
    assert np.array_equal(run_encode(rs, batch, stride=stride), batch)


# ---------------------------------------------------------------------------
# Java host API
# ---------------------------------------------------------------------------

def test_host_api_encode_decode_ragged_golden(gpu, golden_dir):
    import rsamd
    d = np.load(os.path.join(golden_dir, "rs_ragged.npz"), allow_pickle=False)
    rs = rsamd.ReedSolomon.create(4, 2)
    for key in d.files:
        exp = d[key]
        n = exp.shape[1]
        sh = [exp[i].copy() for i in range(4)] + [np.zeros(n, np.uint8) for _ in range(2)]
        rs.encodeParity(sh, 0, n)
        assert all(np.array_equal(a, b) for a, b in zip(sh, exp)), key
        assert rs.isParityCorrect(sh, 0, n)
        assert rs.isParityCorrect(sh, 0, n, np.zeros(n, np.uint8))
        er = [s.copy() for s in sh]
        er[0][:] = 0
        er[5][:] = 0
        rs.decodeMissing(er, [False, True, True, True, True, False], 0, n)  # ReedSolomonTest.java:77-93
        assert all(np.array_equal(a, b) for a, b in zip(er, exp)), key


def test_host_api_offset_range_only(gpu, oracle_lib):
    import rsamd
    rng = np.random.default_rng(7)
    n, off, cnt = 5000, 123, 3001
    sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(6)]
    ref = [s.copy() for s in sh]
    oracle_lib.Codec(4, 2).encode_parity(ref, off, cnt)
    rs = rsamd.ReedSolomon.create(4, 2)
    rs.encodeParity(sh, off, cnt)
    assert all(np.array_equal(a, b) for a, b in zip(sh, ref))  # outside [off, off+cnt) untouched too
    assert rs.isParityCorrect(sh, off, cnt)
    assert not rs.isParityCorrect(sh, 0, n)
    sh[4][off + cnt - 1] ^= 1
    assert not rs.isParityCorrect(sh, off, cnt)
    assert rs.isParityCorrect(sh, off, cnt - 1)


def test_host_api_bytearray_and_large(gpu, oracle_lib):
    """Shards as bytearray (the JNI byte[] analogue) and a multi-chunk size (> 64 MiB staging chunk)."""
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    n = (64 << 20) + 4099
    rng = np.random.default_rng(11)
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(4)]
    sh = [bytearray(d.tobytes()) for d in data] + [bytearray(n) for _ in range(2)]
    rs.encodeParity(sh, 0, n)
    ref = [d.copy() for d in data] + [np.zeros(n, np.uint8) for _ in range(2)]
    oracle_lib.Codec(4, 2).encode_parity(ref, 0, n)
    assert np.frombuffer(bytes(sh[4]), np.uint8).tobytes() == ref[4].tobytes()
    assert np.frombuffer(bytes(sh[5]), np.uint8).tobytes() == ref[5].tobytes()
    sh[1] = bytearray(n)
    rs.decodeMissing(sh, [True, False, True, True, True, True], 0, n)
    assert bytes(sh[1]) == data[1].tobytes()


def test_host_api_every_erasure_pattern_10_4(gpu, oracle_lib):
    import rsamd
    rs = rsamd.ReedSolomon.create(10, 4)
    rng = np.random.default_rng(3)
    n = 777
    base = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(10)] + [np.zeros(n, np.uint8) for _ in range(4)]
    oracle_lib.Codec(10, 4).encode_parity(base, 0, n)
    for miss in list(itertools.combinations(range(14), 4))[::37] + [(0, 1, 2, 3)]:
        sh = [b.copy() for b in base]
        for j in miss:
            sh[j][:] = 0
        rs.decodeMissing(sh, [i not in miss for i in range(14)], 0, n)
        assert all(np.array_equal(a, b) for a, b in zip(sh, base)), miss


@pytest.mark.parametrize("nin,nout,n,off", [(4, 2, 4096, 0), (5, 3, 1001, 7), (1, 1, 1, 0), (12, 7, 333, 1),
                                            (32, 4, 2048, 16), (3, 9, 64, 3)])
def test_code_some_shards_random_rows(gpu, oracle_lib, nin, nout, n, off):
    import rsamd
    rng = np.random.default_rng(nin * 100 + nout)
    rows = rng.integers(0, 256, (nout, nin), dtype=np.uint8)
    inputs = [rng.integers(0, 256, n + off + 5, dtype=np.uint8) for _ in range(nin)]
    outs = [np.full(n + off + 5, 0x5A, np.uint8) for _ in range(nout)]
    ref = [o.copy() for o in outs]
    oracle_lib.code_some_shards(7, rows, inputs, ref, off, n)
    rsamd.codeSomeShards(rows, inputs, nin, outs, nout, off, n)
    assert all(np.array_equal(a, b) for a, b in zip(outs, ref))
    assert rsamd.checkSomeShards(rows, inputs, nin, outs, nout, off, n)
    outs[-1][off + n // 2] ^= 0x80
    assert not rsamd.checkSomeShards(rows, inputs, nin, outs, nout, off, n)


def test_host_api_threads(gpu, oracle_lib):
    """One shared codec used from several threads (the Java codec is a static final)."""
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    oc = oracle_lib.Codec(4, 2)
    errors = []

    def work(seed):
        try:
            rng = np.random.default_rng(seed)
            for _ in range(5):
                n = int(rng.integers(1, 200000))
                sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(4)] + [np.zeros(n, np.uint8)] * 0
                sh += [np.zeros(n, np.uint8), np.zeros(n, np.uint8)]
                ref = [s.copy() for s in sh]
                oc.encode_parity(ref, 0, n)
                rs.encodeParity(sh, 0, n)
                assert all(np.array_equal(a, b) for a, b in zip(sh, ref))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=work, args=(s,)) for s in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


# ---------------------------------------------------------------------------
# Full-size (BASELINE.json configs) through size-independent properties
# ---------------------------------------------------------------------------

def _sample_check(oracle_lib, dev_buf, lay, k, m, stripes, seed=SEED):
    """Copy a few stripes back and check them against the oracle."""
    total = k + m
    c = oracle_lib.Codec(k, m)
    for t in stripes:
        row = dev_buf[t * lay.stripe_stride:(t + 1) * lay.stripe_stride].cpu().numpy()
        sh = [row[i * lay.shard_stride: i * lay.shard_stride + lay.shard_len].copy() for i in range(total)]
        data = oracle_lib.fill_synthetic(k * lay.shard_len, seed, t)
        assert np.array_equal(np.concatenate(sh[:k]), data), t
        ref = [s.copy() for s in sh]
        for p in range(m):
            ref[k + p][:] = 0
        c.encode_parity(ref, 0, lay.shard_len)
        assert all(np.array_equal(a, b) for a, b in zip(sh, ref)), t


@pytest.mark.parametrize("k,m,S,B,miss", [
    (4, 2, 1 << 20, 4096, (0, 1)),      # configs[1]/[2]: 4+2 x 1 MiB x 4096
    (4, 2, 1 << 20, 4096, (0, 5)),      # the reference test's erasure pattern
    (10, 4, 4 << 20, 128, (0, 1, 2, 3)),  # configs[3] per-GPU share (1024 stripes / 8 GPUs)
    (4, 2, 4096, 1 << 20, (2, 3)),      # configs[4]: 1 M small stripes
])
def test_full_size_round_trip(gpu, oracle_lib, k, m, S, B, miss):
    torch = _torch()
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream()
    device.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, st)
    device.encode(rs, buf.data_ptr(), lay, st)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
    assert int(flag.item()) == 0
    _sample_check(oracle_lib, buf, lay, k, m, [0, 1, B // 2, B - 1])
    # erase, decode, compare against the untouched copy of the erased shards
    v = buf.view(B, lay.stripe_stride)
    saved = [v[:, j * lay.shard_stride: j * lay.shard_stride + S].clone() for j in miss]
    for j in miss:
        v[:, j * lay.shard_stride: j * lay.shard_stride + S].fill_(0)
    device.decode(rs, buf.data_ptr(), [i not in miss for i in range(k + m)], lay, st)
    for j, s in zip(miss, saved):
        assert torch.equal(v[:, j * lay.shard_stride: j * lay.shard_stride + S], s), j
    device.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
    assert int(flag.item()) == 0
    del buf, v, saved
    torch.cuda.empty_cache()


def test_copy_kernel(gpu):
    torch = _torch()
    from rsamd import device
    src = torch.randint(0, 256, ((1 << 20) + 7,), dtype=torch.uint8, device="cuda:0")
    dst = torch.zeros_like(src)
    device.copy(dst.data_ptr(), src.data_ptr(), src.numel(), torch.cuda.current_stream())
    assert torch.equal(dst, src)


@pytest.mark.parametrize("offset", [0, 12345])
def test_host_api_pinned_buffers(gpu, oracle_lib, offset):
    """Page-locked host shards take the direct-DMA pipeline (no pinned mirror):
    encode, decode and verify over ~8 chunks, bytes outside the range untouched."""
    import torch
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    n, count = (40 << 20) + 77, (40 << 20) - 12345 - 5
    rng = np.random.default_rng(21)
    sh = [torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(6)]
    for a in sh:
        a[:] = rng.integers(0, 256, n, dtype=np.uint8)
    ref = [a.copy() for a in sh]
    oracle_lib.Codec(4, 2).encode_parity(ref, offset, count)
    rs.encodeParity(sh, offset, count)
    for a, b in zip(sh, ref):
        assert np.array_equal(a, b)
    assert rs.isParityCorrect(sh, offset, count)
    sh[0][offset:offset + count] = 0
    sh[5][offset:offset + count] = 0
    rs.decodeMissing(sh, [False, True, True, True, True, False], offset, count)
    for a, b in zip(sh, ref):
        assert np.array_equal(a[offset:offset + count], b[offset:offset + count])


def test_host_file_paths_pinned(gpu, oracle_lib):
    """rs_file_encode / rs_file_decode on page-locked file and shard buffers."""
    import torch
    import rsamd
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    rs = rsamd.ReedSolomon.create(4, 2)
    n = 50_000_123
    data = torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy()
    data[:] = np.random.default_rng(22).integers(0, 256, n, dtype=np.uint8)
    _, S = file_layout(rs, n)
    sh = [torch.zeros(S, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(6)]
    file_encode_into(rs, data, sh)
    ref = oracle_lib.Codec(4, 2).file_encode(data.tobytes())
    assert np.array_equal(np.stack(sh), ref)
    sh[1][:] = 0
    sh[4][:] = 0
    out = torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy()
    file_decode_into(rs, sh, [True, False, True, True, False, True], S, out)
    assert np.array_equal(out, data)
    assert np.array_equal(np.stack(sh), ref)


@pytest.mark.parametrize("k,m", [(1, 1), (1, 255), (255, 1), (128, 128), (200, 56)])
def test_extreme_shard_counts(gpu, oracle_lib, k, m):
    """k + m up to the reference's limit of 256 (ReedSolomon.java:44-46):
    generic kernel with up to 255 inputs, up to 64 output groups, decode of the
    most erasures the code allows -- host API, device batch API and the
    per-stripe masked call, against the oracle."""
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    T, S = k + m, 4096 + 13  # 16-B vectors plus a byte tail
    rng = np.random.default_rng(T * 7 + k)
    ref = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
    oracle = oracle_lib.Codec(k, m)
    oracle.encode_parity(ref, 0, S)
    rs = rsamd.ReedSolomon.create(k, m)
    sh = [a.copy() if i < k else np.zeros(S, np.uint8) for i, a in enumerate(ref)]
    rs.encodeParity(sh, 0, S)
    assert all(np.array_equal(a, b) for a, b in zip(sh, ref))
    assert rs.isParityCorrect(sh, 0, S)
    # erase as many shards as the code allows: the first min(k, m) data shards, then parity
    miss = list(range(min(k, m))) + list(range(k, k + m - min(k, m)))
    present = [i not in miss for i in range(T)]
    for j in miss:
        sh[j][:] = 0
    rs.decodeMissing(sh, present, 0, S)
    assert all(np.array_equal(a, b) for a, b in zip(sh, ref))
    # device batch: 2 stripes, same pattern, then the masked call with another
    lay = StripeLayout.packed(2, T, S)
    host = np.zeros((2, T, lay.shard_stride), np.uint8)
    host[:, :, :S] = np.stack(ref)
    dev = torch.from_numpy(host.reshape(-1).copy()).to("cuda:0")
    dev.view(2, T, lay.shard_stride)[:, k:, :] = 0
    device.encode(rs, dev.data_ptr(), lay)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy().reshape(2, T, -1)[:, :, :S], host[:, :, :S])
    pats = np.array([present, [i != T - 1 for i in range(T)]], dtype=bool)
    for t in range(2):
        for j in range(T):
            if not pats[t, j]:
                dev.view(2, T, lay.shard_stride)[t, j, :S] = 0x5A
    device.decode_masked(rs, dev.data_ptr(), pats, lay)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy().reshape(2, T, -1)[:, :, :S], host[:, :, :S])


@pytest.mark.parametrize("k,m", [(6, 3), (8, 4), (17, 3)])
def test_compiled_wide_shapes(gpu, oracle_lib, k, m):
    """The compiled 6+m, 8+m and 17+m kernels (kernels.hip dispatch_vec), packed
    and granule batches: encode against the oracle, then every erasure count
    up to m (1 .. m outputs) decoded and compared, and verify clean."""
    torch = _torch()
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    rs = rsamd.ReedSolomon.create(k, m)
    S, B = 64 << 10, 6
    for lay in (StripeLayout.packed(B, k + m, S), device.GranuleLayout.make(B, k + m, S, 16 << 10)):
        buf = torch.zeros(lay.nbytes, dtype=torch.uint8, device="cuda:0")
        st = torch.cuda.current_stream()
        rng = np.random.default_rng(k * 10 + m)
        data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
        for t in range(B):
            for i in range(k):
                if isinstance(lay, StripeLayout):
                    off = t * lay.stripe_stride + i * lay.shard_stride
                    buf[off:off + S] = torch.from_numpy(data[t, i]).to("cuda:0")
                else:
                    device.copy_shard(lay, buf.data_ptr(), t, i, data[t, i].ctypes.data, True, st)
        torch.cuda.synchronize()
        device.encode(rs, buf.data_ptr(), lay, st)

        def shard(t, i):
            if isinstance(lay, StripeLayout):
                off = t * lay.stripe_stride + i * lay.shard_stride
                return buf[off:off + S].cpu().numpy()
            out = np.zeros(S, np.uint8)
            device.copy_shard(lay, buf.data_ptr(), t, i, out.ctypes.data, False, st)
            torch.cuda.synchronize()
            return out

        oc = oracle_lib.Codec(k, m)
        full = []
        for t in range(B):
            ref = [data[t, i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
            oc.encode_parity(ref, 0, S)
            full.append(ref)
            for p in range(m):
                assert np.array_equal(shard(t, k + p), ref[k + p]), (t, p)
        for e in range(1, m + 1):
            miss = sorted(rng.choice(k + m, e, replace=False).tolist())
            zero = np.zeros(S, np.uint8)
            for t in range(B):
                for j in miss:
                    if isinstance(lay, StripeLayout):
                        off = t * lay.stripe_stride + j * lay.shard_stride
                        buf[off:off + S] = 0
                    else:
                        device.copy_shard(lay, buf.data_ptr(), t, j, zero.ctypes.data, True, st)
            torch.cuda.synchronize()
            device.decode(rs, buf.data_ptr(), [i not in miss for i in range(k + m)], lay, st)
            for t in range(B):
                for j in miss:
                    assert np.array_equal(shard(t, j), full[t][j]), (e, miss, t, j)
        flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
        device.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
        assert int(flag.item()) == 0
