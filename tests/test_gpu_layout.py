"""GPU tests of the client file layout path against the
oracle's restatement of ReedSolomonEncoder / ReedSolomonDecoder
(client/ReedSolomonEncoder.java:56-85, client/ReedSolomonDecoder.java:33-103).

Covers the reference's committed fixture (ClientClusterCommTestFiles test.txt)
with every erasure subset, the round-trip tests of ReedSolomonTest.java:70-93,
ragged file sizes around the 4000-byte padding multiple, the fused k=4 kernels
and the generic split/merge paths (other k, block sizes, misaligned buffers).
"""
import hashlib
import itertools
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rand_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def test_reference_fixture_encode_decode(gpu, oracle_lib, golden_dir):
    from rsamd.layout import ReedSolomonDecoder, ReedSolomonEncoder
    raw = open(os.path.join(golden_dir, "reference_test.txt"), "rb").read()
    exp = json.load(open(os.path.join(golden_dir, "rs_small.json")))["reference_test_txt"]
    enc = ReedSolomonEncoder(raw)
    enc.encode()
    shards = enc.getShards()
    assert enc.getPaddedFileSize() == exp["padded_size"] and len(shards[0]) == exp["shard_len"]
    assert enc.getLastChunkIdx() == exp["padded_size"] // 1000 - 1
    assert [hashlib.sha256(s.tobytes()).hexdigest() for s in shards] == exp["shard_sha256"]
    for e in range(0, 3):
        for miss in itertools.combinations(range(6), e):
            sh = [s.copy() for s in shards]
            for j in miss:
                sh[j][:] = 0  # Client.java:235-238 zero-fills the absent shards
            dec = ReedSolomonDecoder(sh, [i not in miss for i in range(6)], len(sh[0]), len(raw))
            assert dec.getFileData() == raw, miss
            assert all(np.array_equal(a, b) for a, b in zip(sh, shards)), miss  # filled in place


@pytest.mark.parametrize("n", [0, 1, 999, 1000, 3999, 4000, 4001, 12345, 123457, 2_000_000])
def test_host_layout_matches_oracle(gpu, oracle_lib, n):
    from rsamd.layout import ReedSolomonDecoder, ReedSolomonEncoder
    data = _rand_bytes(n, n)
    enc = ReedSolomonEncoder(data)
    enc.encode()
    ref = oracle_lib.Codec(4, 2).file_encode(data)
    got = np.stack(enc.getShards()) if n else np.zeros((6, 0), np.uint8)
    assert np.array_equal(got, ref)
    if n:
        sh = [s.copy() for s in enc.getShards()]
        sh[0][:] = 0
        sh[5][:] = 0
        assert ReedSolomonDecoder(sh, [0, 1, 1, 1, 1, 0], len(sh[0]), n).getFileData() == data


def _dev(arr_or_n, pad=0):
    import torch
    if isinstance(arr_or_n, int):
        return torch.zeros(arr_or_n + pad, dtype=torch.uint8, device="cuda:0")
    t = torch.zeros(len(arr_or_n) + pad, dtype=torch.uint8, device="cuda:0")
    if len(arr_or_n):
        t[: len(arr_or_n)] = torch.from_numpy(np.frombuffer(arr_or_n, np.uint8).copy()).to("cuda:0")
    return t


@pytest.mark.parametrize("k,m,block,n,file_off,stride_mode", [
    (4, 2, 1000, 1_234_567, 0, "aligned"),   # fused kernels (the DFS shape)
    (4, 2, 1000, 1_234_567, 0, "exact"),     # stride = S = 8 mod 16 -> generic split/merge + stripe kernels
    (4, 2, 1000, 4000 * 37, 0, "aligned"),   # fused, exact multiple of k*block
    (4, 2, 1000, 9_999, 8, "aligned"),       # fused, 8-aligned file offset
    (4, 2, 1000, 77_777, 3, "aligned"),      # misaligned file -> generic split/merge
    (4, 2, 512, 100_000, 0, "exact"),        # another block size (S % 16 == 0: fused)
    (4, 2, 7, 5_000, 0, "aligned"),          # block % 8 != 0 -> byte split/merge
    (5, 3, 1000, 200_001, 0, "aligned"),     # k != 4 -> generic
    (10, 4, 1000, 500_000, 0, "aligned"),    # config-4 shape
    (4, 6, 1000, 60_000, 0, "aligned"),      # m > 4: fused first parity group + stripe kernel
])
def test_device_layout_paths(gpu, oracle_lib, k, m, block, n, file_off, stride_mode):
    import torch
    import rsamd
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    rs = rsamd.ReedSolomon.create(k, m)
    padded, S = file_layout(rs, n, block)
    data = _rand_bytes(n, k * 1000 + n)
    ref = oracle_lib.Codec(k, m).file_encode(data, block)
    assert ref.shape == (k + m, S)
    fdev = _dev(data, pad=file_off + 16)
    if file_off:
        fdev[file_off: file_off + n] = fdev[:n].clone()
    stride = S if stride_mode == "exact" else (S + 255) // 256 * 256
    sdev = _dev((k + m) * stride)
    encode_file_dev(rs, fdev.data_ptr() + file_off, n, sdev.data_ptr(), stride, block, torch.cuda.current_stream())
    got = sdev.cpu().numpy().reshape(k + m, stride)[:, :S]
    assert np.array_equal(got, ref)
    for miss in [(), (0,), (1, k), (k,), tuple(range(min(m, k)))]:
        s2 = sdev.clone()
        v = s2.view(k + m, stride)
        for j in miss:
            v[j, :S] = 0
        present = [i not in miss for i in range(k + m)]
        out = _dev(n, pad=file_off + 16)
        for wm in (False, True):
            out.zero_()
            decode_file_dev(rs, s2.data_ptr(), S, stride, present, out.data_ptr() + file_off, n, block, wm,
                            torch.cuda.current_stream())
            assert out[file_off: file_off + n].cpu().numpy().tobytes() == data, (miss, wm)
            assert int(out[file_off + n:].sum().item()) == 0  # nothing past the trimmed size
            if wm:
                assert np.array_equal(s2.cpu().numpy().reshape(k + m, stride)[:, :S], ref)


def test_large_file_round_trip(gpu):
    """256 MiB file through the fused kernels: encode, erase 2, decode, compare on device."""
    import torch
    import rsamd
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    rs = rsamd.ReedSolomon.create(4, 2)
    n = (256 << 20) + 12345
    _, S = file_layout(rs, n)
    f = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda:0")
    stride = (S + 255) // 256 * 256
    sh = torch.zeros(6 * stride, dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream()
    encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, stream=st)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    from rsamd import device
    from rsamd.device import StripeLayout
    device.verify(rs, sh.data_ptr(), StripeLayout(1, S, stride, 6 * stride), flag.data_ptr(), st)
    assert int(flag.item()) == 0
    v = sh.view(6, stride)
    v[1].zero_()
    v[4].zero_()
    out = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    decode_file_dev(rs, sh.data_ptr(), S, stride, [1, 0, 1, 1, 0, 1], out.data_ptr(), n, stream=st)
    assert torch.equal(out, f)


@pytest.mark.parametrize("k,m,block,n", [(4, 2, 1000, 80_000_123), (3, 2, 4096, 70_001_111)])
def test_host_file_paths_multi_chunk(gpu, oracle_lib, k, m, block, n):
    """rs_file_encode / rs_file_decode stage ~32 MiB of file per chunk over two
    streams: a file of 2-3 chunks and a ragged last row, every absent shard
    filled in place (decodeMissing semantics), against the oracle."""
    from rsamd.layout import ReedSolomonDecoder, ReedSolomonEncoder
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    enc = ReedSolomonEncoder(data, k, m, block)
    enc.encode()
    shards = enc.getShards()
    ref = oracle_lib.Codec(k, m).file_encode(data, block)
    assert np.array_equal(np.stack(shards), ref)
    for miss in [(), (0,), (1, k + m - 1), (k, k + 1) if m >= 2 else (k,)]:
        sh = [s.copy() for s in shards]
        for j in miss:
            sh[j][:] = 0
        got = ReedSolomonDecoder(sh, [i not in miss for i in range(k + m)], len(sh[0]), n, k, m, block).getFileData()
        assert got == data, miss
        assert all(np.array_equal(a, b) for a, b in zip(sh, shards)), miss
