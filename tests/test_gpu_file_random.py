"""Seeded random cases of the client's file path (ReedSolomonEncoder.java:56-85,
ReedSolomonDecoder.java:62-103) through rs_file_encode / rs_file_decode and
their device forms, against the oracle's restatement, bit-exact: data and
parity shards of the padded, block-interleaved file; the file rebuilt from
the first k present shards with every absent shard filled in place
(decodeMissing semantics); random k, m, block sizes (multiples of 8 and not,
1 byte included), file sizes from empty to ~300 KB and random erasure sets.
"""
import numpy as np
import pytest
from bytes_report import assert_same

pytestmark = pytest.mark.gpu

BLOCKS = [1000, 8, 16, 24, 999, 7, 4096, 1, 1000, 520]


@pytest.mark.parametrize("case", range(24))
def test_file_paths_random(gpu, oracle_lib, case):
    import torch
    import rsamd
    from rsamd.layout import ReedSolomonDecoder, ReedSolomonEncoder, decode_file_dev, encode_file_dev, file_layout
    rng = np.random.default_rng(9000 + case)
    k = int(rng.integers(1, 11))
    m = int(rng.integers(0, 5))
    block = BLOCKS[case % len(BLOCKS)]
    n = int(rng.choice([0, 1, block, k * block, k * block + 1, int(rng.integers(1, 300_001))]))
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    oc = oracle_lib.Codec(k, m)
    ref = oc.file_encode(data, block)  # (k + m, S)

    enc = ReedSolomonEncoder(data, k, m, block)
    enc.encode()
    got = np.stack(enc.getShards()) if ref.shape[1] else np.zeros_like(ref)
    assert_same([got], [ref], (k, m, block, n))
    if n == 0:
        return
    S = ref.shape[1]
    e = int(rng.integers(0, m + 1))
    miss = sorted(int(x) for x in rng.choice(k + m, e, replace=False)) if e else []
    present = [i not in miss for i in range(k + m)]
    sh = [ref[i].copy() for i in range(k + m)]
    for j in miss:
        sh[j][:] = 0
    out = ReedSolomonDecoder(sh, present, S, n, k, m, block).getFileData()
    assert out == data, (k, m, block, n, miss)
    assert_same(sh, ref, (k, m, block, n, miss))  # filled in place
    assert oc.file_decode(ref, present, n, block) == data

    # the device forms on the same case: shards at a 256-rounded stride
    rs = rsamd.ReedSolomon.create(k, m)
    padded, S2 = file_layout(rs, n, block)
    assert S2 == S
    stride = (S + 255) // 256 * 256
    st = torch.cuda.current_stream()
    fdev = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to("cuda:0")
    sdev = torch.zeros((k + m) * stride, dtype=torch.uint8, device="cuda:0")
    encode_file_dev(rs, fdev.data_ptr(), n, sdev.data_ptr(), stride, block, st)
    v = sdev.view(k + m, stride)
    assert np.array_equal(v[:, :S].cpu().numpy(), ref), (k, m, block, n)
    for j in miss:
        v[j, :S] = 0
    odev = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    decode_file_dev(rs, sdev.data_ptr(), S, stride, present, odev.data_ptr(), n, block, True, st)
    assert odev.cpu().numpy().tobytes() == data, (k, m, block, n, miss)
    assert np.array_equal(v[:, :S].cpu().numpy(), ref), (k, m, block, n, miss)  # write_missing


@pytest.mark.parametrize("case", range(10))
def test_file_host_random_large(gpu, oracle_lib, case):
    """Host file calls at sizes that take the mirrored pipeline (shards of
    1 MiB and more): pageable file, shards and output, each a view at a
    random offset (8-byte aligned, or not for one case in four), split and
    merged on the host around the GPU's coding (capi.cpp file_encode_mirrored /
    file_decode_mirrored); random k, m, block and erasures, against the
    oracle."""
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    import rsamd
    rng = np.random.default_rng(9500 + case)
    k = int(rng.integers(1, 11))
    m = int(rng.integers(0, 5))
    block = int(rng.choice([1000, 8, 4096, 520, 24, 1000]))
    n = int(rng.integers(max(1, k) * (1 << 20), max(1, k) * (3 << 20)))
    step = 1 if case % 4 == 3 else 8

    def view(size):
        o = int(rng.integers(0, 4096 // step)) * step
        return np.empty(size + o, np.uint8)[o:o + size]

    rs = rsamd.ReedSolomon.create(k, m)
    oc = oracle_lib.Codec(k, m)
    _, S = file_layout(rs, n, block)
    f = view(n)
    f[:] = rng.integers(0, 256, n, dtype=np.uint8)
    sh = [view(S) for _ in range(k + m)]
    for a in sh:
        a[:] = 0xEE
    file_encode_into(rs, f, sh, block)
    ref = oc.file_encode(f.tobytes(), block)
    assert_same(sh, ref, (k, m, block, n))
    e = int(rng.integers(0, m + 1))
    miss = sorted(int(x) for x in rng.choice(k + m, e, replace=False)) if e else []
    for j in miss:
        sh[j][:] = 0
    out = view(n)
    out[:] = 0x33
    file_decode_into(rs, sh, [i not in miss for i in range(k + m)], S, out, block)
    assert_same([out], [f], (k, m, block, n, miss))
    assert_same(sh, ref, (k, m, block, n, miss))


@pytest.mark.parametrize("case", range(8))
def test_file_host_odd_blocks_pageable_and_pinned(gpu, oracle_lib, case):
    """The host file calls with blocks that are not 8-byte multiples (999,
    1001, 13, 4097) and files that end mid-row, on pageable arrays (the
    mirrored pipeline) and on caller-pinned ones (the direct kernels plus the
    host split / merge; odd blocks fall back to the staged pipeline there),
    every erasure count up to m, against the oracle."""
    import torch
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    import rsamd
    rng = np.random.default_rng(9600 + case)
    k, m = [(4, 2), (3, 2), (6, 3), (2, 1)][case % 4]
    block = [999, 1001, 13, 4097][(case // 2) % 4]
    pinned = case % 2 == 1
    n = int(rng.integers(k * (300 << 10), k * (900 << 10)))
    rs = rsamd.ReedSolomon.create(k, m)
    oc = oracle_lib.Codec(k, m)
    _, S = file_layout(rs, n, block)

    def buf(size):
        if pinned:
            return torch.empty(size, dtype=torch.uint8, pin_memory=True).numpy()
        o = int(rng.integers(0, 64))
        return np.empty(size + o, np.uint8)[o:o + size]

    f = buf(n)
    f[:] = rng.integers(0, 256, n, dtype=np.uint8)
    sh = [buf(S) for _ in range(k + m)]
    for a in sh:
        a[:] = 0xEE
    file_encode_into(rs, f, sh, block)
    ref = oc.file_encode(f.tobytes(), block)
    assert_same(sh, ref, (k, m, block, n, pinned))
    for e in range(m + 1):
        miss = sorted(int(x) for x in rng.choice(k + m, e, replace=False)) if e else []
        for j in miss:
            sh[j][:] = 0
        out = buf(n)
        out[:] = 0x33
        file_decode_into(rs, sh, [i not in miss for i in range(k + m)], S, out, block)
        assert_same([out], [f], (k, m, block, n, miss, pinned))
        assert_same(sh, ref, (k, m, block, n, miss, pinned))


PINNED_GEOMS = [(4, 2, 1000), (1, 1, 8), (10, 4, 1000), (3, 3, 520), (6, 1, 4096), (2, 4, 24), (7, 2, 8192),
                (5, 3, 16), (4, 2, 1000), (9, 4, 4096), (1, 4, 1000), (8, 2, 8), (4, 1, 65536), (2, 2, 40000)]


@pytest.mark.parametrize("case", range(len(PINNED_GEOMS)))
def test_file_pinned_random(gpu, oracle_lib, case):
    """Files and shards in the library's pinned buffers (rs_host_alloc): the
    encode's tiled kernel (layout.hip file_direct_tiled_kernel; 64 KiB of
    block rows per workgroup, one row when a row is larger, the column kernel
    past that) across k, m and block sizes, then a decode with random
    erasures (rebuilt data shards teed into the file by the direct kernels
    when block % 8 == 0), against the oracle."""
    import rsamd
    from rsamd.device import HostBuffer
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    k, m, block = PINNED_GEOMS[case]
    rng = np.random.default_rng(9700 + case)
    kb = k * block
    n = int(rng.integers(kb, max(kb + 1, 3_000_000 // kb * kb))) + int(rng.integers(0, 2)) * kb * 40
    rs = rsamd.ReedSolomon.create(k, m)
    oc = oracle_lib.Codec(k, m)
    _, S = file_layout(rs, n, block)
    f = HostBuffer(n)
    f.array[:] = rng.integers(0, 256, n, dtype=np.uint8)
    sh = [HostBuffer(S) for _ in range(k + m)]
    views = [b.array for b in sh]
    for v in views:
        v[:] = 0xEE
    file_encode_into(rs, f.array, views, block)
    ref = oc.file_encode(f.array.tobytes(), block)
    assert_same(views, list(ref), (k, m, block, n))
    e = int(rng.integers(1, m + 1))
    miss = sorted(int(x) for x in rng.choice(k + m, e, replace=False))
    for j in miss:
        views[j][:] = 0
    # the decode's kernels write rebuilt data shards straight into the file
    # (kernels.hpp DirectTee): 4 KiB of sentinel past the file's end must stay
    out = HostBuffer(n + 4096)
    out.array[:] = 0x33
    file_decode_into(rs, views, [i not in miss for i in range(k + m)], S, out.array[:n], block)
    assert np.array_equal(out.array[:n], f.array), (k, m, block, n, miss)
    assert (out.array[n:] == 0x33).all(), (k, m, block, n, miss)
    assert_same(views, list(ref), (k, m, block, n, miss))
    for b in sh + [f, out]:
        b.free()


@pytest.mark.parametrize("block", [1000, 8, 520])
def test_file_pinned_two_launch_groups(gpu, oracle_lib, block):
    """A pinned file decode whose plan needs two direct launches (six absent
    shards, at most four outputs per launch): the second launch's rebuilt data
    shards reach the file through its own tee entries (kernels.hpp
    DirectTee; block 520 is not a multiple of 8 and merges on the host)."""
    import rsamd
    from rsamd.device import HostBuffer
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    k, m = 8, 6
    rng = np.random.default_rng(7100 + block)
    n = k * block * 300 + int(rng.integers(1, k * block))
    rs = rsamd.ReedSolomon.create(k, m)
    oc = oracle_lib.Codec(k, m)
    _, S = file_layout(rs, n, block)
    f = HostBuffer(n)
    f.array[:] = rng.integers(0, 256, n, dtype=np.uint8)
    sh = [HostBuffer(S) for _ in range(k + m)]
    views = [b.array for b in sh]
    file_encode_into(rs, f.array, views, block)
    ref = oc.file_encode(f.array.tobytes(), block)
    assert_same(views, list(ref), (k, m, block, n))
    miss = [0, 2, 3, 5, 7, 9]  # five data shards (over both launches) and a parity shard
    for j in miss:
        views[j][:] = 0
    out = HostBuffer(n + 4096)
    out.array[:] = 0x33
    file_decode_into(rs, views, [i not in miss for i in range(k + m)], S, out.array[:n], block)
    assert np.array_equal(out.array[:n], f.array), (block, n)
    assert (out.array[n:] == 0x33).all(), (block, n)
    assert_same(views, list(ref), (k, m, block, n, miss))
    for b in sh + [f, out]:
        b.free()


@pytest.mark.parametrize("block", [1000, 8, 520, 1])
def test_file_small_pageable_two_launch_groups(gpu, oracle_lib, block):
    """The small pageable file decode (capi.cpp file_decode_zc_split: the
    survivors staged in the zero-copy buffer, padded to whole 16-byte vectors)
    with a plan of two direct launches, the second signalling completion for
    both (kernels.hpp DirectSignal), then the same file again with one launch.
    Shard lengths that are and are not multiples of 16."""
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    import rsamd
    k, m = 8, 6
    rng = np.random.default_rng(7300 + block)
    for n in (k * block * 37 + int(rng.integers(1, k * block + 1)), k * block * 5):
        rs = rsamd.ReedSolomon.create(k, m)
        oc = oracle_lib.Codec(k, m)
        data = rng.integers(0, 256, n, dtype=np.uint8)
        _, S = file_layout(rs, n, block)
        sh = [np.zeros(S, np.uint8) for _ in range(k + m)]
        file_encode_into(rs, data, sh, block)
        ref = oc.file_encode(data.tobytes(), block)
        assert_same(sh, list(ref), (block, n))
        for miss in ([0, 2, 3, 5, 7, 9], [1, 12]):
            for j in miss:
                sh[j][:] = 0x5A
            out = np.full(n + 64, 0x33, np.uint8)
            file_decode_into(rs, sh, [i not in miss for i in range(k + m)], S, out[:n], block)
            assert np.array_equal(out[:n], data), (block, n, miss)
            assert (out[n:] == 0x33).all(), (block, n, miss)
            assert_same(sh, list(ref), (block, n, miss))
