"""The JNI shim's marshalling (jni/rs_jni_core.c) over the real librsamd
backend on the GPU, through the mock JNI environment of test_jni_core.py:
Java-array in, Java-array out, compared with the oracle byte for byte, for
small calls and calls of more than SLICE bytes per shard (one library call
either way, the arrays pinned only around the library's copy batches), with
the reference's offsets and erasure patterns (ReedSolomon.java:90-104,
175-272; ReedSolomonTest.java:77-93's {0, 5}); and with the mock as a
compacting GC that moves every array between batches.
"""
import ctypes as C

import numpy as np
import pytest

from test_jni_core import SLICE, Jvm, build_mock

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mocklib():
    return build_mock()


@pytest.fixture
def jvm(mocklib):
    return Jvm(mocklib)


@pytest.fixture(scope="module")
def codec104(native):
    h = C.c_void_p()
    assert native.rs_codec_create(10, 4, C.byref(h)) == 0
    yield h
    native.rs_codec_destroy(h)


@pytest.mark.parametrize("k,m,off,cnt", [(4, 2, 17, 100000), (4, 2, 3, SLICE + 4099), (10, 4, 0, 65536),
                                         (10, 4, 5, SLICE + 1)])
def test_encode_decode_through_shim(gpu, oracle_lib, native, jvm, k, m, off, cnt):
    h = C.c_void_p()
    assert native.rs_codec_create(k, m, C.byref(h)) == 0
    try:
        S = off + cnt + 11
        rng = np.random.default_rng(cnt)
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        ref = [d.copy() for d in data]
        oracle_lib.Codec(k, m).encode_parity(ref, off, cnt)
        arrs = [jvm.bytes(d) for d in data]
        jvm.lib.mock_encode_parity(1, h, jvm.objects(arrs), off, cnt)
        assert jvm.exception() == ("", "")
        for i in range(k + m):
            assert np.array_equal(jvm.read(arrs[i], S), ref[i]), i
        jvm.assert_clean()
        assert jvm.lib.mock_is_parity_correct(1, h, jvm.objects(arrs), off, cnt, None) == 1
        # erase and decode: {0, k+m-1} (the reference test's {0, 5} for 4+2), plus one more for 10+4
        miss = [0, k + m - 1] + ([3, 7] if k == 10 else [])
        present = [i not in miss for i in range(k + m)]
        for j in miss:
            arrs[j] = jvm.bytes(np.full(S, 0x5A, np.uint8))
        jvm.lib.mock_decode_missing(1, h, jvm.objects(arrs), jvm.bools(present), off, cnt)
        assert jvm.exception() == ("", "")
        for j in miss:
            got = jvm.read(arrs[j], S)
            assert np.array_equal(got[off:off + cnt], ref[j][off:off + cnt]), j
            assert (got[:off] == 0x5A).all() and (got[off + cnt:] == 0x5A).all()  # outside the range untouched
        jvm.assert_clean()
    finally:
        native.rs_codec_destroy(h)


@pytest.mark.parametrize("cnt", [5000, SLICE + 333])
def test_code_some_shards_through_shim(gpu, oracle_lib, jvm, cnt):
    rng = np.random.default_rng(cnt)
    nin, nout, off = 5, 3, 9
    S = off + cnt + 4
    rows = rng.integers(0, 256, (nout, nin), dtype=np.uint8)
    ins = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(nin)]
    want = [np.zeros(S, np.uint8) for _ in range(nout)]
    oracle_lib.code_some_shards(7, rows, ins, want, off, cnt)
    outs = [jvm.bytes(np.zeros(S, np.uint8)) for _ in range(nout)]
    R = jvm.objects([jvm.bytes(r) for r in rows])
    I = jvm.objects([jvm.bytes(a) for a in ins])
    jvm.lib.mock_code_some_shards(1, R, I, nin, jvm.objects(outs), nout, off, cnt)
    assert jvm.exception() == ("", "")
    for p in range(nout):
        assert np.array_equal(jvm.read(outs[p], S), want[p]), p
    assert jvm.lib.mock_check_some_shards(1, R, I, nin, jvm.objects(outs), nout, off, cnt) == 1
    jvm.assert_clean()


def test_recover_groups_shard_major_through_shim(gpu, oracle_lib, native, jvm):
    """NativeReedSolomon.recoverGroupsShardMajorDevice's marshalling over the
    real entry point: the master's layout on the GPU, a byte[] of flags with
    the offline set growing mid-loop, every chunk back as the oracle encoded
    it, the flags array released untouched."""
    import torch
    k, m, chunk, N, j = 4, 2, 1000, 3001, 1501
    T, L = k + m, N * chunk
    h = C.c_void_p()
    assert native.rs_codec_create(k, m, C.byref(h)) == 0
    rng = np.random.default_rng(21)
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)] + [np.zeros(L, np.uint8) for _ in range(m)]
    oracle_lib.Codec(k, m).encode_parity(rows, 0, L)
    want = np.concatenate(rows)
    flags = np.ones((N, T), np.uint8)
    flags[:j, 1] = 0
    flags[j:, [1, 4]] = 0
    host = want.copy()
    host[1 * L: 2 * L] = 0x3C
    host[4 * L + j * chunk: 5 * L] = 0x3C
    dev = torch.from_numpy(host).to("cuda:0")
    fl = jvm.bytes(flags.ravel())
    jvm.lib.mock_recover_groups_shard_major(1, h, dev.data_ptr(), L, chunk, N, fl, 0)
    assert jvm.exception() == ("", "")
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), want)
    assert np.array_equal(jvm.read(fl, N * T), flags.ravel())
    jvm.assert_clean()
    native.rs_codec_destroy(h)


@pytest.mark.parametrize("k,m,block,flen", [(4, 2, 1000, 90999), (4, 2, 1000, 4000 * (SLICE // 1000 + 7) + 1234),
                                            (10, 4, 1024, 3 * 1024 * 1024 + 5)])
def test_file_encode_decode_through_shim(gpu, oracle_lib, native, jvm, k, m, block, flen):
    """NativeReedSolomon.encodeFile / decodeFile's marshalling over
    rs_file_encode / rs_file_decode: the Java file in, the k+m shards out as
    the oracle's pad + split + encode writes them (ReedSolomonEncoder.java:
    56-85); then {0, k+m-1} erased, the shards rebuilt in place and the file
    back trimmed (ReedSolomonDecoder.java:33-39, 92-103).  The second case
    is more than one slice of block rows per shard."""
    h = C.c_void_p()
    assert native.rs_codec_create(k, m, C.byref(h)) == 0
    try:
        data = np.random.default_rng(flen).integers(0, 256, flen, dtype=np.uint8)
        ref = oracle_lib.Codec(k, m).file_encode(data.tobytes(), block)
        S = ref.shape[1]
        arrs = [jvm.bytes(np.full(S, 0xA5, np.uint8)) for _ in range(k + m)]
        jvm.lib.mock_file_encode(1, h, jvm.bytes(data), block, jvm.objects(arrs))
        assert jvm.exception() == ("", "")
        for i in range(k + m):
            assert np.array_equal(jvm.read(arrs[i], S), ref[i]), i
        jvm.assert_clean()
        present = [i not in (0, k + m - 1) for i in range(k + m)]
        for i in (0, k + m - 1):
            arrs[i] = jvm.bytes(np.zeros(S, np.uint8))
        out = jvm.bytes(np.full(flen, 0x11, np.uint8))
        jvm.lib.mock_file_decode(1, h, jvm.objects(arrs), jvm.bools(present), S, block, out, flen)
        assert jvm.exception() == ("", "")
        assert np.array_equal(jvm.read(out, flen), data)
        for i in range(k + m):
            assert np.array_equal(jvm.read(arrs[i], S), ref[i]), i
        jvm.assert_clean()
    finally:
        native.rs_codec_destroy(h)


def test_direct_buffers_through_shim(gpu, oracle_lib, native, jvm):
    """NativeReedSolomon.allocatePinned / freePinned and the ByteBuffer
    overloads over librsamd: shards and a file in pinned direct buffers from
    the shim's own allocator, coded in place, against the oracle."""
    k, m, n = 4, 2, (4 << 20) + 24
    h = C.c_void_p()
    assert native.rs_codec_create(k, m, C.byref(h)) == 0

    def view(buf, size):
        return np.ctypeslib.as_array(C.cast(jvm.lib.mock_data(buf), C.POINTER(C.c_uint8)), shape=(size,))

    try:
        bufs = [jvm.lib.mock_alloc_pinned(1, n) for _ in range(k + m)]
        assert all(bufs) and jvm.exception() == ("", "")
        rng = np.random.default_rng(5)
        for b in bufs:
            view(b, n)[:] = rng.integers(0, 256, n, dtype=np.uint8)
        ref = [view(b, n).copy() for b in bufs]
        oracle_lib.Codec(k, m).encode_parity(ref, 0, n)
        jvm.lib.mock_encode_parity_direct(1, h, jvm.objects(bufs), 0, n)
        assert jvm.exception() == ("", "")
        assert all(np.array_equal(view(b, n), r) for b, r in zip(bufs, ref))
        for j in (0, 5):
            view(bufs[j], n)[:] = 0
        jvm.lib.mock_decode_missing_direct(1, h, jvm.objects(bufs), jvm.bools([i not in (0, 5) for i in range(6)]), 0,
                                           n)
        assert jvm.exception() == ("", "")
        assert all(np.array_equal(view(b, n), r) for b, r in zip(bufs, ref))
        # the file calls: 3 shards' worth of file, 1000-byte blocks
        flen = 3 * n + 7
        S = -(-flen // 4000) * 1000
        fb = jvm.lib.mock_alloc_pinned(1, flen)
        view(fb, flen)[:] = rng.integers(0, 256, flen, dtype=np.uint8)
        fsh = [jvm.lib.mock_alloc_pinned(1, S) for _ in range(k + m)]
        jvm.lib.mock_file_encode_direct(1, h, fb, flen, 1000, jvm.objects(fsh))
        assert jvm.exception() == ("", "")
        want = oracle_lib.Codec(k, m).file_encode(view(fb, flen).tobytes(), 1000)
        assert all(np.array_equal(view(b, S), w) for b, w in zip(fsh, want))
        out = jvm.lib.mock_alloc_pinned(1, flen)
        view(fsh[0], S)[:] = 0
        jvm.lib.mock_file_decode_direct(1, h, jvm.objects(fsh), jvm.bools([False] + [True] * 5), S, 1000, out, flen)
        assert jvm.exception() == ("", "")
        assert np.array_equal(view(out, flen), view(fb, flen))
        for b in bufs + fsh + [fb, out]:
            jvm.lib.mock_drop_local()
            jvm.lib.mock_free_pinned(1, b)
        assert jvm.exception() == ("", "")
        jvm.assert_clean()
    finally:
        native.rs_codec_destroy(h)


def test_pageable_direct_buffers_through_shim(gpu, oracle_lib, native, jvm):
    """ByteBuffer.allocateDirect-style buffers (pageable C memory, here NumPy
    arrays) through the ByteBuffer overloads: the mirrored pipeline, same
    bytes as the oracle."""
    k, m, n = 4, 2, (3 << 20) + 40
    h = C.c_void_p()
    assert native.rs_codec_create(k, m, C.byref(h)) == 0
    try:
        rng = np.random.default_rng(6)
        bufs = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] + [np.zeros(n, np.uint8) for _ in range(m)]
        ref = [b.copy() for b in bufs]
        oracle_lib.Codec(k, m).encode_parity(ref, 0, n)
        jvm.lib.mock_encode_parity_direct(1, h, jvm.objects([jvm.direct(b) for b in bufs]), 0, n)
        assert jvm.exception() == ("", "")
        assert all(np.array_equal(b, r) for b, r in zip(bufs, ref))
        for j in (1, 4):
            bufs[j][:] = 0
        jvm.lib.mock_decode_missing_direct(1, h, jvm.objects([jvm.direct(b) for b in bufs]),
                                           jvm.bools([j not in (1, 4) for j in range(6)]), 0, n)
        assert jvm.exception() == ("", "")
        assert all(np.array_equal(b, r) for b, r in zip(bufs, ref))
        flen = 4 * n - 3
        f = rng.integers(0, 256, flen + 9, dtype=np.uint8)  # capacity past the file
        S = -(-flen // 4000) * 1000
        fsh = [np.zeros(S, np.uint8) for _ in range(k + m)]
        jvm.lib.mock_file_encode_direct(1, h, jvm.direct(f), flen, 1000, jvm.objects([jvm.direct(b) for b in fsh]))
        assert jvm.exception() == ("", "")
        want = oracle_lib.Codec(k, m).file_encode(f[:flen].tobytes(), 1000)
        assert all(np.array_equal(b, w) for b, w in zip(fsh, want))
        out = np.zeros(flen, np.uint8)
        fsh[2][:] = 0
        jvm.lib.mock_file_decode_direct(1, h, jvm.objects([jvm.direct(b) for b in fsh]),
                                        jvm.bools([j != 2 for j in range(6)]), S, 1000, jvm.direct(out), flen)
        assert jvm.exception() == ("", "")
        assert np.array_equal(out, f[:flen])
        jvm.assert_clean()
    finally:
        native.rs_codec_destroy(h)


@pytest.fixture
def moving(jvm):
    """The mock as a compacting GC: every critical get of an unpinned array
    moves it and unmaps the old mapping (an address kept past a region faults)."""
    jvm.lib.mock_moving(1)
    yield jvm
    jvm.lib.mock_moving(0)


@pytest.mark.parametrize("S", [100_000, (3 << 20) + 4099, (70 << 20) + 8])
def test_moving_arrays_shard_calls(gpu, oracle_lib, native, moving, S):
    """One library call per Java call with the arrays moving between the
    library's copy batches (the small-call pass; the mirrored pipeline's many
    batches): encode, verify, decode {0,5} against the oracle."""
    jvm = moving
    k, m = 4, 2
    h = C.c_void_p()
    assert native.rs_codec_create(k, m, C.byref(h)) == 0
    try:
        rng = np.random.default_rng(S)
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        ref = [d.copy() for d in data]
        oracle_lib.Codec(k, m).encode_parity(ref, 0, S)
        arrs = [jvm.bytes(d) for d in data]
        jvm.lib.mock_encode_parity(1, h, jvm.objects(arrs), 0, S)
        assert jvm.exception() == ("", "")
        assert all(np.array_equal(jvm.read(a, S), r) for a, r in zip(arrs, ref))
        moves = jvm.lib.mock_moves()
        assert moves >= 2 * (k + m)  # the probe and at least one batch each moved every array
        assert jvm.lib.mock_is_parity_correct(1, h, jvm.objects(arrs), 0, S, None) == 1
        for j in (0, 5):
            arrs[j] = jvm.bytes(np.full(S, 0x5A, np.uint8))
        jvm.lib.mock_decode_missing(1, h, jvm.objects(arrs), jvm.bools([i not in (0, 5) for i in range(6)]), 0, S)
        assert jvm.exception() == ("", "")
        assert all(np.array_equal(jvm.read(a, S), r) for a, r in zip(arrs, ref))
        jvm.assert_clean()
    finally:
        native.rs_codec_destroy(h)


@pytest.mark.parametrize("flen", [90_999, 9 << 20])
def test_moving_arrays_file_calls(gpu, oracle_lib, native, moving, flen):
    jvm = moving
    k, m = 4, 2
    h = C.c_void_p()
    assert native.rs_codec_create(k, m, C.byref(h)) == 0
    try:
        data = np.random.default_rng(flen).integers(0, 256, flen, dtype=np.uint8)
        ref = oracle_lib.Codec(k, m).file_encode(data.tobytes(), 1000)
        S = ref.shape[1]
        arrs = [jvm.bytes(np.full(S, 0xA5, np.uint8)) for _ in range(k + m)]
        jvm.lib.mock_file_encode(1, h, jvm.bytes(data), 1000, jvm.objects(arrs))
        assert jvm.exception() == ("", "")
        assert all(np.array_equal(jvm.read(a, S), r) for a, r in zip(arrs, ref))
        for i in (0, 5):
            arrs[i] = jvm.bytes(np.zeros(S, np.uint8))
        out = jvm.bytes(np.full(flen, 0x11, np.uint8))
        jvm.lib.mock_file_decode(1, h, jvm.objects(arrs), jvm.bools([i not in (0, 5) for i in range(6)]), S, 1000,
                                 out, flen)
        assert jvm.exception() == ("", "")
        assert np.array_equal(jvm.read(out, flen), data)
        assert all(np.array_equal(jvm.read(a, S), r) for a, r in zip(arrs, ref))
        jvm.assert_clean()
    finally:
        native.rs_codec_destroy(h)


def test_moving_arrays_code_some_shards(gpu, oracle_lib, moving):
    jvm = moving
    rng = np.random.default_rng(12)
    nin, nout, off, cnt = 6, 2, 3, (2 << 20) + 5
    S = off + cnt + 1
    rows = rng.integers(0, 256, (nout, nin), dtype=np.uint8)
    ins = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(nin)]
    want = [np.zeros(S, np.uint8) for _ in range(nout)]
    oracle_lib.code_some_shards(0, rows, ins, want, off, cnt)
    outs = [jvm.bytes(np.zeros(S, np.uint8)) for _ in range(nout)]
    R = jvm.objects([jvm.bytes(r) for r in rows])
    I = jvm.objects([jvm.bytes(a) for a in ins])
    jvm.lib.mock_code_some_shards(1, R, I, nin, jvm.objects(outs), nout, off, cnt)
    assert jvm.exception() == ("", "")
    assert all(np.array_equal(jvm.read(o, S), w) for o, w in zip(outs, want))
    jvm.assert_clean()


@pytest.mark.parametrize("move,N,grow", [(0, 2049, 1001), (1, 2049, 1001), (1, 600, None), (0, 3001, "many")])
def test_recover_groups_shard_major_host_through_shim(gpu, oracle_lib, native, jvm, move, N, grow):
    """NativeReedSolomon.recoverGroupsShardMajor(byte[][] ...) over the real
    entry point: the master's host arrays (one per server, padded past the
    groups), the offline set growing mid-loop (or changing every other group),
    the arrays moving between batches; every byte as the oracle encoded it."""
    k, m, chunk = 4, 2, 1000
    T, L = k + m, N * chunk
    h = C.c_void_p()
    assert native.rs_codec_create(k, m, C.byref(h)) == 0
    try:
        rng = np.random.default_rng(N + move)
        rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(T)]
        oracle_lib.Codec(k, m).encode_parity(rows, 0, L)
        want = [np.concatenate([r, np.full(77, 0xD7, np.uint8)]) for r in rows]
        flags = np.ones((N, T), np.uint8)
        if grow == "many":
            for g in range(0, N, 2):
                flags[g, int(rng.integers(0, T))] = 0
        elif grow is None:
            flags[:, 2] = 0
        else:
            flags[:grow, 1] = 0
            flags[grow:, [1, 4]] = 0
        arrs = [jvm.bytes(np.concatenate([np.where(np.repeat(flags[:, s], chunk).astype(bool), rows[s], 0x3C)
                                          .astype(np.uint8), np.full(77, 0xD7, np.uint8)])) for s in range(T)]
        jvm.lib.mock_moving(move)
        jvm.lib.mock_recover_groups_shard_major_host(1, h, jvm.objects(arrs), chunk, N, jvm.bytes(flags.ravel()))
        jvm.lib.mock_moving(0)
        assert jvm.exception() == ("", "")
        for s in range(T):
            assert np.array_equal(jvm.read(arrs[s], L + 77), want[s]), s
        jvm.assert_clean()
    finally:
        native.rs_codec_destroy(h)


def test_recover_groups_shard_major_direct_through_shim(gpu, oracle_lib, native, jvm):
    """The ByteBuffer[] overload: the master's arrays in the shim's pinned
    buffers (allocatePinned), coded in place across the link."""
    k, m, chunk, N = 4, 2, 1000, 2049
    T, L = k + m, N * chunk
    h = C.c_void_p()
    assert native.rs_codec_create(k, m, C.byref(h)) == 0

    def view(buf, size):
        return np.ctypeslib.as_array(C.cast(jvm.lib.mock_data(buf), C.POINTER(C.c_uint8)), shape=(size,))

    try:
        rng = np.random.default_rng(77)
        rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(T)]
        oracle_lib.Codec(k, m).encode_parity(rows, 0, L)
        bufs = [jvm.lib.mock_alloc_pinned(1, L) for _ in range(T)]
        for b, r in zip(bufs, rows):
            view(b, L)[:] = r
        flags = np.ones((N, T), np.uint8)
        flags[:, [0, 5]] = 0
        for s in (0, 5):
            view(bufs[s], L)[:] = 0
        jvm.lib.mock_recover_groups_shard_major_direct(1, h, jvm.objects(bufs), chunk, N, jvm.bytes(flags.ravel()))
        assert jvm.exception() == ("", "")
        assert all(np.array_equal(view(b, L), r) for b, r in zip(bufs, rows))
        for b in bufs:
            jvm.lib.mock_drop_local()
            jvm.lib.mock_free_pinned(1, b)
        jvm.assert_clean()
    finally:
        native.rs_codec_destroy(h)


def test_free_pinned_rejects_foreign_buffers(gpu, native, jvm):
    """NativeReedSolomon.freePinned on a direct buffer the shim did not
    allocate, on a slice of one, and twice: IllegalArgumentException each
    time (rs_host_free's check), the real allocation freed exactly once."""
    buf = jvm.lib.mock_alloc_pinned(1, 8192)
    assert buf and jvm.exception() == ("", "")
    jvm.lib.mock_drop_local()
    other = np.zeros(4096, np.uint8)
    jvm.lib.mock_free_pinned(1, jvm.direct(other))
    assert jvm.exception() == ("java/lang/IllegalArgumentException", "rs_host_free: not a live rs_host_alloc buffer")
    jvm.lib.mock_reset()
    inner = jvm.lib.mock_new_direct(C.c_void_p(jvm.lib.mock_data(buf) + 4096), 4096)
    jvm.lib.mock_free_pinned(1, inner)
    assert jvm.exception()[0] == "java/lang/IllegalArgumentException"
    jvm.lib.mock_reset()
    jvm.lib.mock_free_pinned(1, buf)
    assert jvm.exception() == ("", "")
    jvm.lib.mock_free_pinned(1, buf)
    assert jvm.exception()[0] == "java/lang/IllegalArgumentException"
