"""The JNI shim's marshalling (jni/rs_jni_core.c) against a mock JNI
environment (tests/jni_mock/mock_env.c), on CPU.

rs_jni.c only adapts JNIEnv to rs_jni_core's interface; everything the natives
decide -- which exception the reference Java code would throw and with what
text (ReedSolomon.java:277-302 and :175-272, InputOutputByteTableCodingLoop
.java:12-44), local-reference accounting, pinning small calls in critical
regions vs copying large ones slice by slice, which arrays are committed --
is checked here.  A fake coding backend (data movement only) stands in for the
GPU; test_gpu_jni_core.py runs the same marshalling over librsamd on a GPU.

A call is one backend call with the Java arrays movable (rs_set_relocator):
one probing pin of every array (released without copy-back), then the
backend's own pins around its copy batches (the fake pins once per call).
With mock_moving(1) the mock is a compacting GC -- every critical get of an
unpinned array moves it and unmaps the old copy -- so an address kept past a
critical region faults.
"""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import ROOT

SLICE = 32 << 20  # RSJ_SLICE_BYTES

NPE = "java/lang/NullPointerException"
IAE = "java/lang/IllegalArgumentException"
ISE = "java/lang/IllegalStateException"
AIOOBE = "java/lang/ArrayIndexOutOfBoundsException"


def build_mock():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "jni_mock"))
    import mockjni
    return mockjni.load()


class Jvm:
    """Mock Java heap + the natives, with -Xcheck:jni-style books."""

    def __init__(self, lib):
        self.lib = lib
        lib.mock_reset()
        lib.mock_file_record((C.c_int64 * 129)(), 129)  # drop earlier tests' file-call records

    def bytes(self, arr):
        arr = np.ascontiguousarray(arr, dtype=np.uint8)
        o = self.lib.mock_new_bytes(len(arr))
        if len(arr):
            C.memmove(self.lib.mock_data(o), arr.ctypes.data, len(arr))
        return o

    def bools(self, flags):
        o = self.lib.mock_new_bools(len(flags))
        if len(flags):
            a = np.array([1 if f else 0 for f in flags], dtype=np.uint8)
            C.memmove(self.lib.mock_data(o), a.ctypes.data, len(a))
        return o

    def objects(self, elems):
        o = self.lib.mock_new_objects(len(elems))
        for i, e in enumerate(elems):
            self.lib.mock_set(o, i, e)
        return o

    def direct(self, arr):
        """A direct ByteBuffer over a NumPy array's memory (the array must outlive it)."""
        return self.lib.mock_new_direct(arr.ctypes.data, len(arr))

    def read(self, o, n):
        return np.ctypeslib.as_array(C.cast(self.lib.mock_data(o), C.POINTER(C.c_uint8)), shape=(n,)).copy()

    def exception(self):
        return self.lib.mock_exc_class().decode(), self.lib.mock_exc_message().decode()

    def stats(self):
        s = (C.c_longlong * 11)()
        self.lib.mock_stats(s)
        keys = ["live_refs", "max_live_refs", "capacity", "critical_open", "max_critical_open", "violations",
                "bytes_in", "bytes_out", "critical_gets", "commits", "aborts"]
        return dict(zip(keys, list(s)))

    def assert_clean(self):
        st = self.stats()
        assert st["live_refs"] == 0 and st["critical_open"] == 0 and st["violations"] == 0, st
        return st


@pytest.fixture(scope="module")
def mocklib():
    return build_mock()


@pytest.fixture
def jvm(mocklib):
    return Jvm(mocklib)


@pytest.fixture(scope="module")
def codec42(native):
    h = C.c_void_p()
    assert native.rs_codec_create(4, 2, C.byref(h)) == 0
    yield h
    native.rs_codec_destroy(h)


def shard_set(jvm, k, m, S, seed=0, lens=None):
    rng = np.random.default_rng(seed)
    data = [rng.integers(0, 256, (lens[i] if lens else S), dtype=np.uint8) for i in range(k + m)]
    return data, [jvm.bytes(d) for d in data]


def fake_parity(data, k, m, off, cnt):
    out = [d.copy() for d in data]
    for p in range(m):
        x = np.full(cnt, p + 1, dtype=np.uint8)
        for i in range(k):
            x ^= data[i][off:off + cnt]
        out[k + p][off:off + cnt] = x
    return out


def slices(cnt):
    return max(1, -(-cnt // SLICE))


@pytest.mark.parametrize("off,cnt,copy", [(100, 500, 0), (0, SLICE, 0), (7, SLICE + 1, 0), (3, 2 * SLICE + 12345, 0),
                                          (7, SLICE + 1, 1), (100, 500, 1)])
def test_encode_one_call(jvm, codec42, off, cnt, copy):
    """One backend call whatever the size: the probe pins all 6 arrays and
    releases them without copy-back, the backend's pin commits the 2 parity
    arrays and aborts the 4 data arrays, no byte copied on the host; when the
    JVM reports copies, the call copies slices through C buffers."""
    S = off + cnt + 50
    data, arrs = shard_set(jvm, 4, 2, S, seed=cnt)
    jvm.lib.mock_force_copy(copy)
    jvm.lib.mock_encode_parity(0, codec42, jvm.objects(arrs), off, cnt)
    jvm.lib.mock_force_copy(0)
    assert jvm.exception() == ("", "")
    want = fake_parity(data, 4, 2, off, cnt)
    for i in range(6):
        assert np.array_equal(jvm.read(arrs[i], S), want[i]), i
    st = jvm.assert_clean()
    if copy:  # one probing pin, then slices copied in and out
        assert st["critical_gets"] == 6 and st["aborts"] == 6 and st["commits"] == 0
        assert st["bytes_in"] == 4 * cnt and st["bytes_out"] == 2 * cnt
    else:
        assert st["critical_gets"] == 12 and st["commits"] == 2 and st["aborts"] == 10
        assert st["bytes_in"] == 0 and st["bytes_out"] == 0 and st["max_critical_open"] == 6


@pytest.mark.parametrize("cnt", [64, SLICE + 64])
def test_encode_check_order_and_messages(jvm, codec42, cnt):
    S = cnt + 10
    # wrong number of shards: reported before any element is touched (a null one included)
    _, arrs = shard_set(jvm, 4, 1, S)
    jvm.lib.mock_encode_parity(0, codec42, jvm.objects(arrs + [None]), 0, cnt)
    assert jvm.exception() == (IAE, "wrong number of shards: 6") or jvm.exception()[0] == NPE
    jvm.lib.mock_reset()
    jvm.lib.mock_encode_parity(0, codec42, jvm.objects(arrs), 0, cnt)
    assert jvm.exception() == (IAE, "wrong number of shards: 5")
    assert jvm.stats()["max_live_refs"] == 0
    cases = [
        ([S] * 5 + [S + 1], 0, cnt, "Shards are different sizes"),
        ([S] * 6, -1, cnt, "offset is negative: -1"),
        ([S] * 6, 0, -5, "byteCount is negative: -5"),
        ([S] * 6, 11, cnt, f"buffers to small: {cnt}11"),  # Java concatenates the strings (ReedSolomon.java:300)
    ]
    for lens, off, c, msg in cases:
        jvm.lib.mock_reset()
        data, arrs = shard_set(jvm, 4, 2, None, lens=lens)
        jvm.lib.mock_encode_parity(0, codec42, jvm.objects(arrs), off, c)
        assert jvm.exception() == (IAE, msg), (lens, off, c)
        for i in range(6):
            assert np.array_equal(jvm.read(arrs[i], lens[i]), data[i])  # nothing written
        jvm.assert_clean()


def test_encode_null_shard_npe(jvm, codec42):
    _, arrs = shard_set(jvm, 4, 2, 100)
    arrs[3] = None
    jvm.lib.mock_encode_parity(0, codec42, jvm.objects(arrs), 0, 10)
    assert jvm.exception()[0] == NPE
    jvm.assert_clean()
    jvm.lib.mock_reset()
    jvm.lib.mock_encode_parity(0, codec42, None, 0, 10)
    assert jvm.exception()[0] == NPE


def fake_decode(data, present, off, cnt):
    out = [d.copy() for d in data]
    for j, p in enumerate(present):
        if p:
            continue
        x = np.full(cnt, 0x80 ^ j, dtype=np.uint8)
        for i, q in enumerate(present):
            if q:
                x ^= data[i][off:off + cnt]
        out[j][off:off + cnt] = x
    return out


@pytest.mark.parametrize("cnt,copy", [(1000, 0), (SLICE + 1000, 0), (SLICE + 1000, 1)])
def test_decode_roles_and_commit(jvm, codec42, cnt, copy):
    S = cnt + 5
    present = [False, True, True, True, True, False]
    data, arrs = shard_set(jvm, 4, 2, S, seed=5)
    jvm.lib.mock_force_copy(copy)
    jvm.lib.mock_decode_missing(0, codec42, jvm.objects(arrs), jvm.bools(present), 5, cnt)
    jvm.lib.mock_force_copy(0)
    assert jvm.exception() == ("", "")
    want = fake_decode(data, present, 5, cnt)
    for i in range(6):
        assert np.array_equal(jvm.read(arrs[i], S), want[i]), i
    st = jvm.assert_clean()
    if copy:  # (+6: the shardPresent booleans)
        assert st["bytes_in"] == 4 * cnt + 6 and st["bytes_out"] == 2 * cnt
    else:  # the missing shards are committed, the survivors released without copy-back (+6: the probe)
        assert st["commits"] == 2 and st["aborts"] == 4 + 6 and st["bytes_out"] == 0


def test_decode_present_array_checks(jvm, codec42):
    data, arrs = shard_set(jvm, 4, 2, 100)
    # sizes are checked first (ReedSolomon.java:185), then shardPresent[i] for i < 6
    jvm.lib.mock_decode_missing(0, codec42, jvm.objects(arrs), jvm.bools([True] * 5), -1, 10)
    assert jvm.exception() == (IAE, "offset is negative: -1")
    jvm.lib.mock_reset()
    jvm.lib.mock_decode_missing(0, codec42, jvm.objects(arrs), jvm.bools([True] * 5), 0, 10)
    assert jvm.exception() == (AIOOBE, "Index 5 out of bounds for length 5")
    jvm.assert_clean()
    jvm.lib.mock_reset()
    jvm.lib.mock_decode_missing(0, codec42, jvm.objects(arrs), None, 0, 10)
    assert jvm.exception()[0] == NPE
    jvm.assert_clean()
    # a longer shardPresent is fine (Java reads the first 6)
    jvm.lib.mock_reset()
    jvm.lib.mock_decode_missing(0, codec42, jvm.objects(arrs), jvm.bools([True] * 9), 0, 10)
    assert jvm.exception() == ("", "")


@pytest.mark.parametrize("cnt", [300, SLICE + 300])
def test_is_parity_correct(jvm, codec42, cnt):
    S = cnt + 20
    data, _ = shard_set(jvm, 4, 2, S, seed=9)
    good = fake_parity(data, 4, 2, 0, S)
    arrs = [jvm.bytes(d) for d in good]
    assert jvm.lib.mock_is_parity_correct(0, codec42, jvm.objects(arrs), 10, cnt, None) == 1
    jvm.assert_clean()
    bad = [d.copy() for d in good]
    bad[5][10 + cnt - 1] ^= 1
    arrs = [jvm.bytes(d) for d in bad]
    assert jvm.lib.mock_is_parity_correct(0, codec42, jvm.objects(arrs), 10, cnt, None) == 0
    assert jvm.exception() == ("", "")
    # tempBuffer shorter than firstByte + byteCount (ReedSolomon.java:150)
    assert jvm.lib.mock_is_parity_correct(0, codec42, jvm.objects(arrs), 10, cnt, jvm.bytes(np.zeros(cnt))) == 0
    assert jvm.exception() == (IAE, "tempBuffer is not big enough")
    st = jvm.assert_clean()
    assert st["commits"] == 0  # read-only: nothing committed


def fake_code(rows, ins, off, cnt):
    outs = []
    for row in rows:
        x = np.zeros(cnt, dtype=np.uint8)
        for i, a in enumerate(ins):
            x ^= (a[off:off + cnt].astype(np.uint16) + row[i]).astype(np.uint8)
        outs.append(x)
    return outs


@pytest.mark.parametrize("cnt,copy", [(777, 0), (SLICE + 777, 0), (SLICE + 777, 1)])
def test_code_some_shards_extra_entries_ignored(jvm, cnt, copy):
    rng = np.random.default_rng(3)
    nin, nout, off = 3, 2, 13
    S = off + cnt + 3
    ins = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(nin + 1)]  # one extra input (CodingLoop.java:63-73)
    rows = [rng.integers(0, 256, nin + 2, dtype=np.uint8) for _ in range(nout)]  # rows longer than inputCount
    outs = [np.full(S, 0xEE, dtype=np.uint8) for _ in range(nout + 1)]
    ia, oa = [jvm.bytes(a) for a in ins], [jvm.bytes(a) for a in outs]
    jvm.lib.mock_force_copy(copy)
    jvm.lib.mock_code_some_shards(0, jvm.objects([jvm.bytes(r) for r in rows]), jvm.objects(ia), nin,
                                  jvm.objects(oa), nout, off, cnt)
    jvm.lib.mock_force_copy(0)
    assert jvm.exception() == ("", "")
    want = fake_code(rows, ins[:nin], off, cnt)
    for p in range(nout):
        got = jvm.read(oa[p], S)
        assert np.array_equal(got[off:off + cnt], want[p])
        assert (got[:off] == 0xEE).all() and (got[off + cnt:] == 0xEE).all()
    assert (jvm.read(oa[nout], S) == 0xEE).all()
    st = jvm.assert_clean()
    if copy:  # (+ nout * nin: the matrix rows)
        assert st["bytes_in"] == nin * cnt + nout * nin and st["bytes_out"] == nout * cnt
    else:  # the probe, then the backend's pin
        assert st["critical_gets"] == (nin + nout) * 2 and st["commits"] == nout
        assert st["bytes_in"] == nout * nin and st["bytes_out"] == 0
    # checkSomeShards on what was just written: true, then false after a flip
    chk = [jvm.bytes(jvm.read(o, S)) for o in oa[:nout]]
    rows_o = jvm.objects([jvm.bytes(r) for r in rows])
    assert jvm.lib.mock_check_some_shards(0, rows_o, jvm.objects(ia), nin, jvm.objects(chk), nout, off, cnt) == 1
    flipped = jvm.read(chk[1], S)
    flipped[off + cnt // 2] ^= 4
    chk[1] = jvm.bytes(flipped)
    assert jvm.lib.mock_check_some_shards(0, rows_o, jvm.objects(ia), nin, jvm.objects(chk), nout, off, cnt) == 0
    jvm.assert_clean()


def test_code_some_shards_java_exceptions(jvm):
    S = 100
    ins = [jvm.bytes(np.zeros(S)) for _ in range(3)]
    outs = [jvm.bytes(np.zeros(S)) for _ in range(2)]
    rows = [jvm.bytes(np.ones(3)) for _ in range(2)]

    def call(rws, i, nin, o, nout, off, cnt):
        jvm.lib.mock_reset()
        jvm.lib.mock_code_some_shards(0, rws, i, nin, o, nout, off, cnt)
        jvm.assert_clean()
        return jvm.exception()

    R, I, O = jvm.objects(rows), jvm.objects(ins), jvm.objects(outs)
    assert call(R, I, 4, O, 2, 0, 10) == (AIOOBE, "Index 3 out of bounds for length 3")   # inputCount > inputs.length
    assert call(R, I, 3, O, 3, 0, 10) == (AIOOBE, "Index 2 out of bounds for length 2")   # rows shorter than outputs
    assert call(jvm.objects(rows + [None]), I, 3, jvm.objects(outs + [jvm.bytes(np.zeros(S))]), 3, 0, 10)[0] == NPE
    assert call(jvm.objects([rows[0], jvm.bytes(np.ones(2))]), I, 3, O, 2, 0, 10) == (
        AIOOBE, "Index 2 out of bounds for length 2")                                    # short matrix row
    assert call(R, I, 3, O, 2, 95, 10) == (AIOOBE, "Index 100 out of bounds for length 100")  # past the end
    assert call(R, I, 3, O, 2, -1, 10) == (AIOOBE, "Index -1 out of bounds for length 100")
    assert call(R, jvm.objects(ins[:2] + [None]), 3, O, 2, 0, 10)[0] == NPE
    assert call(R, None, 3, O, 2, 0, 10)[0] == NPE
    # no bytes to code: nothing thrown for in-range counts, nothing written
    assert call(R, I, 3, O, 2, 0, 0) == ("", "")
    assert call(R, I, 3, O, 0, 0, 10) == ("", "")


def test_many_shards_local_references(jvm, native):
    """255 + 1 shards: more element references than the 16 a native frame gets
    without EnsureLocalCapacity; every one is deleted before returning."""
    h = C.c_void_p()
    assert native.rs_codec_create(200, 56, C.byref(h)) == 0
    try:
        data, arrs = shard_set(jvm, 200, 56, 64)
        jvm.lib.mock_encode_parity(0, h, jvm.objects(arrs), 0, 64)
        assert jvm.exception() == ("", "")
        st = jvm.assert_clean()
        assert st["max_live_refs"] == 256 and st["capacity"] >= 256
    finally:
        native.rs_codec_destroy(h)


def test_critical_failure_releases_everything(jvm, codec42):
    _, arrs = shard_set(jvm, 4, 2, 100)
    jvm.lib.mock_fail_critical(1)
    jvm.lib.mock_encode_parity(0, codec42, jvm.objects(arrs), 0, 10)
    jvm.lib.mock_fail_critical(0)
    assert jvm.exception()[0] == "java/lang/OutOfMemoryError"
    jvm.assert_clean()


def test_real_backend_without_gpu_throws_illegal_state(jvm, codec42, native):
    """librsamd itself behind the shim: argument errors stay IAE, a missing
    device is IllegalStateException, and no array is written."""
    if native.rs_device_count() > 0:
        pytest.skip("a GPU is visible: tests/test_gpu_jni_core.py covers the real backend")
    data, arrs = shard_set(jvm, 4, 2, 100)
    jvm.lib.mock_encode_parity(1, codec42, jvm.objects(arrs), 0, 200)
    assert jvm.exception() == (IAE, "buffers to small: 2000")
    jvm.lib.mock_reset()
    jvm.lib.mock_encode_parity(1, codec42, jvm.objects(arrs), 0, 50)
    assert jvm.exception()[0] == ISE
    for i in range(6):
        assert np.array_equal(jvm.read(arrs[i], 100), data[i])
    jvm.assert_clean()


# ---- recoverGroupsShardMajorDevice (rs_decode_groups_shard_major_dev) ----

def test_shard_major_marshalling(jvm, codec42):
    """The flags reach the entry point as one byte per shard per group, with
    the device pointer, strides and stream as given.  They are copied out
    (GetBooleanArrayRegion), never pinned: the library call can block, and a
    critical region held across it would stall the GC."""
    n = 7
    flags = np.random.default_rng(3).integers(0, 3, n * 6).astype(np.uint8)
    jvm.lib.mock_shard_major_rc(0)
    jvm.lib.mock_recover_groups_shard_major(0, codec42, 1 << 40, 123456, 1000, n, jvm.bytes(flags), 0xABC)
    assert jvm.exception() == ("", "")
    rec = (C.c_uint64 * 5)()
    got = (C.c_uint8 * len(flags))()
    jvm.lib.mock_shard_major_record(rec, got, len(flags))
    assert list(rec) == [1 << 40, 123456, 1000, n, 0xABC]
    assert bytes(got) == flags.tobytes()
    st = jvm.assert_clean()
    assert st["commits"] == 0 and st["critical_gets"] == 0 and st["bytes_in"] == len(flags)


def test_shard_major_argument_errors(jvm, codec42):
    jvm.lib.mock_recover_groups_shard_major(0, codec42, 1 << 20, 6000, 1000, 2, None, 0)
    assert jvm.exception() == (NPE, "present is null")
    jvm.lib.mock_reset()
    jvm.lib.mock_recover_groups_shard_major(0, codec42, 1 << 20, 6000, 1000, 2, jvm.bytes(np.ones(11, np.uint8)), 0)
    assert jvm.exception() == (IAE, "present has 11 flags; n_groups * total shards is 12")
    jvm.lib.mock_reset()
    jvm.lib.mock_recover_groups_shard_major(0, codec42, 1 << 20, -1, 1000, 2, jvm.bytes(np.ones(12, np.uint8)), 0)
    assert jvm.exception() == (IAE, "negative size")
    jvm.lib.mock_reset()
    jvm.lib.mock_shard_major_rc(-9)  # RS_E_HIP from the entry point -> IllegalStateException
    jvm.lib.mock_recover_groups_shard_major(0, codec42, 1 << 20, 6000, 1000, 2, jvm.bytes(np.ones(12, np.uint8)), 0)
    assert jvm.exception()[0] == ISE
    jvm.lib.mock_shard_major_rc(0)
    jvm.lib.mock_reset()
    jvm.assert_clean()


def test_shard_major_real_backend_rejects_before_any_work(jvm, codec42):
    """Through librsamd (no device needed: every group is validated first):
    a group with fewer than k servers is the reference's exception."""
    flags = np.ones((3, 6), np.uint8)
    flags[1, :3] = 0
    jvm.lib.mock_recover_groups_shard_major(1, codec42, 1 << 20, 3000, 1000, 3, jvm.bytes(flags.ravel()), 0)
    assert jvm.exception() == (IAE, "Not enough shards present")
    jvm.assert_clean()


# ---- the client's file layout: rsj_file_encode / rsj_file_decode ----

def file_calls(jvm):
    """(file length, shard length) of every backend file call since the last read."""
    rec = (C.c_int64 * 129)()
    jvm.lib.mock_file_record(rec, 129)
    return [(rec[1 + 2 * i], rec[2 + 2 * i]) for i in range(min(rec[0], 64))]


def split_file(data, k, m, block):
    """ReedSolomonEncoder.pad + splitFileToShards (ReedSolomonEncoder.java:62-85), numpy."""
    kb = k * block
    padded = len(data) if len(data) % kb == 0 else (len(data) // kb + 1) * kb
    buf = np.zeros(padded, np.uint8)
    buf[:len(data)] = data
    rows = buf.reshape(-1, k, block)
    return [np.ascontiguousarray(rows[:, i, :]).ravel() for i in range(k)] + [np.zeros(padded // k, np.uint8)
                                                                             for _ in range(m)]


def merge_file(shards, k, block, size):
    """mergeShardsToFile + trimPadding (ReedSolomonDecoder.java:62-66, 92-103), numpy."""
    S = len(shards[0])
    return np.stack([s.reshape(-1, block) for s in shards[:k]], axis=1).ravel()[:size] if S else np.zeros(0, np.uint8)


@pytest.fixture(scope="module")
def codec21(native):
    h = C.c_void_p()
    assert native.rs_codec_create(2, 1, C.byref(h)) == 0
    yield h
    native.rs_codec_destroy(h)


FILE_CASES = [(4, 2, 1000, 90999, 0), (4, 2, 1000, 92000, 0), (4, 2, 1000, 0, 0), (4, 2, 8, 4001, 1),
              (2, 1, 4096, 2 * SLICE + 3 * 4096 * 2 + 77, 0), (2, 1, 4096, 2 * SLICE + 3 * 4096 * 2 + 77, 1),
              (2, 1, 3000, 4 * SLICE + 5, 0)]


@pytest.mark.parametrize("k,m,block,flen,copy", FILE_CASES)
def test_file_encode_marshalling(jvm, codec42, codec21, k, m, block, flen, copy):
    """The whole file in, every shard out (data split + parity), committed;
    one library call whatever the size; when the JVM copies, a file of more
    than one slice of block rows per shard goes to the library in slices of
    whole rows through C buffers, the last one holding the ragged end."""
    codec = codec42 if k == 4 else codec21
    data = np.random.default_rng(flen).integers(0, 256, flen, dtype=np.uint8)
    want = split_file(data, k, m, block)
    S = len(want[0])
    want = fake_parity(want, k, m, 0, S)
    arrs = [jvm.bytes(np.full(S, 0xC3, np.uint8)) for _ in range(k + m)]
    jvm.lib.mock_force_copy(copy)
    jvm.lib.mock_file_encode(0, codec, jvm.bytes(data), block, jvm.objects(arrs))
    jvm.lib.mock_force_copy(0)
    assert jvm.exception() == ("", "")
    for i in range(k + m):
        assert np.array_equal(jvm.read(arrs[i], S), want[i]), i
    st = jvm.assert_clean()
    rows, per = S // block, max(1, SLICE // block)
    calls = file_calls(jvm)
    if rows <= per or not copy:
        assert calls == [(flen, S)]  # one call, with the arrays' own lengths
        if not copy:  # the probe, then the backend's pin: shards committed, the file aborted
            assert st["critical_gets"] == (k + m + 1) * 2 and st["commits"] == k + m
            assert st["bytes_in"] == 0 and st["bytes_out"] == 0
    else:
        n = -(-rows // per)
        assert [c[1] for c in calls] == [per * block] * (n - 1) + [(rows - (n - 1) * per) * block]
        assert sum(c[0] for c in calls) == flen
        assert st["bytes_in"] == flen and st["bytes_out"] == (k + m) * S


@pytest.mark.parametrize("k,m,block,flen,copy", FILE_CASES)
def test_file_decode_marshalling(jvm, codec42, codec21, k, m, block, flen, copy):
    """Survivors in, the absent shards rebuilt in place and the trimmed file
    out, sliced like the encode; only the rebuilt shards and the file are
    committed."""
    codec = codec42 if k == 4 else codec21
    data = np.random.default_rng(flen + 1).integers(0, 256, flen, dtype=np.uint8)
    shards = split_file(data, k, m, block)
    S = len(shards[0])
    shards = fake_parity(shards, k, m, 0, S)
    present = [i != 0 for i in range(k + m)]
    want = fake_decode(shards, present, 0, S)
    arrs = [jvm.bytes(shards[i] if present[i] else np.zeros(S, np.uint8)) for i in range(k + m)]
    out = jvm.bytes(np.full(flen + 3, 0x77, np.uint8))
    jvm.lib.mock_force_copy(copy)
    jvm.lib.mock_file_decode(0, codec, jvm.objects(arrs), jvm.bools(present), S, block, out, flen)
    jvm.lib.mock_force_copy(0)
    assert jvm.exception() == ("", "")
    for i in range(k + m):
        assert np.array_equal(jvm.read(arrs[i], S), want[i]), i
    got = jvm.read(out, flen + 3)
    assert np.array_equal(got[:flen], merge_file(want, k, block, flen)) and (got[flen:] == 0x77).all()
    st = jvm.assert_clean()
    rows, per = S // block, max(1, SLICE // block)
    calls = file_calls(jvm)
    if rows > per and copy:
        n = -(-rows // per)
        assert len(calls) == n and sum(c[0] for c in calls) == flen
        assert st["bytes_in"] == (k + m - 1) * S + k + m and st["bytes_out"] == S + flen
    elif not copy:  # one call: the rebuilt shard and the file committed (+ k + m + 1: the probe)
        assert calls == [(flen, S)]
        assert st["commits"] == 2 and st["aborts"] == (k + m - 1) + (k + m + 1)


def test_file_argument_errors(jvm, codec42):
    """The library's own checks and texts (real backend; none needs a device)
    and the shim's: a null file is NullPointerException, a fileOut shorter than
    fileSize ArrayIndexOutOfBoundsException, and nothing is written."""
    def enc(file, block, arrs):
        jvm.lib.mock_reset()
        jvm.lib.mock_file_encode(1, codec42, file, block, jvm.objects(arrs))
        jvm.assert_clean()
        return jvm.exception()

    data = jvm.bytes(np.arange(9000) % 251)
    full = [jvm.bytes(np.zeros(3000, np.uint8)) for _ in range(6)]
    assert enc(None, 1000, full)[0] == NPE
    assert enc(data, 1000, full[:5]) == (IAE, "wrong number of shards: 5")
    assert enc(data, 0, full) == (IAE, "block size must be positive")
    short = full[:5] + [jvm.bytes(np.zeros(2999, np.uint8))]
    assert enc(data, 1000, short) == (IAE, "shard 5 is shorter than 3000")
    assert all((jvm.read(a, 3000) == 0).all() for a in full)

    def dec(arrs, present, cnt, block, out, size, real=1):
        jvm.lib.mock_reset()
        jvm.lib.mock_file_decode(real, codec42, jvm.objects(arrs), present, cnt, block, out, size)
        jvm.assert_clean()
        return jvm.exception()

    out = jvm.bytes(np.zeros(12000, np.uint8))
    ok = jvm.bools([True] * 6)
    assert dec(full, ok, 3001, 1000, out, 9000) == (IAE, "buffers to small: 30010")
    assert dec(full, None, 3000, 1000, out, 9000)[0] == NPE
    assert dec(full, ok, 3000, 1000, None, 9000)[0] == NPE
    assert dec(full, jvm.bools([True] * 5), 3000, 1000, out, 9000) == (AIOOBE, "Index 5 out of bounds for length 5")
    assert dec(full, ok, 3000, 1000, jvm.bytes(np.zeros(8999, np.uint8)), 9000) == (
        AIOOBE, "Index 8999 out of bounds for length 8999")
    assert dec(full, jvm.bools([False, False, False, True, True, True]), 3000, 1000, out, 9000) == (
        IAE, "Not enough shards present")
    assert dec(full, ok, 3000, 1000, out, 12001)[0] == AIOOBE  # fileOut holds 12000
    assert dec(full, ok, 3000, 1000, jvm.bytes(np.zeros(12001, np.uint8)), 12001) == (
        IAE, "file size exceeds k * shard length")
    assert (jvm.read(out, 12000) == 0).all()


def test_file_real_backend_without_gpu_throws_illegal_state(jvm, codec42, native):
    if native.rs_device_count() > 0:
        pytest.skip("a GPU is visible: tests/test_gpu_jni_core.py covers the real backend")
    arrs = [jvm.bytes(np.zeros(1000, np.uint8)) for _ in range(6)]
    jvm.lib.mock_file_encode(1, codec42, jvm.bytes(np.ones(4000, np.uint8)), 1000, jvm.objects(arrs))
    assert jvm.exception()[0] == ISE
    assert all((jvm.read(a, 1000) == 0).all() for a in arrs)
    jvm.assert_clean()


# ---- direct ByteBuffers: pinned allocation and the ByteBuffer overloads ----

def test_direct_encode_decode_marshalling(jvm, codec42):
    """Shards by address and capacity: no critical region, no copy, no local
    reference left; the backend writes the caller's memory in place."""
    S, off, cnt = 5000, 7, 4000
    data = [np.random.default_rng(i).integers(0, 256, S, dtype=np.uint8) for i in range(6)]
    bufs = [d.copy() for d in data]
    jvm.lib.mock_encode_parity_direct(0, codec42, jvm.objects([jvm.direct(b) for b in bufs]), off, cnt)
    assert jvm.exception() == ("", "")
    want = fake_parity(data, 4, 2, off, cnt)
    assert all(np.array_equal(b, w) for b, w in zip(bufs, want))
    present = [True, False, True, True, True, False]
    jvm.lib.mock_decode_missing_direct(0, codec42, jvm.objects([jvm.direct(b) for b in bufs]), jvm.bools(present),
                                       off, cnt)
    assert jvm.exception() == ("", "")
    want = fake_decode(want, present, off, cnt)
    assert all(np.array_equal(b, w) for b, w in zip(bufs, want))
    st = jvm.assert_clean()
    assert st["critical_gets"] == 0 and st["bytes_in"] == 6 and st["bytes_out"] == 0  # (the 6 flags)


def test_direct_argument_errors(jvm, codec42):
    bufs = [np.zeros(100, np.uint8) for _ in range(6)]

    def enc(elems, off=0, cnt=10, real=1):
        jvm.lib.mock_reset()
        jvm.lib.mock_encode_parity_direct(real, codec42, elems, off, cnt)
        jvm.assert_clean()
        return jvm.exception()

    D = [jvm.direct(b) for b in bufs]
    assert enc(None)[0] == NPE
    assert enc(jvm.objects(D[:5])) == (IAE, "wrong number of shards: 5")
    assert enc(jvm.objects(D[:2] + [jvm.bytes(bufs[2])] + D[3:])) == (IAE, "shard 2 is not a direct buffer")
    assert enc(jvm.objects(D[:5] + [None]))[0] == NPE
    assert enc(jvm.objects(D), 95, 10) == (IAE, "buffers to small: 1095")
    jvm.lib.mock_reset()
    jvm.lib.mock_decode_missing_direct(1, codec42, jvm.objects(D), jvm.bools([True] * 5), 0, 10)
    assert jvm.exception() == (AIOOBE, "Index 5 out of bounds for length 5")
    jvm.assert_clean()
    assert all((b == 0).all() for b in bufs)


def test_direct_file_marshalling(jvm, codec42):
    k, m, block, flen = 4, 2, 1000, 90999
    data = np.random.default_rng(4).integers(0, 256, flen + 50, dtype=np.uint8)  # capacity past the file
    want = split_file(data[:flen], k, m, block)
    S = len(want[0])
    want = fake_parity(want, k, m, 0, S)
    bufs = [np.full(S, 0xC3, np.uint8) for _ in range(k + m)]
    jvm.lib.mock_file_encode_direct(0, codec42, jvm.direct(data), flen, block, jvm.objects([jvm.direct(b) for b in bufs]))
    assert jvm.exception() == ("", "")
    assert all(np.array_equal(b, w) for b, w in zip(bufs, want))
    present = [False, True, True, True, True, True]
    out = np.full(flen + 3, 0x77, np.uint8)
    jvm.lib.mock_file_decode_direct(0, codec42, jvm.objects([jvm.direct(b) for b in bufs]), jvm.bools(present), S,
                                    block, jvm.direct(out), flen)
    assert jvm.exception() == ("", "")
    dec = fake_decode(want, present, 0, S)
    assert np.array_equal(out[:flen], merge_file(dec, k, block, flen)) and (out[flen:] == 0x77).all()
    st = jvm.assert_clean()
    assert st["critical_gets"] == 0
    # the file length past the buffer, a heap array where a direct buffer belongs
    jvm.lib.mock_file_encode_direct(1, codec42, jvm.direct(data), len(data) + 1, block,
                                    jvm.objects([jvm.direct(b) for b in bufs]))
    assert jvm.exception() == (AIOOBE, f"Index {len(data)} out of bounds for length {len(data)}")
    jvm.lib.mock_reset()
    jvm.lib.mock_file_encode_direct(1, codec42, jvm.bytes(data), flen, block, jvm.objects([jvm.direct(b) for b in bufs]))
    assert jvm.exception() == (IAE, "fileData is not a direct buffer")
    jvm.lib.mock_reset()
    jvm.lib.mock_file_decode_direct(1, codec42, jvm.objects([jvm.direct(b) for b in bufs]), jvm.bools(present), S,
                                    block, jvm.direct(out[:flen - 1]), flen)
    assert jvm.exception() == (AIOOBE, f"Index {flen - 1} out of bounds for length {flen - 1}")
    jvm.assert_clean()


def test_alloc_free_pinned(jvm, native):
    """allocatePinned hands back a direct buffer of the asked capacity over
    the backend's allocation (one new local reference, which the Java caller
    owns); freePinned returns it."""
    buf = jvm.lib.mock_alloc_pinned(0, 4096)
    assert buf and jvm.exception() == ("", "") and jvm.lib.mock_host_live() == 1
    assert jvm.stats()["live_refs"] == 1
    jvm.lib.mock_drop_local()
    jvm.lib.mock_free_pinned(0, buf)
    assert jvm.lib.mock_host_live() == 0 and jvm.exception() == ("", "")
    assert not jvm.lib.mock_alloc_pinned(0, -1) and jvm.exception() == (IAE, "capacity is negative")
    jvm.lib.mock_reset()
    jvm.lib.mock_free_pinned(0, jvm.bytes(np.zeros(4)))
    assert jvm.exception() == (IAE, "not a direct buffer")
    jvm.lib.mock_reset()
    if native.rs_device_count() == 0:  # the real allocator needs a device
        assert not jvm.lib.mock_alloc_pinned(1, 4096) and jvm.exception()[0] == ISE
    jvm.assert_clean()


@pytest.mark.parametrize("copy", [0, 1])
def test_file_decode_sliced_short_file(jvm, codec21, copy):
    """A decode of shards longer than a slice whose fileSize ends in the
    first block rows: the absent shard is still rebuilt whole (the reference
    decodes all byteCntInShard bytes before it trims) -- in one call, or when
    the JVM copies in slices, the later ones writing no file bytes."""
    k, m, block = 2, 1, 4096
    S = 2 * SLICE + 3 * block
    rng = np.random.default_rng(8)
    shards = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8)]
    shards = fake_parity(shards, k, m, 0, S)
    present = [True, False, True]
    arrs = [jvm.bytes(s if p else np.zeros(S, np.uint8)) for s, p in zip(shards, present)]
    out = jvm.bytes(np.full(10, 0x77, np.uint8))
    jvm.lib.mock_force_copy(copy)
    jvm.lib.mock_file_decode(0, codec21, jvm.objects(arrs), jvm.bools(present), S, block, out, 5)
    jvm.lib.mock_force_copy(0)
    assert jvm.exception() == ("", "")
    want = fake_decode(shards, present, 0, S)
    assert np.array_equal(jvm.read(arrs[1], S), want[1])
    got = jvm.read(out, 10)
    assert np.array_equal(got[:5], want[0][:5]) and (got[5:] == 0x77).all()
    calls = file_calls(jvm)
    if copy:
        assert [c[0] for c in calls] == [5, 0, 0] and sum(c[1] for c in calls) == S
    else:
        assert calls == [(5, S)]
    jvm.assert_clean()


# ---- movable arrays: the mock as a compacting GC ----

@pytest.fixture
def moving(jvm):
    jvm.lib.mock_moving(1)
    yield jvm
    jvm.lib.mock_moving(0)


def test_moving_gc_shard_calls(moving, codec42):
    """Every critical get moves the array (the old mapping unmapped): encode,
    verify, decode and codeSomeShards still land every byte in the arrays'
    current places, and every release names the address its get returned."""
    jvm = moving
    S, off, cnt = 70_000, 5, 60_000
    data, arrs = shard_set(jvm, 4, 2, S, seed=21)
    jvm.lib.mock_encode_parity(0, codec42, jvm.objects(arrs), off, cnt)
    assert jvm.exception() == ("", "")
    want = fake_parity(data, 4, 2, off, cnt)
    assert all(np.array_equal(jvm.read(a, S), w) for a, w in zip(arrs, want))
    assert jvm.lib.mock_is_parity_correct(0, codec42, jvm.objects(arrs), off, cnt, None) == 1
    present = [True, False, True, True, False, True]
    jvm.lib.mock_decode_missing(0, codec42, jvm.objects(arrs), jvm.bools(present), off, cnt)
    assert jvm.exception() == ("", "")
    want = fake_decode(want, present, off, cnt)
    assert all(np.array_equal(jvm.read(a, S), w) for a, w in zip(arrs, want))
    rows = [np.arange(3, dtype=np.uint8) + r for r in range(2)]
    outs = [jvm.bytes(np.zeros(S, np.uint8)) for _ in range(2)]
    jvm.lib.mock_code_some_shards(0, jvm.objects([jvm.bytes(r) for r in rows]), jvm.objects(arrs[:3]), 3,
                                  jvm.objects(outs), 2, off, cnt)
    assert jvm.exception() == ("", "")
    got = fake_code(rows, want[:3], off, cnt)
    assert all(np.array_equal(jvm.read(o, S)[off:off + cnt], g) for o, g in zip(outs, got))
    st = jvm.assert_clean()
    assert jvm.lib.mock_moves() >= 4 * 6  # every call moved every array at least twice
    assert st["violations"] == 0


def test_moving_gc_file_calls(moving, codec42):
    jvm = moving
    k, m, block, flen = 4, 2, 1000, 90_999
    data = np.random.default_rng(22).integers(0, 256, flen, dtype=np.uint8)
    want = fake_parity(split_file(data, k, m, block), k, m, 0, 23_000)
    arrs = [jvm.bytes(np.zeros(23_000, np.uint8)) for _ in range(k + m)]
    jvm.lib.mock_file_encode(0, codec42, jvm.bytes(data), block, jvm.objects(arrs))
    assert jvm.exception() == ("", "")
    assert all(np.array_equal(jvm.read(a, 23_000), w) for a, w in zip(arrs, want))
    out = jvm.bytes(np.zeros(flen, np.uint8))
    present = [False, True, True, True, True, False]
    jvm.lib.mock_file_decode(0, codec42, jvm.objects(arrs), jvm.bools(present), 23_000, block, out, flen)
    assert jvm.exception() == ("", "")
    dec = fake_decode(want, present, 0, 23_000)
    assert np.array_equal(jvm.read(out, flen), merge_file(dec, k, block, flen))
    jvm.assert_clean()
    assert jvm.lib.mock_moves() > 0


# ---- recoverGroupsShardMajor on host arrays (rs_decode_groups_shard_major) ----

def fake_groups(servers, present, chunk):
    """The fake backend's per-group decode over the master's host arrays."""
    out = [s.copy() for s in servers]
    N, T = present.shape
    for g in range(N):
        at = [s[g * chunk:(g + 1) * chunk] for s in servers]
        dec = fake_decode(at, list(present[g]), 0, chunk)
        for s in range(T):
            out[s][g * chunk:(g + 1) * chunk] = dec[s]
    return out


@pytest.mark.parametrize("move", [0, 1])
def test_shard_major_host_marshalling(jvm, codec42, move):
    """byte[][] servers (one per server, groups back to back, padded past the
    groups) and byte[] flags: one backend call over movable arrays, every
    server committed (present chunks are read, absent ones written), the flags
    copied out; the ByteBuffer[] form reaches the same call by address."""
    N, chunk = 9, 100
    rng = np.random.default_rng(40 + move)
    servers = [rng.integers(0, 256, N * chunk + 37, dtype=np.uint8) for _ in range(6)]
    present = np.ones((N, 6), bool)
    present[:5, 0] = False
    present[5:, [0, 3]] = False
    want = fake_groups(servers, present, chunk)
    arrs = [jvm.bytes(s) for s in servers]
    jvm.lib.mock_moving(move)
    jvm.lib.mock_recover_groups_shard_major_host(0, codec42, jvm.objects(arrs), chunk, N,
                                                 jvm.bytes(present.astype(np.uint8).ravel()))
    jvm.lib.mock_moving(0)
    assert jvm.exception() == ("", "")
    for a, w in zip(arrs, want):
        assert np.array_equal(jvm.read(a, N * chunk + 37), w)
    st = jvm.assert_clean()
    assert st["commits"] == 6 and st["critical_gets"] == 12 and st["bytes_in"] == N * 6
    bufs = [s.copy() for s in servers]
    jvm.lib.mock_recover_groups_shard_major_direct(0, codec42, jvm.objects([jvm.direct(b) for b in bufs]), chunk, N,
                                                   jvm.bytes(present.astype(np.uint8).ravel()))
    assert jvm.exception() == ("", "")
    assert all(np.array_equal(b, w) for b, w in zip(bufs, want))
    jvm.assert_clean()


def test_shard_major_host_copying_jvm(jvm, codec42):
    """A JVM that copies: the groups go through C buffers, same results."""
    N, chunk = 5, 64
    rng = np.random.default_rng(44)
    servers = [rng.integers(0, 256, N * chunk, dtype=np.uint8) for _ in range(6)]
    present = np.ones((N, 6), bool)
    present[:, 2] = False
    want = fake_groups(servers, present, chunk)
    arrs = [jvm.bytes(s) for s in servers]
    jvm.lib.mock_force_copy(1)
    jvm.lib.mock_recover_groups_shard_major_host(0, codec42, jvm.objects(arrs), chunk, N,
                                                 jvm.bytes(present.astype(np.uint8).ravel()))
    jvm.lib.mock_force_copy(0)
    assert jvm.exception() == ("", "")
    assert all(np.array_equal(jvm.read(a, N * chunk), w) for a, w in zip(arrs, want))
    jvm.assert_clean()


def test_shard_major_host_argument_errors(jvm, codec42):
    """Java-side checks (null flags, a flag count that is not nGroups x 6,
    negative sizes, the shard count) and the library's (a short server, a
    group with fewer than k present: real backend, no device needed), none
    writing any array."""
    N, chunk = 4, 100
    servers = [np.full(N * chunk, i, np.uint8) for i in range(6)]
    arrs = [jvm.bytes(s) for s in servers]
    ok = jvm.bytes(np.ones(N * 6, np.uint8))

    def call(objs, flags, chunk_len=chunk, n=N, real=0):
        jvm.lib.mock_reset()
        jvm.lib.mock_recover_groups_shard_major_host(real, codec42, objs, chunk_len, n, flags)
        jvm.assert_clean()
        return jvm.exception()

    assert call(jvm.objects(arrs), None) == (NPE, "present is null")
    assert call(jvm.objects(arrs), jvm.bytes(np.ones(23, np.uint8))) == (
        IAE, "present has 23 flags; nGroups * total shards is 24")
    assert call(jvm.objects(arrs), ok, chunk_len=-1) == (IAE, "negative size")
    assert call(jvm.objects(arrs[:5]), ok) == (IAE, "wrong number of shards: 5")
    short = arrs[:5] + [jvm.bytes(np.zeros(N * chunk - 1, np.uint8))]
    assert call(jvm.objects(short), ok, real=1)[0] == IAE
    flags = np.ones((N, 6), np.uint8)
    flags[2, :3] = 0
    assert call(jvm.objects(arrs), jvm.bytes(flags.ravel()), real=1) == (IAE, "Not enough shards present")
    assert all(np.array_equal(jvm.read(a, N * chunk), s) for a, s in zip(arrs, servers))
