"""Movable caller arrays (rs_set_relocator, include/rs_amd.h): the library
may touch caller memory only inside copy batches bracketed by the relocator's
acquire / release, at the addresses the last acquire gave.

The arrays here MOVE at every acquire, the way a compacting GC may move a
JVM's byte[]s between two critical regions: acquire copies each array to a
fresh NumPy buffer and poisons the old one, which stays allocated.  The call's
array arguments are non-canonical stand-in keys.  So a byte read outside a
batch, or from a stale address, reads poison (wrong results), a byte written
there lands in a dead buffer (missing results, and the dead buffer no longer
all poison), and a key dereferenced faults.  Every host entry point is run on
pageable arrays at sizes that take each of its paths (one signalled small
launch, the mirrored pipeline, the file paths' splits and merges, the master's
runs and its per-group form), against the oracle, bit-exact.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POISON = 0xEE
KEY0 = 0x4000_0000_0000_0000  # non-canonical on x86-64: never a real mapping


class _Reloc(C.Structure):
    _fields_ = [("user", C.c_void_p), ("n", C.c_int), ("keys", C.POINTER(C.c_void_p)),
                ("lens", C.POINTER(C.c_int64)),
                ("acquire", C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_void_p))),
                ("release", C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_void_p)))]


class MovingHeap:
    """Arrays that move at every acquire; keys stand in for their addresses."""

    def __init__(self, arrays):
        self.cur = [np.array(a, dtype=np.uint8) for a in arrays]
        self.dead = []
        self.acquires = self.releases = 0
        self.open = False
        n = len(self.cur)
        self.keys = (C.c_void_p * n)(*[KEY0 + (i << 36) for i in range(n)])
        self.lens = (C.c_int64 * n)(*[len(a) for a in self.cur])
        self._acq = _Reloc._fields_[4][1](self._acquire)
        self._rel = _Reloc._fields_[5][1](self._release)
        self.struct = _Reloc(None, n, self.keys, self.lens, self._acq, self._rel)

    def _acquire(self, user, base):
        assert not self.open, "acquire inside an open batch"
        self.open = True
        self.acquires += 1
        for i, a in enumerate(self.cur):
            moved = np.empty(max(1, len(a)), np.uint8)[: len(a)]
            moved[:] = a
            a[:] = POISON
            self.dead.append(a)
            self.cur[i] = moved
            base[i] = moved.ctypes.data if len(a) else KEY0  # (an empty array is never touched)
        return 0

    def _release(self, user, base):
        assert self.open
        self.open = False
        self.releases += 1

    def key(self, i, off=0):
        return C.cast(C.c_void_p(KEY0 + (i << 36) + off), C.POINTER(C.c_uint8))

    def ptrs(self, idx):
        return (C.POINTER(C.c_uint8) * len(idx))(*[self.key(i) for i in idx])

    def __enter__(self):
        from rsamd import _lib
        assert _lib.load().rs_set_relocator(C.byref(self.struct)) == 0
        return self

    def __exit__(self, *exc):
        from rsamd import _lib
        assert _lib.load().rs_set_relocator(None) == 0
        assert not self.open
        assert self.acquires == self.releases
        for d in self.dead:
            assert not np.any(d != POISON), "a byte was written at a stale address"


def _codec(k, m):
    import rsamd
    return rsamd.ReedSolomon.create(k, m)


@pytest.mark.parametrize("S", [1000, 4096, 200_000, 3 << 20])
def test_relocated_encode_decode_verify(gpu, oracle_lib, S):
    from rsamd import _lib
    k, m = 4, 2
    rng = np.random.default_rng(S)
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    want = [a.copy() for a in data] + [np.zeros(S, np.uint8) for _ in range(m)]
    oracle_lib.Codec(k, m).encode_parity(want, 0, S)
    rs = _codec(k, m)
    lib = _lib.load()
    heap = MovingHeap(data + [np.full(S, 7, np.uint8) for _ in range(m)])
    with heap:
        assert lib.rs_encode_parity(rs.handle, heap.ptrs(range(6)), 6, heap.lens, 0, S) == 0, _lib.last_error()
    assert heap.acquires >= 1
    for got, w in zip(heap.cur, want):
        assert np.array_equal(got, w)
    with heap:
        ok = C.c_int(0)
        assert lib.rs_is_parity_correct(rs.handle, heap.ptrs(range(6)), 6, heap.lens, 0, S, None, 0,
                                        C.byref(ok)) == 0
        assert ok.value == 1
    heap.cur[1][S // 2] ^= 1
    with heap:
        assert lib.rs_is_parity_correct(rs.handle, heap.ptrs(range(6)), 6, heap.lens, 0, S, None, 0,
                                        C.byref(ok)) == 0
        assert ok.value == 0
    heap.cur[1][S // 2] ^= 1
    heap.cur[0][:] = 0
    heap.cur[5][:] = 0
    present = np.array([0, 1, 1, 1, 1, 0], np.uint8)
    with heap:
        assert lib.rs_decode_missing(rs.handle, heap.ptrs(range(6)), 6, heap.lens,
                                     present.ctypes.data_as(_lib.u8p), 0, S) == 0, _lib.last_error()
    for got, w in zip(heap.cur, want):
        assert np.array_equal(got, w)


@pytest.mark.parametrize("F", [90_999, 5 << 20])
def test_relocated_file_calls(gpu, oracle_lib, F):
    """rs_file_encode / rs_file_decode (the client's split and merge on the
    host, the coding on the GPU) with the file and every shard movable."""
    from rsamd import _lib
    k, m, blk = 4, 2, 1000
    rng = np.random.default_rng(F)
    data = rng.integers(0, 256, F, dtype=np.uint8)
    want = oracle_lib.Codec(k, m).file_encode(data.tobytes(), blk)
    S = want.shape[1]
    rs = _codec(k, m)
    lib = _lib.load()
    heap = MovingHeap([np.zeros(S, np.uint8) for _ in range(k + m)] + [data])
    with heap:
        assert lib.rs_file_encode(rs.handle, heap.key(6), F, blk, heap.ptrs(range(6)), 6, heap.lens) == 0, \
            _lib.last_error()
    assert np.array_equal(np.stack(heap.cur[:6]), want)
    for s in (0, 5):
        heap.cur[s][:] = 0
    present = np.array([0, 1, 1, 1, 1, 0], np.uint8)
    out = MovingHeap(heap.cur[:6] + [np.zeros(F, np.uint8)])
    with out:
        assert lib.rs_file_decode(rs.handle, out.ptrs(range(6)), 6, out.lens, present.ctypes.data_as(_lib.u8p), S,
                                  blk, out.key(6), F) == 0, _lib.last_error()
    assert np.array_equal(out.cur[6], data)
    assert np.array_equal(np.stack(out.cur[:6]), want)
    # byteCntInShard short of the shard (the generic decode + host merge)
    for s in (0, 5):
        out.cur[s][:] = 0
    tail = MovingHeap(out.cur[:6] + [np.zeros(F, np.uint8)])
    with tail:
        assert lib.rs_file_decode(rs.handle, tail.ptrs(range(6)), 6, tail.lens, present.ctypes.data_as(_lib.u8p),
                                  S - blk, blk, tail.key(6), F) == 0, _lib.last_error()
    assert np.array_equal(tail.cur[6][: (S - blk) * k], data[: (S - blk) * k])


@pytest.mark.parametrize("N,many", [(700, False), (2049, False), (3001, True)])
def test_relocated_shard_major(gpu, oracle_lib, N, many):
    """The master's host arrays movable: runs (small and mirrored) and the
    per-group form (chunks through the DMA pipeline)."""
    from rsamd import _lib
    k, m, chunk = 4, 2, 1000
    T, L = k + m, N * chunk
    rng = np.random.default_rng(N)
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(T)]
    oracle_lib.Codec(k, m).encode_parity(rows, 0, L)
    present = np.ones((N, T), bool)
    if many:
        for g in range(0, N, 2):
            present[g, int(rng.integers(0, T))] = False
    else:
        present[:, 0] = False
        present[N // 2 + 1:, 3] = False
    heap = MovingHeap([np.where(np.repeat(present[:, s], chunk), r, 0x3C).astype(np.uint8)
                       for s, r in enumerate(rows)])
    with heap:
        assert lib_call(heap, present, chunk, N) == 0, _lib.last_error()
    for s in range(T):
        assert np.array_equal(heap.cur[s], rows[s]), s


def lib_call(heap, present, chunk, N):
    from rsamd import _lib
    rs = _codec(4, 2)
    p = np.ascontiguousarray(present).view(np.uint8)
    return _lib.load().rs_decode_groups_shard_major(rs.handle, heap.ptrs(range(6)), 6, heap.lens, chunk, N,
                                                    p.ctypes.data_as(_lib.u8p))


def test_relocated_code_some_shards(gpu, oracle_lib):
    """The CodingLoop plugin (rs_code_some_shards) with movable inputs and outputs."""
    from rsamd import _lib
    rng = np.random.default_rng(3)
    nin, nout, n = 5, 3, 300_000
    rows = [rng.integers(0, 256, nin, dtype=np.uint8) for _ in range(nout)]
    ins = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(nin)]
    want = [np.zeros(n, np.uint8) for _ in range(nout)]
    oracle_lib.code_some_shards(0, np.stack(rows), ins, want, 0, n)
    heap = MovingHeap(ins + [np.zeros(n, np.uint8) for _ in range(nout)])
    rp = (_lib.u8p * nout)(*[r.ctypes.data_as(_lib.u8p) for r in rows])
    with heap:
        assert _lib.load().rs_code_some_shards(rp, heap.ptrs(range(nin)), nin, heap.ptrs(range(nin, nin + nout)), nout,
                                               0, n) == 0, _lib.last_error()
    for got, w in zip(heap.cur[nin:], want):
        assert np.array_equal(got, w)


def test_relocator_acquire_failure_is_reported(gpu):
    """An acquire that fails: the batch is skipped and the call reports
    RS_E_INVALID; a relocator with bad members is refused."""
    from rsamd import _lib
    from rsamd.codec import RS_E_INVALID
    S = 4096
    heap = MovingHeap([np.zeros(S, np.uint8) for _ in range(6)])
    heap.struct.acquire = _Reloc._fields_[4][1](lambda u, b: 1)
    heap._acq = heap.struct.acquire
    lib = _lib.load()
    rs = _codec(4, 2)
    assert lib.rs_set_relocator(C.byref(heap.struct)) == 0
    try:
        rc = lib.rs_encode_parity(rs.handle, heap.ptrs(range(6)), 6, heap.lens, 0, S)
    finally:
        assert lib.rs_set_relocator(None) == 0
    assert rc == RS_E_INVALID and "acquire failed" in _lib.last_error()
    bad = _Reloc(None, 0, heap.keys, heap.lens, heap._acq, heap._rel)
    assert lib.rs_set_relocator(C.byref(bad)) == RS_E_INVALID
