"""GPU tests of the host API's direct path (capi.cpp run_direct, kernels.hip
gf_direct_kernel): page-locked caller shards coded in place across the link by
one kernel, 16-byte vectors when every shard address shares a residue modulo
16, 8-byte vectors when they share one modulo 8, head and tail bytes one per
thread, and the staged pipeline when they share none.  Every case is checked
byte for byte against the oracle (ReedSolomon.java:90-104 encodeParity,
:175-272 decodeMissing, :115-164 isParityCorrect; CodingLoop.java:79-117).
Which path served a call is visible in a kernel trace (gf_direct_kernel vs the
staged copies); here each geometry is chosen so that the path is known.
"""
import numpy as np
import pytest
from bytes_report import assert_same

pytestmark = pytest.mark.gpu

N = (6 << 20) + 13  # above the single-chunk size: pinned calls take the direct path


def _pinned_block(nbytes):
    import torch
    return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).numpy()


def _shards(big, starts, n):
    return [big[s:s + n] for s in starts]


@pytest.mark.parametrize("page,gap,offset", [
    (16, 0, 0),       # one residue modulo 16: 16-byte vectors, no head
    (16, 0, 9),       # same residue 9: 16-byte vectors after a 7-byte head
    (16, 8, 0),       # residues 0 / 8 alternate: 8-byte vectors
    (16, 8, 5),       # 8-byte vectors after a 3-byte head
    (16, 3, 0),       # no common residue modulo 8: the staged pipeline
    (4096, 0, 16),    # one residue modulo 4 KiB (malloc'd arrays): a 4080-byte head to the page
    (4096, 0, 4095),  # a 1-byte head
])
def test_direct_encode_verify_decode(gpu, oracle_lib, page, gap, offset):
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    n = N + offset + 32
    slot = (n + page - 1) // page * page + gap
    big = _pinned_block(6 * slot + 4096 + 64)
    big = big[(-big.ctypes.data) % 4096:]  # page-aligned start
    sh = _shards(big, [i * slot for i in range(6)], n)
    rng = np.random.default_rng(100 + gap * 10 + offset + page)
    for a in sh:
        a[:] = rng.integers(0, 256, n, dtype=np.uint8)
    count = N
    ref = [a.copy() for a in sh]
    oracle_lib.Codec(4, 2).encode_parity(ref, offset, count)
    rs.encodeParity(sh, offset, count)
    for a, b in zip(sh, ref):  # parity in range, every byte outside it untouched
        assert_same([a], [b], '')
    assert rs.isParityCorrect(sh, offset, count)
    for pos in (offset, offset + 1, offset + count // 2, offset + count - 1):  # head, body, tail bytes
        sh[5][pos] ^= 0x10
        assert not rs.isParityCorrect(sh, offset, count), pos
        sh[5][pos] ^= 0x10
    assert rs.isParityCorrect(sh, offset, count)
    for miss in ((0, 5), (0, 1), (2,)):
        for j in miss:
            sh[j][offset:offset + count] = 0
        rs.decodeMissing(sh, [i not in miss for i in range(6)], offset, count)
        for a, b in zip(sh, ref):
            assert_same([a], [b], miss)


def test_direct_pageable_registered(gpu, oracle_lib):
    """Pageable numpy shards of a multi-chunk call: the pages wholly inside
    them are page-locked for the call (HostRegistration, mapped) and coded in
    place, the ragged ends through the staging buffer in the same launches."""
    import rsamd
    rs = rsamd.ReedSolomon.create(10, 4)
    n = (3 << 20) + 4096 + 5
    rng = np.random.default_rng(7)
    sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(10)] + [np.zeros(n, np.uint8) for _ in range(4)]
    ref = [a.copy() for a in sh]
    oracle_lib.Codec(10, 4).encode_parity(ref, 0, n)
    rs.encodeParity(sh, 0, n)
    assert_same(sh, ref, '')
    miss = (0, 3, 7, 12)
    for j in miss:
        sh[j][:] = 0
    rs.decodeMissing(sh, [i not in miss for i in range(14)], 0, n)
    assert_same(sh, ref, '')
    assert rs.isParityCorrect(sh, 0, n)


def test_direct_pageable_offset_range(gpu, oracle_lib):
    """A pageable call on a range far into its arrays: only whole pages inside
    the range are locked, so the kernel's addresses come from inside it."""
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    n, off, cnt = 12 << 20, (3 << 20) + 5, (4 << 20) + 3
    rng = np.random.default_rng(17)
    sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(6)]
    ref = [a.copy() for a in sh]
    oracle_lib.Codec(4, 2).encode_parity(ref, off, cnt)
    rs.encodeParity(sh, off, cnt)
    assert all(np.array_equal(a, b) for a, b in zip(sh, ref))  # outside the range untouched
    assert rs.isParityCorrect(sh, off, cnt)
    sh[2][off:off + cnt] = 0
    rs.decodeMissing(sh, [True, True, False, True, True, True], off, cnt)
    assert_same(sh, ref, '')


@pytest.mark.parametrize("nin,nout", [(7, 9), (32, 2), (33, 1)])
def test_direct_code_some_shards(gpu, oracle_lib, nin, nout):
    """CodingLoop.codeSomeShards / checkSomeShards on pinned buffers: more
    than kMaxOut outputs (several launch groups), the widest direct plan
    (32 inputs) and one input too many (staged)."""
    import rsamd
    n, off = (5 << 20) + 3, 11
    rng = np.random.default_rng(nin * 100 + nout)
    rows = rng.integers(0, 256, (nout, nin), dtype=np.uint8)
    big = _pinned_block((nin + nout) * (n + off + 16))
    step = n + off + 16
    bufs = _shards(big, [i * step for i in range(nin + nout)], n + off)
    for a in bufs[:nin]:
        a[:] = rng.integers(0, 256, n + off, dtype=np.uint8)
    for a in bufs[nin:]:
        a[:] = 0x5A
    inputs, outs = bufs[:nin], bufs[nin:]
    ref = [o.copy() for o in outs]
    oracle_lib.code_some_shards(7, rows, inputs, ref, off, n - off)
    rsamd.codeSomeShards(rows, inputs, nin, outs, nout, off, n - off)
    assert_same(outs, ref, '')
    assert rsamd.checkSomeShards(rows, inputs, nin, outs, nout, off, n - off)
    outs[-1][n - 1] ^= 1  # the last byte of the range
    assert not rsamd.checkSomeShards(rows, inputs, nin, outs, nout, off, n - off)


def test_direct_threads(gpu, oracle_lib):
    """Several threads each coding their own pinned shards at once."""
    import threading
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    oc = oracle_lib.Codec(4, 2)
    errors = []

    def work(seed):
        try:
            rng = np.random.default_rng(seed)
            n = (2 << 20) + int(rng.integers(1, 5000))
            big = _pinned_block(6 * (n + 16))
            sh = _shards(big, [i * (n + 16) for i in range(6)], n)
            for a in sh[:4]:
                a[:] = rng.integers(0, 256, n, dtype=np.uint8)
            for _ in range(3):
                ref = [a.copy() for a in sh]
                oc.encode_parity(ref, 0, n)
                rs.encodeParity(sh, 0, n)
                assert_same(sh, ref, '')
                sh[0][:] = rng.integers(0, 256, n, dtype=np.uint8)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=work, args=(s,)) for s in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


# ---------------------------------------------------------------------------
# The host file API's direct path (capi.cpp file_encode_direct /
# file_decode_direct, layout.hip file_direct_*_kernel): ReedSolomonEncoder's
# pad + split + encode and ReedSolomonDecoder's decode + merge + trim
# (ReedSolomonEncoder.java:56-85, ReedSolomonDecoder.java:36,62-103) on
# page-locked (or per-call locked) file and shard buffers.
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("k,m,n,file_off,pinned,misses", [
    (4, 2, 20_000_003, 0, True, [(), (0, 5), (1, 4), (2,), (4, 5)]),   # ragged file end (pad inside a unit)
    (4, 2, 16_000_000, 8, True, [(0, 1), (3,)]),                     # whole rows; 8-byte-aligned file start
    (4, 2, 9_999_999, 3, True, [(0, 5)]),                            # file start not 8-aligned: staged
    (10, 4, 30_000_001, 0, False, [(0, 3, 7, 12), (13,)]),           # pageable, locked per call
    (3, 5, 7_000_011, 0, True, [(0, 1, 2, 3, 4)]),                   # 5 parity shards (> 4 outputs): staged encode
])
def test_direct_file_paths(gpu, oracle_lib, k, m, n, file_off, pinned, misses):
    import rsamd
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    rs = rsamd.ReedSolomon.create(k, m)
    oc = oracle_lib.Codec(k, m)
    rng = np.random.default_rng(n)
    alloc = _pinned_block if pinned else (lambda nb: np.empty(nb, np.uint8))
    fbuf = alloc(n + 64)
    fbuf = fbuf[(-fbuf.ctypes.data) % 64 + file_off:][:n]
    fbuf[:] = rng.integers(0, 256, n, dtype=np.uint8)
    _, S = file_layout(rs, n)
    sh = [alloc(S) for _ in range(k + m)]
    for a in sh:
        a[:] = 0xEE  # every byte must be written
    file_encode_into(rs, fbuf, sh)
    ref = oc.file_encode(fbuf.tobytes())
    assert_same(sh, ref, '')
    for miss in misses:
        for j in miss:
            sh[j][:] = 0
        out = alloc(n + 64)[8:8 + n]
        out[:] = 0x33
        file_decode_into(rs, sh, [i not in miss for i in range(k + m)], S, out)
        assert_same([out], [fbuf], miss)
        assert_same(sh, ref, miss)  # absent shards rebuilt in place


@pytest.mark.parametrize("k,m,n,block,offs", [
    (4, 2, 12_000_007, 1000, (24, 16, 4088, 8, 0, 4000, 2000)),     # offsets of file, shard 0 .. 5
    (4, 2, 4_096_000, 1000, (0,) * 7),                               # whole pages: locked whole
    (10, 4, 30_000_001, 4096, (8, 40, 4056, 0, 8, 16, 24, 32, 48, 56, 64, 72, 80, 88, 96)),
    (4, 2, 3_000_000, 8, (16, 8, 0, 8, 16, 24, 32)),                # 512 rows per page
    (4, 2, 3_000_000, 1000, (3, 8, 0, 8, 16, 24, 32)),              # file not 8-aligned: staged
    (4, 2, 3_000_000, 999, (8, 8, 0, 8, 16, 24, 32)),               # block not a multiple of 8: staged
])
def test_direct_file_interior(gpu, oracle_lib, k, m, n, block, offs):
    """Pageable host file calls (ReedSolomonEncoder.java:56-85,
    ReedSolomonDecoder.java:36,62-103): the block rows inside whole pages of
    the file and of every shard are page-locked and coded in place, the rows
    either side staged (capi.cpp file_encode_interior / file_decode_interior).
    Shards and file exact against the oracle, and no byte around any array
    written."""
    import rsamd
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    rs = rsamd.ReedSolomon.create(k, m)
    oc = oracle_lib.Codec(k, m)
    rng = np.random.default_rng(n + block)
    _, S = file_layout(rs, n, block)
    guard = 8192

    def place(size, off):  # a view `off` bytes past a page inside a guarded pageable buffer
        raw = np.full(size + off + 2 * guard + 4096, 0xA5, np.uint8)
        start = (-raw.ctypes.data) % 4096 + guard + off
        return raw, raw[start:start + size]

    def guards_intact(raw, view):
        a = view.ctypes.data - raw.ctypes.data
        return bool((raw[:a] == 0xA5).all() and (raw[a + len(view):] == 0xA5).all())

    fraw, fbuf = place(n, offs[0])
    fbuf[:] = rng.integers(0, 256, n, dtype=np.uint8)
    shs = [place(S, o) for o in offs[1:]]
    sh = [v for _, v in shs]
    for a in sh:
        a[:] = 0xEE  # every byte must be written
    file_encode_into(rs, fbuf, sh, block)
    ref = oc.file_encode(fbuf.tobytes(), block)
    assert_same(sh, ref, '')
    assert all(guards_intact(r, v) for r, v in shs) and guards_intact(fraw, fbuf)
    miss = tuple(int(x) for x in rng.choice(k + m, m, replace=False))
    for j in miss:
        sh[j][:] = 0
    oraw, out = place(n, offs[0] + 8 if offs[0] % 8 == 0 else offs[0])
    out[:] = 0x33
    file_decode_into(rs, sh, [i not in miss for i in range(k + m)], S, out, block)
    assert_same([out], [fbuf], miss)
    assert_same(sh, ref, miss)  # absent shards rebuilt in place
    assert all(guards_intact(r, v) for r, v in shs) and guards_intact(oraw, out)


def test_direct_file_interior_threads(gpu, oracle_lib):
    """Four threads at once, each encoding and decoding its own file, with
    every file and shard a slice of ONE pageable buffer, packed back to back
    at 8-byte-aligned odd offsets so neighbouring slices share pages (the
    mirrored pipeline: each thread's chunks through its own slots); every
    result is exact."""
    import threading
    import rsamd
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    k, m, n, block = 4, 2, 3_000_104, 1000
    rs = rsamd.ReedSolomon.create(k, m)
    oc = oracle_lib.Codec(k, m)
    _, S = file_layout(rs, n, block)
    per = n + 2 * n + (k + m) * S + 8 * (k + m + 2)  # file, decoded file, shards (+ 8-byte gaps)
    big = np.empty(4 * per + 4096, np.uint8)
    rng = np.random.default_rng(11)
    jobs = []
    pos = (-big.ctypes.data) % 4096 + 24
    for t in range(4):
        f = big[pos:pos + n]; pos += n + 8
        out = big[pos:pos + n]; pos += n + 8
        sh = []
        for _ in range(k + m):
            sh.append(big[pos:pos + S]); pos += S + 8
        f[:] = rng.integers(0, 256, n, dtype=np.uint8)
        jobs.append((f, out, sh, (t % (k + m), (t + 3) % (k + m))))
    refs = [oc.file_encode(f.tobytes(), block) for f, _, _, _ in jobs]
    errors = []

    def work(j):
        f, out, sh, miss = jobs[j]
        try:
            for _ in range(3):
                file_encode_into(rs, f, sh, block)
                if not np.array_equal(np.stack(sh), refs[j]):
                    errors.append((j, "encode"))
                for s in miss:
                    sh[s][:] = 0
                out[:] = 0
                file_decode_into(rs, sh, [i not in miss for i in range(k + m)], S, out, block)
                if not np.array_equal(out, f) or not np.array_equal(np.stack(sh), refs[j]):
                    errors.append((j, "decode", miss))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((j, repr(e)))

    ts = [threading.Thread(target=work, args=(j,)) for j in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


@pytest.mark.parametrize("n,off", [((64 << 10) + 4100, 3), ((256 << 10) + 8200, 3), ((1 << 20) + 7, 4095),
                                   ((1 << 20) + 8200, 3), (5 << 20, 0)])
def test_direct_interior_and_ends(gpu, oracle_lib, n, off):
    """Pageable calls at ragged offsets and lengths (the mirrored pipeline's
    ramped chunks from 1 MiB per shard, or the zero-copy pass below).  Encode,
    decode and verify must be exact at both ends and inside, and a wrong
    parity byte is found wherever it is."""
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    rng = np.random.default_rng(n + off)
    cnt = n - off - 1
    sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(4)] + [np.zeros(n, np.uint8) for _ in range(2)]
    ref = [a.copy() for a in sh]
    oracle_lib.Codec(4, 2).encode_parity(ref, off, cnt)
    rs.encodeParity(sh, off, cnt)
    assert_same(sh, ref, '')
    assert rs.isParityCorrect(sh, off, cnt)
    for where in (off, off + cnt - 1, off + cnt // 2, off + 4095 if cnt > 8192 else off + 1):
        sh[5][where] ^= 0x5A
        assert not rs.isParityCorrect(sh, off, cnt), where
        sh[5][where] ^= 0x5A
    for miss in ((0, 5), (1, 2)):
        for j in miss:
            sh[j][off:off + cnt] = 0x33
        rs.decodeMissing(sh, [i not in miss for i in range(6)], off, cnt)
        assert_same(sh, ref, miss)


def test_host_buffer_shards_and_file(gpu, oracle_lib):
    """Shards and a file kept in rs_host_alloc memory (rsamd.device.HostBuffer,
    the pinned buffers NativeReedSolomon.allocatePinned hands a JVM): encode,
    decode {0, 5} and the file calls in place, against the oracle."""
    import rsamd
    from rsamd.device import HostBuffer
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    k, m, n = 4, 2, (8 << 20) + 40
    rs = rsamd.ReedSolomon.create(k, m)
    bufs = [HostBuffer(n) for _ in range(k + m)]
    sh = [b.array for b in bufs]
    rng = np.random.default_rng(77)
    for a in sh:
        a[:] = rng.integers(0, 256, n, dtype=np.uint8)
    ref = [a.copy() for a in sh]
    oracle_lib.Codec(k, m).encode_parity(ref, 0, n)
    rs.encodeParity(sh, 0, n)
    assert_same(sh, ref, "encode")
    for j in (0, 5):
        sh[j][:] = 0
    rs.decodeMissing(sh, [i not in (0, 5) for i in range(k + m)], 0, n)
    assert_same(sh, ref, "decode {0,5}")
    flen = 3 * (4 << 20) + 999
    fbuf = HostBuffer(flen)
    fbuf.array[:] = rng.integers(0, 256, flen, dtype=np.uint8)
    _, S = file_layout(rs, flen)
    fsh = [HostBuffer(S) for _ in range(k + m)]
    file_encode_into(rs, fbuf.array, [b.array for b in fsh])
    want = oracle_lib.Codec(k, m).file_encode(fbuf.array.tobytes(), 1000)
    assert_same([b.array for b in fsh], list(want), "file encode")
    out = HostBuffer(flen)
    for j in (0, 5):
        fsh[j].array[:] = 0
    file_decode_into(rs, [b.array for b in fsh], [i not in (0, 5) for i in range(k + m)], S, out.array)
    assert np.array_equal(out.array, fbuf.array)
    for b in bufs + fsh + [fbuf, out]:
        b.free()


def test_host_buffer_view_keeps_its_owner(gpu, oracle_lib):
    """HostBuffer(n).array with the HostBuffer itself dropped: the view keeps
    the pinned allocation alive (its base holds the owner), and the host
    calls still code it in place."""
    import gc
    import rsamd
    from rsamd.device import HostBuffer
    k, m, n = 4, 2, 1 << 20
    views = [HostBuffer(n).array for _ in range(k + m)]
    gc.collect()
    rng = np.random.default_rng(31)
    for v in views[:k]:
        v[:] = rng.integers(0, 256, n, dtype=np.uint8)
    ref = [v.copy() for v in views[:k]] + [np.zeros(n, np.uint8) for _ in range(m)]
    oracle_lib.Codec(k, m).encode_parity(ref, 0, n)
    rsamd.ReedSolomon.create(k, m).encodeParity(views, 0, n)
    assert all(np.array_equal(v, r) for v, r in zip(views, ref))
    half = views[0][n // 2:]  # a slice keeps the owner alive too
    del views
    gc.collect()
    assert np.array_equal(half, ref[0][n // 2:])


def test_host_free_takes_only_live_allocations(gpu):
    """rs_host_free: a foreign pointer, an interior one (a slice) and a second
    free are RS_E_INVALID and free nothing; the allocation itself frees once."""
    import ctypes as C
    from rsamd import _lib
    from rsamd.codec import RS_E_INVALID
    lib = _lib.load()
    p = C.c_void_p()
    assert lib.rs_host_alloc(C.byref(p), 1 << 16) == 0
    foreign = np.zeros(4096, np.uint8)
    assert lib.rs_host_free(C.c_void_p(foreign.ctypes.data)) == RS_E_INVALID
    assert "not a live rs_host_alloc buffer" in _lib.last_error()
    assert lib.rs_host_free(C.c_void_p(p.value + 4096)) == RS_E_INVALID
    C.memset(p, 0x5A, 1 << 16)  # still allocated and mapped
    assert lib.rs_host_free(p) == 0
    assert lib.rs_host_free(p) == RS_E_INVALID
    assert lib.rs_host_free(None) == 0
