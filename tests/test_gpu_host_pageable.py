"""GPU tests of the host calls on pageable caller memory (JVM heap arrays
through JNI), which go through the mirrored pipeline (host.hpp run_mirrored:
chunks copied into the thread's device-mapped pinned slots, coded there by the
direct kernels, copied back).  Sharing must never change a byte: threads
passing the same input arrays, shards that are slices of one allocation
(shared pages), and the same array passed twice.
"""
import threading

import numpy as np
import pytest
from bytes_report import assert_same

pytestmark = pytest.mark.gpu

N = (12 << 20) + 3  # several pipeline chunks per call, ragged end


def test_threads_share_input_arrays(gpu, oracle_lib):
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    rng = np.random.default_rng(31)
    data = [rng.integers(0, 256, N, dtype=np.uint8) for _ in range(4)]
    ref = [d.copy() for d in data] + [np.zeros(N, np.uint8) for _ in range(2)]
    oracle_lib.Codec(4, 2).encode_parity(ref, 0, N)
    errors = []

    def work(seed):
        try:
            for _ in range(3):
                par = [np.full(N, seed, np.uint8) for _ in range(2)]
                rs.encodeParity(data + par, 0, N)  # the same data arrays in every thread
                assert np.array_equal(par[0], ref[4]) and np.array_equal(par[1], ref[5])
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=work, args=(s,)) for s in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def test_shards_are_slices_of_one_allocation(gpu, oracle_lib):
    """Six shards back to back in one array (neighbouring shards share pages)."""
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    big = np.zeros(6 * N, np.uint8)
    big[: 4 * N] = np.random.default_rng(32).integers(0, 256, 4 * N, dtype=np.uint8)
    sh = [big[i * N:(i + 1) * N] for i in range(6)]
    ref = [s.copy() for s in sh]
    oracle_lib.Codec(4, 2).encode_parity(ref, 0, N)
    rs.encodeParity(sh, 0, N)
    assert_same(sh, ref, '')
    sh[1][:] = 0
    sh[4][:] = 0
    rs.decodeMissing(sh, [True, False, True, True, False, True], 0, N)
    assert_same(sh, ref, '')
    assert rs.isParityCorrect(sh, 0, N)


def test_same_array_twice_as_input(gpu, oracle_lib):
    """CodingLoop-level call with one input array passed twice (two slots of
    the mirror hold the same bytes)."""
    import rsamd
    rng = np.random.default_rng(33)
    a = rng.integers(0, 256, N, dtype=np.uint8)
    b = rng.integers(0, 256, N, dtype=np.uint8)
    rows = np.array([[3, 7, 11]], dtype=np.uint8)
    out = [np.zeros(N, np.uint8)]
    ref = [np.zeros(N, np.uint8)]
    oracle_lib.code_some_shards(7, rows, [a, b, a], ref, 0, N)
    rsamd.codeSomeShards(rows, [a, b, a], 3, out, 1, 0, N)
    assert_same([out[0]], [ref[0]], '')


def test_threads_check_the_same_shards(gpu, oracle_lib):
    """Several threads run isParityCorrect on the SAME pageable shards (every
    slot an input; each thread has its own mirror slots and stream), then
    decodes of the same shards into per-thread copies of the absent ones."""
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    rng = np.random.default_rng(33)
    sh = [rng.integers(0, 256, N, dtype=np.uint8) for _ in range(4)] + [np.zeros(N, np.uint8) for _ in range(2)]
    oracle_lib.Codec(4, 2).encode_parity(sh, 0, N)
    errors = []

    def work(seed):
        try:
            for _ in range(4):
                assert rs.isParityCorrect(sh, 0, N)
                mine = list(sh)
                mine[seed % 4] = np.zeros(N, np.uint8)
                present = [i != seed % 4 for i in range(6)]
                rs.decodeMissing(mine, present, 0, N)
                assert np.array_equal(mine[seed % 4], sh[seed % 4])
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=work, args=(s,)) for s in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def test_many_threads_borrow_slot_sets(gpu, oracle_lib):
    """Eight threads at once, each encoding then decoding its own pageable
    shards of a different size: more concurrent calls than the pool keeps idle
    slot sets (host.cpp MirrorPool), every result exact, and again once the
    pool has trimmed back."""
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    errors = []

    def work(t):
        try:
            n = (1 << 20) * (t + 1) + 13 * t
            rng = np.random.default_rng(100 + t)
            sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(4)] + [np.zeros(n, np.uint8) for _ in range(2)]
            ref = [a.copy() for a in sh]
            oracle_lib.Codec(4, 2).encode_parity(ref, 0, n)
            rs.encodeParity(sh, 0, n)
            assert_same(sh, ref, f"thread {t} encode")
            sh[t % 6][:] = 0
            rs.decodeMissing(sh, [i != t % 6 for i in range(6)], 0, n)
            assert_same(sh, ref, f"thread {t} decode")
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    for _ in range(2):
        ts = [threading.Thread(target=work, args=(t,)) for t in range(8)]
        for th in ts:
            th.start()
        for th in ts:
            th.join()
        assert not errors, errors
