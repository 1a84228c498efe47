"""GPU tests of the split small-call pass (capi.cpp run_small): pageable
coding calls from 128 KiB to just under 1 MiB per shard run as two signalled
launches over two page-aligned column ranges of the zero-copy buffer.  The
cut, the page-aligned slot stride and the zeroed 16-byte tail must never
change a byte: ragged sizes either side of the threshold, offsets into larger
arrays, several codes, decodes of every kind of absent set, and threads
alternating split and one-launch calls (each thread's signal sequence)."""
import threading

import numpy as np
import pytest
from bytes_report import assert_same

pytestmark = pytest.mark.gpu

SIZES = [(128 << 10) - 16, 128 << 10, (128 << 10) + 5, 200_003, 262_151, 777_777, (1 << 20) - 1]
CODES = [(4, 2), (10, 4), (6, 3), (3, 1)]


@pytest.mark.parametrize("k,m", CODES)
@pytest.mark.parametrize("S", SIZES)
def test_split_encode_decode(gpu, oracle_lib, k, m, S):
    import rsamd
    rng = np.random.default_rng(S * 31 + k * 7 + m)
    off = int(rng.integers(0, 5000))
    n = S + off + int(rng.integers(0, 300))
    sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k + m)]
    ref = [a.copy() for a in sh]
    rs = rsamd.ReedSolomon.create(k, m)
    oc = oracle_lib.Codec(k, m)
    rs.encodeParity(sh, off, S)
    oc.encode_parity(ref, off, S)
    assert_same(sh, ref, f"encode k={k} m={m} S={S} off={off}")
    assert rs.isParityCorrect(sh, off, S)
    for absent in ({0}, {k + m - 1}, set(range(m)), set(range(k, k + m)) if m else set()):
        present = [i not in absent for i in range(k + m)]
        got = [a.copy() for a in sh]
        for i in absent:
            got[i][off:off + S] = rng.integers(0, 256, S, dtype=np.uint8)
        rs.decodeMissing(got, present, off, S)
        assert_same(got, sh, f"decode {sorted(absent)} k={k} m={m} S={S} off={off}")


def test_split_calls_alternate_with_small_ones_in_threads(gpu, oracle_lib):
    """Four threads, each alternating split calls and one-launch calls (1000 B,
    64 KiB) on its own shards: every call waits on its own signal numbers."""
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    oc = oracle_lib.Codec(4, 2)
    errors = []

    def work(t):
        try:
            rng = np.random.default_rng(700 + t)
            for it in range(6):
                S = [1000, 300_001 + t, 65536, 524_288 + 17 * t][it % 4]
                sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(6)]
                ref = [a.copy() for a in sh]
                oc.encode_parity(ref, 0, S)
                rs.encodeParity(sh, 0, S)
                assert_same(sh, ref, f"thread {t} encode S={S}")
                sh[t % 6][:] = 0
                rs.decodeMissing(sh, [i != t % 6 for i in range(6)], 0, S)
                assert_same(sh, ref, f"thread {t} decode S={S}")
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for th in ts:
        th.start()
    for th in ts:
        th.join()
    assert not errors, errors


def test_split_code_some_shards(gpu, oracle_lib):
    """The CodingLoop-level call on a split size, one input passed twice."""
    import rsamd
    rng = np.random.default_rng(41)
    S = 333_333
    a = rng.integers(0, 256, S, dtype=np.uint8)
    b = rng.integers(0, 256, S, dtype=np.uint8)
    rows = np.array([[3, 7, 11], [1, 2, 250]], dtype=np.uint8)
    out = [np.zeros(S, np.uint8), np.full(S, 9, np.uint8)]
    ref = [np.zeros(S, np.uint8), np.zeros(S, np.uint8)]
    oracle_lib.code_some_shards(7, rows, [a, b, a], ref, 0, S)
    rsamd.codeSomeShards(rows, [a, b, a], 3, out, 2, 0, S)
    assert_same(out, ref, '')


FILES = [(4, 2, 1000, 524_288), (4, 2, 1000, 1_000_003), (4, 2, 1000, 3_999_999), (6, 3, 4096, 2_000_000),
         (10, 4, 1000, 1_400_000), (3, 1, 8, 600_001), (4, 2, 520, 700_000), (2, 2, 1000, 262_000),
         (2, 2, 1000, 263_001), (5, 3, 999, 900_000), (1, 1, 1000, 131_072)]


@pytest.mark.parametrize("k,m,block,F", FILES)
def test_split_file_encode(gpu, oracle_lib, k, m, block, F):
    """The client's file encode on pageable memory at sizes whose shards reach
    128 KiB (capi.cpp file_encode_zc_halves: two launches over two halves of
    the block rows), then file decodes (capi.cpp file_decode_zc_split, halves from 128 KiB)
    of {0}, of the m parity shards and of a data and a parity shard."""
    import rsamd
    from rsamd.layout import file_decode_into, file_encode_into, file_layout
    rng = np.random.default_rng(F + 97 * k + m)
    data = rng.integers(0, 256, F, dtype=np.uint8)
    rs = rsamd.ReedSolomon.create(k, m)
    _, S = file_layout(rs, F, block)
    sh = [np.full(S, 0xA5, np.uint8) for _ in range(k + m)]
    file_encode_into(rs, data, sh, block)
    ref = oracle_lib.Codec(k, m).file_encode(data.tobytes(), block)
    assert_same([np.stack(sh)], [ref], (k, m, block, F))
    for absent in ({0}, set(range(k, k + m)), {k - 1, k + m - 1} if m >= 2 else {k - 1}):
        pres = [i not in absent for i in range(k + m)]
        got = [a.copy() for a in sh]
        for i in absent:
            got[i][:] = 0x3C
        out = np.zeros(F, np.uint8)
        file_decode_into(rs, got, pres, S, out, block)
        assert np.array_equal(out, data), (k, m, block, F, sorted(absent))


@pytest.mark.parametrize("S", [128 << 10, 200_003, 777_777, (1 << 20) - 1])
def test_split_verify(gpu, oracle_lib, S):
    """isParityCorrect split in two launches (only the last one signals): a
    wrong byte in either half, at either side of the cut or at the very end,
    is found; a correct call after a failed one reads true (the mismatch word
    the first launch leaves set is reported and zeroed by the last)."""
    import rsamd
    rng = np.random.default_rng(S + 5)
    k, m = 4, 2
    sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
    oracle_lib.Codec(k, m).encode_parity(sh, 0, S)
    rs = rsamd.ReedSolomon.create(k, m)
    assert rs.isParityCorrect(sh, 0, S)
    n16 = (S + 15) // 16 * 16
    cut = min(n16, (n16 // 2 + 4095) // 4096 * 4096)
    for pos in sorted({0, cut - 1, cut, S - 1, S // 3}):
        for shard in (1, k, k + m - 1):
            sh[shard][pos] ^= 0x41
            assert not rs.isParityCorrect(sh, 0, S), (pos, shard)
            sh[shard][pos] ^= 0x41
            assert rs.isParityCorrect(sh, 0, S), (pos, shard)
