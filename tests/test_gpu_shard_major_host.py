"""The master's recovery loop on HOST arrays (rs_decode_groups_shard_major;
MasterImpl.java:733-743, 794-839 with ChunkserverDiskRecoveryMachine.java:34-48
per group) against the oracle, bit-exact, through the C-ABI.

The master holds each server's chunks of the groups it read back to back in
one array (`servers[s]`, chunk g at g * chunk_len).  Its offline set is the same
for every group and grows when a read fails mid-loop, so the groups form runs
of one presence pattern, each coded as ONE decodeMissing of run-long shards
(pageable arrays: the small-call pass below 1 MiB per shard, the mirrored
pipeline above; rs_host_alloc arrays: the direct kernels in place).  Flags that
change every few groups go to the per-stripe pattern kernels in chunks of
groups.  Every byte of every array -- the pads past n_groups * chunk_len and
the present chunks included -- must come back as the oracle encoded it, and a
call that fails its checks must leave every array untouched.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CODES = [(4, 2), (10, 4), (3, 3), (6, 1)]
CHUNKS = [1000, 1024, 8, 13, 4096, 999, 1000, 2000]
PADS = [0, 8, 256, 4096, 1, 0, 24, 4097]


def _servers(rng, oracle_lib, k, m, N, chunk, pad):
    """The encoded arrays (T arrays of N*chunk bytes + pad random sentinels)."""
    T, L = k + m, N * chunk
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(T)]
    oracle_lib.Codec(k, m).encode_parity(rows, 0, L)  # parity of every group at once (per column)
    return [np.concatenate([r, rng.integers(0, 256, pad, dtype=np.uint8)]) for r in rows]


def _erase(want, present, runs, chunk):
    """Copies of `want` with the runs' offline chunks overwritten; flags set."""
    got = [w.copy() for w in want]
    for g0, g1, miss in runs:
        for s in miss:
            present[g0:g1, s] = False
            got[s][g0 * chunk: g1 * chunk] = 0x3C
    return got


def _check(got, want, what):
    for s, (g, w) in enumerate(zip(got, want)):
        if not np.array_equal(g, w):
            i = int(np.flatnonzero(g != w)[0])
            raise AssertionError(f"{what}: first wrong byte server {s} offset {i}")


def _pinned_copies(arrs):
    from rsamd.device import HostBuffer
    held = [HostBuffer(max(1, len(a))) for a in arrs]
    out = []
    for h, a in zip(held, arrs):
        v = h.array[: len(a)]
        v[:] = a
        out.append(v)
    return held, out


@pytest.mark.parametrize("case", range(24))
def test_host_shard_major_random(gpu, oracle_lib, case):
    """Seeded: codes 4+2 / 10+4 / 3+3 / 6+1, chunks that are and are not
    multiples of 8 or 16, pads of 0 to 4 KiB + 1 past each server's groups,
    one to five runs with their own offline sets (empty and shrinking ones
    too), random bytes in every chunk (survivors: the first k present,
    ReedSolomon.java:210-222).  Every third case on rs_host_alloc arrays."""
    from rsamd.recovery import recover_groups_shard_major
    rng = np.random.default_rng(9100 + case)
    k, m = CODES[case % len(CODES)]
    T = k + m
    chunk = CHUNKS[case % len(CHUNKS)]
    pad = PADS[(case // 2) % len(PADS)]
    N = int(rng.integers(1, 3001)) if case % 4 else int(rng.integers(1100, 2600))  # some runs >= 1 MiB
    want = _servers(rng, oracle_lib, k, m, N, chunk, pad)
    cuts = sorted(set(int(x) for x in rng.integers(1, N, int(rng.integers(0, 5))))) if N > 1 else []
    bounds = [0] + cuts + [N]
    runs = []
    for g0, g1 in zip(bounds[:-1], bounds[1:]):
        e = int(rng.integers(0, m + 1))
        runs.append((g0, g1, [int(x) for x in rng.choice(T, e, replace=False)] if e else []))
    present = np.ones((N, T), bool)
    got = _erase(want, present, runs, chunk)
    held = None
    if case % 3 == 2:
        held, got = _pinned_copies(got)
    recover_groups_shard_major(got, present, chunk, data_shards=k, parity_shards=m)
    _check(got, want, f"k={k} m={m} chunk={chunk} pad={pad} N={N} runs={bounds} pinned={held is not None}")
    for h in held or []:
        h.free()


@pytest.mark.parametrize("pinned", [False, True])
def test_host_shard_major_like_the_master(gpu, oracle_lib, pinned):
    """4+2, 1000-byte chunks, 2 MB per server: offline {0} and {0,5} for every
    group (one run: the mirrored pipeline / the direct kernels), a set that
    grows at an odd group (the second run starts 8 bytes off a 16-byte
    boundary), a failure after a clean run, and a growth late enough that the
    second run is a small call."""
    from rsamd.recovery import recover_groups_shard_major
    k, m, chunk, N = 4, 2, 1000, 2049
    rng = np.random.default_rng(31 + pinned)
    want = _servers(rng, oracle_lib, k, m, N, chunk, 64)
    cases = {
        "offline_0": [(0, N, (0,))],
        "offline_0_5": [(0, N, (0, 5))],
        "grows_mid_loop": [(0, 1001, (0,)), (1001, N, (0, 3))],
        "fails_after_clean_run": [(0, 1001, ()), (1001, N, (2,))],
        "grows_late": [(0, 2000, (1,)), (2000, N, (1, 4))],
    }
    for name, runs in cases.items():
        present = np.ones((N, k + m), bool)
        got = _erase(want, present, runs, chunk)
        held = None
        if pinned:
            held, got = _pinned_copies(got)
        recover_groups_shard_major(got, present, chunk)
        _check(got, want, name)
        for h in held or []:
            h.free()


@pytest.mark.parametrize("chunk,pad,k,m", [(1000, 0, 4, 2), (13, 8, 4, 2), (4096, 256, 4, 2), (1000, 16, 10, 4),
                                           (1000, 0, 20, 4)])
def test_host_shard_major_many_runs(gpu, oracle_lib, chunk, pad, k, m):
    """Flags that change every one to three groups (not the master's loop;
    more runs than the call codes one by one): chunks of groups through the
    per-stripe pattern kernels -- or, for a code too wide for the pattern
    table (20+4), run by run -- with the same results."""
    from rsamd.recovery import recover_groups_shard_major
    rng = np.random.default_rng(chunk + pad + k)
    T = k + m
    N = 3001 if T <= 20 else 200
    want = _servers(rng, oracle_lib, k, m, N, chunk, pad)
    present = np.ones((N, T), bool)
    runs, g = [], 0
    while g < N:
        n = int(rng.integers(1, 4))
        e = int(rng.integers(0, m + 1))
        runs.append((g, min(N, g + n), [int(x) for x in rng.choice(T, e, replace=False)] if e else []))
        g += n
    got = _erase(want, present, runs, chunk)
    recover_groups_shard_major(got, present, chunk, data_shards=k, parity_shards=m)
    _check(got, want, f"{k}+{m} chunk={chunk} pad={pad}")


def test_host_shard_major_checks_touch_nothing(gpu):
    """The argument checks, in order, before anything is written: wrong
    server count, a short server, a group with fewer than k present (late in
    the batch, after runs that would decode) -> IllegalArgumentException."""
    import ctypes as C
    import rsamd
    from rsamd import _lib
    from rsamd.codec import IllegalArgumentException, RS_E_INVALID, RS_E_NOT_ENOUGH, RS_E_WRONG_NSHARDS
    from rsamd.recovery import recover_groups_shard_major
    N, T, chunk = 3000, 6, 1000
    rng = np.random.default_rng(5)
    servers = [rng.integers(0, 256, N * chunk, dtype=np.uint8) for _ in range(T)]
    before = [s.copy() for s in servers]
    present = np.ones((N, T), bool)
    present[:1500, 1] = False
    present[2999, :3] = False  # undecodable
    with pytest.raises(IllegalArgumentException) as e:
        recover_groups_shard_major(servers, present, chunk)
    assert e.value.code == RS_E_NOT_ENOUGH and "Not enough shards present" in str(e.value)
    _check(servers, before, "not enough")
    present[2999, :3] = True
    short = servers[:5] + [servers[5][: N * chunk - 1]]
    with pytest.raises(IllegalArgumentException) as e:
        recover_groups_shard_major(short, present, chunk)
    assert e.value.code == RS_E_INVALID
    _check(servers, before, "short server")
    rs = rsamd.ReedSolomon.create(4, 2)
    ptrs = (_lib.u8p * 5)(*[s.ctypes.data_as(_lib.u8p) for s in servers[:5]])
    lens = (C.c_int64 * 5)(*[len(s) for s in servers[:5]])
    rc = _lib.load().rs_decode_groups_shard_major(rs.handle, ptrs, 5, lens, chunk, N,
                                                  present.view(np.uint8).ctypes.data_as(_lib.u8p))
    assert rc == RS_E_WRONG_NSHARDS and _lib.last_error() == "wrong number of shards: 5"
    _check(servers, before, "wrong count")


def test_host_shard_major_any_nonzero_flag(gpu, oracle_lib):
    """A flag is present when nonzero (the Java boolean[]): random nonzero
    bytes in every present flag still form two runs."""
    import ctypes as C
    import rsamd
    from rsamd import _lib
    k, m, chunk, N = 4, 2, 1000, 1026
    rng = np.random.default_rng(19)
    want = _servers(rng, oracle_lib, k, m, N, chunk, 0)
    flags = rng.integers(1, 256, (N, k + m), dtype=np.uint8)
    flags[:500, 0] = 0
    flags[500:, 2] = 0
    flags[500:, 5] = 0
    got = [w.copy() for w in want]
    got[0][: 500 * chunk] = 0x3C
    for s in (2, 5):
        got[s][500 * chunk:] = 0x3C
    rs = rsamd.ReedSolomon.create(k, m)
    ptrs = (_lib.u8p * 6)(*[g.ctypes.data_as(_lib.u8p) for g in got])
    lens = (C.c_int64 * 6)(*[len(g) for g in got])
    rc = _lib.load().rs_decode_groups_shard_major(rs.handle, ptrs, 6, lens, chunk, N, flags.ctypes.data_as(_lib.u8p))
    assert rc == 0, _lib.last_error()
    _check(got, want, "nonzero flags")
