"""GPU parity of the 8-byte-vector kernels (gf_vec8_kernel, gf_masked8_kernel):
stripe batches whose base and strides are multiples of 8 but not of 16, the
DFS's 1000-byte chunk groups packed back to back (ChunkserverDiskRecoveryMachine
.java:34-48; the 6 x 1000-B groups of MasterImpl.java:794-839).  Encode
(ReedSolomon.java:90-104), uniform decode (ReedSolomon.java:175-272, the
reference test's {0,5}: ReedSolomonTest.java:77-93) and verify
(ReedSolomon.java:115-164) through the C-ABI, bit-exact against the oracle.
Shapes: 1000/1000 (125 vectors, two vectors per lane leave 3 lanes idle),
1004/1016 (a 4-byte tail on the byte kernel), 10+4 and 3+3 (the runtime-k
build), and 8-aligned stripe strides with 16-aligned shard strides."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _encoded(oracle_lib, k, m, S, B, seed):
    rng = np.random.default_rng(seed)
    batch = np.zeros((B, k + m, S), np.uint8)
    batch[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    c = oracle_lib.Codec(k, m)
    for t in range(B):
        c.encode_parity([batch[t, i] for i in range(k + m)], 0, S)
    return batch


def _to_dev(torch, batch, shard_stride, stripe_stride):
    B, T, S = batch.shape
    host = np.zeros(B * stripe_stride, np.uint8)
    v = np.lib.stride_tricks.as_strided(host, (B, T, S), (stripe_stride, shard_stride, 1))
    v[...] = batch
    return torch.from_numpy(host).to("cuda:0")


def _from_dev(dev, B, T, S, shard_stride, stripe_stride):
    host = dev.cpu().numpy()
    return np.lib.stride_tricks.as_strided(host, (B, T, S), (stripe_stride, shard_stride, 1)).copy()


@pytest.mark.parametrize("k,m,S,shard_stride,stripe_pad", [(4, 2, 1000, 1000, 0), (4, 2, 1004, 1016, 0),
                                                           (10, 4, 1000, 1000, 0), (3, 3, 2040, 2040, 0),
                                                           (4, 2, 4096, 4096, 8), (4, 2, 1000, 1000, 8)])
def test_vec8_encode_decode_verify(gpu, oracle_lib, k, m, S, shard_stride, stripe_pad):
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    T, B = k + m, 700
    stripe_stride = T * shard_stride + stripe_pad
    want = _encoded(oracle_lib, k, m, S, B, S + k)
    lay = StripeLayout(B, S, shard_stride, stripe_stride)
    rs = rsamd.ReedSolomon.create(k, m)
    st = torch.cuda.current_stream()
    # encode over garbage parity
    clob = want.copy()
    clob[:, k:] = 0xA5
    dev = _to_dev(torch, clob, shard_stride, stripe_stride)
    device.encode(rs, dev.data_ptr(), lay, st)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_from_dev(dev, B, T, S, shard_stride, stripe_stride), want)
    # verify: clean, then one flipped byte in the last stripe's last parity byte
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.verify(rs, dev.data_ptr(), lay, flag.data_ptr(), st)
    assert int(flag.item()) == 0
    bad = want.copy()
    bad[-1, -1, -1] ^= 1
    dev_bad = _to_dev(torch, bad, shard_stride, stripe_stride)
    device.verify(rs, dev_bad.data_ptr(), lay, flag.data_ptr(), st)
    assert int(flag.item()) == 1
    # uniform decode of {0, T-1} (4+2: the reference test's {0,5}) and of {1}
    for miss in [(0, T - 1), (1,)]:
        clob = want.copy()
        clob[:, list(miss)] = 0x3C
        dev = _to_dev(torch, clob, shard_stride, stripe_stride)
        device.decode(rs, dev.data_ptr(), [i not in miss for i in range(T)], lay, st)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_from_dev(dev, B, T, S, shard_stride, stripe_stride), want)


@pytest.mark.parametrize("offset", [136, 64])
def test_line_owner_kernel_edges(gpu, oracle_lib, offset):
    """The line-owner kernel (gf_group8_kernel: 4+2 x 1000-B groups packed
    back to back, outputs one run of consecutive shards) writes whole 128-byte
    lines, rewriting the input bytes that share a line with an output with
    their own values -- but never a byte outside the batch.  The batch sits
    inside a guarded buffer (base 8- but not 16-aligned, or 64-aligned); every
    run of consecutive shards is erased and rebuilt (encode: 4-5; decodes:
    {0}, {0,1}, {1,2}, {2,3}, {3,4}, {5}, and {0,5}, where every group boundary
    line is rebuilt by both groups and the earlier one writes it whole) and
    every other byte, guards included, must be unchanged."""
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    k, m, S, B = 4, 2, 1000, 701
    T = k + m
    want = _encoded(oracle_lib, k, m, S, B, 11)
    guard = 512
    host = np.full(guard + offset + B * T * S + guard, 0x77, np.uint8)
    host[guard + offset: guard + offset + B * T * S] = want.reshape(-1)
    lay = StripeLayout(B, S, S, T * S)
    rs = rsamd.ReedSolomon.create(k, m)
    st = torch.cuda.current_stream()
    for miss in [(4, 5), (0,), (0, 1), (1, 2), (2, 3), (3, 4), (5,), (0, 5)]:
        clob = host.copy()
        v = clob[guard + offset: guard + offset + B * T * S].reshape(B, T, S)
        v[:, list(miss)] = 0x3C
        dev = torch.from_numpy(clob).to("cuda:0")
        base = dev.data_ptr() + guard + offset
        if miss == (4, 5):
            device.encode(rs, base, lay, st)
        else:
            device.decode(rs, base, [i not in miss for i in range(T)], lay, st)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dev.cpu().numpy(), host, err_msg=f"erased {miss}")


@pytest.mark.parametrize("offset", [136, 64])
def test_line_owner_kernel_per_group_patterns(gpu, oracle_lib, offset):
    """The line-owner kernel with a presence pattern per group (the master's
    recovery, MasterImpl.java:794-839): random patterns of <= 2 erasures, plus
    undecodable and complete groups, and runs that meet across a group
    boundary ({5} in one group, {0} in the next).  A group rewrites a
    neighbour's bytes only where that neighbour rebuilds nothing there; every
    byte outside the rebuilt shards, guards included, must be unchanged."""
    import itertools
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    k, m, S, B = 4, 2, 1000, 603
    T = k + m
    want = _encoded(oracle_lib, k, m, S, B, 13)
    guard = 512
    host = np.full(guard + offset + B * T * S + guard, 0x77, np.uint8)
    host[guard + offset: guard + offset + B * T * S] = want.reshape(-1)
    allp = [[i not in mi for i in range(T)] for e in range(3) for mi in itertools.combinations(range(T), e)]
    rng = np.random.default_rng(offset)
    pres = np.array([allp[i] for i in rng.integers(0, len(allp), B)], dtype=bool)
    pres[0] = [False] + [True] * (T - 1)            # the batch's first byte is rebuilt
    pres[-1] = [True] * (T - 1) + [False]           # ... and its last
    pres[10] = [True] * (T - 1) + [False]           # {5} next to {0}: both groups write one line
    pres[11] = [False] + [True] * (T - 1)
    pres[30:40] = [False] + [True] * (T - 2) + [False]  # a run of {0,5} groups
    pres[50] = [False] + [True] * (T - 2) + [False]     # {0,5} between an undecodable group ...
    pres[51] = [False, False, False, True, True, True]
    pres[49] = [True] * (T - 1) + [False]               # ... and a {5}
    pres[60] = [True] * (T - 2) + [False, False]        # {4,5} before a singular-free {0,1}
    pres[61] = [False, False] + [True] * (T - 2)
    pres[20] = [False, False, False, True, True, True]  # undecodable: untouched, counted
    n_bad = 2
    words = pres.astype(np.uint32) @ (1 << np.arange(T, dtype=np.uint32))
    clob = host.copy()
    v = clob[guard + offset: guard + offset + B * T * S].reshape(B, T, S)
    v[~pres] = 0x3C
    expect = host.copy()
    expect[guard + offset: guard + offset + B * T * S].reshape(B, T, S)[20] = v[20]
    expect[guard + offset: guard + offset + B * T * S].reshape(B, T, S)[51] = v[51]
    dev = torch.from_numpy(clob).to("cuda:0")
    base = dev.data_ptr() + guard + offset
    bits = torch.from_numpy(words.view(np.int32)).to("cuda:0")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    rs = rsamd.ReedSolomon.create(k, m)
    device.decode_masked_bits(rs, base, bits.data_ptr(), StripeLayout(B, S, S, T * S), bad.data_ptr(),
                              torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert int(bad.item()) == n_bad
    np.testing.assert_array_equal(dev.cpu().numpy(), expect)
    # the same patterns as host flags (rs_decode_batch_masked_dev), stripes 20 and 51 made decodable
    for t in (20, 51):
        pres[t] = True
        pres[t, [0, 1]] = False
        v[t] = want[t]
        v[t, [0, 1]] = 0x3C
    dev = torch.from_numpy(clob).to("cuda:0")
    device.decode_masked(rs, dev.data_ptr() + guard + offset, pres, StripeLayout(B, S, S, T * S),
                         torch.cuda.current_stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy(), host)
