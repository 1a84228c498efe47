"""GPU parity of the run-time compiled XOR-network kernels (csrc/xornet.cpp).

rs_debug_xornet(2) routes every launch with >= 2 KiB of columns through the
bitsliced kernel generated for its matrix (compiled by hiprtc on first use);
the columns past the last whole 2 KiB chunk go to the table kernels.  Each
case is checked against the oracle (encode: InputOutputByteTableCodingLoop.java
:12-44; decode: ReedSolomon.java:175-272) byte for byte, and the compiled-kernel
count proves the generated kernels ran.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED


@pytest.fixture
def xornet_forced(native):
    before = native.rs_debug_xornet(2)
    yield native
    native.rs_debug_xornet(-1)
    assert native.rs_debug_xornet(-1) >= before


def _batch(oracle_lib, k, m, S, B, seed):
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    ref = np.zeros((B, k + m, S), dtype=np.uint8)
    ref[:, :k] = data
    c = oracle_lib.Codec(k, m)
    for t in range(B):
        sh = [np.ascontiguousarray(ref[t, i]) for i in range(k + m)]
        c.encode_parity(sh, 0, S)
        for i in range(k, k + m):
            ref[t, i] = sh[i]
    return ref


def _dev(torch, host, stride):
    B, T, S = host.shape
    h = np.zeros((B, T, stride), dtype=np.uint8)
    h[:, :, :S] = host
    return torch.from_numpy(h.reshape(-1)).to("cuda:0")


def _host(buf, B, T, S, stride):
    return buf.cpu().numpy().reshape(B, T, stride)[:, :, :S]


@pytest.mark.parametrize("k,m,S,B,pad", [
    (4, 2, 8192, 5, 0),          # whole 2 KiB chunks
    (10, 4, 6 * 2048 + 53, 3, 256),  # ragged: xornet + vector tail + byte tail
    (17, 3, 4096 + 2048, 2, 512),    # nout = 3
    (6, 6, 2048 * 3, 2, 0),          # nout = 6: two launch groups (4 + 2 outputs)
    (1, 1, 2048, 4, 0),
])
def test_encode_decode_verify(gpu, oracle_lib, xornet_forced, k, m, S, B, pad):
    import torch

    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    native = xornet_forced
    n0 = native.rs_debug_xornet(2)
    ref = _batch(oracle_lib, k, m, S, B, seed=k * 31 + m)
    stride = (S + 15) // 16 * 16 + pad
    lay = StripeLayout(B, S, stride, stride * (k + m))
    work = ref.copy()
    work[:, k:] = 0
    buf = _dev(torch, work, stride)
    st = torch.cuda.current_stream()
    rs = rsamd.ReedSolomon.create(k, m)
    device.encode(rs, buf.data_ptr(), lay, st)
    assert np.array_equal(_host(buf, B, k + m, S, stride), ref), "encode differs from the oracle"
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
    assert int(flag.item()) == 0
    # one flipped bit in the xornet-coded columns and one in the tail columns
    for col in sorted({7, S - 1}):
        bad = ref.copy()
        bad[B - 1, k + m - 1, col] ^= 0x40
        b2 = _dev(torch, bad, stride)
        flag.zero_()
        device.verify(rs, b2.data_ptr(), lay, flag.data_ptr(), st)
        assert int(flag.item()) == 1, col
    # decode: up to m erasures, spread over data and parity
    rng = np.random.default_rng(k + m)
    for _ in range(3):
        miss = sorted(rng.choice(k + m, size=min(m, 4), replace=False).tolist())
        work = ref.copy()
        work[:, miss] = 0xA5
        buf = _dev(torch, work, stride)
        device.decode(rs, buf.data_ptr(), [i not in miss for i in range(k + m)], lay, st)
        assert np.array_equal(_host(buf, B, k + m, S, stride), ref), f"decode {miss}"
    assert native.rs_debug_xornet(2) >= max(1, n0)  # generated kernels compiled (mode 2 fails loudly if not)


def test_same_bytes_as_table_kernels(gpu, native):
    """The two kernel families on the same random batch (10+4, ragged)."""
    import torch

    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    k, m, S, B = 10, 4, 3 * 2048 + 1000, 16
    lay = StripeLayout.packed(B, k + m, S)
    outs = []
    for mode in (0, 2):
        native.rs_debug_xornet(mode)
        try:
            buf = torch.zeros(lay.nbytes, dtype=torch.uint8, device="cuda:0")
            st = torch.cuda.current_stream()
            # S is not a multiple of 8: fill a rounded-down length, the rest stays zero
            device.fill_synthetic(buf.data_ptr(), k, StripeLayout(B, S // 8 * 8, lay.shard_stride, lay.stripe_stride),
                                  SEED, 0, st)
            rs = rsamd.ReedSolomon.create(k, m)
            device.encode(rs, buf.data_ptr(), lay, st)
            device.decode(rs, buf.data_ptr(), [i not in (1, 4, 11, 12) for i in range(k + m)], lay, st)
            outs.append(buf.cpu().numpy())
        finally:
            native.rs_debug_xornet(-1)
    assert np.array_equal(outs[0], outs[1])


def test_full_size_10p4_default_threshold(gpu, oracle_lib, native):
    """configs[3] per-GPU share through the XOR-network kernel at the default size threshold."""
    import torch

    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    n0 = native.rs_debug_xornet(1)
    k, m, S, B = 10, 4, 4 << 20, 128
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream()
    device.fill_synthetic(buf.data_ptr(), k, lay, SEED, 0, st)
    device.encode(rs, buf.data_ptr(), lay, st)
    torch.cuda.synchronize()
    assert native.rs_debug_xornet(-1) >= max(1, n0)  # compiled (or reused) the 10+4 encode network
    c = oracle_lib.Codec(k, m)
    for t in (0, B - 1):
        row = buf[t * lay.stripe_stride:(t + 1) * lay.stripe_stride].cpu().numpy()
        sh = [row[i * lay.shard_stride: i * lay.shard_stride + S].copy() for i in range(k + m)]
        ref = [s.copy() for s in sh]
        for p in range(m):
            ref[k + p][:] = 0
        c.encode_parity(ref, 0, S)
        assert all(np.array_equal(a, b) for a, b in zip(sh, ref)), t
    del buf
    torch.cuda.empty_cache()
