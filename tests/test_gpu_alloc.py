"""GPU tests of rs_dev_alloc / rs_dev_free (rsamd.device.DeviceBuffer): a
physically contiguous stripe pool and a hipMalloc one both code bit-exactly
(encode, verify, decode against the oracle)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED


@pytest.mark.parametrize("contiguous", [True, False])
def test_stripe_pool_codes_exactly(gpu, oracle_lib, contiguous):
    import ctypes as C
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import DeviceBuffer, StripeLayout
    k, m, S, B = 4, 2, 1 << 20, 256
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    pool = DeviceBuffer(lay.nbytes, contiguous=contiguous)
    assert pool.data_ptr() % 256 == 0 and pool.numel() == lay.nbytes
    if not contiguous:
        assert pool.contiguous is False
    st = torch.cuda.current_stream()
    device.fill_synthetic(pool.data_ptr(), k, lay, SEED, 0, st)
    device.encode(rs, pool.data_ptr(), lay, st)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    device.verify(rs, pool.data_ptr(), lay, flag.data_ptr(), st)
    torch.cuda.synchronize()
    assert int(flag.item()) == 0
    hip = C.CDLL("libamdhip64.so")
    row = np.empty(lay.stripe_stride, np.uint8)
    for t in (0, B - 1):
        assert hip.hipMemcpy(row.ctypes.data_as(C.c_void_p), C.c_void_p(pool.data_ptr() + t * lay.stripe_stride),
                             C.c_size_t(lay.stripe_stride), 2) == 0  # hipMemcpyDeviceToHost
        sh = [row[i * lay.shard_stride: i * lay.shard_stride + S].copy() for i in range(k + m)]
        assert np.array_equal(np.concatenate(sh[:k]), oracle_lib.fill_synthetic(k * S, SEED, t))
        ref = [x.copy() for x in sh]
        ref[4][:] = 0
        ref[5][:] = 0
        oracle_lib.Codec(k, m).encode_parity(ref, 0, S)
        assert all(np.array_equal(a, b) for a, b in zip(sh, ref)), t
    pool.free()
    pool.free()  # idempotent
