"""GPU tests with no slack: every buffer a call touches ends exactly where the
call's arguments say it ends, at the end of its own allocation.

The round-3 fault (hipErrorIllegalAddress after rs_file_decode_dev on
4+2 x block 1000 x 1,234,567 bytes, S = 309,000, S % 16 == 8) surfaced in a
test whose output buffer had 16 bytes of slack inside a torch caching-allocator
segment, where a small overrun touches mapped memory and only faults once in
many runs.  Here the file, the shard batch and the output are each their own
rs_dev_alloc allocation of exactly the bytes the call describes:
  * against the bounds-checking build (make -C csrc bounds, RSAMD_TEST_LIB),
    any kernel access outside those bytes fails the test deterministically
    (tests/conftest.py bounds_check; csrc/bounds.hpp);
  * against the product build, the same calls run with 4 KiB canaries on both
    sides of every buffer, so any stray write is caught too.
Shapes: the faulting one (with and without write_missing, every erasure set
of ReedSolomonDecoder.java:33-103's callers), exact strides (S % 16 == 8 on an
8-aligned stride), tiled-decode last tiles of 1..R-1 rows, ragged single
stripes (launch_gf's vector + byte tail), the master's 1000-byte chunk groups
(the line-owner kernel) and per-group bitmasks.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GUARD = 4096
CANARY = 0xA5


class Tight:
    """nbytes of HBM with GUARD canary bytes on each side, or (guard=False)
    exactly nbytes, ending at the end of its own allocation."""

    def __init__(self, nbytes, guard=True, off=0):
        from rsamd.device import DeviceBuffer
        self.n, self.g = nbytes, (GUARD if guard else 0) + off  # off: the buffer's start past an aligned one
        self.buf = DeviceBuffer(max(1, nbytes + 2 * self.g - off), contiguous=False)
        self.t = self.buf.tensor()
        self.t.fill_(CANARY)

    def ptr(self):
        return self.buf.data_ptr() + self.g

    def view(self):
        return self.t[self.g: self.g + self.n]

    def check(self):
        if self.g >= GUARD:
            head = self.t[: self.g].cpu().numpy()
            tail = self.t[self.g + self.n:].cpu().numpy()
            assert (head == CANARY).all(), f"write before the buffer at {int(np.argmax(head != CANARY)) - self.g}"
            assert (tail == CANARY).all(), f"write past the buffer at +{int(np.argmax(tail != CANARY))}"

    def free(self):
        self.buf.free()


def _bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


@pytest.mark.parametrize("guard", [False, True], ids=["no-slack", "canary"])
@pytest.mark.parametrize("k,m,block,n,stride_mode", [
    (4, 2, 1000, 1_234_567, "aligned"),   # round 3's faulting shape: S % 16 == 8, last tile 5 of 8 rows
    (4, 2, 1000, 1_234_567, "exact"),     # stride = S: generic split/merge + 8-byte kernels
    (4, 2, 1000, 4000 * 37, "aligned"),   # S = 37000: last tile 5 rows, file ends on a row
    (4, 2, 1000, 4000 * 9 - 1, "aligned"),  # one tile + 1 row, ragged file end
    (4, 2, 1000, 4000 * 15 + 7, "aligned"),  # last tile 8 rows - 1 ... ragged
    (4, 2, 512, 100_000, "exact"),        # S % 16 == 0
    (4, 2, 1000, 7, "aligned"),           # a one-row file
    (10, 4, 1000, 500_003, "aligned"),    # generic paths
])
def test_file_paths_no_slack(gpu, oracle_lib, guard, k, m, block, n, stride_mode):
    import torch
    import rsamd
    from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
    rs = rsamd.ReedSolomon.create(k, m)
    _, S = file_layout(rs, n, block)
    stride = S if stride_mode == "exact" else (S + 255) // 256 * 256
    data = _bytes(n, n + k)
    ref = oracle_lib.Codec(k, m).file_encode(data.tobytes(), block)
    st = torch.cuda.current_stream()
    f = Tight(n, guard)
    f.view().copy_(torch.from_numpy(data).to("cuda:0"))
    sh_bytes = (k + m - 1) * stride + S  # the last shard ends the batch
    sh = Tight(sh_bytes, guard)
    encode_file_dev(rs, f.ptr(), n, sh.ptr(), stride, block, st)
    torch.cuda.synchronize()
    got = np.empty((k + m, S), np.uint8)
    host = sh.view().cpu().numpy()
    for i in range(k + m):
        got[i] = host[i * stride: i * stride + S]
    assert np.array_equal(got, ref)
    f.check()
    sh.check()
    for miss in [(), (0,), (1, k), (k,), (k + m - 1,), tuple(range(min(m, k)))]:
        present = [i not in miss for i in range(k + m)]
        for wm in (False, True):
            s2 = Tight(sh_bytes, guard)
            s2.view().copy_(sh.view())
            v = s2.view()
            for j in miss:
                v[j * stride: j * stride + S] = 0
            out = Tight(n, guard)
            decode_file_dev(rs, s2.ptr(), S, stride, present, out.ptr(), n, block, wm, st)
            torch.cuda.synchronize()
            assert np.array_equal(out.view().cpu().numpy(), data), (miss, wm)
            if wm:
                h2 = s2.view().cpu().numpy()
                for i in range(k + m):
                    assert np.array_equal(h2[i * stride: i * stride + S], ref[i]), (miss, i)
            out.check()
            s2.check()
            out.free()
            s2.free()
    f.free()
    sh.free()


@pytest.mark.parametrize("guard", [False, True], ids=["no-slack", "canary"])
@pytest.mark.parametrize("k,m,S,B,stride,off", [
    (4, 2, 309_000, 1, 309_248, 0),   # the faulting test's write_missing launch: one ragged stripe
    (4, 2, 309_000, 3, 309_000, 0),   # 8-aligned stride
    (4, 2, 4096 + 8, 7, 4096 + 16, 0),
    (4, 2, 1000, 4099, 1000, 0),      # the master's chunk groups, back to back: line-owner kernel
    (4, 2, 24, 5, 24, 0),             # below the vector width: byte kernel only
    (10, 4, 65536 + 24, 3, 65536 + 32, 0),
    (4, 2, 1_048_000, 1, 1_048_576, 8),  # 8 bytes off 16 with 16-byte strides: 8-column peel + 16-byte kernels
    (4, 2, 65_536, 5, 65_536, 8),        # the same over several stripes
])
def test_stripe_batches_no_slack(gpu, oracle_lib, guard, k, m, S, B, stride, off):
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    rs = rsamd.ReedSolomon.create(k, m)
    T = k + m
    lay = StripeLayout(B, S, stride, T * stride)
    nbytes = (B - 1) * lay.stripe_stride + (T - 1) * stride + S
    buf = Tight(nbytes, guard, off)
    st = torch.cuda.current_stream()
    data = _bytes(B * k * S, S + B)
    host = np.zeros(nbytes, np.uint8)
    for t in range(B):
        for i in range(k):
            o = t * lay.stripe_stride + i * stride
            host[o: o + S] = data[(t * k + i) * S: (t * k + i + 1) * S]
    buf.view().copy_(torch.from_numpy(host).to("cuda:0"))
    device.encode(rs, buf.ptr(), lay, st)
    flag = Tight(4, guard)
    flag.view().zero_()
    device.verify(rs, buf.ptr(), lay, flag.ptr(), st)
    torch.cuda.synchronize()
    assert int(flag.view().view(torch.int32).item()) == 0
    enc = buf.view().cpu().numpy()
    oc = oracle_lib.Codec(k, m)
    for t in sorted({0, B // 2, B - 1}):
        shards = [enc[t * lay.stripe_stride + i * stride:][:S].copy() for i in range(T)]
        ref = [s.copy() for s in shards[:k]] + [np.zeros(S, np.uint8) for _ in range(m)]
        oc.encode_parity(ref, 0, S)
        for p in range(m):
            assert np.array_equal(shards[k + p], ref[k + p]), (t, p)
    # uniform decode, then per-stripe bitmasks with a different pattern per stripe
    miss = (0, T - 1)
    dec = buf.view()
    for t in range(B):
        for j in miss:
            o = t * lay.stripe_stride + j * stride
            dec[o: o + S] = 0
    device.decode(rs, buf.ptr(), [i not in miss for i in range(T)], lay, st)
    torch.cuda.synchronize()
    assert np.array_equal(buf.view().cpu().numpy(), enc)
    rng = np.random.default_rng(B)
    present = np.ones((B, T), bool)
    for t in range(B):
        present[t, rng.choice(T, size=int(rng.integers(0, m + 1)), replace=False)] = False
        for j in np.flatnonzero(~present[t]):
            o = t * lay.stripe_stride + j * stride
            dec[o: o + S] = 0
    bits = Tight(4 * B, guard)
    bits.view().copy_(torch.from_numpy(device.presence_bits(present).view(np.uint8)).to("cuda:0"))
    bad = Tight(4, guard)
    bad.view().zero_()
    device.decode_masked_bits(rs, buf.ptr(), bits.ptr(), lay, bad.ptr(), st)
    torch.cuda.synchronize()
    assert int(bad.view().view(torch.int32).item()) == 0
    assert np.array_equal(buf.view().cpu().numpy(), enc)
    for x in (buf, flag, bits, bad):
        x.check()
        x.free()


def test_bounds_build_flags_an_overrun(gpu):
    """The checker itself (bounds-checking build only; the product build would
    really overrun): a batch whose arguments describe 16 bytes more than its
    allocation holds is reported -- by the host check of the declared range
    and by the kernels' accesses past the allocation, which are redirected
    instead of made."""
    import ctypes as C
    import torch
    import rsamd
    from rsamd import _lib, device
    from rsamd.device import StripeLayout
    lib = _lib.load()
    if not hasattr(lib, "rs_bounds_report"):
        pytest.skip("product library: the overrun would be real (run with RSAMD_TEST_LIB=lib/bounds/librsamd.so)")
    k, m, S, B = 4, 2, 4096, 3
    lay = StripeLayout.packed(B, k + m, S)
    buf = Tight(lay.nbytes - 16, guard=False)
    rs = rsamd.ReedSolomon.create(k, m)
    device.encode(rs, buf.ptr(), lay, torch.cuda.current_stream())
    torch.cuda.synchronize()
    n, addr, ln, where = C.c_ulonglong(), C.c_ulonglong(), C.c_ulonglong(), C.c_uint()
    lib.rs_bounds_report(C.byref(n), C.byref(addr), C.byref(ln), C.byref(where))
    assert n.value >= 2 and where.value == 900003, (n.value, where.value)
    buf.free()
