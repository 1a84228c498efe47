"""CPU check of the generated bitsliced XOR-network kernels (csrc/xornet.cpp).

The library generates one HIP kernel per coefficient matrix (rs_xornet_source)
and compiles it at run time for gfx950.  Here the SAME generated source is
compiled for the host by clang with a small shim (builtins as plain C, one
call per (block, lane)) and run over a stripe batch; its outputs must equal the
oracle's codeSomeShards (InputOutputByteTableCodingLoop.java:12-44) byte for
byte, and the verify variant must flag exactly the corrupted batches.  This
pins the generator's math -- the bit-plane transposes, the per-coefficient bit
matrices and the XOR folding -- before any GPU run; tests/test_gpu_xornet.py
checks the compiled kernels on the device.
"""
import ctypes as C
import hashlib
import os
import subprocess

import numpy as np
import pytest

CLANG = "/opt/rocm/llvm/bin/clang++"
BUILD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "build", "xornet_host")

SHIM = r"""
#include <cstdint>
#include <cstring>
struct rs_dim3 { unsigned x, y, z; };
static rs_dim3 blockIdx, threadIdx;
#define __global__
#define __device__
#define __forceinline__ inline
#define __launch_bounds__(n)
static inline unsigned rs_bitop3(unsigned a, unsigned b, unsigned c, unsigned tt) {
    unsigned r = 0;
    for (int idx = 0; idx < 8; ++idx)
        if ((tt >> idx) & 1) r |= ((idx & 4) ? a : ~a) & ((idx & 2) ? b : ~b) & ((idx & 1) ? c : ~c);
    return r;
}
#define __builtin_amdgcn_bitop3_b32(a, b, c, t) rs_bitop3((a), (b), (c), (t))
#define __builtin_nontemporal_load(p) (*(p))
#define __builtin_nontemporal_store(v, p) (*(p) = (v))
#define __hip_atomic_fetch_or(p, v, o, s) (*(p) |= (v))
#ifndef __HIP_MEMORY_SCOPE_AGENT
#define __HIP_MEMORY_SCOPE_AGENT 0
#endif
"""

DRIVER = r"""
extern "C" void run_all(unsigned char *base, const int *in_idx, const int *out_idx, unsigned long long stripe_stride,
                        unsigned long long shard_stride, unsigned chunks, unsigned n_stripes, unsigned rot,
                        int *mismatch) {
    unsigned l = 0;
    while ((1ull << l) < chunks) ++l;
    XorNetArgs a;
    a.base = base; a.in_idx = in_idx; a.out_idx = out_idx; a.stripe_stride = stripe_stride;
    a.shard_stride = shard_stride; a.chunks = chunks; a.n_items = chunks * n_stripes;
    a.cdiv_m = (unsigned)(((1ull << 32) * ((1ull << l) - chunks)) / chunks + 1);
    a.cdiv_s1 = l < 1 ? l : 1u; a.cdiv_s2 = l > 1 ? l - 1 : 0u;
    a.xcd_span = a.n_items / 8u; a.rot = rot % chunks; a.mismatch = mismatch;
    for (unsigned b = 0; b < a.n_items; ++b)
        for (unsigned t = 0; t < 64; ++t) {
            blockIdx.x = b; threadIdx.x = t;
            rsamd_xornet(a);
        }
}
"""


def generated_source(native, rows, verify):
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    nout, nin = rows.shape
    ops = C.c_int()
    n = native.rs_xornet_source(rows.ctypes.data_as(C.POINTER(C.c_uint8)), nin, nout, int(verify), None, 0,
                                C.byref(ops))
    assert n > 0
    buf = C.create_string_buffer(n + 1)
    assert native.rs_xornet_source(rows.ctypes.data_as(C.POINTER(C.c_uint8)), nin, nout, int(verify), buf, n + 1,
                                   None) == n
    return buf.value.decode(), ops.value


def host_kernel(native, rows, verify):
    src, ops = generated_source(native, rows, verify)
    key = hashlib.sha256((src + SHIM + DRIVER).encode()).hexdigest()[:16]
    os.makedirs(BUILD, exist_ok=True)
    so = os.path.join(BUILD, f"xn_{key}.so")
    if not os.path.exists(so):
        cpp = so[:-3] + ".cpp"
        with open(cpp, "w") as f:
            f.write(SHIM + src + DRIVER)
        subprocess.run([CLANG, "-O1", "-std=c++17", "-shared", "-fPIC", "-w", cpp, "-o", so], check=True)
    lib = C.CDLL(so)
    lib.run_all.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_ulonglong, C.c_ulonglong, C.c_uint, C.c_uint,
                            C.c_uint, C.c_void_p]
    return lib, ops


def run_batch(lib, buf, in_idx, out_idx, stripe_stride, shard_stride, chunks, n_stripes, mismatch=None, rot=0):
    ii = np.ascontiguousarray(in_idx, dtype=np.int32)
    oo = np.ascontiguousarray(out_idx, dtype=np.int32)
    mm = np.zeros(1, dtype=np.int32) if mismatch is None else mismatch
    lib.run_all(buf.ctypes.data, ii.ctypes.data, oo.ctypes.data, stripe_stride, shard_stride, chunks, n_stripes, rot,
                mm.ctypes.data)
    return int(mm[0])


def check_matrix(native, oracle_lib, rows, seed, S=4096, n_stripes=3, pad=256, verify=True, rot=0):
    """Batch of n_stripes stripes [inputs..., outputs...] of S bytes (2 KiB
    chunks), shard stride S + pad: emulated kernel vs the oracle."""
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    nout, nin = rows.shape
    rng = np.random.default_rng(seed)
    stride = S + pad
    total = nin + nout
    buf = np.zeros(n_stripes * total * stride, dtype=np.uint8)
    view = buf.reshape(n_stripes, total, stride)
    view[:, :nin, :S] = rng.integers(0, 256, (n_stripes, nin, S), dtype=np.uint8)
    # shard order inside a stripe: outputs first, then inputs reversed (index lists are not identity)
    in_idx = [total - 1 - i for i in range(nin)]
    out_idx = list(range(nout))
    perm = view.copy()
    for i in range(nin):
        perm[:, in_idx[i]] = view[:, i]
    view[:] = perm
    lib, ops = host_kernel(native, rows, False)
    run_batch(lib, buf, in_idx, out_idx, total * stride, stride, S // 2048, n_stripes, rot=rot)
    for t in range(n_stripes):
        ins = [np.ascontiguousarray(view[t, in_idx[i], :S]) for i in range(nin)]
        outs = [np.zeros(S, np.uint8) for _ in range(nout)]
        oracle_lib.code_some_shards(7, rows, ins, outs, 0, S)
        for p in range(nout):
            assert np.array_equal(view[t, out_idx[p], :S], outs[p]), f"stripe {t} output {p}"
        assert not view[t, :, S:].any(), "wrote into the pad"
    if verify:
        vlib, _ = host_kernel(native, rows, True)
        assert run_batch(vlib, buf, in_idx, out_idx, total * stride, stride, S // 2048, n_stripes) == 0
        view[n_stripes - 1, out_idx[-1], S - 1] ^= 0x10
        assert run_batch(vlib, buf, in_idx, out_idx, total * stride, stride, S // 2048, n_stripes) == 1
    return ops


@pytest.mark.parametrize("k,m", [(4, 2), (10, 4), (17, 3), (1, 1)])
def test_encode_matrices(native, oracle_lib, k, m):
    G = oracle_lib.build_matrix(k, k + m)
    ops = check_matrix(native, oracle_lib, G[k:], seed=k * 100 + m)
    if (k, m) == (10, 4):
        assert ops < 1250  # network + transposes per 32 columns (vs 2 x 1046 for the table kernel)


@pytest.mark.parametrize("present", [
    [0, 1, 1, 1, 1, 0], [0, 0, 1, 1, 1, 1], [1, 1, 0, 0, 1, 1], [1, 0, 1, 1, 1, 1],
])
def test_decode_matrices_4p2(native, oracle_lib, present):
    codec = oracle_lib.Codec(4, 2)
    _, _, rows = codec.decode_rows(present)
    check_matrix(native, oracle_lib, rows, seed=sum(present), verify=False)


def test_decode_matrix_10p4_four_erasures(native, oracle_lib):
    codec = oracle_lib.Codec(10, 4)
    _, _, rows = codec.decode_rows([0, 0, 0, 0] + [1] * 10)
    check_matrix(native, oracle_lib, rows, seed=7, n_stripes=2)


@pytest.mark.parametrize("nin,nout,seed", [(1, 4, 1), (3, 1, 2), (7, 3, 3), (12, 4, 4), (2, 2, 5)])
def test_random_matrices(native, oracle_lib, nin, nout, seed):
    rng = np.random.default_rng(seed)
    rows = rng.integers(0, 256, (nout, nin), dtype=np.uint8)
    rows[0, 0] = 0  # zero, one and 255 coefficients
    if nin > 1:
        rows[0, 1] = 1
        rows[-1, -1] = 255
    check_matrix(native, oracle_lib, rows, seed=seed, n_stripes=2)


def test_chunk_rotation_covers_every_chunk(native, oracle_lib):
    """Block order with a per-stripe chunk rotation (3 chunks, rotation 2)."""
    G = oracle_lib.build_matrix(4, 6)
    check_matrix(native, oracle_lib, G[4:], seed=3, S=3 * 2048, n_stripes=4, verify=False, rot=2)


def test_zero_row_writes_zeros(native, oracle_lib):
    rows = np.zeros((2, 3), dtype=np.uint8)
    rows[1] = [5, 6, 7]
    check_matrix(native, oracle_lib, rows, seed=11, n_stripes=1)


def test_source_rejects_bad_shapes(native):
    rows = np.zeros((5, 2), dtype=np.uint8)
    assert native.rs_xornet_source(rows.ctypes.data_as(C.POINTER(C.c_uint8)), 2, 5, 0, None, 0, None) < 0
    assert native.rs_xornet_source(rows.ctypes.data_as(C.POINTER(C.c_uint8)), 0, 1, 0, None, 0, None) < 0
