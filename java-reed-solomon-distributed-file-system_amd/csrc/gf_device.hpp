// gf_device.hpp -- device-side GF(2^8) helpers shared by kernels.hip and the
// kernel microbenchmark (tools/kbench.hip).  See kernels.hip for the design.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "bounds.hpp"

namespace rsamd {
namespace dev {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Selector bytes of one input dword (four GF elements).
struct Sel {
    uint32_t c0, c1, c2;
};
__device__ __forceinline__ Sel selectors(uint32_t x) {
    return Sel{x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

// The three partial products c*x0, c*(x1<<3), c*(x2<<6) of four bytes.
// v_perm_b32(S0, S1, sel): selector byte 0..3 picks byte of S1, 4..7 of S0.
__device__ __forceinline__ void terms(const uint32_t *t, const Sel &s, uint32_t &a, uint32_t &b,
                                      uint32_t &c) {
    a = __builtin_amdgcn_perm(t[1], t[0], s.c0);
    b = __builtin_amdgcn_perm(t[3], t[2], s.c1);
    c = __builtin_amdgcn_perm(t[4], t[4], s.c2);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Folds input i's three terms into acc.  Terms are paired across inputs so
// every v_bitop3_b32 takes two new terms: an odd input leaves its third term
// in `carry`, the next (even) input consumes it.  N inputs then cost
// (3N - 1) / 2 ops (15 for N = 10) instead of 2N - 1 (19); fold_end() adds
// the carry an even N leaves behind.  `i` is a compile-time constant after
// unrolling, so the branches fold away.
__device__ __forceinline__ void fold_terms(int i, uint32_t &acc, uint32_t &carry, uint32_t a, uint32_t b,
                                           uint32_t c) {
    if (i == 0) {
        acc = xor3(a, b, c);
    } else if (i & 1) {
        acc = xor3(acc, a, b);
        carry = c;
    } else {
        acc = xor3(xor3(acc, carry, a), b, c);
    }
}
__device__ __forceinline__ uint32_t fold_end(int n, uint32_t acc, uint32_t carry) {
    return (n % 2 == 0) ? acc ^ carry : acc;
}

// Fold the 3*N terms of one output dword with 3-input XORs.
template <int N>
__device__ __forceinline__ uint32_t dot_dword(const uint32_t (&T)[N][5], const Sel (&s)[N]) {
    uint32_t a, b, c, acc = 0, carry = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        terms(T[i], s[i], a, b, c);
        fold_terms(i, acc, carry, a, b, c);
    }
    return fold_end(N, acc, carry);
}

__device__ __forceinline__ void flag_mismatch(int *mismatch) {
    __hip_atomic_fetch_or(RSAMD_G(mismatch, 4), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Early-exit hint for verify launches: a plain load, possibly stale (a block
// that misses an earlier mismatch just does its own check).  Not an atomic:
// the compiler models an atomic load as a possible clobber of every later
// load, which turns the scalar table loads into per-lane vector loads
// (252 VGPRs and 2 waves per SIMD for the 10+4 verify kernel).
__device__ __forceinline__ bool mismatch_seen(const int *mismatch) { return *RSAMD_G(mismatch, 4) != 0; }

// A small host call's completion signal (kernels.hpp DirectSignal), after a
// block's last store: the block's stores are made visible system-wide and it
// counts itself done on `ctr`; the last block resets `ctr`, moves the verify
// word (if any) into flag[1] and releases `seq` into flag[0].  Vector atomics
// on global memory only.
__device__ __forceinline__ void signal_done(uint32_t *flag, uint32_t *ctr, uint32_t seq, int *mismatch) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x != 0) return;
    const uint32_t prev = __hip_atomic_fetch_add(RSAMD_G(ctr, 4), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1 != gridDim.x) return;
    __hip_atomic_store(RSAMD_G(ctr, 4), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t mm = 0;
    if (mismatch) {
        mm = uint32_t(__hip_atomic_load(RSAMD_G(mismatch, 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        __hip_atomic_store(RSAMD_G(mismatch, 4), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_store(RSAMD_G(flag + 1, 4), mm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(RSAMD_G(flag, 4), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace dev
}  // namespace rsamd
