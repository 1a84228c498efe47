// gf_device.hpp -- device-side GF(2^8) helpers shared by kernels.hip and the
// kernel microbenchmark (tools/kbench.hip).  See kernels.hip for the design.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

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

// Fold the 3*N terms of one output dword with 3-input XORs.
template <int N>
__device__ __forceinline__ uint32_t dot_dword(const uint32_t (&T)[N][5], const Sel (&s)[N]) {
    uint32_t a, b, c;
    terms(T[0], s[0], a, b, c);
    uint32_t acc = xor3(a, b, c);
#pragma unroll
    for (int i = 1; i < N; ++i) {
        terms(T[i], s[i], a, b, c);
        acc = xor3(acc, a, b);
        acc ^= c;
    }
    return acc;
}

__device__ __forceinline__ void flag_mismatch(int *mismatch) {
    __hip_atomic_fetch_or(mismatch, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool mismatch_seen(const int *mismatch) {
    return __hip_atomic_load(mismatch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

}  // namespace dev
}  // namespace rsamd
