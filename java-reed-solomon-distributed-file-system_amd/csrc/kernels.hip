// kernels.hip -- gfx950 kernels of the Reed-Solomon engine.
//
// The one hot operation is the GF(2^8) matrix-times-shards product of
// CodingLoop.codeSomeShards (CodingLoop.java:79-85; default loop
// InputOutputByteTableCodingLoop.java:12-44):
//     out[p][b] = XOR_i mul(row[p][i], in[i][b])
// Encode (ReedSolomon.java:90-104) and decode (ReedSolomon.java:175-272, fused
// to one pass by the host, see codec.cpp) both run it; only the coefficient
// rows and the shard index lists differ.
//
// Design:
//  * Byte-stream, HBM-bound: each input byte is read once and each output byte
//    written once -- (nin + nout) bytes per column, not the Java loop's
//    nin*nout read-modify-write passes.  16 bytes per lane per shard
//    (global_load_dwordx4 / global_store_dwordx4), 1 KiB per wave-instruction.
//  * No tables in memory on the hot path.  Multiplication by the constant c is
//    linear over GF(2), so c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6] with
//    8/8/4-entry tables that fit in 2/2/1 registers; one v_perm_b32 looks up
//    four bytes of a dword at once.  The tables are wave-uniform (scalar
//    loads) and the 3*nin terms of an output are folded with v_bitop3_b32
//    (3-input XOR, gfx950).  Per (input, output) pair and dword: 3 v_perm +
//    1.5 v_bitop3; per input dword 5 ops of selector extraction.  No LDS, no
//    MFMA (GF(2^8) is not a float contraction).
//  * Work item = (stripe, run of 256*U vectors of it): block-uniform index
//    math on the scalar unit, lanes take consecutive 16-byte vectors, so every
//    wave-instruction touches one contiguous KiB of one shard.
#include "kernels.hpp"

#include <algorithm>
#include <climits>
#include <cstdlib>

namespace rsamd {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;

struct VecArgs {
    uint8_t *base;
    const uint32_t *tabs;
    const int32_t *in_idx;
    const int32_t *out_idx;
    uint64_t stripe_stride;
    uint64_t shard_stride;
    uint32_t nvec;     // full 16-byte vectors per shard
    uint32_t chunks;   // work items per stripe
    uint32_t n_items;  // work items in this launch
    int nin;           // generic kernel only
    int *mismatch;     // Mode::Verify only
};

struct ByteArgs {
    uint8_t *base;
    const uint32_t *tabs;
    const int32_t *in_idx;
    const int32_t *out_idx;
    uint64_t stripe_stride;
    uint64_t shard_stride;
    uint64_t col0;
    uint64_t ncols;
    uint64_t total;  // n_stripes * ncols
    int nin, nout;
    int *mismatch;
};

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

// ---------------------------------------------------------------------------
// Vector kernel, compile-time shape: K inputs, M outputs, U vectors per lane.
// ---------------------------------------------------------------------------
template <int K, int M, int U, bool VERIFY>
__global__ void __launch_bounds__(kThreads) gf_vec_kernel(VecArgs a) {
    uint32_t T[M][K][5];  // wave-uniform: lives in SGPRs
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int p = 0; p < M; ++p)
#pragma unroll
            for (int j = 0; j < 5; ++j) T[p][i][j] = a.tabs[(i * M + p) * 5 + j];
    uint64_t in_off[K], out_off[M];
#pragma unroll
    for (int i = 0; i < K; ++i) in_off[i] = uint64_t(a.in_idx[i]) * a.shard_stride;
#pragma unroll
    for (int p = 0; p < M; ++p) out_off[p] = uint64_t(a.out_idx[p]) * a.shard_stride;

    for (uint32_t item = blockIdx.x; item < a.n_items; item += gridDim.x) {
        if (VERIFY && mismatch_seen(a.mismatch)) return;
        const uint32_t stripe = item / a.chunks;
        const uint32_t chunk = item - stripe * a.chunks;
        uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride;
        const uint32_t v0 = chunk * uint32_t(kThreads * U) + threadIdx.x;

        u32x4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t v = v0 + u * kThreads;
            if (v < a.nvec) {
#pragma unroll
                for (int i = 0; i < K; ++i)
                    x[u][i] = *reinterpret_cast<const u32x4 *>(sb + in_off[i] + uint64_t(v) * 16);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t v = v0 + u * kThreads;
            if (v >= a.nvec) continue;
            u32x4 acc[M];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                Sel s[K];
#pragma unroll
                for (int i = 0; i < K; ++i) s[i] = selectors(x[u][i][w]);
#pragma unroll
                for (int p = 0; p < M; ++p) acc[p][w] = dot_dword<K>(T[p], s);
            }
#pragma unroll
            for (int p = 0; p < M; ++p) {
                u32x4 *dst = reinterpret_cast<u32x4 *>(sb + out_off[p] + uint64_t(v) * 16);
                if (VERIFY) {
                    const u32x4 have = *dst;
                    if (have[0] != acc[p][0] || have[1] != acc[p][1] || have[2] != acc[p][2] ||
                        have[3] != acc[p][3])
                        flag_mismatch(a.mismatch);
                } else {
                    *dst = acc[p];
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Vector kernel, runtime input count (any k), M outputs, one vector per lane.
// ---------------------------------------------------------------------------
template <int M, bool VERIFY>
__global__ void __launch_bounds__(kThreads) gf_vec_generic_kernel(VecArgs a) {
    uint64_t out_off[M];
#pragma unroll
    for (int p = 0; p < M; ++p) out_off[p] = uint64_t(a.out_idx[p]) * a.shard_stride;

    for (uint32_t item = blockIdx.x; item < a.n_items; item += gridDim.x) {
        if (VERIFY && mismatch_seen(a.mismatch)) return;
        const uint32_t stripe = item / a.chunks;
        const uint32_t chunk = item - stripe * a.chunks;
        uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride;
        const uint32_t v = chunk * uint32_t(kThreads) + threadIdx.x;
        if (v >= a.nvec) continue;
        u32x4 acc[M];
#pragma unroll
        for (int p = 0; p < M; ++p) acc[p] = u32x4{0, 0, 0, 0};
#pragma unroll 2
        for (int i = 0; i < a.nin; ++i) {
            const u32x4 x =
                *reinterpret_cast<const u32x4 *>(sb + uint64_t(a.in_idx[i]) * a.shard_stride + uint64_t(v) * 16);
            uint32_t T[M][5];
#pragma unroll
            for (int p = 0; p < M; ++p)
#pragma unroll
                for (int j = 0; j < 5; ++j) T[p][j] = a.tabs[(i * M + p) * 5 + j];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const Sel s = selectors(x[w]);
#pragma unroll
                for (int p = 0; p < M; ++p) {
                    uint32_t t0, t1, t2;
                    terms(T[p], s, t0, t1, t2);
                    acc[p][w] = xor3(acc[p][w], t0, t1) ^ t2;
                }
            }
        }
#pragma unroll
        for (int p = 0; p < M; ++p) {
            u32x4 *dst = reinterpret_cast<u32x4 *>(sb + out_off[p] + uint64_t(v) * 16);
            if (VERIFY) {
                const u32x4 have = *dst;
                if (have[0] != acc[p][0] || have[1] != acc[p][1] || have[2] != acc[p][2] || have[3] != acc[p][3])
                    flag_mismatch(a.mismatch);
            } else {
                *dst = acc[p];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Byte kernel: any alignment; also the <16-byte tail of aligned shards.
// One thread per (stripe, column byte).
// ---------------------------------------------------------------------------
template <bool VERIFY>
__global__ void __launch_bounds__(kThreads) gf_byte_kernel(ByteArgs a) {
    const uint64_t step = uint64_t(gridDim.x) * kThreads;
    for (uint64_t idx = uint64_t(blockIdx.x) * kThreads + threadIdx.x; idx < a.total; idx += step) {
        if (VERIFY && mismatch_seen(a.mismatch)) return;
        const uint64_t stripe = idx / a.ncols;
        const uint64_t col = a.col0 + (idx - stripe * a.ncols);
        uint8_t *sb = a.base + stripe * a.stripe_stride + col;
        uint32_t acc[kMaxOut] = {0, 0, 0, 0};
        for (int i = 0; i < a.nin; ++i) {
            const Sel s = selectors(sb[uint64_t(a.in_idx[i]) * a.shard_stride]);
            for (int p = 0; p < a.nout; ++p) {
                uint32_t t0, t1, t2;
                terms(a.tabs + (i * a.nout + p) * 5, s, t0, t1, t2);
                acc[p] = xor3(acc[p], t0, t1) ^ t2;
            }
        }
        for (int p = 0; p < a.nout; ++p) {
            uint8_t *dst = sb + uint64_t(a.out_idx[p]) * a.shard_stride;
            if (VERIFY) {
                if (*dst != uint8_t(acc[p])) flag_mismatch(a.mismatch);
            } else {
                *dst = uint8_t(acc[p]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Synthetic data and the reference copy kernel (benchmark support).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t n) {
    uint64_t z = seed + n * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(kThreads)
    fill_synthetic_kernel(uint8_t *base, uint64_t words_per_stripe, uint64_t words_per_shard,
                          uint64_t n_words, uint64_t shard_stride, uint64_t stripe_stride, uint64_t seed,
                          uint64_t stripe0) {
    const uint64_t step = uint64_t(gridDim.x) * kThreads;
    for (uint64_t idx = uint64_t(blockIdx.x) * kThreads + threadIdx.x; idx < n_words; idx += step) {
        const uint64_t t = idx / words_per_stripe;
        const uint64_t w = idx - t * words_per_stripe;
        const uint64_t shard = w / words_per_shard;
        const uint64_t col = (w - shard * words_per_shard) * 8;
        *reinterpret_cast<uint64_t *>(base + t * stripe_stride + shard * shard_stride + col) =
            splitmix64_at(seed ^ (stripe0 + t), w + 1);
    }
}

__global__ void __launch_bounds__(kThreads) copy_kernel(u32x4 *dst, const u32x4 *src, uint64_t nvec) {
    const uint64_t step = uint64_t(gridDim.x) * kThreads;
    for (uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x; i < nvec; i += step) dst[i] = src[i];
}

__global__ void copy_tail_kernel(uint8_t *dst, const uint8_t *src, uint64_t n) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

// ---------------------------------------------------------------------------
// Host-side dispatch.
// ---------------------------------------------------------------------------
unsigned max_blocks() {
    static const unsigned v = [] {
        const char *e = std::getenv("RSAMD_MAX_BLOCKS");
        long x = e ? std::atol(e) : 0;
        return x > 0 ? unsigned(x) : 0u;  // 0: one block per work item
    }();
    return v;
}

template <int K, int M, int U>
hipError_t launch_vec_t(VecArgs a, unsigned grid, Mode mode, hipStream_t s) {
    if (mode == Mode::Verify)
        hipLaunchKernelGGL((gf_vec_kernel<K, M, U, true>), dim3(grid), dim3(kThreads), 0, s, a);
    else
        hipLaunchKernelGGL((gf_vec_kernel<K, M, U, false>), dim3(grid), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

template <int M>
hipError_t launch_vec_generic_t(VecArgs a, unsigned grid, Mode mode, hipStream_t s) {
    if (mode == Mode::Verify)
        hipLaunchKernelGGL((gf_vec_generic_kernel<M, true>), dim3(grid), dim3(kThreads), 0, s, a);
    else
        hipLaunchKernelGGL((gf_vec_generic_kernel<M, false>), dim3(grid), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

// Vector units per lane for a shape: 2 for narrow stripes (keeps 8 x 16 B of
// loads in flight per lane), 1 for wide ones and for short shards.
int units_for(int nin, uint32_t nvec) {
    if (nvec <= uint32_t(kThreads)) return 1;
    return nin <= 4 ? 2 : 1;
}

hipError_t dispatch_vec(VecArgs a, int nout, int U, unsigned grid, Mode mode, hipStream_t s) {
#define RSAMD_CASE(K, M, UU) \
    if (a.nin == K && nout == M && U == UU) return launch_vec_t<K, M, UU>(a, grid, mode, s);
    RSAMD_CASE(4, 1, 1) RSAMD_CASE(4, 2, 1) RSAMD_CASE(4, 3, 1) RSAMD_CASE(4, 4, 1)
    RSAMD_CASE(4, 1, 2) RSAMD_CASE(4, 2, 2) RSAMD_CASE(4, 3, 2) RSAMD_CASE(4, 4, 2)
    RSAMD_CASE(10, 1, 1) RSAMD_CASE(10, 2, 1) RSAMD_CASE(10, 3, 1) RSAMD_CASE(10, 4, 1)
#undef RSAMD_CASE
    switch (nout) {
    case 1: return launch_vec_generic_t<1>(a, grid, mode, s);
    case 2: return launch_vec_generic_t<2>(a, grid, mode, s);
    case 3: return launch_vec_generic_t<3>(a, grid, mode, s);
    case 4: return launch_vec_generic_t<4>(a, grid, mode, s);
    }
    return hipErrorInvalidValue;
}

bool is_specialised(int nin) { return nin == 4 || nin == 10; }

hipError_t launch_bytes(const Geometry &g, const DevPlan &p, size_t col0, size_t ncols, Mode mode, int *mismatch,
                        hipStream_t s) {
    ByteArgs a{g.base, p.tabs, p.in_idx, p.out_idx, g.stripe_stride, g.shard_stride, col0, ncols,
               uint64_t(g.n_stripes) * ncols, p.nin, p.nout, mismatch};
    if (a.total == 0) return hipSuccess;
    const uint64_t want = (a.total + kThreads - 1) / kThreads;
    const unsigned grid = unsigned(std::min<uint64_t>(want, 65536));
    if (mode == Mode::Verify)
        hipLaunchKernelGGL((gf_byte_kernel<true>), dim3(grid), dim3(kThreads), 0, s, a);
    else
        hipLaunchKernelGGL((gf_byte_kernel<false>), dim3(grid), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_gf(const Geometry &g, const DevPlan &p, Mode mode, int *mismatch, hipStream_t s) {
    if (g.n_stripes == 0 || g.len == 0 || p.nout == 0) return hipSuccess;
    if (p.nout > kMaxOut || p.nin < 1) return hipErrorInvalidValue;
    uint8_t *base = g.base + g.col0;
    const bool aligned = (reinterpret_cast<uintptr_t>(base) % 16 == 0) && g.shard_stride % 16 == 0 &&
                         g.stripe_stride % 16 == 0;
    if (!aligned || g.len / 16 > UINT32_MAX) return launch_bytes(g, p, g.col0, g.len, mode, mismatch, s);

    const uint32_t nvec = uint32_t(g.len / 16);
    if (nvec > 0) {
        const int U = is_specialised(p.nin) ? units_for(p.nin, nvec) : 1;
        const uint32_t per_item = uint32_t(kThreads) * U;
        const uint32_t chunks = (nvec + per_item - 1) / per_item;
        // Work items are 32-bit: split very large batches by stripe ranges.
        const size_t stripes_per_launch = std::max<size_t>(1, (size_t(UINT32_MAX) / chunks));
        for (size_t t0 = 0; t0 < g.n_stripes; t0 += stripes_per_launch) {
            const size_t nst = std::min(stripes_per_launch, g.n_stripes - t0);
            VecArgs a{base + t0 * g.stripe_stride, p.tabs, p.in_idx, p.out_idx, g.stripe_stride, g.shard_stride,
                      nvec, chunks, uint32_t(nst * chunks), p.nin, mismatch};
            unsigned grid = a.n_items;
            if (max_blocks() && grid > max_blocks()) grid = max_blocks();
            hipError_t e = dispatch_vec(a, p.nout, U, grid, mode, s);
            if (e != hipSuccess) return e;
        }
    }
    const size_t tail = g.len % 16;
    if (tail) return launch_bytes(g, p, g.col0 + size_t(nvec) * 16, tail, mode, mismatch, s);
    return hipSuccess;
}

hipError_t launch_fill_synthetic(uint8_t *base, int k, size_t n_stripes, size_t shard_len, size_t shard_stride,
                                 size_t stripe_stride, uint64_t seed, uint64_t stripe0, hipStream_t s) {
    if (n_stripes == 0 || shard_len == 0) return hipSuccess;
    if (shard_len % 8 || shard_stride % 8 || stripe_stride % 8 || reinterpret_cast<uintptr_t>(base) % 8)
        return hipErrorInvalidValue;
    const uint64_t wps = shard_len / 8;
    const uint64_t wpst = wps * uint64_t(k);
    const uint64_t n = wpst * n_stripes;
    const unsigned grid = unsigned(std::min<uint64_t>((n + kThreads - 1) / kThreads, 1u << 16));
    hipLaunchKernelGGL(fill_synthetic_kernel, dim3(grid), dim3(kThreads), 0, s, base, wpst, wps, n, uint64_t(shard_stride),
                       uint64_t(stripe_stride), seed, stripe0);
    return hipGetLastError();
}

hipError_t launch_copy(uint8_t *dst, const uint8_t *src, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    size_t head = 0;
    if (reinterpret_cast<uintptr_t>(dst) % 16 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0) {
        const uint64_t nvec = n / 16;
        if (nvec) {
            const unsigned grid = unsigned(std::min<uint64_t>((nvec + kThreads - 1) / kThreads, 1u << 16));
            hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(kThreads), 0, s, reinterpret_cast<u32x4 *>(dst),
                               reinterpret_cast<const u32x4 *>(src), nvec);
        }
        head = nvec * 16;
    }
    const uint64_t rest = n - head;
    if (rest) {
        const unsigned grid = unsigned((rest + kThreads - 1) / kThreads);
        hipLaunchKernelGGL(copy_tail_kernel, dim3(grid), dim3(kThreads), 0, s, dst + head, src + head, rest);
    }
    return hipGetLastError();
}

}  // namespace rsamd
