// kbench.hip -- microbenchmark of encode-kernel variants on one MI355X.
//
// Sweeps the knobs of the hot kernel (vectors per lane, non-temporal loads /
// stores, persistent vs one-shot grid) on the BASELINE config-2 shape
// (4+2 x 1 MiB x 4096 stripes, 24 GiB resident), plus pure-memory references
// with the same access pattern (XOR instead of GF multiply, and a plain copy),
// so the gap between "the kernel" and "the memory system" is visible.
// Each GF variant's parity is compared against the first variant's.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../java-.../csrc tools/kbench.hip -o kbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "gf_device.hpp"

using namespace rsamd;
using namespace rsamd::dev;

#define CHECK(x)                                                                             \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

struct Args {
    uint8_t *base;
    const uint32_t *tabs;
    uint64_t stripe_stride, shard_stride;
    uint32_t nvec, chunks, n_items;
};

enum Op { GF = 0, XOR = 1 };

template <int K, int M, int U, int BLK, bool NTL, bool NTS, int OP>
__global__ void __launch_bounds__(BLK) enc_kernel(Args a) {
    uint32_t T[M][K][5];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int p = 0; p < M; ++p)
#pragma unroll
            for (int j = 0; j < 5; ++j) T[p][i][j] = a.tabs[(i * M + p) * 5 + j];
    for (uint32_t item = blockIdx.x; item < a.n_items; item += gridDim.x) {
        const uint32_t stripe = item / a.chunks;
        const uint32_t chunk = item - stripe * a.chunks;
        uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride;
        const uint32_t v0 = chunk * uint32_t(BLK * U) + threadIdx.x;
        u32x4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t v = v0 + u * BLK;
            if (v < a.nvec) {
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const u32x4 *src = reinterpret_cast<const u32x4 *>(sb + i * a.shard_stride + uint64_t(v) * 16);
                    x[u][i] = NTL ? __builtin_nontemporal_load(src) : *src;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t v = v0 + u * BLK;
            if (v >= a.nvec) continue;
            u32x4 acc[M];
            if (OP == GF) {
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    Sel s[K];
#pragma unroll
                    for (int i = 0; i < K; ++i) s[i] = selectors(x[u][i][w]);
#pragma unroll
                    for (int p = 0; p < M; ++p) acc[p][w] = dot_dword<K>(T[p], s);
                }
            } else {
#pragma unroll
                for (int p = 0; p < M; ++p) {
                    acc[p] = x[u][0] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
                    for (int i = 1; i < K; ++i) acc[p] ^= x[u][i];
                }
            }
#pragma unroll
            for (int p = 0; p < M; ++p) {
                u32x4 *dst = reinterpret_cast<u32x4 *>(sb + (K + p) * a.shard_stride + uint64_t(v) * 16);
                if (NTS)
                    __builtin_nontemporal_store(acc[p], dst);
                else
                    *dst = acc[p];
            }
        }
    }
}


// Tables staged per input: the M*5 table dwords of input i+1 are loaded while
// input i is computed; sched_barrier fences keep the scheduler from hoisting all
// K*M*5 table loads to the top (which spills SGPRs into VGPR lanes).
template <int K, int M, int BLK, bool NTL, bool NTS>
__global__ void __launch_bounds__(BLK) enc_staged_kernel(Args a) {
    for (uint32_t item = blockIdx.x; item < a.n_items; item += gridDim.x) {
        const uint32_t stripe = item / a.chunks;
        const uint32_t chunk = item - stripe * a.chunks;
        uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride;
        const uint32_t v = chunk * uint32_t(BLK) + threadIdx.x;
        if (v >= a.nvec) continue;
        u32x4 x[K];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const u32x4 *src = reinterpret_cast<const u32x4 *>(sb + i * a.shard_stride + uint64_t(v) * 16);
            x[i] = NTL ? __builtin_nontemporal_load(src) : *src;
        }
        u32x4 acc[M];
        uint32_t Tc[M][5];
#pragma unroll
        for (int p = 0; p < M; ++p)
#pragma unroll
            for (int j = 0; j < 5; ++j) Tc[p][j] = a.tabs[p * 5 + j];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            uint32_t Tn[M][5];
            if (i + 1 < K) {
#pragma unroll
                for (int p = 0; p < M; ++p)
#pragma unroll
                    for (int j = 0; j < 5; ++j) Tn[p][j] = a.tabs[((i + 1) * M + p) * 5 + j];
            }
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const Sel s = selectors(x[i][w]);
#pragma unroll
                for (int p = 0; p < M; ++p) {
                    uint32_t t0, t1, t2;
                    terms(Tc[p], s, t0, t1, t2);
                    acc[p][w] = i == 0 ? xor3(t0, t1, t2) : xor3(acc[p][w], t0, t1) ^ t2;
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            if (i + 1 < K) {
#pragma unroll
                for (int p = 0; p < M; ++p)
#pragma unroll
                    for (int j = 0; j < 5; ++j) Tc[p][j] = Tn[p][j];
            }
        }
#pragma unroll
        for (int p = 0; p < M; ++p) {
            u32x4 *dst = reinterpret_cast<u32x4 *>(sb + (K + p) * a.shard_stride + uint64_t(v) * 16);
            if (NTS)
                __builtin_nontemporal_store(acc[p], dst);
            else
                *dst = acc[p];
        }
    }
}


template <int BLK, bool NTL, bool NTS>
__global__ void __launch_bounds__(BLK) copy_kernel(u32x4 *dst, const u32x4 *src, uint64_t nvec, int unroll_dummy) {
    const uint64_t step = uint64_t(gridDim.x) * BLK;
    for (uint64_t i = uint64_t(blockIdx.x) * BLK + threadIdx.x; i < nvec; i += step) {
        u32x4 v = NTL ? __builtin_nontemporal_load(src + i) : src[i];
        if (NTS)
            __builtin_nontemporal_store(v, dst + i);
        else
            dst[i] = v;
    }
}

__global__ void fill_kernel(uint64_t *p, uint64_t n, uint64_t seed) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

struct Ctx {
    size_t pad = 0;  // extra bytes between shards (shard_stride = S + pad)
    size_t cap = 0;  // bytes allocated at buf: every shape is checked against it on the host
    uint8_t *buf;
    uint32_t *tabs;
    size_t S, B, total;
    hipEvent_t e0, e1;
    std::vector<uint8_t> ref_parity;  // parity of stripes 0..3 and B-4..B-1 from the first GF variant
};

std::vector<uint8_t> sample_parity(Ctx &c, int K, int M) {
    std::vector<uint8_t> out;
    for (size_t t : {size_t(0), size_t(1), c.B - 2, c.B - 1}) {
        std::vector<uint8_t> h(M * c.S);
        const size_t sh = c.S + c.pad;
        for (int p = 0; p < M; ++p)
            CHECK(hipMemcpy(h.data() + p * c.S, c.buf + t * c.total * sh + (K + p) * sh, c.S, hipMemcpyDeviceToHost));
        out.insert(out.end(), h.begin(), h.end());
    }
    return out;
}

template <int K, int M, int U, int BLK, bool NTL, bool NTS, int OP>
void run_enc(Ctx &c, const char *name, unsigned grid_cap, int reps) {
    const uint32_t nvec = uint32_t(c.S / 16);
    const uint32_t per = BLK * U;
    const uint32_t chunks = (nvec + per - 1) / per;
    const uint64_t sh = c.S + c.pad;
    Args a{c.buf, c.tabs, uint64_t(c.total * sh), sh, nvec, chunks, uint32_t(c.B * chunks)};
    unsigned grid = a.n_items;
    if (grid_cap && grid > grid_cap) grid = grid_cap;
    CHECK(hipMemset(c.buf + K * c.S, 0, M * c.S));  // poison stripe 0 parity so a no-op variant shows
    hipLaunchKernelGGL((enc_kernel<K, M, U, BLK, NTL, NTS, OP>), dim3(grid), dim3(BLK), 0, 0, a);
    CHECK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(c.e0, 0));
        hipLaunchKernelGGL((enc_kernel<K, M, U, BLK, NTL, NTS, OP>), dim3(grid), dim3(BLK), 0, 0, a);
        CHECK(hipEventRecord(c.e1, 0));
        CHECK(hipEventSynchronize(c.e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, c.e0, c.e1));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double ms = ts[ts.size() / 2];
    const double bytes = double(K + M) * c.S * c.B;
    const char *ok = "-";
    if (OP == GF) {
        auto p = sample_parity(c, K, M);
        if (c.ref_parity.empty()) c.ref_parity = p;
        ok = (p == c.ref_parity) ? "ok" : "MISMATCH";
    }
    std::printf("%-44s pad=%6zu  %8.3f ms  %7.1f GB/s  %5.1f%% of 8 TB/s  %s\n", name, c.pad, ms, bytes / ms / 1e6,
                bytes / ms / 1e6 / 80.0, ok);
    std::fflush(stdout);
}


template <int K, int M, int BLK, bool NTL, bool NTS>
void run_staged(Ctx &c, const char *name, int reps) {
    const uint32_t nvec = uint32_t(c.S / 16);
    const uint32_t chunks = (nvec + BLK - 1) / BLK;
    const uint64_t sh = c.S + c.pad;
    Args a{c.buf, c.tabs, uint64_t(c.total * sh), sh, nvec, chunks, uint32_t(c.B * chunks)};
    const unsigned grid = a.n_items;
    CHECK(hipMemset(c.buf + K * c.S, 0, M * c.S));
    hipLaunchKernelGGL((enc_staged_kernel<K, M, BLK, NTL, NTS>), dim3(grid), dim3(BLK), 0, 0, a);
    CHECK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(c.e0, 0));
        hipLaunchKernelGGL((enc_staged_kernel<K, M, BLK, NTL, NTS>), dim3(grid), dim3(BLK), 0, 0, a);
        CHECK(hipEventRecord(c.e1, 0));
        CHECK(hipEventSynchronize(c.e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, c.e0, c.e1));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double ms = ts[ts.size() / 2];
    const double bytes = double(K + M) * c.S * c.B;
    auto p = sample_parity(c, K, M);
    if (c.ref_parity.empty()) c.ref_parity = p;
    std::printf("%-44s pad=%6zu  %8.3f ms  %7.1f GB/s  %5.1f%% of 8 TB/s  %s\n", name, c.pad, ms, bytes / ms / 1e6,
                bytes / ms / 1e6 / 80.0, p == c.ref_parity ? "ok" : "MISMATCH");
    std::fflush(stdout);
}

// Same shape, loads/stores through buffer intrinsics with explicit cache-policy
// bits (gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16).
template <int K, int M, int LAUX, int SAUX>
__global__ void __launch_bounds__(64) enc_buf_kernel(Args a) {
    uint32_t T[M][K][5];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int p = 0; p < M; ++p)
#pragma unroll
            for (int j = 0; j < 5; ++j) T[p][i][j] = a.tabs[(i * M + p) * 5 + j];
    const uint32_t item = blockIdx.x;
    const uint32_t stripe = item / a.chunks;
    const uint32_t v = (item - stripe * a.chunks) * 64u + threadIdx.x;
    if (v >= a.nvec) return;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(sb, 0, 0x7fffffff, 0x00020000);
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const uint32_t off = uint32_t(i * a.shard_stride + uint64_t(v) * 16);
        x[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, LAUX));
    }
    u32x4 acc[M];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        Sel s[K];
#pragma unroll
        for (int i = 0; i < K; ++i) s[i] = selectors(x[i][w]);
#pragma unroll
        for (int p = 0; p < M; ++p) acc[p][w] = dot_dword<K>(T[p], s);
    }
#pragma unroll
    for (int p = 0; p < M; ++p) {
        const uint32_t off = uint32_t((K + p) * a.shard_stride + uint64_t(v) * 16);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, acc[p]), rs, off, 0, SAUX);
    }
}

template <int K, int M, int LAUX, int SAUX>
void run_buf(Ctx &c, const char *name, int reps) {
    const uint32_t nvec = uint32_t(c.S / 16);
    const uint32_t chunks = (nvec + 63) / 64;
    const uint64_t sh = c.S + c.pad;
    Args a{c.buf, c.tabs, uint64_t(c.total * sh), sh, nvec, chunks, uint32_t(c.B * chunks)};
    hipLaunchKernelGGL((enc_buf_kernel<K, M, LAUX, SAUX>), dim3(a.n_items), dim3(64), 0, 0, a);
    CHECK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(c.e0, 0));
        hipLaunchKernelGGL((enc_buf_kernel<K, M, LAUX, SAUX>), dim3(a.n_items), dim3(64), 0, 0, a);
        CHECK(hipEventRecord(c.e1, 0));
        CHECK(hipEventSynchronize(c.e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, c.e0, c.e1));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double ms = ts[ts.size() / 2];
    const double bytes = double(K + M) * c.S * c.B;
    auto p = sample_parity(c, K, M);
    if (c.ref_parity.empty()) c.ref_parity = p;
    std::printf("%-44s pad=%6zu  %8.3f ms  %7.1f GB/s  %5.1f%% of 8 TB/s  %s\n", name, c.pad, ms, bytes / ms / 1e6,
                bytes / ms / 1e6 / 80.0, p == c.ref_parity ? "ok" : "MISMATCH");
    std::fflush(stdout);
}

template <int BLK, bool NTL, bool NTS>
void run_copy(Ctx &c, const char *name, unsigned grid, int reps) {
    const size_t n = c.B * c.total * c.S / 2;
    const uint64_t nvec = n / 16;
    std::vector<float> ts;
    for (int r = 0; r < reps + 1; ++r) {
        CHECK(hipEventRecord(c.e0, 0));
        hipLaunchKernelGGL((copy_kernel<BLK, NTL, NTS>), dim3(grid), dim3(BLK), 0, 0,
                           reinterpret_cast<u32x4 *>(c.buf + n), reinterpret_cast<const u32x4 *>(c.buf), nvec, 0);
        CHECK(hipEventRecord(c.e1, 0));
        CHECK(hipEventSynchronize(c.e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, c.e0, c.e1));
        if (r) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double ms = ts[ts.size() / 2];
    std::printf("%-44s grid=%8u  %8.3f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", name, grid, ms, 2.0 * n / ms / 1e6,
                2.0 * n / ms / 1e6 / 80.0);
    std::fflush(stdout);
}

bool setup_shape(Ctx &c, int K, int M, size_t S, size_t B) {
    const size_t need = B * size_t(K + M) * (S + c.pad);
    if (need > c.cap || size_t(K) * M * 20 > 64 * 1024) {  // never launch past the allocation
        std::printf("--- skip %d+%d S=%zu B=%zu pad=%zu: needs %zu bytes > %zu allocated\n", K, M, S, B, c.pad, need,
                    c.cap);
        return false;
    }
    c.S = S;
    c.B = B;
    c.total = K + M;
    c.ref_parity.clear();
    const size_t bytes = c.B * c.total * (c.S + c.pad);
    hipLaunchKernelGGL(fill_kernel, dim3(65536), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(c.buf), bytes / 8,
                       0x5EEDull + K);
    GfMatrix g = build_generator(K, K + M);
    std::vector<uint32_t> tabs;
    for (int i = 0; i < K; ++i)
        for (int p = 0; p < M; ++p) {
            PermTable t = perm_table(g.at(K + p, i));
            tabs.insert(tabs.end(), {t.t0lo, t.t0hi, t.t1lo, t.t1hi, t.t2});
        }
    CHECK(hipMemcpy(c.tabs, tabs.data(), tabs.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipDeviceSynchronize());
    std::printf("--- %d+%d x %zu KiB x %zu stripes (%.1f GiB)\n", K, M, S >> 10, B, bytes / 1073741824.0);
    return true;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 7;
    Ctx c;
    c.cap = size_t(24) << 30;
    CHECK(hipMalloc(&c.buf, c.cap));
    CHECK(hipMalloc(&c.tabs, 64 * 1024));
    CHECK(hipEventCreate(&c.e0));
    CHECK(hipEventCreate(&c.e1));

    for (size_t pad : {size_t(0), size_t(512), size_t(1024), size_t(2048), size_t(4096), size_t(8192),
                       size_t(12288), size_t(16384), size_t(65536)}) {
        c.pad = pad;
        if (!setup_shape(c, 10, 4, size_t(4) << 20, 120)) continue;
        run_enc<10, 4, 1, 64, true, true, GF>(c, "gf 10+4 staged? (enc_kernel) B64", 0, reps);
        run_staged<10, 4, 64, true, true>(c, "staged 10+4 B64", reps);
    }
    for (size_t pad : {size_t(0), size_t(256), size_t(512), size_t(1024), size_t(2048), size_t(4096)}) {
        c.pad = pad;
        if (!setup_shape(c, 4, 2, 4096, 900000)) continue;
        run_enc<4, 2, 1, 64, true, true, GF>(c, "gf 4+2 4KiB B64", 0, reps);
    }
    for (size_t pad : {size_t(0), size_t(2048), size_t(8192), size_t(16384)}) {
        c.pad = pad;
        if (!setup_shape(c, 4, 2, size_t(1) << 20, 3900)) continue;
        run_enc<4, 2, 1, 64, true, true, GF>(c, "gf 4+2 1MiB B64", 0, reps);
    }
    return 0;
}
