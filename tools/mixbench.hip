// mixbench.hip -- how far is the 4+2 encode from what HBM gives its access
// pattern?  One run, one 24 GiB buffer (the BASELINE config-2 footprint), all
// kernels in the encode kernel's shape (one wave per block, one 16-byte vector
// per lane, non-temporal loads and stores, one-shot grid):
//   rd1 / wr1 / cp1   read-only, write-only, copy: one contiguous stream
//   rd4               read-only over the 4 data shards of each stripe (4
//                     streams 1 MiB apart, the encode's read side alone)
//   wr2               write-only over the 2 parity shards (its write side alone)
//   xor42             4+2 with XOR instead of the GF multiply (memory reference)
//   gf42              the production-shaped 4+2 encode
//   gf42x             gf42 with an XCD-contiguous blockIdx remap (the XCD that
//                     gets every 8th block codes one contiguous eighth)
//   xor42r            xor42 with the 4 loads issued in a per-wave rotated order
//   gf42p1 / gf42p3   gf42 at wave priority 1 / 3 until its loads are issued
// plus the additive model R / rate(rd4) + W / rate(wr2) for the encode.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ijava-reed-solomon-distributed-file-system_amd/csrc \
//          tools/mixbench.hip java-reed-solomon-distributed-file-system_amd/csrc/gf256.cpp -o tools/bin/mixbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gf256.hpp"
#include "gf_device.hpp"

using namespace rsamd;
using namespace rsamd::dev;

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e = (x);                                                                       \
        if (e != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

constexpr int K = 4, M = 2;
constexpr uint32_t kMagic = 0x9E3779B9u;

struct Geo {
    uint8_t *base;
    const uint32_t *tabs;  // [K][M][5]
    uint32_t *sink;
    uint64_t stripe_stride, shard_stride;
    uint32_t nvec, chunks, n_items;
};

__device__ __forceinline__ u32x4 ld(const uint8_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}
__device__ __forceinline__ void st(uint8_t *p, const u32x4 &v) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
}

// One contiguous stream: OP 0 read, 1 write, 2 copy (first half -> second half).
template <int OP>
__global__ void __launch_bounds__(64) flat_kernel(uint8_t *p, uint64_t nvec, uint32_t *sink) {
    const uint64_t i = uint64_t(blockIdx.x) * 64 + threadIdx.x;
    if (i >= nvec) return;
    if (OP == 0) {
        const u32x4 v = ld(p + i * 16);
        const uint32_t x = v[0] ^ v[1] ^ v[2] ^ v[3];
        if (x == kMagic) sink[threadIdx.x] = x;
    } else if (OP == 1) {
        const uint32_t a = uint32_t(i);
        st(p + i * 16, u32x4{a, a ^ 1u, a ^ 2u, a ^ 3u});
    } else {
        st(p + (nvec + i) * 16, ld(p + i * 16));
    }
}

// Stripe-shaped kernels.  OP: 0 rd4, 1 wr2, 2 xor42, 3 gf42.  XCD: remap
// blockIdx so XCD x (blocks x, x+8, ...) codes items [x*n/8, (x+1)*n/8).
// ROT (XOR only): the 4 loads are issued starting at shard (item % 4).
template <int OP, bool XCD, bool ROT, int PRIO = 0>
__global__ void __launch_bounds__(64) stripe_kernel(Geo a) {
    // Tables first: s_setprio counts as a memory clobber, so loads placed
    // after it could no longer be scalar loads.
    uint32_t T[M][K][5];
    if (OP == 3) {
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int p = 0; p < M; ++p)
#pragma unroll
                for (int j = 0; j < 5; ++j) T[p][i][j] = a.tabs[(i * M + p) * 5 + j];
    }
    if (PRIO) __builtin_amdgcn_s_setprio(PRIO);  // issue this wave's loads ahead of computing waves
    uint32_t item = blockIdx.x;
    if (XCD) item = (item % 8u) * (a.n_items / 8u) + item / 8u;
    const uint32_t stripe = item / a.chunks;
    const uint32_t v = (item - stripe * a.chunks) * 64u + threadIdx.x;
    if (v >= a.nvec) return;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(v) * 16;
    if (OP == 1) {
        const uint32_t t = item * 64u + threadIdx.x;
#pragma unroll
        for (int p = 0; p < M; ++p) st(sb + uint64_t(K + p) * a.shard_stride, u32x4{t, t + 1u, t + 2u, uint32_t(p)});
        return;
    }
    u32x4 x[K];
    if (ROT) {  // XOR only (commutative): x[j] holds shard (j + r) % 4
        const uint32_t r = item % 4u;
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = ld(sb + uint64_t((j + r) % 4u) * a.shard_stride);
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = ld(sb + uint64_t(i) * a.shard_stride);
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    if (OP == 0) {
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < K; ++i) s ^= x[i][0] ^ x[i][1] ^ x[i][2] ^ x[i][3];
        if (s == kMagic) a.sink[threadIdx.x] = s;
        return;
    }
    u32x4 acc[M];
    if (OP == 2) {
#pragma unroll
        for (int p = 0; p < M; ++p) {
            acc[p] = x[0] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
            for (int i = 1; i < K; ++i) acc[p] ^= x[i];
        }
    } else {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            Sel s[K];
#pragma unroll
            for (int i = 0; i < K; ++i) s[i] = selectors(x[i][w]);
#pragma unroll
            for (int p = 0; p < M; ++p) acc[p][w] = dot_dword<K>(T[p], s);
        }
    }
#pragma unroll
    for (int p = 0; p < M; ++p) st(sb + uint64_t(K + p) * a.shard_stride, acc[p]);
}

hipEvent_t e0, e1;

template <class F>
double median_ms(F launch, int reps) {
    launch();
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(e0, 0));
        launch();
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

void report(const char *name, double bytes, double ms) {
    std::printf("%-44s %12.0f B  %8.3f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", name, bytes, ms, bytes / ms / 1e6,
                bytes / ms / 1e6 / 80.0);
    std::fflush(stdout);
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 9;
    const size_t S = size_t(1) << 20, B = 4096;
    const size_t total = B * (K + M) * S;  // 24 GiB
    uint8_t *buf = nullptr;
    uint32_t *sink = nullptr, *tabs = nullptr;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipMalloc(&buf, total));
    CHECK(hipMalloc(&sink, 256));
    CHECK(hipMalloc(&tabs, 4096));
    CHECK(hipMemset(buf, 0x37, total));
    {
        GfMatrix g = build_generator(K, K + M);
        std::vector<uint32_t> t;
        for (int i = 0; i < K; ++i)
            for (int p = 0; p < M; ++p) {
                const PermTable pt = perm_table(g.at(K + p, i));
                t.insert(t.end(), {pt.t0lo, pt.t0hi, pt.t1lo, pt.t1hi, pt.t2});
            }
        if (t.size() * 4 > 4096) return 1;
        CHECK(hipMemcpy(tabs, t.data(), t.size() * 4, hipMemcpyHostToDevice));
    }
    std::printf("--- one MI355X, %zu GiB buffer (4+2 x 1 MiB x %zu stripes), median of %d\n", total >> 30, B, reps);

    const uint64_t nvec = total / 16;  // all launches stay inside [buf, buf + total)
    const double t_rd1 = median_ms([&] { hipLaunchKernelGGL(flat_kernel<0>, dim3(unsigned(nvec / 64)), dim3(64), 0, 0, buf, nvec, sink); }, reps);
    report("rd1  read-only, 1 stream", double(total), t_rd1);
    const double t_wr1 = median_ms([&] { hipLaunchKernelGGL(flat_kernel<1>, dim3(unsigned(nvec / 64)), dim3(64), 0, 0, buf, nvec, sink); }, reps);
    report("wr1  write-only, 1 stream", double(total), t_wr1);
    const uint64_t half = nvec / 2;
    const double t_cp1 = median_ms([&] { hipLaunchKernelGGL(flat_kernel<2>, dim3(unsigned(half / 64)), dim3(64), 0, 0, buf, half, sink); }, reps);
    report("cp1  copy 1:1", double(total), t_cp1);

    const uint32_t nv = uint32_t(S / 16), chunks = (nv + 63) / 64;
    const Geo g{buf, tabs, sink, uint64_t((K + M) * S), uint64_t(S), nv, chunks, uint32_t(B * chunks)};
    const dim3 grid(g.n_items);
    const double R = double(B) * K * S, W = double(B) * M * S;
    const double t_rd4 = median_ms([&] { hipLaunchKernelGGL((stripe_kernel<0, false, false>), grid, dim3(64), 0, 0, g); }, reps);
    report("rd4  read 4 data shards per stripe", R, t_rd4);
    const double t_wr2 = median_ms([&] { hipLaunchKernelGGL((stripe_kernel<1, false, false>), grid, dim3(64), 0, 0, g); }, reps);
    report("wr2  write 2 parity shards per stripe", W, t_wr2);
    const double t_x = median_ms([&] { hipLaunchKernelGGL((stripe_kernel<2, false, false>), grid, dim3(64), 0, 0, g); }, reps);
    report("xor42 (memory reference)", R + W, t_x);
    const double t_g = median_ms([&] { hipLaunchKernelGGL((stripe_kernel<3, false, false>), grid, dim3(64), 0, 0, g); }, reps);
    report("gf42  encode", R + W, t_g);
    const double t_gx = median_ms([&] { hipLaunchKernelGGL((stripe_kernel<3, true, false>), grid, dim3(64), 0, 0, g); }, reps);
    report("gf42x encode, XCD-contiguous items", R + W, t_gx);
    const double t_xr = median_ms([&] { hipLaunchKernelGGL((stripe_kernel<2, false, true>), grid, dim3(64), 0, 0, g); }, reps);
    report("xor42r memory reference, rotated load order", R + W, t_xr);
    const double t_p1 = median_ms([&] { hipLaunchKernelGGL((stripe_kernel<3, false, false, 1>), grid, dim3(64), 0, 0, g); }, reps);
    report("gf42p1 encode, setprio 1 while issuing loads", R + W, t_p1);
    const double t_p3 = median_ms([&] { hipLaunchKernelGGL((stripe_kernel<3, false, false, 3>), grid, dim3(64), 0, 0, g); }, reps);
    report("gf42p3 encode, setprio 3 while issuing loads", R + W, t_p3);
    const double t_g2 = median_ms([&] { hipLaunchKernelGGL((stripe_kernel<3, false, false>), grid, dim3(64), 0, 0, g); }, reps);
    report("gf42  encode (again, drift check)", R + W, t_g2);
    report("model: rd4 time + wr2 time", R + W, t_rd4 + t_wr2);
    report("model: R/rate(rd1) + W/rate(wr1)", R + W, R / (total / t_rd1) + W / (total / t_wr1));
    return 0;
}
