// HBM ceiling by read/write mix: a kernel in the product
// kernels' shape (kernels.hip gf_vec_kernel: one-wave workgroups, one 16-byte
// vector per lane per shard, a one-shot grid, non-temporal loads and stores,
// the XCD block remap, an occupancy cap through dynamic LDS) over stripes of
// R input and W output shards of 1 MiB; each output is the XOR of the inputs
// and its index (no GF arithmetic: the probe prices the traffic alone).
// Prints one JSON line per (R, W, pad): the algorithmic bytes over the mean
// HIP-event launch time, and the fraction of 8 TB/s.
//
//   hipcc --offload-arch=gfx950 -O3 -I java-reed-solomon-distributed-file-system_amd/csrc -o /tmp/mix_probe tools/mix_probe.hip
//   /tmp/mix_probe [GiB per launch, default 24] [f: the file-encode variants only | s: by size]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "gf_device.hpp"

namespace {

constexpr int kWave = 64;
constexpr uint64_t kShard = uint64_t(1) << 20;
constexpr uint32_t kChunks = uint32_t(kShard / 16 / kWave);  // workgroups per stripe

using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

// PLANAR: the fused file encode's streams (layout.hip file_encode_kernel) --
// the inputs read from one file of 1 KiB blocks dealt round-robin over the R
// input shards (a wave reads the whole R KiB block row), each output one
// region of `plane` bytes (the shard arrays, a shard stride apart) -- instead
// of 1 MiB shards in stripes.
// LOAD8: two plain 8-byte loads per lane and stream (layout.hip IO_PLAIN8).
template <int R, int W, bool PLANAR, bool LOAD8>
__global__ void __launch_bounds__(kWave) mix_kernel(uint8_t *base, uint32_t xcd_span, uint64_t plane) {
    uint32_t b = blockIdx.x;
    if (xcd_span && b < 8u * xcd_span) b = (b & 7u) * xcd_span + (b >> 3);
    const uint32_t stripe = b / kChunks, chunk = b % kChunks;
    // PLANAR: vector v of shard s is file bytes [(b * R + s) * 1024 + 16 lane, +16), outputs after the file
    uint8_t *sb = PLANAR ? base + uint64_t(b) * R * 1024 + threadIdx.x * 16
                         : base + uint64_t(stripe) * (R + W) * kShard + (uint64_t(chunk) * kWave + threadIdx.x) * 16;
    uint8_t *ob = PLANAR ? base + (uint64_t(b) * kWave + threadIdx.x) * 16 : sb;  // output w at ob + (R + w) * plane
    const uint64_t step = PLANAR ? 1024 : kShard, ostep = PLANAR ? plane : kShard;
    u32x4 acc = u32x4{0u, 0u, 0u, 0u};
    u32x4 x[R > 0 ? R : 1];
#pragma unroll
    for (int s = 0; s < R; ++s) {
        if (LOAD8) {
            using u32x2 = __attribute__((ext_vector_type(2))) uint32_t;
            const u32x2 lo = *reinterpret_cast<const u32x2 *>(sb + s * step);
            const u32x2 hi = *reinterpret_cast<const u32x2 *>(sb + s * step + 8);
            x[s] = u32x4{lo.x, lo.y, hi.x, hi.y};
        } else {
            x[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(sb + s * step));
        }
    }
#pragma unroll
    for (int s = 0; s < R; ++s) acc ^= x[s];
    if (W == 0) {  // read-only: keep the loads alive
        if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) *reinterpret_cast<u32x4 *>(sb) = acc;
    }
#pragma unroll
    for (int w = 0; w < W; ++w)
        __builtin_nontemporal_store(acc ^ u32x4{uint32_t(w), 0u, 0u, 0u},
                                    reinterpret_cast<u32x4 *>(ob + uint64_t(R + w) * ostep));
}

// The fused file encode itself at 1 KiB blocks (layout.hip file_encode_kernel
// with the geometry taken out): 4 inputs from the file, the 4 data shards
// written back out, 2 parity shards.  GF: the parity through the product's
// GF(2^8) fold (gf_device.hpp, tables as scalar loads first), else XORs.
// STORE_FIRST: the data shards stored before the parity is computed (the
// product's order), else every store after the compute.
template <bool GF, bool STORE_FIRST, bool LOAD8>
__global__ void __launch_bounds__(kWave) file_probe_kernel(uint8_t *base, uint32_t xcd_span, uint64_t plane,
                                                           const uint32_t *tabs) {
    constexpr int K = 4, M = 2;
    uint32_t b = blockIdx.x;
    if (xcd_span && b < 8u * xcd_span) b = (b & 7u) * xcd_span + (b >> 3);
    const uint8_t *fb = base + uint64_t(b) * K * 1024 + threadIdx.x * 16;
    uint8_t *ob = base + uint64_t(K) * plane + (uint64_t(b) * kWave + threadIdx.x) * 16;
    uint32_t T[M][K][5];
    if (GF) {
#pragma unroll
        for (int p = 0; p < M; ++p)
#pragma unroll
            for (int i = 0; i < K; ++i)
#pragma unroll
                for (int j = 0; j < 5; ++j) T[p][i][j] = tabs[(i * M + p) * 5 + j];
    }
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        if (LOAD8) {
            using u32x2 = __attribute__((ext_vector_type(2))) uint32_t;
            const u32x2 lo = *reinterpret_cast<const u32x2 *>(fb + i * 1024);
            const u32x2 hi = *reinterpret_cast<const u32x2 *>(fb + i * 1024 + 8);
            x[i] = u32x4{lo.x, lo.y, hi.x, hi.y};
        } else {
            x[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(fb + i * 1024));
        }
    }
    if (STORE_FIRST) {
#pragma unroll
        for (int i = 0; i < K; ++i) __builtin_nontemporal_store(x[i], reinterpret_cast<u32x4 *>(ob + uint64_t(i) * plane));
    }
    u32x4 acc[M];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        if (GF) {
            rsamd::dev::Sel sl[K];
#pragma unroll
            for (int i = 0; i < K; ++i) sl[i] = rsamd::dev::selectors(x[i][w]);
#pragma unroll
            for (int p = 0; p < M; ++p) acc[p][w] = rsamd::dev::dot_dword<K>(T[p], sl);
        } else {
#pragma unroll
            for (int p = 0; p < M; ++p) acc[p][w] = x[0][w] ^ x[1][w] ^ x[2][w] ^ (x[3][w] + uint32_t(p));
        }
    }
    if (!STORE_FIRST) {
#pragma unroll
        for (int i = 0; i < K; ++i) __builtin_nontemporal_store(x[i], reinterpret_cast<u32x4 *>(ob + uint64_t(i) * plane));
    }
#pragma unroll
    for (int p = 0; p < M; ++p) __builtin_nontemporal_store(acc[p], reinterpret_cast<u32x4 *>(ob + uint64_t(K + p) * plane));
}

template <bool GF, bool STORE_FIRST, bool LOAD8>
void run_file(uint8_t *buf, uint64_t total_bytes, const uint32_t *tabs) {
    const uint64_t plane = total_bytes / (10 * kShard) * kShard;
    const uint32_t grid = uint32_t(plane / 1024);
    for (size_t pad : {size_t(0), size_t(10240), size_t(11520), size_t(12544), size_t(14848)}) {
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        for (int i = 0; i < 3; ++i) file_probe_kernel<GF, STORE_FIRST, LOAD8><<<grid, kWave, pad>>>(buf, grid / 8u, plane, tabs);
        CHECK(hipGetLastError());
        const int reps = 10;
        CHECK(hipEventRecord(a));
        for (int i = 0; i < reps; ++i) file_probe_kernel<GF, STORE_FIRST, LOAD8><<<grid, kWave, pad>>>(buf, grid / 8u, plane, tabs);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double bytes = 10.0 * double(plane), s = ms / 1e3 / reps;
        std::printf("{\"file_encode\": 1, \"gf\": %d, \"store_first\": %d, \"load8\": %d, \"lds_pad\": %zu, "
                    "\"bytes\": %.0f, \"ms\": %.4f, \"frac\": %.4f}\n",
                    int(GF), int(STORE_FIRST), int(LOAD8), pad, bytes, s * 1e3, bytes / s / 8e12);
        std::fflush(stdout);
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
    }
}

template <int R, int W, bool PLANAR = false, bool LOAD8 = false>
void run(uint8_t *buf, uint64_t total_bytes, size_t pad) {
    const uint64_t stripes = total_bytes / (uint64_t(R + W) * kShard);
    const uint32_t grid = uint32_t(stripes * kChunks);
    const uint64_t plane = stripes * kShard;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) mix_kernel<R, W, PLANAR, LOAD8><<<grid, kWave, pad>>>(buf, grid / 8u, plane);
    CHECK(hipGetLastError());
    const int reps = 10;
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) mix_kernel<R, W, PLANAR, LOAD8><<<grid, kWave, pad>>>(buf, grid / 8u, plane);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double bytes = double(R + W) * double(stripes) * double(kShard), s = ms / 1e3 / reps;
    std::printf("{\"reads\": %d, \"writes\": %d, \"planar\": %d, \"load8\": %d, \"lds_pad\": %zu, \"stripes\": %llu, "
                "\"ms\": %.4f, \"TBps\": %.3f, \"frac\": %.4f}\n",
                R, W, int(PLANAR), int(LOAD8), pad, (unsigned long long)stripes, s * 1e3, bytes / s / 1e12, bytes / s / 8e12);
    std::fflush(stdout);
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
}

template <int R, int W, bool PLANAR = false, bool LOAD8 = false>
void sweep(uint8_t *buf, uint64_t total) {
    for (size_t pad : {size_t(0), size_t(10240), size_t(12544), size_t(14848)}) run<R, W, PLANAR, LOAD8>(buf, total, pad);
}

}  // namespace

int main(int argc, char **argv) {
    const double gib = argc > 1 ? std::atof(argv[1]) : 24.0;
    const uint64_t total = uint64_t(gib * double(uint64_t(1) << 30));
    uint8_t *buf = nullptr;
    CHECK(hipMalloc(&buf, total));
    CHECK(hipMemset(buf, 0x5a, total));
    CHECK(hipDeviceSynchronize());
    uint32_t *tabs = nullptr;
    CHECK(hipMalloc(&tabs, 40 * sizeof(uint32_t)));
    {
        uint32_t h[40];
        for (int i = 0; i < 40; ++i) h[i] = 0x9e3779b9u * uint32_t(i + 1);
        CHECK(hipMemcpy(tabs, h, sizeof h, hipMemcpyHostToDevice));
    }
    if (argc > 2 && argv[2][0] == 'f') {  // the file-encode variants only
        run_file<false, false, false>(buf, total, tabs);
        run_file<false, true, false>(buf, total, tabs);
        run_file<true, false, false>(buf, total, tabs);
        run_file<true, true, false>(buf, total, tabs);
        run_file<true, true, true>(buf, total, tabs);
        run_file<true, false, true>(buf, total, tabs);
        return 0;
    }
    if (argc > 2 && argv[2][0] == 's') {  // the GF file encode by bytes per launch, in the one allocation
        for (double w : {2.5, 5.0, 10.0, 15.0, 20.0, 24.0})
            if (w <= gib) run_file<true, true, true>(buf, uint64_t(w * double(uint64_t(1) << 30)), tabs);
        return 0;
    }
    sweep<1, 0>(buf, total);
    sweep<0, 1>(buf, total);
    sweep<1, 1>(buf, total);
    sweep<4, 2>(buf, total);
    sweep<4, 4>(buf, total);
    sweep<4, 5>(buf, total);
    sweep<4, 6>(buf, total);
    sweep<10, 4>(buf, total);
    sweep<4, 6, true>(buf, total);
    sweep<4, 6, true, true>(buf, total);
    sweep<4, 6, false, true>(buf, total);
    sweep<4, 2, true>(buf, total);
    CHECK(hipFree(buf));
    return 0;
}
