// file_granule_mem.hip -- the fused file kernels' access pattern (row f1)
// with the shards packed (1 GiB apart for a 4 GiB file) or in the granule
// layout (include/rs_amd.h: granule g of every shard stored together).  XOR
// reference kernels in the product kernels' shape: a wave takes one 1 KiB
// column chunk, reads the K KiB of the file that hold it (the 1000-B block
// interleave simplified to 1 KiB blocks) and writes K data + M parity KiB
// (encode), or reads K shards' KiB and writes the K KiB of file (decode).
// XCD-contiguous block order, warmed up.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/file_granule_mem.hip -o tools/bin/file_granule_mem
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e = (x);                                                                       \
        if (e != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld(const uint8_t *p) { return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p)); }
__device__ __forceinline__ void st(uint8_t *p, const u32x4 &v) { __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p)); }

// Shard s, column c: packed (G == 0) s*S + c; granule (c/G)*nsh*G + s*G + c%G.
__device__ __forceinline__ uint64_t shard_addr(uint64_t c, int s, uint64_t S, uint64_t G, int nsh) {
    return G ? (c / G) * nsh * G + uint64_t(s) * G + c % G : uint64_t(s) * S + c;
}

template <int K, int M, bool DEC>
__global__ void __launch_bounds__(64) file_kernel(const uint8_t *file, uint8_t *fout, uint8_t *shards, uint64_t S,
                                                  uint64_t G, uint32_t xcd_span) {
    uint32_t b = blockIdx.x;
    if (xcd_span && b < 8u * xcd_span) b = (b & 7u) * xcd_span + (b >> 3);
    const uint64_t c = uint64_t(b) * 1024 + threadIdx.x * 16u;
    const uint64_t f = uint64_t(b) * 1024 * K + threadIdx.x * 16u;
    u32x4 x[K];
    if (!DEC) {
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = ld(file + f + i * 1024);
#pragma unroll
        for (int i = 0; i < K; ++i) st(shards + shard_addr(c, i, S, G, K + M), x[i]);
#pragma unroll
        for (int p = 0; p < M; ++p) {
            u32x4 acc = x[0] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
            for (int i = 1; i < K; ++i) acc ^= x[i];
            st(shards + shard_addr(c, K + p, S, G, K + M), acc);
        }
    } else {  // survivors 1..K (shard 0 missing), written back as file blocks
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = ld(shards + shard_addr(c, i + 1, S, G, K + M));
#pragma unroll
        for (int i = 0; i < K; ++i) st(fout + f + i * 1024, x[i]);
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    constexpr int K = 4, M = 2;
    const size_t F = size_t(4) << 30, S = F / K;
    uint8_t *file = nullptr, *fout = nullptr, *sh = nullptr;
    CHECK(hipMalloc(&file, F));
    CHECK(hipMalloc(&fout, F));
    CHECK(hipMalloc(&sh, (K + M) * S));
    CHECK(hipMemset(file, 0x11, F));
    CHECK(hipMemset(sh, 0x22, (K + M) * S));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const uint32_t n = uint32_t(S / 1024);
    for (int rep = 0; rep < 2; ++rep)
        for (size_t G : {size_t(0), size_t(16384), size_t(32768), size_t(65536), size_t(262144)})
            for (int dec = 0; dec < 2; ++dec) {
                auto launch = [&] {
                    if (dec) hipLaunchKernelGGL((file_kernel<K, M, true>), dim3(n), dim3(64), 0, 0, file, fout, sh, S, G, n / 8);
                    else hipLaunchKernelGGL((file_kernel<K, M, false>), dim3(n), dim3(64), 0, 0, file, fout, sh, S, G, n / 8);
                };
                for (int w = 0; w < 30; ++w) launch();
                CHECK(hipGetLastError());
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
                const double ms = ts[ts.size() / 2];
                const double bytes = dec ? double(F) + K * double(S) : double(F) + (K + M) * double(S);
                std::printf("file 4 GiB %s shards %-8s %-7zu %7.3f ms  %.3f of 8 TB/s\n", dec ? "decode" : "encode",
                            G ? "granule" : "packed", G, ms, bytes / ms / 1e6 / 8000.0);
                std::fflush(stdout);
            }
    return 0;
}
