// interleave_mem.hip -- is the 10+4 read/write interleaving cost a property of
// the number of concurrent streams?  XOR memory references of the encode
// (read K shards, write M) for two stripe layouts in HBM:
//   packed      [stripe][shard][S]: a wave's K+M vectors lie S bytes apart
//               (the layout every bench leg uses)
//   interleave  [stripe][granule][shard][G]: the stripe's shards are cut into
//               G-byte granules and granule g of every shard is stored
//               together, so a wave's K reads and M writes lie in one
//               (K+M)*G-byte run
// Same kernel shape as the product kernels (one wave per 1 KiB column chunk,
// 16-B non-temporal loads and stores), plain and XCD-contiguous block orders,
// warmed up.  Pools: 10+4 x 4 MiB x 128 and 4+2 x 1 MiB x 4096.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/interleave_mem.hip -o tools/bin/interleave_mem
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

struct Geo {
    uint8_t *base;
    uint64_t stripe_stride;  // bytes per stripe
    uint64_t shard_stride;   // packed: S; interleave: G
    uint64_t gran_stride;    // interleave: (K+M)*G; packed: unused
    uint32_t gran_chunks;    // 1 KiB chunks per granule (interleave)
    uint32_t chunks, n_items, xcd_span;
    int interleave;
};

template <int K, int M>
__global__ void __launch_bounds__(64) enc_kernel(Geo a) {
    uint32_t b = blockIdx.x;
    if (a.xcd_span && b < 8u * a.xcd_span) b = (b & 7u) * a.xcd_span + (b >> 3);
    const uint32_t stripe = b / a.chunks, chunk = b - stripe * a.chunks;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + threadIdx.x * 16u;
    if (a.interleave) {
        const uint32_t g = chunk / a.gran_chunks, w = chunk - g * a.gran_chunks;
        sb += uint64_t(g) * a.gran_stride + uint64_t(w) * 1024;
    } else {
        sb += uint64_t(chunk) * 1024;
    }
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(sb + uint64_t(i) * a.shard_stride));
#pragma unroll
    for (int p = 0; p < M; ++p) {
        u32x4 acc = x[0] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
        for (int i = 1; i < K; ++i) acc ^= x[i];
        __builtin_nontemporal_store(acc, reinterpret_cast<u32x4 *>(sb + uint64_t(K + p) * a.shard_stride));
    }
}

hipEvent_t e0, e1;

template <class F>
double median_ms(F launch, int reps) {
    launch();
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    for (int w = 0; w < 30; ++w) launch();
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

template <int K, int M>
void shape(uint8_t *buf, size_t S, size_t B, int reps, const char *name) {
    const uint32_t chunks = uint32_t(S / 1024);
    const double bytes = double(B) * (K + M) * S;
    for (int rep = 0; rep < 2; ++rep)
        for (size_t G : {size_t(0), size_t(1024), size_t(4096), size_t(16384), size_t(32768), size_t(65536), size_t(131072),
                          size_t(262144), size_t(524288), size_t(1) << 20, size_t(2) << 20})
            for (int order = 0; order < 2; ++order) {
                if (G >= S) continue;
                Geo g{buf, uint64_t((K + M) * S), G ? G : S, uint64_t((K + M) * G), uint32_t(G / 1024), chunks,
                      uint32_t(B * chunks), order ? uint32_t(B * chunks / 8) : 0u, G ? 1 : 0};
                const double ms = median_ms([&] { hipLaunchKernelGGL((enc_kernel<K, M>), dim3(g.n_items), dim3(64), 0, 0, g); }, reps);
                char leg[64];
                if (G) std::snprintf(leg, sizeof leg, "interleave G=%zu", G);
                else std::snprintf(leg, sizeof leg, "packed");
                std::printf("%-16s %-20s %-5s %7.3f ms  %.3f of 8 TB/s\n", name, leg, order ? "xcd" : "plain", ms,
                            bytes / ms / 1e6 / 8000.0);
                std::fflush(stdout);
            }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    const size_t cap = size_t(26) << 30;
    uint8_t *buf = nullptr;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipMalloc(&buf, cap));
    CHECK(hipMemset(buf, 0x37, cap));
    shape<10, 4>(buf, size_t(4) << 20, 128, reps, "10+4 4MiB x128");
    shape<4, 2>(buf, size_t(1) << 20, 4096, reps, "4+2 1MiB x4096");
    CHECK(hipFree(buf));
    return 0;
}
