// pattern_mem.hip -- XOR memory references for the 4+2 x 1 MiB x 4096 decode
// access patterns next to the encode's: which shards of each stripe a wave
// reads and which it writes, with the product kernels' shape (one wave per
// 1 KiB column chunk, 16-B non-temporal loads and stores) and block orders
// (plain, XCD-contiguous, 3/8-stripe rotation).  Patterns:
//   enc     read 0-3, write 4-5      dec0    read 1-4, write 0
//   dec01   read 2-5, write 0-1      dec05   read 1-4, write 0 and 5
//   rd4     read 1-4 only            wr1     write 0 only
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pattern_mem.hip -o tools/bin/pattern_mem
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
    uint32_t *sink;
    uint64_t stripe_stride, shard_stride;
    uint32_t chunks, n_items, xcd_span, rot;
};

// R0..R0+NR-1 read (consecutive shards), W0 and W1 written (W1 < 0: one output).
template <int R0, int NR, int W0, int W1>
__global__ void __launch_bounds__(64) pat_kernel(Geo a) {
    uint32_t b = blockIdx.x;
    if (a.xcd_span && b < 8u * a.xcd_span) b = (b & 7u) * a.xcd_span + (b >> 3);
    const uint32_t stripe = b / a.chunks;
    uint32_t chunk = b - stripe * a.chunks;
    if (a.rot) chunk = (chunk + stripe * a.rot) % a.chunks;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(chunk) * 1024 + threadIdx.x * 16u;
    u32x4 acc = u32x4{b, threadIdx.x, 1u, 2u};
#pragma unroll
    for (int i = 0; i < NR; ++i) acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(sb + uint64_t(R0 + i) * a.shard_stride));
    if (W0 < 0) {
        if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9E3779B9u) a.sink[threadIdx.x] = acc[0];
        return;
    }
    __builtin_nontemporal_store(acc, reinterpret_cast<u32x4 *>(sb + uint64_t(W0) * a.shard_stride));
    if (W1 >= 0) __builtin_nontemporal_store(acc + 1u, reinterpret_cast<u32x4 *>(sb + uint64_t(W1) * a.shard_stride));
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

template <int R0, int NR, int W0, int W1>
void leg(const Geo &g, int reps, const char *name, const char *order) {
    const double ms = median_ms([&] { hipLaunchKernelGGL((pat_kernel<R0, NR, W0, W1>), dim3(g.n_items), dim3(64), 0, 0, g); }, reps);
    const int shards = NR + (W0 >= 0) + (W1 >= 0);
    std::printf("4+2 1MiB x4096  %-6s %-6s %7.3f ms  %.3f of 8 TB/s\n", name, order, ms,
                double(g.n_items) * 1024.0 * shards / ms / 1e6 / 8000.0);
    std::fflush(stdout);
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    const size_t S = size_t(1) << 20, B = 4096, K = 4, M = 2;
    uint8_t *buf = nullptr;
    uint32_t *sink = nullptr;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipMalloc(&buf, B * (K + M) * S));
    CHECK(hipMalloc(&sink, 256));
    CHECK(hipMemset(buf, 0x37, B * (K + M) * S));
    const uint32_t chunks = uint32_t(S / 1024);
    static const char *orders[] = {"plain", "xcd", "rot"};
    for (int rep = 0; rep < 2; ++rep)
        for (int order = 0; order < 3; ++order) {
            Geo g{buf, sink, uint64_t((K + M) * S), uint64_t(S), chunks, uint32_t(B * chunks), 0, 0};
            if (order == 1) g.xcd_span = g.n_items / 8u;
            if (order == 2) g.rot = 3u * chunks / 8u - 1u;
            leg<0, 4, 4, 5>(g, reps, "enc", orders[order]);
            leg<1, 4, 0, -1>(g, reps, "dec0", orders[order]);
            leg<2, 4, 0, 1>(g, reps, "dec01", orders[order]);
            leg<1, 4, 0, 5>(g, reps, "dec05", orders[order]);
            leg<1, 4, -1, -1>(g, reps, "rd4", orders[order]);
            leg<0, 0, 0, -1>(g, reps, "wr1", orders[order]);
        }
    CHECK(hipFree(buf));
    return 0;
}
