// orderbench.hip -- does the order in which blocks walk a stripe batch change
// the HBM rate?  The production kernels map block b to (stripe b / chunks,
// chunk b % chunks): consecutive blocks are consecutive 1 KiB columns of one
// stripe.  For the BASELINE shapes that run below the 4+2 x 1 MiB rate --
// 10+4 x 4 MiB (14 streams exactly 4 MiB apart; a 4 KiB shard pad lifts it)
// and 4+2 x 4 KiB x 1 M stripes -- this sweeps the block -> (stripe, chunk)
// map with the encode kernel's access shape (one wave per block, one 16-byte
// vector per lane of every shard, non-temporal), XOR instead of the GF
// multiply so only the memory side is measured:
//   ORDER 0  stripe-major (production)
//   ORDER 1  chunk-major: block b -> stripe b % B, chunk b / B
//   ORDER 2  stripe-major with an XCD-contiguous remap (every 8th block -> one
//            contiguous eighth of the items)
//   ORDER 3  stripe-major, each stripe's chunk order rotated by rot * stripe
//   ORDER 5  XCD-contiguous remap + rotation
//   ORDER 4  stripe-major over pairs of stripes: chunk-interleaved (block b ->
//            stripe 2*(b / (2*chunks)) + b % 2, chunk (b / 2) % chunks)
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/orderbench.hip -o tools/bin/orderbench
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
    uint64_t stripe_stride, shard_stride;
    uint32_t nvec, chunks, n_items, n_stripes;
    uint32_t rot;  // ORDER 3 / 5: chunk rotation per stripe
};

template <int K, int M, int ORDER>
__global__ void __launch_bounds__(64) xor_kernel(Geo a) {
    uint32_t b = blockIdx.x, stripe, chunk;
    if (ORDER == 2 || ORDER == 5) b = (b % 8u) * (a.n_items / 8u) + b / 8u;
    if (ORDER == 1) {
        stripe = b % a.n_stripes;
        chunk = b / a.n_stripes;
    } else if (ORDER == 4) {
        stripe = 2u * (b / (2u * a.chunks)) + (b & 1u);
        chunk = (b >> 1) % a.chunks;
    } else {
        stripe = b / a.chunks;
        chunk = b - stripe * a.chunks;
        if (ORDER == 3 || ORDER == 5) chunk = uint32_t((chunk + uint64_t(a.rot) * stripe) % a.chunks);
    }
    const uint32_t v = chunk * 64u + threadIdx.x;
    if (v >= a.nvec) return;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(v) * 16;
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i)
        x[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(sb + uint64_t(i) * a.shard_stride));
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
void sweep(uint8_t *buf, size_t cap, size_t S, size_t B, size_t pad, int reps) {
    const size_t sh = S + pad;
    const size_t need = B * (K + M) * sh;
    if (need > cap || S % 1024 || B % 16) {  // never launch past the allocation
        std::printf("--- skip %d+%d S=%zu B=%zu pad=%zu (%zu > %zu bytes)\n", K, M, S, B, pad, need, cap);
        return;
    }
    const uint32_t nvec = uint32_t(S / 16), chunks = (nvec + 63) / 64;
    Geo g{buf, uint64_t((K + M) * sh), uint64_t(sh), nvec, chunks, uint32_t(B * chunks), uint32_t(B), 7};
    const double bytes = double(K + M) * S * B;
    std::printf("--- %d+%d x %zu KiB x %zu stripes, shard pad %zu B (%.1f GiB)\n", K, M, S >> 10, B, pad,
                need / 1073741824.0);
    auto line = [&](const char *name, double t) {
        std::printf("  xor %-40s %8.3f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", name, t, bytes / t / 1e6,
                    bytes / t / 1e6 / 80.0);
    };
    line("ORDER 0 stripe-major (production)",
         median_ms([&] { hipLaunchKernelGGL((xor_kernel<K, M, 0>), dim3(g.n_items), dim3(64), 0, 0, g); }, reps));
    line("ORDER 2 XCD-contiguous",
         median_ms([&] { hipLaunchKernelGGL((xor_kernel<K, M, 2>), dim3(g.n_items), dim3(64), 0, 0, g); }, reps));
    for (uint32_t rot : {1u, 3u, 7u, 31u, 127u, 509u, chunks / 2 + 1, chunks / 3 + 1}) {
        g.rot = rot % chunks;
        char name[96];
        std::snprintf(name, sizeof name, "ORDER 3 rotation %u", g.rot);
        line(name, median_ms([&] { hipLaunchKernelGGL((xor_kernel<K, M, 3>), dim3(g.n_items), dim3(64), 0, 0, g); }, reps));
        std::snprintf(name, sizeof name, "ORDER 5 XCD + rotation %u", g.rot);
        line(name, median_ms([&] { hipLaunchKernelGGL((xor_kernel<K, M, 5>), dim3(g.n_items), dim3(64), 0, 0, g); }, reps));
    }
    std::fflush(stdout);
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 7;
    const size_t cap = size_t(24) << 30;
    uint8_t *buf = nullptr;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipMalloc(&buf, cap));
    CHECK(hipMemset(buf, 0x5b, cap));
    sweep<10, 4>(buf, cap, size_t(4) << 20, 128, 0, reps);
    sweep<10, 4>(buf, cap, size_t(4) << 20, 128, 4096, reps);
    sweep<4, 2>(buf, cap, 4096, size_t(1) << 20, 0, reps);
    sweep<4, 2>(buf, cap, size_t(1) << 20, 4000, 0, reps);
    return 0;
}
