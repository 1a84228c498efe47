// skew_mem.hip -- packed 10+4 x 4 MiB stripes: can a workgroup-level shard
// skew through LDS recover what a per-shard pad recovers?
//
// The packed layout's shards sit a power of two apart (4 MiB), so the K loads
// a wave issues at one column hit the same address bits; the same batch with
// every shard 4 KiB further on codes 3-4 points faster under the occupancy
// caps (bench cfg3_10p4_4MiB_x128_pad4K).  XOR-reference kernels (the encode's
// traffic, XOR instead of the GF product):
//   base  one wave per block, 1 KiB column chunk of every shard, pad P bytes
//         between shards, dynamic LDS D bytes per block (occupancy cap)
//   skew  W waves per block own W consecutive 1 KiB chunks of one stripe;
//         wave w loads chunk (w + i*S) mod W of shard i into LDS, then, after
//         a barrier, codes chunk w from LDS and stores it (OUT=1: parity p is
//         stored at chunk (w + (K+p)*S) mod W, its inputs read from LDS)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/skew_mem.hip -o tools/bin/skew_mem
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

__device__ __forceinline__ u32x4 ld(const uint8_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}
__device__ __forceinline__ void st(uint8_t *p, const u32x4 &v) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
}

struct Geo {
    uint8_t *base;
    uint64_t stripe_stride, shard_stride;
    uint32_t chunks;    // 1 KiB chunks per shard
    uint32_t xcd_span;  // 0: plain block order
};

__device__ __forceinline__ uint32_t order(uint32_t b, uint32_t span) {
    return (span && b < 8u * span) ? (b & 7u) * span + (b >> 3) : b;
}

template <int K, int M>
__global__ void __launch_bounds__(64) base_kernel(Geo a) {
    const uint32_t b = order(blockIdx.x, a.xcd_span);
    const uint32_t stripe = b / a.chunks, chunk = b - stripe * a.chunks;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(chunk) * 1024 + threadIdx.x * 16u;
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = ld(sb + uint64_t(i) * a.shard_stride);
#pragma unroll
    for (int p = 0; p < M; ++p) {
        u32x4 acc = x[0] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
        for (int i = 1; i < K; ++i) acc ^= x[i];
        st(sb + uint64_t(K + p) * a.shard_stride, acc);
    }
}

template <int K, int M, int W, int S, int OUT>
__global__ void __launch_bounds__(64 * W) skew_kernel(Geo a) {
    extern __shared__ u32x4 lds[];  // [K][W][64]
    const uint32_t groups = a.chunks / W;
    const uint32_t b = order(blockIdx.x, a.xcd_span);
    const uint32_t stripe = b / groups, g = b - stripe * groups;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(g) * W * 1024 + lane * 16u;
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = ld(sb + uint64_t(i) * a.shard_stride + ((w + i * S) % W) * 1024u);
#pragma unroll
    for (int i = 0; i < K; ++i) lds[(i * W + (w + i * S) % W) * 64 + lane] = x[i];
    __syncthreads();
    if (!OUT) {
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = lds[(i * W + w) * 64 + lane];
#pragma unroll
        for (int p = 0; p < M; ++p) {
            u32x4 acc = x[0] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
            for (int i = 1; i < K; ++i) acc ^= x[i];
            st(sb + uint64_t(K + p) * a.shard_stride + w * 1024u, acc);
        }
    } else {
#pragma unroll
        for (int p = 0; p < M; ++p) {
            const uint32_t c = (w + (K + p) * S) % W;
            u32x4 acc = lds[c * 64 + lane] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
            for (int i = 1; i < K; ++i) acc ^= lds[(i * W + c) * 64 + lane];
            st(sb + uint64_t(K + p) * a.shard_stride + c * 1024u, acc);
        }
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

void report(size_t B, const char *name, double bytes, double ms) {
    std::printf("10+4 4MiB x%-5zu %-44s %7.3f ms  %.3f of 8 TB/s\n", B, name, ms, bytes / ms / 1e6 / 8000.0);
    std::fflush(stdout);
}

constexpr int K = 10, M = 4;

template <int W, int S, int OUT>
void run_skew(uint8_t *buf, size_t B, size_t stride, int span_on, int reps) {
    const size_t Sh = size_t(4) << 20;
    Geo g{buf, uint64_t((K + M) * stride), uint64_t(stride), uint32_t(Sh / 1024), 0};
    const uint32_t blocks = uint32_t(B * (g.chunks / W));
    if (span_on) g.xcd_span = blocks / 8u;
    const size_t lds = size_t(K) * W * 1024;
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(skew_kernel<K, M, W, S, OUT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    char name[96];
    std::snprintf(name, sizeof name, "skew W=%d S=%d out=%d pad=%zu %s", W, S, OUT, stride - Sh, span_on ? "xcd" : "plain");
    report(B, name, double(B) * (K + M) * Sh,
           median_ms([&] { hipLaunchKernelGGL((skew_kernel<K, M, W, S, OUT>), dim3(blocks), dim3(64 * W), lds, 0, g); }, reps));
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 7;
    const size_t Sh = size_t(4) << 20;
    const size_t cap = size_t(14) * (Sh + 8192) * 1024 + (size_t(1) << 20);
    uint8_t *buf = nullptr;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipMalloc(&buf, cap));
    CHECK(hipMemset(buf, 0x37, cap));
    for (int round = 0; round < 2; ++round) {
        for (size_t B : {size_t(128), size_t(1024)}) {
            for (size_t pad : {size_t(0), size_t(1024), size_t(2048), size_t(4096)}) {
                for (int dyn : {0, 10240, 12544}) {
                    for (int span_on = 0; span_on < 2; ++span_on) {
                        const size_t stride = Sh + pad;
                        Geo g{buf, uint64_t((K + M) * stride), uint64_t(stride), uint32_t(Sh / 1024), 0};
                        const uint32_t blocks = uint32_t(B * g.chunks);
                        if (span_on) g.xcd_span = blocks / 8u;
                        char name[96];
                        std::snprintf(name, sizeof name, "base pad=%zu lds=%d %s", pad, dyn, span_on ? "xcd" : "plain");
                        report(B, name, double(B) * (K + M) * Sh,
                               median_ms([&] { hipLaunchKernelGGL((base_kernel<K, M>), dim3(blocks), dim3(64), dyn, 0, g); }, reps));
                    }
                }
            }
            for (int span_on = 0; span_on < 2; ++span_on) {
                run_skew<4, 1, 0>(buf, B, Sh, span_on, reps);
                run_skew<8, 1, 0>(buf, B, Sh, span_on, reps);
                run_skew<8, 1, 1>(buf, B, Sh, span_on, reps);
                run_skew<8, 0, 0>(buf, B, Sh, span_on, reps);
                run_skew<8, 3, 0>(buf, B, Sh, span_on, reps);
                run_skew<16, 1, 0>(buf, B, Sh, span_on, reps);
                run_skew<16, 1, 1>(buf, B, Sh, span_on, reps);
                run_skew<8, 1, 0>(buf, B, Sh + 4096, span_on, reps);
            }
        }
    }
    CHECK(hipFree(buf));
    return 0;
}
