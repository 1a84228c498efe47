// phase_mem.hip -- can a chip-wide read phase / write phase schedule beat the
// 10+4 x 4 MiB encode's access-pattern ceiling (reads alone 0.86,
// writes alone 0.75-0.88, interleaved 0.73)?
//
// Memory-reference kernels (XOR in place of the GF product) on the
// 10+4 x 4 MiB x 128 pool:
//   oneshot   the product kernel's shape: one wave per 1 KiB column chunk,
//             one-shot grid, XCD remap (the existing ceiling, wide_mem.hip)
//   phased    persistent grid, one or two 256-thread workgroups per CU.  Per
//             phase each wave reads U consecutive 1 KiB chunks of all K data
//             shards, folds them into U*M parity vectors held in registers,
//             then stores them.  BAR 0: no synchronisation (phases stay
//             aligned only by equal work); 1: a grid barrier at the start of
//             every phase; 2: also one between the reads and the stores.
// The barrier is for timing only (no data crosses workgroups): one relaxed
// agent-scope atomic add per workgroup, a relaxed agent-scope poll with
// s_sleep, every spin bounded (an error word reports a timeout).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/phase_mem.hip -o tools/bin/phase_mem
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
    uint32_t chunks;    // 1 KiB column chunks per shard
    uint32_t n_items;   // stripes * chunks
    uint32_t xcd_span;  // oneshot only
    uint32_t *ctr;      // barrier counter (phased)
    uint32_t ctr_base;  // counter value at launch start
    uint32_t *err;
    uint32_t phases;
};

template <int K, int M>
__global__ void __launch_bounds__(64) oneshot_kernel(Geo a) {
    uint32_t b = blockIdx.x;
    if (a.xcd_span && b < 8u * a.xcd_span) b = (b & 7u) * a.xcd_span + (b >> 3);
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

// Timing-only grid barrier (see the header).  Returns after every workgroup
// of the grid has arrived `n` times in this launch, or after the spin bound.
__device__ __forceinline__ void grid_arrive_wait(const Geo &a, uint32_t n) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(a.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t target = a.ctr_base + n * gridDim.x;
        uint32_t spins = 0;
        while (int32_t(__hip_atomic_load(a.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 22)) {
                __hip_atomic_fetch_add(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
}

template <int K, int M, int U, int BAR, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) phased_kernel(Geo a) {
    const uint32_t waves = gridDim.x * 4u;
    const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t arrivals = 0;
    for (uint32_t ph = 0; ph < a.phases; ++ph) {
        if (BAR >= 1) grid_arrive_wait(a, ++arrivals);
        const uint32_t g = (ph * waves + wave) * U;  // first chunk of this wave's group
        const uint32_t stripe = g / a.chunks, chunk = g - stripe * a.chunks;
        uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(chunk) * 1024 + lane * 16u;
        u32x4 acc[U][M];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x4 x[K];
#pragma unroll
            for (int i = 0; i < K; ++i) x[i] = ld(sb + uint64_t(i) * a.shard_stride + u * 1024);
#pragma unroll
            for (int p = 0; p < M; ++p) {
                acc[u][p] = x[0] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
                for (int i = 1; i < K; ++i) acc[u][p] ^= x[i];
            }
        }
        if (BAR >= 2) grid_arrive_wait(a, ++arrivals);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int p = 0; p < M; ++p) st(sb + uint64_t(K + p) * a.shard_stride + u * 1024, acc[u][p]);
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

void report(const char *name, double bytes, double ms) {
    std::printf("%-48s %7.3f ms  %7.1f GB/s  %.3f of 8 TB/s\n", name, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 8000.0);
    std::fflush(stdout);
}

int n_cu = 0;
uint32_t host_ctr = 0;  // counter value the device holds between launches

template <int K, int M, int U, int BAR, int WPE>
void run_phased(Geo g, double bytes, int reps) {
    const int wg_per_cu = WPE;  // 4 waves per workgroup, WPE waves per SIMD
    const uint32_t grid = uint32_t(n_cu * wg_per_cu);
    const uint32_t per_phase = grid * 4u * U;
    if (g.n_items % per_phase) {
        std::printf("skip U=%d WPE=%d: %u chunks not a multiple of %u\n", U, WPE, g.n_items, per_phase);
        return;
    }
    g.phases = g.n_items / per_phase;
    const uint32_t arrivals = BAR == 0 ? 0 : g.phases * uint32_t(BAR);
    const double ms = median_ms(
        [&] {
            g.ctr_base = host_ctr;
            hipLaunchKernelGGL((phased_kernel<K, M, U, BAR, WPE>), dim3(grid), dim3(256), 0, 0, g);
            host_ctr += arrivals * grid;
        },
        reps);
    uint32_t err = 0;
    CHECK(hipMemcpy(&err, g.err, 4, hipMemcpyDeviceToHost));
    char name[96];
    std::snprintf(name, sizeof name, "phased U=%-2d BAR=%d %d WG/CU (%u phases, %.0f MiB rd)%s", U, BAR, WPE, g.phases,
                  double(per_phase) * K / 1024.0, err ? " SPIN-TIMEOUT" : "");
    report(name, bytes, ms);
    if (err) std::exit(3);
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    const size_t B = argc > 2 ? size_t(std::atoi(argv[2])) : 128;
    constexpr int K = 10, M = 4;
    const size_t S = size_t(4) << 20;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    n_cu = prop.multiProcessorCount;
    std::printf("CUs %d, 10+4 x 4 MiB x %zu\n", n_cu, B);
    uint8_t *buf = nullptr;
    uint32_t *ctr = nullptr;
    const size_t cap = B * (K + M) * S;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipMalloc(&buf, cap));
    CHECK(hipMalloc(&ctr, 256));
    CHECK(hipMemset(buf, 0x37, cap));
    CHECK(hipMemset(ctr, 0, 256));
    const uint32_t chunks = uint32_t(S / 1024);
    Geo g{buf, uint64_t((K + M) * S), uint64_t(S), chunks, uint32_t(B * chunks), 0, ctr, 0, ctr + 32, 0};
    const double bytes = double(B) * (K + M) * S;
    for (int rep = 0; rep < 2; ++rep) {
        g.xcd_span = g.n_items / 8u;
        report("oneshot xcd", bytes, median_ms([&] { hipLaunchKernelGGL((oneshot_kernel<K, M>), dim3(g.n_items), dim3(64), 0, 0, g); }, reps));
        g.xcd_span = 0;
        report("oneshot plain", bytes, median_ms([&] { hipLaunchKernelGGL((oneshot_kernel<K, M>), dim3(g.n_items), dim3(64), 0, 0, g); }, reps));
        run_phased<K, M, 4, 0, 1>(g, bytes, reps);
        run_phased<K, M, 8, 0, 1>(g, bytes, reps);
        run_phased<K, M, 4, 0, 2>(g, bytes, reps);
        run_phased<K, M, 8, 1, 1>(g, bytes, reps);
        run_phased<K, M, 8, 2, 1>(g, bytes, reps);
        run_phased<K, M, 4, 1, 2>(g, bytes, reps);
        run_phased<K, M, 4, 2, 2>(g, bytes, reps);
        run_phased<K, M, 16, 1, 1>(g, bytes, reps);
    }
    CHECK(hipFree(buf));
    CHECK(hipFree(ctr));
    return 0;
}
