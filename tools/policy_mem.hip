// policy_mem.hip -- cache-policy bits of the streaming stores and loads on the
// encode access pattern (XOR in place of the GF product; same one-shot grid,
// one wave per 1 KiB column chunk, XCD remap or 3/8 rotation as the product
// kernels use).  Stores: nt (the product kernels' __builtin_nontemporal_store),
// plain, sc1, sc0 sc1, nt sc1, nt sc0 sc1; loads nt.  (Load variants written
// as separate inline-asm loads faulted: the compiler may reuse a register an
// in-flight asm load still targets.)  The
// guide's table: plain / sc0 / nt stores keep the line in the XCD's L2, sc1 /
// sc0 sc1 drop it.  Pools: 4+2 x 1 MiB x 4096 and 10+4 x 4 MiB x 128, write-only
// and read-k-write-m.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/policy_mem.hip -o tools/bin/policy_mem
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
    uint32_t chunks, n_items, xcd_span, rot;
};

enum { ST_NT, ST_PLAIN, ST_SC1, ST_SC01, ST_NTSC1, ST_NTSC01 };
enum { LD_NT };

template <int P>
__device__ __forceinline__ void st(uint8_t *p, const u32x4 &v) {
    if (P == ST_NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
    if (P == ST_PLAIN) *reinterpret_cast<u32x4 *>(p) = v;
    if (P == ST_SC1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    if (P == ST_SC01) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    if (P == ST_NTSC1) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    if (P == ST_NTSC01) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ uint8_t *item(const Geo &a) {
    uint32_t b = blockIdx.x;
    if (a.xcd_span && b < 8u * a.xcd_span) b = (b & 7u) * a.xcd_span + (b >> 3);
    const uint32_t stripe = b / a.chunks;
    uint32_t chunk = b - stripe * a.chunks;
    if (a.rot) chunk = (chunk + stripe * a.rot) % a.chunks;
    return a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(chunk) * 1024 + threadIdx.x * 16u;
}

// WO: write the M parity shards only; else read K, write M.
template <int K, int M, int SP, int LP, bool WO>
__global__ void __launch_bounds__(64) enc_kernel(Geo a) {
    uint8_t *sb = item(a);
    if (WO) {
        const uint32_t t = blockIdx.x * 64u + threadIdx.x;
#pragma unroll
        for (int p = 0; p < M; ++p) st<SP>(sb + uint64_t(K + p) * a.shard_stride, u32x4{t, t + 1u, t + 2u, uint32_t(p)});
        return;
    }
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(sb + uint64_t(i) * a.shard_stride));
#pragma unroll
    for (int p = 0; p < M; ++p) {
        u32x4 acc = x[0] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
        for (int i = 1; i < K; ++i) acc ^= x[i];
        st<SP>(sb + uint64_t(K + p) * a.shard_stride, acc);
    }
}

hipEvent_t e0, e1;

template <class F>
double median_ms(F launch, int reps) {
    launch();
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    for (int w = 0; w < 20; ++w) launch();  // a few ms of load before timing
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

const char *st_name[] = {"nt", "plain", "sc1", "sc0 sc1", "nt sc1", "nt sc0 sc1"};
const char *ld_name[] = {"nt"};

template <int K, int M, int SP, int LP, bool WO>
void leg(const Geo &g, int reps, const char *shape, const char *order) {
    const double ms = median_ms([&] { hipLaunchKernelGGL((enc_kernel<K, M, SP, LP, WO>), dim3(g.n_items), dim3(64), 0, 0, g); }, reps);
    const double bytes = double(g.n_items) * 1024.0 * (WO ? M : K + M);
    std::printf("%-16s %-6s %-10s store %-11s load %-7s %7.3f ms  %.3f of 8 TB/s\n", shape, order,
                WO ? "write-only" : "rd k wr m", st_name[SP], WO ? "-" : ld_name[LP], ms, bytes / ms / 1e6 / 8000.0);
    std::fflush(stdout);
}

template <int K, int M>
void shape(uint8_t *buf, size_t S, size_t B, int reps, const char *name) {
    const uint32_t chunks = uint32_t(S / 1024);
    for (int order = 0; order < 2; ++order) {
        Geo g{buf, uint64_t((K + M) * S), uint64_t(S), chunks, uint32_t(B * chunks), 0, 0};
        if (order == 0) g.xcd_span = g.n_items / 8u;
        else g.rot = 3u * chunks / 8u - 1u;
        const char *o = order ? "rot" : "xcd";
        for (int rep = 0; rep < 2; ++rep) {
            leg<K, M, ST_NT, LD_NT, true>(g, reps, name, o);
            leg<K, M, ST_PLAIN, LD_NT, true>(g, reps, name, o);
            leg<K, M, ST_SC1, LD_NT, true>(g, reps, name, o);
            leg<K, M, ST_SC01, LD_NT, true>(g, reps, name, o);
            leg<K, M, ST_NTSC1, LD_NT, true>(g, reps, name, o);
            leg<K, M, ST_NTSC01, LD_NT, true>(g, reps, name, o);
            leg<K, M, ST_NT, LD_NT, false>(g, reps, name, o);
            leg<K, M, ST_SC1, LD_NT, false>(g, reps, name, o);
            leg<K, M, ST_SC01, LD_NT, false>(g, reps, name, o);
            leg<K, M, ST_NTSC1, LD_NT, false>(g, reps, name, o);
            leg<K, M, ST_NTSC01, LD_NT, false>(g, reps, name, o);
        }
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    const size_t cap = size_t(28) << 30;
    uint8_t *buf = nullptr;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipMalloc(&buf, cap));
    CHECK(hipMemset(buf, 0x37, cap));
    shape<4, 2>(buf, size_t(1) << 20, 4096, reps, "4+2 1MiB x4096");
    shape<10, 4>(buf, size_t(4) << 20, 128, reps, "10+4 4MiB x128");
    CHECK(hipFree(buf));
    return 0;
}
