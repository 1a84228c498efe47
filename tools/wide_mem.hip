// wide_mem.hip -- is the 10+4 x 4 MiB encode's 0.72 of HBM peak set by its
// memory access pattern?  Memory-reference kernels in the encode kernel's
// exact shape (one wave per block, one 16-byte non-temporal vector per lane
// per shard, one-shot grid, stripe-major blocks with the XCD remap) but with
// XOR instead of the GF product, on the 4+2 x 1 MiB x 4096 and
// 10+4 x 4 MiB x 128 / x 1024 pools:
//   rdK+M   read every shard (the verify kernel's traffic)
//   rdK     read the K data shards
//   wrM     write the M parity shards
//   xorKM   read K, write M (the encode's traffic)
//   xorKM_sep  the same, loads of a wave completed before its stores issue
//   xorKM_pad  shards 4 KiB apart more than packed
// `sweep` runs the encode traffic over pads, block orders (identity, XCD
// remap, 3/8-stripe chunk rotation) and 1 / 2 / 4 KiB of each shard per wave.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/wide_mem.hip -o tools/bin/wide_mem
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
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

__device__ __forceinline__ u32x4 ld(const uint8_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}
__device__ __forceinline__ void st(uint8_t *p, const u32x4 &v) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
}

// OP 0: read all K+M; 1: read K; 2: write M; 3: read K -> write M; 4: as 3, loads drained first.
// V: 16-byte vectors per lane per shard (1 KiB apart): a wave covers V KiB of each shard.
template <int K, int M, int OP, int V = 1>
__global__ void __launch_bounds__(64) wide_kernel(Geo a) {
    uint32_t b = blockIdx.x;
    if (a.xcd_span && b < 8u * a.xcd_span) b = (b & 7u) * a.xcd_span + (b >> 3);
    const uint32_t stripe = b / a.chunks;
    uint32_t chunk = b - stripe * a.chunks;
    if (a.rot) chunk = (chunk + stripe * a.rot) % a.chunks;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(chunk) * 1024 * V + threadIdx.x * 16u;
    if (V > 1) {  // encode traffic only
        u32x4 x[K][V];
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int v = 0; v < V; ++v) x[i][v] = ld(sb + uint64_t(i) * a.shard_stride + v * 1024);
#pragma unroll
        for (int p = 0; p < M; ++p)
#pragma unroll
            for (int v = 0; v < V; ++v) {
                u32x4 acc = x[0][v] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
                for (int i = 1; i < K; ++i) acc ^= x[i][v];
                st(sb + uint64_t(K + p) * a.shard_stride + v * 1024, acc);
            }
        return;
    }
    if (OP == 2) {
        const uint32_t t = b * 64u + threadIdx.x;
#pragma unroll
        for (int p = 0; p < M; ++p) st(sb + uint64_t(K + p) * a.shard_stride, u32x4{t, t + 1u, t + 2u, uint32_t(p)});
        return;
    }
    constexpr int NR = OP == 0 ? K + M : K;
    u32x4 x[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) x[i] = ld(sb + uint64_t(i) * a.shard_stride);
    if (OP <= 1) {
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < NR; ++i) s ^= x[i][0] ^ x[i][1] ^ x[i][2] ^ x[i][3];
        if (s == 0x9E3779B9u) a.sink[threadIdx.x] = s;
        return;
    }
    if (OP == 4) __builtin_amdgcn_s_waitcnt(0);  // every load of the wave back before any store
    u32x4 acc[M];
#pragma unroll
    for (int p = 0; p < M; ++p) {
        acc[p] = x[0] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
        for (int i = 1; i < K; ++i) acc[p] ^= x[i];
    }
#pragma unroll
    for (int p = 0; p < M; ++p) st(sb + uint64_t(K + p) * a.shard_stride, acc[p]);
}

// Encode traffic with a choice of cache policy: LP / SP = 1 plain, 0 non-temporal.
template <int K, int M, int LP, int SP>
__global__ void __launch_bounds__(64) policy_kernel(Geo a) {
    uint32_t b = blockIdx.x;
    if (a.xcd_span && b < 8u * a.xcd_span) b = (b & 7u) * a.xcd_span + (b >> 3);
    const uint32_t stripe = b / a.chunks;
    uint32_t chunk = b - stripe * a.chunks;
    if (a.rot) chunk = (chunk + stripe * a.rot) % a.chunks;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(chunk) * 1024 + threadIdx.x * 16u;
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const u32x4 *p = reinterpret_cast<const u32x4 *>(sb + uint64_t(i) * a.shard_stride);
        x[i] = LP ? *p : __builtin_nontemporal_load(p);
    }
#pragma unroll
    for (int p = 0; p < M; ++p) {
        u32x4 acc = x[0] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
        for (int i = 1; i < K; ++i) acc ^= x[i];
        u32x4 *q = reinterpret_cast<u32x4 *>(sb + uint64_t(K + p) * a.shard_stride);
        if (SP) *q = acc;
        else __builtin_nontemporal_store(acc, q);
    }
}

// File-encode traffic reference: a wave reads K KiB of the file contiguously
// (16 B per lane per instruction) and writes K data + M parity KiB, one KiB to
// each of K+M shards (shard stride S).  file_decode reference (DEC): reads K
// shards' KiB, writes K KiB of file.
template <int K, int M, bool DEC>
__global__ void __launch_bounds__(64) file_ref_kernel(const uint8_t *file, uint8_t *fout, uint8_t *shards,
                                                      uint64_t S, uint32_t xcd_span, uint32_t n_items) {
    uint32_t b = blockIdx.x;
    if (xcd_span && b < 8u * xcd_span) b = (b & 7u) * xcd_span + (b >> 3);
    const uint64_t col = uint64_t(b) * 1024 + threadIdx.x * 16u;  // column within each shard
    if (!DEC) {
        u32x4 x[K];
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = ld(file + uint64_t(b) * 1024 * K + uint64_t(i) * 1024 + threadIdx.x * 16u);
#pragma unroll
        for (int i = 0; i < K; ++i) st(shards + uint64_t(i) * S + col, x[i]);
#pragma unroll
        for (int p = 0; p < M; ++p) {
            u32x4 acc = x[0] + u32x4{uint32_t(p), 0, 0, 0};
#pragma unroll
            for (int i = 1; i < K; ++i) acc ^= x[i];
            st(shards + uint64_t(K + p) * S + col, acc);
        }
    } else {
        u32x4 x[K];
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = ld(shards + uint64_t(i + 1) * S + col);
#pragma unroll
        for (int i = 0; i < K; ++i) st(fout + uint64_t(b) * 1024 * K + uint64_t(i) * 1024 + threadIdx.x * 16u, x[i]);
    }
}

// Same traffic as the encode, but no wave both reads and writes: even blocks
// read the K data shards of item b/2, odd blocks write the M parity shards of
// item b/2 (interleaved in dispatch order).  Tells a per-wave (CU-side)
// read/write mixing cost from a DRAM-side one.
template <int K, int M>
__global__ void __launch_bounds__(64) split_roles_kernel(Geo a) {
    uint32_t b = blockIdx.x >> 1;
    if (a.xcd_span && b < 8u * a.xcd_span) b = (b & 7u) * a.xcd_span + (b >> 3);
    const uint32_t stripe = b / a.chunks;
    uint32_t chunk = b - stripe * a.chunks;
    if (a.rot) chunk = (chunk + stripe * a.rot) % a.chunks;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(chunk) * 1024 + threadIdx.x * 16u;
    if (blockIdx.x & 1) {
        const uint32_t t = b * 64u + threadIdx.x;
#pragma unroll
        for (int p = 0; p < M; ++p) st(sb + uint64_t(K + p) * a.shard_stride, u32x4{t, t + 1u, t + 2u, uint32_t(p)});
        return;
    }
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = ld(sb + uint64_t(i) * a.shard_stride);
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) s ^= x[i][0] ^ x[i][1] ^ x[i][2] ^ x[i][3];
    if (s == 0x9E3779B9u) a.sink[threadIdx.x] = s;
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

void report(const char *shape, const char *name, double bytes, double ms) {
    std::printf("%-22s %-34s %7.3f ms  %7.1f GB/s  %.3f of 8 TB/s\n", shape, name, ms, bytes / ms / 1e6,
                bytes / ms / 1e6 / 8000.0);
    std::fflush(stdout);
}

template <int K, int M, int V>
double enc(uint8_t *buf, size_t S, size_t B, size_t stride, uint32_t *sink, int order, int reps) {
    const uint32_t chunks = uint32_t(S / (1024 * V));
    Geo g{buf, sink, uint64_t((K + M) * stride), uint64_t(stride), chunks, uint32_t(B * chunks), 0, 0};
    if (order == 1) g.xcd_span = g.n_items / 8u;
    if (order == 2) g.rot = 3u * chunks / 8u - 1u;
    const dim3 grid(g.n_items);
    return median_ms([&] { hipLaunchKernelGGL((wide_kernel<K, M, 3, V>), grid, dim3(64), 0, 0, g); }, reps);
}

template <int K, int M>
void sweep(uint8_t *buf, size_t cap, uint32_t *sink, size_t S, size_t B, int reps) {
    static const char *orders[] = {"plain", "xcd", "rot3/8"};
    for (size_t pad : {size_t(0), size_t(4096), size_t(8192), size_t(65536 + 4096), size_t(1) << 20}) {
        const size_t stride = S + pad;
        if (B * (K + M) * stride > cap) continue;
        for (int order = 0; order < 3; ++order) {
            char name[96];
            std::snprintf(name, sizeof name, "%d+%d %zuKiB x%zu", K, M, S >> 10, B);
            const double bytes = double(B) * (K + M) * S;
            char leg[96];
            std::snprintf(leg, sizeof leg, "pad %7zu %-6s 1 KiB/wave", pad, orders[order]);
            report(name, leg, bytes, enc<K, M, 1>(buf, S, B, stride, sink, order, reps));
            std::snprintf(leg, sizeof leg, "pad %7zu %-6s 2 KiB/wave", pad, orders[order]);
            report(name, leg, bytes, enc<K, M, 2>(buf, S, B, stride, sink, order, reps));
            std::snprintf(leg, sizeof leg, "pad %7zu %-6s 4 KiB/wave", pad, orders[order]);
            report(name, leg, bytes, enc<K, M, 4>(buf, S, B, stride, sink, order, reps));
        }
    }
}

template <int K, int M>
void policies(uint8_t *buf, uint32_t *sink, size_t S, size_t B, int reps) {
    const size_t stride = S;
    const uint32_t chunks = uint32_t(S / 1024);
    static const char *names[] = {"nt load / nt store", "nt load / plain store", "plain load / nt store",
                                  "plain load / plain store"};
    for (int order = 0; order < 2; ++order)
        for (int v = 0; v < 4; ++v) {
            Geo g{buf, sink, uint64_t((K + M) * stride), uint64_t(stride), chunks, uint32_t(B * chunks), 0, 0};
            if (order == 0) g.xcd_span = g.n_items / 8u;
            else g.rot = 3u * chunks / 8u - 1u;
            const dim3 grid(g.n_items);
            double ms = 0;
            if (v == 0) ms = median_ms([&] { hipLaunchKernelGGL((policy_kernel<K, M, 0, 0>), grid, dim3(64), 0, 0, g); }, reps);
            if (v == 1) ms = median_ms([&] { hipLaunchKernelGGL((policy_kernel<K, M, 0, 1>), grid, dim3(64), 0, 0, g); }, reps);
            if (v == 2) ms = median_ms([&] { hipLaunchKernelGGL((policy_kernel<K, M, 1, 0>), grid, dim3(64), 0, 0, g); }, reps);
            if (v == 3) ms = median_ms([&] { hipLaunchKernelGGL((policy_kernel<K, M, 1, 1>), grid, dim3(64), 0, 0, g); }, reps);
            char name[64], leg[96];
            std::snprintf(name, sizeof name, "%d+%d %zuKiB x%zu", K, M, S >> 10, B);
            std::snprintf(leg, sizeof leg, "%s %s", order ? "rot" : "xcd", names[v]);
            report(name, leg, double(B) * (K + M) * S, ms);
        }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    if (argc > 2 && std::string(argv[2]) == "roles") {
        const size_t cap = size_t(60) << 30;
        uint8_t *buf = nullptr;
        uint32_t *sink = nullptr;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        CHECK(hipMalloc(&buf, cap));
        CHECK(hipMalloc(&sink, 256));
        CHECK(hipMemset(buf, 0x37, cap));
        struct Shape { int k, m; size_t S, B; } shapes[] = {{10, 4, size_t(4) << 20, 128}, {4, 2, size_t(1) << 20, 4096}};
        for (const Shape &sh : shapes) {
            const uint32_t chunks = uint32_t(sh.S / 1024);
            for (int order = 0; order < 2; ++order) {
                Geo g{buf, sink, uint64_t((sh.k + sh.m) * sh.S), uint64_t(sh.S), chunks, uint32_t(sh.B * chunks), 0, 0};
                if (order == 0) g.xcd_span = g.n_items / 8u;
                else g.rot = 3u * chunks / 8u - 1u;
                const double bytes = double(sh.B) * (sh.k + sh.m) * sh.S;
                char name[64];
                std::snprintf(name, sizeof name, "%d+%d %zuKiB x%zu", sh.k, sh.m, sh.S >> 10, sh.B);
                const char *o = order ? "rot" : "xcd";
                double mixed, split;
                if (sh.k == 10) {
                    mixed = median_ms([&] { hipLaunchKernelGGL((wide_kernel<10, 4, 3>), dim3(g.n_items), dim3(64), 0, 0, g); }, reps);
                    split = median_ms([&] { hipLaunchKernelGGL((split_roles_kernel<10, 4>), dim3(2 * g.n_items), dim3(64), 0, 0, g); }, reps);
                } else {
                    mixed = median_ms([&] { hipLaunchKernelGGL((wide_kernel<4, 2, 3>), dim3(g.n_items), dim3(64), 0, 0, g); }, reps);
                    split = median_ms([&] { hipLaunchKernelGGL((split_roles_kernel<4, 2>), dim3(2 * g.n_items), dim3(64), 0, 0, g); }, reps);
                }
                char leg[96];
                std::snprintf(leg, sizeof leg, "%s read+write in every wave", o);
                report(name, leg, bytes, mixed);
                std::snprintf(leg, sizeof leg, "%s reader waves + writer waves", o);
                report(name, leg, bytes, split);
            }
        }
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "file") {
        const size_t F = size_t(4) << 30, S = F / 4;  // 4 GiB file, 4+2 shards of 1 GiB
        uint8_t *file = nullptr, *fout = nullptr, *sh = nullptr;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        CHECK(hipMalloc(&file, F));
        CHECK(hipMalloc(&fout, F));
        CHECK(hipMalloc(&sh, 6 * S));
        CHECK(hipMemset(file, 0x11, F));
        CHECK(hipMemset(sh, 0x22, 6 * S));
        const uint32_t n = uint32_t(S / 1024);
        for (int xcd = 0; xcd < 2; ++xcd) {
            const uint32_t span = xcd ? n / 8 : 0;
            report("file 4 GiB -> 4+2", xcd ? "encode traffic, xcd" : "encode traffic, plain", double(F) + 6.0 * S,
                   median_ms([&] { hipLaunchKernelGGL((file_ref_kernel<4, 2, false>), dim3(n), dim3(64), 0, 0, file, fout, sh, S, span, n); }, reps));
            report("4+2 -> file 4 GiB", xcd ? "decode traffic (4 shards -> file), xcd" : "decode traffic, plain",
                   double(F) + 4.0 * S,
                   median_ms([&] { hipLaunchKernelGGL((file_ref_kernel<4, 2, true>), dim3(n), dim3(64), 0, 0, file, fout, sh, S, span, n); }, reps));
        }
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "policy") {
        const size_t cap = size_t(60) << 30;
        uint8_t *buf = nullptr;
        uint32_t *sink = nullptr;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        CHECK(hipMalloc(&buf, cap));
        CHECK(hipMalloc(&sink, 256));
        CHECK(hipMemset(buf, 0x37, cap));
        policies<10, 4>(buf, sink, size_t(4) << 20, 128, reps);
        policies<10, 4>(buf, sink, size_t(4) << 20, 1024, reps);
        policies<4, 2>(buf, sink, size_t(1) << 20, 4096, reps);
        CHECK(hipFree(buf));
        return 0;
    }
    const size_t cap = size_t(60) << 30;
    uint8_t *buf = nullptr;
    uint32_t *sink = nullptr;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipMalloc(&buf, cap));
    CHECK(hipMalloc(&sink, 256));
    CHECK(hipMemset(buf, 0x37, cap));
    sweep<10, 4>(buf, cap, sink, size_t(4) << 20, 128, reps);
    sweep<10, 4>(buf, cap, sink, size_t(4) << 20, 1024, reps);
    sweep<4, 2>(buf, cap, sink, size_t(1) << 20, 4096, reps);
    CHECK(hipFree(buf));
    return 0;
}
