// group_mem.hip -- what does the access pattern of 4+2 x 1000-B chunk groups
// packed back to back (stride 1000, group stride 6000; the master's recovery
// batches, ChunkserverDiskRecoveryMachine.java:34-48) allow on MI355X?
// Memory-reference kernels with XOR in place of the GF product, in the
// 8-byte-aligned kernels' shapes (kernels.hip gf_vec8_kernel / gf_masked8_kernel),
// over 4 M groups (24 GB):
//   x8     one 8-byte vector per lane: read 4 data shards, write 2 (two waves per group)
//   x16    16-byte vectors at 8-byte alignment plus the half vector (one wave per group)
//   rd8    read the 4 data shards only (x8 shape)
//   wr8    write the 2 parity shards only (x8 shape)
//   sep8   read 4000 B per group from this pool, write 2000 B per group to a
//          second pool (the same bytes, reads and writes in different pages)
//   copy   a 16-byte copy of 16 GB into a second pool (the streaming ceiling)
//   x8 at strides 1024 / 1008, and xal: stride 1000 with the parity region
//          written as aligned 16-byte stores (is the partial-line write the cost?)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/group_mem.hip -o tools/bin/group_mem
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

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a8 __attribute__((ext_vector_type(4), aligned(8)));

constexpr uint64_t S = 1000, G = 6000;

template <typename V>
__device__ __forceinline__ V ld(const uint8_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const V *>(p));
}
template <typename V>
__device__ __forceinline__ void st(uint8_t *p, const V &v) {
    __builtin_nontemporal_store(v, reinterpret_cast<V *>(p));
}

// OP 0: read 4 -> write 2 in place; 1: read only (sink); 2: write only; 3: read here, write to `out`.
template <int OP>
__global__ void __launch_bounds__(64) x8_kernel(uint8_t *base, uint8_t *out, uint32_t *sink) {
    const uint32_t group = blockIdx.x >> 1, v = (blockIdx.x & 1) * 64 + threadIdx.x;
    if (v >= S / 8) return;
    uint8_t *g = base + uint64_t(group) * G + v * 8;
    u32x2 acc{0, 0};
    if (OP != 2) {
        u32x2 x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = ld<u32x2>(g + i * S);
        acc = x[0] ^ x[1] ^ x[2] ^ x[3];
    }
    if (OP == 1) {
        if ((acc[0] ^ acc[1]) == 0x12345678u) *sink = acc[0];
        return;
    }
    uint8_t *o = OP == 3 ? out + uint64_t(group) * 2 * S + v * 8 : g + 4 * S;
    st<u32x2>(o, acc);
    st<u32x2>(o + S, acc ^ u32x2{1, 1});
}

// x8 at any shard stride SS (group stride 6 * SS), in place.
template <uint64_t SS>
__global__ void __launch_bounds__(64) x8s_kernel(uint8_t *base) {
    const uint32_t group = blockIdx.x >> 1, v = (blockIdx.x & 1) * 64 + threadIdx.x;
    if (v >= S / 8) return;
    uint8_t *g = base + uint64_t(group) * 6 * SS + v * 8;
    u32x2 x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = ld<u32x2>(g + i * SS);
    const u32x2 acc = x[0] ^ x[1] ^ x[2] ^ x[3];
    st<u32x2>(g + 4 * SS, acc);
    st<u32x2>(g + 5 * SS, acc ^ u32x2{1, 1});
}

// Stride 1000, reads as x8, but the 2000-byte parity region of a group (16-byte
// aligned at both ends) written as aligned 16-byte stores: wave w of the group
// stores region bytes [1024 w, 1024 w + 1024) clipped to 2000.
__global__ void __launch_bounds__(64) xal_kernel(uint8_t *base) {
    const uint32_t group = blockIdx.x >> 1, w = blockIdx.x & 1, v = w * 64 + threadIdx.x;
    uint8_t *g = base + uint64_t(group) * G;
    u32x2 acc{0, 0};
    if (v < S / 8) {
        u32x2 x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = ld<u32x2>(g + v * 8 + i * S);
        acc = x[0] ^ x[1] ^ x[2] ^ x[3];
    }
    const uint32_t off = w * 1024 + threadIdx.x * 16;
    if (off < 2 * S) st<u32x4>(g + 4 * S + off, u32x4{acc[0], acc[1], acc[0] ^ 1u, acc[1] ^ 1u});
}

// Stride 1000, x8's loads and per-shard spans, but each output shard's bytes
// stored as 16-byte-aligned pairs of lanes' 8-byte vectors (the lane whose
// address is 16-aligned takes its neighbour's half by ds_bpermute; edge lanes
// store 8 bytes): does the store granularity alone matter?
__global__ void __launch_bounds__(64) xpair_kernel(uint8_t *base) {
    const uint32_t group = blockIdx.x >> 1, v = (blockIdx.x & 1) * 64 + threadIdx.x;
    const bool act = v < S / 8;
    uint8_t *g = base + uint64_t(group) * G + uint64_t(v) * 8;
    u32x2 acc{0, 0};
    if (act) {
        u32x2 x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = ld<u32x2>(g + i * S);
        acc = x[0] ^ x[1] ^ x[2] ^ x[3];
    }
    const int nb = (threadIdx.x + 1) & 63;
    const bool nb_act = threadIdx.x < 63 && v + 1 < S / 8;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const u32x2 mine = acc ^ u32x2{uint32_t(p), uint32_t(p)};
        const u32x2 next{uint32_t(__builtin_amdgcn_ds_bpermute(nb << 2, int(mine[0]))),
                         uint32_t(__builtin_amdgcn_ds_bpermute(nb << 2, int(mine[1])))};
        if (!act) continue;
        uint8_t *q = g + (4 + p) * S;
        const bool lead = (reinterpret_cast<uintptr_t>(q) & 15) == 0;
        const bool prev_leads = !lead && threadIdx.x > 0;  // the lane before stored this half
        if (lead && nb_act)
            st<u32x4>(q, u32x4{mine[0], mine[1], next[0], next[1]});
        else if (!prev_leads)
            st<u32x2>(q, mine);
    }
}

__global__ void __launch_bounds__(64) x16_kernel(uint8_t *base) {
    const uint32_t group = blockIdx.x, v = threadIdx.x;
    if (v > S / 16) return;
    uint8_t *g = base + uint64_t(group) * G + v * 16;
    if (v < S / 16) {
        u32x4a8 x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = ld<u32x4a8>(g + i * S);
        const u32x4a8 acc = x[0] ^ x[1] ^ x[2] ^ x[3];
        st<u32x4a8>(g + 4 * S, acc);
        st<u32x4a8>(g + 5 * S, acc ^ u32x4a8{1, 1, 1, 1});
    } else {
        u32x2 x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = ld<u32x2>(g + i * S);
        const u32x2 acc = x[0] ^ x[1] ^ x[2] ^ x[3];
        st<u32x2>(g + 4 * S, acc);
        st<u32x2>(g + 5 * S, acc ^ u32x2{1, 1});
    }
}

__global__ void __launch_bounds__(64) copy_kernel(const uint8_t *src, uint8_t *dst) {
    const uint64_t i = (uint64_t(blockIdx.x) * 64 + threadIdx.x) * 16;
    st<u32x4>(dst + i, ld<u32x4>(src + i));
}

static hipEvent_t e0, e1;

template <typename F>
double median_ms(F launch, int reps) {
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(e0, 0));
        launch();
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

static void report(const char *leg, double bytes, double ms) {
    std::printf("{\"leg\": \"%s\", \"ms\": %.4f, \"hbm_frac\": %.4f}\n", leg, ms, bytes / (ms * 1e-3) / 8e12);
    std::fflush(stdout);
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 10;
    const uint32_t B = 4u << 20;
    const size_t pool = size_t(B) * 6 * 1024, out_bytes = size_t(B) * 2 * S;  // room for 1 KiB slots
    uint8_t *base = nullptr, *out = nullptr;
    uint32_t *sink = nullptr;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipExtMallocWithFlags(reinterpret_cast<void **>(&base), pool, hipDeviceMallocContiguous));
    CHECK(hipMalloc(&out, std::max(out_bytes, size_t(16) << 30)));
    CHECK(hipMalloc(&sink, 256));
    CHECK(hipMemset(base, 0x37, pool));
    CHECK(hipMemset(out, 0x11, std::max(out_bytes, size_t(16) << 30)));
    const double all = double(B) * G, rd = double(B) * 4 * S, wr = double(B) * 2 * S;
    for (int rep = 0; rep < 2; ++rep) {
        report("x8 read 4 -> write 2 in place", all,
               median_ms([&] { hipLaunchKernelGGL(x8_kernel<0>, dim3(2 * B), dim3(64), 0, 0, base, out, sink); }, reps));
        report("x16 read 4 -> write 2 in place", all,
               median_ms([&] { hipLaunchKernelGGL(x16_kernel, dim3(B), dim3(64), 0, 0, base); }, reps));
        report("rd8 read 4 only", rd,
               median_ms([&] { hipLaunchKernelGGL(x8_kernel<1>, dim3(2 * B), dim3(64), 0, 0, base, out, sink); }, reps));
        report("wr8 write 2 only", wr,
               median_ms([&] { hipLaunchKernelGGL(x8_kernel<2>, dim3(2 * B), dim3(64), 0, 0, base, out, sink); }, reps));
        report("sep8 read 4 here -> write 2 to a second pool", all,
               median_ms([&] { hipLaunchKernelGGL(x8_kernel<3>, dim3(2 * B), dim3(64), 0, 0, base, out, sink); }, reps));
        report("x8 stride 1024 (1 KiB slots) in place", all,
               median_ms([&] { hipLaunchKernelGGL(x8s_kernel<1024>, dim3(2 * B), dim3(64), 0, 0, base); }, reps));
        report("x8 stride 1008 in place", all,
               median_ms([&] { hipLaunchKernelGGL(x8s_kernel<1008>, dim3(2 * B), dim3(64), 0, 0, base); }, reps));
        report("xpair stride 1000, 8-byte loads, per-shard 16-byte-aligned paired stores", all,
               median_ms([&] { hipLaunchKernelGGL(xpair_kernel, dim3(2 * B), dim3(64), 0, 0, base); }, reps));
        report("xal stride 1000, parity region as aligned 16-byte stores", all,
               median_ms([&] { hipLaunchKernelGGL(xal_kernel, dim3(2 * B), dim3(64), 0, 0, base); }, reps));
        const size_t n = size_t(16) << 30;
        report("copy 16 GB -> second pool", 2.0 * n,
               median_ms([&] { hipLaunchKernelGGL(copy_kernel, dim3(uint32_t(n / 1024)), dim3(64), 0, 0, base, out); }, reps));
    }
    return 0;
}
