// masked_ref.hip -- memory reference for the per-stripe-pattern decode (row f2):
// the access pattern of gf_masked_kernel with XOR in place of the GF products.
// Per stripe, from its presence bitmask: load the first K present shards' 16-B
// vectors (all up front, as the product kernel does), XOR them, store the
// result into every absent shard (at most MS).  Same wave shape, one-shot grid
// and chunk rotation as the product kernel, so a probe running both on one pool
// (tools/masked_ref_probe.py) separates the pattern's cost from the kernel's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC tools/masked_ref.hip -o tools/bin/libmasked_ref.so
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct RefArgs {
    uint8_t *base;
    const uint32_t *bits;
    uint64_t stripe_stride, shard_stride;
    uint32_t chunks, nvec, rot;
};

template <int K, int T, int MS>
__global__ void __launch_bounds__(64) masked_xor_ref(RefArgs a) {
    const uint32_t b = blockIdx.x;
    const uint32_t stripe = b / a.chunks;
    uint32_t chunk = b - stripe * a.chunks;
    if (a.rot) chunk = uint32_t((uint64_t(chunk) + uint64_t(stripe) * a.rot) % a.chunks);
    const uint32_t v = chunk * 64u + threadIdx.x;
    const uint32_t bits = __builtin_amdgcn_readfirstlane(a.bits[stripe]) & ((1u << T) - 1u);
    if (__builtin_popcount(bits) < K || bits == (1u << T) - 1u || v >= a.nvec) return;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(v) * 16u;
    u32x4 x[K];
    uint32_t rem = bits;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const int i = __builtin_ctz(rem);
        rem &= rem - 1u;
        x[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(sb + uint64_t(i) * a.shard_stride));
    }
    u32x4 acc = x[0];
#pragma unroll
    for (int j = 1; j < K; ++j) acc ^= x[j];
    uint32_t miss = ~bits & ((1u << T) - 1u);
#pragma unroll
    for (int p = 0; p < MS; ++p) {
        if (miss) {
            const int i = __builtin_ctz(miss);
            miss &= miss - 1u;
            __builtin_nontemporal_store(acc ^ uint32_t(p), reinterpret_cast<u32x4 *>(sb + uint64_t(i) * a.shard_stride));
        }
    }
}
}  // namespace

// 10+4 only (the f2 bench geometry); shard_len a multiple of 1 KiB.
extern "C" int masked_ref_launch(uint8_t *base, const uint32_t *bits, uint32_t n_stripes, uint64_t shard_len,
                                 uint64_t shard_stride, uint64_t stripe_stride, uint32_t rot, hipStream_t s) {
    if (shard_len % 1024 || !n_stripes) return 1;
    RefArgs a{base, bits, stripe_stride, shard_stride, uint32_t(shard_len / 1024), uint32_t(shard_len / 16), rot};
    const uint64_t blocks = uint64_t(n_stripes) * a.chunks;
    if (blocks >= (1ull << 31)) return 1;
    hipLaunchKernelGGL((masked_xor_ref<10, 14, 4>), dim3(uint32_t(blocks)), dim3(64), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
