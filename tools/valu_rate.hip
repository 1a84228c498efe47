// valu_rate.hip -- issue rate of the VALU instructions the coding kernels are
// made of (v_perm_b32, v_bitop3_b32, v_bfi_b32, v_xor_b32, v_lshlrev_b32), on
// every CU at 8 waves per SIMD, 8 independent accumulator chains per wave, and
// one dependent chain at 1 wave per SIMD (latency).  Prints wave64
// instructions per SIMD per cycle (cycles from s_memtime inside the kernel;
// the wall clock gives the effective clock).
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/bin/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

constexpr int kIters = 4096;

#define OP_XOR(d, a, b) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b))
#define OP_BITOP3(d, a, b) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(d))
#define OP_BITOP3S(d, a, b) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xd8" : "=v"(d) : "v"(a), "v"(b), "s"(smask))
#define OP_PERM(d, a, b) asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(d))
#define OP_PERMS(d, a, b) asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(d) : "s"(smask), "v"(b), "v"(a))
#define OP_BFI(d, a, b) asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(d) : "s"(smask), "v"(a), "v"(d))
#define OP_SHL(d, a, b) asm volatile("v_lshlrev_b32 %0, 3, %1" : "=v"(d) : "v"(a))

#define KERNEL(NAME, OP)                                                                         \
    __global__ void __launch_bounds__(256) NAME(unsigned *out, unsigned seed, unsigned smask,   \
                                                unsigned smask2, unsigned long long *cyc) {     \
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11,   \
                 a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19, x = seed * 23 + threadIdx.x, y = x * 29; \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                              \
        for (int i = 0; i < kIters; ++i) {                                                       \
            OP(a0, x, y); OP(a1, y, x); OP(a2, x, y); OP(a3, y, x);                              \
            OP(a4, x, y); OP(a5, y, x); OP(a6, x, y); OP(a7, y, x);                              \
        }                                                                                        \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                              \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
        if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                        \
    }                                                                                            \
    __global__ void __launch_bounds__(64) NAME##_chain(unsigned *out, unsigned seed, unsigned smask, \
                                                       unsigned smask2, unsigned long long *cyc) { \
        unsigned a0 = threadIdx.x ^ seed, x = seed * 23 + threadIdx.x, y = x * 29;               \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                              \
        for (int i = 0; i < kIters; ++i) {                                                       \
            OP(a0, x, y); OP(a0, y, a0); OP(a0, x, a0); OP(a0, a0, y);                           \
            OP(a0, x, a0); OP(a0, y, a0); OP(a0, a0, y); OP(a0, x, a0);                          \
        }                                                                                        \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                              \
        out[blockIdx.x * 64 + threadIdx.x] = a0;                                                 \
        if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                        \
    }

KERNEL(k_xor, OP_XOR)
KERNEL(k_bitop3, OP_BITOP3)
KERNEL(k_bitop3s, OP_BITOP3S)
KERNEL(k_perm, OP_PERM)
KERNEL(k_perms, OP_PERMS)
KERNEL(k_bfi, OP_BFI)
KERNEL(k_shl, OP_SHL)

typedef void (*Kern)(unsigned *, unsigned, unsigned, unsigned, unsigned long long *);

int run(const char *name, Kern k, Kern chain, unsigned *out, unsigned long long *cyc, unsigned long long *hcyc) {
    const int cus = 256, blocks = cus * 8;  // 256-thread blocks, 8 per CU = 8 waves per SIMD
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1u, 0x0F0F0F0Fu, 0x03020100u, cyc);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 2u, 0x0F0F0F0Fu, 0x03020100u, cyc);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipMemcpy(hcyc, cyc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double avg = 0;
    for (int b = 0; b < blocks; ++b) avg += double(hcyc[b]);
    avg /= blocks;
    // per SIMD: 8 waves x kIters x 8 instructions
    const double instr_per_simd = 8.0 * kIters * 8;
    const double wall_ghz_equiv = instr_per_simd / (ms * 1e6);  // instructions per ns per SIMD
    hipLaunchKernelGGL(chain, dim3(cus * 4), dim3(64), 0, 0, out, 3u, 0x0F0F0F0Fu, 0x03020100u, cyc);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(hcyc, cyc, cus * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double lat = 0;
    for (int b = 0; b < cus * 4; ++b) lat += double(hcyc[b]);
    lat /= cus * 4;
    std::printf("%-10s throughput: %.3f instr/cycle/SIMD (s_memtime), %.3f instr/ns/SIMD (wall %.3f ms); "
                "dependent chain: %.2f cycles/instr\n",
                name, instr_per_simd / avg, wall_ghz_equiv, ms, lat / (kIters * 8.0));
    return 0;
}

int main() {
    unsigned *out;
    unsigned long long *cyc;
    static unsigned long long hcyc[256 * 8];
    CHECK(hipMalloc(&out, 256 * 8 * 256 * sizeof(unsigned)));
    CHECK(hipMalloc(&cyc, 256 * 8 * sizeof(unsigned long long)));
    if (run("xor", k_xor, k_xor_chain, out, cyc, hcyc) || run("bitop3", k_bitop3, k_bitop3_chain, out, cyc, hcyc) ||
        run("bitop3_s", k_bitop3s, k_bitop3s_chain, out, cyc, hcyc) ||
        run("perm", k_perm, k_perm_chain, out, cyc, hcyc) || run("perm_ss", k_perms, k_perms_chain, out, cyc, hcyc) ||
        run("bfi_s", k_bfi, k_bfi_chain, out, cyc, hcyc) || run("lshl", k_shl, k_shl_chain, out, cyc, hcyc))
        return 1;
    CHECK(hipFree(out));
    CHECK(hipFree(cyc));
    return 0;
}
