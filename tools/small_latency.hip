// small_latency.hip -- where a small host call's time goes.
//
// Times, from C (no Python in the loop), per call in microseconds (median of
// N calls after warm-up):
//   lib_dec1000     rs_decode_missing 4+2 x 1000 B, {0} absent (the recovery
//                   machine's call, ChunkserverDiskRecoveryMachine.java:44)
//   lib_dec1000_05  the same, {0,5} absent
//   lib_enc4k       rs_encode_parity 4+2 x 4 KiB
//   lib_enc64k      rs_encode_parity 4+2 x 64 KiB
//   lib_fencF, lib_fdecF_0, lib_fdecF_05
//                   rs_file_encode / rs_file_decode ({0}, {0,5} absent) of an
//                   F-byte file, 1000-byte blocks (the client's small files)
// and the pieces such a call is made of, on this process's own stream:
//   launch_only     hipLaunchKernelGGL of an empty kernel, no wait (host cost)
//   empty_sync      empty kernel + hipStreamSynchronize
//   empty_query     empty kernel + hipEventRecord + spin on hipEventQuery
//   empty_flag      one-wave kernel stores a sequence number into coherent
//                   host memory; the CPU spins on it (no runtime wait)
//   xor_sync_S      memcpy 4 x S in -> kernel over the mapped buffer (4 loads,
//                   2 stores per 16 B) -> hipStreamSynchronize -> memcpy 2 x S out
//   xor_flag_S      the same, the kernel's last block storing the flag
//   graph_sync      the xor kernel as a one-node hipGraph + hipStreamSynchronize
// argv[1] == "spin": hipSetDeviceFlags(hipDeviceScheduleSpin) first.
// SL_SIZES=a,b,... replaces the encode / verify shard sizes 4096 and 65536.
// argv[1] == "lib200": only 200 calls of each library call (for a rocprofv3
// --kernel-trace --memory-copy-trace --hip-runtime-trace of exactly those).
//
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/small_latency.hip \
//          -Iinclude -Ljava-reed-solomon-distributed-file-system_amd/lib -lrsamd \
//          -Wl,-rpath,$PWD/java-reed-solomon-distributed-file-system_amd/lib -o tools/bin/small_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "rs_amd.h"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

__global__ void empty_kernel() {}

__global__ void flag_kernel(uint32_t *flag, uint32_t seq) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 4 inputs, 2 outputs of n16 16-byte vectors, S apart, in mapped host memory.
// With flag: each block fences its stores at system scope and counts itself
// done; the last one stores seq into *flag (and resets the counter).
__global__ void xor_kernel(u32x4 *base, uint64_t stride16, uint64_t n16, uint32_t *ctr, uint32_t *flag,
                           uint32_t seq) {
    const uint64_t v = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (v < n16) {
        u32x4 a = base[v], b = base[stride16 + v], c = base[2 * stride16 + v], d = base[3 * stride16 + v];
        base[4 * stride16 + v] = a ^ b ^ c ^ d;
        base[5 * stride16 + v] = a ^ (b + c) ^ d;
    }
    if (!flag) return;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median_us(int reps, const std::function<void()> &fn) {
    for (int i = 0; i < 20; ++i) fn();
    std::vector<double> t(reps);
    for (int i = 0; i < reps; ++i) {
        const double t0 = now_us();
        fn();
        t[i] = now_us() - t0;
    }
    std::sort(t.begin(), t.end());
    return t[reps / 2];
}

static void spin_until(volatile uint32_t *flag, uint32_t seq) {
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
    }
}

int main(int argc, char **argv) {
    const std::string mode = argc > 1 ? argv[1] : "";
    if (mode == "spin") CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    CK(hipSetDevice(0));
    const int reps = mode == "lib200" ? 200 : 2000;
    std::printf("{\"mode\": \"%s\"", mode.c_str());

    // ---- library calls -------------------------------------------------------
    rs_codec *codec = nullptr;
    if (rs_codec_create(4, 2, &codec)) return 1;
    // SL_SIZES=a,b,...: the encode / verify shard sizes instead of 4096 and 65536
    std::vector<size_t> sizes{1000, 4096, 65536};
    if (const char *e = std::getenv("SL_SIZES")) {
        sizes.assign(1, 1000);
        for (const char *p = e; *p;) {
            char *end = nullptr;
            const size_t v = std::strtoull(p, &end, 10);
            if (end == p) break;
            if (v && v != 1000) sizes.push_back(v);
            p = *end == ',' ? end + 1 : end;
        }
    }
    for (size_t S : sizes) {
        std::vector<std::vector<uint8_t>> sh(6, std::vector<uint8_t>(S));
        for (int i = 0; i < 6; ++i)
            for (size_t b = 0; b < S; ++b) sh[i][b] = uint8_t(b * 7 + i * 13 + (b >> 8));
        uint8_t *p[6];
        int64_t lens[6];
        for (int i = 0; i < 6; ++i) {
            p[i] = sh[i].data();
            lens[i] = int64_t(S);
        }
        int rc = 0;
        if (S == 1000) {
            if (rs_encode_parity(codec, p, 6, lens, 0, int32_t(S))) return 1;
            const uint8_t pres0[6] = {0, 1, 1, 1, 1, 1}, pres05[6] = {0, 1, 1, 1, 1, 0};
            const double d0 = median_us(reps, [&] { rc |= rs_decode_missing(codec, p, 6, lens, pres0, 0, int32_t(S)); });
            const double d05 = median_us(reps, [&] { rc |= rs_decode_missing(codec, p, 6, lens, pres05, 0, int32_t(S)); });
            std::printf(", \"lib_dec1000\": %.2f, \"lib_dec1000_05\": %.2f", d0, d05);
        } else {
            const double e = median_us(reps, [&] { rc |= rs_encode_parity(codec, p, 6, lens, 0, int32_t(S)); });
            int ok = 0;
            const double v = median_us(reps, [&] { rc |= rs_is_parity_correct(codec, p, 6, lens, 0, int32_t(S), nullptr, 0, &ok); });
            if (!ok) {
                std::fprintf(stderr, "verify reported a mismatch after encode\n");
                return 1;
            }
            std::printf(", \"lib_enc%zuk\": %.2f, \"lib_ver%zuk\": %.2f", S >> 10, e, S >> 10, v);
        }
        if (rc) {
            std::fprintf(stderr, "library call failed: %s\n", rs_last_error_message());
            return 1;
        }
    }
    // the client's file calls on small files (1000-byte blocks): encode, and
    // decode with {0} and {0,5} absent
    for (size_t F : {size_t(90999), size_t(256) << 10, size_t(1) << 20}) {
        const size_t blk = 1000, S = (F + 4 * blk - 1) / (4 * blk) * blk;
        std::vector<uint8_t> file(F), back(F);
        for (size_t b = 0; b < F; ++b) file[b] = uint8_t(b * 31 + (b >> 9));
        std::vector<std::vector<uint8_t>> sh(6, std::vector<uint8_t>(S));
        uint8_t *p[6];
        int64_t lens[6];
        for (int i = 0; i < 6; ++i) {
            p[i] = sh[i].data();
            lens[i] = int64_t(S);
        }
        int rc = 0;
        const double e = median_us(reps / 4, [&] {
            rc |= rs_file_encode(codec, file.data(), int64_t(F), int32_t(blk), p, 6, lens);
        });
        const uint8_t pres0[6] = {0, 1, 1, 1, 1, 1}, pres05[6] = {0, 1, 1, 1, 1, 0};
        const double d0 = median_us(reps / 4, [&] {
            rc |= rs_file_decode(codec, p, 6, lens, pres0, int32_t(S), int32_t(blk), back.data(), int64_t(F));
        });
        const double d05 = median_us(reps / 4, [&] {
            rc |= rs_file_decode(codec, p, 6, lens, pres05, int32_t(S), int32_t(blk), back.data(), int64_t(F));
        });
        if (rc || back != file) {
            std::fprintf(stderr, "file call failed or wrong: %s\n", rs_last_error_message());
            return 1;
        }
        std::printf(", \"lib_fenc%zu\": %.2f, \"lib_fdec%zu_0\": %.2f, \"lib_fdec%zu_05\": %.2f", F, e, F, d0, F, d05);
    }
    rs_codec_destroy(codec);
    if (mode == "lib200") {
        std::printf("}\n");
        return 0;
    }

    // ---- the pieces ------------------------------------------------------------
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    uint32_t *hflag = nullptr, *dflag = nullptr, *ctr = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&hflag), 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&dflag), hflag, 0));
    CK(hipMalloc(reinterpret_cast<void **>(&ctr), 256));
    CK(hipMemset(ctr, 0, 256));
    *hflag = 0;
    uint32_t seq = 0;

    {  // host cost of a launch
        for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        CK(hipStreamSynchronize(s));
        const double t0 = now_us();
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        const double t1 = now_us();
        CK(hipStreamSynchronize(s));
        std::printf(", \"launch_only\": %.2f", (t1 - t0) / reps);
    }
    std::printf(", \"empty_sync\": %.2f", median_us(reps, [&] {
                    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
                    CK(hipStreamSynchronize(s));
                }));
    std::printf(", \"empty_query\": %.2f", median_us(reps, [&] {
                    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
                    CK(hipEventRecord(ev, s));
                    while (hipEventQuery(ev) == hipErrorNotReady) {
                    }
                }));
    std::printf(", \"empty_flag\": %.2f", median_us(reps, [&] {
                    ++seq;
                    hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, dflag, seq);
                    spin_until(hflag, seq);
                }));
    CK(hipStreamSynchronize(s));

    // the zero-copy buffer a small call stages through
    const size_t cap = size_t(6) << 20;
    uint8_t *zc = nullptr, *zc_dev = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&zc), cap, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&zc_dev), zc, 0));
    for (size_t S : {size_t(1024), size_t(4096), size_t(65536)}) {
        std::vector<std::vector<uint8_t>> sh(6, std::vector<uint8_t>(S, 1));
        const uint64_t n16 = S / 16;
        const unsigned grid = unsigned((n16 + 255) / 256);
        auto copy_in = [&] {
            for (int i = 0; i < 4; ++i) std::memcpy(zc + i * S, sh[i].data(), S);
        };
        auto copy_out = [&] {
            for (int i = 4; i < 6; ++i) std::memcpy(sh[i].data(), zc + i * S, S);
        };
        const double ts = median_us(reps, [&] {
            copy_in();
            hipLaunchKernelGGL(xor_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<u32x4 *>(zc_dev), S / 16, n16,
                               ctr, nullptr, 0u);
            CK(hipStreamSynchronize(s));
            copy_out();
        });
        const double tf = median_us(reps, [&] {
            copy_in();
            ++seq;
            hipLaunchKernelGGL(xor_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<u32x4 *>(zc_dev), S / 16, n16,
                               ctr, dflag, seq);
            spin_until(hflag, seq);
            copy_out();
        });
        CK(hipStreamSynchronize(s));
        // check the flagged path's outputs are the kernel's
        for (size_t b = 0; b < S; b += 997)
            if (sh[4][b] != uint8_t(1 ^ 1 ^ 1 ^ 1)) {
                std::fprintf(stderr, "xor_flag output wrong at %zu\n", b);
                return 1;
            }
        std::printf(", \"xor_sync_%zuk\": %.2f, \"xor_flag_%zuk\": %.2f", S >> 10, ts, S >> 10, tf);
    }
    {  // one-node graph
        const size_t S = 4096;
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        hipLaunchKernelGGL(xor_kernel, dim3(1), dim3(256), 0, s, reinterpret_cast<u32x4 *>(zc_dev), S / 16,
                           uint64_t(S / 16), ctr, nullptr, 0u);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        std::printf(", \"graph_sync\": %.2f", median_us(reps, [&] {
                        CK(hipGraphLaunch(ge, s));
                        CK(hipStreamSynchronize(s));
                    }));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    CK(hipStreamSynchronize(s));
    std::printf("}\n");
    CK(hipHostFree(zc));
    CK(hipHostFree(hflag));
    CK(hipFree(ctr));
    return 0;
}
