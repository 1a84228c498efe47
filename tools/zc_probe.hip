// zc_probe.hip -- can a kernel code host-resident shards over PCIe faster than
// the DMA pipeline (host.cpp run_chunks: 0.86 of the link bound)?
//
// The pipeline's 4+2 x 64 MiB encode moves 256 MiB up and 128 MiB down in 48
// hipMemcpyAsync calls; the measured time sits ~0.5 ms above the link bound,
// about 10 us per copy.  A kernel that loads the data shards straight from
// page-locked host memory and stores the parity straight back has no copies
// at all and keeps both link directions busy at once.  Legs (all pinned,
// hipHostMalloc; `reg` = malloc + hipHostRegister, as the JNI path pins):
//   dma_up / dma_down / dma_both   hipMemcpyAsync of the same bytes
//   zc_read / zc_write             kernel-side loads only / stores only
//   zc_xor42 (blocks, vec)         4 loads -> 2 stores per column (encode traffic)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/zc_probe.hip -o build/probes/zc_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

struct Ptrs {
    const uint8_t *in[4];
    uint8_t *out[2];
};

// Grid-stride over 16-byte columns; V vectors per lane in flight per shard.
template <int V, int MODE>  // MODE 0: encode traffic, 1: loads only, 2: stores only
__global__ void __launch_bounds__(256) zc_kernel(Ptrs p, uint64_t nvec, uint32_t *sink) {
    const uint64_t step = uint64_t(gridDim.x) * blockDim.x * V;
    uint32_t s = 0;
    for (uint64_t v0 = (uint64_t(blockIdx.x) * blockDim.x * V) + threadIdx.x; v0 < nvec; v0 += step) {
        u32x4 x[4][V];
        if (MODE != 2) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const uint64_t v = v0 + uint64_t(j) * blockDim.x;
                    x[i][j] = v < nvec ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p.in[i]) + v)
                                       : u32x4{0, 0, 0, 0};
                }
        }
        if (MODE == 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < V; ++j) s ^= x[i][j][0] ^ x[i][j][3];
            continue;
        }
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const uint64_t v = v0 + uint64_t(j) * blockDim.x;
            if (v >= nvec) continue;
            u32x4 a = MODE == 2 ? u32x4{uint32_t(v), 1, 2, 3} : (x[0][j] ^ x[1][j] ^ x[2][j] ^ x[3][j]);
            u32x4 b = MODE == 2 ? a : (x[0][j] ^ (x[1][j] + x[2][j]) ^ x[3][j]);
            __builtin_nontemporal_store(a, reinterpret_cast<u32x4 *>(p.out[0]) + v);
            __builtin_nontemporal_store(b, reinterpret_cast<u32x4 *>(p.out[1]) + v);
        }
    }
    if (s == 0x9E3779B9u) sink[0] = s;
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

void report(const char *mem, const char *name, double up, double down, double ms) {
    std::printf("%-5s %-36s %8.3f ms  up %6.2f GB/s  down %6.2f GB/s  user(4 data shards) %6.2f GiB/s\n", mem, name,
                ms, up / ms / 1e6, down / ms / 1e6, up / ms * 1e3 / double(1 << 30));
    std::fflush(stdout);
}

template <int V, int MODE>
double run_zc(const Ptrs &p, uint64_t nvec, uint32_t *sink, int blocks, int reps) {
    return median_ms([&] { hipLaunchKernelGGL((zc_kernel<V, MODE>), dim3(blocks), dim3(256), 0, 0, p, nvec, sink); }, reps);
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    const size_t n = size_t(64) << 20;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    uint32_t *sink = nullptr;
    CHECK(hipMalloc(&sink, 256));
    uint8_t *dev = nullptr;
    CHECK(hipMalloc(&dev, 6 * n));
    for (int mem = 0; mem < 2; ++mem) {
        uint8_t *h[6];
        for (int i = 0; i < 6; ++i) {
            if (mem == 0) {
                CHECK(hipHostMalloc(reinterpret_cast<void **>(&h[i]), n, hipHostMallocDefault));
            } else {
                h[i] = static_cast<uint8_t *>(std::aligned_alloc(4096, n));
                CHECK(hipHostRegister(h[i], n, hipHostRegisterMapped));
            }
            std::memset(h[i], 0x11 * (i + 1), n);
        }
        Ptrs p;
        for (int i = 0; i < 4; ++i) {
            void *d = nullptr;
            CHECK(hipHostGetDevicePointer(&d, h[i], 0));
            p.in[i] = static_cast<const uint8_t *>(d);
        }
        for (int i = 0; i < 2; ++i) {
            void *d = nullptr;
            CHECK(hipHostGetDevicePointer(&d, h[4 + i], 0));
            p.out[i] = static_cast<uint8_t *>(d);
        }
        const char *mname = mem ? "reg" : "pin";
        hipStream_t s1, s2;
        CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
        CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        const double up = 4.0 * n, down = 2.0 * n;
        report(mname, "dma_up (4 x 64 MiB)", up, 0, median_ms([&] {
                   for (int i = 0; i < 4; ++i) CHECK(hipMemcpyAsync(dev + i * n, h[i], n, hipMemcpyHostToDevice, 0));
               }, reps));
        report(mname, "dma_down (2 x 64 MiB)", 0, down, median_ms([&] {
                   for (int i = 0; i < 2; ++i) CHECK(hipMemcpyAsync(h[4 + i], dev + (4 + i) * n, n, hipMemcpyDeviceToHost, 0));
               }, reps));
        report(mname, "dma_both (two streams)", up, down, median_ms([&] {
                   hipEvent_t ev;
                   CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                   CHECK(hipEventRecord(ev, 0));
                   CHECK(hipStreamWaitEvent(s1, ev, 0));
                   CHECK(hipStreamWaitEvent(s2, ev, 0));
                   for (int i = 0; i < 4; ++i) CHECK(hipMemcpyAsync(dev + i * n, h[i], n, hipMemcpyHostToDevice, s1));
                   for (int i = 0; i < 2; ++i) CHECK(hipMemcpyAsync(h[4 + i], dev + (4 + i) * n, n, hipMemcpyDeviceToHost, s2));
                   hipEvent_t a, b;
                   CHECK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
                   CHECK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
                   CHECK(hipEventRecord(a, s1));
                   CHECK(hipEventRecord(b, s2));
                   CHECK(hipStreamWaitEvent(0, a, 0));
                   CHECK(hipStreamWaitEvent(0, b, 0));
                   CHECK(hipEventDestroy(a));
                   CHECK(hipEventDestroy(b));
                   CHECK(hipEventDestroy(ev));
               }, reps));
        const uint64_t nvec = n / 16;
        for (int blocks : {256, 512, 1024, 2048, 4096}) {
            char name[64];
            std::snprintf(name, sizeof name, "zc_read  blocks=%d V=1", blocks);
            report(mname, name, up, 0, run_zc<1, 1>(p, nvec, sink, blocks, reps));
            std::snprintf(name, sizeof name, "zc_write blocks=%d V=1", blocks);
            report(mname, name, 0, down, run_zc<1, 2>(p, nvec, sink, blocks, reps));
            std::snprintf(name, sizeof name, "zc_xor42 blocks=%d V=1", blocks);
            report(mname, name, up, down, run_zc<1, 0>(p, nvec, sink, blocks, reps));
            std::snprintf(name, sizeof name, "zc_xor42 blocks=%d V=2", blocks);
            report(mname, name, up, down, run_zc<2, 0>(p, nvec, sink, blocks, reps));
            std::snprintf(name, sizeof name, "zc_xor42 blocks=%d V=4", blocks);
            report(mname, name, up, down, run_zc<4, 0>(p, nvec, sink, blocks, reps));
        }
        CHECK(hipStreamDestroy(s1));
        CHECK(hipStreamDestroy(s2));
        for (int i = 0; i < 6; ++i) {
            if (mem == 0) {
                CHECK(hipHostFree(h[i]));
            } else {
                CHECK(hipHostUnregister(h[i]));
                std::free(h[i]);
            }
        }
    }
    return 0;
}
