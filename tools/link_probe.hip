// Host<->device link rates by mechanism: SDMA async copies (hipMemcpyAsync)
// against copy kernels that read or write page-locked host memory through its
// device mapping, one direction and both at once.  Decides how the host
// pipeline (capi.cpp run_chunks) should move its chunk outputs.
//   hipcc -O3 --offload-arch=gfx950 tools/link_probe.hip -o tools/bin/link_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Segment copy: blockIdx.y selects the segment, grid-stride over 16-B words.
struct Seg {
    const u32x4 *src;
    u32x4 *dst;
    size_t n16;
};
struct Segs {
    Seg s[8];
};

__global__ void __launch_bounds__(256) seg_copy(Segs a) {
    const Seg g = a.s[blockIdx.y];
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < g.n16; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(g.src + i), g.dst + i);
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t seg = size_t(8) << 20, nseg = 6, reps = 10;
    const size_t total = seg * nseg;
    uint8_t *h_in, *h_out, *d_in, *d_out;
    CK(hipHostMalloc(reinterpret_cast<void **>(&h_in), total, hipHostMallocMapped));
    CK(hipHostMalloc(reinterpret_cast<void **>(&h_out), total, hipHostMallocMapped));
    std::memset(h_in, 1, total);
    std::memset(h_out, 2, total);
    // registered pageable memory, as HostRegistration does it
    uint8_t *r_out = static_cast<uint8_t *>(std::aligned_alloc(4096, total));
    std::memset(r_out, 3, total);
    CK(hipHostRegister(r_out, total, hipHostRegisterDefault));
    uint8_t *r_out_dev = nullptr, *h_in_dev = nullptr, *h_out_dev = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&r_out_dev), r_out, 0));
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&h_in_dev), h_in, 0));
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&h_out_dev), h_out, 0));
    std::printf("registered host %p -> device %p; hostmalloc %p -> %p\n", (void *)r_out, (void *)r_out_dev,
                (void *)h_out, (void *)h_out_dev);
    CK(hipMalloc(reinterpret_cast<void **>(&d_in), total));
    CK(hipMalloc(reinterpret_cast<void **>(&d_out), total));
    CK(hipMemset(d_out, 4, total));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));

    auto sdma_h2d = [&](hipStream_t s) {
        for (size_t i = 0; i < nseg; ++i) CK(hipMemcpyAsync(d_in + i * seg, h_in + i * seg, seg, hipMemcpyHostToDevice, s));
    };
    auto sdma_d2h = [&](hipStream_t s, uint8_t *dst) {
        for (size_t i = 0; i < nseg; ++i) CK(hipMemcpyAsync(dst + i * seg, d_out + i * seg, seg, hipMemcpyDeviceToHost, s));
    };
    auto kern = [&](hipStream_t s, const uint8_t *src, uint8_t *dst, int blocks) {
        Segs a{};
        for (size_t i = 0; i < nseg; ++i)
            a.s[i] = {reinterpret_cast<const u32x4 *>(src + i * seg), reinterpret_cast<u32x4 *>(dst + i * seg), seg / 16};
        hipLaunchKernelGGL(seg_copy, dim3(blocks, nseg), dim3(256), 0, s, a);
        CK(hipGetLastError());
    };
    auto run = [&](const char *name, double bytes_per_rep, auto &&body) {
        body();
        CK(hipDeviceSynchronize());
        const double t0 = now();
        for (size_t r = 0; r < reps; ++r) body();
        CK(hipDeviceSynchronize());
        const double t = (now() - t0) / reps;
        std::printf("%-48s %8.1f GB/s  (%.3f ms per rep)\n", name, bytes_per_rep / t / 1e9, t * 1e3);
        std::fflush(stdout);
    };
    const double B = double(total);
    run("sdma h2d (6 x 8 MiB)", B, [&] { sdma_h2d(s1); });
    run("sdma d2h hostmalloc", B, [&] { sdma_d2h(s2, h_out); });
    run("sdma d2h registered", B, [&] { sdma_d2h(s2, r_out); });
    run("sdma h2d + sdma d2h registered", 2 * B, [&] { sdma_h2d(s1); sdma_d2h(s2, r_out); });
    for (int blocks : {16, 32, 64, 128, 256, 1024}) {
        char name[96];
        std::snprintf(name, sizeof name, "kernel d2h registered, %d x 6 blocks", blocks);
        run(name, B, [&] { kern(s2, d_out, r_out_dev, blocks); });
        std::snprintf(name, sizeof name, "kernel h2d hostmalloc, %d x 6 blocks", blocks);
        run(name, B, [&] { kern(s1, h_in_dev, d_in, blocks); });
        std::snprintf(name, sizeof name, "sdma h2d + kernel d2h reg, %d x 6 blocks", blocks);
        run(name, 2 * B, [&] { sdma_h2d(s1); kern(s2, d_out, r_out_dev, blocks); });
        std::snprintf(name, sizeof name, "kernel h2d + kernel d2h reg, %d x 6 blocks", blocks);
        run(name, 2 * B, [&] { kern(s1, h_in_dev, d_in, blocks); kern(s2, d_out, r_out_dev, blocks); });
    }
    // check the kernel wrote the registered buffer
    CK(hipMemset(d_out, 7, total));
    CK(hipDeviceSynchronize());  // s2 is non-blocking: order it after the memset
    kern(s2, d_out, r_out_dev, 64);
    CK(hipDeviceSynchronize());
    size_t bad = 0;
    for (size_t i = 0; i < total; ++i) bad += r_out[i] != 7;
    std::printf("kernel d2h check: %zu bad bytes\n", bad);
    CK(hipHostUnregister(r_out));
    std::free(r_out);
    return bad != 0;
}
