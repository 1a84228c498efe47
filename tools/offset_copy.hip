// offset_copy.hip -- does the relative offset between a read stream and a
// write stream change the copy rate?  If the read/write interleaving cost of
// the coding kernels is per HBM channel, a copy whose source and destination
// sit in the same channel at the same moment should run slower than one whose
// destination is shifted into other channels.  Copies 2 GiB from `src` to
// `src + 2 GiB + d` for d over 0-8 KiB in 256-B steps and powers of two up to
// 64 MiB, with the coding kernels' shape (one wave per 1 KiB chunk, 16-B
// non-temporal loads and stores, XCD-contiguous block order), warmed up.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/offset_copy.hip -o tools/bin/offset_copy
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

__global__ void __launch_bounds__(64) copy_kernel(const uint8_t *src, uint8_t *dst, uint32_t xcd_span) {
    uint32_t b = blockIdx.x;
    if (xcd_span && b < 8u * xcd_span) b = (b & 7u) * xcd_span + (b >> 3);
    const uint64_t o = uint64_t(b) * 1024 + threadIdx.x * 16u;
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + o));
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(dst + o));
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    const size_t n = size_t(2) << 30, maxd = size_t(64) << 20;
    uint8_t *buf = nullptr;
    CHECK(hipMalloc(&buf, 2 * n + maxd + 4096));
    CHECK(hipMemset(buf, 0x11, 2 * n + maxd + 4096));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const uint32_t blocks = uint32_t(n / 1024);
    std::vector<size_t> ds;
    for (size_t d = 0; d <= 8192; d += 256) ds.push_back(d);
    for (size_t d = 16384; d <= maxd; d *= 2) ds.push_back(d);
    for (int pass = 0; pass < 2; ++pass)
        for (size_t d : ds) {
            for (int order = 0; order < 2; ++order) {
                const uint32_t span = order ? blocks / 8u : 0u;
                auto launch = [&] { hipLaunchKernelGGL(copy_kernel, dim3(blocks), dim3(64), 0, 0, buf, buf + n + d, span); };
                for (int w = 0; w < 20; ++w) launch();
                CHECK(hipGetLastError());
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
                const double ms = ts[ts.size() / 2];
                std::printf("pass %d d %9zu %-5s %.3f ms  %.3f of 8 TB/s\n", pass, d, order ? "xcd" : "plain", ms,
                            2.0 * n / ms / 1e6 / 8000.0);
                std::fflush(stdout);
            }
        }
    CHECK(hipFree(buf));
    return 0;
}
