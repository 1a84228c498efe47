// Host memcpy bandwidth between pageable and pinned (hipHostMalloc) memory
// with 1..16 threads -- the ceiling of staging pageable buffers ourselves.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double run(uint8_t *dst, const uint8_t *src, size_t n, int nt, int reps) {
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) {
        std::vector<std::thread> th;
        const size_t per = (n + nt - 1) / nt;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([=] {
                const size_t a = std::min(n, t * per), b = std::min(n, (t + 1) * per);
                std::memcpy(dst + a, src + a, b - a);
            });
        for (auto &x : th) x.join();
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return double(n) * reps / s / 1e9;
}

int main() {
    const size_t n = size_t(256) << 20;
    uint8_t *page = static_cast<uint8_t *>(std::malloc(n));
    uint8_t *page2 = static_cast<uint8_t *>(std::malloc(n));
    uint8_t *pin = nullptr;
    if (hipHostMalloc(reinterpret_cast<void **>(&pin), n, hipHostMallocDefault) != hipSuccess) return 1;
    std::memset(page, 1, n);
    std::memset(page2, 2, n);
    std::memset(pin, 3, n);
    for (int nt : {1, 2, 4, 8, 16}) {
        const double in = run(pin, page, n, nt, 4), out = run(page2, pin, n, nt, 4), pp = run(page2, page, n, nt, 4);
        std::printf("threads %2d  pageable->pinned %6.1f GB/s  pinned->pageable %6.1f GB/s  pageable->pageable %6.1f GB/s\n",
                    nt, in, out, pp);
    }
    return 0;
}
