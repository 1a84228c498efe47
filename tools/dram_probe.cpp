// dram_probe.cpp -- host DRAM copy bandwidth on one NUMA node, CPU only (no
// GPU): the ceiling under the pageable host calls' copies.
//
// Bound to the CPUs given (argv[1], a cpulist; memory first-touched after the
// bind, so it lies on that node), it times over ~2 s each:
//   read_T      T threads summing a 1 GiB buffer (DRAM read bandwidth)
//   memcpy_T    T threads memcpy 1 GiB -> 1 GiB (bytes copied per second)
//   pool        the library's own copy pool (csrc/copy_pool.cpp, compiled in):
//               batches of 6 x 16 MiB jobs, 32-byte streaming stores, its 15
//               workers + the caller -- the copies of a pageable encodeParity
//   pool_4k     the same with the source on 4 KiB pages (MADV_NOHUGEPAGE; a
//               JVM heap without -XX:+UseTransparentHugePages), else THP
//   gather      the pool's gather of 1000-byte rows 4000 bytes apart into
//               contiguous shards (a file encode's split)
// and prints one JSON line.  Bytes: copies count each byte once (DRAM moves
// it twice: read + write, no read-for-ownership with streaming stores).
//
// argv[2] == "pool": the pool and gather legs only.  Build:
//   g++ -O2 -std=c++17 -pthread -Ijava-reed-solomon-distributed-file-system_amd/csrc \
//       tools/dram_probe.cpp java-reed-solomon-distributed-file-system_amd/csrc/copy_pool.cpp \
//       -o build/probes/dram_probe
#include <sched.h>
#include <sys/mman.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "copy_pool.hpp"

namespace {
double secs_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

uint8_t *alloc(size_t n, bool huge) {
    void *p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) std::exit(1);
    madvise(p, n, huge ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
    return static_cast<uint8_t *>(p);
}

// first touch from T threads (pages land on the bound node)
void touch(uint8_t *p, size_t n, int T) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([=] {
            const size_t a = n / T * t, b = t == T - 1 ? n : n / T * (t + 1);
            std::memset(p + a, int(t + 1), b - a);
        });
    for (auto &x : th) x.join();
}

template <class Fn>
double rate_mt(int T, size_t bytes_per_pass, Fn fn) {  // GB/s over >= 2 s
    size_t passes = 0;
    const auto t0 = std::chrono::steady_clock::now();
    while (secs_since(t0) < 2.0) {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back([&, t] { fn(t); });
        for (auto &x : th) x.join();
        ++passes;
    }
    return double(bytes_per_pass) * passes / secs_since(t0) / 1e9;
}

std::vector<int> cpulist(const char *s) {
    std::vector<int> out;
    std::string str(s);
    size_t i = 0;
    while (i < str.size()) {
        size_t j = str.find(',', i);
        if (j == std::string::npos) j = str.size();
        const std::string part = str.substr(i, j - i);
        const size_t d = part.find('-');
        const int a = std::atoi(part.c_str()), b = d == std::string::npos ? a : std::atoi(part.c_str() + d + 1);
        for (int c = a; c <= b; ++c) out.push_back(c);
        i = j + 1;
    }
    return out;
}
}  // namespace

int main(int argc, char **argv) {
    if (argc > 1) {
        cpu_set_t set;
        CPU_ZERO(&set);
        for (int c : cpulist(argv[1])) CPU_SET(c, &set);
        if (sched_setaffinity(0, sizeof set, &set)) return 2;
    }
    const size_t n = size_t(1) << 30;
    uint8_t *src = alloc(n, true), *dst = alloc(n, true), *src4k = alloc(n, false);
    touch(src, n, 16);
    touch(dst, n, 16);
    touch(src4k, n, 16);
    const bool pool_only = argc > 2 && std::string(argv[2]) == "pool";  // the pool and the gather only
    std::printf("{\"cpus\": \"%s\"", argc > 1 && std::strlen(argv[1]) < 200 ? argv[1] : "(node)");
    for (int T : {1, 2, 4, 8, 16}) {
        if (pool_only) break;
        std::atomic<uint64_t> sink{0};
        const double r = rate_mt(T, n, [&](int t) {
            const uint64_t *p = reinterpret_cast<const uint64_t *>(src + n / T * t);
            uint64_t s = 0;
            for (size_t i = 0; i < n / T / 8; i += 8) s += p[i] ^ p[i + 1] ^ p[i + 2] ^ p[i + 3] ^ p[i + 4] ^ p[i + 5] ^ p[i + 6] ^ p[i + 7];
            sink += s;
        });
        const double c = rate_mt(T, n, [&](int t) { std::memcpy(dst + n / T * t, src + n / T * t, n / T); });
        std::printf(", \"read_%d_GBps\": %.1f, \"memcpy_%d_GBps\": %.1f", T, r, T, c);
    }
    rsamd::CopyPool &pool = rsamd::CopyPool::get();
    for (int which = 0; which < 2; ++which) {
        const uint8_t *s = which ? src4k : src;
        const size_t job = size_t(16) << 20;
        size_t bytes = 0, at = 0;
        const auto t0 = std::chrono::steady_clock::now();
        while (secs_since(t0) < 2.0) {
            std::vector<rsamd::CopyJob> jobs;
            for (int j = 0; j < 6; ++j, at = (at + job) % n) jobs.push_back({dst + at, s + at, job});
            pool.copy(jobs);
            bytes += 6 * job;
        }
        std::printf(", \"%s_GBps\": %.1f", which ? "pool_4k" : "pool", double(bytes) / secs_since(t0) / 1e9);
    }
    {  // the file split's gather: 1000-B rows 4000 B apart -> 4 contiguous shards of a 256 MiB file
        const size_t blk = 1000, rows = (size_t(256) << 20) / (4 * blk);
        size_t bytes = 0;
        const auto t0 = std::chrono::steady_clock::now();
        while (secs_since(t0) < 2.0) {
            std::vector<rsamd::CopyJob> jobs;
            for (size_t b0 = 0; b0 < rows; b0 += 256)
                for (int i = 0; i < 4; ++i) {
                    const size_t nr = std::min<size_t>(256, rows - b0);
                    jobs.push_back({dst + size_t(i) * rows * blk + b0 * blk, src + (b0 * 4 + size_t(i)) * blk, blk, nr,
                                    blk, 4 * blk});
                }
            pool.copy(jobs);
            bytes += rows * 4 * blk;
        }
        std::printf(", \"gather_GBps\": %.1f", double(bytes) / secs_since(t0) / 1e9);
    }
    std::printf(", \"pool_threads\": %d}\n", pool.workers() + 1);
    return 0;
}
