// pool_batch_probe.cpp -- per-batch time of the copy pool against the calling
// thread alone (CPU only): `njobs` jobs of n bytes, 3000 batches with a 10 us
// gap between them (a small call's GPU part), median and p90 microseconds.
//   g++ -O2 -std=c++17 -pthread -Ijava-reed-solomon-distributed-file-system_amd/csrc
//       tools/pool_batch_probe.cpp java-reed-solomon-distributed-file-system_amd/csrc/copy_pool.cpp
//       -o build/probes/pool_batch_probe
//   build/probes/pool_batch_probe N NJOBS
#include "copy_pool.hpp"
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
using namespace rsamd;
int main(int argc, char **argv) {
    size_t n = argc > 1 ? atol(argv[1]) : 65536;
    int njobs = argc > 2 ? atoi(argv[2]) : 4;
    std::vector<std::vector<uint8_t>> src(njobs, std::vector<uint8_t>(n, 1)), dst(njobs, std::vector<uint8_t>(n));
    std::vector<CopyJob> jobs;
    for (int i = 0; i < njobs; ++i) jobs.push_back({dst[i].data(), src[i].data(), n});
    auto &pool = CopyPool::get();
    for (int mode = 0; mode < 2; ++mode) {
        std::vector<double> t;
        for (int it = 0; it < 3000; ++it) {
            auto t0 = std::chrono::steady_clock::now();
            if (mode) pool.copy(jobs); else CopyPool::copy_here(jobs);
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
            // gap like a small call's GPU part
            auto g0 = std::chrono::steady_clock::now();
            while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - g0).count() < 10) {}
        }
        std::sort(t.begin(), t.end());
        printf("%s n=%zu jobs=%d median %.2f us p90 %.2f\n", mode ? "pool" : "here", n, njobs, t[t.size()/2], t[t.size()*9/10]);
    }
}
