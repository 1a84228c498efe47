// copy_pool_check.cpp -- CPU check of the host copy pool (csrc/copy_pool.cpp):
// strided row copies into contiguous destinations (the streaming gather of
// a file's block rows into shard columns), with a second destination (the
// tee into the pinned slots), random row lengths, strides and alignments;
// every byte is compared with a plain copy and nothing past the destination
// may be written.  Then several threads hand the pool batches at once (the
// process-wide pool serves every concurrent call), more of them than it has
// batch slots, each batch checked.  Built
// and run by tests/test_copy_pool.py, with and without idle spinning.
#include "copy_pool.hpp"
#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>
int main() {  // copy_pool.cpp gathers, tees, zero fills: every byte against a plain copy
    std::mt19937_64 rng(1);
    int bad = 0, cases = 0;
    for (int it = 0; it < 3000; ++it) {
        size_t n = 1 + rng() % 5000, rows = 1 + rng() % 300, sstride = n + rng() % 9000;
        if (it % 3 == 0) n = 1000, sstride = 4000;
        size_t doff = rng() % 64, soff = rng() % 64, d2off = rng() % 64;
        if (it % 4 == 1) d2off = doff % 16 + 16 * (rng() % 3);  // destinations agreeing modulo 16
        std::vector<uint8_t> src(soff + sstride * rows + n), dst(doff + n * rows + 64, 0xEE), dst2(d2off + n * rows + 64, 0xDD);
        for (auto &b : src) b = uint8_t(rng());
        rsamd::CopyJob j{dst.data() + doff, src.data() + soff, n, rows, n, sstride};
        if (it % 2) { j.dst2 = dst2.data() + d2off; j.dst2_stride = n; }
        if (it % 5 == 4) {  // zero fill rows (a file's padding) through the same pool
            rsamd::CopyJob z{dst.data() + doff, nullptr, n, rows, n, 0};
            rsamd::CopyPool::get().copy({z});
            for (size_t x = 0; x < n * rows; ++x)
                if (dst[doff + x]) { ++bad; printf("zero fill n=%zu\n", n); break; }
        }
        rsamd::CopyPool::get().copy({j});
        ++cases;
        for (size_t r = 0; r < rows; ++r) {
            if (memcmp(dst.data() + doff + r * n, src.data() + soff + r * sstride, n)) { ++bad; printf("bad n=%zu rows=%zu r=%zu\n", n, rows, r); break; }
            if (j.dst2 && memcmp(dst2.data() + d2off + r * n, src.data() + soff + r * sstride, n)) { ++bad; printf("bad2 n=%zu rows=%zu r=%zu\n", n, rows, r); break; }
        }
        if (dst[doff + n * rows] != 0xEE || (doff && dst[doff - 1] != 0xEE)) { ++bad; printf("overrun n=%zu\n", n); }
        if (j.dst2 && (dst2[d2off + n * rows] != 0xDD || (d2off && dst2[d2off - 1] != 0xDD))) { ++bad; printf("overrun2 n=%zu\n", n); }
    }
    // a contiguous run teed into strided rows (a decode's data shard into its
    // slot and the file): every byte of both destinations, nothing past them
    for (int it = 0; it < 600; ++it) {
        const size_t n = 8 + rng() % 3000, rows = 1 + rng() % 400, d2stride = n + rng() % 5000;
        const size_t soff = rng() % 64, doff = rng() % 64, d2off = rng() % 64;
        std::vector<uint8_t> src(soff + n * rows), dst(doff + n * rows + 64, 0xEE), dst2(d2off + d2stride * rows + 64, 0xDD);
        for (auto &b : src) b = uint8_t(rng());
        rsamd::CopyJob j{dst.data() + doff, src.data() + soff, n, rows, n, n};
        j.dst2 = dst2.data() + d2off;
        j.dst2_stride = d2stride;
        rsamd::CopyPool::get().copy({j});
        ++cases;
        if (memcmp(dst.data() + doff, src.data() + soff, n * rows) || dst[doff + n * rows] != 0xEE) {
            ++bad;
            printf("tee run n=%zu rows=%zu\n", n, rows);
        }
        for (size_t r = 0; r < rows; ++r) {
            if (memcmp(dst2.data() + d2off + r * d2stride, src.data() + soff + r * n, n)) { ++bad; printf("tee rows n=%zu r=%zu\n", n, r); break; }
            if (r + 1 < rows && d2stride > n && dst2[d2off + r * d2stride + n] != 0xDD) { ++bad; printf("tee gap n=%zu\n", n); break; }
        }
    }
    // concurrent callers: 6 threads x 300 batches of 1-6 jobs, 1 B to 3 MiB
    // each; then 24 threads x 60 batches, more callers than the pool has batch
    // slots (those copy alone)
    std::atomic<int> cbad{0}, ccases{0};
    for (const int nt : {6, 24}) {
    std::vector<std::thread> ts;
    for (int t = 0; t < nt; ++t)
        ts.emplace_back([&, t, nt] {
            std::mt19937_64 r(100 + t + 1000 * nt);
            for (int it = 0; it < (nt == 6 ? 300 : 60); ++it) {
                const int nj = 1 + int(r() % 6);
                std::vector<std::vector<uint8_t>> srcs(nj), dsts(nj);
                std::vector<rsamd::CopyJob> jobs;
                for (int q = 0; q < nj; ++q) {
                    const size_t n = 1 + r() % ((r() % 4 == 0) ? (3u << 20) : 70000u);
                    srcs[q].resize(n);
                    for (size_t x = 0; x < n; x += 8) srcs[q][x] = uint8_t(r());
                    dsts[q].assign(n + 1, 0xEE);
                    jobs.push_back({dsts[q].data(), srcs[q].data(), n});
                }
                rsamd::CopyPool::get().copy(jobs);
                ++ccases;
                for (int q = 0; q < nj; ++q)
                    if (memcmp(dsts[q].data(), srcs[q].data(), srcs[q].size()) || dsts[q].back() != 0xEE) ++cbad;
            }
        });
    for (auto &th : ts) th.join();
    }
    printf("%d concurrent batches, %d bad\n", ccases.load(), cbad.load());
    bad += cbad.load();
    printf("%d cases, %d bad\n", cases, bad);
    return bad != 0;
}
