// copy_pool_check.cpp -- CPU check of the host copy pool (csrc/copy_pool.cpp):
// strided row copies into contiguous destinations (the streaming gather of
// a file's block rows into shard columns), with a second destination (the
// tee into the pinned slots), random row lengths, strides and alignments;
// every byte is compared with a plain copy and nothing past the destination
// may be written.  Built and run by tests/test_copy_pool.py.
#include "copy_pool.hpp"
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>
int main() {  // copy_pool.cpp gathers, tees, zero fills: every byte against a plain copy
    std::mt19937_64 rng(1);
    int bad = 0, cases = 0;
    for (int it = 0; it < 3000; ++it) {
        size_t n = 1 + rng() % 5000, rows = 1 + rng() % 300, sstride = n + rng() % 9000;
        if (it % 3 == 0) n = 1000, sstride = 4000;
        size_t doff = rng() % 64, soff = rng() % 64, d2off = rng() % 64;
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
    }
    printf("%d cases, %d bad\n", cases, bad);
    return bad != 0;
}
