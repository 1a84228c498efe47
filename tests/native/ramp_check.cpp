// ramp_check.cpp -- CPU check of the mirrored pipeline's chunking (csrc/host.cpp
// ramp_bounds, mirror_chunk_bytes): for many call sizes, chunk sizes and
// granules, the boundaries start at 0, end at the call's size, strictly
// increase, every chunk but the last is a whole number of granules, no chunk
// is wider than a chunk plus the granules the rounding leaves over, and a
// call of more than two chunks ramps up and down (a quarter and a half chunk
// first and last).  Built against the product objects by tests/test_copy_pool.py.
#include <cstdio>
#include <random>
#include <vector>

#include "host.hpp"

int main() {
    std::mt19937_64 rng(5);
    int bad = 0, cases = 0;
    auto fail = [&](const char *what, size_t total, size_t chunk, size_t g) {
        if (bad++ < 10) std::printf("%s: total=%zu chunk=%zu granule=%zu\n", what, total, chunk, g);
    };
    for (int it = 0; it < 200000; ++it) {
        const size_t g = it % 3 == 0 ? 1 : (it % 3 == 1 ? 4096 : 1 + rng() % 5000);
        const size_t total = 1 + rng() % (it % 2 ? (size_t(1) << 28) : 100000);
        const size_t chunk = 1 + rng() % (size_t(1) << 24);
        const std::vector<size_t> b = rsamd::host::ramp_bounds(total, chunk, g);
        ++cases;
        if (b.size() < 2 || b.front() != 0 || b.back() != total) {
            fail("ends", total, chunk, g);
            continue;
        }
        const size_t c = std::max(g, chunk / g * g);
        const size_t n = b.size() - 1;
        for (size_t j = 0; j < n; ++j) {
            const size_t w = b[j + 1] - b[j];
            if (w == 0) fail("empty chunk", total, chunk, g);
            if (j + 1 < n && w % g) fail("not whole granules", total, chunk, g);
            if (w > c + n * g + c / 2 + g) fail("too wide", total, chunk, g);
        }
        // a call of several chunks starts with a quarter chunk and ends short too
        if (total > 2 * (c / 4 + c / 2) + 2 * g && n > 3 && b[1] > c / 4 + g) fail("no ramp", total, chunk, g);
    }
    for (int nslots : {3, 6, 14, 20})
        for (size_t total : {size_t(1000), size_t(1) << 20, size_t(64) << 20, size_t(1) << 30}) {
            const size_t c = rsamd::host::mirror_chunk_bytes(total, nslots, 4096);
            ++cases;
            if (c == 0 || c % 4096 || c * size_t(nslots) > (size_t(64) << 20) + 4096 * size_t(nslots))
                fail("mirror_chunk_bytes", total, size_t(nslots), 4096);
        }
    std::printf("%d cases, %d bad\n", cases, bad);
    return bad != 0;
}
