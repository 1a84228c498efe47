// copy_pool.cpp -- see copy_pool.hpp.
#include "copy_pool.hpp"
#include "tuning.hpp"

#include <algorithm>
#include <cstring>

#include <immintrin.h>

namespace rsamd {

namespace {
constexpr size_t kPiece = size_t(1) << 20;  // bytes per work item

// Streaming (non-temporal) copy: the destination's lines are written without
// being read first and without displacing the cache.  Every pool copy is
// between caller memory and the pinned mirror, which the GPU reads (or has
// written) across the link, so no CPU cache would keep either side.  The
// sfence makes the stores globally visible before the piece is reported done.
__attribute__((target("avx2"))) void copy_stream(uint8_t *dst, const uint8_t *src, size_t n) {
    size_t head = (32 - reinterpret_cast<uintptr_t>(dst) % 32) % 32;
    if (head > n) head = n;
    std::memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    for (; n >= 128; n -= 128, dst += 128, src += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + 64));
        const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst), a);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + 96), d);
    }
    std::memcpy(dst, src, n);
    _mm_sfence();
}

// TUNING builds: RSAMD_COPY_NT=0 copies with memcpy instead (A/B).
bool use_stream() {
    static const bool on = [] {
        const char *e = tuning_env("RSAMD_COPY_NT");
        return __builtin_cpu_supports("avx2") && !(e && e[0] == '0');
    }();
    return on;
}

void copy_piece(const CopyJob &j) {
    if (j.n >= 4096 && use_stream())
        copy_stream(static_cast<uint8_t *>(j.dst), static_cast<const uint8_t *>(j.src), j.n);
    else
        std::memcpy(j.dst, j.src, j.n);
}
}  // namespace

CopyPool &CopyPool::get() {
    static CopyPool *pool = [] {
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        // + the caller: <= 16 copying threads (TUNING builds: RSAMD_COPY_THREADS)
        return new CopyPool(int(tuning_size("RSAMD_COPY_THREADS", std::min(15u, std::max(2u, hw / 2)))));
    }();
    return *pool;
}

CopyPool::CopyPool(int n) {
    for (int i = 0; i < n; ++i) {
        threads_.emplace_back([this] { run(); });
        threads_.back().detach();
    }
}

void CopyPool::run() {
    std::unique_lock<std::mutex> lock(mu_);
    for (;;) {
        work_cv_.wait(lock, [this] { return !queue_.empty(); });
        Piece p = queue_.front();
        queue_.pop_front();
        lock.unlock();
        copy_piece(p.job);
        lock.lock();
        if (--*p.pending == 0) done_cv_.notify_all();
    }
}

void CopyPool::copy(const std::vector<CopyJob> &jobs) {
    size_t pending = 0;
    {
        std::lock_guard<std::mutex> lock(mu_);
        for (const CopyJob &j : jobs)
            for (size_t off = 0; off < j.n; off += kPiece) {
                const size_t n = std::min(kPiece, j.n - off);
                queue_.push_back({{static_cast<uint8_t *>(j.dst) + off, static_cast<const uint8_t *>(j.src) + off, n},
                                  &pending});
                ++pending;
            }
    }
    if (pending == 0) return;
    work_cv_.notify_all();
    // The caller works too: take this batch's pieces (or anyone's) until the
    // queue is empty, then wait for the pieces still being copied.
    std::unique_lock<std::mutex> lock(mu_);
    while (pending > 0) {
        if (!queue_.empty()) {
            Piece p = queue_.front();
            queue_.pop_front();
            lock.unlock();
            copy_piece(p.job);
            lock.lock();
            if (--*p.pending == 0) done_cv_.notify_all();
            continue;
        }
        done_cv_.wait(lock, [&] { return pending == 0 || !queue_.empty(); });
    }
}

}  // namespace rsamd
