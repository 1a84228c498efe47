// copy_pool.cpp -- see copy_pool.hpp.
#include "copy_pool.hpp"
#include "tuning.hpp"

#include <algorithm>
#include <cstring>

namespace rsamd {

namespace {
constexpr size_t kPiece = size_t(1) << 20;  // bytes per work item
}

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
        std::memcpy(p.job.dst, p.job.src, p.job.n);
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
            std::memcpy(p.job.dst, p.job.src, p.job.n);
            lock.lock();
            if (--*p.pending == 0) done_cv_.notify_all();
            continue;
        }
        done_cv_.wait(lock, [&] { return pending == 0 || !queue_.empty(); });
    }
}

}  // namespace rsamd
