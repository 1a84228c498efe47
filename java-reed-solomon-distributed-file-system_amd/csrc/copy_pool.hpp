// copy_pool.hpp -- parallel host memcpy for the host-buffer pipeline.
//
// Pageable caller buffers (what JNI hands us) are staged through pinned
// mirrors so the PCIe copies run as async DMA in both directions at once; the
// pageable <-> pinned memcpy is split over a small process-wide worker pool so
// it keeps up with the link (measured on the MI355X host: one thread ~23 GB/s,
// 8 threads ~71 GB/s, 16 threads 100-126 GB/s; the link moves ~57 GB/s each
// way -- tools/memcpy_probe.cpp).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <thread>
#include <vector>

namespace rsamd {

// n bytes from src to dst, or `rows` rows of n bytes each, row r at
// src + r * src_stride and dst + r * dst_stride (block rows of a file and the
// columns of a shard).  src == nullptr writes zeros (a file's padding).  With
// dst2, every row also goes to dst2 + r * dst2_stride, from the same thread
// right after the first (the second read hits the core's cache).
struct CopyJob {
    void *dst;
    const void *src;
    size_t n;
    size_t rows = 1;
    size_t dst_stride = 0, src_stride = 0;
    void *dst2 = nullptr;
    size_t dst2_stride = 0;
};

// Caller arrays that may move between copy batches (a JVM's heap arrays;
// rs_amd.h rs_set_relocator).  The library touches caller memory only by
// copy jobs -- CopyPool::copy and CopyPool::copy_here -- so the arrays need
// to stay put only while one batch runs: with a relocator set on the calling
// thread, each batch first calls acquire (which pins every array and writes
// its current address into base[i]), rewrites every job address inside
// [keys[i], keys[i] + lens[i]) to the same offset from base[i], copies, then
// calls release.  The keys are stand-ins the call's pointers were made from;
// they are never dereferenced.
struct Relocator {
    void *user = nullptr;
    int n = 0;
    const uint8_t *const *keys = nullptr;
    const int64_t *lens = nullptr;
    int (*acquire)(void *user, uint8_t **base) = nullptr;
    void (*release)(void *user, uint8_t **base) = nullptr;
};
// The calling thread's relocator (nullptr: none; the struct is copied, the
// key and length arrays it points to must outlive the setting).
void set_thread_relocator(const Relocator *r);
bool thread_relocating();
// True, and cleared, when an acquire failed on this thread since the last
// call (that batch was not copied).
bool take_relocation_failure();

class CopyPool {
public:
    // The process-wide pool (created on first use, never destroyed: its
    // threads are detached so process exit never waits on them).
    static CopyPool &get();

    // Copy every job, split into pieces over the workers and the calling
    // thread; returns when all bytes are copied.  Safe to call from several
    // threads at once.
    void copy(const std::vector<CopyJob> &jobs);
    // The same on the calling thread alone with plain memcpy / memset (small
    // calls: the pool's wake-up costs more than their bytes).
    static void copy_here(const std::vector<CopyJob> &jobs);

    int workers() const { return int(threads_.size()); }

private:
    explicit CopyPool(int n);
    void run();
    void copy_batch(const std::vector<CopyJob> &jobs);

    // One posted batch: its pieces (the caller's), claimed one at a time by
    // an atomic counter.  kSlots batches (callers) at once; a caller that
    // finds none free copies alone.
    enum : uint32_t { kFree = 0, kFilling = 1, kActive = 2, kDraining = 3 };
    struct Slot {
        std::atomic<uint32_t> state{kFree};
        const CopyJob *pieces = nullptr;
        size_t n = 0;
        std::atomic<size_t> next{0}, done{0};
        std::atomic<int> refs{0};  // threads that may touch the batch
    };
    static constexpr int kSlots = 16;
    bool work_on(Slot &s);

    Slot slots_[kSlots];
    std::atomic<uint64_t> posted_{0};  // batches posted so far (a sleeper's wake-up condition)
    std::atomic<int> sleepers_{0};
    std::mutex mu_;                    // sleeping workers only
    std::condition_variable work_cv_;
    int spin_us_ = 0;                  // how long an idle thread polls before it sleeps
    std::vector<std::thread> threads_;
};

}  // namespace rsamd
