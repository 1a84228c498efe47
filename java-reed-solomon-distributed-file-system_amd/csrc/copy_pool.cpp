// copy_pool.cpp -- see copy_pool.hpp.
#include "copy_pool.hpp"
#include "tuning.hpp"

#include <algorithm>
#include <chrono>
#include <cstring>

#include <immintrin.h>

namespace rsamd {

namespace {
constexpr size_t kPiece = size_t(1) << 20;  // bytes per work item

// Streaming (non-temporal) copy: the destination's lines are written without
// being read first and without displacing the cache.  Every pool copy is
// between caller memory and the pinned mirror, which the GPU reads (or has
// written) across the link, so no CPU cache would keep either side.
// copy_piece's sfence makes the stores globally visible before the piece is
// reported done.
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
}

// TUNING builds: RSAMD_COPY_NT=0 copies with memcpy instead (A/B).
bool use_stream() {
    static const bool on = [] {
        const char *e = tuning_env("RSAMD_COPY_NT");
        return __builtin_cpu_supports("avx2") && !(e && e[0] == '0');
    }();
    return on;
}

// Rows shorter than this are copied with plain stores (TUNING builds:
// RSAMD_COPY_NT_MIN): a streaming store that fills only part of a line
// (a short row's head and tail) costs the line a read-modify-write.
size_t stream_min() {
    static const size_t v = tuning_size("RSAMD_COPY_NT_MIN", 256);
    return v;
}

void copy_row(uint8_t *dst, const uint8_t *src, size_t n) {
    if (!src)
        std::memset(dst, 0, n);
    else if (n >= stream_min() && use_stream())
        copy_stream(dst, src, n);
    else
        std::memcpy(dst, src, n);
}

// Destination bytes [x0, x0 + len) of a gather whose destination is `rows`
// rows of n bytes back to back, row r's source at src + r * src_stride.
void gather_plain(uint8_t *dst, const uint8_t *src, size_t n, size_t src_stride, size_t x0, size_t len) {
    while (len) {
        const size_t r = x0 / n, c = x0 % n, take = std::min(len, n - c);
        std::memcpy(dst + x0, src + r * src_stride + c, take);
        x0 += take;
        len -= take;
    }
}

// A gather into a contiguous destination (a file's block rows into one
// shard's column run: rows of n >= 32 bytes, sources src_stride apart) as
// whole 32-byte streaming stores along the destination.  Copying row by row
// instead leaves each short row's first and last line partly written by
// streaming stores, which costs those lines a read-modify-write.  A vector
// that straddles two rows is assembled from both.
// With `prefetch` = p > 0, the row p rows on is prefetched as each row
// starts: the rows are short runs src_stride apart (a file's 1000-byte blocks
// 4000 bytes apart), where the hardware prefetchers restart at every row and
// each row's first lines miss.
__attribute__((target("avx2"))) void gather_stream(uint8_t *dst, const uint8_t *src, size_t n, size_t rows,
                                                   size_t src_stride, size_t prefetch) {
    const size_t total = n * rows;
    size_t x = std::min(total, (32 - reinterpret_cast<uintptr_t>(dst) % 32) % 32);
    gather_plain(dst, src, n, src_stride, 0, x);
    size_t r = x / n, c = x % n;
    const uint8_t *sp = src + r * src_stride + c;
    auto fetch = [&](size_t row) {  // one row, line by line
        if (row >= rows) return;
        const char *p = reinterpret_cast<const char *>(src + row * src_stride);
        for (size_t l = 0; l < n; l += 64) _mm_prefetch(p + l, _MM_HINT_T0);
    };
    auto ahead = [&](size_t row) {  // entering `row`: the row `prefetch` rows on
        if (prefetch) fetch(row + prefetch);
    };
    for (size_t q = 1; q <= prefetch; ++q) fetch(r + q);
    for (; x + 32 <= total; x += 32) {
        __m256i v;
        if (c + 32 <= n) {
            v = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(sp));
            sp += 32;
            c += 32;
        } else {  // the vector's bytes end one row and start the next
            alignas(32) uint8_t tmp[32];
            const size_t a = n - c;
            std::memcpy(tmp, sp, a);
            ++r;
            sp = src + r * src_stride;
            std::memcpy(tmp + a, sp, 32 - a);
            sp += 32 - a;
            c = 32 - a;
            v = _mm256_load_si256(reinterpret_cast<const __m256i *>(tmp));
            ahead(r);
        }
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + x), v);
        if (c == n) {
            ++r;
            c = 0;
            sp = src + r * src_stride;
            ahead(r);
        }
    }
    gather_plain(dst, src, n, src_stride, x, total - x);
}

// Rows ahead the gather prefetches (TUNING builds: RSAMD_COPY_PREFETCH, 0 = none).
// 256 MiB pageable file encode, three alternated runs each: none 39.5-40.6
// GiB/s; 1 row 44.4-45.5; 2 rows 44.9-45.5; 3 rows 43.4-45.4
// (profiles/r5/host_legs_prefetch_r7d.txt, host_legs_pfdist_r7i.txt).
size_t prefetch_rows() {
    static const size_t v = tuning_size("RSAMD_COPY_PREFETCH", 2);
    return v;
}

void copy_piece(const CopyJob &j) {
    uint8_t *d = static_cast<uint8_t *>(j.dst), *d2 = static_cast<uint8_t *>(j.dst2);
    const uint8_t *s = static_cast<const uint8_t *>(j.src);
    // rows into a contiguous destination: along the destination
    auto gathers = [&](size_t dst_stride) {
        return s && j.rows > 1 && dst_stride == j.n && j.n >= 32 && use_stream() && !tuning_size("RSAMD_COPY_ROWWISE", 0);
    };
    if (gathers(j.dst_stride) && (!d2 || gathers(j.dst2_stride))) {
        // Two passes, the second reading the source again from this core's
        // cache: one pass loading each 16 bytes once and streaming them to both
        // destinations (16-byte stores; a caller's array and its slot agree only
        // modulo 16) made the 256 MiB pageable file encode slower, 35.1-35.5
        // GiB/s against 37.0-37.4 (profiles/r5/host_legs_dual_r6u.txt; deleted).
        // (TUNING builds: RSAMD_COPY_PREFETCH=0 turns the row prefetch off, A/B)
        gather_stream(d, s, j.n, j.rows, j.src_stride, prefetch_rows());
        if (d2) gather_stream(d2, s, j.n, j.rows, j.src_stride, 0);
    } else if (s && d2 && j.rows > 1 && j.src_stride == j.n && j.dst_stride == j.n && use_stream()) {
        // a contiguous run teed into rows (a decode's data shard into its slot
        // and the file): the run in one stream, then the rows from this core's cache
        copy_stream(d, s, j.n * j.rows);
        for (size_t r = 0; r < j.rows; ++r) copy_row(d2 + r * j.dst2_stride, s + r * j.n, j.n);
    } else {
        for (size_t r = 0; r < j.rows; ++r) {
            const uint8_t *src = s ? s + r * j.src_stride : nullptr;
            copy_row(d + r * j.dst_stride, src, j.n);
            if (d2) copy_row(d2 + r * j.dst2_stride, src, j.n);
        }
    }
    _mm_sfence();
}
}  // namespace

// ---- relocation (copy_pool.hpp Relocator) ----------------------------------
namespace {
thread_local Relocator t_reloc;
thread_local bool t_reloc_on = false;
thread_local bool t_reloc_failed = false;

// The batch's jobs with every address inside a key range moved to its array's
// current base.
template <class P>
P rebase(P p, uint8_t *const *base) {
    if (!p) return p;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    for (int i = 0; i < t_reloc.n; ++i) {
        const uintptr_t k = reinterpret_cast<uintptr_t>(t_reloc.keys[i]);
        if (a >= k && a - k <= uintptr_t(t_reloc.lens[i]))
            return reinterpret_cast<P>(reinterpret_cast<uintptr_t>(base[i]) + (a - k));
    }
    return p;
}

// Runs `fn` over the jobs, relocated when this thread has a relocator: false
// (nothing copied, the failure recorded) when its acquire fails.
template <class Fn>
void with_relocation(const std::vector<CopyJob> &jobs, Fn fn) {
    if (!t_reloc_on || jobs.empty()) {
        fn(jobs);
        return;
    }
    std::vector<uint8_t *> base(size_t(std::max(1, t_reloc.n)), nullptr);
    if (t_reloc.acquire(t_reloc.user, base.data()) != 0) {
        t_reloc_failed = true;
        return;
    }
    std::vector<CopyJob> moved(jobs);
    for (CopyJob &j : moved) {
        j.dst = rebase(j.dst, base.data());
        j.src = rebase(j.src, base.data());
        j.dst2 = rebase(j.dst2, base.data());
    }
    fn(moved);
    t_reloc.release(t_reloc.user, base.data());
}
}  // namespace

void set_thread_relocator(const Relocator *r) {
    t_reloc_on = r != nullptr;
    t_reloc = r ? *r : Relocator{};
    t_reloc_failed = false;
}
bool thread_relocating() { return t_reloc_on; }
bool take_relocation_failure() {
    const bool f = t_reloc_failed;
    t_reloc_failed = false;
    return f;
}

void CopyPool::copy_here(const std::vector<CopyJob> &jobs) {
    with_relocation(jobs, [](const std::vector<CopyJob> &js) {
        for (const CopyJob &j : js)
            for (size_t r = 0; r < j.rows; ++r) {
                uint8_t *dst = static_cast<uint8_t *>(j.dst) + r * j.dst_stride;
                const uint8_t *src = j.src ? static_cast<const uint8_t *>(j.src) + r * j.src_stride : nullptr;
                if (src)
                    std::memcpy(dst, src, j.n);
                else
                    std::memset(dst, 0, j.n);
                if (j.dst2) {
                    uint8_t *d2 = static_cast<uint8_t *>(j.dst2) + r * j.dst2_stride;
                    if (src)
                        std::memcpy(d2, src, j.n);
                    else
                        std::memset(d2, 0, j.n);
                }
            }
    });
}

CopyPool &CopyPool::get() {
    static CopyPool *pool = [] {
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        // + the caller: <= 16 copying threads (TUNING builds: RSAMD_COPY_THREADS)
        return new CopyPool(int(tuning_size("RSAMD_COPY_THREADS", std::min(15u, std::max(2u, hw / 2)))));
    }();
    return *pool;
}

// spin_us_: an idle thread (a worker with nothing to claim, a caller waiting
// for its batch's last pieces) polls for this long before it sleeps (a
// caller: yields): the mirrored pipeline hands the pool a batch per chunk, and
// a sleeping thread's wake-up costs more than a small chunk's copy.  4+2
// pageable encodeParity per call, 0 -> 50 us (profiles/r5/host_sizes_r5v.txt):
// 1 MiB shards 309-378 -> 235-269 us, 2 MiB 465-547 -> 354-394, 4 MiB
// 620-656 -> 556-567; 200 us is no better (TUNING builds: RSAMD_POOL_SPIN_US).
CopyPool::CopyPool(int n) {
    spin_us_ = int(tuning_size("RSAMD_POOL_SPIN_US", 50));
    for (int i = 0; i < n; ++i) {
        threads_.emplace_back([this] { run(); });
        threads_.back().detach();
    }
}

// Claims and copies pieces of slot s's batch while any are left; true if it
// copied one.  A worker holds a reference while it may touch the slot's
// batch, so the batch's owner returns (and its pieces go) only after every
// claimant has let go; the slots themselves live as long as the pool.
bool CopyPool::work_on(Slot &s) {
    if (s.state.load(std::memory_order_acquire) != kActive) return false;
    s.refs.fetch_add(1, std::memory_order_acq_rel);
    bool did = false;
    if (s.state.load(std::memory_order_acquire) == kActive) {
        for (;;) {
            const size_t i = s.next.fetch_add(1, std::memory_order_acq_rel);
            if (i >= s.n) break;
            copy_piece(s.pieces[i]);
            s.done.fetch_add(1, std::memory_order_acq_rel);
            did = true;
        }
    }
    s.refs.fetch_sub(1, std::memory_order_acq_rel);
    return did;
}

// Workers poll the slots; one sleeps only after spin_us_ of continuous
// idleness, and a caller posting a batch wakes the sleepers.  Pieces are
// claimed with an atomic counter, not under a lock: with a mutex-guarded queue
// the 15 workers polling for a batch met at the mutex, and a small batch cost
// 17 us more through the pool than on the calling thread alone (4 x 64 KiB;
// tools/pool_batch_probe.cpp, profiles/r6/pool_probe_r6y.txt).
void CopyPool::run() {
    using clock = std::chrono::steady_clock;
    auto idle_since = clock::now();
    for (;;) {
        bool did = false;
        for (Slot &s : slots_) did = work_on(s) || did;
        if (did) {
            idle_since = clock::now();
            continue;
        }
        if (clock::now() - idle_since < std::chrono::microseconds(spin_us_)) {
            for (int i = 0; i < 32; ++i) _mm_pause();
            continue;
        }
        std::unique_lock<std::mutex> lock(mu_);
        const uint64_t seen = posted_.load(std::memory_order_seq_cst);
        sleepers_.fetch_add(1, std::memory_order_seq_cst);
        bool any = false;
        for (Slot &s : slots_) any = any || s.state.load(std::memory_order_seq_cst) == kActive;
        if (!any) work_cv_.wait(lock, [&] { return posted_.load(std::memory_order_seq_cst) != seen; });
        sleepers_.fetch_sub(1, std::memory_order_seq_cst);
        idle_since = clock::now();
    }
}

void CopyPool::copy(const std::vector<CopyJob> &jobs) {
    with_relocation(jobs, [this](const std::vector<CopyJob> &js) { copy_batch(js); });
}

void CopyPool::copy_batch(const std::vector<CopyJob> &jobs) {
    std::vector<CopyJob> pieces;
    for (const CopyJob &j : jobs) {
        if (j.n == 0 || j.rows == 0) continue;
        const uint8_t *src = static_cast<const uint8_t *>(j.src);
        uint8_t *dst = static_cast<uint8_t *>(j.dst);
        uint8_t *dst2 = static_cast<uint8_t *>(j.dst2);
        if (j.rows == 1) {
            for (size_t off = 0; off < j.n; off += kPiece) {
                CopyJob piece{dst + off, src ? src + off : nullptr, std::min(kPiece, j.n - off)};
                piece.dst2 = dst2 ? dst2 + off : nullptr;
                pieces.push_back(piece);
            }
            continue;
        }
        // rows: pieces of about kPiece bytes of whole rows
        const size_t per = std::max<size_t>(1, kPiece / j.n);
        for (size_t r = 0; r < j.rows; r += per)
            pieces.push_back({dst + r * j.dst_stride, src ? src + r * j.src_stride : nullptr, j.n,
                              std::min(per, j.rows - r), j.dst_stride, j.src_stride,
                              dst2 ? dst2 + r * j.dst2_stride : nullptr, j.dst2_stride});
    }
    if (pieces.empty()) return;
    // A free slot (every slot taken by other callers' batches: this thread copies alone)
    Slot *slot = nullptr;
    for (Slot &s : slots_) {
        uint32_t free = kFree;
        if (s.state.compare_exchange_strong(free, kFilling, std::memory_order_acq_rel)) {
            slot = &s;
            break;
        }
    }
    if (!slot || pieces.size() == 1) {
        if (slot) slot->state.store(kFree, std::memory_order_release);
        for (const CopyJob &p : pieces) copy_piece(p);
        return;
    }
    slot->pieces = pieces.data();
    slot->n = pieces.size();
    slot->next.store(0, std::memory_order_relaxed);
    slot->done.store(0, std::memory_order_relaxed);
    slot->state.store(kActive, std::memory_order_seq_cst);
    posted_.fetch_add(1, std::memory_order_seq_cst);
    if (sleepers_.load(std::memory_order_seq_cst) > 0) {
        { std::lock_guard<std::mutex> lock(mu_); }
        work_cv_.notify_all();
    }
    // The caller works too, then waits for the pieces others still copy.
    work_on(*slot);
    const auto t0 = std::chrono::steady_clock::now();
    while (slot->done.load(std::memory_order_acquire) < slot->n) {
        if (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(spin_us_))
            for (int i = 0; i < 32; ++i) _mm_pause();
        else
            std::this_thread::yield();
    }
    // Retire the batch: no new claimant after this, and the last one gone
    // before the pieces (this frame's vector) go.
    slot->state.store(kDraining, std::memory_order_seq_cst);
    while (slot->refs.load(std::memory_order_acquire) != 0) _mm_pause();
    slot->state.store(kFree, std::memory_order_release);
}

}  // namespace rsamd
