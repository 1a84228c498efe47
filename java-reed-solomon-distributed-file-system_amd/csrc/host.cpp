// host.cpp -- the host side of the host-buffer entry points (host.hpp):
// thread-local error text, per-(thread, device) staging contexts, page-locking
// of pageable caller buffers, and the chunked H2D -> kernels -> D2H pipeline
// with its zero-copy path for single-chunk calls.
#include "host.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <thread>

#include "../../include/rs_amd.h"
#include "bounds.hpp"
#include "codec.hpp"
#include "copy_pool.hpp"
#include "tuning.hpp"

#include <sys/syscall.h>
#include <unistd.h>

namespace rsamd {
namespace host {

namespace {
void release_all(std::map<int, ThreadCtx *> &ctx);
void orphan(std::map<int, ThreadCtx *> &&ctx);
ThreadCtx *adopt_idle(int dev);

// This thread's contexts (device -> context), released when the thread exits
// (JVM and gRPC worker pools create and retire threads) or by rs_thread_release.
// Not for the process's main thread: its thread-locals are destroyed inside
// exit() (glibc runs them before the atexit handlers), where the HIP runtime
// may already be shutting down.  Whichever thread loaded the library (a JVM
// loads it from a worker) is released like any other.
//
// The exiting thread makes no HIP call: its contexts go to the reaper thread
// (orphan), which frees their buffers from a live thread and keeps their
// streams and events for the next new thread (adopt_idle).  Thread-local destructors run
// in the reverse order of their first use, across libraries, so the HIP
// runtime's own per-thread state (created lazily, by the first stream or
// launch of the thread, after this object) may already be gone when this
// destructor runs; streams and events destroyed from here went through it.
// Both GPU faults of rounds 3 and 4 surfaced a few calls after worker threads
// had exited that way.
bool on_main_thread() { return pid_t(syscall(SYS_gettid)) == getpid(); }
struct ThreadContexts {
    std::map<int, ThreadCtx *> m;
    ~ThreadContexts() {
        if (!on_main_thread() && !process_exiting() && !m.empty()) orphan(std::move(m));
    }
};

thread_local std::string t_err;
thread_local ThreadContexts t_ctx;
}  // namespace

int fail(int code, const std::string &msg) {
    t_err = msg;
    return code;
}

const char *last_error() { return t_err.c_str(); }

int hip_fail(hipError_t e, const char *where) {
    char buf[256];
    std::snprintf(buf, sizeof buf, "HIP error %s (%s) in %s", hipGetErrorName(e), hipGetErrorString(e), where);
    t_err = buf;
    return RS_E_HIP;
}

// ---------------------------------------------------------------------------
// Per-(thread, device) staging context for the host-buffer API.
// ---------------------------------------------------------------------------
int need_device() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(RS_E_NO_DEVICE, "no HIP device available");
    return RS_OK;
}

// Streams and hardware queues.  HIP maps streams onto a few hardware queues
// (GPU_MAX_HW_QUEUES, 4); two streams on one queue run in order.  With H2D
// copies, kernels and D2H copies on three streams, which queue each got
// depended on the streams the process had made before: the same 4+2 x 64 MiB
// pinned encode ran at 34 or 44 GiB/s depending only on how many torch
// streams existed first (tools/host_queues.py, profiles/r3/host_queues_*.txt),
// because a D2H copy (a blit kernel) queued behind an H2D copy's wait
// serialises the two directions.  Measured over 0-5 prior streams:
//   three plain streams                34.3, then 44.0-44.7
//   D2H / H2D at low / high priority   44.4, 44.4, 44.4, 43.0, 40.6, 42.4
//   three CU-masked streams            43.2-44.4
//   D2H on the kernel stream           44.1-45.0   <- used
// The D2H of chunk j now runs before chunk j+1's kernel on one stream, which
// costs nothing (that kernel waits for its own, longer upload anyway), and
// only two streams must differ: uploads (stream3) and the rest (stream).
#ifndef RSAMD_PIPE_MODE
#define RSAMD_PIPE_MODE 3  // A/B: 0 plain streams, 1 priorities, 2 CU-masked streams, 3 D2H on the kernel stream
#endif
hipError_t create_pipeline_streams(ThreadCtx *c) {
    int least = 0, greatest = 0;
    if (RSAMD_PIPE_MODE == 2) {
        int dev = 0, ncu = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        std::vector<uint32_t> mask(size_t(ncu + 31) / 32, 0xFFFFFFFFu);
        if (e == hipSuccess) e = hipExtStreamCreateWithCUMask(&c->stream, uint32_t(mask.size()), mask.data());
        if (e == hipSuccess) e = hipExtStreamCreateWithCUMask(&c->stream2, uint32_t(mask.size()), mask.data());
        if (e == hipSuccess) e = hipExtStreamCreateWithCUMask(&c->stream3, uint32_t(mask.size()), mask.data());
        return e;
    }
    if (RSAMD_PIPE_MODE != 1 || hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess || least == greatest) {
        (void)hipGetLastError();
        hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream3, hipStreamNonBlocking);
        return e;
    }
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, least);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, greatest);
    return e;
}

int thread_ctx(ThreadCtx **out) {
    int dev = 0;
    RS_HIP(hipGetDevice(&dev));
    auto it = t_ctx.m.find(dev);
    if (it == t_ctx.m.end()) {
        ThreadCtx *c = adopt_idle(dev);  // a retired thread's streams and events, if any
        if (c) {
            it = t_ctx.m.emplace(dev, c).first;
            *out = c;
            bounds::allow(c->flag, 256);
            return RS_OK;
        }
        c = new ThreadCtx;
        hipError_t e = create_pipeline_streams(c);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ready, hipEventDisableTiming);
        for (int b = 0; b < kStageBufs && e == hipSuccess; ++b) {
            e = hipEventCreateWithFlags(&c->coded[b], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&c->freed[b], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&c->loaded[b], hipEventDisableTiming);
        }
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&c->flag), 256);
        if (e == hipSuccess) e = hipMemset(c->flag, 0, 256);  // the verify word and the signal's block counter
        if (e != hipSuccess) {
            delete c;
            return hip_fail(e, "thread context");
        }
        it = t_ctx.m.emplace(dev, c).first;
    }
    *out = it->second;
    bounds::allow(it->second->flag, 256);
    return RS_OK;
}

namespace {
// A context's buffers (staging, mirrors, zero-copy and masked slots, plan
// images): the memory a retired thread should give back.  Streams, events
// and the flag stay.
void free_buffers(ThreadCtx *c) {
    for (MaskedSlot &sl : c->masked) {
        if (sl.done) (void)hipEventSynchronize(sl.done);
        if (sl.dev) (void)hipFree(sl.dev);
        if (sl.host) (void)hipHostFree(sl.host);
        sl.dev = sl.host = nullptr;
        sl.dev_cap = sl.host_cap = 0;
    }
    if (c->mirror) (void)hipHostFree(c->mirror);
    if (c->stage) (void)hipFree(c->stage);
    if (c->plan) (void)hipFree(c->plan);
    if (c->file) (void)hipFree(c->file);
    if (c->zc) (void)hipHostFree(c->zc);
    if (c->sig) (void)hipHostFree(c->sig);
    c->sig = c->sig_dev = nullptr;
    c->mirror = c->stage = c->plan = c->file = c->zc = c->zc_dev = nullptr;
    c->mirror_cap = c->stage_cap = c->plan_cap = c->file_cap = c->zc_cap = 0;
}

void release_all(std::map<int, ThreadCtx *> &ctx) {
    if (ctx.empty()) return;  // a thread that never coded makes no HIP call here
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto &kv : ctx) {
        ThreadCtx *c = kv.second;
        (void)hipSetDevice(kv.first);
        free_buffers(c);
        if (c->stream) (void)hipStreamDestroy(c->stream);
        if (c->stream2) (void)hipStreamDestroy(c->stream2);
        if (c->stream3) (void)hipStreamDestroy(c->stream3);
        if (c->ready) (void)hipEventDestroy(c->ready);
        for (int b = 0; b < kStageBufs; ++b) {
            if (c->coded[b]) (void)hipEventDestroy(c->coded[b]);
            if (c->freed[b]) (void)hipEventDestroy(c->freed[b]);
            if (c->loaded[b]) (void)hipEventDestroy(c->loaded[b]);
        }
        if (c->flag) (void)hipFree(c->flag);
        for (MaskedSlot &sl : c->masked) {
            if (sl.done) (void)hipEventDestroy(sl.done);
            if (sl.uploaded) (void)hipEventDestroy(sl.uploaded);
        }
        delete c;
    }
    ctx.clear();
    (void)hipSetDevice(cur);
}
}  // namespace

namespace {
// The reaper: one long-lived thread, started by the first exiting worker,
// that releases orphaned contexts.  It never touches a ThreadCtx of its own
// and stops releasing once exit() has begun (as ~Codec does).
struct Orphanage {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::map<int, ThreadCtx *>> q;
    bool started = false;
    std::map<int, std::vector<ThreadCtx *>> idle;  // device -> retired contexts, buffers freed
};

Orphanage &orphanage() {
    static Orphanage *o = new Orphanage;  // never destroyed: the reaper may outlive exit()
    return *o;
}

void reaper() {
    Orphanage &o = orphanage();
    for (;;) {
        std::map<int, ThreadCtx *> m;
        {
            std::unique_lock<std::mutex> lock(o.mu);
            o.cv.wait(lock, [&] { return !o.q.empty(); });
            m = std::move(o.q.front());
            o.q.pop_front();
        }
        // Give the memory back and keep the streams and events for the next
        // new thread (thread_ctx): a JVM or gRPC pool that retires and
        // creates workers then makes no stream churn at all.  Each context is
        // freed under exit_mutex with the exit flag checked inside it, so no
        // free runs once exit() has begun (codec.cpp).
        for (auto &kv : m) {
            std::lock_guard<std::mutex> exit_lock(exit_mutex());
            if (process_exiting()) return;
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(kv.first);
            free_buffers(kv.second);
            (void)hipSetDevice(cur);
        }
        std::lock_guard<std::mutex> lock(o.mu);
        for (auto &kv : m) o.idle[kv.first].push_back(kv.second);
    }
}

// A retired context for this device, or nullptr.
ThreadCtx *adopt_idle(int dev) {
    Orphanage &o = orphanage();
    std::lock_guard<std::mutex> lock(o.mu);
    auto it = o.idle.find(dev);
    if (it == o.idle.end() || it->second.empty()) return nullptr;
    ThreadCtx *c = it->second.back();
    it->second.pop_back();
    return c;
}

void orphan(std::map<int, ThreadCtx *> &&ctx) {
    Orphanage &o = orphanage();
    std::lock_guard<std::mutex> lock(o.mu);
    o.q.push_back(std::move(ctx));
    if (!o.started) {
        o.started = true;
        std::thread(reaper).detach();
    }
    o.cv.notify_one();
}
}  // namespace

void release_thread_contexts() {
    release_all(t_ctx.m);
    release_idle_mirror_sets();
}

int grow(uint8_t **buf, size_t *cap, size_t want) {
    if (*cap >= want) {
        bounds::allow(*buf, *cap);
        return RS_OK;
    }
    if (*buf) RS_HIP(hipFree(*buf));
    *buf = nullptr;
    *cap = 0;
    RS_HIP(hipMalloc(reinterpret_cast<void **>(buf), want));
    *cap = want;
    bounds::allow(*buf, *cap);
    return RS_OK;
}

int grow_pinned(uint8_t **buf, size_t *cap, size_t want) {
    if (*cap >= want) return RS_OK;
    if (*buf) RS_HIP(hipHostFree(*buf));
    *buf = nullptr;
    *cap = 0;
    RS_HIP(hipHostMalloc(reinterpret_cast<void **>(buf), want, hipHostMallocDefault));
    *cap = want;
    return RS_OK;
}

// ---------------------------------------------------------------------------
// Host-buffer pipeline.  A call is cut into chunks staged through kStageBufs
// device buffers.  `stream3` carries every H2D copy and `stream` every kernel
// and D2H copy, each in chunk order, so chunk j's D2H runs beside chunk j+1's
// H2D; events hand each buffer from its upload to its kernels and back (after
// its D2H) to the H2D that reuses it.  (Two streams that each ran H2D ->
// kernel -> D2H fell into lockstep and never overlapped the directions; why
// the D2H copies share the kernels' stream: create_pipeline_streams.)
//
// The link is full duplex only for async copies from page-locked memory
// (57 GB/s one way, 97 GB/s both ways; pageable copies share one staged path
// at 56 GB/s in total, even from two host threads -- tools/pcie_probe.py).
// Pinned callers are copied directly.  Pageable callers (JNI arrays) go
// through a pinned mirror of each staging buffer: the pool of copy_pool.hpp
// fills chunk j's inputs into the mirror while the GPU moves chunk j-1, and
// drains chunk j-1's outputs once their D2H is done.
// ---------------------------------------------------------------------------
constexpr size_t kChunk = size_t(32) << 20;        // max bytes per slot per chunk
constexpr size_t kMinChunk = size_t(4) << 20;      // min bytes per slot per chunk (~8 chunks per call)
constexpr size_t kMirrorBytes = size_t(24) << 20;  // pinned mirror bytes per staging buffer
constexpr size_t kZeroCopyBytes = size_t(64) << 20; // single-chunk calls up to this size run zero-copy

// Bytes per slot per chunk for a call of `total` bytes per slot and `nslots`
// slots per buffer.
size_t chunks_per_call() {
    static const size_t v = [] {
        const char *e = tuning_env("RSAMD_CHUNKS");
        const long n = e ? std::atol(e) : 0;
        return n > 0 ? size_t(n) : size_t(8);
    }();
    return v;
}

size_t chunk_bytes(size_t total, int nslots, bool pinned) {
    const size_t per = chunks_per_call();
    size_t c = std::max(kMinChunk * 8 / per, (total / per + 255) / 256 * 256);
    // TUNING builds: RSAMD_MIRROR_BYTES overrides the mirror size per buffer
    static const size_t mirror = rsamd::tuning_size("RSAMD_MIRROR_BYTES", kMirrorBytes);
    if (!pinned) c = std::min(c, std::max<size_t>(size_t(1) << 20, mirror / size_t(std::max(1, nslots))));
    return std::min(kChunk, c);
}

// True when every non-null pointer is page-locked host memory known to HIP:
// pinned by the caller (torch pin_memory, hipHostMalloc, a pooled direct
// buffer).  The library itself never page-locks caller memory.
bool all_pinned(const uint8_t *const *ptrs, int n) {
    if (rsamd::thread_relocating()) return false;  // movable arrays (rs_set_relocator): stand-in addresses
    for (int i = 0; i < n; ++i) {
        if (!ptrs[i]) continue;
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, ptrs[i]) != hipSuccess) {
            (void)hipGetLastError();  // pageable memory: clear the sticky error
            return false;
        }
        if (attr.type != hipMemoryTypeHost) return false;
    }
    return true;
}

namespace {


int n_bufs(size_t n_chunks) { return int(std::min<size_t>(kStageBufs, std::max<size_t>(1, n_chunks))); }

int run_chunks_impl(ThreadCtx *ctx, size_t n_chunks, size_t buf_bytes, bool pinned, const ChunkIo &io,
                    const ChunkCode &code);

}  // namespace

int run_chunks(ThreadCtx *ctx, size_t n_chunks, size_t buf_bytes, bool pinned, const ChunkIo &io,
               const ChunkCode &code) {
    const int rc = run_chunks_impl(ctx, n_chunks, buf_bytes, pinned, io, code);
    if (rc) {
        (void)hipStreamSynchronize(ctx->stream3);
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamSynchronize(ctx->stream2);
    }
    return rc;
}

// Bytes above which a zero-copy pass's host copies go to the copy pool
// (TUNING builds: RSAMD_ZC_POOL_MIN).
size_t zc_pool_min() {
    static const size_t v = tuning_size("RSAMD_ZC_POOL_MIN", size_t(2) << 20);
    return v;
}

size_t zero_copy_limit() {
    static const size_t v = [] {
        const char *e = tuning_env("RSAMD_ZC_BYTES");
        return e ? size_t(std::strtoull(e, nullptr, 10)) : kZeroCopyBytes;
    }();
    return v;
}

int zero_copy_buffer(ThreadCtx *ctx, size_t buf_bytes) {
    if (ctx->zc_cap < buf_bytes) {
        if (ctx->zc) RS_HIP(hipHostFree(ctx->zc));
        ctx->zc = ctx->zc_dev = nullptr;
        ctx->zc_cap = 0;
        // TUNING builds: RSAMD_ZC_ALLOC 1 = mapped + the caller's NUMA policy, 2 = mapped non-coherent
        const size_t how = tuning_size("RSAMD_ZC_ALLOC", 0);
        const unsigned flags = how == 1 ? (hipHostMallocMapped | hipHostMallocNumaUser)
                             : how == 2 ? (hipHostMallocMapped | hipHostMallocNonCoherent)
                                        : (hipHostMallocMapped | hipHostMallocCoherent);
        RS_HIP(hipHostMalloc(reinterpret_cast<void **>(&ctx->zc), buf_bytes, flags));
        ctx->zc_cap = buf_bytes;
        RS_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&ctx->zc_dev), ctx->zc, 0));
    }
    bounds::allow(ctx->zc_dev, ctx->zc_cap);
    return RS_OK;
}

int next_signal(ThreadCtx *ctx, uint32_t **flag_dev, uint32_t **ctr, uint32_t *seq) {
    if (!ctx->sig) {
        RS_HIP(hipHostMalloc(reinterpret_cast<void **>(&ctx->sig), 256, hipHostMallocMapped | hipHostMallocCoherent));
        RS_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&ctx->sig_dev), ctx->sig, 0));
        __atomic_store_n(&ctx->sig[0], 0u, __ATOMIC_RELEASE);
        __atomic_store_n(&ctx->sig[1], 0u, __ATOMIC_RELEASE);
    }
    if (++ctx->sig_seq == 0) ctx->sig_seq = 1;
    *flag_dev = ctx->sig_dev;
    *ctr = reinterpret_cast<uint32_t *>(ctx->flag) + kSignalCtr;
    *seq = ctx->sig_seq;
    bounds::allow(ctx->sig_dev, 8);
    return RS_OK;
}

int wait_signal(ThreadCtx *ctx, uint32_t seq, uint32_t *mismatch) {
    // Spin: a small call's kernel ends a few microseconds after its launch, and
    // the stream's own completion costs ~3 us more to observe.
    // Past 100 us the stream is asked now and then whether it failed or went
    // idle without the signal.
    // A later launch of the same stream may already have signalled past seq
    // (the sequence numbers only grow, modulo 2^32).
    auto reached = [&] { return int32_t(__atomic_load_n(&ctx->sig[0], __ATOMIC_ACQUIRE) - seq) >= 0; };
    static const auto query_after = std::chrono::microseconds(tuning_size("RSAMD_SIGNAL_QUERY_US", 100));
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spins = 1;; ++spins) {
        if (reached()) break;
        if (spins % 64 != 0 || std::chrono::steady_clock::now() - t0 < query_after) continue;
        const hipError_t e = hipStreamQuery(ctx->stream);
        if (e == hipErrorNotReady) {
            (void)hipGetLastError();
            std::this_thread::yield();
            continue;
        }
        if (reached()) break;
        if (e != hipSuccess) return hip_fail(e, "small call (hipStreamQuery)");
        return fail(RS_E_HIP, "small call: the stream is idle and the kernel's completion signal is missing");
    }
    if (mismatch) *mismatch = __atomic_load_n(&ctx->sig[1], __ATOMIC_ACQUIRE);
    return RS_OK;
}

namespace {

// Single-chunk calls (<= 4 MiB per shard) skip the DMA pipeline: the inputs
// are copied into a coherent, device-mapped host buffer, the kernels read and
// write it over the link directly, and the outputs are copied back -- one
// launch and one stream sync instead of an async copy per shard each way and
// the event hand-offs.  Measured per call (tools/small_call_bench.py, 4+2,
// pageable): 1000-B shards 130 -> 36 us, 64 KiB 180 -> 40 us, 1 MiB 390-500
// -> 280-306 us, 4 MiB 810-1100 -> 660-725 us.  RSAMD_ZC_BYTES sets the size
// limit of the staging buffer (0 disables).

int run_zero_copy(ThreadCtx *ctx, size_t buf_bytes, const ChunkIo &io, const ChunkCode &code) {
    int zrc = zero_copy_buffer(ctx, buf_bytes);
    if (zrc) return zrc;
    std::vector<Xfer> in, out;
    io(0, &in, &out);
    // Host copies on the calling thread; the copy pool only above 2 MiB (its
    // wake-up costs more than a small memcpy; TUNING builds: RSAMD_ZC_POOL_MIN).
    // (Streaming stores on the calling thread instead of memcpy: no better,
    // profiles/r5/host_sizes_r5v.txt.)
    const bool use_pool = buf_bytes > zc_pool_min();
    auto copy = [&](const std::vector<rsamd::CopyJob> &jobs) {
        if (use_pool)
            rsamd::CopyPool::get().copy(jobs);
        else
            rsamd::CopyPool::copy_here(jobs);
    };
    std::vector<rsamd::CopyJob> jobs;
    for (const Xfer &x : in) jobs.push_back({ctx->zc + x.off, x.host, x.n});
    copy(jobs);
    int rc = code(0, ctx->zc_dev, ctx->stream);
    if (rc) return rc;
    RS_HIP(hipStreamSynchronize(ctx->stream));
    jobs.clear();
    for (const Xfer &x : out) jobs.push_back({x.host, ctx->zc + x.off, x.n});
    copy(jobs);
    return RS_OK;
}

// Stream of the pipeline's H2D copies: a stream of their own, so chunk j+1's
// upload is not queued behind chunk j's kernels (file decode: 4 x 8 MiB of
// uploads, then 90 us of kernels, per 1.05 ms chunk).  RSAMD_PIPE_STREAMS=2
// puts them back on the kernel stream.
hipStream_t upload_stream(const ThreadCtx *ctx) {
    static const bool two = [] {
        const char *e = tuning_env("RSAMD_PIPE_STREAMS");
        return e && std::atoi(e) == 2;
    }();
    return two ? ctx->stream : ctx->stream3;
}

int run_chunks_impl(ThreadCtx *ctx, size_t n_chunks, size_t buf_bytes, bool pinned, const ChunkIo &io,
                    const ChunkCode &code) {
    if (n_chunks == 1 && buf_bytes <= zero_copy_limit()) return run_zero_copy(ctx, buf_bytes, io, code);
    const int nbuf = n_bufs(n_chunks);
    int rc = grow(&ctx->stage, &ctx->stage_cap, buf_bytes * size_t(nbuf));
    if (rc) return rc;
    const bool staged = !pinned;
    if (staged) {
        rc = grow_pinned(&ctx->mirror, &ctx->mirror_cap, buf_bytes * size_t(nbuf));
        if (rc) return rc;
    }
    hipStream_t up_s = upload_stream(ctx), in_s = ctx->stream, out_s = RSAMD_PIPE_MODE == 3 ? ctx->stream : ctx->stream2;
    rsamd::CopyPool &pool = rsamd::CopyPool::get();
    // Staged outputs are drained nbuf - 1 chunks behind (their D2H is long
    // done by then), in the same pool batch as the next chunk's inputs.  A
    // mirror's output bytes are drained before the D2H that reuses it is issued.
    const size_t lag = size_t(std::max(1, nbuf - 1));
    std::deque<std::pair<size_t, std::vector<Xfer>>> pending;
    std::vector<Xfer> in, out;
    std::vector<rsamd::CopyJob> jobs;
    auto queue_drain = [&]() -> int {  // the oldest pending chunk: mirror -> caller
        const size_t pj = pending.front().first;
        RS_HIP(hipEventSynchronize(ctx->freed[pj % nbuf]));
        const uint8_t *mir = ctx->mirror + (pj % nbuf) * buf_bytes;
        for (const Xfer &x : pending.front().second) jobs.push_back({x.host, mir + x.off, x.n});
        pending.pop_front();
        return RS_OK;
    };
    for (size_t j = 0; j < n_chunks; ++j) {
        const size_t b = j % nbuf;
        uint8_t *dev = ctx->stage + b * buf_bytes;
        uint8_t *mir = staged ? ctx->mirror + b * buf_bytes : nullptr;
        in.clear();
        out.clear();
        io(j, &in, &out);
        if (staged) {
            jobs.clear();
            if (pending.size() >= lag) {
                rc = queue_drain();
                if (rc) return rc;
            }
            if (j >= size_t(nbuf)) RS_HIP(hipEventSynchronize(ctx->loaded[b]));  // chunk j - nbuf's H2D done
            for (const Xfer &x : in) jobs.push_back({mir + x.off, x.host, x.n});
            pool.copy(jobs);
        }
        if (j >= size_t(nbuf)) RS_HIP(hipStreamWaitEvent(up_s, ctx->freed[b], 0));  // device buffer free
        for (const Xfer &x : in)
            RS_HIP(hipMemcpyAsync(dev + x.off, staged ? mir + x.off : x.host, x.n, hipMemcpyHostToDevice, up_s));
        RS_HIP(hipEventRecord(ctx->loaded[b], up_s));
        if (up_s != in_s) RS_HIP(hipStreamWaitEvent(in_s, ctx->loaded[b], 0));
        rc = code(j, dev, in_s);
        if (rc) return rc;
        RS_HIP(hipEventRecord(ctx->coded[b], in_s));
        RS_HIP(hipStreamWaitEvent(out_s, ctx->coded[b], 0));
        for (const Xfer &x : out)
            RS_HIP(hipMemcpyAsync(staged ? mir + x.off : x.host, dev + x.off, x.n, hipMemcpyDeviceToHost, out_s));
        RS_HIP(hipEventRecord(ctx->freed[b], out_s));
        if (staged && !out.empty()) pending.emplace_back(j, out);
    }
    while (!pending.empty()) {
        jobs.clear();
        rc = queue_drain();
        if (rc) return rc;
        pool.copy(jobs);
    }
    RS_HIP(hipEventRecord(ctx->ready, out_s));
    RS_HIP(hipStreamWaitEvent(in_s, ctx->ready, 0));
    RS_HIP(hipStreamSynchronize(in_s));
    return RS_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// The mirrored pipeline (host.hpp).  Slot b of the call's slot set holds one
// chunk laid out as the caller's code expects; a chunk's life is
//   copy-in (pool, caller -> slot) -> kernels over the slot's device address
//   (ctx->stream, event done[b]) -> copy-out (pool, slot -> caller).
// The copy batch issued before chunk j's launch holds chunk j's inputs and
// the outputs of every earlier chunk whose kernels have completed; only the
// chunk that last used slot b must have been drained before the slot is
// refilled, so the CPU runs up to nbuf - 1 chunks ahead of the GPU.
// ---------------------------------------------------------------------------
namespace {
// Pinned bytes per slot (TUNING builds: RSAMD_MIRROR_BYTES).
// 64 MiB: a direct kernel over a chunk costs ~70 us on top of its bytes, so
// larger chunks run closer to the link (4+2 x 64 MiB, no host copies: 0.893 of
// the link bound at 24 MiB slots, 0.953 at 48 MiB; with the copies 0.853 /
// 0.888; 16 MiB 0.832; profiles/r5/host_legs_r5d.txt, r5e).  With 6 chunks per
// call (mirror_chunk_bytes) instead of 8 in 48 MiB slots, the bench's host legs
// (encode / decode {0,1} / file encode / file decode {0,5}, mean of four child
// processes alternated with the others) read 0.872 / 0.870 / 0.716 / 0.880 of
// the link bound against 0.854 / 0.839 / 0.691 / 0.845; 96 MiB slots with 4
// chunks and 128 MiB with 3 read the same as 64 MiB with 6 within a point
// (profiles/r5/host_legs_bigchunks_r6r.txt, host_legs_bigchunks2_r6s.txt).
size_t mirror_slot_bytes() {
    static const size_t v = rsamd::tuning_size("RSAMD_MIRROR_BYTES", size_t(64) << 20);
    return v;
}

// Slots in use (<= kMirrorBufs; TUNING builds: RSAMD_MIRROR_NBUF).  Three let
// the CPU copy one chunk in and drain one out while the GPU codes a third.
int mirror_nbuf() {
    static const int v = int(std::max<size_t>(2, std::min<size_t>(kMirrorBufs, rsamd::tuning_size("RSAMD_MIRROR_NBUF", 3))));
    return v;
}

// The slots, shared by the process's threads: a call takes an idle set of
// its device for its duration (or makes one), so the pinned memory follows the
// number of concurrent large pageable calls, not the number of threads that
// ever made one (a JVM's I/O pool); at most kIdleSets idle sets per device are
// kept, the rest freed when returned.
struct MirrorSet {
    int dev = 0;
    uint8_t *buf = nullptr, *dev_ptr = nullptr;  // host and device addresses of the slots
    size_t cap = 0;
    hipEvent_t done[kMirrorBufs] = {};  // slot b's kernels done (its outputs may be drained)
};

constexpr size_t kIdleSets = 4;
// Pinned bytes idle sets may hold per device (a set of three 64 MiB slots is
// 192 MiB): beyond it a returned set is freed.  rs_thread_release frees every
// idle set (release_idle_mirror_sets).
constexpr size_t kIdleBytes = size_t(384) << 20;

struct MirrorPool {
    std::mutex mu;
    std::map<int, std::vector<MirrorSet *>> idle;  // device -> idle sets
};

MirrorPool &mirror_pool() {
    static MirrorPool *p = new MirrorPool;  // never destroyed: no HIP calls at exit
    return *p;
}

void free_set(MirrorSet *s) {
    if (s->buf) (void)hipHostFree(s->buf);
    for (hipEvent_t &ev : s->done)
        if (ev) (void)hipEventDestroy(ev);
    delete s;
}

// An idle set of the current device with at least `bytes` of slots (the
// largest idle one, grown if needed), or a new one.
int acquire_set(size_t bytes, MirrorSet **out) {
    *out = nullptr;
    int dev = 0;
    RS_HIP(hipGetDevice(&dev));
    MirrorSet *s = nullptr;
    {
        MirrorPool &p = mirror_pool();
        std::lock_guard<std::mutex> lock(p.mu);
        std::vector<MirrorSet *> &v = p.idle[dev];
        if (!v.empty()) {
            auto best = std::max_element(v.begin(), v.end(), [](MirrorSet *a, MirrorSet *b) { return a->cap < b->cap; });
            s = *best;
            v.erase(best);
        }
    }
    if (!s) {
        s = new MirrorSet;
        s->dev = dev;
    }
    *out = s;  // (returned by release_set also on the error paths below)
    if (s->cap < bytes) {
        if (s->buf) RS_HIP(hipHostFree(s->buf));
        s->buf = s->dev_ptr = nullptr;
        s->cap = 0;
        // TUNING builds: RSAMD_MIRROR_ALLOC 0 = hipHostMallocDefault, 1 = non-coherent,
        // 2 = coherent, 3 = mapped, pages placed by the calling thread's NUMA policy
        // (A/B of where and how the slots are pinned).  The default places the slots
        // by the caller's policy: a service bound to the GPU's NUMA node (as bench.py
        // binds its host legs) gets them there, 4+2 x 64 MiB pageable encode 0.853 ->
        // 0.882 of the link bound, file encode 0.852 -> 0.861, file decode 0.733 ->
        // 0.779 (profiles/r5/host_legs_r5e.txt).
        const size_t how = rsamd::tuning_size("RSAMD_MIRROR_ALLOC", 3);
        const unsigned flags = how == 1 ? (hipHostMallocMapped | hipHostMallocNonCoherent)
                             : how == 2 ? (hipHostMallocMapped | hipHostMallocCoherent)
                             : how == 3 ? (hipHostMallocMapped | hipHostMallocNumaUser)
                                        : hipHostMallocDefault;
        RS_HIP(hipHostMalloc(reinterpret_cast<void **>(&s->buf), bytes, flags));
        s->cap = bytes;
        RS_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&s->dev_ptr), s->buf, 0));
    }
    for (hipEvent_t &ev : s->done)
        if (!ev) RS_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    bounds::allow(s->dev_ptr, s->cap);
    return RS_OK;
}

// Back to the pool once nothing of the call uses it (the caller has
// synchronised); beyond kIdleSets idle sets per device it is freed.
void release_set(MirrorSet *s) {
    if (!s) return;
    {
        MirrorPool &p = mirror_pool();
        std::lock_guard<std::mutex> lock(p.mu);
        std::vector<MirrorSet *> &v = p.idle[s->dev];
        size_t held = s->cap;
        for (const MirrorSet *x : v) held += x->cap;
        if ((v.size() < kIdleSets && held <= kIdleBytes) || process_exiting()) {
            v.push_back(s);
            return;
        }
    }
    free_set(s);
}
}  // namespace

void release_idle_mirror_sets() {
    if (process_exiting()) return;
    std::vector<MirrorSet *> drop;
    {
        MirrorPool &p = mirror_pool();
        std::lock_guard<std::mutex> lock(p.mu);
        for (auto &kv : p.idle) {
            drop.insert(drop.end(), kv.second.begin(), kv.second.end());
            kv.second.clear();
        }
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (MirrorSet *s : drop) {
        (void)hipSetDevice(s->dev);
        free_set(s);
    }
    (void)hipSetDevice(cur);
}

namespace {

// TUNING builds: RSAMD_TRACE=<file> appends one JSON line per mirrored call
// with every chunk's copy batch (host ns from the call's start), launch, and
// kernel start / end (GPU events, on the same clock through a reference event
// synchronised at the start), and which chunks each batch drained.
struct MirrorTrace {
    const char *path = nullptr;
    std::chrono::steady_clock::time_point t0;
    hipEvent_t ref = nullptr;
    std::vector<hipEvent_t> ks, ke;
    std::vector<int64_t> cb, ce, launched;
    std::vector<std::vector<size_t>> drained;
    int64_t now() const {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    }
    void begin(hipStream_t s, size_t n) {
        path = tuning_env("RSAMD_TRACE");
        if (!path) return;
        (void)hipEventCreate(&ref);
        ks.assign(n, nullptr);
        ke.assign(n, nullptr);
        for (size_t j = 0; j < n; ++j) {
            (void)hipEventCreate(&ks[j]);
            (void)hipEventCreate(&ke[j]);
        }
        cb.assign(n, 0);
        ce.assign(n, 0);
        launched.assign(n, 0);
        drained.assign(n, {});
        (void)hipStreamSynchronize(s);
        (void)hipEventRecord(ref, s);
        (void)hipEventSynchronize(ref);
        t0 = std::chrono::steady_clock::now();
    }
    void end(hipStream_t s, size_t bytes) {
        if (!path) return;
        (void)hipStreamSynchronize(s);
        const int64_t total = now();
        FILE *f = std::fopen(path, "a");
        if (f) {
            std::fprintf(f, "{\"bytes\": %zu, \"total_ns\": %lld, \"chunks\": [", bytes, (long long)total);
            for (size_t j = 0; j < cb.size(); ++j) {
                float a = 0, b = 0;
                (void)hipEventElapsedTime(&a, ref, ks[j]);
                (void)hipEventElapsedTime(&b, ref, ke[j]);
                std::fprintf(f, "%s{\"j\": %zu, \"copy\": [%lld, %lld], \"launch\": %lld, \"kernel\": [%lld, %lld], \"drained\": [",
                             j ? ", " : "", j, (long long)cb[j], (long long)ce[j], (long long)launched[j],
                             (long long)(a * 1e6), (long long)(b * 1e6));
                for (size_t q = 0; q < drained[j].size(); ++q) std::fprintf(f, "%s%zu", q ? ", " : "", drained[j][q]);
                std::fprintf(f, "]}");
            }
            std::fprintf(f, "]}\n");
            std::fclose(f);
        }
    }
    ~MirrorTrace() {  // also when the call returned early with an error
        for (hipEvent_t e : ks)
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : ke)
            if (e) (void)hipEventDestroy(e);
        if (ref) (void)hipEventDestroy(ref);
    }
};

int run_mirrored_impl(ThreadCtx *ctx, MirrorSet *ms, int nbuf, size_t n_chunks, size_t buf_bytes,
                      const ChunkIo &io, const ChunkCode &code, const ChunkSide &side) {
    int rc = RS_OK;
    MirrorTrace tr;
    tr.begin(ctx->stream, n_chunks);
    // One stream: chunks alternating over two streams (one chunk's kernel
    // starting while the previous one drains) ran two kernels at a time at the
    // same aggregate rate (0.831 / 0.805 of the link bound, 0.893 / 0.888 without
    // host copies; profiles/r5/host_legs_r5d.txt, r5e).  TUNING builds:
    // RSAMD_MIRROR_STREAMS=2; stream2 then first waits for what the caller
    // queued on stream (the verify flag's reset).
    const int nstreams = int(std::min<size_t>(2, std::max<size_t>(1, rsamd::tuning_size("RSAMD_MIRROR_STREAMS", 1))));
    hipStream_t ss[2] = {ctx->stream, ctx->stream2};
    if (nstreams > 1) {
        RS_HIP(hipEventRecord(ctx->ready, ctx->stream));
        RS_HIP(hipStreamWaitEvent(ctx->stream2, ctx->ready, 0));
    }
    rsamd::CopyPool &pool = rsamd::CopyPool::get();
    // TUNING builds: RSAMD_MIRROR_NOCOPY=1 skips the host copies (wrong
    // results; the kernels' rate on the slots without CPU memory traffic)
    const bool nocopy = rsamd::tuning_size("RSAMD_MIRROR_NOCOPY", 0) != 0;
    struct Pending {
        size_t j;
        std::vector<Xfer> out;
        std::vector<rsamd::CopyJob> after;  // side copies behind the chunk's kernels
    };
    std::deque<Pending> pending;  // launched, slot not yet released: outputs not copied out (chunk order)
    std::vector<rsamd::CopyJob> jobs;
    std::vector<Xfer> in, out;
    size_t batch = 0;  // the chunk whose copy batch is being built (trace)
    auto drain_front = [&]() {
        const Pending &p = pending.front();
        if (tr.path) tr.drained[batch].push_back(p.j);
        const uint8_t *slot = ms->buf + (p.j % size_t(nbuf)) * buf_bytes;
        for (const Xfer &x : p.out) jobs.push_back({x.host, slot + x.off, x.n});
        jobs.insert(jobs.end(), p.after.begin(), p.after.end());
        pending.pop_front();
    };
    auto done = [&](size_t j) {  // chunk j's kernels have completed
        const hipError_t e = hipEventQuery(ms->done[j % size_t(nbuf)]);
        if (e == hipErrorNotReady) (void)hipGetLastError();
        return e == hipSuccess;
    };
    for (size_t j = 0; j < n_chunks; ++j) {
        const size_t b = j % size_t(nbuf);
        batch = j;
        jobs.clear();
        // the slot's previous chunk first (waited for), then whatever else is done
        while (!pending.empty() && pending.front().j + size_t(nbuf) <= j) {
            RS_HIP(hipEventSynchronize(ms->done[pending.front().j % size_t(nbuf)]));
            drain_front();
        }
        while (!pending.empty() && done(pending.front().j)) drain_front();
        in.clear();
        out.clear();
        io(j, &in, &out);
        uint8_t *slot = ms->buf + b * buf_bytes;
        for (const Xfer &x : in) jobs.push_back({slot + x.off, x.host, x.n});
        std::vector<rsamd::CopyJob> after;
        if (side) side(j, slot, &jobs, &after);
        if (tr.path) tr.cb[j] = tr.now();
        if (!nocopy) pool.copy(jobs);
        hipStream_t st = ss[j % size_t(nstreams)];
        if (tr.path) {
            tr.ce[j] = tr.now();
            (void)hipEventRecord(tr.ks[j], st);
        }
        rc = code(j, ms->dev_ptr + b * buf_bytes, st);
        if (rc) return rc;
        if (tr.path) {
            (void)hipEventRecord(tr.ke[j], st);
            tr.launched[j] = tr.now();
        }
        RS_HIP(hipEventRecord(ms->done[b], st));
        // (also with no outputs -- verify: the slot's inputs may not be
        // refilled before the chunk's kernels have read them)
        pending.push_back({j, out, std::move(after)});
    }
    batch = n_chunks - 1;
    while (!pending.empty()) {
        jobs.clear();
        RS_HIP(hipEventSynchronize(ms->done[pending.front().j % size_t(nbuf)]));
        drain_front();
        while (!pending.empty() && done(pending.front().j)) drain_front();
        if (!nocopy) pool.copy(jobs);
    }
    if (nstreams > 1) {  // stream carries on behind both (the caller reads the verify flag next)
        RS_HIP(hipEventRecord(ctx->ready, ctx->stream2));
        RS_HIP(hipStreamWaitEvent(ctx->stream, ctx->ready, 0));
    }
    RS_HIP(hipStreamSynchronize(ctx->stream));
    tr.end(ctx->stream, buf_bytes);
    return RS_OK;
}
}  // namespace

size_t mirror_chunk_bytes(size_t total, int nslots, size_t granule) {
    granule = std::max<size_t>(1, granule);
    // 6 chunks per call when they fit the slot (mirror_slot_bytes), never
    // under 2 MiB per slot:
    // calls up to 3 MiB per shard then run as 4 equal chunks (ramp_bounds), 4
    // MiB as 5.  Each chunk costs a pool batch, a launch and an event; against
    // a 256 KiB floor (7-11 chunks) 4+2 calls of 1 / 2 / 4 MiB per shard took
    // 196-198 / 309-320 / 495-507 us instead of 227-285 / 359-384 / 564-584,
    // 4 and 16 MiB files 233-275 / 555-573 instead of 264-360 / 636-917; 64 MiB
    // calls are unchanged (profiles/r5/host_sizes_chunkmin_r6k.txt).  TUNING
    // builds: RSAMD_MIRROR_CHUNKS, RSAMD_MIRROR_CHUNK_MIN.
    const size_t per = std::max<size_t>(1, rsamd::tuning_size("RSAMD_MIRROR_CHUNKS", 6));
    size_t c = std::max<size_t>(rsamd::tuning_size("RSAMD_MIRROR_CHUNK_MIN", size_t(2) << 20), total / per);
    c = std::min(c, mirror_slot_bytes() / size_t(std::max(1, nslots)));
    c = std::max(granule, c / granule * granule);
    return c;
}

std::vector<size_t> ramp_bounds(size_t total, size_t chunk, size_t granule) {
    granule = std::max<size_t>(1, granule);
    chunk = std::max(granule, chunk / granule * granule);
    auto g = [&](size_t x) { return std::max(granule, x / granule * granule); };
    std::vector<size_t> sizes;
    const size_t q = g(chunk / 4), h = g(chunk / 2);
    if (total <= 2 * (q + h)) {  // short call: up to 4 equal chunks
        const size_t n = std::max<size_t>(1, std::min<size_t>(4, total / granule));
        const size_t each = g((total + n - 1) / n);
        for (size_t done = 0; done < total; done += each) sizes.push_back(std::min(each, total - done));
    } else {  // a quarter and a half chunk either side of whole chunks
        // (granule-sized pieces up to the last one, which takes the remainder)
        const size_t mid = total - 2 * (q + h), nbody = (mid + chunk - 1) / chunk;
        const size_t each = g(mid / nbody);
        sizes = {q, h};
        for (size_t i = 0; i < nbody && each * (i + 1) <= mid; ++i) sizes.push_back(each);
        sizes.push_back(h);
        size_t sum = 0;
        for (size_t x : sizes) sum += x;
        sizes.push_back(total - sum);
    }
    std::vector<size_t> b{0};
    for (size_t x : sizes) b.push_back(b.back() + x);
    return b;
}

int run_mirrored(ThreadCtx *ctx, size_t n_chunks, size_t buf_bytes, const ChunkIo &io, const ChunkCode &code,
                 const ChunkSide &side) {
    const int nbuf = int(std::min<size_t>(size_t(mirror_nbuf()), std::max<size_t>(1, n_chunks)));
    MirrorSet *ms = nullptr;
    int rc = acquire_set(buf_bytes * size_t(nbuf), &ms);
    if (!rc) rc = run_mirrored_impl(ctx, ms, nbuf, n_chunks, buf_bytes, io, code, side);
    if (rc) {  // nothing of the call left in flight before the slots go back
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamSynchronize(ctx->stream2);
    }
    release_set(ms);
    return rc;
}

}  // namespace host

#if RSAMD_BOUNDS
// ---------------------------------------------------------------------------
// The bounds-checking build's host half (bounds.hpp): one process-wide table,
// set by the outermost Scope of a call and widened by allow(), uploaded to
// both translation units' device copies.
// ---------------------------------------------------------------------------
namespace bounds {
namespace {
std::recursive_mutex g_mu;
thread_local int t_depth = 0;
thread_local bool t_passive = false;  // inside a stream capture: no checking
BoundsTable g_table;
BoundsReport g_seen;  // accumulated over calls until rs_bounds_report

void put(const BoundsTable &t) {
    (void)bounds_put_kernels(t);
    (void)bounds_put_layout(t);
}

void take() {
    for (auto fn : {bounds_take_kernels, bounds_take_layout}) {
        BoundsReport r;
        if (fn(&r) != hipSuccess || r.count == 0) continue;
        if (g_seen.count == 0) {
            g_seen.addr = r.addr;
            g_seen.len = r.len;
            g_seen.where = r.where;
        }
        g_seen.count += r.count;
    }
}
}  // namespace

Scope::Scope(const void *stream) {
    g_mu.lock();
    if (t_depth++ > 0) return;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    t_passive = stream && hipStreamIsCapturing(static_cast<hipStream_t>(const_cast<void *>(stream)), &st) == hipSuccess &&
                st != hipStreamCaptureStatusNone;
    if (t_passive) return;
    (void)hipDeviceSynchronize();
    g_table = BoundsTable{};
    g_table.n = 0;
    put(g_table);
}

Scope::~Scope() {
    if (--t_depth == 0 && !t_passive) {
        (void)hipDeviceSynchronize();
        take();
        g_table = BoundsTable{};  // outside a call: everything allowed
        put(g_table);
    }
    g_mu.unlock();
}

// A host-side finding (a declared range not inside a live allocation).
void note(uint64_t addr, uint64_t len, unsigned where) {
    if (g_seen.count++ == 0) {
        g_seen.addr = addr;
        g_seen.len = len;
        g_seen.where = where;
    }
}

void allow(const void *p, size_t n, bool check_alloc) {
    if (!p || n == 0) return;
    std::lock_guard<std::recursive_mutex> lock(g_mu);
    if (t_depth == 0 || t_passive) return;
    if (check_alloc) {
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
            (void)hipGetLastError();
            note(reinterpret_cast<uint64_t>(p), n, 900001);  // not in any live allocation
        } else if (attr.type == hipMemoryTypeDevice) {
            hipDeviceptr_t base = nullptr;
            size_t size = 0;
            if (hipMemGetAddressRange(&base, &size, const_cast<void *>(p)) != hipSuccess) {
                (void)hipGetLastError();
                note(reinterpret_cast<uint64_t>(p), n, 900002);
            } else if (static_cast<const uint8_t *>(p) + n > static_cast<const uint8_t *>(base) + size) {
                note(reinterpret_cast<uint64_t>(p), n, 900003);  // runs past its allocation:
                n = size_t(static_cast<const uint8_t *>(base) + size - static_cast<const uint8_t *>(p));  // kernels get the part inside
            }
        }
    }
    if (g_table.n == kBoundsAll) return;
    if (g_table.n == kBoundsMax) {  // table full: stop checking for the rest of the call
        g_table.n = kBoundsAll;
        put(g_table);
        return;
    }
    const uint64_t lo = reinterpret_cast<uint64_t>(p);
    for (uint32_t i = 0; i < g_table.n; ++i)
        if (g_table.lo[i] == lo && g_table.hi[i] == lo + n) return;
    g_table.lo[g_table.n] = lo;
    g_table.hi[g_table.n] = lo + n;
    ++g_table.n;
    put(g_table);  // widens the table: kernels already running see a superset
}

void report(BoundsReport *out) {
    std::lock_guard<std::recursive_mutex> lock(g_mu);
    *out = g_seen;
    g_seen = BoundsReport{};
}
}  // namespace bounds
#endif

}  // namespace rsamd
