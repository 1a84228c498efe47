// host.cpp -- the host side of the host-buffer entry points (host.hpp):
// thread-local error text, per-(thread, device) staging contexts, page-locking
// of pageable caller buffers, and the chunked H2D -> kernels -> D2H pipeline
// with its zero-copy path for single-chunk calls.
#include "host.hpp"

#include <algorithm>
#include <atomic>
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
        if (process_exiting()) return;
        // Give the memory back and keep the streams and events for the next
        // new thread (thread_ctx): a JVM or gRPC pool that retires and
        // creates workers then makes no stream churn at all.
        int cur = 0;
        (void)hipGetDevice(&cur);
        for (auto &kv : m) {
            (void)hipSetDevice(kv.first);
            free_buffers(kv.second);
        }
        (void)hipSetDevice(cur);
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

void release_thread_contexts() { release_all(t_ctx.m); }

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

namespace {
struct HostRegistry;
HostRegistry &host_registry();
std::mutex &registry_mutex(HostRegistry &reg);
bool registry_holds_locked(HostRegistry &reg, const void *p);  // below: locked for a call by HostRegistration
}

// True when every non-null pointer is page-locked host memory known to HIP
// and stays so for the call: memory that HostRegistration locked for another
// thread's call reads as pinned too, but is unlocked when that call ends, so
// it counts as pageable here (the caller then locks it and shares that
// registration by reference count).  The registry's lock is held across each
// pointer's attribute query and registry lookup: a registration released
// between the two would otherwise read as the caller's own pinning, and the
// call would run on pages nobody keeps locked.
bool all_pinned(const uint8_t *const *ptrs, int n) {
    HostRegistry &reg = host_registry();
    std::lock_guard<std::mutex> guard(registry_mutex(reg));
    for (int i = 0; i < n; ++i) {
        if (!ptrs[i]) continue;
        if (registry_holds_locked(reg, ptrs[i])) return false;
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, ptrs[i]) != hipSuccess) {
            (void)hipGetLastError();  // pageable memory: clear the sticky error
            return false;
        }
        if (attr.type != hipMemoryTypeHost) return false;
    }
    return true;
}

// Page-locks pageable caller memory for the duration of one call
// (hipHostRegister: ~0.2 ms per 64 MiB the first time a range is seen,
// microseconds after) so the direct kernels code it in place.  Since the
// end of round 4 only ranges made of whole pages of the caller's own bytes
// are locked (capi.cpp run_direct_interior, whole_pages): a lock rounded out
// to pages reached into neighbouring allocations, which the runtime locks
// for its own pageable copies, and every GPU fault of rounds 3 and 4 surfaced
// in such a copy after calls that had locked NumPy memory.
//
// Registrations go through a process-wide registry of page ranges: calls on
// the same caller buffers (several threads, or one array passed twice) share
// one registration by reference count, and a range that partly overlaps a
// registered one is not registered again -- registering the same pages twice
// and unregistering one while the other is in use aborts inside the HIP
// runtime.  All or nothing: if any range cannot be locked the call is staged.
// The destructor releases after the call's kernels have completed, also on
// its error paths.  Off unless rs_set_host_register(1) (TUNING builds:
// RSAMD_HOST_REGISTER=1 at load).
namespace {

struct HostRegistry {
    std::mutex mu;
    std::map<uintptr_t, std::pair<uintptr_t, int>> regs;  // page start -> (page end, references)
};

std::atomic<int64_t> g_unregister_failures{0};

HostRegistry &host_registry() {
    static HostRegistry *r = new HostRegistry;  // never destroyed: no HIP calls at exit
    return *r;
}

std::mutex &registry_mutex(HostRegistry &reg) { return reg.mu; }

bool registry_holds_locked(HostRegistry &reg, const void *p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    auto next = reg.regs.upper_bound(a);
    if (next == reg.regs.begin()) return false;
    const auto prev = std::prev(next);
    return a >= prev->first && a < prev->second.first;
}

// Drops this call's references; the last one unregisters.  Caller holds reg.mu.
void release_locked(HostRegistry &reg, std::vector<uintptr_t> &held) {
    for (uintptr_t ps : held) {
        auto it = reg.regs.find(ps);
        if (it != reg.regs.end() && --it->second.second == 0) {
            const hipError_t e = hipHostUnregister(reinterpret_cast<void *>(ps));
            if (e != hipSuccess) {  // never seen; said once, as it would leave the pages locked
                (void)hipGetLastError();
                g_unregister_failures.fetch_add(1);
                static std::atomic<bool> said{false};
                if (!said.exchange(true))
                    std::fprintf(stderr, "librsamd: hipHostUnregister(%p) failed: %s\n", reinterpret_cast<void *>(ps),
                                 hipGetErrorString(e));
            }
            reg.regs.erase(it);
        }
    }
    held.clear();
}

}  // namespace

namespace {
// Off by default (include/rs_amd.h rs_set_host_register); a TUNING build's
// RSAMD_HOST_REGISTER=1 sets the initial value.
std::atomic<int> &host_register_flag() {
    static std::atomic<int> *f = new std::atomic<int>([] {
        const char *e = tuning_env("RSAMD_HOST_REGISTER");
        return e && e[0] == '1' ? 1 : 0;
    }());
    return *f;
}
}  // namespace

int set_host_register(int enable) {
    if (enable < 0) return host_register_flag().load();
    return host_register_flag().exchange(enable ? 1 : 0);
}

bool HostRegistration::lock(const std::vector<std::pair<const uint8_t *, size_t>> &ranges) {
    if (!host_register_flag().load()) return false;
    // The call's page ranges, sorted and merged: shards that are slices of
    // one allocation (sharing boundary pages) become one registration.
    constexpr uintptr_t kPage = 4096;
    std::vector<std::pair<uintptr_t, uintptr_t>> pages;
    for (const auto &r : ranges) {
        if (!r.first || r.second == 0) continue;
        const uintptr_t a = reinterpret_cast<uintptr_t>(r.first);
        pages.push_back({a & ~(kPage - 1), (a + r.second + kPage - 1) & ~(kPage - 1)});
    }
    std::sort(pages.begin(), pages.end());
    std::vector<std::pair<uintptr_t, uintptr_t>> merged;
    for (const auto &pr : pages) {
        if (!merged.empty() && pr.first <= merged.back().second)
            merged.back().second = std::max(merged.back().second, pr.second);
        else
            merged.push_back(pr);
    }
    HostRegistry &reg = host_registry();
    std::lock_guard<std::mutex> guard(reg.mu);
    for (const auto &pr : merged) {
        const uintptr_t ps = pr.first, pe = pr.second;
        auto next = reg.regs.upper_bound(ps);  // first registration starting after ps
        if (next != reg.regs.begin()) {
            auto prev = std::prev(next);
            if (prev->second.first >= pe) {  // already covered: share it
                ++prev->second.second;
                held_.push_back(prev->first);
                continue;
            }
            if (prev->second.first > ps) {  // partial overlap
                release_locked(reg, held_);
                return false;
            }
        }
        if ((next != reg.regs.end() && next->first < pe) ||
            hipHostRegister(reinterpret_cast<void *>(ps), pe - ps, hipHostRegisterMapped) != hipSuccess) {
            (void)hipGetLastError();
            release_locked(reg, held_);
            return false;
        }
        reg.regs.emplace(ps, std::make_pair(pe, 1));
        held_.push_back(ps);
    }
    return true;
}

int registry_state(int64_t *out, int n) {
    int64_t v[3] = {0, 0, g_unregister_failures.load()};
    {
        HostRegistry &reg = host_registry();
        std::lock_guard<std::mutex> guard(reg.mu);
        v[0] = int64_t(reg.regs.size());
        for (const auto &kv : reg.regs) v[1] += int64_t((kv.second.first - kv.first) / 4096);
    }
    for (int i = 0; out && i < n && i < 3; ++i) out[i] = v[i];
    return 3;
}

HostRegistration::~HostRegistration() {
    if (held_.empty()) return;
    HostRegistry &reg = host_registry();
    std::lock_guard<std::mutex> guard(reg.mu);
    release_locked(reg, held_);
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

int zero_copy_buffer(ThreadCtx *ctx, size_t buf_bytes) {
    if (ctx->zc_cap < buf_bytes) {
        if (ctx->zc) RS_HIP(hipHostFree(ctx->zc));
        ctx->zc = ctx->zc_dev = nullptr;
        ctx->zc_cap = 0;
        RS_HIP(hipHostMalloc(reinterpret_cast<void **>(&ctx->zc), buf_bytes,
                             hipHostMallocMapped | hipHostMallocCoherent));
        ctx->zc_cap = buf_bytes;
        RS_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&ctx->zc_dev), ctx->zc, 0));
    }
    bounds::allow(ctx->zc_dev, ctx->zc_cap);
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
size_t zero_copy_limit() {
    static const size_t v = [] {
        const char *e = tuning_env("RSAMD_ZC_BYTES");
        return e ? size_t(std::strtoull(e, nullptr, 10)) : kZeroCopyBytes;
    }();
    return v;
}

int run_zero_copy(ThreadCtx *ctx, size_t buf_bytes, const ChunkIo &io, const ChunkCode &code) {
    int zrc = zero_copy_buffer(ctx, buf_bytes);
    if (zrc) return zrc;
    std::vector<Xfer> in, out;
    io(0, &in, &out);
    // Host copies on the calling thread; the copy pool only above 2 MiB (its
    // wake-up costs more than a small memcpy).
    const bool use_pool = buf_bytes > (size_t(2) << 20);
    std::vector<rsamd::CopyJob> jobs;
    for (const Xfer &x : in) jobs.push_back({ctx->zc + x.off, x.host, x.n});
    if (use_pool) {
        rsamd::CopyPool::get().copy(jobs);
    } else {
        for (const rsamd::CopyJob &j : jobs) std::memcpy(j.dst, j.src, j.n);
    }
    int rc = code(0, ctx->zc_dev, ctx->stream);
    if (rc) return rc;
    RS_HIP(hipStreamSynchronize(ctx->stream));
    jobs.clear();
    for (const Xfer &x : out) jobs.push_back({x.host, ctx->zc + x.off, x.n});
    if (use_pool) {
        rsamd::CopyPool::get().copy(jobs);
    } else {
        for (const rsamd::CopyJob &j : jobs) std::memcpy(j.dst, j.src, j.n);
    }
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
