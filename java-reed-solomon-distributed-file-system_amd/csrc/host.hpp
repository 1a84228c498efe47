// host.hpp -- host side of the C-ABI's host-buffer entry points: error text,
// the per-(thread, device) staging context, page-locking of caller buffers
// and the chunked H2D -> kernels -> D2H pipeline (host.cpp).  capi.cpp builds
// every host-buffer call of include/rs_amd.h on these.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include "copy_pool.hpp"

namespace rsamd {
namespace host {

// ---- errors: the thread's last message (rs_last_error_message) ------------
int fail(int code, const std::string &msg);
int hip_fail(hipError_t e, const char *where);
const char *last_error();

#define RS_HIP(call)                                                  \
    do {                                                              \
        hipError_t e_ = (call);                                       \
        if (e_ != hipSuccess) return ::rsamd::host::hip_fail(e_, #call); \
    } while (0)

// ---- per-(thread, device) context ------------------------------------------
// Per-call staging of rs_decode_batch_masked_dev (stripe pattern ids or
// bitmasks, plus records on the dedupe path): pinned host + device bytes,
// reused only after `done` (recorded on the caller's stream behind the
// call's kernels) has completed.  The upload runs on the context's H2D
// stream and the caller's stream waits for `uploaded`, so it overlaps the
// previous call's kernels instead of queueing behind them.
struct MaskedSlot {
    uint8_t *dev = nullptr;
    size_t dev_cap = 0;
    uint8_t *host = nullptr;
    size_t host_cap = 0;
    hipEvent_t done = nullptr;
    hipEvent_t uploaded = nullptr;
};

#ifndef RSAMD_STAGE_BUFS
#define RSAMD_STAGE_BUFS 3  // A/B builds: make KDEFS=-DRSAMD_STAGE_BUFS=n
#endif
constexpr int kStageBufs = RSAMD_STAGE_BUFS;  // staging buffers of the host-buffer pipeline
#ifndef RSAMD_MIRROR_BUFS
#define RSAMD_MIRROR_BUFS 4  // A/B builds: make KDEFS=-DRSAMD_MIRROR_BUFS=n
#endif
constexpr int kMirrorBufs = RSAMD_MIRROR_BUFS;  // slots of the mirrored pipeline (run_mirrored)

struct ThreadCtx {
    hipStream_t stream = nullptr;   // host pipeline: kernels, in chunk order
    hipStream_t stream2 = nullptr;  // host pipeline: D2H copies, in chunk order
    hipStream_t stream3 = nullptr;  // host pipeline: H2D copies, in chunk order
    hipEvent_t ready = nullptr;     // joins stream2 back into stream
    hipEvent_t coded[kStageBufs] = {};   // buffer b's kernels done (stream -> stream2)
    hipEvent_t freed[kStageBufs] = {};   // buffer b's D2H done (stream2 -> stream3, and the host)
    hipEvent_t loaded[kStageBufs] = {};  // buffer b's H2D done (stream3 -> stream; its pinned mirror may be refilled)
    uint8_t *stage = nullptr;       // kStageBufs device staging buffers
    size_t stage_cap = 0;
    uint8_t *mirror = nullptr;      // their pinned host mirrors (pageable callers only)
    size_t mirror_cap = 0;
    uint8_t *plan = nullptr;   // per-call plan images (rs_code_some_shards)
    size_t plan_cap = 0;
    int *flag = nullptr;       // verify result
    uint8_t *file = nullptr;   // file staging (rs_file_encode / rs_file_decode)
    size_t file_cap = 0;
    uint8_t *zc = nullptr;      // small calls: coherent, device-mapped host buffer the kernels use directly
    uint8_t *zc_dev = nullptr;  // its device address
    size_t zc_cap = 0;
    // Small calls' completion signal (kernels.hpp DirectSignal): two coherent,
    // device-mapped host words the kernel stores into and the thread spins on;
    // the block counter is a word of `flag` (kSignalCtr).
    uint32_t *sig = nullptr, *sig_dev = nullptr;
    uint32_t sig_seq = 0;
    bool flag_dirty = true;  // the verify word may be nonzero (zeroed by a memset before the next verify)
    // rs_decode_batch_masked_dev: two staging slots used in turn, so a call's
    // host-side preparation overlaps the previous call's kernels.
    MaskedSlot masked[2];
    int masked_next = 0;
};

int need_device();
// The calling thread's context on its current device (created on first use).
int thread_ctx(ThreadCtx **out);
// Frees every context of the calling thread and every idle pooled slot set
// (rs_thread_release).
void release_thread_contexts();
// Frees the process's idle mirrored-pipeline slot sets (pinned host memory).
void release_idle_mirror_sets();
// Device / pinned-host buffers that only grow.
int grow(uint8_t **buf, size_t *cap, size_t want);
int grow_pinned(uint8_t **buf, size_t *cap, size_t want);
// The context's coherent, device-mapped host buffer (zc / zc_dev) with at
// least buf_bytes.
int zero_copy_buffer(ThreadCtx *ctx, size_t buf_bytes);
// Largest staging buffer of a single zero-copy pass.
size_t zero_copy_limit();
// Bytes above which a zero-copy pass copies with the copy pool (below, on the
// calling thread: the pool's hand-off costs more than a small memcpy).
size_t zc_pool_min();

// ---- small calls' completion signal ---------------------------------------
constexpr size_t kSignalCtr = 16;  // int index into ThreadCtx::flag of the block counter
// The context's signal words (allocated on first use) and the next call's
// sequence number (never 0).
int next_signal(ThreadCtx *ctx, uint32_t **flag_dev, uint32_t **ctr, uint32_t *seq);
// Spins until the launch signalled `seq` (or a later launch on the stream its
// own, higher number); *mismatch (may be NULL) gets the
// verify word.  A stream that went idle without the signal, or failed, is an
// error (nothing then spins forever).
int wait_signal(ThreadCtx *ctx, uint32_t seq, uint32_t *mismatch);

// ---- the chunked pipeline --------------------------------------------------
// Bytes per slot per chunk for a call of `total` bytes per slot and `nslots`
// slots per buffer.
size_t chunk_bytes(size_t total, int nslots, bool pinned);
// True when every non-null pointer is page-locked host memory known to HIP
// (the caller's own pinning: the library never page-locks caller memory).
bool all_pinned(const uint8_t *const *ptrs, int n);
inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// One host <-> device transfer of a chunk: host bytes [host, host + n) and
// bytes [off, off + n) of the chunk's staging buffer.
struct Xfer {
    uint8_t *host;
    size_t off;
    size_t n;
};
using ChunkIo = std::function<void(size_t j, std::vector<Xfer> *in, std::vector<Xfer> *out)>;
using ChunkCode = std::function<int(size_t j, uint8_t *buf, hipStream_t s)>;

// Runs n_chunks chunks of buf_bytes each: io(j) names chunk j's inputs and
// outputs, code(j) enqueues its kernels on the given stream.  Returns once
// every output has reached host memory -- also on an error, so no copy into
// or out of caller memory is still in flight when the caller gets control.
int run_chunks(ThreadCtx *ctx, size_t n_chunks, size_t buf_bytes, bool pinned, const ChunkIo &io,
               const ChunkCode &code);

// ---- the mirrored pipeline (pageable callers) ----------------------------------
// Pageable caller memory (JVM heap arrays through JNI) cannot be read by the
// GPU, and the library does not page-lock it.  Its bytes are
// copied by the copy pool into device-mapped pinned slots that the direct
// kernels code in place across the link, and the outputs copied back out,
// chunk by chunk: chunk j's inputs are copied while the GPU codes chunk j-1 and
// chunk j-2's outputs are drained, so the CPU copies hide behind the link.
//
// Per-slot chunk bytes for a call of `total` bytes per slot over `nslots`
// slots (multiples of `granule`, at least one granule).
size_t mirror_chunk_bytes(size_t total, int nslots, size_t granule);
// Chunk boundaries over [0, total) in units of `granule`: chunks of `chunk`
// bytes, the first and last two shorter (a quarter, a half), so the pipeline
// fills and drains quickly.  bounds.front() == 0, bounds.back() == total.
std::vector<size_t> ramp_bounds(size_t total, size_t chunk, size_t granule);
// Runs bounds.size() - 1 chunks through the slots: io(j) names chunk j's host
// inputs and outputs (offsets into a slot of buf_bytes), code(j, dev, s)
// enqueues its kernels on s over the slot's device address.  Returns once
// every output is in caller memory; on an error, once nothing of the call is
// in flight.
// side(j, slot, before, after), when given, adds host copies of chunk j that
// are not slot transfers (a file split into its data shards, shards merged into
// a file): `before` run in the batch with chunk j's inputs, `after` in the
// batch that drains its outputs; slot is chunk j's slot (host address).
using ChunkSide = std::function<void(size_t j, uint8_t *slot, std::vector<rsamd::CopyJob> *before,
                                     std::vector<rsamd::CopyJob> *after)>;
int run_mirrored(ThreadCtx *ctx, size_t n_chunks, size_t buf_bytes, const ChunkIo &io, const ChunkCode &code,
                 const ChunkSide &side = nullptr);

}  // namespace host
}  // namespace rsamd
