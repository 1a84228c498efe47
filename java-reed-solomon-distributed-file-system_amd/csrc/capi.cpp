// capi.cpp -- the extern "C" boundary (include/rs_amd.h).
//
// Host-buffer entry points mirror ReedSolomon.java / CodingLoop.java one for
// one (argument meaning, check order, exception text); they stage the byte
// range to the GPU through host.hpp's pipeline, run the kernels of
// kernels.hip / layout.hip and copy results back.
// Device entry points enqueue the same kernels on a caller's stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rs_amd.h"
#include "bounds.hpp"
#include "codec.hpp"
#include "copy_pool.hpp"
#include "gf256.hpp"
#include "host.hpp"
#include "kernels.hpp"
#include "layout.hpp"
#include "tuning.hpp"

struct rs_codec {
    rsamd::Codec *impl;
};

namespace {

using rsamd::Codec;
using rsamd::DevPlan;
using rsamd::Geometry;
using rsamd::Mode;
using rsamd::Plan;
using namespace rsamd::host;
namespace bounds = rsamd::bounds;

// Bounds-checking build (bounds.hpp): the bytes a stripe batch's arguments
// describe -- stripe t's shard s at base + t * stripe_stride + s * shard_stride,
// len bytes each.  A no-op in the product build.
void allow_batch(const uint8_t *base, size_t n_stripes, size_t len, size_t shard_stride, size_t stripe_stride,
                 int total) {
    if (!base || n_stripes == 0 || len == 0 || total < 1) return;
    bounds::allow(base, (n_stripes - 1) * stripe_stride + size_t(total - 1) * shard_stride + len);
}

// Direct path: the caller's page-locked shards coded in place across the link,
// one launch_gf_direct per launch group on the context's stream (kernels.hip
// gf_direct_kernel: 0.96 of the link bound against 0.86 for the staged
// pipeline, profiles/r3/zc_probe_r3s2b.txt).  *taken = false, and nothing
// enqueued, when a shard has no device address, the plan is wider than
// kMaxDirectIn inputs, or the shards' addresses share no 8-byte residue: the
// caller then stages the call.  In a TUNING build RSAMD_DIRECT=0 turns it off.
bool direct_enabled() {
    static const bool on = [] {
        const char *e = rsamd::tuning_env("RSAMD_DIRECT");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Device address of page-locked host memory (nullptr if it has none).
uint8_t *host_dev_addr(const void *p) {
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, const_cast<void *>(p), 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<uint8_t *>(d);
}

// Bytes per shard from which a caller-pinned call is coded in place by the
// direct kernel instead of being copied through the zero-copy staging buffer
// (TUNING builds: RSAMD_DIRECT_MIN, read per call).  4+2 encodeParity per
// call on pinned shards, staged -> direct (tools/direct_small_probe.py,
// profiles/r3/direct_small_r3s2k.txt): 4 KiB 26.3 -> 29.7 us, 64 KiB
// 38.8 -> 31.8 us, 256 KiB 96.3 -> 50.5 us.
size_t direct_min_bytes() { return rsamd::tuning_size("RSAMD_DIRECT_MIN", size_t(64) << 10); }

// Bytes per shard from which a pageable call takes the mirrored pipeline
// instead of the single zero-copy staging pass (TUNING builds:
// RSAMD_MIRROR_MIN, read per call).  Below 1 MiB the pipeline's per-chunk
// latency outweighs its overlap: 4+2 encodeParity per call, zero-copy /
// mirrored, 256 KiB shards 84 / 181-251 us, 512 KiB 145-169 / 208-287 us;
// even at 1 MiB (profiles/r5/host_sizes_r5u.txt, host_sizes_r5v.txt).
size_t mirror_min_bytes() { return rsamd::tuning_size("RSAMD_MIRROR_MIN", size_t(1) << 20); }

// The direct kernels' plans for columns [offset, offset+count) of the slots:
// false (nothing enqueued) when a shard has no device address, a plan is
// wider than kMaxDirectIn inputs, or the addresses share no 8-byte residue.
// addr(slot) gives a slot's device address (nullptr: none).
bool direct_plans(const std::vector<DevPlan> &plans, const std::vector<int> &in_slots,
                  const std::vector<int> &out_slots, const std::function<uint8_t *(int)> &addr,
                  std::vector<rsamd::DirectPlan> *out) {
    if (!direct_enabled() || plans.empty()) return false;
    std::vector<rsamd::DirectPlan> dp(plans.size());
    auto dev_addr = [&](int slot, uint8_t **a) {
        *a = addr(slot);
        return *a != nullptr;
    };
    for (size_t g = 0; g < plans.size(); ++g) {
        const DevPlan &p = plans[g];
        if (p.nin > rsamd::kMaxDirectIn || p.nin > int(in_slots.size())) return false;
        dp[g].nin = p.nin;
        dp[g].nout = p.nout;
        dp[g].tabs = p.tabs;
        for (int i = 0; i < p.nin; ++i) {
            uint8_t *a = nullptr;
            if (!dev_addr(in_slots[i], &a)) return false;
            dp[g].in[i] = a;
        }
        for (int q = 0; q < p.nout; ++q) {
            const size_t o = g * size_t(rsamd::kMaxOut) + size_t(q);
            if (o >= out_slots.size() || !dev_addr(out_slots[o], &dp[g].out[q])) return false;
        }
    }
    // Every address must share one residue modulo 8 (launch_gf_direct's
    // narrowest vector).
    const uintptr_t r8 = reinterpret_cast<uintptr_t>(dp[0].in[0]) % 8;
    for (const rsamd::DirectPlan &d : dp) {
        for (int i = 0; i < d.nin; ++i)
            if (reinterpret_cast<uintptr_t>(d.in[i]) % 8 != r8) return false;
        for (int q = 0; q < d.nout; ++q)
            if (reinterpret_cast<uintptr_t>(d.out[q]) % 8 != r8) return false;
    }
    *out = std::move(dp);
    return true;
}

int launch_direct(ThreadCtx *ctx, const std::vector<rsamd::DirectPlan> &dp, size_t count, Mode mode) {
    for (const rsamd::DirectPlan &d : dp) {
        for (int i = 0; i < d.nin; ++i) bounds::allow(d.in[i], count);
        for (int q = 0; q < d.nout; ++q) bounds::allow(d.out[q], count);
    }
    for (size_t g = 0; g < dp.size(); ++g) {
        const hipError_t e = rsamd::launch_gf_direct(dp[g], count, mode, ctx->flag, ctx->stream);
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(ctx->stream);
            return hip_fail(e, "launch_gf_direct");
        }
    }
    RS_HIP(hipStreamSynchronize(ctx->stream));
    return RS_OK;
}

// Caller-pinned arrays: [offset, offset+count) coded in place by the direct
// kernels.  *taken = false (nothing enqueued) when direct_plans refuses.
int run_direct(ThreadCtx *ctx, const std::vector<DevPlan> &plans, const std::vector<int> &in_slots,
               const std::vector<int> &out_slots, uint8_t *const *host, size_t offset, size_t count, Mode mode,
               bool *taken) {
    *taken = false;
    std::vector<rsamd::DirectPlan> dp;
    if (!direct_plans(plans, in_slots, out_slots, [&](int sl) { return host_dev_addr(host[sl] + offset); }, &dp))
        return RS_OK;
    *taken = true;
    return launch_direct(ctx, dp, count, mode);
}

// Pageable caller arrays (JNI heap arrays): copied chunk by chunk into the
// context's device-mapped pinned slots and coded there in place by the direct
// kernels, the copies overlapped with the link (host.hpp run_mirrored).  The
// library never page-locks caller memory.  *taken = false
// (nothing done) when a plan is wider than the direct kernels take.
constexpr size_t kMirrorAlign = 4096;  // slots on page boundaries: the kernels' waves move whole lines

int run_mirror_host(ThreadCtx *ctx, const std::vector<DevPlan> &plans, int nslots, const std::vector<int> &in_slots,
                    const std::vector<int> &out_slots, uint8_t *const *host, size_t offset, size_t count, Mode mode,
                    bool *taken) {
    *taken = false;
    if (!direct_enabled() || plans.empty()) return RS_OK;
    for (const DevPlan &p : plans)
        if (p.nin > rsamd::kMaxDirectIn) return RS_OK;
    const size_t chunk = mirror_chunk_bytes(count, nslots, kMirrorAlign);
    const std::vector<size_t> cb = ramp_bounds(count, chunk, kMirrorAlign);
    size_t widest = 0;
    for (size_t j = 0; j + 1 < cb.size(); ++j) widest = std::max(widest, cb[j + 1] - cb[j]);
    const size_t slot_stride = round_up(widest, kMirrorAlign);
    auto io = [&](size_t j, std::vector<Xfer> *in, std::vector<Xfer> *out) {
        const size_t lo = cb[j], n = cb[j + 1] - lo;
        for (int s : in_slots) in->push_back({host[s] + offset + lo, size_t(s) * slot_stride, n});
        if (mode == Mode::Code)
            for (int s : out_slots) out->push_back({host[s] + offset + lo, size_t(s) * slot_stride, n});
    };
    auto code = [&](size_t j, uint8_t *dev, hipStream_t st) -> int {
        std::vector<rsamd::DirectPlan> dp;
        if (!direct_plans(plans, in_slots, out_slots, [&](int sl) { return dev + size_t(sl) * slot_stride; }, &dp))
            return fail(RS_E_HIP, "direct plans over the mirror slots");
        for (const rsamd::DirectPlan &d : dp) RS_HIP(rsamd::launch_gf_direct(d, cb[j + 1] - cb[j], mode, ctx->flag, st));
        return RS_OK;
    };
    *taken = true;
    return run_mirrored(ctx, cb.size() - 1, slot_stride * size_t(nslots), io, code);
}

// Small calls (one zero-copy pass, one launch group): the inputs are copied
// into the context's coherent, device-mapped buffer, ONE direct-kernel launch
// codes it in place over the link -- 16-byte vectors, its head and tail bytes
// in the same launch -- and signals its completion into host memory, where
// this thread spins (kernels.hpp DirectSignal); then the outputs are copied
// back.  Against the staged pass it replaces (the stripe kernels over the
// buffer, then a stream synchronisation), measured from C on one MI355X
// (tools/small_latency.hip, profiles/r6/small_latency_*.json): 4+2 x 1000 B
// decodeMissing 18.6 -> see DESIGN.md 5.2 -- at 1000 B the stripe kernels had
// no whole 1 KiB wave span and coded every byte in the byte kernel (8.7 us of
// GPU time), and a stream synchronisation observes a finished kernel ~3 us
// later than the spin does.  *taken = false (nothing done) for plans of more
// than one launch group or wider than the direct kernels take.
bool small_signal_enabled() { return rsamd::tuning_size("RSAMD_SMALL_SIGNAL", 1) != 0; }  // TUNING builds: A/B
// Launches of a split small call (run_small), the bytes per shard from which
// calls split, and the alignment of the cuts (TUNING builds: A/B knobs).
size_t small_parts() {
    static const size_t v = std::min<size_t>(8, std::max<size_t>(1, rsamd::tuning_size("RSAMD_SMALL_PARTS", 2)));
    return v;
}
size_t small_parts_min() {
    static const size_t v = rsamd::tuning_size("RSAMD_SMALL_PARTS_MIN", size_t(128) << 10);
    return v;
}
// Staging bytes above which the small file passes (file_encode_zc_split,
// file_decode_zc_split) copy with the copy pool: 8 MiB, against 2 MiB for the
// shard calls (zc_pool_min).  4+2, 3 MiB file, calling thread / pool,
// alternated: encode 170-174 / 176-187 us, decode {0,5} 151-169 / 170-186;
// 10+4 3 MiB file 154-156 / 184-200.  The shard calls keep 2 MiB: at 10+4
// the calling thread lost from 192 KiB per shard (profiles/r6/zcpool_*_r6bk.txt, zcpool2_42_r6bk.txt).
// TUNING builds: RSAMD_FILE_ZC_POOL_MIN.
size_t file_zc_pool_min() {
    static const size_t v = rsamd::tuning_size("RSAMD_FILE_ZC_POOL_MIN", size_t(8) << 20);
    return v;
}
size_t small_parts_align() {
    static const size_t v = std::max<size_t>(256, rsamd::tuning_size("RSAMD_SMALL_PARTS_ALIGN", 4096));
    return v;
}

int run_small(ThreadCtx *ctx, const std::vector<DevPlan> &plans, int nslots, const std::vector<int> &in_slots,
              const std::vector<int> &out_slots, uint8_t *const *host, size_t offset, size_t count, Mode mode,
              int *result, bool *taken) {
    *taken = false;
    if (plans.size() != 1 || count == 0 || !small_signal_enabled()) return RS_OK;
    // The kernel codes whole 16-byte vectors: each slot's bytes past `count`
    // up to the next 16 are zeroed (0 codes to 0, so a verify compares them
    // equal) and coded too, no byte tail in the launch (at 1000-byte shards
    // the tail's per-input byte loads cost several link round trips).
    const size_t n16 = round_up(count, 16);
    // From 128 KiB per shard a coding call runs as two launches over two
    // column ranges, each signalling: the second range's copy-in overlaps the
    // first range's kernel, the first range's copy-out the second's.  4+2
    // encodeParity per call, from C (profiles/r6/small_parts_ab_r6ay.txt):
    // 256 KiB 77 -> 64 us, 512 KiB 130-137 -> 113-117, 768 KiB 171-198 -> 141-148.
    // The cut is on a page boundary: cuts inside a page (the CPU copying into
    // the page whose other half the GPU is reading) made each later launch
    // 25-50 us slower.  Three or four ranges are no better than two.  A
    // verify splits too, only its last launch signalling: the launches before
    // leave their mismatches in the device word, which the last one's signal
    // reports and zeroes.  TUNING builds: RSAMD_SMALL_PARTS,
    // RSAMD_SMALL_PARTS_MIN, RSAMD_SMALL_PARTS_ALIGN, RSAMD_SMALL_PARTS_VERIFY.
    static const bool split_verify = rsamd::tuning_size("RSAMD_SMALL_PARTS_VERIFY", 1) != 0;
    const size_t parts =
        (mode == Mode::Code || split_verify) && count >= small_parts_min() ? small_parts() : 1;
    const size_t cut_align = small_parts_align();
    std::vector<size_t> cut(parts + 1, n16);
    cut[0] = 0;
    for (size_t j = 1; j < parts; ++j) cut[j] = std::min(n16, round_up(n16 * j / parts, cut_align));
    // (split: the slots on page boundaries too, so no page holds bytes of two ranges)
    const size_t ss = round_up(count, parts > 1 ? cut_align : 256), bytes = ss * size_t(nslots);
    if (bytes > zero_copy_limit()) return RS_OK;
    int rc = zero_copy_buffer(ctx, bytes);
    if (rc) return rc;
    std::vector<rsamd::DirectPlan> dp;
    if (!direct_plans(plans, in_slots, out_slots, [&](int sl) { return ctx->zc_dev + size_t(sl) * ss; }, &dp))
        return RS_OK;
    std::vector<rsamd::DirectSignal> sg(parts);
    for (rsamd::DirectSignal &g : sg) {
        rc = next_signal(ctx, &g.flag, &g.ctr, &g.seq);
        if (rc) return rc;
    }
    size_t last = 0;  // the last non-empty range
    for (size_t j = 0; j < parts; ++j)
        if (cut[j] < cut[j + 1]) last = j;
    *taken = true;
    // host copies on this thread; the copy pool only above 2 MiB (as run_zero_copy)
    const bool use_pool = bytes > zc_pool_min();
    std::vector<rsamd::CopyJob> jobs;
    auto copy = [&]() {
        if (use_pool)
            rsamd::CopyPool::get().copy(jobs);
        else
            rsamd::CopyPool::copy_here(jobs);
        jobs.clear();
    };
    const rsamd::DirectPlan &d = dp[0];
    for (int i = 0; i < d.nin; ++i) bounds::allow(d.in[i], n16);
    for (int q = 0; q < d.nout; ++q) bounds::allow(d.out[q], n16);
    for (size_t j = 0; j < parts; ++j) {
        const size_t lo = cut[j], hi = cut[j + 1];
        if (lo == hi) continue;
        const size_t end = std::min(hi, count);
        for (int s : in_slots) {
            if (end > lo) jobs.push_back({ctx->zc + size_t(s) * ss + lo, host[s] + offset + lo, end - lo});
            if (hi > count) std::memset(ctx->zc + size_t(s) * ss + count, 0, hi - count);
        }
        copy();
        rsamd::DirectPlan dj = d;
        for (int i = 0; i < dj.nin; ++i) dj.in[i] += lo;
        for (int q = 0; q < dj.nout; ++q) dj.out[q] += lo;
        const rsamd::DirectSignal *sj = mode == Mode::Verify && j != last ? nullptr : &sg[j];
        const hipError_t e = rsamd::launch_gf_direct(dj, hi - lo, mode, ctx->flag, ctx->stream, nullptr, sj);
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(ctx->stream);
            return hip_fail(e, "launch_gf_direct (small call)");
        }
    }
    for (size_t j = 0; j < parts; ++j) {
        const size_t lo = cut[j], end = std::min(cut[j + 1], count);
        if (cut[j] == cut[j + 1] || (mode == Mode::Verify && j != last)) continue;
        uint32_t mm = 0;
        rc = wait_signal(ctx, sg[j].seq, &mm);
        if (rc) {
            (void)hipStreamSynchronize(ctx->stream);
            return rc;
        }
        if (mode == Mode::Verify) {
            *result = mm ? 0 : 1;
            return RS_OK;
        }
        if (end > lo)
            for (int s : out_slots) jobs.push_back({host[s] + offset + lo, ctx->zc + size_t(s) * ss + lo, end - lo});
        copy();
    }
    return RS_OK;
}

// Stage [offset, offset+count) of the host shards (slot-indexed), run every
// launch group of `plans`, copy results back.
//   in_slots:  slots copied host -> device (coding inputs, plus the checked
//              shards in Verify mode)
//   out_slots: slots copied device -> host afterwards (Code mode)
int run_host(const std::vector<DevPlan> &plans, int nslots, const std::vector<int> &in_slots,
             const std::vector<int> &out_slots, uint8_t *const *host, size_t offset, size_t count, Mode mode,
             int *result) {
    ThreadCtx *ctx = nullptr;
    int rc = thread_ctx(&ctx);
    if (rc) return rc;
    // Small calls stay on the zero-copy staging path (direct_min_bytes): skip the
    // per-buffer pointer queries.  Larger calls: caller-pinned arrays are coded
    // in place by the direct kernels, pageable ones through the mirrored
    // pipeline (or, for plans the direct kernels cannot take, the DMA pipeline).
    const size_t dmin = direct_min_bytes();
    const bool pinned = count >= std::min(dmin, size_t(1) << 20) && all_pinned(host, nslots);
    // The verify word (ctx->flag): a small call's signal leaves it zero
    // (kernels.hpp DirectSignal); every other verify may leave it set, so the
    // next verify zeroes it first (a memset is a dispatch of its own: ~4 us of
    // a small call).
    if (!pinned && count < mirror_min_bytes()) {
        if (mode == Mode::Verify && ctx->flag_dirty) {
            RS_HIP(hipMemsetAsync(ctx->flag, 0, sizeof(int), ctx->stream));
            ctx->flag_dirty = false;
        }
        bool taken = false;
        rc = run_small(ctx, plans, nslots, in_slots, out_slots, host, offset, count, mode, result, &taken);
        if (rc) ctx->flag_dirty = true;
        if (rc || taken) return rc;
    }
    if (mode == Mode::Verify) {
        if (ctx->flag_dirty) RS_HIP(hipMemsetAsync(ctx->flag, 0, sizeof(int), ctx->stream));
        ctx->flag_dirty = true;
    }
    if (pinned || count >= mirror_min_bytes()) {
        bool taken = false;
        rc = pinned ? run_direct(ctx, plans, in_slots, out_slots, host, offset, count, mode, &taken)
                    : run_mirror_host(ctx, plans, nslots, in_slots, out_slots, host, offset, count, mode, &taken);
        if (rc) return rc;
        if (taken) {
            if (mode == Mode::Verify) {
                int h = 0;
                RS_HIP(hipMemcpy(&h, ctx->flag, sizeof(int), hipMemcpyDeviceToHost));
                *result = h ? 0 : 1;
            }
            return RS_OK;
        }
    }
    const size_t chunk = std::min(count, chunk_bytes(count, nslots, pinned));
    const size_t slot_stride = round_up(std::max<size_t>(chunk, 1), 256);
    auto io = [&](size_t j, std::vector<Xfer> *in, std::vector<Xfer> *out) {
        const size_t done = j * chunk, n = std::min(chunk, count - done);
        for (int s : in_slots) in->push_back({host[s] + offset + done, size_t(s) * slot_stride, n});
        if (mode == Mode::Code)
            for (int s : out_slots) out->push_back({host[s] + offset + done, size_t(s) * slot_stride, n});
    };
    auto code = [&](size_t j, uint8_t *buf, hipStream_t st) -> int {
        Geometry g;
        g.base = buf;
        g.n_stripes = 1;
        g.col0 = 0;
        g.len = std::min(chunk, count - j * chunk);
        g.shard_stride = slot_stride;
        g.stripe_stride = slot_stride * size_t(nslots);
        for (const DevPlan &p : plans) RS_HIP(rsamd::launch_gf(g, p, mode, ctx->flag, st));
        return RS_OK;
    };
    rc = run_chunks(ctx, (count + chunk - 1) / chunk, slot_stride * size_t(nslots), pinned, io, code);
    if (rc) return rc;
    if (mode == Mode::Verify) {
        int h = 0;
        RS_HIP(hipMemcpy(&h, ctx->flag, sizeof(int), hipMemcpyDeviceToHost));
        *result = h ? 0 : 1;
    }
    return RS_OK;
}

// ReedSolomon.checkBuffersAndSizes (ReedSolomon.java:277-302), same order and text.
// shards == NULL with check_ptrs false: the sizes only (rs_check_buffers_and_sizes).
int check_buffers_and_sizes(const Codec &c, uint8_t *const *shards, int nshards, const int64_t *lens,
                            int64_t offset, int64_t count, bool check_ptrs = true) {
    if (nshards != c.total()) return fail(RS_E_WRONG_NSHARDS, "wrong number of shards: " + std::to_string(nshards));
    if ((check_ptrs && !shards) || !lens) return fail(RS_E_INVALID, "shards and shard_lens must not be NULL");
    for (int i = 1; i < nshards; ++i)
        if (lens[i] != lens[0]) return fail(RS_E_SIZE_MISMATCH, "Shards are different sizes");
    if (offset < 0) return fail(RS_E_NEG_OFFSET, "offset is negative: " + std::to_string(offset));
    if (count < 0) return fail(RS_E_NEG_COUNT, "byteCount is negative: " + std::to_string(count));
    if (lens[0] < offset + count)  // Java concatenates the two ints (ReedSolomon.java:300)
        return fail(RS_E_TOO_SMALL, "buffers to small: " + std::to_string(count) + std::to_string(offset));
    for (int i = 0; check_ptrs && i < nshards; ++i)
        if (!shards[i] && lens[i] > 0) return fail(RS_E_INVALID, "shard " + std::to_string(i) + " is NULL");
    return RS_OK;
}

int code_with_plan(const Plan &plan, int nslots, uint8_t *const *host, size_t offset, size_t count, Mode mode,
                   int *result) {
    int rc = need_device();
    if (rc) return rc;
    std::vector<DevPlan> plans;
    RS_HIP(plan.device_plans(&plans));
    std::vector<int> in = plan.in_idx();
    if (mode == Mode::Verify) in.insert(in.end(), plan.out_idx().begin(), plan.out_idx().end());
    return run_host(plans, nslots, in, plan.out_idx(), host, offset, count, mode, result);
}

// Plan for explicit rows (CodingLoop API): slots 0..nin-1 inputs, nin.. outputs.
// Uploaded per call to the thread context (rows change per call).
int code_rows(const uint8_t *const *rows, const uint8_t *const *inputs, int nin, uint8_t *const *outputs, int nout,
              int32_t offset, int32_t count, Mode mode, int *result) {
    if (nout <= 0 || count <= 0) {  // the Java loops do nothing
        if (result) *result = 1;
        return RS_OK;
    }
    if (!rows || !inputs || !outputs || nin < 1)
        return fail(RS_E_INVALID, "matrix_rows, inputs and outputs must not be NULL; input_count >= 1");
    if (offset < 0) return fail(RS_E_INVALID, "offset is negative: " + std::to_string(offset));
    for (int p = 0; p < nout; ++p)
        if (!rows[p] || !outputs[p]) return fail(RS_E_INVALID, "NULL matrix row or output");
    for (int i = 0; i < nin; ++i)
        if (!inputs[i]) return fail(RS_E_INVALID, "NULL input");
    int rc = need_device();
    if (rc) return rc;
    rsamd::GfMatrix m(nout, nin);
    for (int p = 0; p < nout; ++p)
        for (int i = 0; i < nin; ++i) m.at(p, i) = rows[p][i];
    std::vector<int> in_idx(nin), out_idx(nout);
    for (int i = 0; i < nin; ++i) in_idx[i] = i;
    for (int p = 0; p < nout; ++p) out_idx[p] = nin + p;
    Plan plan(in_idx, out_idx, m);

    ThreadCtx *ctx = nullptr;
    rc = thread_ctx(&ctx);
    if (rc) return rc;
    std::vector<std::vector<uint8_t>> images;
    size_t total = 0;
    for (int g = 0; g < plan.groups(); ++g) {
        images.push_back(plan.image(g));
        total += images.back().size();
    }
    rc = grow(&ctx->plan, &ctx->plan_cap, total);
    if (rc) return rc;
    std::vector<DevPlan> plans;
    size_t off = 0;
    for (int g = 0; g < plan.groups(); ++g) {
        RS_HIP(hipMemcpyAsync(ctx->plan + off, images[g].data(), images[g].size(), hipMemcpyHostToDevice,
                              ctx->stream));
        plans.push_back(rsamd::dev_plan_at(ctx->plan + off, nin, std::min(rsamd::kMaxOut, nout - g * rsamd::kMaxOut)));
        off += images[g].size();
    }
    std::vector<uint8_t *> slots(size_t(nin) + nout);
    for (int i = 0; i < nin; ++i) slots[i] = const_cast<uint8_t *>(inputs[i]);
    for (int p = 0; p < nout; ++p) slots[nin + p] = outputs[p];
    std::vector<int> in_slots = in_idx;
    if (mode == Mode::Verify) in_slots.insert(in_slots.end(), out_idx.begin(), out_idx.end());
    return run_host(plans, nin + nout, in_slots, out_idx, slots.data(), size_t(offset), size_t(count), mode, result);
}


// ---------------------------------------------------------------------------
// Client file layout (ReedSolomonEncoder / ReedSolomonDecoder).
// ---------------------------------------------------------------------------
int file_layout(const Codec &c, int64_t file_len, int64_t block, int64_t *padded, int64_t *S) {
    if (file_len < 0) return fail(RS_E_INVALID, "file length is negative: " + std::to_string(file_len));
    if (block < 1) return fail(RS_E_INVALID, "block size must be positive");
    const int64_t mult = int64_t(c.k()) * block;  // ConfigVariables.FILE_SIZE_MULTIPLE
    *padded = file_len % mult == 0 ? file_len : file_len / mult * mult + mult;  // ReedSolomonEncoder.java:76-85
    *S = *padded / c.k();
    return RS_OK;
}

int file_encode_dev(const Codec &c, const uint8_t *file, size_t file_len, size_t block, uint8_t *shards,
                    size_t stride, hipStream_t s) {
    int64_t padded = 0, S = 0;
    int rc = file_layout(c, int64_t(file_len), int64_t(block), &padded, &S);
    if (rc) return rc;
    if (S == 0) return RS_OK;
    if (!shards || (!file && file_len)) return fail(RS_E_INVALID, "NULL device buffer");
    if (stride < size_t(S)) return fail(RS_E_INVALID, "shard_stride is smaller than the shard length");
    rsamd::FileGeom g;
    g.file = file;
    g.file_len = file_len;
    g.block = block;
    g.k = c.k();
    g.S = size_t(S);
    g.shards = shards;
    g.shard_stride = stride;
    bounds::allow(file, file_len);
    allow_batch(shards, 1, size_t(S), stride, 0, c.total());
    std::vector<DevPlan> plans;
    RS_HIP(c.encode_plan().device_plans(&plans));
    Geometry sg{shards, 1, 0, size_t(S), stride, stride * size_t(c.total())};
    size_t first = 0;
    if (rsamd::file_fusable(g, true)) {
        RS_HIP(rsamd::launch_file_encode_fused(g, plans.empty() ? nullptr : &plans[0], s));
        first = plans.empty() ? 0 : 1;
    } else {
        RS_HIP(rsamd::launch_split(g, s));
    }
    for (size_t i = first; i < plans.size(); ++i) RS_HIP(rsamd::launch_gf(sg, plans[i], Mode::Code, nullptr, s));
    return RS_OK;
}

int file_decode_dev(const Codec &c, uint8_t *shards, size_t S, size_t stride, const uint8_t *present, size_t block,
                    uint8_t *file_out, size_t file_size, bool write_missing, hipStream_t s) {
    if (!present) return fail(RS_E_INVALID, "present must not be NULL");
    if (block < 1) return fail(RS_E_INVALID, "block size must be positive");
    if (S % block) return fail(RS_E_INVALID, "shard length " + std::to_string(S) + " is not a multiple of the block size");
    if (file_size > S * size_t(c.k())) return fail(RS_E_INVALID, "file size exceeds k * shard length");
    if (stride < S) return fail(RS_E_INVALID, "shard_stride is smaller than the shard length");
    int n_present = 0;
    for (int i = 0; i < c.total(); ++i) n_present += present[i] ? 1 : 0;
    if (n_present < c.k()) return fail(RS_E_NOT_ENOUGH, "Not enough shards present");
    if (S == 0 || (file_size == 0 && !write_missing)) return RS_OK;
    if (!shards || (!file_out && file_size)) return fail(RS_E_INVALID, "NULL device buffer");
    rsamd::FileGeom g;
    g.file_out = file_out;
    g.file_len = file_size;
    g.block = block;
    g.k = c.k();
    g.S = S;
    g.shards = shards;
    g.shard_stride = stride;
    bounds::allow(file_out, file_size);
    allow_batch(shards, 1, S, stride, 0, c.total());
    std::shared_ptr<const Plan> plan;
    int n_missing_data = 0;
    for (int i = 0; i < c.k(); ++i) n_missing_data += present[i] ? 0 : 1;
    const bool fused = rsamd::file_fusable(g, false) && n_missing_data <= rsamd::kMaxOut;
    if (write_missing || !fused) {
        if (n_present < c.total()) {  // reconstruct every absent shard in place, then merge
            int rc = c.decode_plan(present, &plan);
            if (rc) return fail(rc, rc == RS_E_SINGULAR ? "Matrix is singular" : "Not enough shards present");
            std::vector<DevPlan> plans;
            RS_HIP(plan->device_plans(&plans));
            Geometry sg{shards, 1, 0, S, stride, stride * size_t(c.total())};
            for (const DevPlan &p : plans) RS_HIP(rsamd::launch_gf(sg, p, Mode::Code, nullptr, s));
        }
        if (file_size == 0) return RS_OK;
        if (!rsamd::file_fusable(g, false)) {
            RS_HIP(rsamd::launch_merge(g, s));
            return RS_OK;
        }
        std::vector<uint8_t> all(c.total(), 1);  // every shard now holds its bytes: pure merge
        int rc = c.decode_plan(all.data(), &plan, true);
        if (rc) return fail(rc, "decode plan");
    } else {
        int rc = c.decode_plan(present, &plan, true);
        if (rc) return fail(rc, rc == RS_E_SINGULAR ? "Matrix is singular" : "Not enough shards present");
    }
    rsamd::FileDecodePlan fp;
    RS_HIP(plan->device_file_plan(c.k(), &fp));
    RS_HIP(rsamd::launch_file_decode_fused(g, fp, s));
    return RS_OK;
}


// Host file paths (rs_file_encode / rs_file_decode): whole block rows per
// chunk through run_chunks, each staging buffer laid out as [file bytes of
// the rows][shard 0 .. total-1 columns of the rows].  (Whole-file pageable
// copies ran ~5x below PCIe rate.)
struct FileChunks {
    size_t R = 0, rows = 0, n = 0;   // block rows per chunk, rows in all, chunks
    size_t fbytes = 0, sstride = 0;  // staged file bytes and shard stride per buffer
    size_t buf_bytes = 0;
};

FileChunks file_chunks(int k, int total, size_t S, size_t block, bool pinned) {
    FileChunks f;
    f.rows = S / block;
    const size_t per_shard = chunk_bytes(S, k + total, pinned);
    f.R = std::min(f.rows, std::max<size_t>(1, per_shard / block));
    f.n = (f.rows + f.R - 1) / f.R;
    f.fbytes = round_up(f.R * size_t(k) * block, 256);
    f.sstride = round_up(f.R * block, 256);
    f.buf_bytes = f.fbytes + f.sstride * size_t(total);
    return f;
}

// ReedSolomonEncoder's split (ReedSolomonEncoder.java:56-60, the arraycopy
// per block) of block rows [r0, r1) as copy jobs: data shard i's block of row
// r is file bytes [(r k + i) blk, +blk), zeros past the file's end (the
// padding).  Row r goes to dst[i] + r * blk and, with dst2, to dst2[i] +
// (r - row2) * blk as well (one read, two writes).
// Rows per block of the split / merge jobs: each block's jobs, one per shard,
// are queued together, so the copy threads work on one ~1 MB stretch of the
// file at a time and read it from DRAM once, in order (4 shards x 1000-B
// blocks, split and tee: +10-25% over one job per shard on a CPU test box,
// tests/native; TUNING builds: RSAMD_COPY_ROW_BLOCK, 0 = one block).
size_t row_block() { return rsamd::tuning_size("RSAMD_COPY_ROW_BLOCK", 256); }

void split_jobs(const uint8_t *file, size_t file_len, size_t blk, int k, uint8_t *const *dst, uint8_t *const *dst2,
                size_t row2, size_t r0, size_t r1, std::vector<rsamd::CopyJob> *jobs) {
    const size_t kb = size_t(k) * blk;
    const size_t full = std::min(r1, std::max(r0, file_len / kb));  // rows wholly inside the file
    const size_t rb = row_block() ? row_block() : std::max<size_t>(1, r1 - r0);
    for (size_t b0 = r0; b0 < full; b0 += rb) {
        const size_t b1 = std::min(full, b0 + rb);
        for (int i = 0; i < k; ++i) {
            rsamd::CopyJob job{dst[i] + b0 * blk, file + (b0 * size_t(k) + size_t(i)) * blk, blk, b1 - b0, blk, kb};
            job.dst2 = dst2 ? dst2[i] + (b0 - row2) * blk : nullptr;
            job.dst2_stride = blk;
            jobs->push_back(job);
        }
    }
    for (size_t r = full; r < r1; ++r)  // the last row: the file's bytes, then the padding's zeros
        for (int i = 0; i < k; ++i) {
            const size_t f0 = (r * size_t(k) + size_t(i)) * blk;
            const size_t have = f0 < file_len ? std::min(blk, file_len - f0) : 0;
            for (uint8_t *d : {dst[i] + r * blk, dst2 ? dst2[i] + (r - row2) * blk : nullptr}) {
                if (!d) continue;
                if (have) jobs->push_back({d, file + f0, have});
                if (have < blk) jobs->push_back({d + have, nullptr, blk - have});
            }
        }
}

// ReedSolomonDecoder's merge and trim (ReedSolomonDecoder.java:62-66, 92-103)
// of block rows [r0, r1) as copy jobs: data shard d's block of row r is file
// bytes [(r k + d) blk, +blk), clipped to the file.  src[d] holds shard d's
// bytes from row r0 on; shards with only[d] == false are skipped.
void merge_jobs(int k, size_t blk, uint8_t *file_out, size_t file_size, const uint8_t *const *src,
                const std::vector<bool> &only, size_t r0, size_t r1, std::vector<rsamd::CopyJob> *jobs) {
    const size_t kb = size_t(k) * blk;
    const size_t rb = row_block() ? row_block() : std::max<size_t>(1, r1 - r0);
    for (size_t b0 = r0; b0 < r1; b0 += rb) {  // blocks of rows, every shard's jobs of a block together
        const size_t b1 = std::min(r1, b0 + rb);
        for (int d = 0; d < k; ++d) {
            if (!only[d]) continue;
            for (size_t r = b0; r < b1;) {
                const size_t f0 = (r * size_t(k) + size_t(d)) * blk;
                if (f0 >= file_size) break;
                if (f0 + blk <= file_size) {  // whole blocks up to the first that crosses the file's end
                    const size_t last = std::min(b1, (file_size - size_t(d) * blk - blk) / kb + 1);
                    jobs->push_back({file_out + f0, src[d] + (r - r0) * blk, blk, last - r, kb, blk});
                    r = last;
                } else {
                    jobs->push_back({file_out + f0, src[d] + (r - r0) * blk, file_size - f0});
                    ++r;
                }
            }
        }
    }
}

// Data shard d's rows [a0, a1) copied from src to dst (both at row a0) and
// merged into the file in the same pass: each row is read once and written
// twice (ReedSolomonDecoder.java:92-103's merge; the rows whose file block is
// cut by the file's end, or lies past it, get their file bytes clipped).
void tee_jobs(int k, size_t blk, uint8_t *file_out, size_t file_size, int d, const uint8_t *src, uint8_t *dst,
              size_t a0, size_t a1, std::vector<rsamd::CopyJob> *jobs) {
    const size_t kb = size_t(k) * blk, lead = size_t(d + 1) * blk;
    const size_t whole_rows = file_size >= lead ? (file_size - lead) / kb + 1 : 0;  // rows with a whole file block
    const size_t w1 = std::min(a1, std::max(a0, whole_rows));
    if (w1 > a0) {
        rsamd::CopyJob j{dst, src, blk, w1 - a0, blk, blk};
        j.dst2 = file_out + (a0 * size_t(k) + size_t(d)) * blk;
        j.dst2_stride = kb;
        jobs->push_back(j);
    }
    if (a1 > w1) {
        jobs->push_back({dst + (w1 - a0) * blk, src + (w1 - a0) * blk, (a1 - w1) * blk});
        const size_t f0 = (w1 * size_t(k) + size_t(d)) * blk;
        if (f0 < file_size) jobs->push_back({file_out + f0, src + (w1 - a0) * blk, std::min(blk, file_size - f0)});
    }
}

// Direct path of the host file calls on caller-pinned memory (layout.hpp
// FileDirect): the fused kernel reads the file in place across the link and
// writes the parity shards in place, while the copy pool splits the file into
// the data shards on the host (they are the file's own bytes: only coded bytes
// cross the link, 1.5 file sizes for 4+2 instead of 2.5).  *taken = false,
// nothing enqueued, when the code or a pointer does not fit the direct kernels
// (more than kMaxOut outputs, k above kMaxDirectIn, no device address, not
// 8-byte aligned): the call is staged.
int file_encode_direct(const Codec &c, const uint8_t *file, size_t file_len, size_t blk, uint8_t *const *shards,
                       size_t S, ThreadCtx *ctx, bool *taken) {
    *taken = false;
    if (!direct_enabled() || c.m() > rsamd::kMaxOut || c.k() > rsamd::kMaxDirectIn) return RS_OK;
    rsamd::FileDirect d;
    d.k = c.k();
    d.nout = c.m();
    d.block = blk;
    d.units = S / 8;
    d.file_len = file_len;
    d.file = host_dev_addr(file);
    if (!d.file) return RS_OK;
    for (int i = c.k(); i < c.total(); ++i)  // data shards (out[0 .. k)) stay null: split on the host
        if (!(d.out[i] = host_dev_addr(shards[i]))) return RS_OK;
    if (c.m() > 0) {
        std::vector<DevPlan> plans;
        RS_HIP(c.encode_plan().device_plans(&plans));
        d.tabs = plans[0].tabs;
    }
    if (!rsamd::file_direct_ok(d)) return RS_OK;
    bounds::allow(d.file, file_len);
    for (int i = c.k(); i < c.total(); ++i) bounds::allow(d.out[i], S);
    if (c.m() > 0) RS_HIP(rsamd::launch_file_encode_direct(d, ctx->stream));
    *taken = true;
    std::vector<rsamd::CopyJob> jobs;
    split_jobs(file, file_len, blk, c.k(), shards, nullptr, 0, 0, S / blk, &jobs);
    rsamd::CopyPool::get().copy(jobs);
    RS_HIP(hipStreamSynchronize(ctx->stream));
    return RS_OK;
}

// Small pageable files (one zero-copy pass): the file is copied into the
// context's device-mapped buffer, the fused direct kernel codes the parity
// there (reading the file over the link, writing only the parity back), and
// the host splits the data shards from the caller's file while it runs -- the
// link carries the file and the parity instead of the file and every shard
// (TUNING builds: RSAMD_FILE_ZC_SPLIT=0 keeps the all-GPU pass).  4+2 encode
// per call, all-GPU / split: 88 KB 39 / 36 us, 256 KiB 53 / 42-44, 1 MiB
// 126 / 85-86, 3 MiB 254 / 175 (profiles/r5/host_sizes_tile8_r5zz.txt).
// *taken = false when the kernel cannot take the geometry (block % 8, k, m,
// size).
// The same pass as two launches over two halves of the block rows (as
// run_small's split, from 128 KiB per shard): the second half of the file is
// copied in while the first half is coded, the first half's parity copied out
// while the second half is coded.  Each half's file bytes and parity sit on
// pages of their own in the staging buffer.  *taken = false when the kernel
// refuses the halves' geometry.
int file_encode_zc_halves(const Codec &c, const uint8_t *file, size_t file_len, size_t blk, uint8_t *const *shards,
                          size_t S, ThreadCtx *ctx, bool *taken) {
    *taken = false;
    const int k = c.k(), m = c.m();
    const size_t A = small_parts_align(), rows = S / blk, kb = size_t(k) * blk;
    const size_t r[3] = {0, rows / 2, rows};
    size_t at = 0, fo[2], flen[2], po[2][rsamd::kMaxOut];
    for (int h = 0; h < 2; ++h) {
        const size_t b0 = r[h] * kb;
        flen[h] = file_len > b0 ? std::min(file_len - b0, (r[h + 1] - r[h]) * kb) : 0;
        fo[h] = at;
        at += round_up(std::max<size_t>(flen[h], 1), A);
    }
    for (int h = 0; h < 2; ++h)
        for (int p = 0; p < m; ++p) {
            po[h][p] = at;
            at += round_up(std::max<size_t>((r[h + 1] - r[h]) * blk, 1), A);
        }
    if (at > (size_t(64) << 20)) return RS_OK;
    int rc = zero_copy_buffer(ctx, at);
    if (rc) return rc;
    std::vector<DevPlan> plans;
    RS_HIP(c.encode_plan().device_plans(&plans));
    rsamd::FileDirect d[2];
    for (int h = 0; h < 2; ++h) {
        d[h].k = k;
        d[h].nout = m;
        d[h].block = blk;
        d[h].units = (r[h + 1] - r[h]) * blk / 8;
        d[h].file_len = flen[h];
        d[h].file = ctx->zc_dev + fo[h];
        for (int p = 0; p < m; ++p) d[h].out[k + p] = ctx->zc_dev + po[h][p];
        d[h].tabs = plans[0].tabs;
        if (!rsamd::file_direct_ok(d[h]) || d[h].units == 0) return RS_OK;
    }
    for (int h = 0; h < 2; ++h) {
        rc = next_signal(ctx, &d[h].sig.flag, &d[h].sig.ctr, &d[h].sig.seq);
        if (rc) return rc;
    }
    *taken = true;
    const bool pool = at > file_zc_pool_min();
    auto copy = [&](std::vector<rsamd::CopyJob> &jobs) {
        if (pool)
            rsamd::CopyPool::get().copy(jobs);
        else
            rsamd::CopyPool::copy_here(jobs);
        jobs.clear();
    };
    std::vector<rsamd::CopyJob> jobs;
    for (int h = 0; h < 2; ++h) {
        if (flen[h]) jobs.push_back({ctx->zc + fo[h], file + r[h] * kb, flen[h]});
        copy(jobs);
        bounds::allow(d[h].file, std::max<size_t>(flen[h], 1));
        for (int p = 0; p < m; ++p) bounds::allow(d[h].out[k + p], d[h].units * 8);
        const hipError_t e = rsamd::launch_file_encode_direct(d[h], ctx->stream);
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(ctx->stream);
            return hip_fail(e, "launch_file_encode_direct (small file, halves)");
        }
    }
    split_jobs(file, file_len, blk, k, shards, nullptr, 0, 0, rows, &jobs);
    copy(jobs);
    for (int h = 0; h < 2; ++h) {
        rc = wait_signal(ctx, d[h].sig.seq, nullptr);
        if (rc) {
            (void)hipStreamSynchronize(ctx->stream);
            return rc;
        }
        for (int p = 0; p < m; ++p)
            jobs.push_back({shards[k + p] + r[h] * blk, ctx->zc + po[h][p], (r[h + 1] - r[h]) * blk});
        copy(jobs);
    }
    return RS_OK;
}

int file_encode_zc_split(const Codec &c, const uint8_t *file, size_t file_len, size_t blk, uint8_t *const *shards,
                         size_t S, ThreadCtx *ctx, bool *taken) {
    *taken = false;
    const int k = c.k(), m = c.m();
    if (!rsamd::tuning_size("RSAMD_FILE_ZC_SPLIT", 1) || !direct_enabled() || m < 1 || m > rsamd::kMaxOut ||
        k > rsamd::kMaxDirectIn || blk % 8 || S % 8)
        return RS_OK;
    if (small_signal_enabled() && small_parts() > 1 && S >= small_parts_min() && S % blk == 0 && S / blk >= 2) {
        int rc = file_encode_zc_halves(c, file, file_len, blk, shards, S, ctx, taken);
        if (rc || *taken) return rc;
    }
    const size_t fbytes = round_up(std::max<size_t>(file_len, 1), 256), stride = round_up(S, 256);
    const size_t need = fbytes + size_t(m) * stride;
    if (need > (size_t(64) << 20)) return RS_OK;
    int rc = zero_copy_buffer(ctx, need);
    if (rc) return rc;
    rsamd::FileDirect d;
    d.k = k;
    d.nout = m;
    d.block = blk;
    d.units = S / 8;
    d.file_len = file_len;
    d.file = ctx->zc_dev;
    for (int p = 0; p < m; ++p) d.out[k + p] = ctx->zc_dev + fbytes + size_t(p) * stride;
    std::vector<DevPlan> plans;
    RS_HIP(c.encode_plan().device_plans(&plans));
    d.tabs = plans[0].tabs;
    if (!rsamd::file_direct_ok(d)) return RS_OK;
    // Completion by the kernel's signal (run_small) instead of a stream
    // synchronisation below 2 MiB, where the ~3 us the synchronisation adds
    // is a measurable part of the call: 90,999-B file 20.3 -> 17.4 us
    // (profiles/r6/small_latency_files_{off,on}_r6s1.json).
    const bool signal = small_signal_enabled() && need <= (size_t(2) << 20) && d.units > 0;
    if (signal) {
        rc = next_signal(ctx, &d.sig.flag, &d.sig.ctr, &d.sig.seq);
        if (rc) return rc;
    }
    *taken = true;
    const bool pool = need > file_zc_pool_min();
    auto copy = [&](const std::vector<rsamd::CopyJob> &jobs) {
        if (pool)
            rsamd::CopyPool::get().copy(jobs);
        else
            rsamd::CopyPool::copy_here(jobs);
    };
    std::vector<rsamd::CopyJob> jobs;
    if (file_len) jobs.push_back({ctx->zc, file, file_len});
    copy(jobs);
    bounds::allow(d.file, file_len);
    for (int p = 0; p < m; ++p) bounds::allow(d.out[k + p], S);
    const hipError_t e = rsamd::launch_file_encode_direct(d, ctx->stream);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(ctx->stream);
        return hip_fail(e, "launch_file_encode_direct (small file)");
    }
    jobs.clear();
    split_jobs(file, file_len, blk, k, shards, nullptr, 0, 0, S / blk, &jobs);
    copy(jobs);
    if (signal) {
        rc = wait_signal(ctx, d.sig.seq, nullptr);
        if (rc) {
            (void)hipStreamSynchronize(ctx->stream);
            return rc;
        }
    } else {
        RS_HIP(hipStreamSynchronize(ctx->stream));
    }
    jobs.clear();
    for (int p = 0; p < m; ++p) jobs.push_back({shards[k + p], ctx->zc + fbytes + size_t(p) * stride, S});
    copy(jobs);
    return RS_OK;
}

// The staged form of the host file encode: chunks of block rows through
// run_chunks.  file_len fills every row but the last (the padded layout).
int file_encode_staged(const Codec &c, const uint8_t *file, size_t file_len, size_t blk, uint8_t *const *shards,
                       size_t S, ThreadCtx *ctx, bool pinned) {
    const size_t kb = size_t(c.k()) * blk;
    const FileChunks f = file_chunks(c.k(), c.total(), S, blk, pinned);
    auto flen_of = [&](size_t r0, size_t rc_rows) {  // every row holds file bytes
        return std::min(rc_rows * kb, file_len - r0 * kb);
    };
    auto io = [&](size_t j, std::vector<Xfer> *in, std::vector<Xfer> *out) {
        const size_t r0 = j * f.R, rc_rows = std::min(f.R, f.rows - r0);
        in->push_back({const_cast<uint8_t *>(file) + r0 * kb, 0, flen_of(r0, rc_rows)});
        for (int i = 0; i < c.total(); ++i)
            out->push_back({shards[i] + r0 * blk, f.fbytes + size_t(i) * f.sstride, rc_rows * blk});
    };
    auto code = [&](size_t j, uint8_t *buf, hipStream_t st) -> int {
        const size_t r0 = j * f.R, rc_rows = std::min(f.R, f.rows - r0);
        return file_encode_dev(c, buf, flen_of(r0, rc_rows), blk, buf + f.fbytes, f.sstride, st);
    };
    return run_chunks(ctx, f.n, f.buf_bytes, pinned, io, code);
}

// Mirrored form of the host file calls (pageable callers, host.hpp
// run_mirrored) -- the file layout on the CPU, the coding on the GPU.  A
// file's data shards are its own bytes rearranged (ReedSolomonEncoder.java:
// 56-60 splits, ReedSolomonDecoder.java:92-103 merges), so they need not
// cross the link in both directions: the CPU moves them between the caller's
// file and shard arrays (the same pass that fills the pinned slots), and only
// the bytes the GPU codes cross the link -- data in, parity (or rebuilt shards)
// out: a 4+2 file encode moves 1.5 file sizes across the link instead of 2.5.
// The slots hold shard columns of whole block rows (one slot per shard,
// page-aligned), coded by the shard direct kernels.
//
// Chunk boundaries in block rows, and the slot stride, for `nslots` slots.
std::vector<size_t> mirror_row_bounds(size_t rows, size_t blk, int nslots, size_t *slot_stride) {
    const size_t per = mirror_chunk_bytes(rows * blk, nslots, blk);
    std::vector<size_t> b = ramp_bounds(rows, std::max<size_t>(1, per / blk), 1);
    size_t widest = 0;
    for (size_t j = 0; j + 1 < b.size(); ++j) widest = std::max(widest, b[j + 1] - b[j]);
    *slot_stride = round_up(widest * blk, kMirrorAlign);
    return b;
}

// Codes chunk j's columns of the slots: every launch group of `plans` over the
// slot-indexed shards.  `sig` (may be null): the last launch signals its
// completion (run_small), the stream having ordered the others before it.
int code_slots(const std::vector<DevPlan> &plans, const std::vector<int> &in_slots, const std::vector<int> &out_slots,
               uint8_t *dev, size_t slot_stride, size_t n, Mode mode, int *flag, hipStream_t st,
               const rsamd::DirectSignal *sig = nullptr) {
    std::vector<rsamd::DirectPlan> dp;
    if (!direct_plans(plans, in_slots, out_slots, [&](int sl) { return dev + size_t(sl) * slot_stride; }, &dp))
        return fail(RS_E_HIP, "direct plans over the mirror slots");
    for (size_t i = 0; i < dp.size(); ++i)
        RS_HIP(rsamd::launch_gf_direct(dp[i], n, mode, flag, st, nullptr, i + 1 == dp.size() ? sig : nullptr));
    return RS_OK;
}

// File encode: the CPU splits each chunk's block rows into the caller's data
// shards and the data slots at once; the GPU codes the parity slots, which are
// copied out.  *taken = false (nothing done) when the direct kernels cannot
// take the code (more than kMaxDirectIn data shards).
int file_encode_mirrored(const Codec &c, const uint8_t *file, size_t file_len, size_t blk, uint8_t *const *shards,
                         size_t S, ThreadCtx *ctx, bool *taken) {
    *taken = false;
    const int k = c.k(), T = c.total();
    if (!direct_enabled() || k > rsamd::kMaxDirectIn) return RS_OK;
    std::vector<DevPlan> plans;
    if (c.m() > 0) RS_HIP(c.encode_plan().device_plans(&plans));
    std::vector<int> in_slots(k), out_slots(c.m());
    for (int i = 0; i < k; ++i) in_slots[i] = i;
    for (int p = 0; p < c.m(); ++p) out_slots[p] = k + p;
    size_t ss = 0;
    const std::vector<size_t> cb = mirror_row_bounds(S / blk, blk, T, &ss);
    auto io = [&](size_t j, std::vector<Xfer> *, std::vector<Xfer> *out) {
        const size_t r0 = cb[j], n = (cb[j + 1] - r0) * blk;
        for (int p = 0; p < c.m(); ++p) out->push_back({shards[k + p] + r0 * blk, size_t(k + p) * ss, n});
    };
    auto side = [&](size_t j, uint8_t *slot, std::vector<rsamd::CopyJob> *before, std::vector<rsamd::CopyJob> *) {
        std::vector<uint8_t *> sl(k);
        for (int i = 0; i < k; ++i) sl[i] = slot + size_t(i) * ss;  // slot i holds the chunk's rows from cb[j]
        split_jobs(file, file_len, blk, k, shards, sl.data(), cb[j], cb[j], cb[j + 1], before);
    };
    auto code = [&](size_t j, uint8_t *dev, hipStream_t st) -> int {
        if (plans.empty()) return RS_OK;  // no parity: the split is the whole call
        return code_slots(plans, in_slots, out_slots, dev, ss, (cb[j + 1] - cb[j]) * blk, Mode::Code, nullptr, st);
    };
    *taken = true;
    return run_mirrored(ctx, cb.size() - 1, ss * size_t(T), io, code, side);
}

// Direct path of the host file decode on caller-pinned memory: the absent
// shards rebuilt in place across the link by the shard direct kernels (the
// survivors read, the rebuilt shards written: only coded bytes cross the
// link), while the copy pool merges the present data shards into the file.
// When the file is device-mapped too (and everything 8-byte aligned, block %
// 8 == 0) the kernels store each rebuilt data shard into the file as well
// (kernels.hpp DirectTee): the extra bytes travel device-to-host, the
// direction the survivors leave idle, and no merge waits for the kernels.
// Otherwise the rebuilt data shards are merged once the kernels are done.
// *taken = false, nothing enqueued, when the direct kernels cannot take the
// plan or a shard has no device address.
int file_decode_pinned(const Codec &c, uint8_t *const *shards, const uint8_t *present, const std::vector<int> &missing,
                       size_t blk, uint8_t *file_out, size_t file_size, size_t rows_needed, ThreadCtx *ctx,
                       bool *taken) {
    *taken = false;
    const int k = c.k();
    std::shared_ptr<const Plan> plan;
    std::vector<rsamd::DirectPlan> dp;
    if (!missing.empty()) {
        int rc = c.decode_plan(present, &plan);
        if (rc) return fail(rc, rc == RS_E_SINGULAR ? "Matrix is singular" : "Not enough shards present");
        std::vector<DevPlan> plans;
        RS_HIP(plan->device_plans(&plans));
        if (!direct_plans(plans, plan->in_idx(), plan->out_idx(), [&](int sl) { return host_dev_addr(shards[sl]); },
                          &dp))
            return RS_OK;
    }
    const size_t n = rows_needed * blk;
    // TUNING builds: RSAMD_FILE_DEC_TEE=0 merges the rebuilt data shards on the host (A/B)
    uint8_t *const fdev = dp.empty() ? nullptr : host_dev_addr(file_out);
    const bool tee = fdev && rsamd::tuning_size("RSAMD_FILE_DEC_TEE", 1) && blk % 8 == 0 &&
                     reinterpret_cast<uintptr_t>(fdev) % 8 == 0 && reinterpret_cast<uintptr_t>(dp[0].in[0]) % 8 == 0;
    std::vector<rsamd::DirectTee> tees(dp.size());
    for (size_t g = 0; g < dp.size(); ++g) {
        tees[g].file = fdev;
        tees[g].file_size = file_size;
        tees[g].blk = blk;
        tees[g].k = uint64_t(k);
        for (int q = 0; q < dp[g].nout; ++q) {
            const int sidx = plan->out_idx()[g * size_t(rsamd::kMaxOut) + size_t(q)];
            tees[g].data[q] = sidx < k ? sidx : -1;
        }
    }
    if (tee) bounds::allow(fdev, file_size);
    for (size_t g = 0; g < dp.size(); ++g) {
        const rsamd::DirectPlan &d = dp[g];
        for (int i = 0; i < d.nin; ++i) bounds::allow(d.in[i], n);
        for (int q = 0; q < d.nout; ++q) bounds::allow(d.out[q], n);
        const hipError_t e = rsamd::launch_gf_direct(d, n, Mode::Code, nullptr, ctx->stream, tee ? &tees[g] : nullptr);
        if (e != hipSuccess) {  // the groups already launched finish before the caller gets control
            (void)hipStreamSynchronize(ctx->stream);
            return hip_fail(e, "launch_gf_direct (file decode)");
        }
    }
    *taken = true;
    std::vector<const uint8_t *> src(shards, shards + k);
    std::vector<bool> now(static_cast<size_t>(k), false), later(static_cast<size_t>(k), false);
    for (int d = 0; d < k; ++d) {
        if (present[d])
            now[d] = true;
        else
            later[d] = true;
    }
    std::vector<rsamd::CopyJob> jobs;
    merge_jobs(k, blk, file_out, file_size, src.data(), now, 0, rows_needed, &jobs);
    rsamd::CopyPool::get().copy(jobs);
    RS_HIP(hipStreamSynchronize(ctx->stream));
    if (tee) return RS_OK;  // the kernels wrote the rebuilt data shards' file bytes
    jobs.clear();
    merge_jobs(k, blk, file_out, file_size, src.data(), later, 0, rows_needed, &jobs);
    rsamd::CopyPool::get().copy(jobs);
    return RS_OK;
}

// Block rows a file decode must code: all of them when a shard is rebuilt,
// else only those holding file bytes.
size_t file_rows_needed(int k, size_t S, size_t blk, const std::vector<int> &missing, size_t file_size) {
    const size_t rows = S / blk, kb = size_t(k) * blk;
    return missing.empty() ? std::min(rows, (file_size + kb - 1) / kb) : rows;
}

// Small pageable file decodes (one zero-copy pass): the survivors are copied
// into the context's device-mapped buffer, the direct kernels rebuild the
// absent shards there, and the host merges the present data shards into the
// file meanwhile; then the rebuilt shards are copied out, a rebuilt data
// shard into the file in the same pass (tee_jobs).  Only the survivors and
// the rebuilt shards cross the link; with nothing absent the call is the
// merge alone, on the host (TUNING builds: RSAMD_FILE_ZC_SPLIT=0 keeps the
// all-GPU pass).  *taken = false when the direct kernels cannot take the plan.
int file_decode_zc_split(const Codec &c, uint8_t *const *shards, const uint8_t *present, const std::vector<int> &surv,
                         const std::vector<int> &missing, size_t blk, uint8_t *file_out, size_t file_size,
                         size_t rows_needed, ThreadCtx *ctx, bool *taken) {
    *taken = false;
    const int k = c.k(), T = c.total();
    if (!rsamd::tuning_size("RSAMD_FILE_ZC_SPLIT", 1) || !direct_enabled() || k > rsamd::kMaxDirectIn) return RS_OK;
    std::vector<const uint8_t *> src(shards, shards + k);
    std::vector<bool> now(static_cast<size_t>(k), false);
    for (int d = 0; d < k; ++d) now[d] = present[d] != 0;
    std::vector<rsamd::CopyJob> jobs;
    if (missing.empty()) {  // mergeShardsToFile alone
        merge_jobs(k, blk, file_out, file_size, src.data(), now, 0, rows_needed, &jobs);
        if (file_size > zc_pool_min())
            rsamd::CopyPool::get().copy(jobs);
        else
            rsamd::CopyPool::copy_here(jobs);
        *taken = true;
        return RS_OK;
    }
    std::shared_ptr<const Plan> plan;
    int rc = c.decode_plan(present, &plan);
    if (rc) return fail(rc, rc == RS_E_SINGULAR ? "Matrix is singular" : "Not enough shards present");
    std::vector<DevPlan> plans;
    RS_HIP(plan->device_plans(&plans));
    for (const DevPlan &p : plans)
        if (p.nin > rsamd::kMaxDirectIn) return RS_OK;
    // From 128 KiB per shard: two signalled passes over two halves of the
    // block rows (as file_encode_zc_halves), each half's slots on pages of
    // their own; the second half's survivors are copied in while the first
    // half is coded, the first half's rebuilt shards copied out (and teed into
    // the file) while the second half is coded.
    if (small_signal_enabled() && small_parts() > 1 && rows_needed >= 2 && rows_needed * blk >= small_parts_min()) {
        const size_t A = small_parts_align(), r[3] = {0, rows_needed / 2, rows_needed};
        size_t base[2], st[2], nh[2], at = 0;
        for (int h = 0; h < 2; ++h) {
            nh[h] = (r[h + 1] - r[h]) * blk;
            st[h] = round_up(round_up(nh[h], 16), A);
            base[h] = at;
            at += st[h] * size_t(T);
        }
        if (at <= (size_t(64) << 20)) {
            rc = zero_copy_buffer(ctx, at);
            if (rc) return rc;
            rsamd::DirectSignal sg[2];
            for (rsamd::DirectSignal &g : sg) {
                rc = next_signal(ctx, &g.flag, &g.ctr, &g.seq);
                if (rc) return rc;
            }
            *taken = true;
            const bool pool = at > file_zc_pool_min();
            auto copy = [&]() {
                if (pool)
                    rsamd::CopyPool::get().copy(jobs);
                else
                    rsamd::CopyPool::copy_here(jobs);
                jobs.clear();
            };
            for (int h = 0; h < 2; ++h) {
                const size_t n16 = round_up(nh[h], 16);
                for (int sidx : surv) {
                    jobs.push_back({ctx->zc + base[h] + size_t(sidx) * st[h], shards[sidx] + r[h] * blk, nh[h]});
                    if (n16 > nh[h]) std::memset(ctx->zc + base[h] + size_t(sidx) * st[h] + nh[h], 0, n16 - nh[h]);
                }
                copy();
                rc = code_slots(plans, plan->in_idx(), plan->out_idx(), ctx->zc_dev + base[h], st[h], n16, Mode::Code,
                                nullptr, ctx->stream, &sg[h]);
                if (rc) {
                    (void)hipStreamSynchronize(ctx->stream);
                    return rc;
                }
            }
            merge_jobs(k, blk, file_out, file_size, src.data(), now, 0, rows_needed, &jobs);
            copy();
            for (int h = 0; h < 2; ++h) {
                rc = wait_signal(ctx, sg[h].seq, nullptr);
                if (rc) {
                    (void)hipStreamSynchronize(ctx->stream);
                    return rc;
                }
                for (int sidx : missing) {
                    const uint8_t *slot = ctx->zc + base[h] + size_t(sidx) * st[h];
                    if (sidx < k)
                        tee_jobs(k, blk, file_out, file_size, sidx, slot, shards[sidx] + r[h] * blk, r[h], r[h + 1],
                                 &jobs);
                    else
                        jobs.push_back({shards[sidx] + r[h] * blk, slot, nh[h]});
                }
                copy();
            }
            return RS_OK;
        }
    }
    const size_t n = rows_needed * blk, ss = round_up(std::max<size_t>(n, 1), 256), need = ss * size_t(T);
    if (need > (size_t(64) << 20)) return RS_OK;
    rc = zero_copy_buffer(ctx, need);
    if (rc) return rc;
    *taken = true;
    const bool pool = need > file_zc_pool_min();
    auto copy = [&](const std::vector<rsamd::CopyJob> &js) {
        if (pool)
            rsamd::CopyPool::get().copy(js);
        else
            rsamd::CopyPool::copy_here(js);
    };
    // Below 2 MiB the last launch signals its completion (run_small) and the
    // slots are coded in whole 16-byte vectors: the survivors' bytes past n
    // up to the next 16 are zeroed (the slots' stride leaves room), no byte
    // tail in the launch; the rebuilt pad bytes are never copied out.
    // 90,999-B file, {0,5} absent: 27.5 -> 16.3 us (profiles/r6/
    // small_latency_files_{off,on}_r6s1.json).
    const bool signal = small_signal_enabled() && need <= (size_t(2) << 20) && n > 0;
    rsamd::DirectSignal sg;
    if (signal) {
        rc = next_signal(ctx, &sg.flag, &sg.ctr, &sg.seq);
        if (rc) return rc;
    }
    const size_t ncode = signal ? round_up(n, 16) : n;
    for (int sidx : surv) {
        jobs.push_back({ctx->zc + size_t(sidx) * ss, shards[sidx], n});
        if (ncode > n) std::memset(ctx->zc + size_t(sidx) * ss + n, 0, ncode - n);
    }
    copy(jobs);
    rc = code_slots(plans, plan->in_idx(), plan->out_idx(), ctx->zc_dev, ss, ncode, Mode::Code, nullptr, ctx->stream,
                    signal ? &sg : nullptr);
    if (rc) {
        (void)hipStreamSynchronize(ctx->stream);
        return rc;
    }
    jobs.clear();
    merge_jobs(k, blk, file_out, file_size, src.data(), now, 0, rows_needed, &jobs);
    copy(jobs);
    if (signal) {
        rc = wait_signal(ctx, sg.seq, nullptr);
        if (rc) {
            (void)hipStreamSynchronize(ctx->stream);
            return rc;
        }
    } else {
        RS_HIP(hipStreamSynchronize(ctx->stream));
    }
    jobs.clear();
    for (int sidx : missing) {
        const uint8_t *slot = ctx->zc + size_t(sidx) * ss;
        if (sidx < k)
            tee_jobs(k, blk, file_out, file_size, sidx, slot, shards[sidx], 0, rows_needed, &jobs);
        else
            jobs.push_back({shards[sidx], slot, n});
    }
    copy(jobs);
    return RS_OK;
}

// The staged form of the host file decode (rs_file_decode's whole-shard
// case): chunks of block rows through run_chunks.
int file_decode_staged(const Codec &c, uint8_t *const *shards, size_t S, const uint8_t *present,
                       const std::vector<int> &surv, const std::vector<int> &missing, size_t blk, uint8_t *file_out,
                       size_t file_size, ThreadCtx *ctx, bool pinned) {
    const size_t kb = size_t(c.k()) * blk;
    const FileChunks f = file_chunks(c.k(), c.total(), S, blk, pinned);
    const size_t rows_needed = file_rows_needed(c.k(), S, blk, missing, file_size);
    if (rows_needed == 0) return RS_OK;
    auto flen_of = [&](size_t r0, size_t rc_rows) {
        const size_t fo = r0 * kb;
        return file_size > fo ? std::min(rc_rows * kb, file_size - fo) : size_t(0);
    };
    auto io = [&](size_t j, std::vector<Xfer> *in, std::vector<Xfer> *out) {
        const size_t r0 = j * f.R, rc_rows = std::min(f.R, f.rows - r0), n = rc_rows * blk;
        for (int sidx : surv) in->push_back({shards[sidx] + r0 * blk, f.fbytes + size_t(sidx) * f.sstride, n});
        for (int sidx : missing) out->push_back({shards[sidx] + r0 * blk, f.fbytes + size_t(sidx) * f.sstride, n});
        const size_t flen = flen_of(r0, rc_rows);
        if (flen) out->push_back({file_out + r0 * kb, 0, flen});
    };
    auto code = [&](size_t j, uint8_t *buf, hipStream_t st) -> int {
        const size_t r0 = j * f.R, rc_rows = std::min(f.R, f.rows - r0);
        return file_decode_dev(c, buf + f.fbytes, rc_rows * blk, f.sstride, present, blk, buf, flen_of(r0, rc_rows),
                               true, st);
    };
    return run_chunks(ctx, (rows_needed + f.R - 1) / f.R, f.buf_bytes, pinned, io, code);
}

// File decode: the survivors' rows go to their slots, the GPU rebuilds the
// absent shards' slots, which are copied out to the caller's arrays; the CPU
// merges each chunk's data shards into the file (present ones from the
// caller's arrays, rebuilt ones from their slots) behind the chunk's kernels.
// With no shard absent there is nothing to code and the merge is the call.
// *taken = false (nothing done) when the direct kernels cannot take the code.
int file_decode_mirrored(const Codec &c, uint8_t *const *shards, const uint8_t *present, const std::vector<int> &surv,
                         const std::vector<int> &missing, size_t blk, uint8_t *file_out, size_t file_size,
                         size_t rows_needed, ThreadCtx *ctx, bool *taken) {
    *taken = false;
    const int k = c.k(), T = c.total();
    if (!direct_enabled() || k > rsamd::kMaxDirectIn) return RS_OK;
    std::shared_ptr<const Plan> plan;
    std::vector<DevPlan> plans;
    if (!missing.empty()) {
        int rc = c.decode_plan(present, &plan);
        if (rc) return fail(rc, rc == RS_E_SINGULAR ? "Matrix is singular" : "Not enough shards present");
        RS_HIP(plan->device_plans(&plans));
    }
    size_t ss = 0;
    const std::vector<size_t> cb = mirror_row_bounds(rows_needed, blk, T, &ss);
    // the chunk's data shards into the file: present ones from the caller's
    // arrays, rebuilt ones from their slots
    const std::vector<bool> all(size_t(k), true);
    auto merge = [&](size_t r0, size_t r1, const uint8_t *slot, std::vector<rsamd::CopyJob> *jobs) {
        std::vector<const uint8_t *> src(k);
        for (int d = 0; d < k; ++d) src[d] = present[d] ? shards[d] + r0 * blk : slot + size_t(d) * ss;
        merge_jobs(k, blk, file_out, file_size, src.data(), all, r0, r1, jobs);
    };
    if (missing.empty()) {  // nothing to rebuild: the merge alone (mergeShardsToFile)
        std::vector<rsamd::CopyJob> jobs;
        merge(0, rows_needed, nullptr, &jobs);
        rsamd::CopyPool::get().copy(jobs);
        *taken = true;
        return RS_OK;
    }
    // Data shards go to the file in the pass that moves them anyway (TUNING
    // builds: RSAMD_DECODE_TEE=0 merges them in a pass of their own): present
    // ones from the caller's arrays into their slots and the file, rebuilt ones
    // from their slots into the caller's arrays and the file.
    const bool tee = rsamd::tuning_size("RSAMD_DECODE_TEE", 1) != 0;
    auto io = [&](size_t j, std::vector<Xfer> *in, std::vector<Xfer> *out) {
        const size_t r0 = cb[j], n = (cb[j + 1] - r0) * blk;
        for (int sidx : surv)
            if (!tee || sidx >= k) in->push_back({shards[sidx] + r0 * blk, size_t(sidx) * ss, n});
        for (int sidx : missing)
            if (!tee || sidx >= k) out->push_back({shards[sidx] + r0 * blk, size_t(sidx) * ss, n});
    };
    auto side = [&](size_t j, uint8_t *slot, std::vector<rsamd::CopyJob> *before, std::vector<rsamd::CopyJob> *after) {
        const size_t r0 = cb[j], r1 = cb[j + 1];
        if (!tee) return merge(r0, r1, slot, after);
        const size_t rb = row_block() ? row_block() : std::max<size_t>(1, r1 - r0);
        for (size_t b0 = r0; b0 < r1; b0 += rb) {  // blocks of rows, every shard's jobs of a block together
            const size_t b1 = std::min(r1, b0 + rb);
            for (int d = 0; d < k; ++d) {
                uint8_t *mine = shards[d] + b0 * blk, *sl = slot + size_t(d) * ss + (b0 - r0) * blk;
                if (present[d])
                    tee_jobs(k, blk, file_out, file_size, d, mine, sl, b0, b1, before);
                else
                    tee_jobs(k, blk, file_out, file_size, d, sl, mine, b0, b1, after);
            }
        }
    };
    auto code = [&](size_t j, uint8_t *dev, hipStream_t st) -> int {
        return code_slots(plans, plan->in_idx(), plan->out_idx(), dev, ss, (cb[j + 1] - cb[j]) * blk, Mode::Code,
                          nullptr, st);
    };
    *taken = true;
    return run_mirrored(ctx, cb.size() - 1, ss * size_t(T), io, code, side);
}

// rs_file_decode when byteCntInShard is the whole shard: one pass per chunk
// -- upload the first k present shards, rebuild every absent shard and merge
// the data shards into the file chunk on the GPU, download the rebuilt shards
// (decodeMissing fills them in, ReedSolomonDecoder.java:36) and the file bytes.
// Same checks, order and messages as rs_decode_missing + the merge.
int file_decode_chunked(const Codec &c, uint8_t *const *shards, const int64_t *lens, const uint8_t *present,
                        int32_t block, uint8_t *file_out, int64_t file_size) {
    const int T = c.total(), k = c.k();
    const int64_t S = lens[0];
    int rc = check_buffers_and_sizes(c, shards, T, lens, 0, S);
    if (rc) return rc;
    int n_present = 0;
    for (int i = 0; i < T; ++i) n_present += present[i] ? 1 : 0;
    if (n_present < k) return fail(RS_E_NOT_ENOUGH, "Not enough shards present");
    if (n_present < T) {
        std::shared_ptr<const Plan> plan;
        rc = c.decode_plan(present, &plan);
        if (rc) return fail(rc, rc == RS_E_SINGULAR ? "Matrix is singular" : "Not enough shards present");
    }
    if (file_size < 0 || file_size > S * k) return fail(RS_E_INVALID, "file size exceeds k * shard length");
    if (file_size > 0 && !file_out) return fail(RS_E_INVALID, "file_out is NULL");
    if (S == 0 || (file_size == 0 && n_present == T)) return RS_OK;
    rc = need_device();
    if (rc) return rc;
    ThreadCtx *ctx = nullptr;
    rc = thread_ctx(&ctx);
    if (rc) return rc;
    const size_t blk = size_t(block);
    std::vector<const uint8_t *> bufs(shards, shards + T);
    bufs.push_back(file_out);
    const bool pinned = all_pinned(bufs.data(), int(bufs.size()));
    const bool big = file_chunks(k, T, size_t(S), blk, false).n > 1 || size_t(S) >= direct_min_bytes();
    std::vector<int> surv, missing;
    for (int i = 0; i < T; ++i) {
        if (present[i] && int(surv.size()) < k) surv.push_back(i);
        if (!present[i]) missing.push_back(i);
    }
    const size_t rows_needed = file_rows_needed(k, size_t(S), blk, missing, size_t(file_size));
    bool taken = false;
    if (pinned) {  // direct path: the absent shards rebuilt in place, the file merged on the host
        rc = file_decode_pinned(c, shards, present, missing, blk, file_out, size_t(file_size), rows_needed, ctx,
                                &taken);
    } else if (big && size_t(S) >= mirror_min_bytes()) {
        rc = file_decode_mirrored(c, shards, present, surv, missing, blk, file_out, size_t(file_size), rows_needed,
                                  ctx, &taken);
    } else {
        rc = file_decode_zc_split(c, shards, present, surv, missing, blk, file_out, size_t(file_size), rows_needed,
                                  ctx, &taken);
    }
    if (rc || taken) return rc;
    return file_decode_staged(c, shards, size_t(S), present, surv, missing, blk, file_out, size_t(file_size), ctx,
                              pinned);
}

// Next staging slot of this thread with >= bytes on both sides, once the
// kernels of the call that last used it have completed.
int masked_slot(size_t bytes, MaskedSlot **out, ThreadCtx **ctx_out) {
    ThreadCtx *ctx = nullptr;
    int rc = thread_ctx(&ctx);
    if (rc) return rc;
    *ctx_out = ctx;
    MaskedSlot &sl = ctx->masked[ctx->masked_next];
    ctx->masked_next ^= 1;
    if (!sl.uploaded) RS_HIP(hipEventCreateWithFlags(&sl.uploaded, hipEventDisableTiming));
    if (!sl.done) RS_HIP(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    else RS_HIP(hipEventSynchronize(sl.done));
    if (sl.host_cap < bytes) {
        if (sl.host) RS_HIP(hipHostFree(sl.host));
        sl.host = nullptr;
        sl.host_cap = 0;
        RS_HIP(hipHostMalloc(reinterpret_cast<void **>(&sl.host), bytes, hipHostMallocDefault));
        sl.host_cap = bytes;
    }
    rc = grow(&sl.dev, &sl.dev_cap, bytes);
    if (rc) return rc;
    *out = &sl;
    return RS_OK;
}

// host -> device copy of a slot's first `bytes` on the context's H2D stream;
// `stream` waits for it.
int upload_slot(ThreadCtx *ctx, MaskedSlot *sl, size_t bytes, hipStream_t stream) {
    RS_HIP(hipMemcpyAsync(sl->dev, sl->host, bytes, hipMemcpyHostToDevice, ctx->stream3));
    RS_HIP(hipEventRecord(sl->uploaded, ctx->stream3));
    RS_HIP(hipStreamWaitEvent(stream, sl->uploaded, 0));
    return RS_OK;
}

// One launch per output group over the pattern tables; plan_ids holds the
// stripes' presence bitmasks.
int launch_pattern_groups(const Codec &c, const rsamd::PatternTables &pt, const Geometry &geo, size_t pattern_bytes,
                          const int32_t *bits, int32_t *bad, hipStream_t stream) {
    for (int g = 0; g < pt.groups; ++g) {
        rsamd::MaskedPlan mp;
        mp.records = pt.records + size_t(g) * pt.npat * pt.rec_stride;
        mp.rec_stride = pt.rec_stride;
        mp.plan_ids = bits;
        mp.nin = c.k();
        mp.mslots = pt.mslots;
        mp.mask_table = pt.mask_table;
        mp.mask_bits = c.total();
        mp.bad = g == 0 ? bad : nullptr;
        mp.pattern_bytes = pattern_bytes;
        RS_HIP(rsamd::launch_gf_masked(geo, mp, stream));
    }
    return RS_OK;
}

// Presence bitmasks of present[0 .. n) rows into bits.  RS_OK, or
// RS_E_NOT_ENOUGH when a row has fewer than k flags set, or RS_E_SINGULAR when
// a row's pattern has no record in table.  Large batches use host threads.
// Codes of up to 8 shards read a row as one 8-byte word: every nonzero flag
// byte becomes 0x01, and one multiply gathers byte i into bit i of the top
// byte (the partial products of 0x0102040810204080 never overlap, so no
// carries).  4-5x faster than the per-byte loop (1.4 against 5.5-7.5 ms per
// 1 M rows of 6 on one core): this runs before the first kernel of a call.
int presence_bits(const uint8_t *present, size_t n, int T, int k, const int32_t *table, uint32_t *bits) {
    auto run = [&](size_t t0, size_t t1) {
        int rc = RS_OK;
        // rows whose 8-byte read stays inside present[0 .. n*T)
        const size_t word_end = T <= 8 && n * size_t(T) >= 8 ? std::min(t1, (n * size_t(T) - 8) / size_t(T) + 1) : t0;
        const uint64_t keep = T >= 8 ? ~uint64_t(0) : (uint64_t(1) << (8 * T)) - 1;
        size_t t = t0;
        for (; t < word_end; ++t) {
            uint64_t x;
            std::memcpy(&x, present + t * T, 8);
            x &= keep;
            const uint64_t nz =
                ((((x & 0x7F7F7F7F7F7F7F7FULL) + 0x7F7F7F7F7F7F7F7FULL) | x) >> 7) & 0x0101010101010101ULL;
            const uint32_t b = uint32_t((nz * 0x0102040810204080ULL) >> 56);
            bits[t] = b;
            if (table[b] < 0) rc = __builtin_popcount(b) < k ? RS_E_NOT_ENOUGH : (rc ? rc : RS_E_SINGULAR);
        }
        for (; t < t1; ++t) {
            const uint8_t *row = present + t * T;
            uint32_t b = 0;
            for (int i = 0; i < T; ++i) b |= uint32_t(row[i] != 0) << i;
            bits[t] = b;
            if (table[b] < 0) rc = __builtin_popcount(b) < k ? RS_E_NOT_ENOUGH : (rc ? rc : RS_E_SINGULAR);
        }
        return rc;
    };
    const size_t nthreads =
        n >= (size_t(1) << 18) ? std::min<size_t>(8, std::max(1u, std::thread::hardware_concurrency())) : 1;
    if (nthreads <= 1) return run(0, n);
    std::vector<std::thread> pool;
    std::vector<int> rcs(nthreads, RS_OK);
    const size_t per = (n + nthreads - 1) / nthreads;
    for (size_t w = 1; w < nthreads; ++w)
        pool.emplace_back([&, w] { rcs[w] = run(std::min(n, w * per), std::min(n, (w + 1) * per)); });
    rcs[0] = run(0, std::min(n, per));
    for (auto &th : pool) th.join();
    int rc = RS_OK;
    for (int r : rcs) {
        if (r == RS_E_NOT_ENOUGH) return r;
        if (r) rc = r;
    }
    return rc;
}

// n_stripes presence patterns (rows of present) over the stripes of geo:
// pattern_bytes 0 -> one per stripe of geo; otherwise geo is the packed view of
// a granule batch and each pattern covers pattern_bytes batch columns
// (rsamd::MaskedPlan::pattern_bytes).
int decode_masked_dev(const Codec &c, const uint8_t *present, size_t n_stripes, const Geometry &geo,
                      size_t pattern_bytes, hipStream_t stream) {
    const int T = c.total(), k = c.k();

    // Codes with a pattern table: upload the stripes' presence bitmasks, the
    // kernels look their records up (no per-call plan building).
    rsamd::PatternTables pt;
    std::string err;
    if (c.pattern_tables(&pt, &err) == RS_OK) {
        MaskedSlot *sl = nullptr;
        ThreadCtx *ctx = nullptr;
        int rc = masked_slot(n_stripes * sizeof(uint32_t), &sl, &ctx);
        if (rc) return rc;
        uint32_t *bits = reinterpret_cast<uint32_t *>(sl->host);
        rc = presence_bits(present, n_stripes, T, k, pt.host_mask_table, bits);
        if (rc) return fail(rc, rc == RS_E_SINGULAR ? "Matrix is singular" : "Not enough shards present");
        rc = upload_slot(ctx, sl, n_stripes * sizeof(uint32_t), stream);
        if (rc) return rc;
        rc = launch_pattern_groups(c, pt, geo, pattern_bytes, reinterpret_cast<const int32_t *>(sl->dev), nullptr,
                                   stream);
        if (rc) return rc;
        RS_HIP(hipEventRecord(sl->done, stream));
        return RS_OK;
    }

    // Wide codes: distinct presence patterns -> per-call record ids (ordered
    // map of the flag vector).
    std::vector<std::vector<uint8_t>> pats;
    std::vector<int32_t> pid(n_stripes);
    std::vector<uint8_t> key(T);
    std::map<std::vector<uint8_t>, int32_t> ids;
    for (size_t t = 0; t < n_stripes; ++t) {
        int np = 0;
        for (int i = 0; i < T; ++i) np += (key[i] = present[t * T + i] ? 1 : 0);
        if (np < k) return fail(RS_E_NOT_ENOUGH, "Not enough shards present");
        auto it = ids.find(key);
        if (it == ids.end()) {
            pats.push_back(key);
            it = ids.emplace(key, int32_t(pats.size() - 1)).first;
        }
        pid[t] = it->second;
    }
    std::vector<std::shared_ptr<const Plan>> plans(pats.size());
    size_t max_missing = 0;
    for (size_t q = 0; q < pats.size(); ++q) {
        int rc = c.decode_plan(pats[q].data(), &plans[q]);
        if (rc) return fail(rc, rc == RS_E_SINGULAR ? "Matrix is singular" : "Not enough shards present");
        max_missing = std::max(max_missing, plans[q]->out_idx().size());
    }
    if (max_missing == 0) return RS_OK;
    const int ms = std::min<int>(c.m(), rsamd::kMaxOut);
    const size_t groups = (max_missing + ms - 1) / ms;
    const rsamd::MaskedRecordLayout L = rsamd::masked_record_layout(k, ms);
    const size_t npat = pats.size();
    const size_t ids_off = groups * npat * L.bytes;
    const size_t bytes = ids_off + n_stripes * sizeof(int32_t);
    MaskedSlot *sl = nullptr;
    ThreadCtx *ctx = nullptr;
    int rc = masked_slot(bytes, &sl, &ctx);
    if (rc) return rc;
    for (size_t g = 0; g < groups; ++g)
        for (size_t q = 0; q < npat; ++q) rsamd::fill_masked_record(*plans[q], int(g), ms, L, sl->host + (g * npat + q) * L.bytes);
    std::memcpy(sl->host + ids_off, pid.data(), n_stripes * sizeof(int32_t));
    rc = upload_slot(ctx, sl, bytes, stream);
    if (rc) return rc;
    for (size_t g = 0; g < groups; ++g) {
        rsamd::MaskedPlan mp;
        mp.records = sl->dev + g * npat * L.bytes;
        mp.rec_stride = L.bytes;
        mp.plan_ids = reinterpret_cast<const int32_t *>(sl->dev + ids_off);
        mp.nin = k;
        mp.mslots = ms;
        mp.pattern_bytes = pattern_bytes;
        RS_HIP(rsamd::launch_gf_masked(geo, mp, stream));
    }
    RS_HIP(hipEventRecord(sl->done, stream));
    return RS_OK;
}

int decode_masked_bits_dev(const Codec &c, const uint32_t *dev_bits, const Geometry &geo, size_t pattern_bytes,
                           int32_t *dev_bad, hipStream_t stream) {
    if (!dev_bits) return fail(RS_E_INVALID, "NULL device buffer");
    rsamd::PatternTables pt;
    std::string err;
    int rc = c.pattern_tables(&pt, &err);
    if (rc) return fail(rc, err);
    return launch_pattern_groups(c, pt, geo, pattern_bytes, reinterpret_cast<const int32_t *>(dev_bits), dev_bad,
                                 stream);
}

// The packed view of a granule batch (rs_amd.h): n_stripes * shard_len / G
// stripes of G-byte shards.  RS_OK, or RS_E_INVALID for a bad shape.
int granule_view(int total_shards, uint8_t *base, size_t n_stripes, size_t shard_len, size_t granule, Geometry *geo) {
    if (granule == 0 || (shard_len % granule != 0 && granule % shard_len != 0))
        return fail(RS_E_INVALID, "shard_len " + std::to_string(shard_len) + " and the granule " +
                                      std::to_string(granule) + " must divide one another");
    if ((n_stripes * shard_len) % granule != 0)
        return fail(RS_E_INVALID, "the granule " + std::to_string(granule) + " does not divide the batch's " +
                                      std::to_string(n_stripes * shard_len) + " columns");
    *geo = Geometry{base, n_stripes * shard_len / granule, 0, granule, granule, size_t(total_shards) * granule};
    return RS_OK;
}

// rs_decode_groups_shard_major's form for flags that change every few groups
// (not the master's loop): chunks of whole groups staged through the DMA
// pipeline (host.hpp run_chunks), each chunk's slots laid out as the caller's
// arrays ([server][groups * chunk_len]) and decoded in HBM by the per-stripe
// pattern kernels, one launch group per output slot group -- the groups read
// as stripes of chunk_len-byte shards (stripe stride chunk_len).  Every group
// is checked (presence_bits) before anything is copied.  The servers with an
// absent chunk in a chunk's groups are copied back whole over those groups
// (their present chunks come back unchanged).
int groups_host_per_group(const Codec &c, const rsamd::PatternTables &pt, uint8_t *const *servers, size_t cl,
                          size_t n_groups, const uint8_t *present) {
    const int T = c.total(), k = c.k();
    MaskedSlot *sl = nullptr;
    ThreadCtx *ctx = nullptr;
    int rc = masked_slot(n_groups * sizeof(uint32_t), &sl, &ctx);
    if (rc) return rc;
    uint32_t *bits = reinterpret_cast<uint32_t *>(sl->host);
    rc = presence_bits(present, n_groups, T, k, pt.host_mask_table, bits);
    if (rc) return fail(rc, rc == RS_E_SINGULAR ? "Matrix is singular" : "Not enough shards present");
    const bool pinned = all_pinned(servers, T);
    const size_t G = std::min(n_groups, std::max<size_t>(1, chunk_bytes(n_groups * cl, T, pinned) / cl));
    const size_t n_chunks = (n_groups + G - 1) / G, ss = round_up(G * cl, 256);
    const uint32_t full = T >= 32 ? ~0u : (1u << T) - 1;
    std::vector<uint32_t> absent(n_chunks, 0);  // per chunk: servers with an absent chunk
    for (size_t g = 0; g < n_groups; ++g) absent[g / G] |= ~bits[g] & full;
    rc = upload_slot(ctx, sl, n_groups * sizeof(uint32_t), ctx->stream);
    if (rc) return rc;
    const int32_t *dbits = reinterpret_cast<const int32_t *>(sl->dev);
    auto io = [&](size_t j, std::vector<Xfer> *in, std::vector<Xfer> *out) {
        const size_t g0 = j * G, n = std::min(G, n_groups - g0);
        for (int s = 0; s < T; ++s) {
            in->push_back({servers[s] + g0 * cl, size_t(s) * ss, n * cl});
            if (absent[j] >> s & 1) out->push_back({servers[s] + g0 * cl, size_t(s) * ss, n * cl});
        }
    };
    auto code = [&](size_t j, uint8_t *buf, hipStream_t st) -> int {
        const size_t g0 = j * G, n = std::min(G, n_groups - g0);
        const Geometry geo{buf, n, 0, cl, ss, cl, T};
        return launch_pattern_groups(c, pt, geo, 0, dbits + g0, nullptr, st);
    };
    rc = run_chunks(ctx, n_chunks, ss * size_t(T), pinned, io, code);
    RS_HIP(hipEventRecord(sl->done, ctx->stream));
    return rc;
}

// Runs of consecutive chunk groups with one presence pattern (the master's
// offline set only grows, MasterImpl.java:794-806: one or a few runs), each
// with its decode plan (null: every shard present).  Every group of the runs
// found is checked (RS_E_NOT_ENOUGH / RS_E_SINGULAR); past max_runs runs the
// search stops with *per_group = true and the rest unchecked.
struct GroupRun {
    size_t g0, n;
    std::shared_ptr<const Plan> plan;
};

size_t max_group_runs(size_t bytes_per_server, int total) {
    return std::min<size_t>(4096, std::max<size_t>(8, (bytes_per_server >> 27) * size_t(total)));
}

int group_runs(const Codec &c, const uint8_t *present, size_t n_groups, size_t max_runs, std::vector<GroupRun> *runs,
               bool *per_group) {
    const int T = c.total(), k = c.k();
    const size_t rowb = size_t(T);
    *per_group = false;
    runs->clear();
    auto same_flags = [&](const uint8_t *a, const uint8_t *b) {
        for (int i = 0; i < T; ++i)
            if ((a[i] != 0) != (b[i] != 0)) return false;
        return true;
    };
    for (size_t g = 0; g < n_groups;) {
        if (runs->size() == max_runs) {
            *per_group = true;
            break;
        }
        const uint8_t *p = present + g * rowb;
        int np = 0;
        for (int i = 0; i < T; ++i) np += p[i] ? 1 : 0;
        if (np < k) return fail(RS_E_NOT_ENOUGH, "Not enough shards present");
        // Extend the run: byte-identical rows by memcmp blocks that double
        // while they match and halve when they do not (rows [g, g+n) all equal
        // row g, so rows [g+n, g+n+a) are compared with rows [g, g+a), a <= n:
        // 4 M groups cost about one pass over the flags); from the first row
        // that differs in bytes, row by row on the flags' meaning (nonzero).
        size_t n = 1, a = 1;
        bool exact = true;
        while (g + n < n_groups) {
            if (exact) {
                a = std::min(a, n_groups - g - n);
                if (std::memcmp(present + (g + n) * rowb, p, a * rowb) == 0) {
                    n += a;
                    a = n;
                } else if (a > 1) {
                    a /= 2;
                } else {
                    exact = false;
                }
            } else if (same_flags(present + (g + n) * rowb, p)) {
                ++n;
            } else {
                break;
            }
        }
        GroupRun r{g, n, nullptr};
        if (np < T) {
            int rc = c.decode_plan(p, &r.plan);
            if (rc) return fail(rc, rc == RS_E_SINGULAR ? "Matrix is singular" : "Not enough shards present");
        }
        runs->push_back(r);
        g += n;
    }
    return RS_OK;
}

// Live rs_host_alloc buffers: rs_host_free frees only these, so a foreign
// pointer, a slice of a buffer or a second free is RS_E_INVALID instead of
// undefined behaviour in the runtime.
struct HostAllocs {
    std::mutex mu;
    std::set<void *> live;
};
HostAllocs &host_allocs() {
    static HostAllocs *h = new HostAllocs;  // never destroyed: no teardown order at exit
    return *h;
}

const Codec *impl(const rs_codec *c) { return c ? c->impl : nullptr; }

// A host entry point's result, with a relocator's failed acquire (a batch
// that was not copied, copy_pool.hpp) reported as RS_E_INVALID.
int reloc_checked(int rc) {
    if (rsamd::take_relocation_failure() && rc == RS_OK) return fail(RS_E_INVALID, "relocator: acquire failed");
    return rc;
}

}  // namespace

extern "C" {

int rs_codec_create(int data_shards, int parity_shards, rs_codec **out) {
    if (!out) return fail(RS_E_INVALID, "out must not be NULL");
    Codec *c = nullptr;
    std::string err;
    int rc = Codec::create(data_shards, parity_shards, &c, &err);
    if (rc) return fail(rc, err);
    *out = new rs_codec{c};
    return RS_OK;
}

void rs_codec_destroy(rs_codec *codec) {
    if (!codec) return;
    delete codec->impl;  // frees its device plan copies, except once exit() has begun (codec.cpp free_device)
    delete codec;
}

int rs_codec_data_shard_count(const rs_codec *c) { return impl(c) ? impl(c)->k() : RS_E_INVALID; }
int rs_codec_parity_shard_count(const rs_codec *c) { return impl(c) ? impl(c)->m() : RS_E_INVALID; }
int rs_codec_total_shard_count(const rs_codec *c) { return impl(c) ? impl(c)->total() : RS_E_INVALID; }

int rs_codec_matrix(const rs_codec *c, uint8_t *out_rows) {
    if (!impl(c) || !out_rows) return fail(RS_E_INVALID, "NULL argument");
    const auto &d = impl(c)->matrix().data();
    std::memcpy(out_rows, d.data(), d.size());
    return RS_OK;
}

int rs_codec_decode_matrix(const rs_codec *c, const uint8_t *present, int nshards, int *survivors, int *missing,
                           int *n_missing, uint8_t *rows) {
    if (!impl(c) || !present || !survivors || !missing || !n_missing || !rows)
        return fail(RS_E_INVALID, "NULL argument");
    if (nshards != impl(c)->total()) return fail(RS_E_WRONG_NSHARDS, "wrong number of shards: " + std::to_string(nshards));
    std::shared_ptr<const Plan> plan;
    int rc = impl(c)->decode_plan(present, &plan);
    if (rc == RS_E_NOT_ENOUGH) return fail(rc, "Not enough shards present");
    if (rc == RS_E_SINGULAR) return fail(rc, "Matrix is singular");
    const int k = impl(c)->k();
    for (int i = 0; i < k; ++i) survivors[i] = plan->in_idx()[i];
    *n_missing = int(plan->out_idx().size());
    for (int j = 0; j < *n_missing; ++j) missing[j] = plan->out_idx()[j];
    std::memcpy(rows, plan->rows().data().data(), plan->rows().data().size());
    return RS_OK;
}

const char *rs_last_error_message(void) { return rsamd::host::last_error(); }

int rs_abi_version(void) { return RS_AMD_ABI_VERSION; }

void rs_thread_release(void) { rsamd::host::release_thread_contexts(); }

int rs_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int rs_encode_parity(const rs_codec *codec, uint8_t *const *shards, int nshards, const int64_t *shard_lens,
                     int32_t offset, int32_t byte_count) {
    return reloc_checked([&]() -> int {
        bounds::Scope bs;
        const Codec *c = impl(codec);
        if (!c) return fail(RS_E_INVALID, "codec is NULL");
        int rc = check_buffers_and_sizes(*c, shards, nshards, shard_lens, offset, byte_count);
        if (rc) return rc;
        if (byte_count == 0 || c->m() == 0) return RS_OK;
        return code_with_plan(c->encode_plan(), c->total(), shards, size_t(offset), size_t(byte_count), Mode::Code,
                              nullptr);
    }());
}

int rs_decode_missing(const rs_codec *codec, uint8_t *const *shards, int nshards, const int64_t *shard_lens,
                      const uint8_t *present, int32_t offset, int32_t byte_count) {
    return reloc_checked([&]() -> int {
        bounds::Scope bs;
        const Codec *c = impl(codec);
        if (!c) return fail(RS_E_INVALID, "codec is NULL");
        int rc = check_buffers_and_sizes(*c, shards, nshards, shard_lens, offset, byte_count);
        if (rc) return rc;
        if (!present) return fail(RS_E_INVALID, "present must not be NULL");
        int n_present = 0;
        for (int i = 0; i < c->total(); ++i) n_present += present[i] ? 1 : 0;
        if (n_present == c->total()) return RS_OK;  // ReedSolomon.java:190-194
        if (n_present < c->k()) return fail(RS_E_NOT_ENOUGH, "Not enough shards present");
        std::shared_ptr<const Plan> plan;
        rc = c->decode_plan(present, &plan);
        if (rc == RS_E_SINGULAR) return fail(rc, "Matrix is singular");
        if (rc) return fail(rc, "Not enough shards present");
        if (byte_count == 0) return RS_OK;
        return code_with_plan(*plan, c->total(), shards, size_t(offset), size_t(byte_count), Mode::Code, nullptr);
    }());
}

int rs_is_parity_correct(const rs_codec *codec, uint8_t *const *shards, int nshards, const int64_t *shard_lens,
                         int32_t first_byte, int32_t byte_count, const uint8_t *temp, int64_t temp_len,
                         int *result) {
    return reloc_checked([&]() -> int {
        bounds::Scope bs;
        const Codec *c = impl(codec);
        if (!c || !result) return fail(RS_E_INVALID, "codec and result must not be NULL");
        int rc = check_buffers_and_sizes(*c, shards, nshards, shard_lens, first_byte, byte_count);
        if (rc) return rc;
        if (temp && temp_len < int64_t(first_byte) + byte_count)
            return fail(RS_E_TEMP_TOO_SMALL, "tempBuffer is not big enough");
        if (byte_count == 0 || c->m() == 0) {
            *result = 1;
            return RS_OK;
        }
        return code_with_plan(c->verify_plan(), c->total(), shards, size_t(first_byte), size_t(byte_count),
                              Mode::Verify, result);
    }());
}

int rs_code_some_shards(const uint8_t *const *matrix_rows, const uint8_t *const *inputs, int input_count,
                        uint8_t *const *outputs, int output_count, int32_t offset, int32_t byte_count) {
    return reloc_checked([&]() -> int {
        bounds::Scope bs;
        return code_rows(matrix_rows, inputs, input_count, outputs, output_count, offset, byte_count, Mode::Code,
                         nullptr);
    }());
}

int rs_check_some_shards(const uint8_t *const *matrix_rows, const uint8_t *const *inputs, int input_count,
                         const uint8_t *const *to_check, int check_count, int32_t offset, int32_t byte_count,
                         int *result) {
    return reloc_checked([&]() -> int {
        if (!result) return fail(RS_E_INVALID, "result must not be NULL");
        bounds::Scope bs;
        return code_rows(matrix_rows, inputs, input_count, const_cast<uint8_t *const *>(to_check), check_count, offset,
                         byte_count, Mode::Verify, result);
    }());
}

int rs_encode_batch_dev(const rs_codec *codec, uint8_t *dev_base, size_t n_stripes, size_t shard_len,
                        size_t shard_stride, size_t stripe_stride, void *stream) {
    const Codec *c = impl(codec);
    if (!c || (!dev_base && n_stripes && shard_len)) return fail(RS_E_INVALID, "NULL codec or device base");
    bounds::Scope bs(stream);
    allow_batch(dev_base, n_stripes, shard_len, shard_stride, stripe_stride, c->total());
    std::vector<DevPlan> plans;
    RS_HIP(c->encode_plan().device_plans(&plans));
    Geometry g{dev_base, n_stripes, 0, shard_len, shard_stride, stripe_stride, c->total()};
    for (const DevPlan &p : plans)
        RS_HIP(rsamd::launch_gf(g, p, Mode::Code, nullptr, static_cast<hipStream_t>(stream)));
    return RS_OK;
}

int rs_decode_batch_dev(const rs_codec *codec, uint8_t *dev_base, const uint8_t *present, size_t n_stripes,
                        size_t shard_len, size_t shard_stride, size_t stripe_stride, void *stream) {
    const Codec *c = impl(codec);
    if (!c || !present || (!dev_base && n_stripes && shard_len))
        return fail(RS_E_INVALID, "NULL codec, presence pattern or device base");
    int n_present = 0;
    for (int i = 0; i < c->total(); ++i) n_present += present[i] ? 1 : 0;
    if (n_present == c->total()) return RS_OK;
    if (n_present < c->k()) return fail(RS_E_NOT_ENOUGH, "Not enough shards present");
    std::shared_ptr<const Plan> plan;
    int rc = c->decode_plan(present, &plan);
    if (rc) return fail(rc, rc == RS_E_SINGULAR ? "Matrix is singular" : "Not enough shards present");
    bounds::Scope bs(stream);
    allow_batch(dev_base, n_stripes, shard_len, shard_stride, stripe_stride, c->total());
    std::vector<DevPlan> plans;
    RS_HIP(plan->device_plans(&plans));
    Geometry g{dev_base, n_stripes, 0, shard_len, shard_stride, stripe_stride, c->total()};
    for (const DevPlan &p : plans)
        RS_HIP(rsamd::launch_gf(g, p, Mode::Code, nullptr, static_cast<hipStream_t>(stream)));
    return RS_OK;
}

int rs_decode_groups_shard_major_dev(const rs_codec *codec, uint8_t *dev_base, size_t server_stride, size_t chunk_len,
                                     size_t n_groups, const uint8_t *present, void *stream) {
    const Codec *c = impl(codec);
    if (!c) return fail(RS_E_INVALID, "codec is NULL");
    if (!present) return fail(RS_E_INVALID, "present must not be NULL");
    if (n_groups == 0 || chunk_len == 0) return RS_OK;
    if (!dev_base) return fail(RS_E_INVALID, "NULL device base");
    const int T = c->total();
    if (n_groups > SIZE_MAX / chunk_len || server_stride > SIZE_MAX / size_t(T))
        return fail(RS_E_INVALID, "n_groups * chunk_len or server_stride * total overflows");
    if (server_stride < n_groups * chunk_len)
        return fail(RS_E_INVALID, "server_stride " + std::to_string(server_stride) + " is smaller than n_groups * chunk_len");
    // Flags that change every few groups (not the master's loop) would make
    // many small launches: past max_runs runs the groups go to the per-stripe
    // pattern kernels instead, the layout read as n_groups stripes of
    // chunk_len-byte shards (stripe stride chunk_len, shard stride
    // server_stride) -- one launch, every group checked before it.  That
    // launch reads 0.53 of peak against 0.85 for runs (4 M groups, a random
    // pattern each: profiles/r4/shard_major_runs_r4zk.txt), and a run costs
    // about 15 us of launches, so runs pay while they number fewer than one
    // per ~160 MB of the batch: one per 128 MiB, at least 8.
    std::vector<GroupRun> runs;
    bool per_group = false;
    int rc0 = group_runs(*c, present, n_groups, max_group_runs(n_groups * chunk_len, T), &runs, &per_group);
    if (rc0) return rc0;
    if (per_group && n_groups > size_t(INT32_MAX)) return fail(RS_E_INVALID, "too many groups");
    int rc = need_device();
    if (rc) return rc;
    bounds::Scope bs(stream);
    allow_batch(dev_base, 1, n_groups * chunk_len, server_stride, 0, T);
    if (per_group) {
        const Geometry geo{dev_base, n_groups, 0, chunk_len, server_stride, chunk_len, T};
        return decode_masked_dev(*c, present, n_groups, geo, 0, static_cast<hipStream_t>(stream));
    }
    for (const GroupRun &r : runs) {
        if (!r.plan) continue;
        std::vector<DevPlan> plans;
        RS_HIP(r.plan->device_plans(&plans));
        // the run is ONE stripe of n * chunk_len-byte shards, server_stride apart
        Geometry g{dev_base + r.g0 * chunk_len, 1, 0, r.n * chunk_len, server_stride, server_stride * size_t(T), T};
        for (const DevPlan &p : plans)
            RS_HIP(rsamd::launch_gf(g, p, Mode::Code, nullptr, static_cast<hipStream_t>(stream)));
    }
    return RS_OK;
}

int rs_decode_groups_shard_major(const rs_codec *codec, uint8_t *const *servers, int nservers,
                                 const int64_t *server_lens, size_t chunk_len, size_t n_groups, const uint8_t *present) {
    return reloc_checked([&]() -> int {
        bounds::Scope bs;
        const Codec *c = impl(codec);
        if (!c) return fail(RS_E_INVALID, "codec is NULL");
        const int T = c->total();
        if (nservers != T) return fail(RS_E_WRONG_NSHARDS, "wrong number of shards: " + std::to_string(nservers));
        if (!servers || !server_lens || !present) return fail(RS_E_INVALID, "servers, server_lens and present must not be NULL");
        if (n_groups == 0 || chunk_len == 0) return RS_OK;
        if (n_groups > size_t(INT64_MAX) / chunk_len) return fail(RS_E_INVALID, "n_groups * chunk_len overflows");
        const size_t span = n_groups * chunk_len;
        for (int s = 0; s < T; ++s) {
            if (!servers[s]) return fail(RS_E_INVALID, "server " + std::to_string(s) + " is NULL");
            if (server_lens[s] < 0 || size_t(server_lens[s]) < span)
                return fail(RS_E_INVALID, "server " + std::to_string(s) + " holds " + std::to_string(server_lens[s]) +
                                              " bytes; n_groups * chunk_len is " + std::to_string(span));
        }
        std::vector<GroupRun> runs;
        bool per_group = false;
        int rc = group_runs(*c, present, n_groups, max_group_runs(span, T), &runs, &per_group);
        if (rc) return rc;
        rsamd::PatternTables pt;
        std::string err;
        if (per_group && c->pattern_tables(&pt, &err) != RS_OK) {  // wide codes: every run, one by one
            rc = group_runs(*c, present, n_groups, SIZE_MAX, &runs, &per_group);
            if (rc) return rc;
        }
        rc = need_device();
        if (rc) return rc;
        if (per_group) return groups_host_per_group(*c, pt, servers, chunk_len, n_groups, present);
        // each run: ONE decodeMissing of n * chunk_len-byte shards at offset g0 * chunk_len
        for (const GroupRun &r : runs) {
            if (!r.plan) continue;
            rc = code_with_plan(*r.plan, T, servers, r.g0 * chunk_len, r.n * chunk_len, Mode::Code, nullptr);
            if (rc) return rc;
        }
        return RS_OK;
    }());
}

int rs_set_relocator(const rs_relocator *r) {
    if (!r) {
        rsamd::set_thread_relocator(nullptr);
        return RS_OK;
    }
    if (r->n < 1 || !r->keys || !r->lens || !r->acquire || !r->release)
        return fail(RS_E_INVALID, "relocator: n >= 1 and keys, lens, acquire, release are required");
    rsamd::Relocator rr;
    rr.user = r->user;
    rr.n = r->n;
    rr.keys = r->keys;
    rr.lens = r->lens;
    rr.acquire = r->acquire;
    rr.release = r->release;
    rsamd::set_thread_relocator(&rr);
    return RS_OK;
}

int rs_decode_batch_masked_dev(const rs_codec *codec, uint8_t *dev_base, const uint8_t *present, size_t n_stripes,
                               size_t shard_len, size_t shard_stride, size_t stripe_stride, void *stream) {
    const Codec *c = impl(codec);
    if (!c) return fail(RS_E_INVALID, "codec is NULL");
    if (!present) return fail(RS_E_INVALID, "present must not be NULL");
    if (n_stripes == 0 || shard_len == 0) return RS_OK;
    if (!dev_base) return fail(RS_E_INVALID, "NULL device base");
    if (n_stripes > size_t(INT32_MAX)) return fail(RS_E_INVALID, "too many stripes");
    const Geometry geo{dev_base, n_stripes, 0, shard_len, shard_stride, stripe_stride, c->total()};
    bounds::Scope bs(stream);
    allow_batch(dev_base, n_stripes, shard_len, shard_stride, stripe_stride, c->total());
    return decode_masked_dev(*c, present, n_stripes, geo, 0, static_cast<hipStream_t>(stream));
}

int rs_decode_granule_masked_dev(const rs_codec *codec, uint8_t *dev_base, const uint8_t *present, size_t n_stripes,
                                 size_t shard_len, size_t granule, void *stream) {
    const Codec *c = impl(codec);
    if (!c) return fail(RS_E_INVALID, "codec is NULL");
    if (!present) return fail(RS_E_INVALID, "present must not be NULL");
    if (n_stripes == 0 || shard_len == 0) return RS_OK;
    if (!dev_base) return fail(RS_E_INVALID, "NULL device base");
    if (n_stripes > size_t(INT32_MAX)) return fail(RS_E_INVALID, "too many stripes");
    Geometry geo;
    int rc = granule_view(c->total(), dev_base, n_stripes, shard_len, granule, &geo);
    if (rc) return rc;
    bounds::Scope bs(stream);
    bounds::allow(dev_base, n_stripes * shard_len * size_t(c->total()));
    return decode_masked_dev(*c, present, n_stripes, geo, shard_len, static_cast<hipStream_t>(stream));
}

int rs_decode_batch_masked_bits_dev(const rs_codec *codec, uint8_t *dev_base, const uint32_t *dev_present_bits,
                                    size_t n_stripes, size_t shard_len, size_t shard_stride, size_t stripe_stride,
                                    int32_t *dev_bad_count, void *stream) {
    const Codec *c = impl(codec);
    if (!c) return fail(RS_E_INVALID, "codec is NULL");
    if (n_stripes == 0 || shard_len == 0) return RS_OK;
    if (!dev_base) return fail(RS_E_INVALID, "NULL device buffer");
    if (n_stripes > size_t(INT32_MAX)) return fail(RS_E_INVALID, "too many stripes");
    const Geometry geo{dev_base, n_stripes, 0, shard_len, shard_stride, stripe_stride, c->total()};
    bounds::Scope bs(stream);
    allow_batch(dev_base, n_stripes, shard_len, shard_stride, stripe_stride, c->total());
    bounds::allow(dev_present_bits, n_stripes * sizeof(uint32_t));
    bounds::allow(dev_bad_count, sizeof(int32_t));
    return decode_masked_bits_dev(*c, dev_present_bits, geo, 0, dev_bad_count, static_cast<hipStream_t>(stream));
}

int rs_decode_granule_masked_bits_dev(const rs_codec *codec, uint8_t *dev_base, const uint32_t *dev_present_bits,
                                      size_t n_stripes, size_t shard_len, size_t granule, int32_t *dev_bad_count,
                                      void *stream) {
    const Codec *c = impl(codec);
    if (!c) return fail(RS_E_INVALID, "codec is NULL");
    if (n_stripes == 0 || shard_len == 0) return RS_OK;
    if (!dev_base) return fail(RS_E_INVALID, "NULL device buffer");
    if (n_stripes > size_t(INT32_MAX)) return fail(RS_E_INVALID, "too many stripes");
    Geometry geo;
    int rc = granule_view(c->total(), dev_base, n_stripes, shard_len, granule, &geo);
    if (rc) return rc;
    bounds::Scope bs(stream);
    bounds::allow(dev_base, n_stripes * shard_len * size_t(c->total()));
    bounds::allow(dev_present_bits, n_stripes * sizeof(uint32_t));
    bounds::allow(dev_bad_count, sizeof(int32_t));
    return decode_masked_bits_dev(*c, dev_present_bits, geo, shard_len, dev_bad_count,
                                  static_cast<hipStream_t>(stream));
}

int rs_verify_batch_dev(const rs_codec *codec, const uint8_t *dev_base, size_t n_stripes, size_t shard_len,
                        size_t shard_stride, size_t stripe_stride, int *dev_mismatch, void *stream) {
    const Codec *c = impl(codec);
    if (!c || !dev_mismatch || (!dev_base && n_stripes && shard_len))
        return fail(RS_E_INVALID, "NULL codec, device base or mismatch flag");
    bounds::Scope bs(stream);
    allow_batch(dev_base, n_stripes, shard_len, shard_stride, stripe_stride, c->total());
    bounds::allow(dev_mismatch, sizeof(int));
    std::vector<DevPlan> plans;
    RS_HIP(c->verify_plan().device_plans(&plans));
    Geometry g{const_cast<uint8_t *>(dev_base), n_stripes, 0, shard_len, shard_stride, stripe_stride};
    for (const DevPlan &p : plans)
        RS_HIP(rsamd::launch_gf(g, p, Mode::Verify, dev_mismatch, static_cast<hipStream_t>(stream)));
    return RS_OK;
}

int rs_file_layout(const rs_codec *codec, int64_t file_len, int32_t block, int64_t *padded_len, int64_t *shard_len) {
    const Codec *c = impl(codec);
    if (!c || !padded_len || !shard_len) return fail(RS_E_INVALID, "NULL argument");
    return file_layout(*c, file_len, block, padded_len, shard_len);
}

int rs_file_encode_dev(const rs_codec *codec, const uint8_t *dev_file, size_t file_len, size_t block,
                       uint8_t *dev_shards, size_t shard_stride, void *stream) {
    const Codec *c = impl(codec);
    if (!c) return fail(RS_E_INVALID, "codec is NULL");
    bounds::Scope bs(stream);
    return file_encode_dev(*c, dev_file, file_len, block, dev_shards, shard_stride, static_cast<hipStream_t>(stream));
}

int rs_file_decode_dev(const rs_codec *codec, uint8_t *dev_shards, size_t shard_len, size_t shard_stride,
                       const uint8_t *present, size_t block, uint8_t *dev_file_out, size_t file_size,
                       int write_missing, void *stream) {
    const Codec *c = impl(codec);
    if (!c) return fail(RS_E_INVALID, "codec is NULL");
    bounds::Scope bs(stream);
    return file_decode_dev(*c, dev_shards, shard_len, shard_stride, present, block, dev_file_out, file_size,
                           write_missing != 0, static_cast<hipStream_t>(stream));
}

int rs_file_encode(const rs_codec *codec, const uint8_t *file, int64_t file_len, int32_t block,
                   uint8_t *const *shards_out, int nshards, const int64_t *shard_lens) {
    return reloc_checked([&]() -> int {
        bounds::Scope bs;
        const Codec *c = impl(codec);
        if (!c) return fail(RS_E_INVALID, "codec is NULL");
        int64_t padded = 0, S = 0;
        int rc = file_layout(*c, file_len, block, &padded, &S);
        if (rc) return rc;
        if (nshards != c->total()) return fail(RS_E_WRONG_NSHARDS, "wrong number of shards: " + std::to_string(nshards));
        if (!shards_out || !shard_lens || (!file && file_len)) return fail(RS_E_INVALID, "NULL argument");
        for (int i = 0; i < nshards; ++i)
            if (shard_lens[i] < S || (!shards_out[i] && S)) return fail(RS_E_INVALID, "shard " + std::to_string(i) + " is shorter than " + std::to_string(S));
        if (S == 0) return RS_OK;
        rc = need_device();
        if (rc) return rc;
        ThreadCtx *ctx = nullptr;
        rc = thread_ctx(&ctx);
        if (rc) return rc;
        const size_t blk = size_t(block);
        std::vector<const uint8_t *> bufs(shards_out, shards_out + nshards);
        bufs.push_back(file);
        const bool pinned = all_pinned(bufs.data(), int(bufs.size()));
        const bool big = file_chunks(c->k(), c->total(), size_t(S), blk, false).n > 1 || size_t(S) >= direct_min_bytes();
        bool taken = false;
        if (pinned)
            rc = file_encode_direct(*c, file, size_t(file_len), blk, shards_out, size_t(S), ctx, &taken);
        else if (big && size_t(S) >= mirror_min_bytes())
            rc = file_encode_mirrored(*c, file, size_t(file_len), blk, shards_out, size_t(S), ctx, &taken);
        else
            rc = file_encode_zc_split(*c, file, size_t(file_len), blk, shards_out, size_t(S), ctx, &taken);
        if (rc || taken) return rc;
        return file_encode_staged(*c, file, size_t(file_len), blk, shards_out, size_t(S), ctx, pinned);
    }());
}

int rs_file_decode(const rs_codec *codec, uint8_t *const *shards, int nshards, const int64_t *shard_lens,
                   const uint8_t *present, int32_t byte_cnt_in_shard, int32_t block, uint8_t *file_out,
                   int64_t file_size) {
    return reloc_checked([&]() -> int {
        bounds::Scope bs;
        const Codec *c = impl(codec);
        if (!c) return fail(RS_E_INVALID, "codec is NULL");
        if (nshards == c->total() && shards && shard_lens && present && byte_cnt_in_shard == shard_lens[0] &&
            block >= 1 && shard_lens[0] % block == 0)
            return file_decode_chunked(*c, shards, shard_lens, present, block, file_out, file_size);
        // decodeMissing(shards, shardPresent, 0, byteCntInShard)  (ReedSolomonDecoder.java:36)
        int rc = rs_decode_missing(codec, shards, nshards, shard_lens, present, 0, byte_cnt_in_shard);
        if (rc) return rc;
        // mergeShardsToFile + trimPadding (ReedSolomonDecoder.java:92-103, 62-66) over shards[0].length
        const int64_t S = shard_lens[0];
        if (block < 1 || S % block) return fail(RS_E_INVALID, "shard length " + std::to_string(S) + " is not a multiple of the block size");
        if (file_size < 0 || file_size > S * c->k()) return fail(RS_E_INVALID, "file size exceeds k * shard length");
        if (file_size == 0) return RS_OK;
        if (!file_out) return fail(RS_E_INVALID, "file_out is NULL");
        // The shards are complete now: the merge is a pure byte permutation, done
        // on the host (copy jobs, as every other host path moves caller bytes).
        std::vector<const uint8_t *> src(shards, shards + c->k());
        const std::vector<bool> every(size_t(c->k()), true);
        std::vector<rsamd::CopyJob> jobs;
        merge_jobs(c->k(), size_t(block), file_out, size_t(file_size), src.data(), every, 0, size_t(S / block), &jobs);
        if (size_t(file_size) > zc_pool_min())
            rsamd::CopyPool::get().copy(jobs);
        else
            rsamd::CopyPool::copy_here(jobs);
        return RS_OK;
    }());
}

int rs_fill_synthetic_dev(uint8_t *dev_base, int data_shards, size_t n_stripes, size_t shard_len, size_t shard_stride,
                          size_t stripe_stride, uint64_t seed, uint64_t stripe0, void *stream) {
    if (!dev_base || data_shards < 1) return fail(RS_E_INVALID, "NULL device base or data_shards < 1");
    if (shard_len % 8) return fail(RS_E_INVALID, "shard_len must be a multiple of 8");
    bounds::Scope bs(stream);
    allow_batch(dev_base, n_stripes, shard_len, shard_stride, stripe_stride, data_shards);
    RS_HIP(rsamd::launch_fill_synthetic(dev_base, data_shards, n_stripes, shard_len, shard_stride, stripe_stride,
                                        seed, stripe0, static_cast<hipStream_t>(stream)));
    return RS_OK;
}

int rs_dev_alloc(void **out, size_t bytes, int contiguous, int *got_contiguous) {
    if (!out) return fail(RS_E_INVALID, "out must not be NULL");
    *out = nullptr;
    if (got_contiguous) *got_contiguous = 0;
    int rc = need_device();
    if (rc) return rc;
    const size_t n = std::max<size_t>(bytes, 1);
    if (contiguous) {
        if (hipExtMallocWithFlags(out, n, hipDeviceMallocContiguous) == hipSuccess) {
            if (got_contiguous) *got_contiguous = 1;
            return RS_OK;
        }
        (void)hipGetLastError();  // no contiguous range of that size: plain hipMalloc
        *out = nullptr;
    }
    RS_HIP(hipMalloc(out, n));
    return RS_OK;
}

int rs_dev_free(void *ptr) {
    if (ptr) RS_HIP(hipFree(ptr));
    return RS_OK;
}

// Caller-owned pinned buffers: the same flags as the mirror slots (mapped,
// pages placed by the calling thread's NUMA policy), so shards the caller
// keeps here take the in-place direct path (all_pinned).
int rs_host_alloc(void **out, size_t bytes) {
    if (!out) return fail(RS_E_INVALID, "out must not be NULL");
    *out = nullptr;
    int rc = need_device();
    if (rc) return rc;
    RS_HIP(hipHostMalloc(out, std::max<size_t>(bytes, 1), hipHostMallocMapped | hipHostMallocNumaUser));
    HostAllocs &h = host_allocs();
    std::lock_guard<std::mutex> lock(h.mu);
    h.live.insert(*out);
    return RS_OK;
}

int rs_host_free(void *ptr) {
    if (!ptr) return RS_OK;
    {
        HostAllocs &h = host_allocs();
        std::lock_guard<std::mutex> lock(h.mu);
        if (!h.live.erase(ptr))  // a foreign pointer, an interior one (a slice), or freed twice
            return fail(RS_E_INVALID, "rs_host_free: not a live rs_host_alloc buffer");
    }
    RS_HIP(hipHostFree(ptr));
    return RS_OK;
}

int rs_check_buffers_and_sizes(const rs_codec *codec, int nshards, const int64_t *shard_lens, int64_t offset,
                               int64_t byte_count) {
    if (!codec) return fail(RS_E_INVALID, "NULL codec");
    return check_buffers_and_sizes(*codec->impl, nullptr, nshards, shard_lens, offset, byte_count, false);
}

size_t rs_shard_stride_recommended(int total_shards, size_t shard_len) {
    if (total_shards < 1 || shard_len == 0) return 0;
    if (total_shards >= 8 && shard_len >= (size_t(1) << 20)) return round_up(shard_len, 4096) + 4096;
    return round_up(shard_len, 256);
}

size_t rs_granule_recommended(int total_shards) {
    if (total_shards < 1) return 0;
    size_t g = size_t(1) << 20;
    while (g > 4096 && size_t(total_shards) * g > (size_t(512) << 10)) g >>= 1;
    return g;
}

int rs_granule_copy_shard(uint8_t *dev_base, int total_shards, size_t n_stripes, size_t shard_len, size_t granule,
                          size_t stripe, int shard, void *buf, int to_granules, void *stream) {
    if (!dev_base || !buf) return fail(RS_E_INVALID, "NULL pointer");
    if (stripe >= n_stripes)
        return fail(RS_E_INVALID, "stripe " + std::to_string(stripe) + " outside [0, " + std::to_string(n_stripes) + ")");
    if (total_shards < 1 || shard < 0 || shard >= total_shards)
        return fail(RS_E_INVALID, "shard " + std::to_string(shard) + " outside [0, " + std::to_string(total_shards) + ")");
    if (granule == 0 || shard_len == 0 || (shard_len % granule != 0 && granule % shard_len != 0))
        return fail(RS_E_INVALID, "shard_len " + std::to_string(shard_len) + " and the granule " +
                                      std::to_string(granule) + " must divide one another");
    int rc = need_device();
    if (rc) return rc;
    // batch column x of the stripe's first byte; granule row x / G, offset x % G
    const size_t x = stripe * shard_len, pitch = size_t(total_shards) * granule;
    uint8_t *g0 = dev_base + (x / granule) * pitch + size_t(shard) * granule + x % granule;
    const size_t width = std::min(shard_len, granule), rows = std::max<size_t>(1, shard_len / granule);
    const hipStream_t st = static_cast<hipStream_t>(stream);
    if (to_granules)
        RS_HIP(hipMemcpy2DAsync(g0, pitch, buf, width, width, rows, hipMemcpyDefault, st));
    else
        RS_HIP(hipMemcpy2DAsync(buf, width, g0, pitch, width, rows, hipMemcpyDefault, st));
    return RS_OK;
}

int rs_copy_dev(uint8_t *dst, const uint8_t *src, size_t n, void *stream) {
    if ((!dst || !src) && n) return fail(RS_E_INVALID, "NULL pointer");
    bounds::Scope bs(stream);
    bounds::allow(dst, n);
    bounds::allow(src, n);
    RS_HIP(rsamd::launch_copy(dst, src, n, static_cast<hipStream_t>(stream)));
    return RS_OK;
}

}  // extern "C"

#if RSAMD_BOUNDS
// Bounds-checking build only (bounds.hpp): the accesses outside every declared
// range since the last call -- count, the first one's address, bytes and site
// (translation unit * 100000 + line; 1 = kernels.hip, 2 = layout.hip).
extern "C" RS_API int rs_bounds_report(unsigned long long *count, unsigned long long *addr, unsigned long long *len,
                                unsigned *where) {
    rsamd::BoundsReport r;
    rsamd::bounds::report(&r);
    if (count) *count = r.count;
    if (addr) *addr = r.addr;
    if (len) *len = r.len;
    if (where) *where = r.where;
    return RS_OK;
}
#endif
