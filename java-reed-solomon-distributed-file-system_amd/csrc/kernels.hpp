// kernels.hpp -- launchers for the gfx950 kernels in kernels.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace rsamd {

// A device-resident coding plan for ONE launch: nout <= kMaxOut outputs, each
// the GF dot product of a coefficient row with the nin input shards.
// Device memory layout (one allocation, see Codec::device_plan):
//   uint32 tabs[nin][nout][5]   PermTable of coefficient row[p][i]
//   int32  in_idx[nin]          shard index of input i inside a stripe
//   int32  out_idx[nout]        shard index of output p inside a stripe
constexpr int kMaxOut = 4;
struct DevPlan {
    const uint32_t *tabs = nullptr;
    const int32_t *in_idx = nullptr;
    const int32_t *out_idx = nullptr;
    int nin = 0, nout = 0;
};

// Stripe-batched layout: shard s of stripe t at base + t*stripe_stride + s*shard_stride,
// bytes [col0, col0 + len) of every shard take part.
struct Geometry {
    uint8_t *base = nullptr;
    size_t n_stripes = 0;
    size_t col0 = 0;
    size_t len = 0;
    size_t shard_stride = 0;
    size_t stripe_stride = 0;
    int total = 0;  // shards per stripe (k + m) when the caller knows it, else 0
};

enum class Mode { Code, Verify };

// Codes (or, with Mode::Verify, checks into *mismatch) every stripe of g with plan p.
// Returns hipSuccess or the first launch error.
hipError_t launch_gf(const Geometry &g, const DevPlan &p, Mode mode, int *mismatch, hipStream_t s);

// Per-stripe presence patterns (rs_decode_batch_masked_dev).  records holds one
// fixed-size record per distinct pattern (masked_record_layout); plan_ids[t]
// selects stripe t's record.  A record with nout == 0 leaves its stripes alone.
struct MaskedRecordLayout {
    size_t in_idx, out_idx, tabs, bytes;  // byte offsets inside a record; nout is an int32 at 0
};
MaskedRecordLayout masked_record_layout(int nin, int mslots);

//
// With mask_table set, plan_ids[t] is instead stripe t's presence bitmask
// (bit i = shard i present) and its record is mask_table[bits] (-1: not
// decodable; bits >= 2^mask_bits is never looked up).  Such stripes are left
// alone and, when bad is set, counted there once (atomicAdd per stripe).
struct MaskedPlan {
    const uint8_t *records = nullptr;
    size_t rec_stride = 0;
    const int32_t *plan_ids = nullptr;
    int nin = 0;
    int mslots = 0;  // output slots per record (<= kMaxOut)
    const int32_t *mask_table = nullptr;
    int mask_bits = 0;
    int32_t *bad = nullptr;
    // 0: plan_ids[t] is view stripe t's.  Otherwise the Geometry is the packed
    // view of a granule batch (rs_amd.h) and plan_ids holds one entry per
    // logical stripe of pattern_bytes columns: view stripe t's column c belongs
    // to logical stripe (t * (col0 + len) + c) / pattern_bytes.
    size_t pattern_bytes = 0;
};

hipError_t launch_gf_masked(const Geometry &g, const MaskedPlan &p, hipStream_t s);

// Shards in page-locked host memory, coded in place across the link by one
// kernel (host-buffer calls, capi.cpp run_direct).  in / out are the device
// addresses of each shard's first byte (hipHostGetDevicePointer); tabs are a
// DevPlan's.  hipErrorInvalidValue when the plan is too wide or the shards'
// addresses do not share an 8-byte residue (the caller then stages).
constexpr int kMaxDirectIn = 32;
struct DirectPlan {
    const uint8_t *in[kMaxDirectIn] = {};
    uint8_t *out[kMaxOut] = {};
    const uint32_t *tabs = nullptr;
    int nin = 0, nout = 0;
};
// The file tee of a direct decode (capi.cpp file_decode_pinned): every output
// that is data shard d < k is also stored into its blocks of the client's
// file -- column c = r * blk + w of data shard d is file byte (r k + d) blk + w
// (ReedSolomonDecoder.java:92-103), clipped to the file's size -- so a rebuilt
// data shard reaches the file in the pass that writes it.  The shard
// addresses and the file's must be 8-byte aligned and blk % 8 == 0 (every
// 8-byte unit then lies in one block); the outputs start at column 0.
struct DirectTee {
    uint8_t *file = nullptr;  // device address
    uint64_t file_size = 0, blk = 0, k = 0;
    int data[kMaxOut] = {-1, -1, -1, -1};  // output q's data shard, or -1 (parity)
};
static_assert(kMaxOut == 4, "DirectTee::data initialises kMaxOut entries");
// Completion signal of a small host call (capi.cpp run_small): every block
// makes its stores visible system-wide and counts itself done on `ctr` (a
// device word, zero between calls); the last block resets it, stores the
// verify result (the device word `mismatch`, then zeroed) into flag[1] and
// `seq` into flag[0] -- coherent host memory the calling thread spins on
// instead of waiting for the stream (small calls).
struct DirectSignal {
    uint32_t *flag = nullptr;  // device address of the coherent host words
    uint32_t *ctr = nullptr;
    uint32_t seq = 0;
};
hipError_t launch_gf_direct(const DirectPlan &p, size_t n, Mode mode, int *mismatch, hipStream_t s,
                            const DirectTee *tee = nullptr, const DirectSignal *sig = nullptr);

hipError_t launch_fill_synthetic(uint8_t *base, int k, size_t n_stripes, size_t shard_len,
                                 size_t shard_stride, size_t stripe_stride, uint64_t seed,
                                 uint64_t stripe0, hipStream_t s);

hipError_t launch_copy(uint8_t *dst, const uint8_t *src, size_t n, hipStream_t s);

}  // namespace rsamd
