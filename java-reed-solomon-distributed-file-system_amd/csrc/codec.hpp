// codec.hpp -- the host-side mirror of ReedSolomon.java: generator matrix,
// encode plan, cached fused decode plans, and their device-resident copies.
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <list>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gf256.hpp"
#include "kernels.hpp"
#include "layout.hpp"

namespace rsamd {

// A coding plan: out[idx_out[p]] = XOR_i rows[p][i] * in[idx_in[i]], split into
// launch groups of at most kMaxOut outputs.  Host-only until uploaded.
class Plan {
public:
    Plan(std::vector<int> in_idx, std::vector<int> out_idx, GfMatrix rows);
    ~Plan();  // frees the device copies (hipFree synchronises the device first)
    Plan(const Plan &) = delete;
    Plan &operator=(const Plan &) = delete;
    const std::vector<int> &in_idx() const { return in_idx_; }
    const std::vector<int> &out_idx() const { return out_idx_; }
    const GfMatrix &rows() const { return rows_; }
    int groups() const { return int((out_idx_.size() + kMaxOut - 1) / kMaxOut); }

    // Per-group device plans on the calling thread's current device; uploaded
    // once per device on first use (upload(): the host waits for that copy
    // only) and then immutable.
    hipError_t device_plans(std::vector<DevPlan> *out) const;

    // The flat image uploaded for group g (exposed for per-call uploads).
    std::vector<uint8_t> image(int g) const;

    // Device image of a data-only decode plan for the fused decode-to-file
    // kernel (layout.hpp FileDecodePlan); k data shards, <= kMaxOut missing.
    hipError_t device_file_plan(int k, FileDecodePlan *out) const;

private:
    std::vector<int> in_idx_, out_idx_;
    GfMatrix rows_;
    mutable std::mutex mu_;
    mutable std::map<int, void *> dev_;       // device id -> allocation of all groups
    mutable std::map<int, void *> dev_file_;  // device id -> FileDecodePlan image
};

// Copy host -> device on a private non-blocking stream of device dev and wait
// for that copy alone (not for work queued on the caller's or the null stream).
hipError_t upload(int dev, void *dst, const void *src, size_t n);

// Device memory freed outside process teardown only: once exit() has begun the
// HIP runtime may already be gone, and the process releases everything anyway.
void free_device(int dev, void *p);
// True once exit() has begun (an atexit hook): device frees are skipped then.
bool process_exiting();
// Held by the exit hook while it sets process_exiting(): hold it around HIP
// calls made from a thread that may outlive exit() and check the flag inside.
std::mutex &exit_mutex();
// Frees p later, in a batch with other deferred frees (codec.cpp).
void free_device_deferred(int dev, void *p);
void flush_deferred_frees();

// Offsets of one group's image: tabs, then in_idx, then out_idx.
struct PlanLayout {
    size_t tabs, in_idx, out_idx, bytes;
};
PlanLayout plan_layout(int nin, int nout);
DevPlan dev_plan_at(const void *base, int nin, int nout);

// Fill one masked record (kernels.hpp MaskedRecordLayout) with output group g
// (at most ms outputs) of plan p.
void fill_masked_record(const Plan &p, int g, int ms, const MaskedRecordLayout &L, uint8_t *rec);

// Every decodable presence pattern of a code as device-resident masked
// records, looked up by presence bitmask (rs_decode_batch_masked_bits_dev).
struct PatternTables {
    const uint8_t *records = nullptr;     // groups blocks of npat records each
    size_t rec_stride = 0, npat = 0;
    const int32_t *mask_table = nullptr;       // [2^total]: pattern id, or -1 (not decodable)
    const int32_t *host_mask_table = nullptr;  // the same ids in host memory
    int groups = 0, mslots = 0;
    size_t bytes = 0;  // the device allocation: records, then mask_table
};
constexpr int kMaxPatternBits = 20;        // k + m for a bitmask table (4 MiB of ids)
constexpr size_t kMaxPatterns = 1u << 16;  // decodable patterns in one table

// Distinct decode plans a codec keeps (least recently used evicted first):
// every decodable pattern of a wide code would otherwise stay resident.
constexpr size_t kMaxDecodePlans = 4096;

class Codec {
public:
    static int create(int k, int m, Codec **out, std::string *err);
    ~Codec();  // frees the pattern tables' device memory

    int k() const { return k_; }
    int m() const { return m_; }
    int total() const { return k_ + m_; }
    const GfMatrix &matrix() const { return matrix_; }
    const Plan &encode_plan() const { return *encode_; }
    const Plan &verify_plan() const { return *encode_; }

    // Fused decode plan for a presence pattern (cached, thread-safe).  Inputs =
    // the first k present shards (ReedSolomon.java:210-223); outputs = every
    // absent shard in ascending order; rows: Dinv[j] for a missing data shard j,
    // parityRow[p] * Dinv for a missing parity shard.
    // With data_only, outputs are the absent DATA shards only (the fused
    // decode-to-file path needs no parity).  Returns 0, RS_E_NOT_ENOUGH or
    // RS_E_SINGULAR.
    int decode_plan(const uint8_t *present, std::shared_ptr<const Plan> *out, bool data_only = false) const;
    // The same plan built fresh, outside the cache.
    int make_decode_plan(const uint8_t *present, bool data_only, std::shared_ptr<const Plan> *out) const;

    // The pattern tables on the calling thread's current device, built on
    // first use (every bitmask with >= k present bits gets decode_plan's
    // record; blocking upload) and then immutable.  RS_E_INVALID when
    // k + m > kMaxPatternBits or the code has more than kMaxPatterns decodable
    // patterns (use the host-pattern call), RS_E_HIP on a HIP error.
    int pattern_tables(PatternTables *out, std::string *err) const;

private:
    Codec(int k, int m);
    int k_, m_;
    GfMatrix matrix_;
    std::unique_ptr<Plan> encode_;
    mutable std::mutex mu_;
    struct CacheEntry {
        std::shared_ptr<const Plan> plan;
        std::list<std::vector<uint8_t>>::iterator lru;
    };
    mutable std::map<std::vector<uint8_t>, CacheEntry> decode_cache_;
    mutable std::list<std::vector<uint8_t>> lru_;  // most recently used first
    mutable std::mutex pat_mu_;
    mutable std::map<int, PatternTables> patterns_;  // device id -> tables (freed by ~Codec)
    mutable std::vector<int32_t> host_mask_table_;
    mutable std::string pattern_refusal_;  // set once the code is found too wide for a table
};

}  // namespace rsamd
