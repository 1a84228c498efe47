// codec.cpp -- see codec.hpp.
#include "codec.hpp"

#include <algorithm>

#include <atomic>
#include <cstdlib>
#include <cstring>

#include "../../include/rs_amd.h"
#include "bounds.hpp"

namespace rsamd {

namespace {
std::atomic<bool> g_exiting{false};
const bool g_exit_hook = [] {
    // Under exit_mutex: a thread that makes HIP calls holding it (the reaper,
    // host.cpp) either finishes them before exit() goes on or sees the flag.
    std::atexit([] {
        std::lock_guard<std::mutex> lock(exit_mutex());
        g_exiting.store(true);
    });
    return true;
}();
}  // namespace

bool process_exiting() { return g_exiting.load(); }

std::mutex &exit_mutex() {
    static std::mutex *mu = new std::mutex;  // never destroyed: used from atexit
    return *mu;
}

hipError_t upload(int dev, void *dst, const void *src, size_t n) {
    // One non-blocking stream per device, created on first use and kept for the
    // process: the copy waits for nothing queued elsewhere (a hipMemcpy on the
    // null stream would wait for a caller's in-flight work on that stream).
    static std::mutex mu;
    static std::map<int, hipStream_t> streams;
    hipStream_t s = nullptr;
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = streams.find(dev);
        if (it == streams.end()) {
            const hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
            if (e != hipSuccess) return e;
            it = streams.emplace(dev, s).first;
        }
        s = it->second;
    }
    hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e;
}

void free_device(int dev, void *p) {
    if (!p || g_exiting.load()) return;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return;
    if (cur != dev) (void)hipSetDevice(dev);
    (void)hipFree(p);
    if (cur != dev) (void)hipSetDevice(cur);
}

namespace {
// Device copies of evicted decode plans wait here and are freed in batches:
// hipFree synchronises the whole device, so freeing each one as the LRU
// evicts it would stall the thread building a new plan on every stream's
// in-flight work, once per eviction.  A kernel still using an evicted plan is
// covered the same way (hipFree waits for it).
constexpr size_t kDeferredFreeBatch = 64;
std::mutex g_grave_mu;
std::vector<std::pair<int, void *>> g_grave;
}  // namespace

void free_device_deferred(int dev, void *p) {
    if (!p || g_exiting.load()) return;
    std::vector<std::pair<int, void *>> batch;
    {
        std::lock_guard<std::mutex> lock(g_grave_mu);
        g_grave.emplace_back(dev, p);
        if (g_grave.size() < kDeferredFreeBatch) return;
        batch.swap(g_grave);
    }
    for (auto &kv : batch) free_device(kv.first, kv.second);
}

void flush_deferred_frees() {
    std::vector<std::pair<int, void *>> batch;
    {
        std::lock_guard<std::mutex> lock(g_grave_mu);
        batch.swap(g_grave);
    }
    for (auto &kv : batch) free_device(kv.first, kv.second);
}

PlanLayout plan_layout(int nin, int nout) {
    PlanLayout l;
    l.tabs = 0;
    l.in_idx = size_t(nin) * nout * sizeof(PermTable);
    l.out_idx = l.in_idx + size_t(nin) * sizeof(int32_t);
    l.bytes = (l.out_idx + size_t(nout) * sizeof(int32_t) + 255) & ~size_t(255);
    return l;
}

DevPlan dev_plan_at(const void *base, int nin, int nout) {
    const PlanLayout l = plan_layout(nin, nout);
    const uint8_t *b = static_cast<const uint8_t *>(base);
    DevPlan p;
    p.tabs = reinterpret_cast<const uint32_t *>(b + l.tabs);
    p.in_idx = reinterpret_cast<const int32_t *>(b + l.in_idx);
    p.out_idx = reinterpret_cast<const int32_t *>(b + l.out_idx);
    p.nin = nin;
    p.nout = nout;
    return p;
}

Plan::Plan(std::vector<int> in_idx, std::vector<int> out_idx, GfMatrix rows)
    : in_idx_(std::move(in_idx)), out_idx_(std::move(out_idx)), rows_(std::move(rows)) {}

std::vector<uint8_t> Plan::image(int g) const {
    const int nin = int(in_idx_.size());
    const int p0 = g * kMaxOut;
    const int nout = std::min<int>(kMaxOut, int(out_idx_.size()) - p0);
    const PlanLayout l = plan_layout(nin, nout);
    std::vector<uint8_t> img(l.bytes, 0);
    // tabs[i][p] (input-major so one input's tables are contiguous)
    for (int i = 0; i < nin; ++i)
        for (int p = 0; p < nout; ++p) {
            const PermTable t = perm_table(rows_.at(p0 + p, i));
            std::memcpy(img.data() + l.tabs + (size_t(i) * nout + p) * sizeof(PermTable), &t, sizeof t);
        }
    for (int i = 0; i < nin; ++i) {
        const int32_t v = in_idx_[i];
        std::memcpy(img.data() + l.in_idx + i * sizeof(int32_t), &v, sizeof v);
    }
    for (int p = 0; p < nout; ++p) {
        const int32_t v = out_idx_[p0 + p];
        std::memcpy(img.data() + l.out_idx + p * sizeof(int32_t), &v, sizeof v);
    }
    return img;
}

Plan::~Plan() {
    for (auto &kv : dev_) free_device_deferred(kv.first, kv.second);
    for (auto &kv : dev_file_) free_device_deferred(kv.first, kv.second);
}

hipError_t Plan::device_plans(std::vector<DevPlan> *out) const {
    // The line-owner kernel (gf_group8_kernel) finds runs of consecutive
    // output shards off out_idx and needs it ascending; every plan the codec
    // builds is (encode: the parity rows in order; decode: the absent shards in
    // index order), and a plan that is not never reaches a kernel.
    if (!std::is_sorted(out_idx_.begin(), out_idx_.end()) ||
        std::adjacent_find(out_idx_.begin(), out_idx_.end()) != out_idx_.end())
        return hipErrorInvalidValue;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const int nin = int(in_idx_.size());
    std::lock_guard<std::mutex> lock(mu_);
    auto it = dev_.find(dev);
    std::vector<size_t> offs;
    size_t total = 0;
    for (int g = 0; g < groups(); ++g) {
        offs.push_back(total);
        total += plan_layout(nin, std::min<int>(kMaxOut, int(out_idx_.size()) - g * kMaxOut)).bytes;
    }
    if (it == dev_.end()) {
        void *buf = nullptr;
        e = hipMalloc(&buf, total ? total : 256);
        if (e != hipSuccess) return e;
        for (int g = 0; g < groups(); ++g) {
            const std::vector<uint8_t> img = image(g);
            e = upload(dev, static_cast<uint8_t *>(buf) + offs[g], img.data(), img.size());
            if (e != hipSuccess) {
                (void)hipFree(buf);
                return e;
            }
        }
        it = dev_.emplace(dev, buf).first;
    }
    bounds::allow(it->second, total ? total : 256);
    out->clear();
    for (int g = 0; g < groups(); ++g) {
        const int nout = std::min<int>(kMaxOut, int(out_idx_.size()) - g * kMaxOut);
        out->push_back(dev_plan_at(static_cast<uint8_t *>(it->second) + offs[g], nin, nout));
    }
    return hipSuccess;
}

hipError_t Plan::device_file_plan(int k, FileDecodePlan *out) const {
    const int E = int(out_idx_.size());
    if (E > kMaxOut || int(in_idx_.size()) != k) return hipErrorInvalidValue;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const size_t tabs_bytes = size_t(k) * E * sizeof(PermTable);
    std::lock_guard<std::mutex> lock(mu_);
    auto it = dev_file_.find(dev);
    if (it == dev_file_.end()) {
        std::vector<uint8_t> img(tabs_bytes + 2 * size_t(k) * sizeof(int32_t));
        for (int j = 0; j < k; ++j)
            for (int r = 0; r < E; ++r) {
                const PermTable t = perm_table(rows_.at(r, j));
                std::memcpy(img.data() + (size_t(j) * E + r) * sizeof(PermTable), &t, sizeof t);
            }
        for (int j = 0; j < k; ++j) {
            const int32_t v = in_idx_[j];
            std::memcpy(img.data() + tabs_bytes + j * sizeof(int32_t), &v, sizeof v);
        }
        for (int i = 0; i < k; ++i) {  // data shard i: survivor position, or -(row + 1)
            int32_t src = 0;
            for (int j = 0; j < k; ++j)
                if (in_idx_[j] == i) src = j;
            for (int r = 0; r < E; ++r)
                if (out_idx_[r] == i) src = -(r + 1);
            std::memcpy(img.data() + tabs_bytes + (k + i) * sizeof(int32_t), &src, sizeof src);
        }
        void *buf = nullptr;
        e = hipMalloc(&buf, img.size());
        if (e != hipSuccess) return e;
        e = upload(dev, buf, img.data(), img.size());
        if (e != hipSuccess) {
            (void)hipFree(buf);
            return e;
        }
        it = dev_file_.emplace(dev, buf).first;
    }
    const uint8_t *b = static_cast<const uint8_t *>(it->second);
    bounds::allow(b, tabs_bytes + 2 * size_t(k) * sizeof(int32_t));
    out->tabs = reinterpret_cast<const uint32_t *>(b);
    out->in_idx = reinterpret_cast<const int32_t *>(b + tabs_bytes);
    out->dsrc = reinterpret_cast<const int32_t *>(b + tabs_bytes + size_t(k) * sizeof(int32_t));
    out->n_missing_data = E;
    return hipSuccess;
}

Codec::Codec(int k, int m) : k_(k), m_(m), matrix_(build_generator(k, k + m)) {
    std::vector<int> in(k), out(m);
    for (int i = 0; i < k; ++i) in[i] = i;
    for (int p = 0; p < m; ++p) out[p] = k + p;
    std::vector<int> parity(m);
    for (int p = 0; p < m; ++p) parity[p] = k + p;
    encode_.reset(new Plan(in, out, matrix_.select_rows(parity)));  // parityRows, ReedSolomon.java:53-56
}

Codec::~Codec() {
    for (auto &kv : patterns_) free_device(kv.first, const_cast<uint8_t *>(kv.second.records));
    decode_cache_.clear();  // the plans' device copies join the deferred list ...
    encode_.reset();
    flush_deferred_frees();  // ... and go now, with every other pending one
}

int Codec::create(int k, int m, Codec **out, std::string *err) {
    if (256 < k + m) {  // ReedSolomon.java:44-46
        *err = "too many shards - max is 256";
        return RS_E_TOO_MANY_SHARDS;
    }
    if (k < 1 || m < 0) {
        *err = "shard counts must satisfy data >= 1 and parity >= 0";
        return RS_E_INVALID;
    }
    *out = new Codec(k, m);
    return RS_OK;
}

int Codec::decode_plan(const uint8_t *present, std::shared_ptr<const Plan> *out, bool data_only) const {
    std::vector<uint8_t> key(total() + 1);
    for (int i = 0; i < total(); ++i) key[i] = present[i] ? 1 : 0;
    key[total()] = data_only ? 1 : 0;
    {
        std::lock_guard<std::mutex> lock(mu_);
        auto it = decode_cache_.find(key);
        if (it != decode_cache_.end()) {
            lru_.splice(lru_.begin(), lru_, it->second.lru);
            *out = it->second.plan;
            return RS_OK;
        }
    }
    std::shared_ptr<const Plan> plan;
    const int rc = make_decode_plan(present, data_only, &plan);
    if (rc) return rc;
    std::shared_ptr<const Plan> evicted;  // destroyed after the lock is released
    std::lock_guard<std::mutex> lock(mu_);
    auto it = decode_cache_.find(key);
    if (it != decode_cache_.end()) {  // another thread built it meanwhile
        *out = it->second.plan;
        return RS_OK;
    }
    lru_.push_front(key);
    decode_cache_.emplace(key, CacheEntry{plan, lru_.begin()});
    if (decode_cache_.size() > kMaxDecodePlans) {
        auto victim = decode_cache_.find(lru_.back());
        evicted = std::move(victim->second.plan);
        decode_cache_.erase(victim);
        lru_.pop_back();
    }
    *out = plan;
    return RS_OK;
}

int Codec::make_decode_plan(const uint8_t *present, bool data_only, std::shared_ptr<const Plan> *out) const {
    std::vector<int> surv, missing;
    for (int i = 0; i < total(); ++i) {
        if (present[i] && int(surv.size()) < k_) surv.push_back(i);
        if (!present[i] && (!data_only || i < k_)) missing.push_back(i);
    }
    if (int(surv.size()) < k_) return RS_E_NOT_ENOUGH;
    GfMatrix dinv;
    if (!matrix_.select_rows(surv).invert(&dinv)) return RS_E_SINGULAR;
    // One row per missing shard over the survivors.  Java's second pass codes
    // missing parity from ALL data shards (ReedSolomon.java:259-271); every
    // present data shard is a survivor and Dinv's row for it is the unit vector
    // selecting it, so parityRow * Dinv reproduces that pass bit for bit.
    GfMatrix rows(int(missing.size()), k_);
    for (size_t r = 0; r < missing.size(); ++r) {
        const int j = missing[r];
        if (j < k_) {
            for (int c = 0; c < k_; ++c) rows.at(int(r), c) = dinv.at(j, c);
        } else {
            GfMatrix prow = matrix_.select_rows({j});
            GfMatrix fused = prow.times(dinv);
            for (int c = 0; c < k_; ++c) rows.at(int(r), c) = fused.at(0, c);
        }
    }
    *out = std::make_shared<const Plan>(surv, missing, std::move(rows));
    return RS_OK;
}

void fill_masked_record(const Plan &p, int g, int ms, const MaskedRecordLayout &L, uint8_t *rec) {
    const int k = int(p.in_idx().size());
    const int nm = int(p.out_idx().size());
    const int32_t nout = std::max(0, std::min(ms, nm - g * ms));
    std::memset(rec, 0, L.bytes);
    std::memcpy(rec, &nout, sizeof nout);
    for (int i = 0; i < k; ++i) {
        const int32_t v = p.in_idx()[i];
        std::memcpy(rec + L.in_idx + i * 4, &v, 4);
    }
    for (int q = 0; q < nout; ++q) {
        const int row = g * ms + q;
        const int32_t v = p.out_idx()[row];
        std::memcpy(rec + L.out_idx + q * 4, &v, 4);
        for (int i = 0; i < k; ++i) {
            const PermTable t = perm_table(p.rows().at(row, i));
            std::memcpy(rec + L.tabs + (size_t(i) * ms + q) * sizeof t, &t, sizeof t);
        }
    }
}

int Codec::pattern_tables(PatternTables *out, std::string *err) const {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        *err = "hipGetDevice failed";
        return RS_E_HIP;
    }
    std::lock_guard<std::mutex> lock(pat_mu_);
    auto it = patterns_.find(dev);
    if (it != patterns_.end()) {
        *out = it->second;
        bounds::allow(out->records, out->bytes);
        return RS_OK;
    }
    const int T = total();
    if (pattern_refusal_.empty() && T > kMaxPatternBits)
        pattern_refusal_ =
            "presence bitmasks need k + m <= " + std::to_string(kMaxPatternBits) + " (got " + std::to_string(T) + ")";
    const uint32_t n = T > kMaxPatternBits ? 0 : 1u << T;
    size_t npat = 0;
    for (uint32_t bits = 0; pattern_refusal_.empty() && bits < n; ++bits) npat += __builtin_popcount(bits) >= k_ ? 1 : 0;
    if (pattern_refusal_.empty() && npat > kMaxPatterns)
        pattern_refusal_ = "code has " + std::to_string(npat) + " decodable presence patterns (> " +
                           std::to_string(kMaxPatterns) + "); use rs_decode_batch_masked_dev";
    if (!pattern_refusal_.empty()) {
        *err = pattern_refusal_;
        return RS_E_INVALID;
    }
    std::vector<int32_t> table(n, -1);
    std::vector<std::shared_ptr<const Plan>> plans;
    plans.reserve(npat);
    std::vector<uint8_t> present(T);
    size_t max_missing = 0;
    for (uint32_t bits = 0; bits < n; ++bits) {
        if (__builtin_popcount(bits) < k_) continue;
        for (int i = 0; i < T; ++i) present[i] = (bits >> i) & 1;
        std::shared_ptr<const Plan> p;
        // Host-side plans only (the records are filled from them): built
        // outside the LRU, so 2^(k+m) patterns do not flush its hot plans.
        const int rc = make_decode_plan(present.data(), false, &p);
        if (rc == RS_E_SINGULAR) continue;  // stays -1: such stripes are skipped and counted
        if (rc) {
            *err = "decode plan";
            return rc;
        }
        table[bits] = int32_t(plans.size());
        max_missing = std::max(max_missing, p->out_idx().size());
        plans.push_back(std::move(p));
    }
    PatternTables t;
    t.npat = plans.size();
    t.mslots = std::max(1, std::min(m_, kMaxOut));
    t.groups = int(std::max<size_t>(1, (max_missing + t.mslots - 1) / t.mslots));
    const MaskedRecordLayout L = masked_record_layout(k_, t.mslots);
    t.rec_stride = L.bytes;
    const size_t rec_bytes = size_t(t.groups) * t.npat * L.bytes;
    std::vector<uint8_t> img(rec_bytes + size_t(n) * sizeof(int32_t));
    for (int g = 0; g < t.groups; ++g)
        for (size_t q = 0; q < t.npat; ++q) fill_masked_record(*plans[q], g, t.mslots, L, img.data() + (g * t.npat + q) * L.bytes);
    std::memcpy(img.data() + rec_bytes, table.data(), size_t(n) * sizeof(int32_t));
    void *buf = nullptr;
    if (hipMalloc(&buf, img.size()) != hipSuccess || upload(dev, buf, img.data(), img.size()) != hipSuccess) {
        if (buf) (void)hipFree(buf);
        *err = "pattern table upload failed";
        return RS_E_HIP;
    }
    if (host_mask_table_.empty()) host_mask_table_ = std::move(table);  // same ids on every device; never resized after
    t.host_mask_table = host_mask_table_.data();
    t.records = static_cast<const uint8_t *>(buf);
    t.mask_table = reinterpret_cast<const int32_t *>(static_cast<const uint8_t *>(buf) + rec_bytes);
    t.bytes = img.size();
    bounds::allow(t.records, t.bytes);
    patterns_.emplace(dev, t);
    *out = t;
    return RS_OK;
}

}  // namespace rsamd
