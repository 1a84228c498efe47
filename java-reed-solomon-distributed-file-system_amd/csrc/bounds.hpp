// bounds.hpp -- the bounds-checking build (make BOUNDS=1; never the product).
//
// Every global load and store of the kernels goes through RSAMD_G(p, n) (or a
// helper that takes the call site's line through __builtin_LINE()).  In the
// product build RSAMD_G is the identity and nothing below exists.  In the
// bounds build the C-ABI entry point that launches a kernel declares, for the
// duration of the call, the byte ranges it may touch -- the caller's batch as
// its arguments describe it (not the allocation around it), the plan tables,
// the call's staging buffers (bounds::allow) -- and each checked access tests
// [p, p + n) against them.  An access outside every range is counted, the
// first one is recorded with its site (translation unit * 100000 + line), and
// it is redirected to a scratch sink, so the run goes on without touching the
// stray address.  rs_bounds_report (bounds build only) returns and clears the
// record; tests/conftest.py checks it after every GPU test when the loaded
// library exports it.
//
// Scope: a call's kernels run between a device synchronisation before the
// ranges are set and one after, under a process-wide lock, so the table is
// exact for every kernel of the call.  Outside any call (and inside a stream
// capture, where the replay runs later) the table allows everything.
//
// Each declared range is itself checked on the host against the live
// allocation holding it (hipPointerGetAttributes / hipMemGetAddressRange):
// a range in freed memory, or one running past its allocation, is reported
// the same way (site 9000xx), so a stale plan table or a caller buffer shorter
// than its arguments say is caught even though the kernels stay inside it.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#ifndef RSAMD_BOUNDS
#define RSAMD_BOUNDS 0
#endif

namespace rsamd {

constexpr uint32_t kBoundsMax = 96;
constexpr uint32_t kBoundsAll = 0xFFFFFFFFu;  // BoundsTable::n: no checking

struct BoundsTable {
    uint32_t n = kBoundsAll;
    uint32_t pad = 0;
    uint64_t lo[kBoundsMax] = {};
    uint64_t hi[kBoundsMax] = {};
};

struct BoundsReport {
    unsigned long long count = 0;  // accesses outside every range
    unsigned long long addr = 0;   // the first one: address, bytes, site
    unsigned long long len = 0;
    unsigned int where = 0;
    unsigned int pad = 0;
};

// Per translation unit (each .hip file has its own device table).
hipError_t bounds_put_kernels(const BoundsTable &t);
hipError_t bounds_take_kernels(BoundsReport *r);
hipError_t bounds_put_layout(const BoundsTable &t);
hipError_t bounds_take_layout(BoundsReport *r);

namespace bounds {
#if RSAMD_BOUNDS
// The current call may touch [p, p + n).  check_alloc = false: the range may
// end inside the page after its allocation's last byte (whole-line reads).
void allow(const void *p, size_t n, bool check_alloc = true);
// RAII around one C-ABI call (nests: the outermost one acts).
class Scope {
public:
    explicit Scope(const void *stream = nullptr);
    ~Scope();
    Scope(const Scope &) = delete;
    Scope &operator=(const Scope &) = delete;
};
// The accesses caught since the last report (and clears them).
void report(BoundsReport *out);
#else
inline void allow(const void *, size_t, bool = true) {}
class Scope {
public:
    explicit Scope(const void * = nullptr) {}
};
#endif
}  // namespace bounds

}  // namespace rsamd

// ---- device side (the .hip translation units, which define RSAMD_TU_ID) ----
#if RSAMD_BOUNDS && defined(RSAMD_TU_ID)
namespace rsamd {
namespace dev {
static __device__ BoundsTable g_bounds;
static __device__ BoundsReport g_bounds_bad;
static __device__ __attribute__((aligned(16))) uint8_t g_bounds_sink[256];

template <class T>
__device__ __forceinline__ T *bounds_guard(T *p, uint64_t n, uint32_t line) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t cnt = g_bounds.n;
    if (cnt == kBoundsAll) return p;
    for (uint32_t i = 0; i < cnt && i < kBoundsMax; ++i)
        if (a >= g_bounds.lo[i] && a + n <= g_bounds.hi[i]) return p;
    if (atomicAdd(&g_bounds_bad.count, 1ull) == 0) {
        g_bounds_bad.addr = a;
        g_bounds_bad.len = n;
        g_bounds_bad.where = uint32_t(RSAMD_TU_ID) * 100000u + line;
    }
    return (T *)(void *)g_bounds_sink;
}
}  // namespace dev
}  // namespace rsamd
#define RSAMD_G(p, n) ::rsamd::dev::bounds_guard((p), uint64_t(n), uint32_t(__LINE__))
#define RSAMD_GL(p, n, line) ::rsamd::dev::bounds_guard((p), uint64_t(n), uint32_t(line))
// Host halves of the per-TU table (bounds_put_* / bounds_take_*).
#define RSAMD_BOUNDS_TU(suffix)                                                                       \
    namespace rsamd {                                                                                 \
    hipError_t bounds_put_##suffix(const BoundsTable &t) {                                            \
        return hipMemcpyToSymbol(HIP_SYMBOL(dev::g_bounds), &t, sizeof t);                            \
    }                                                                                                 \
    hipError_t bounds_take_##suffix(BoundsReport *r) {                                                \
        hipError_t e = hipMemcpyFromSymbol(r, HIP_SYMBOL(dev::g_bounds_bad), sizeof *r);              \
        const BoundsReport zero{};                                                                    \
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(dev::g_bounds_bad), &zero, sizeof zero); \
        return e;                                                                                     \
    }                                                                                                 \
    }
#else
#define RSAMD_G(p, n) (p)
#define RSAMD_GL(p, n, line) (p)
#define RSAMD_BOUNDS_TU(suffix)
#endif
