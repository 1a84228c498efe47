// kernels.hip -- gfx950 kernels of the Reed-Solomon engine.
//
// The one hot operation is the GF(2^8) matrix-times-shards product of
// CodingLoop.codeSomeShards (CodingLoop.java:79-85; default loop
// InputOutputByteTableCodingLoop.java:12-44):
//     out[p][b] = XOR_i mul(row[p][i], in[i][b])
// Encode (ReedSolomon.java:90-104) and decode (ReedSolomon.java:175-272, fused
// to one pass by the host, see codec.cpp) both run it; only the coefficient
// rows and the shard index lists differ.  Verification (isParityCorrect,
// ReedSolomon.java:115-164) is the same product compared instead of stored.
//
// Design:
//  * Byte-stream, HBM-bound: each input byte is read once and each output byte
//    written once -- (nin + nout) bytes per column, not the Java loop's
//    nin*nout read-modify-write passes.  16 bytes per lane per shard
//    (global_load_dwordx4 / global_store_dwordx4 with the non-temporal hint),
//    1 KiB per wave-instruction.
//  * No tables in memory on the hot path.  Multiplication by the constant c is
//    linear over GF(2), so c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6] with
//    8/8/4-entry tables that fit in 2/2/1 registers; one v_perm_b32 looks up
//    four bytes of a dword at once (gf_device.hpp).  The tables are
//    wave-uniform scalar loads and the 3*nin terms of an output are folded
//    with v_bitop3_b32 (3-input XOR, gfx950).  No MFMA (GF(2^8) is not a
//    float contraction).
//  * Work item = one wave = 64 consecutive 16-byte vectors of one stripe; a
//    one-shot grid (one block per item, 64 threads).
//  * Occupancy is capped on purpose: a launch asks for dynamic LDS it never
//    touches, so a CU holds 11-16 of these waves instead of 32 (vec_lds_pad,
//    masked_lds_pad), and capped launches run in plain block order
//    (block_order): 4+2 encode 0.836 -> 0.874 of HBM peak.
//  * Every global access goes through RSAMD_G (bounds.hpp): the identity in
//    the product, a range check in the bounds-checking build.
#define RSAMD_TU_ID 1
#include "kernels.hpp"

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdlib>

#include "gf_device.hpp"
#include "tuning.hpp"

namespace rsamd {
namespace {

using namespace dev;

constexpr int kThreads = 256;  // byte / fill / copy kernels
constexpr int kWave = 64;      // vector kernels: one wave per block
// A dispatch's grid is at most 2^32 - 1 work-items per dimension (the AQL
// packet's grid size is 32-bit), so one-shot grids of one-wave blocks are cut
// into launches of at most this many blocks.
constexpr size_t kMaxGridBlocks = size_t(UINT32_MAX) / kWave;
constexpr uint64_t kSmallBytes = 16384;  // columns below which a ragged launch uses the byte kernel alone
constexpr uint64_t kLinePeelMinBytes = uint64_t(256) << 20;  // head peel (launch_gf_tables) from this many columns
// Division by a launch-invariant divisor with a multiply-high (Granlund and
// Montgomery): q = (t + ((n - t) >> s1)) >> s2, t = mulhi(n, m), exact for all
// 32-bit n.  The block -> (stripe, chunk) map divides wave-uniform values, and
// a plain `/` compiles to a float-reciprocal sequence on the VALU (21 of the
// 4+2 encode's 288 VALU ops); this stays on the scalar unit.
struct FastDiv {
    uint32_t m, s1, s2;
};
FastDiv make_fastdiv(uint32_t d) {
    uint32_t l = 0;
    while ((uint64_t(1) << l) < d) ++l;
    return FastDiv{uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << l) - d)) / d + 1), l < 1 ? l : 1u,
                   l > 1 ? l - 1 : 0u};
}
__device__ __forceinline__ uint32_t fast_div(uint32_t n, const FastDiv &f) {
    const uint32_t t = __umulhi(n, f.m);
    return (t + ((n - t) >> f.s1)) >> f.s2;
}

struct VecArgs {
    uint8_t *base;
    const uint32_t *tabs;
    const int32_t *in_idx;
    const int32_t *out_idx;
    uint64_t stripe_stride;
    uint64_t shard_stride;
    uint32_t nvec;     // full 16-byte vectors per shard
    uint32_t chunks;   // blocks per stripe = ceil(nvec / 64)
    uint32_t n_items;  // blocks in this launch
    uint32_t rot;      // block order (block_item): chunk rotation per stripe
    uint32_t xcd_span; // block order: XCD-contiguous remap span (0 = off)
    FastDiv cdiv;      // division by chunks
    int nin;           // generic kernel only
    int *mismatch;     // Mode::Verify only
};

struct ByteArgs {
    uint8_t *base;
    const uint32_t *tabs;
    const int32_t *in_idx;
    const int32_t *out_idx;
    uint64_t stripe_stride;
    uint64_t shard_stride;
    uint64_t col0;
    uint64_t ncols;
    uint64_t total;  // n_stripes * ncols
    int nin, nout;
    int *mismatch;
};

#ifndef RSAMD_LOAD_NT
#define RSAMD_LOAD_NT 1  // A/B builds: 0 = plain loads
#endif
#ifndef RSAMD_STORE_NT
#define RSAMD_STORE_NT 1  // A/B builds: 0 = plain stores
#endif
__device__ __forceinline__ u32x4 load_stream(const uint8_t *p, uint32_t line = __builtin_LINE()) {
    p = RSAMD_GL(p, 16, line);
    if (!RSAMD_LOAD_NT) return *reinterpret_cast<const u32x4 *>(p);
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}

// Streaming store of one 16-byte vector.  RSAMD_STORE_SC1=1 (A/B builds)
// adds the sc1 bit to the non-temporal store (global_store_dwordx4 ... sc1 nt).
// The stores come after every load of the kernel, so the inline asm cannot
// upset the compiler's vmcnt bookkeeping for a later load.
#ifndef RSAMD_STORE_SC1
#define RSAMD_STORE_SC1 0
#endif
__device__ __forceinline__ void store_stream(uint8_t *p, const u32x4 &v, uint32_t line = __builtin_LINE()) {
    p = RSAMD_GL(p, 16, line);
    if (RSAMD_STORE_SC1)
        asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if (!RSAMD_STORE_NT)
        *reinterpret_cast<u32x4 *>(p) = v;
    else
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
}

template <bool VERIFY>
__device__ __forceinline__ void emit(uint8_t *p, const u32x4 &v, int *mismatch, uint32_t line = __builtin_LINE()) {
    if (VERIFY) {
        const u32x4 have = load_stream(p, line);
        if (have[0] != v[0] || have[1] != v[1] || have[2] != v[2] || have[3] != v[3]) flag_mismatch(mismatch);
    } else {
        store_stream(p, v, line);
    }
}

// Block -> (stripe, chunk) of the one-shot grids.  Stripe-major: the blocks
// of one stripe are its consecutive 1 KiB column chunks, with two
// refinements whose use block_order() picks per geometry from measurements:
//  * rot != 0: each stripe's chunk order is rotated by rot * stripe, so the
//    stripes in flight no longer start at the same offsets modulo the shard
//    stride;
//  * xcd_span != 0: over the first 8 * xcd_span blocks, XCD x (which gets
//    every 8th block) walks items [x * xcd_span, (x+1) * xcd_span), one
//    contiguous range per XCD instead of every 8th chunk.
// Both are bijections on [0, n_items); blocks past 8 * xcd_span keep the
// identity map.
__device__ __forceinline__ void block_item(uint32_t chunks, const FastDiv &cdiv, uint32_t rot, uint32_t xcd_span,
                                           uint32_t &stripe, uint32_t &chunk) {
    uint32_t b = blockIdx.x;
    if (xcd_span && b < 8u * xcd_span) b = (b & 7u) * xcd_span + (b >> 3);
    stripe = fast_div(b, cdiv);
    chunk = b - stripe * chunks;
    if (rot) {  // stripe * rot < n_items: fits 32 bits
        const uint32_t p = stripe * rot;
        chunk += p - fast_div(p, cdiv) * chunks;
        if (chunk >= chunks) chunk -= chunks;
    }
}

// The staged coding loop of gf_vec_kernel and gf_masked_kernel, as a macro
// so each kernel keeps it inline in its own body (moved into a device
// function behind the kernel's early exits, the same code was scheduled with
// every table load hoisted: 146 VGPRs and 3 waves per SIMD at 10+4).
//
// Input vectors: K <= 4 loads all K up front.  Wide codes load AHEAD of them
// up front and the rest two at a time, as each input pair is folded in and its
// registers free up.  The tables are staged one input (pair) at a time: the
// M*5 dwords of the next input are fetched while the current one is folded
// in, and sched_barrier stops the scheduler from hoisting all K*M*5 of them,
// which overflows the SGPR file at 10+4 (it spills into VGPR lanes: 3x
// slower).  For K <= 4 the terms are folded in pairs across inputs
// (fold_terms: 1.5 v_bitop3_b32 per input and output dword instead of 2); the
// carried term costs M*4 VGPRs, so wider codes fold each input alone.
//   in: sb, TABS, IN_IDX, OUT_IDX, SHARD_STRIDE, AHEAD; out: out_off[M], acc[M] (u32x4)
//
// gf_vec_kernel<10,4> with all 10 loads up front needs 72 VGPRs (7 waves per
// SIMD); with 5 ahead and a budget of 8 waves it needs 62, unspilled.  On one
// pool, alternating builds (tools/lib_ab_same.py, profiles/r2/lib_ab_same_r2ak.txt
// and r2al): 10+4 x 128 encode +0.4-1.0, decode +0.9-1.4, verify +1.2-1.9,
// x 1024 +0.3 points of peak; 4+2 unchanged (same code).  gf_masked_kernel keeps
// all loads up front at 7 waves (its comment).  Raising wave priority while
// loads issue (s_setprio 3) cost 2-9 points; s_sleep before the stores was
// neutral (lib_ab_same_r2ai.txt).
#ifndef RSAMD_VEC_WAVES
#define RSAMD_VEC_WAVES 8  // gf_vec_kernel register budget, waves per SIMD (A/B builds: make KDEFS=...)
#endif
#ifndef RSAMD_VEC_AHEAD
#define RSAMD_VEC_AHEAD 5  // gf_vec_kernel, wide codes: inputs loaded before the first fold
#endif
// The pair loop loads input i+q+AHEAD after folding the pair at i; with
// AHEAD < 2 input i+1 would be read before it is loaded.
static_assert(RSAMD_VEC_AHEAD >= 2, "RSAMD_VEC_AHEAD must be >= 2");
// Per output count (A/B builds, profiles/r3/ahead_ab_r3zh.txt, 10+4 x 4 MiB x 128, one
// pool): one output (a single lost shard) reads 0.749 in the granule view at 5 ahead,
// 0.740-0.742 at 2 or 4, 0.73 with all 10 up front; two outputs with all 10 up front
// gain 0.8 points in the granule view and lose 0.8 packed.  Both stay at 5.
#ifndef RSAMD_VEC_AHEAD_M1
#define RSAMD_VEC_AHEAD_M1 RSAMD_VEC_AHEAD  // ... for one output (A/B)
#endif
#ifndef RSAMD_VEC_AHEAD_M2
#define RSAMD_VEC_AHEAD_M2 RSAMD_VEC_AHEAD  // ... for two outputs (A/B; >= K: all up front)
#endif
static_assert(RSAMD_VEC_AHEAD_M1 >= 2 && RSAMD_VEC_AHEAD_M2 >= 2, "lookahead must be >= 2");
#ifndef RSAMD_MASKED_WAVES
#define RSAMD_MASKED_WAVES 7  // gf_masked_kernel: see the comment on it
#endif
#define RSAMD_CODE_VECTORS(K, M, TABS, IN_IDX, OUT_IDX, SHARD_STRIDE, AHEAD)                              \
    constexpr bool kCarry = (K) <= 4;                                                                     \
    uint64_t out_off[M]; /* read before any store so these stay scalar loads */                          \
    _Pragma("unroll") for (int p = 0; p < (M); ++p) out_off[p] = uint64_t((OUT_IDX)[p]) * (SHARD_STRIDE); \
    constexpr int kAhead = kCarry ? (K) : ((K) < (AHEAD) ? (K) : (AHEAD));                                \
    u32x4 x[K];                                                                                           \
    _Pragma("unroll") for (int i = 0; i < kAhead; ++i) x[i] = load_stream(sb + uint64_t((IN_IDX)[i]) * (SHARD_STRIDE)); \
    uint32_t fa[M][4];                                                                                    \
    if (kCarry) {                                                                                         \
        uint32_t Tc[M][5], fc[M][4];                                                                      \
        _Pragma("unroll") for (int p = 0; p < (M); ++p)                                                   \
            _Pragma("unroll") for (int j = 0; j < 5; ++j) Tc[p][j] = (TABS)[p * 5 + j];                   \
        _Pragma("unroll") for (int i = 0; i < (K); ++i) {                                                 \
            uint32_t Tn[M][5];                                                                            \
            if (i + 1 < (K)) {                                                                            \
                _Pragma("unroll") for (int p = 0; p < (M); ++p)                                           \
                    _Pragma("unroll") for (int j = 0; j < 5; ++j) Tn[p][j] = (TABS)[((i + 1) * (M) + p) * 5 + j]; \
            }                                                                                             \
            _Pragma("unroll") for (int w = 0; w < 4; ++w) {                                               \
                const Sel s = selectors(x[i][w]);                                                         \
                _Pragma("unroll") for (int p = 0; p < (M); ++p) {                                         \
                    uint32_t t0, t1, t2;                                                                  \
                    terms(Tc[p], s, t0, t1, t2);                                                          \
                    fold_terms(i, fa[p][w], fc[p][w], t0, t1, t2);                                        \
                }                                                                                         \
            }                                                                                             \
            __builtin_amdgcn_sched_barrier(0);                                                            \
            if (i + 1 < (K)) {                                                                            \
                _Pragma("unroll") for (int p = 0; p < (M); ++p)                                           \
                    _Pragma("unroll") for (int j = 0; j < 5; ++j) Tc[p][j] = Tn[p][j];                    \
            }                                                                                             \
        }                                                                                                 \
        _Pragma("unroll") for (int p = 0; p < (M); ++p)                                                   \
            _Pragma("unroll") for (int w = 0; w < 4; ++w) fa[p][w] = fold_end((K), fa[p][w], fc[p][w]);   \
    } else {                                                                                              \
        /* wide codes: inputs in pairs, both tables loaded at the top of the pair */                      \
        _Pragma("unroll") for (int i = 0; i < (K); i += 2) {                                              \
            const int n2 = (i + 1 < (K)) ? 2 : 1;                                                         \
            uint32_t T2[2][M][5];                                                                         \
            _Pragma("unroll") for (int q = 0; q < 2; ++q)                                                 \
                if (q < n2)                                                                               \
                    _Pragma("unroll") for (int p = 0; p < (M); ++p)                                       \
                        _Pragma("unroll") for (int j = 0; j < 5; ++j) T2[q][p][j] = (TABS)[((i + q) * (M) + p) * 5 + j]; \
            _Pragma("unroll") for (int w = 0; w < 4; ++w) {                                               \
                const Sel s0 = selectors(x[i][w]);                                                        \
                const Sel s1 = selectors(x[n2 == 2 ? i + 1 : i][w]);                                      \
                _Pragma("unroll") for (int p = 0; p < (M); ++p) {                                         \
                    uint32_t t0, t1, t2;                                                                  \
                    terms(T2[0][p], s0, t0, t1, t2);                                                      \
                    if (n2 == 2) {                                                                        \
                        uint32_t u0, u1, u2;                                                              \
                        terms(T2[1][p], s1, u0, u1, u2);                                                  \
                        const uint32_t h = i == 0 ? xor3(t0, t1, t2) : xor3(xor3(fa[p][w], t0, t1), t2, u0); \
                        fa[p][w] = i == 0 ? xor3(h, u0, u1) ^ u2 : xor3(h, u1, u2);                       \
                    } else {                                                                              \
                        fa[p][w] = i == 0 ? xor3(t0, t1, t2) : xor3(fa[p][w], t0, t1) ^ t2;              \
                    }                                                                                     \
                }                                                                                         \
            }                                                                                             \
            /* the pair's registers are free: load the inputs kAhead further on */                         \
            _Pragma("unroll") for (int q = 0; q < 2; ++q)                                                 \
                if (i + q + kAhead < (K) && q < n2)                                                       \
                    x[i + q + kAhead] = load_stream(sb + uint64_t((IN_IDX)[i + q + kAhead]) * (SHARD_STRIDE)); \
            __builtin_amdgcn_sched_barrier(0);                                                            \
        }                                                                                                 \
    }                                                                                                     \
    u32x4 acc[M];                                                                                         \
    _Pragma("unroll") for (int p = 0; p < (M); ++p)                                                       \
        _Pragma("unroll") for (int w = 0; w < 4; ++w) acc[p][w] = fa[p][w];

// ---------------------------------------------------------------------------
// Vector kernel, compile-time shape: K inputs, M outputs.
// Block = one wave = 64 consecutive 16-byte vectors of every shard of one
// stripe: the 64-thread, one-vector-per-lane, non-temporal, one-shot-grid
// shape measured fastest on MI355X (tools/kbench.hip).
// With no grid-stride loop nothing stored by the launch can alias the
// coefficient tables, so every table load is a scalar load.
// ---------------------------------------------------------------------------
template <int K, int M, bool VERIFY>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(RSAMD_VEC_WAVES, 8))) gf_vec_kernel(VecArgs a) {
    if (VERIFY && mismatch_seen(a.mismatch)) return;
    uint32_t stripe, chunk;
    block_item(a.chunks, a.cdiv, a.rot, a.xcd_span, stripe, chunk);
    const uint32_t v = chunk * uint32_t(kWave) + threadIdx.x;
    if (v >= a.nvec) return;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(v) * 16;
    const uint32_t *tabs = RSAMD_G(a.tabs, K * M * 20);
    const int32_t *in_idx = RSAMD_G(a.in_idx, K * 4), *out_idx = RSAMD_G(a.out_idx, M * 4);
    RSAMD_CODE_VECTORS(K, M, tabs, in_idx, out_idx, a.shard_stride,
                       M == 1 ? RSAMD_VEC_AHEAD_M1 : M == 2 ? RSAMD_VEC_AHEAD_M2 : RSAMD_VEC_AHEAD)
    if (VERIFY) {  // as in gf_masked_kernel: keep the compares' inputs from being sunk
#pragma unroll
        for (int p = 0; p < M; ++p) asm volatile("" : "+v"(acc[p]));
    }
#pragma unroll
    for (int p = 0; p < M; ++p) emit<VERIFY>(sb + out_off[p], acc[p], a.mismatch);
}

// ---------------------------------------------------------------------------
// Vector kernel, runtime input count (any k), M outputs.  Inputs go in groups
// of RSAMD_GEN_GROUP, software-pipelined: group g+1's loads are issued before
// group g is folded in, so a wave keeps up to 2 * RSAMD_GEN_GROUP input
// vectors in flight (the compiled shapes load theirs up front or 5 ahead).
// Every group condition is wave-uniform.
// ---------------------------------------------------------------------------
#ifndef RSAMD_GEN_GROUP
#define RSAMD_GEN_GROUP 4  // A/B builds: 1 = one input ahead (the round-2 form)
#endif
template <int M, bool VERIFY>
__global__ void __launch_bounds__(kWave) gf_vec_generic_kernel(VecArgs a) {
    if (VERIFY && mismatch_seen(a.mismatch)) return;
    uint32_t stripe, chunk;
    block_item(a.chunks, a.cdiv, a.rot, a.xcd_span, stripe, chunk);
    const uint32_t v = chunk * uint32_t(kWave) + threadIdx.x;
    if (v >= a.nvec) return;
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(v) * 16;
    constexpr int G = RSAMD_GEN_GROUP;
    const int nin = a.nin;
    const uint32_t *tabs = RSAMD_G(a.tabs, nin * M * 20);
    const int32_t *in_idx = RSAMD_G(a.in_idx, nin * 4), *out_idx = RSAMD_G(a.out_idx, M * 4);
    uint64_t out_off[M];
#pragma unroll
    for (int p = 0; p < M; ++p) out_off[p] = uint64_t(out_idx[p]) * a.shard_stride;
    u32x4 acc[M];
#pragma unroll
    for (int p = 0; p < M; ++p) acc[p] = u32x4{0, 0, 0, 0};
    u32x4 cur[G];
#pragma unroll
    for (int q = 0; q < G; ++q)
        if (q < nin) cur[q] = load_stream(sb + uint64_t(in_idx[q]) * a.shard_stride);
    for (int i0 = 0; i0 < nin; i0 += G) {
        u32x4 nxt[G];
#pragma unroll
        for (int q = 0; q < G; ++q)
            if (i0 + G + q < nin) nxt[q] = load_stream(sb + uint64_t(in_idx[i0 + G + q]) * a.shard_stride);
#pragma unroll
        for (int q = 0; q < G; ++q) {
            if (i0 + q >= nin) break;
            uint32_t T[M][5];
#pragma unroll
            for (int p = 0; p < M; ++p)
#pragma unroll
                for (int j = 0; j < 5; ++j) T[p][j] = tabs[((i0 + q) * M + p) * 5 + j];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const Sel s = selectors(cur[q][w]);
#pragma unroll
                for (int p = 0; p < M; ++p) {
                    uint32_t t0, t1, t2;
                    terms(T[p], s, t0, t1, t2);
                    acc[p][w] = xor3(acc[p][w], t0, t1) ^ t2;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < G; ++q)
            if (i0 + G + q < nin) cur[q] = nxt[q];
    }
#pragma unroll
    for (int p = 0; p < M; ++p) emit<VERIFY>(sb + out_off[p], acc[p], a.mismatch);
}

// ---------------------------------------------------------------------------
// Masked vector kernel: the coding plan is chosen PER STRIPE from a table of
// records (one per distinct presence pattern).  The record index, shard
// indices, output count and tables are block-uniform scalar loads; stripes
// whose record has nout == 0 return at once.  Same wave shape as
// gf_vec_kernel; up to MS outputs per launch.
// ---------------------------------------------------------------------------
struct MaskedArgs {
    uint8_t *base;
    const uint8_t *records;
    uint64_t rec_stride;
    const int32_t *plan_ids;
    uint64_t stripe_stride;
    uint64_t shard_stride;
    uint32_t nvec, chunks, n_items;
    uint32_t rot, xcd_span;                      // block order (block_item)
    FastDiv cdiv;                                // division by chunks
    uint32_t rec_in_idx, rec_out_idx, rec_tabs;  // byte offsets inside a record
    int nin;                                     // generic kernel only
    const int32_t *mask_table;                   // MaskedPlan::mask_table
    int mask_bits;
    int32_t *bad;
    // Patterns per logical stripe of a granule batch (MaskedPlan::pattern_bytes):
    // pat_on != 0 -> the block's pattern is plan_ids[(pat_chunk0 + stripe *
    // chunks + chunk) / pdiv], its 1 KiB column chunk counted along the batch's
    // byte columns; plan_ids is then not offset per launch.
    uint32_t pat_on, pat_chunk0;
    FastDiv pdiv;
    uint32_t pat_chunks;  // 1 KiB chunks per logical stripe (pdiv's divisor)
};

// The plan index of the block at (stripe, chunk) and whether it holds the
// first column of that pattern's stripe (the one that counts an undecodable
// stripe).  Block-uniform scalar work.
template <bool PAT>
__device__ __forceinline__ uint32_t masked_pattern(const MaskedArgs &a, uint32_t stripe, uint32_t chunk, bool &first) {
    if (!PAT) {
        first = chunk == 0;
        return stripe;
    }
    const uint32_t x = a.pat_chunk0 + stripe * a.chunks + chunk;
    const uint32_t t = fast_div(x, a.pdiv);
    first = x == t * a.pat_chunks;
    return t;
}

// Stripe t's record, or nullptr when its presence bitmask is not decodable.
// No side effects: the caller counts an undecodable stripe (count_undecodable)
// on the path that returns.  A store that could reach the record loads would
// make the compiler read the record -- tables included -- with per-lane
// vector loads instead of scalar loads (97 VGPRs and 4 waves per SIMD for
// 4+2, 256 VGPRs and 1 wave for 10+4).
__device__ __forceinline__ const uint8_t *masked_record(const uint8_t *records, uint64_t rec_stride,
                                                        const int32_t *plan_ids, const int32_t *mask_table,
                                                        int mask_bits, uint64_t t) {
    int32_t id = *RSAMD_G(plan_ids + t, 4);
    if (mask_table) {
        const uint32_t bits = uint32_t(id);
        id = (bits >> mask_bits) ? -1 : *RSAMD_G(mask_table + bits, 4);
        if (id < 0) return nullptr;
    }
    return RSAMD_G(records + uint64_t(id) * rec_stride, rec_stride);
}

// One count per undecodable stripe: by the thread that owns its column 0.
__device__ __forceinline__ void count_undecodable(int32_t *bad, bool col0) {
    if (bad && col0) atomicAdd(RSAMD_G(bad, 4), 1);
}

// Register budget for 7 waves per SIMD (72 VGPRs).  At 10+4 the kernel needs
// 73 and ran at 6 waves, about 1.5 points under an XOR reference of its own
// access pattern; at 72 it spills 5 dwords per lane (20 B of scratch) and runs
// at or above that reference, 0.744-0.750 against 0.735-0.745 for the uniform
// decode on the same pool (tools/masked_ref_probe.py,
// profiles/r2/masked_ref_r2af.txt).  The same budget on gf_vec_kernel<10,4>
// (8 waves, 56 B spilled) cost 9 points (masked_ref_r2ae.txt).
template <int K, int MS, bool PAT>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(RSAMD_MASKED_WAVES, 8))) gf_masked_kernel(MaskedArgs a) {
    uint32_t stripe, chunk;
    block_item(a.chunks, a.cdiv, a.rot, a.xcd_span, stripe, chunk);
    const uint32_t v = chunk * uint32_t(kWave) + threadIdx.x;
    bool first = v == 0;
    uint32_t pat = stripe;
    if constexpr (PAT) pat = masked_pattern<PAT>(a, stripe, chunk, first);
    const uint8_t *rec = masked_record(a.records, a.rec_stride, a.plan_ids, a.mask_table, a.mask_bits, pat);
    if (!rec) {
        count_undecodable(a.bad, first && (PAT ? threadIdx.x == 0 : true));
        return;
    }
    const int nout = *reinterpret_cast<const int32_t *>(rec);
    if (nout == 0 || v >= a.nvec) return;
    const int32_t *in_idx = reinterpret_cast<const int32_t *>(rec + a.rec_in_idx);
    const int32_t *out_idx = reinterpret_cast<const int32_t *>(rec + a.rec_out_idx);
    const uint32_t *tabs = reinterpret_cast<const uint32_t *>(rec + a.rec_tabs);
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(v) * 16;
    RSAMD_CODE_VECTORS(K, MS, tabs, in_idx, out_idx, a.shard_stride, K)
    // Pin the accumulators before the stores: their only uses are the
    // `p < nout` stores, and without this LLVM sinks each output's whole
    // perm/fold chain into its store block, past every table stage, so all
    // K*MS*5 table dwords are live at once (10+4: 106 SGPRs, spilled into
    // VGPR lanes, 154 VGPRs, 0.40 of peak; pinned: 73 VGPRs, no spill).
#pragma unroll
    for (int p = 0; p < MS; ++p) asm volatile("" : "+v"(acc[p]));
#pragma unroll
    for (int p = 0; p < MS; ++p)
        if (p < nout) store_stream(sb + out_off[p], acc[p]);
}

template <int MS, bool PAT>
__global__ void __launch_bounds__(kWave) gf_masked_generic_kernel(MaskedArgs a) {
    uint32_t stripe, chunk;
    block_item(a.chunks, a.cdiv, a.rot, a.xcd_span, stripe, chunk);
    const uint32_t v = chunk * uint32_t(kWave) + threadIdx.x;
    const uint8_t *rec;
    if constexpr (PAT) {
        bool first;
        const uint32_t pat = masked_pattern<PAT>(a, stripe, chunk, first);
        rec = masked_record(a.records, a.rec_stride, a.plan_ids, a.mask_table, a.mask_bits, pat);
        if (!rec) {
            count_undecodable(a.bad, first && threadIdx.x == 0);
            return;
        }
    } else {
        rec = masked_record(a.records, a.rec_stride, a.plan_ids, a.mask_table, a.mask_bits, stripe);
        if (!rec) {
            count_undecodable(a.bad, v == 0);
            return;
        }
    }
    const int nout = *reinterpret_cast<const int32_t *>(rec);
    if (nout == 0 || v >= a.nvec) return;
    const int32_t *in_idx = reinterpret_cast<const int32_t *>(rec + a.rec_in_idx);
    const int32_t *out_idx = reinterpret_cast<const int32_t *>(rec + a.rec_out_idx);
    const uint32_t *tabs = reinterpret_cast<const uint32_t *>(rec + a.rec_tabs);
    uint8_t *sb = a.base + uint64_t(stripe) * a.stripe_stride + uint64_t(v) * 16;
    uint64_t out_off[MS];
#pragma unroll
    for (int p = 0; p < MS; ++p) out_off[p] = uint64_t(out_idx[p]) * a.shard_stride;
    u32x4 acc[MS];
#pragma unroll
    for (int p = 0; p < MS; ++p) acc[p] = u32x4{0, 0, 0, 0};
    // inputs in pipelined groups, as gf_vec_generic_kernel
    constexpr int G = RSAMD_GEN_GROUP;
    const int nin = a.nin;
    u32x4 cur[G];
#pragma unroll
    for (int q = 0; q < G; ++q)
        if (q < nin) cur[q] = load_stream(sb + uint64_t(in_idx[q]) * a.shard_stride);
    for (int i0 = 0; i0 < nin; i0 += G) {
        u32x4 nxt[G];
#pragma unroll
        for (int q = 0; q < G; ++q)
            if (i0 + G + q < nin) nxt[q] = load_stream(sb + uint64_t(in_idx[i0 + G + q]) * a.shard_stride);
#pragma unroll
        for (int q = 0; q < G; ++q) {
            if (i0 + q >= nin) break;
            uint32_t T[MS][5];
#pragma unroll
            for (int p = 0; p < MS; ++p)
#pragma unroll
                for (int j = 0; j < 5; ++j) T[p][j] = tabs[((i0 + q) * MS + p) * 5 + j];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const Sel s = selectors(cur[q][w]);
#pragma unroll
                for (int p = 0; p < MS; ++p) {
                    uint32_t t0, t1, t2;
                    terms(T[p], s, t0, t1, t2);
                    acc[p][w] = xor3(acc[p][w], t0, t1) ^ t2;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < G; ++q)
            if (i0 + G + q < nin) cur[q] = nxt[q];
    }
#pragma unroll
    for (int p = 0; p < MS; ++p)
        if (p < nout) store_stream(sb + out_off[p], acc[p]);
}

// 8-byte-aligned kernels: batches whose base and strides are multiples of 8
// but not of 16 -- the DFS's 1000-byte chunk groups packed back to back
// (ChunkserverDiskRecoveryMachine.java:34-48, MasterImpl.java:794-839), and
// shards below 16 KiB whose length leaves an 8-byte tail (small_with_tail8).
// The built form: every lane codes one 8-byte vector (W = 2), 125 lanes per
// 1000-byte shard, two waves per stripe.  The A/B form (U16): a lane codes a
// 16-byte vector at an 8-byte-aligned address (W = 4, global_load_dwordx4)
// and the shard's last half vector takes W = 2: 62 + 1 lanes, one wave per
// stripe.  K > 0 issues all K loads before the first fold; K == 0 (runtime
// k) loads input by input.  a.nvec counts lanes' vectors.
//
// Measured on 4 M chunk groups of 4+2 x 1000 B packed back to back
// (tools/chunk_group_probe.py; profiles/r2/chunk_groups_r2bi.txt, cg_ab_r2bk.txt):
// 8-byte form encode / decode 0.590 / 0.590 of peak, per-group bitmasks
// 0.604-0.605; 16-byte form 0.51-0.60 / 0.50-0.60 and 0.556 (it needs 65
// VGPRs: capped at 8 waves it spills, at 7 it ran 0.513); the byte kernel
// they replace 0.049 and 0.042.  An XOR reference of the same access pattern
// reads 0.486 (8-byte) and 0.420 (16-byte) and its write-only half 0.325
// (tools/group_mem.hip, profiles/r2/group_mem_r2bk.txt): the 1000-byte write
// runs set the rate.  With 1 KiB slots (stride 1024) the same kernels run
// 0.71-0.73 (chunk_groups_r2bm.txt).  Plain (temporal) stores, which could let
// L2 merge the halves of a line two waves write, cost 10-14 points at either
// stride (profiles/r2/ab/cg_st8_r2cb.txt).  Both families take the 8-byte form
// (RSAMD_VEC8_U16 / RSAMD_MASKED8_U16 = 1 for A/B builds).
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4a8 __attribute__((ext_vector_type(4), aligned(8)));
#ifndef RSAMD_VEC8_U16
#define RSAMD_VEC8_U16 0
#endif
#ifndef RSAMD_MASKED8_U16
#define RSAMD_MASKED8_U16 0
#endif

template <int W>
struct Vec8;
template <>
struct Vec8<2> {
    typedef u32x2 T;
};
template <>
struct Vec8<4> {
    typedef u32x4a8 T;
};

template <int W>
__device__ __forceinline__ typename Vec8<W>::T load8(const uint8_t *p, uint32_t line = __builtin_LINE()) {
    return __builtin_nontemporal_load(reinterpret_cast<const typename Vec8<W>::T *>(RSAMD_GL(p, W * 4, line)));
}

// sb: the lane's vector in shard 0 of its stripe; tabs[nin][MS][5].  With
// W = 4 and half set, the lane's vector is only its low 8 bytes (a shard's
// last half vector): it loads and stores 8 bytes and codes zeros above them,
// so every lane runs the same fold.
template <int W, int K, int MS, bool VERIFY>
__device__ __forceinline__ void code8(uint8_t *sb, bool half, const uint32_t *tabs, const int32_t *in_idx,
                                      const int32_t *out_idx, int nin, int nout, uint64_t shard_stride,
                                      int *mismatch) {
    typedef typename Vec8<W>::T V;
    auto ld = [&](const uint8_t *p) -> V {
        if (W == 4 && half) {
            const u32x2 h = load8<2>(p);
            V x;
            x[0] = h[0];
            x[1] = h[1];
#pragma unroll
            for (int w = 2; w < W; ++w) x[w] = 0;
            return x;
        }
        return load8<W>(p);
    };
    uint64_t out_off[MS];
#pragma unroll
    for (int p = 0; p < MS; ++p) out_off[p] = uint64_t(out_idx[p]) * shard_stride;
    uint32_t acc[MS][W];
    auto fold = [&](int i, const V &x) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const Sel sl = selectors(x[w]);
#pragma unroll
            for (int p = 0; p < MS; ++p) {
                uint32_t t0, t1, t2;
                terms(tabs + (i * MS + p) * 5, sl, t0, t1, t2);
                acc[p][w] = i == 0 ? xor3(t0, t1, t2) : xor3(acc[p][w], t0, t1) ^ t2;
            }
        }
    };
    if constexpr (K > 0) {
        V x[K];
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = ld(sb + uint64_t(in_idx[i]) * shard_stride);
#pragma unroll
        for (int i = 0; i < K; ++i) fold(i, x[i]);
    } else {
        for (int i = 0; i < nin; ++i) fold(i, ld(sb + uint64_t(in_idx[i]) * shard_stride));
    }
#pragma unroll
    for (int p = 0; p < MS; ++p) {
        if (p >= nout) continue;
        uint8_t *q = sb + out_off[p];
        if (VERIFY) {
            const V have = ld(q);
            bool diff = false;
#pragma unroll
            for (int w = 0; w < W; ++w) diff |= have[w] != acc[p][w];
            if (diff) flag_mismatch(mismatch);
        } else if (W == 4 && half) {
            __builtin_nontemporal_store(u32x2{acc[p][0], acc[p][1]}, reinterpret_cast<u32x2 *>(RSAMD_G(q, 8)));
        } else {
            V v;
#pragma unroll
            for (int w = 0; w < W; ++w) v[w] = acc[p][w];
            __builtin_nontemporal_store(v, reinterpret_cast<V *>(RSAMD_G(q, W * 4)));
        }
    }
}

// Lane vector v of a stripe: U16, whole 16-byte vectors below nfull16, then
// the half vector; otherwise 8-byte vectors throughout.
template <bool U16, int K, int MS, bool VERIFY>
__device__ __forceinline__ void code8_lane(uint8_t *stripe_base, uint32_t v, uint32_t nfull16, const uint32_t *tabs,
                                           const int32_t *in_idx, const int32_t *out_idx, int nin, int nout,
                                           uint64_t shard_stride, int *mismatch) {
    uint8_t *sb = stripe_base + uint64_t(v) * (U16 ? 16 : 8);
    if (U16)
        code8<4, K, MS, VERIFY>(sb, v >= nfull16, tabs, in_idx, out_idx, nin, nout, shard_stride, mismatch);
    else
        code8<2, K, MS, VERIFY>(sb, false, tabs, in_idx, out_idx, nin, nout, shard_stride, mismatch);
}

template <int K, int MS>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(8, 8))) gf_masked8_kernel(MaskedArgs a) {
    uint32_t stripe, chunk;
    block_item(a.chunks, a.cdiv, a.rot, a.xcd_span, stripe, chunk);
    const uint32_t v = chunk * uint32_t(kWave) + threadIdx.x;
    const uint8_t *rec = masked_record(a.records, a.rec_stride, a.plan_ids, a.mask_table, a.mask_bits, stripe);
    if (!rec) {
        count_undecodable(a.bad, v == 0);
        return;
    }
    const int nout = *reinterpret_cast<const int32_t *>(rec);
    if (nout == 0 || v >= a.nvec) return;
    code8_lane<RSAMD_MASKED8_U16, K, MS, false>(a.base + uint64_t(stripe) * a.stripe_stride, v, a.pat_chunk0,
                             reinterpret_cast<const uint32_t *>(rec + a.rec_tabs),
                             reinterpret_cast<const int32_t *>(rec + a.rec_in_idx),
                             reinterpret_cast<const int32_t *>(rec + a.rec_out_idx), a.nin, nout, a.shard_stride,
                             nullptr);
}

struct Vec8Args {
    VecArgs v;
    uint32_t nfull16;
};

template <int K, int M, bool VERIFY>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(8, 8))) gf_vec8_kernel(Vec8Args a8) {
    const VecArgs &a = a8.v;
    if (VERIFY && mismatch_seen(a.mismatch)) return;
    uint32_t stripe, chunk;
    block_item(a.chunks, a.cdiv, a.rot, a.xcd_span, stripe, chunk);
    const uint32_t v = chunk * uint32_t(kWave) + threadIdx.x;
    if (v >= a.nvec) return;
    code8_lane<RSAMD_VEC8_U16, K, M, VERIFY>(a.base + uint64_t(stripe) * a.stripe_stride, v, a8.nfull16,
                                             RSAMD_G(a.tabs, a.nin * M * 20), RSAMD_G(a.in_idx, a.nin * 4),
                                             RSAMD_G(a.out_idx, M * 4), a.nin, M, a.shard_stride, a.mismatch);
}

// ---------------------------------------------------------------------------
// Line-owner kernel for chunk groups packed back to back: the master's
// 6 x 1000-byte groups (ChunkserverDiskRecoveryMachine.java:34-48,
// MasterImpl.java:794-839) at shard stride 1000, group stride 6000.  There
// every shard starts and ends inside a 128-byte line.  The 8-byte kernels
// above read and write it as 1000-byte runs of 8-byte lanes split over two
// waves: lines written piecewise by two waves, a partially written line at
// each end of an output shard, and reads that split lines into separate
// requests.  HBM serves partial lines with read-modify-writes; the 8-byte
// kernels ran at 0.59 of peak against 0.72 for the same groups in 1 KiB slots.
//
// Here ONE wave owns a group, and every line it touches it touches whole:
//  * phase 0: each input shard's lines (the shard's bytes rounded out to
//    128-byte lines) as aligned 16-byte loads into LDS;
//  * phase 1: each lane codes 8-byte columns of every output from LDS into
//    registers, then (the input lines no longer needed) parks them in LDS in
//    memory order, one slot per run of consecutive output shards;
//  * phase 2: each run is stored as whole aligned lines (16-byte non-temporal
//    stores).  The bytes of a run's first and last line that lie outside it
//    belong to the neighbouring shard; when nobody writes that shard in this
//    launch (a shard of this group that is not an output -- runs are maximal
//    -- or a neighbouring group's shard that group does not rebuild), the wave
//    loads those bytes (with the input loads) and writes them back unchanged,
//    so HBM sees no partial line.  Otherwise (or at the batch's ends) the line
//    stays partial.
// Shards of >= 256 bytes keep two runs of one group on different lines.
// Measured on 4 M groups (profiles/r3/): encode and decode
// {0,1} 0.745 of peak against 0.590 for the 8-byte kernels, per-group
// bitmasks 0.70 against 0.605, PMC traffic 1.05x / 1.08x the algorithmic
// bytes (the rounding to lines).  Variants measured and dropped (A/B builds):
// 8-byte lane loads straight from HBM 0.645, no write-back of the foreign
// bytes 0.578, plain stores 0.58, two groups per wave 0.62, loading a line
// shared by two input shards once 0.60 (its loads took two round trips).
// ---------------------------------------------------------------------------
struct GroupArgs {
    uint8_t *base;            // stripe 0 of this launch
    uint64_t stripe_stride;   // = total * len
    uint8_t *lo, *hi;         // the batch's bytes: [lo, hi)
    uint32_t len;             // shard length = shard stride (multiple of 8, >= 256)
    uint32_t total;           // shards per stripe
    uint32_t n_items;         // stripes in this launch (one wave each)
    uint32_t xcd_span;        // block order: XCD-contiguous remap span (0 = off)
    // one plan for every stripe (MASKED = false)
    const uint32_t *tabs;     // tabs[nin][MS][5]
    const int32_t *in_idx;
    const int32_t *out_idx;   // ascending: every Plan lists its outputs in shard order (codec.cpp)
    // a record per stripe (MASKED = true), as MaskedArgs
    const uint8_t *records;
    uint64_t rec_stride;
    const int32_t *plan_ids;  // offset to this launch's stripe 0
    const int32_t *mask_table;
    int mask_bits;
    int32_t *bad;
    uint32_t rec_in_idx, rec_out_idx, rec_tabs;
    uint32_t has_prev;        // stripe 0 of this launch has a predecessor in the batch
    uint32_t has_next_last;   // the launch's last stripe has a successor in the batch
};

typedef uint32_t u32x2a __attribute__((ext_vector_type(2)));

// One wave per stripe; shards of 256 .. kGroupMaxLen bytes, so one pass of
// 2 x 1 KiB loads per input covers a shard's lines and a lane codes at most
// kGroupIters 8-byte columns.  The LDS area first holds the input lines, then
// (after every lane has its columns in registers) the output runs: 5 KiB per
// wave at 4+2 x 1000 B.  Three or four outputs hold up to 32 accumulator
// registers per lane: a budget of 5 waves per SIMD, unspilled.
constexpr uint32_t kGroupMaxLen = 1792;
#ifndef RSAMD_GROUP_FOREIGN
#define RSAMD_GROUP_FOREIGN 1  // A/B: 0 = never write foreign bytes back (a run's ragged ends as 8-byte stores)
#endif
#ifndef RSAMD_GROUP_FOREIGN_LDS
#define RSAMD_GROUP_FOREIGN_LDS 1  // foreign bytes of a survivor's line from LDS: 0 never, 1 per-group records, 2 always
#endif
constexpr int kGroupIters = 4;

template <int K, int MS, bool MASKED>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(MS >= 3 ? 5 : 8, 8))) gf_group8_kernel(GroupArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint32_t t = blockIdx.x;
    if (a.xcd_span && t < 8u * a.xcd_span) t = (t & 7u) * a.xcd_span + (t >> 3);
    const uint32_t lane = threadIdx.x;
    const uint32_t len = a.len;
    const int T = int(a.total);
    uint8_t *sb = a.base + uint64_t(t) * a.stripe_stride;
    const bool has_prev = t > 0 || a.has_prev, has_next = t + 1 < a.n_items || a.has_next_last;

    // Inputs, outputs and the neighbours' claims on this stripe's edge shards,
    // all known before any load: the first K present shards are the survivors
    // (ReedSolomon.java:210-223) and every absent shard is an output, in
    // ascending order -- read off the stripe's bitmask (MASKED) or the plan.
    int sidx[K], oidx[MS];
    int nout;
    const uint32_t *tabs;
    bool prev_busy, next_busy;  // the previous stripe rebuilds its last shard / the next its first
    uint32_t bits = 0;
    if (MASKED) {
        bits = uint32_t(*RSAMD_G(a.plan_ids + t, 4));
        const uint32_t bp = has_prev ? uint32_t(*RSAMD_G(a.plan_ids + (int64_t(t) - 1), 4)) : 0u;
        const uint32_t bn = has_next ? uint32_t(*RSAMD_G(a.plan_ids + (t + 1), 4)) : 0u;
        const uint32_t full = (1u << a.mask_bits) - 1u;
        if ((bits >> a.mask_bits) || __builtin_popcount(bits) < K) {
            count_undecodable(a.bad, lane == 0);
            return;
        }
        if (bits == full) return;  // nothing missing
        uint32_t rest = bits, miss = ~bits & full;
        nout = __builtin_popcount(miss);
#pragma unroll
        for (int i = 0; i < K; ++i) {
            sidx[i] = __builtin_ctz(rest);
            rest &= rest - 1u;
        }
#pragma unroll
        for (int p = 0; p < MS; ++p) {
            oidx[p] = miss ? __builtin_ctz(miss) : T;
            miss &= miss - 1u;
        }
        // conservative: an absent shard of an undecodable neighbour counts as rebuilt
        prev_busy = !has_prev || (bp >> a.mask_bits) || !((bp >> (T - 1)) & 1u);
        next_busy = !has_next || (bn >> a.mask_bits) || !(bn & 1u);
        // The record's tables.  Its id is read before any vector load (there
        // it stays a scalar load; behind the input loads the compiler read it
        // per lane, and the tables with it).  The pointer is formed after the
        // id check: a pointer that may be null is a generic one, which may
        // alias LDS, and the tables would then be read with per-lane loads.
        const int32_t id = *RSAMD_G(a.mask_table + bits, 4);
        if (id < 0) {  // a singular survivor matrix
            count_undecodable(a.bad, lane == 0);
            return;
        }
        tabs = reinterpret_cast<const uint32_t *>(RSAMD_G(a.records + uint64_t(id) * a.rec_stride + a.rec_tabs, K * MS * 20));
    } else {
        nout = MS;
        tabs = RSAMD_G(a.tabs, K * MS * 20);
#pragma unroll
        for (int i = 0; i < K; ++i) sidx[i] = *RSAMD_G(a.in_idx + i, 4);
#pragma unroll
        for (int p = 0; p < MS; ++p) oidx[p] = *RSAMD_G(a.out_idx + p, 4);
        prev_busy = !has_prev || oidx[MS - 1] == T - 1;
        next_busy = !has_next || oidx[0] == 0;
    }

    // Runs of consecutive output shards and their LDS slots (memory order).
    // Every array is indexed by the unrolled p only (a runtime index would
    // put it in scratch): run_start[p] marks the first output of a run,
    // run_lds[p] its slot, run_last[p] the last shard of p's run.
    bool run_start[MS];
    uint32_t out_lds[MS], run_lds[MS];
    int run_last[MS];
    {
        uint32_t cum = 0;
        int cur_p0 = 0;
#pragma unroll
        for (int p = 0; p < MS; ++p) {
            run_start[p] = p < nout && (p == 0 || oidx[p] != oidx[p - 1] + 1);
            if (run_start[p] && p > 0) {
                cum += (uint32_t(p - cur_p0) * len + 256u + 15u) & ~15u;
                cur_p0 = p;
            }
            run_lds[p] = cum;
            const uint8_t *r0 = sb + uint64_t(oidx[cur_p0]) * len;
            out_lds[p] = cum + uint32_t(reinterpret_cast<uintptr_t>(r0) & 127u) + uint32_t(p - cur_p0) * len;
        }
        int last = 0;
#pragma unroll
        for (int p = MS - 1; p >= 0; --p) {
            if (p < nout && (p == nout - 1 || (p + 1 < MS && run_start[p + 1]))) last = oidx[p];
            run_last[p] = last;
        }
    }

    // Phase 0: each input shard's whole lines (16-byte aligned loads, one
    // pass), and the foreign bytes of each run's first and last line where
    // nobody writes them -- all loads issued together.
    const uint32_t islot = (len + 256u + 15u) & ~15u;
    uint32_t in_off[K];
    u32x4 r[K][2];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const uint8_t *si = sb + uint64_t(sidx[i]) * len;
        in_off[i] = uint32_t(reinterpret_cast<uintptr_t>(si) & 127u);
        const uint8_t *ai = si - in_off[i];
        const uint32_t span = (in_off[i] + len + 127u) & ~127u;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t q = uint32_t(h) * 16u * kWave + 16u * lane;
            if (q < span) r[i][h] = load_stream(ai + q);
        }
    }
    bool head[MS], tail[MS], fin[MS], fin_lds[MS];
    uint32_t foff[MS], fsrc[MS];
    u32x2a fv[MS];
#pragma unroll
    for (int p = 0; p < MS; ++p) {
        fin[p] = fin_lds[p] = false;
        if (!run_start[p]) continue;
        const int s0 = oidx[p], s1 = run_last[p];
        uint8_t *r0 = sb + uint64_t(s0) * len, *r1 = sb + uint64_t(s1 + 1) * len;
        uint8_t *l0 = r0 - (reinterpret_cast<uintptr_t>(r0) & 127u);  // pointer arithmetic keeps the
        uint8_t *l1 = r1 + ((128u - (reinterpret_cast<uintptr_t>(r1) & 127u)) & 127u);  // global address space
        head[p] = RSAMD_GROUP_FOREIGN && (s0 > 0 || !prev_busy);
        tail[p] = RSAMD_GROUP_FOREIGN && (s1 + 1 < T || !next_busy);
        uint8_t *q = lane < 16 ? l0 + 8u * lane : r1 + 8u * (lane - 16);
        fin[p] = lane < 16 ? (head[p] && q < r0) : (lane < 32 && tail[p] && q < l1);
        foff[p] = run_lds[p] + uint32_t(q - l0);
        // A neighbour shard of this stripe that is a survivor has the line in
        // LDS after phase 0: read the bytes there instead of loading the line
        // again.  Per-group records only (A/B in RSAMD_GROUP_FOREIGN_LDS).
        if (RSAMD_GROUP_FOREIGN_LDS == 2 || (RSAMD_GROUP_FOREIGN_LDS == 1 && MASKED)) {
            const int nb = lane < 16 ? s0 - 1 : s1 + 1;
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (sidx[i] == nb) {
                    fin_lds[p] = fin[p];
                    fsrc[p] = uint32_t(i) * islot + uint32_t(q - (sb + uint64_t(sidx[i]) * len)) + in_off[i];
                }
        }
        if (fin[p] && !fin_lds[p]) fv[p] = *reinterpret_cast<const u32x2a *>(RSAMD_G(q, 8));
    }

#pragma unroll
    for (int i = 0; i < K; ++i) {
        const uint32_t span = (in_off[i] + len + 127u) & ~127u;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t q = uint32_t(h) * 16u * kWave + 16u * lane;
            if (q < span) *reinterpret_cast<u32x4 *>(lds + i * islot + q) = r[i][h];
        }
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < MS; ++p)
        if (fin_lds[p]) fv[p] = *reinterpret_cast<const u32x2a *>(lds + fsrc[p]);

    // Phase 1: 8-byte columns of every output, from LDS into registers.  The
    // tables are read through the constant address space: they are not
    // written while the kernel runs, and a load behind a barrier from a
    // global pointer cannot be proven unclobbered (it would be read per lane).
    const __attribute__((address_space(4))) uint32_t *ctabs =
        (const __attribute__((address_space(4))) uint32_t *)(tabs);
    const uint32_t nw = len / 8;
    uint32_t acc[kGroupIters][MS][2];
#pragma unroll
    for (int it = 0; it < kGroupIters; ++it) {
        const uint32_t v = uint32_t(it) * kWave + lane;
        if (v < nw) {
            u32x2a x[K];
#pragma unroll
            for (int i = 0; i < K; ++i) x[i] = *reinterpret_cast<const u32x2a *>(lds + i * islot + in_off[i] + 8u * v);
#pragma unroll
            for (int w = 0; w < 2; ++w) {
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const Sel sl = selectors(x[i][w]);
#pragma unroll
                    for (int p = 0; p < MS; ++p) {
                        uint32_t t0, t1, t2, tp[5];
#pragma unroll
                        for (int j = 0; j < 5; ++j) tp[j] = ctabs[(i * MS + p) * 5 + j];
                        terms(tp, sl, t0, t1, t2);
                        acc[it][p][w] = i == 0 ? xor3(t0, t1, t2) : xor3(acc[it][p][w], t0, t1) ^ t2;
                    }
                }
            }
        }
    }
    __syncthreads();  // every lane is done with the input lines: LDS now takes the outputs

#pragma unroll
    for (int it = 0; it < kGroupIters; ++it) {
        const uint32_t v = uint32_t(it) * kWave + lane;
        if (v < nw) {
#pragma unroll
            for (int p = 0; p < MS; ++p)
                if (p < nout)
                    *reinterpret_cast<u32x2a *>(lds + out_lds[p] + 8u * v) = u32x2a{acc[it][p][0], acc[it][p][1]};
        }
    }
#pragma unroll
    for (int p = 0; p < MS; ++p)
        if (fin[p]) *reinterpret_cast<u32x2a *>(lds + foff[p]) = fv[p];
    __syncthreads();
    // Phase 2: each run's lines, as aligned 16-byte stores (8-byte halves where
    // a partial line starts or ends mid-vector).
#pragma unroll
    for (int p = 0; p < MS; ++p) {
        if (!run_start[p]) continue;
        const int s0 = oidx[p], s1 = run_last[p];
        uint8_t *r0 = sb + uint64_t(s0) * len, *r1 = sb + uint64_t(s1 + 1) * len;
        uint8_t *l0 = r0 - (reinterpret_cast<uintptr_t>(r0) & 127u);
        uint8_t *l1 = r1 + ((128u - (reinterpret_cast<uintptr_t>(r1) & 127u)) & 127u);
        uint8_t *w0 = head[p] ? l0 : r0, *w1 = tail[p] ? l1 : r1;
        uint8_t *x0 = w0 - (reinterpret_cast<uintptr_t>(w0) & 15u);
        for (uint8_t *q = x0 + 16u * lane; q < w1; q += 16u * kWave) {
            const u32x4 v = *reinterpret_cast<const u32x4 *>(lds + run_lds[p] + (q - l0));
            const bool lo_in = q >= w0 && q + 8 <= w1, hi_in = q + 8 >= w0 && q + 16 <= w1;
            if (lo_in && hi_in)
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(RSAMD_G(q, 16)));
            else if (lo_in)
                __builtin_nontemporal_store(u32x2a{v[0], v[1]}, reinterpret_cast<u32x2a *>(RSAMD_G(q, 8)));
            else if (hi_in)
                __builtin_nontemporal_store(u32x2a{v[2], v[3]}, reinterpret_cast<u32x2a *>(RSAMD_G(q + 8, 8)));
        }
    }
}

// Masked byte kernel: any alignment, and the <16-byte tails.
struct MaskedByteArgs {
    uint8_t *base;
    const uint8_t *records;
    uint64_t rec_stride;
    const int32_t *plan_ids;
    uint64_t stripe_stride, shard_stride, col0, ncols, total;
    uint32_t rec_in_idx, rec_out_idx, rec_tabs;
    int nin, mslots;
    const int32_t *mask_table;
    int mask_bits;
    int32_t *bad;
    uint64_t pat_bytes, row_bytes;  // MaskedPlan::pattern_bytes (0: per stripe); the view's full shard length
    uint64_t count_col;             // per-stripe patterns: the column whose thread counts an undecodable stripe
};

__global__ void __launch_bounds__(kThreads) gf_masked_byte_kernel(MaskedByteArgs a) {
    const uint64_t step = uint64_t(gridDim.x) * kThreads;
    for (uint64_t idx = uint64_t(blockIdx.x) * kThreads + threadIdx.x; idx < a.total; idx += step) {
        const uint64_t stripe = idx / a.ncols;
        const uint64_t col = a.col0 + (idx - stripe * a.ncols);
        uint64_t pat = stripe;
        bool first = col == a.count_col;
        if (a.pat_bytes) {
            const uint64_t x = stripe * a.row_bytes + col;
            pat = x / a.pat_bytes;
            first = x == pat * a.pat_bytes;
        }
        const uint8_t *rec = masked_record(a.records, a.rec_stride, a.plan_ids, a.mask_table, a.mask_bits, pat);
        if (!rec) {
            count_undecodable(a.bad, first);
            continue;
        }
        const int nout = *reinterpret_cast<const int32_t *>(rec);
        if (nout == 0) continue;
        const int32_t *in_idx = reinterpret_cast<const int32_t *>(rec + a.rec_in_idx);
        const int32_t *out_idx = reinterpret_cast<const int32_t *>(rec + a.rec_out_idx);
        const uint32_t *tabs = reinterpret_cast<const uint32_t *>(rec + a.rec_tabs);
        uint8_t *sb = a.base + stripe * a.stripe_stride + col;
        uint32_t acc[kMaxOut] = {0, 0, 0, 0};
        for (int i = 0; i < a.nin; ++i) {
            const Sel s = selectors(*RSAMD_G(sb + uint64_t(in_idx[i]) * a.shard_stride, 1));
            for (int p = 0; p < nout; ++p) {
                uint32_t t0, t1, t2;
                terms(tabs + (i * a.mslots + p) * 5, s, t0, t1, t2);
                acc[p] = xor3(acc[p], t0, t1) ^ t2;
            }
        }
        for (int p = 0; p < nout; ++p) *RSAMD_G(sb + uint64_t(out_idx[p]) * a.shard_stride, 1) = uint8_t(acc[p]);
    }
}

// ---------------------------------------------------------------------------
// Byte kernel: any alignment; also the <16-byte tail of aligned shards.
// One thread per (stripe, column byte).
// ---------------------------------------------------------------------------
template <bool VERIFY>
__global__ void __launch_bounds__(kThreads) gf_byte_kernel(ByteArgs a) {
    const uint64_t step = uint64_t(gridDim.x) * kThreads;
    for (uint64_t idx = uint64_t(blockIdx.x) * kThreads + threadIdx.x; idx < a.total; idx += step) {
        if (VERIFY && mismatch_seen(a.mismatch)) return;
        const uint64_t stripe = idx / a.ncols;
        const uint64_t col = a.col0 + (idx - stripe * a.ncols);
        uint8_t *sb = a.base + stripe * a.stripe_stride + col;
        const uint32_t *tabs = RSAMD_G(a.tabs, a.nin * a.nout * 20);
        const int32_t *in_idx = RSAMD_G(a.in_idx, a.nin * 4), *out_idx = RSAMD_G(a.out_idx, a.nout * 4);
        uint32_t acc[kMaxOut] = {0, 0, 0, 0};
        for (int i = 0; i < a.nin; ++i) {
            const Sel s = selectors(*RSAMD_G(sb + uint64_t(in_idx[i]) * a.shard_stride, 1));
            for (int p = 0; p < a.nout; ++p) {
                uint32_t t0, t1, t2;
                terms(tabs + (i * a.nout + p) * 5, s, t0, t1, t2);
                acc[p] = xor3(acc[p], t0, t1) ^ t2;
            }
        }
        for (int p = 0; p < a.nout; ++p) {
            uint8_t *dst = RSAMD_G(sb + uint64_t(out_idx[p]) * a.shard_stride, 1);
            if (VERIFY) {
                if (*dst != uint8_t(acc[p])) flag_mismatch(a.mismatch);
            } else {
                *dst = uint8_t(acc[p]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Synthetic data and the reference copy kernel (benchmark support).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t n) {
    uint64_t z = seed + n * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(kThreads)
    fill_synthetic_kernel(uint8_t *base, uint64_t words_per_stripe, uint64_t words_per_shard,
                          uint64_t n_words, uint64_t shard_stride, uint64_t stripe_stride, uint64_t seed,
                          uint64_t stripe0) {
    const uint64_t step = uint64_t(gridDim.x) * kThreads;
    for (uint64_t idx = uint64_t(blockIdx.x) * kThreads + threadIdx.x; idx < n_words; idx += step) {
        const uint64_t t = idx / words_per_stripe;
        const uint64_t w = idx - t * words_per_stripe;
        const uint64_t shard = w / words_per_shard;
        const uint64_t col = (w - shard * words_per_shard) * 8;
        *reinterpret_cast<uint64_t *>(RSAMD_G(base + t * stripe_stride + shard * shard_stride + col, 8)) =
            splitmix64_at(seed ^ (stripe0 + t), w + 1);
    }
}

// Same access shape as the vector kernels: one wave per block, one 16-byte
// vector per lane, non-temporal both ways, one-shot grid.
__global__ void __launch_bounds__(kWave) copy_kernel(uint8_t *dst, const uint8_t *src, uint64_t nvec) {
    const uint64_t i = uint64_t(blockIdx.x) * kWave + threadIdx.x;
    if (i < nvec) __builtin_nontemporal_store(load_stream(src + i * 16), reinterpret_cast<u32x4 *>(RSAMD_G(dst + i * 16, 16)));
}

__global__ void copy_tail_kernel(uint8_t *dst, const uint8_t *src, uint64_t n) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) *RSAMD_G(dst + i, 1) = *RSAMD_G(src + i, 1);
}

// ---------------------------------------------------------------------------
// Direct kernel: shards in page-locked HOST memory, coded in place over the
// link (the host-buffer entry points, capi.cpp run_direct).  Every input
// vector is loaded across PCIe and every output vector stored back across it,
// so the link carries H2D and D2H at once with no copy engine, no staging
// buffer and no per-chunk hand-off.  tools/zc_probe.hip, profiles/r3/
// zc_probe_r3s2b.txt: 4 host loads -> 2 host stores per column run at 50.3-50.6
// GiB/s of data shards, 0.96 of the link bound, where the chunked DMA
// pipeline reaches 0.86.  The link, not the GF arithmetic, is the bound, so
// the kernel keeps a plain shape: a grid-stride loop over W-byte vectors
// (W = 16, or 8 when the shards' addresses agree only modulo 8), one input
// at a time, the pointers as wave-uniform kernel arguments.  Bytes before the
// first aligned vector (head) and after the last (tail) go one per thread.
// ---------------------------------------------------------------------------
struct DirectArgs {
    const uint8_t *in[kMaxDirectIn];
    uint8_t *out[kMaxOut];
    const uint32_t *tabs;  // [nin][M][5]
    uint64_t head;         // bytes before the first W-aligned vector
    uint64_t nvec;         // W-byte vectors after the head
    uint64_t n;            // bytes per shard
    int nin;
    int *mismatch;
    DirectTee tee;         // TEE kernels only
    DirectSignal sig;      // sig.flag == nullptr: no completion signal
};

// The completion signal (kernels.hpp DirectSignal), after a block's last store.
__device__ __forceinline__ void signal_done(const DirectSignal &sg, int *mismatch) {
    dev::signal_done(sg.flag, sg.ctr, sg.seq, mismatch);
}

// The tee store of one 8-byte unit of data shard d at column c (unit-aligned,
// so inside one block), clipped to the file (the padding's rows are not file
// bytes).
__device__ __forceinline__ void tee8(const DirectTee &t, int d, uint64_t c, uint32_t lo, uint32_t hi) {
    const uint64_t r = c / t.blk;
    const uint64_t f = r * t.k * t.blk + uint64_t(d) * t.blk + (c - r * t.blk);
    if (f + 8 <= t.file_size) {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store(u32x2{lo, hi}, reinterpret_cast<u32x2 *>(RSAMD_G(t.file + f, 8)));
        return;
    }
    const uint64_t x = uint64_t(lo) | uint64_t(hi) << 32;
    for (uint64_t b = f; b < t.file_size && b < f + 8; ++b) *RSAMD_G(t.file + b, 1) = uint8_t(x >> (8 * (b - f)));
}

// The same for a 16-byte vector at column c: one 16-byte store when both
// halves lie in one block row and in the file (consecutive lanes then cover
// whole lines with one instruction), else two 8-byte ones.
__device__ __forceinline__ void tee16(const DirectTee &t, int d, uint64_t c, const u32x4 &y) {
    const uint64_t r = c / t.blk, w = c - r * t.blk;
    const uint64_t f = r * t.k * t.blk + uint64_t(d) * t.blk + w;
    if (w + 16 <= t.blk && f + 16 <= t.file_size) {
        typedef uint32_t u32x4_a8 __attribute__((ext_vector_type(4), aligned(8)));
        __builtin_nontemporal_store(u32x4_a8{y[0], y[1], y[2], y[3]}, reinterpret_cast<u32x4_a8 *>(RSAMD_G(t.file + f, 16)));
        return;
    }
    tee8(t, d, c, y[0], y[1]);
    tee8(t, d, c + 8, y[2], y[3]);
}

template <int W>
struct DirectVec;
template <>
struct DirectVec<16> {
    typedef u32x4 T;
    static constexpr int kDwords = 4;
};
template <>
struct DirectVec<8> {
    typedef uint32_t T __attribute__((ext_vector_type(2)));
    static constexpr int kDwords = 2;
};

// Input i's W bytes at `off` folded into acc.
template <int W, int M>
__device__ __forceinline__ void direct_fold(const DirectArgs &a, int i, const typename DirectVec<W>::T &x,
                                            uint32_t (&acc)[M][DirectVec<W>::kDwords]) {
    uint32_t T[M][5];
#pragma unroll
    for (int p = 0; p < M; ++p)
#pragma unroll
        for (int j = 0; j < 5; ++j) T[p][j] = *RSAMD_G(a.tabs + ((i * M + p) * 5 + j), 4);
#pragma unroll
    for (int w = 0; w < DirectVec<W>::kDwords; ++w) {
        const Sel s = selectors(x[w]);
#pragma unroll
        for (int p = 0; p < M; ++p) {
            uint32_t t0, t1, t2;
            terms(T[p], s, t0, t1, t2);
            acc[p][w] = xor3(acc[p][w], t0, t1) ^ t2;
        }
    }
}

// PRE (small calls, kernels.hpp DirectSignal): the inputs are loaded eight at
// a time before any is folded, so a thread waits for one link round trip per
// eight inputs instead of one per input -- a small call has too few waves to
// hide them.  The streaming form keeps one input in flight per thread (its
// many waves hide the latency; its ISA is unchanged).
template <int W, int M, bool VERIFY, bool TEE, bool PRE>
__global__ void __launch_bounds__(kThreads) gf_direct_kernel(DirectArgs a) {
    typedef typename DirectVec<W>::T V;
    constexpr int D = DirectVec<W>::kDwords;
    const uint64_t step = uint64_t(gridDim.x) * kThreads;
    for (uint64_t v = uint64_t(blockIdx.x) * kThreads + threadIdx.x; v < a.nvec; v += step) {
        if (VERIFY && mismatch_seen(a.mismatch)) break;  // (the completion signal below still runs)
        const uint64_t off = a.head + v * W;
        uint32_t acc[M][D];
#pragma unroll
        for (int p = 0; p < M; ++p)
#pragma unroll
            for (int w = 0; w < D; ++w) acc[p][w] = 0;
        if constexpr (PRE) {
            constexpr int kPre = 8;
            for (int i0 = 0; i0 < a.nin; i0 += kPre) {
                V x[kPre];
#pragma unroll
                for (int j = 0; j < kPre; ++j)
                    if (i0 + j < a.nin) x[j] = __builtin_nontemporal_load(reinterpret_cast<const V *>(RSAMD_G(a.in[i0 + j] + off, W)));
#pragma unroll
                for (int j = 0; j < kPre; ++j)
                    if (i0 + j < a.nin) direct_fold<W, M>(a, i0 + j, x[j], acc);
            }
        } else {
            for (int i = 0; i < a.nin; ++i) {
                const V x = __builtin_nontemporal_load(reinterpret_cast<const V *>(RSAMD_G(a.in[i] + off, W)));
                direct_fold<W, M>(a, i, x, acc);
            }
        }
#pragma unroll
        for (int p = 0; p < M; ++p) {
            V y;
#pragma unroll
            for (int w = 0; w < D; ++w) y[w] = acc[p][w];
            V *dst = reinterpret_cast<V *>(RSAMD_G(a.out[p] + off, W));
            if (VERIFY) {
                const V have = __builtin_nontemporal_load(dst);
                bool same = true;
#pragma unroll
                for (int w = 0; w < D; ++w) same = same && have[w] == y[w];
                if (!same) flag_mismatch(a.mismatch);
            } else {
                __builtin_nontemporal_store(y, dst);
                if (TEE && a.tee.data[p] >= 0) {
                    if constexpr (W == 16)
                        tee16(a.tee, a.tee.data[p], off, y);
                    else
                        tee8(a.tee, a.tee.data[p], off, y[0], y[1]);
                }
            }
        }
    }
    // head bytes (< 4 KiB) and tail bytes (< W): block 0, one byte per thread
    const uint64_t tail0 = a.head + a.nvec * W;
    const uint64_t nbytes = a.head + (a.n - tail0);
    for (uint64_t t = threadIdx.x; blockIdx.x == 0 && t < nbytes; t += kThreads) {
        const uint64_t b = t < a.head ? t : tail0 + (t - a.head);
        uint32_t acc[M] = {};
        for (int i = 0; i < a.nin; ++i) {
            const Sel s = selectors(*RSAMD_G(a.in[i] + b, 1));
#pragma unroll
            for (int p = 0; p < M; ++p) {
                uint32_t t0, t1, t2;
                terms(RSAMD_G(a.tabs + (i * M + p) * 5, 20), s, t0, t1, t2);
                acc[p] = xor3(acc[p], t0, t1) ^ t2;
            }
        }
#pragma unroll
        for (int p = 0; p < M; ++p) {
            if (VERIFY) {
                if (*RSAMD_G(a.out[p] + b, 1) != uint8_t(acc[p])) flag_mismatch(a.mismatch);
            } else {
                *RSAMD_G(a.out[p] + b, 1) = uint8_t(acc[p]);
                if (TEE && a.tee.data[p] >= 0) {
                    const uint64_t r = b / a.tee.blk;
                    const uint64_t f = r * a.tee.k * a.tee.blk + uint64_t(a.tee.data[p]) * a.tee.blk + (b - r * a.tee.blk);
                    if (f < a.tee.file_size) *RSAMD_G(a.tee.file + f, 1) = uint8_t(acc[p]);
                }
            }
        }
    }
    if (a.sig.flag) signal_done(a.sig, VERIFY ? a.mismatch : nullptr);
}

// ---------------------------------------------------------------------------
// Host-side dispatch.
// ---------------------------------------------------------------------------
#ifndef RSAMD_VEC_LDS_PAD
#define RSAMD_VEC_LDS_PAD -1  // A/B: dynamic LDS bytes per wave of gf_vec_kernel (-1: the table below)
#endif
// Occupancy cap of the vector kernels.  A one-wave workgroup that asks for
// `pad` bytes of (unused) dynamic LDS leaves 160 KiB / pad waves per CU, and
// fewer waves in flight stream HBM better: at the VGPR limit (32 waves per
// CU) the 4+2 encode reads 0.836 of peak, at 12 waves 0.860.  Measured per
// shape on one pool, pads alternated (tools/occ_sweep.py,
// profiles/r3/occ_sweep_r3zs.txt; fractions of 8 TB/s, pad in bytes):
//   shape                        0      10240  11520  12544  13568  14848  16384  20480
//   4+2 granule encode         0.836  0.847  0.852  0.861  0.860  0.855  0.828  0.777
//   4+2 granule decode {0}     0.796  0.797  0.813  0.837  0.837  0.830  0.803  0.754
//   4+2 granule decode {0,5}   0.800  0.813  0.814  0.820  0.822  0.819  0.804  0.762
//   4+2 granule verify         0.887  0.933  0.950  0.897  0.844  0.788  0.731  0.669
//   4+2 packed encode          0.801  0.828  0.852  0.860  0.857  0.844  0.811  0.762
//   4+2 x 4 KiB packed encode  0.760  0.791  0.795  0.807  0.813  0.814  0.801  0.759
//   10+4 granule encode        0.801  0.814  0.812  0.803  0.792  0.778  0.758  0.733
//   10+4 granule decode {0,1}  0.795  0.794  0.793  0.798  0.818  0.843  0.845  0.821
//   10+4 granule decode {0}    0.747  0.765  0.773  0.780  0.784  0.789  0.796  0.802
//   10+4 granule verify        0.827  0.807  0.800  0.768  0.753  0.729  0.684  0.632
//   10+4 packed encode         0.737  0.758  0.761  0.764  0.765  0.754  0.744  0.713
// The table below takes each column's best per (k, outputs, verify), checked
// again in plain block order (block_order: capped launches), which moved the
// 4+2 decodes' best to 12544 ({0} 0.877 against 0.872 at 13568, encode a tie;
// profiles/r3/occ_plain_r3zz3.txt, occ_plain2_r3zz4.txt).
size_t vec_lds_pad(int k, int m, bool verify) {
    if (const char *e = tuning_env("RSAMD_VEC_LDS_PAD")) return size_t(std::atol(e));  // per launch: sweeps
    if (RSAMD_VEC_LDS_PAD >= 0) return size_t(RSAMD_VEC_LDS_PAD);
    if (k == 4) return verify ? 11520 : 12544;
    if (k == 10) {
        if (verify) return 0;
        return m >= 4 ? 10240 : m == 3 ? 13568 : m == 2 ? 16384 : 20480;
    }
    // 17+m (the upstream library's benchmark code, compiled like 10+m): 17+3
    // granule encode / decode {0,1,2} 0.777 / 0.770 at 16384 B against the
    // runtime-k kernel's 0.760-0.766 / 0.748-0.765 at its best cap (tools/gpu_k17.sh,
    // profiles/r3/k17_r3s2v.txt, k17_r3s2w.txt).
    if (k == 17) return verify ? 0 : 16384;
    // 6+m and 8+m, compiled since the end of round 3 (tools/gpu_k68.sh,
    // profiles/r3/k68_r3s2w2.txt; runtime-k kernel at its best cap -> compiled):
    // 8+4 encode 0.805 -> 0.827 (10240 B), decode {0} 0.758 -> 0.777 (16384);
    // 6+3 encode 0.834 -> 0.855, decode {0,1} 0.848 -> 0.869 (14848).
    if (k == 8) return verify ? 0 : m == 1 ? 16384 : m == 2 ? 12544 : 10240;
    if (k == 6) return verify ? 0 : m == 1 ? 16384 : 14848;
    // The runtime-k kernel (every other k; called with k = 0), since it loads
    // its inputs in pipelined groups of 4.  Granule batches, one pool per
    // shape, builds alternated (tools/gpu_gen.sh, profiles/r3/gen_r3s2q.txt),
    // best group-of-1 build (the round-2 kernel, uncapped) -> groups of 4 here:
    // 17+3 encode 0.742 -> 0.759, {0,1,2} 0.742 -> 0.762; 8+4 encode 0.797 ->
    // 0.805; 8+4 decode {0} 0.69 -> 0.772 (at 12544); 6+3 encode 0.811 -> 0.84,
    // {0,1} 0.80 -> 0.852.  Verify stays uncapped (as 10+4 verify).
    if (verify) return 0;
    return m == 1 ? 12544 : 10240;
}

// The same cap for the per-stripe-pattern kernels (gf_masked_kernel), granule
// batches with a random pattern per stripe (tools/occ_sweep2.py --family
// masked, profiles/r3/occ_sweep2_r3zt.txt): config[4] 0.797 uncapped, 0.824
// at 12544 B; 4+2 x 1 MiB 0.80 -> 0.829 at 12544; 10+4 x 4 MiB with 4 erasures
// 0.76-0.79 -> 0.80-0.806 at 10240.  (The copy kernel, two streams per wave,
// is best uncapped: 0.851, and 0.78 at 10240.)
// The runtime-k masked kernel (other k, called with k = 0 or the code's k)
// takes 10240 since it loads in pipelined groups (tools/occ_sweep2.py --family
// masked, profiles/r3/masked_gen_r3s2t.txt; granule batches, random erasures
// per stripe, one-input-ahead build uncapped -> groups of 4 at 10240): 6+3
// 0.77-0.78 -> 0.833, 8+4 0.72 -> 0.72-0.725, 17+3 0.71-0.75 -> 0.73.
size_t masked_lds_pad(int k, int ms) {
    (void)ms;
    return tuning_size("RSAMD_MASKED_LDS_PAD", k == 4 ? 12544 : 10240);
}

template <int K, int M>
hipError_t launch_vec_t(VecArgs a, Mode mode, hipStream_t s) {
    const size_t lds = vec_lds_pad(K, M, mode == Mode::Verify);
    if (mode == Mode::Verify)
        hipLaunchKernelGGL((gf_vec_kernel<K, M, true>), dim3(a.n_items), dim3(kWave), lds, s, a);
    else
        hipLaunchKernelGGL((gf_vec_kernel<K, M, false>), dim3(a.n_items), dim3(kWave), lds, s, a);
    return hipGetLastError();
}

template <int M>
hipError_t launch_vec_generic_t(VecArgs a, Mode mode, hipStream_t s) {
    if (mode == Mode::Verify)
        hipLaunchKernelGGL((gf_vec_generic_kernel<M, true>), dim3(a.n_items), dim3(kWave), vec_lds_pad(0, M, true), s, a);
    else
        hipLaunchKernelGGL((gf_vec_generic_kernel<M, false>), dim3(a.n_items), dim3(kWave), vec_lds_pad(0, M, false), s, a);
    return hipGetLastError();
}

// Compile-time shapes for the BASELINE geometries (4+2 and 10+4 with any
// erasure count), and for 6+m, 8+m and 17+m (the common wider codes and the
// upstream library's benchmark code); every other shape runs the runtime-k
// kernel, capped and in plain order like them (block_order: capped).
hipError_t dispatch_vec(VecArgs a, int nout, Mode mode, hipStream_t s) {
#define RSAMD_CASE(K, M) \
    if (a.nin == K && nout == M) return launch_vec_t<K, M>(a, mode, s);
    RSAMD_CASE(4, 1) RSAMD_CASE(4, 2) RSAMD_CASE(4, 3) RSAMD_CASE(4, 4)
    RSAMD_CASE(10, 1) RSAMD_CASE(10, 2) RSAMD_CASE(10, 3) RSAMD_CASE(10, 4)
    RSAMD_CASE(17, 1) RSAMD_CASE(17, 2) RSAMD_CASE(17, 3)
    RSAMD_CASE(6, 1) RSAMD_CASE(6, 2) RSAMD_CASE(6, 3)
    RSAMD_CASE(8, 1) RSAMD_CASE(8, 2) RSAMD_CASE(8, 3) RSAMD_CASE(8, 4)
#undef RSAMD_CASE
    switch (nout) {
    case 1: return launch_vec_generic_t<1>(a, mode, s);
    case 2: return launch_vec_generic_t<2>(a, mode, s);
    case 3: return launch_vec_generic_t<3>(a, mode, s);
    case 4: return launch_vec_generic_t<4>(a, mode, s);
    }
    return hipErrorInvalidValue;
}

// Block order of a launch (block_item): a table tuned on MI355X with the real
// encode kernel (tools/sweep_order.sh, tools/ab_order_encode.sh; results in
// profiles/r1/block_order_sweep.txt), fraction of HBM peak:
//
//   shards x size     stripe-major   XCD-contiguous   rotation (~3/8 stripe)
//   4+2  x 16 KiB         0.78           0.81              0.73
//   4+2  x 256 KiB        0.78           0.81              0.75
//   4+2  x 512 KiB        0.77           0.80              0.79
//   4+2  x 1 MiB          0.78           0.79              0.81-0.82
//   4+2  x 2 MiB          0.77           0.79              0.69-0.70
//   4+2  x 4 MiB          0.76           0.77              0.76
//   4+2  x 8 MiB          0.74           0.79              0.73
//   10+4 x 1 MiB          0.73           0.73              0.77
//   10+4 x 4 MiB          0.70           0.70              0.72
//   4+2  x 4 KiB          0.72           0.80              --
//   4+2  x 1 MiB + 1 KiB pad   0.75      0.80              0.75
//   4+2  x 1 MiB + 4 KiB pad   0.62      0.78              0.74
//   10+4 x 4 MiB + 4 KiB pad   0.75      0.71              0.74
//
// On a physically contiguous pool (rs_dev_alloc; profiles/r1/order_ab/
// orders_contiguous_pool*.txt, 512k_rotation.txt) the table holds except at
// 512 KiB, where a quarter-stripe rotation (127 chunks; 3/8 = 191 gives 0.78)
// reaches 0.809 against 0.791 for the XCD remap (0.787 / 0.785 on hipMalloc).
//
// The XCD-contiguous remap is the default; rotation wins at 512 KiB and 1 MiB
// shards on stripe-aligned strides and for wide (>= 14-shard) stripes of
// >= 1 MiB, and loses badly elsewhere (2 MiB, padded strides), so it is used
// exactly there.  In a TUNING=1 build (tuning.hpp) RSAMD_BLOCK_ROT (rotation
// in chunks, 0 = off) and RSAMD_BLOCK_XCD (0 / 1) override the table for A/B runs.  (Remapping
// within groups of 8 * N blocks instead of the whole launch measured worse.)
struct BlockOrder {
    uint32_t rot, xcd_span;
};

// With an occupancy cap (vec_lds_pad / masked_lds_pad > 0: `capped`) plain
// order wins everywhere it was measured (tools/occ_sweep.py --cross,
// profiles/r3/occ_order_r3zy.txt; tools/pattern_sweep.py,
// profiles/r3/order_caps_r3zz.txt): 4+2 granule encode 0.874 against 0.863
// with the XCD remap, every 4+2 decode pattern 0.851-0.878 against
// 0.817-0.861, per-stripe patterns 0.848-0.861 against 0.824-0.833; 4+2 packed
// 0.869 against 0.863 rotated; 10+4 granule 0.810 against 0.808 and packed
// x 128 0.774 against 0.770.  The table above stays for uncapped launches.
BlockOrder block_order(uint32_t chunks, uint32_t total_shards, uint64_t shard_stride, uint32_t n_items,
                       int nout = 0, bool capped = false) {
    // read at every launch (TUNING builds only): sweeps change them between legs
    const char *er = tuning_env("RSAMD_BLOCK_ROT"), *ex = tuning_env("RSAMD_BLOCK_XCD");
    const int env_rot = er ? std::atoi(er) : -1;
    const int env_xcd = ex ? std::atoi(ex) : -1;
    const bool half = chunks == 512 && shard_stride % (uint64_t(512) << 10) == 0;
    // Wide stripes (>= 14 shards of >= 1 MiB): rotation up to 256 stripes per
    // launch, the XCD remap beyond (10+4 x 4 MiB on contiguous pools: 128 and
    // 256 stripes 0.72-0.75 rotated vs 0.70-0.71 remapped; 512 a tie at 0.70;
    // 1024 0.753 remapped vs 0.70 rotated -- profiles/r2/order_pad_*.txt).
    const uint32_t stripes = n_items / std::max(1u, chunks);
    const bool rotate = (chunks == 1024 && shard_stride % (uint64_t(1) << 20) == 0) || half ||
                        (total_shards >= 14 && chunks >= 1024 && stripes <= 256);
    const uint32_t step = half ? chunks / 4u - 1u : 3u * chunks / 8u - 1u;
    const uint32_t rot = env_rot >= 0 ? uint32_t(env_rot) : (rotate ? step : 0u);
    // The 4+2 granule view (64 KiB granules) keeps the XCD remap.  Plain order
    // read +0.5 points for two-output plans on one box (encode 0.850-0.851 vs
    // 0.845-0.847 in fresh processes, profiles/r2/order_ab_headline_r2bs.txt)
    // but -0.3 on another (0.842 vs 0.845 on one pool, granule_decode_r2bu.txt)
    // with one 0.841 run among four (placement_layouts_r2br.txt); the remap read
    // 0.8444-0.8467 on every box and process.  nout is kept for such rules.
    (void)nout;
    const bool xcd = env_xcd >= 0 ? env_xcd != 0 : !rotate;
    // (Not for packed wide stripes beyond 256: 10+4 x 4 MiB x 1024 keeps the
    // XCD remap, 0.775 against 0.762 plain.)
    const bool wide_many = total_shards >= 14 && chunks >= 1024 && stripes > 256;
    if (capped && !wide_many && env_rot < 0 && env_xcd < 0) return BlockOrder{0u, 0u};
    return BlockOrder{chunks > 1 ? rot % chunks : 0u, xcd ? n_items / 8u : 0u};
}

hipError_t launch_bytes(const Geometry &g, const DevPlan &p, size_t col0, size_t ncols, Mode mode, int *mismatch,
                        hipStream_t s) {
    ByteArgs a{g.base, p.tabs, p.in_idx, p.out_idx, g.stripe_stride, g.shard_stride, col0, ncols,
               uint64_t(g.n_stripes) * ncols, p.nin, p.nout, mismatch};
    if (a.total == 0) return hipSuccess;
    const uint64_t want = (a.total + kThreads - 1) / kThreads;
    const unsigned grid = unsigned(std::min<uint64_t>(want, 65536));
    if (mode == Mode::Verify)
        hipLaunchKernelGGL((gf_byte_kernel<true>), dim3(grid), dim3(kThreads), 0, s, a);
    else
        hipLaunchKernelGGL((gf_byte_kernel<false>), dim3(grid), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

// PAT (a.pat_on) is a template argument, not a uniform branch.  As a branch
// in one kernel, the pattern divide changed the 10+4 kernel's register
// allocation (scratch 20 -> 8 B per lane).  On one pool that build ran packed
// batches at 0.727 against 0.754 and the granule view at 0.796 against 0.752
// (tools/masked_ab.py, profiles/r2/ab/masked_ab_r2bc.txt).  As a template,
// PAT = false compiles to the old kernel instruction for instruction and
// PAT = true (granule batches, the only callers of pattern_bytes) keeps the
// faster allocation: 0.78-0.79 against 0.75 for the view with repeated
// patterns on one pool (masked_ab_r2bd.txt).
template <int K, int MS>
hipError_t launch_masked_t(const MaskedArgs &a, hipStream_t s) {
    if (a.pat_on)
        hipLaunchKernelGGL((gf_masked_kernel<K, MS, true>), dim3(a.n_items), dim3(kWave), masked_lds_pad(K, MS), s, a);
    else
        hipLaunchKernelGGL((gf_masked_kernel<K, MS, false>), dim3(a.n_items), dim3(kWave), masked_lds_pad(K, MS), s, a);
    return hipGetLastError();
}

template <int MS>
hipError_t launch_masked_generic_t(const MaskedArgs &a, hipStream_t s) {
    if (a.pat_on)
        hipLaunchKernelGGL((gf_masked_generic_kernel<MS, true>), dim3(a.n_items), dim3(kWave), masked_lds_pad(0, MS), s, a);
    else
        hipLaunchKernelGGL((gf_masked_generic_kernel<MS, false>), dim3(a.n_items), dim3(kWave), masked_lds_pad(0, MS), s, a);
    return hipGetLastError();
}

// RSAMD_MASKED_WIDE=0 routes k = 10 to the runtime-k masked kernel (A/B runs).
bool masked_wide_enabled() {
    static const bool on = [] {
        const char *e = tuning_env("RSAMD_MASKED_WIDE");
        return !(e && e[0] == '0');
    }();
    return on;
}

hipError_t dispatch_masked(const MaskedArgs &a, int ms, hipStream_t s) {
#define RSAMD_CASE(K, M) \
    if (a.nin == K && ms == M) return launch_masked_t<K, M>(a, s);
    // k = 10 (10+4, 4 erasures per stripe, tools/masked_wide_probe.py):
    // 0.66 of peak, against 0.62 for the runtime-k kernel.
    RSAMD_CASE(4, 1) RSAMD_CASE(4, 2) RSAMD_CASE(4, 3) RSAMD_CASE(4, 4)
    if (masked_wide_enabled()) {
        RSAMD_CASE(10, 1) RSAMD_CASE(10, 2) RSAMD_CASE(10, 3) RSAMD_CASE(10, 4)
    }
#undef RSAMD_CASE
    switch (ms) {
    case 1: return launch_masked_generic_t<1>(a, s);
    case 2: return launch_masked_generic_t<2>(a, s);
    case 3: return launch_masked_generic_t<3>(a, s);
    case 4: return launch_masked_generic_t<4>(a, s);
    }
    return hipErrorInvalidValue;
}

template <int K, int MS>
hipError_t launch_masked8_t(const MaskedArgs &a, hipStream_t s) {
    hipLaunchKernelGGL((gf_masked8_kernel<K, MS>), dim3(a.n_items), dim3(kWave), tuning_size("RSAMD_MASKED8_LDS_PAD", 0),
                       s, a);
    return hipGetLastError();
}

hipError_t dispatch_masked8(const MaskedArgs &a, int ms, hipStream_t s) {
    const bool k4 = a.nin == 4;
    switch (ms) {
    case 1: return k4 ? launch_masked8_t<4, 1>(a, s) : launch_masked8_t<0, 1>(a, s);
    case 2: return k4 ? launch_masked8_t<4, 2>(a, s) : launch_masked8_t<0, 2>(a, s);
    case 3: return k4 ? launch_masked8_t<4, 3>(a, s) : launch_masked8_t<0, 3>(a, s);
    case 4: return k4 ? launch_masked8_t<4, 4>(a, s) : launch_masked8_t<0, 4>(a, s);
    }
    return hipErrorInvalidValue;
}

template <int K, int M>
hipError_t launch_vec8_t(const Vec8Args &a, Mode mode, hipStream_t s) {
    if (mode == Mode::Verify)
        hipLaunchKernelGGL((gf_vec8_kernel<K, M, true>), dim3(a.v.n_items), dim3(kWave), tuning_size("RSAMD_VEC8_LDS_PAD", 0),
                           s, a);
    else
        hipLaunchKernelGGL((gf_vec8_kernel<K, M, false>), dim3(a.v.n_items), dim3(kWave), tuning_size("RSAMD_VEC8_LDS_PAD", 0),
                           s, a);
    return hipGetLastError();
}

hipError_t dispatch_vec8(const Vec8Args &a, int nout, Mode mode, hipStream_t s) {
    const bool k4 = a.v.nin == 4;
    switch (nout) {
    case 1: return k4 ? launch_vec8_t<4, 1>(a, mode, s) : launch_vec8_t<0, 1>(a, mode, s);
    case 2: return k4 ? launch_vec8_t<4, 2>(a, mode, s) : launch_vec8_t<0, 2>(a, mode, s);
    case 3: return k4 ? launch_vec8_t<4, 3>(a, mode, s) : launch_vec8_t<0, 3>(a, mode, s);
    case 4: return k4 ? launch_vec8_t<4, 4>(a, mode, s) : launch_vec8_t<0, 4>(a, mode, s);
    }
    return hipErrorInvalidValue;
}

template <int K, int MS, bool MASKED>
hipError_t launch_group8_t(const GroupArgs &a, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((gf_group8_kernel<K, MS, MASKED>), dim3(a.n_items), dim3(kWave), lds, s, a);
    return hipGetLastError();
}

// RSAMD_GROUP8=0 (TUNING builds) keeps such batches on the 8-byte kernels (A/B runs).
bool group8_enabled() {
    static const bool on = [] {
        const char *e = tuning_env("RSAMD_GROUP8");
        return !(e && e[0] == '0');
    }();
    return on;
}

// LDS of one wave: the nin input slots, reused for the output runs (at worst
// one run per output, each rounded out to lines).
// The LDS a launch asks per wave also caps the waves per CU, and the two
// forms want different caps (4 M groups of 4+2 x 1000 B, extra LDS per wave
// on top of the 5 KiB the inputs need; profiles/r3/cg_pad_r3k.txt):
//   extra LDS                     0      1 KiB   2.5 KiB   5 KiB
//   waves per CU                 32       26       21       16
//   encode / decode {0,1}       0.708    0.726    0.730    0.692
//   per-group bitmasks          0.667    0.635    0.585    0.503
// One plan for every group: all its waves stream, and fewer of them in flight
// keep DRAM pages open longer; per-group records: each wave first waits for a
// chain of dependent scalar loads, and more waves hide it.  So a uniform plan
// asks for (nin + ms) slots (21 waves per CU), per-group records for the
// max(nin, ms) slots they use (32).
#ifndef RSAMD_GROUP_LDS_PAD
#define RSAMD_GROUP_LDS_PAD 0  // extra LDS bytes per wave (A/B builds)
#endif
#ifndef RSAMD_GROUP_LDS_MODE
#define RSAMD_GROUP_LDS_MODE 0  // A/B: 0 per form (below), 1 both at max(nin, ms) slots, 2 both at nin + ms
#endif
size_t group8_lds(size_t len, int nin, int ms, bool masked) {
    const size_t slot = (len + 256 + 15) / 16 * 16;
    const bool wide = RSAMD_GROUP_LDS_MODE == 2 || (RSAMD_GROUP_LDS_MODE == 0 && !masked);
    return (wide ? size_t(nin + ms) : std::max(size_t(nin), size_t(ms))) * slot +
           tuning_size("RSAMD_GROUP_LDS_PAD_ENV", RSAMD_GROUP_LDS_PAD);  // per launch in TUNING builds
}

// The line-owner kernel takes k = 4 codes on stripes of back-to-back shards
// (shard stride = shard length, stripe stride = total shards x that) of
// 8-byte multiples >= 256 bytes, 8-byte but not 16-byte aligned (aligned
// batches keep the 16-byte kernels), small enough for LDS.
constexpr size_t kGroupLdsMax = 32768;
bool group8_geometry(const Geometry &g, int nin, int ms) {
    const uintptr_t b = reinterpret_cast<uintptr_t>(g.base);
    return nin == 4 && ms >= 1 && ms <= kMaxOut && g.total > 0 && g.col0 == 0 && g.len == g.shard_stride &&
           g.len % 8 == 0 && g.len >= 256 && g.len <= kGroupMaxLen && b % 8 == 0 &&
           g.stripe_stride == size_t(g.total) * g.len && group8_lds(g.len, nin, ms, false) <= kGroupLdsMax &&
           group8_enabled();
}

template <bool MASKED>
hipError_t launch_group8(const Geometry &g, GroupArgs a, int ms, hipStream_t s) {
    const size_t lds = group8_lds(g.len, 4, ms, MASKED);
    a.stripe_stride = g.stripe_stride;
    a.lo = g.base;
    a.hi = g.base + g.n_stripes * g.stripe_stride;
    // Phase 0 reads whole 128-byte lines, so the batch's first and last line
    // may be read past its ends (never written there: a foreign byte is
    // written back only inside the batch).  A line never crosses a page.
    const uintptr_t line_lo = reinterpret_cast<uintptr_t>(a.lo) & ~uintptr_t(127);
    bounds::allow(a.lo, size_t(a.hi - a.lo));
    bounds::allow(reinterpret_cast<const void *>(line_lo),
                  ((reinterpret_cast<uintptr_t>(a.hi) + 127) & ~uintptr_t(127)) - line_lo, false);
    a.len = uint32_t(g.len);
    a.total = uint32_t(g.total);
    const int32_t *ids0 = a.plan_ids;
    for (size_t t0 = 0; t0 < g.n_stripes; t0 += kMaxGridBlocks) {
        const size_t nst = std::min<size_t>(kMaxGridBlocks, g.n_stripes - t0);
        a.base = g.base + t0 * g.stripe_stride;
        a.n_items = uint32_t(nst);
        const char *gx = tuning_env("RSAMD_GROUP_XCD");  // A/B (TUNING builds): 0 = plain order
        a.xcd_span = gx && gx[0] == '0' ? 0u : uint32_t(nst / 8);
        a.plan_ids = ids0 ? ids0 + t0 : nullptr;
        a.has_prev = t0 > 0;
        a.has_next_last = t0 + nst < g.n_stripes;
        hipError_t e = hipErrorInvalidValue;
        switch (ms) {
        case 1: e = launch_group8_t<4, 1, MASKED>(a, lds, s); break;
        case 2: e = launch_group8_t<4, 2, MASKED>(a, lds, s); break;
        case 3: e = launch_group8_t<4, 3, MASKED>(a, lds, s); break;
        case 4: e = launch_group8_t<4, 4, MASKED>(a, lds, s); break;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// Lanes per stripe of the 8-byte-aligned kernels and the bytes they cover:
// whole 16-byte vectors plus a half, or 8-byte vectors.
struct Lanes8 {
    uint32_t nvec, nfull16;
    size_t covered;
};
Lanes8 lanes8(size_t len, bool u16) {
    if (u16) {
        const size_t full = len / 16, half = (len % 16) >= 8 ? 1 : 0;
        return Lanes8{uint32_t(full + half), uint32_t(full), full * 16 + half * 8};
    }
    return Lanes8{uint32_t(len / 8), 0, len / 8 * 8};
}

// `counts`: this launch covers the first column of its call's range, and
// counts each undecodable stripe there (per-stripe patterns).  A launch that
// codes a tail or a head peel's remainder does not: every stripe is counted
// once per call (include/rs_amd.h rs_decode_batch_masked_bits_dev).
hipError_t launch_masked_bytes(const Geometry &g, const MaskedPlan &p, const MaskedRecordLayout &l, size_t col0,
                               size_t ncols, bool counts, hipStream_t s) {
    MaskedByteArgs a{g.base, p.records, p.rec_stride, p.plan_ids, g.stripe_stride, g.shard_stride, col0, ncols,
                     uint64_t(g.n_stripes) * ncols, uint32_t(l.in_idx), uint32_t(l.out_idx), uint32_t(l.tabs),
                     p.nin, p.mslots, p.mask_table, p.mask_bits, p.bad, p.pattern_bytes, g.col0 + g.len,
                     counts ? uint64_t(col0) : UINT64_MAX};
    if (a.total == 0) return hipSuccess;
    const unsigned grid = unsigned(std::min<uint64_t>((a.total + kThreads - 1) / kThreads, 65536));
    hipLaunchKernelGGL(gf_masked_byte_kernel, dim3(grid), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace

namespace {

// Shards of a few KiB whose length leaves an 8-byte remainder after the
// 16-byte vectors (S = 1000 at stride 1008 or 1024) take the 8-byte kernels
// even when 16-byte aligned: one launch instead of the 16-byte kernel plus a
// byte-kernel tail launch, 0.59 of peak against 0.54 at stride 1008
// (profiles/r2/chunk_groups_r2bl.txt).
bool small_with_tail8(size_t len) { return len % 16 == 8 && len < 16384; }

// RSAMD_MASKED8=0 sends 8-byte-aligned batches to the byte kernel (A/B runs).
bool masked8_enabled() {
    static const bool on = [] {
        const char *e = tuning_env("RSAMD_MASKED8");
        return !(e && e[0] == '0');
    }();
    return on;
}

// 8-byte vectors (gf_masked8_kernel), then the < 8-byte tail on the byte kernel.
hipError_t launch_masked8(const Geometry &g, const MaskedPlan &p, const MaskedRecordLayout &l, hipStream_t s) {
    uint8_t *base = g.base + g.col0;
    const Lanes8 n = lanes8(g.len, RSAMD_MASKED8_U16);
    if (n.nvec > 0) {
        const uint32_t chunks = (n.nvec + kWave - 1) / kWave;
        const size_t stripes_per_launch = std::max<size_t>(1, kMaxGridBlocks / chunks);
        for (size_t t0 = 0; t0 < g.n_stripes; t0 += stripes_per_launch) {
            const size_t nst = std::min(stripes_per_launch, g.n_stripes - t0);
            const BlockOrder o = block_order(chunks, uint32_t(g.stripe_stride / std::max<size_t>(1, g.shard_stride)),
                                             g.shard_stride, uint32_t(nst * chunks));
            // pat_chunk0 carries nfull16 (the 8-byte kernels take no per-row patterns)
            MaskedArgs a{base + t0 * g.stripe_stride, p.records, p.rec_stride, p.plan_ids + t0, g.stripe_stride,
                         g.shard_stride, n.nvec, chunks, uint32_t(nst * chunks), o.rot, o.xcd_span,
                         make_fastdiv(chunks), uint32_t(l.in_idx), uint32_t(l.out_idx), uint32_t(l.tabs), p.nin,
                         p.mask_table, p.mask_bits, p.bad, 0u, n.nfull16, make_fastdiv(1), 1u};
            hipError_t e = dispatch_masked8(a, p.mslots, s);
            if (e != hipSuccess) return e;
        }
    }
    if (n.covered < g.len) return launch_masked_bytes(g, p, l, g.col0 + n.covered, g.len - n.covered, false, s);
    return hipSuccess;
}

// Columns to code on the byte kernel before the vector kernels (0: none).
size_t head_peel(const Geometry &g) {
    // Head peel: the first columns on the byte kernel, so the rest starts on a
    // boundary every shard shares (strides its multiples).
    //  * For batches of >= 256 MiB of columns: a wave's 1 KiB (else a 128-B
    //    line, for strides that are line but not 1 KiB multiples), so each
    //    wave covers whole lines instead of sharing a partial line with each
    //    neighbour; at most 1/1024 of a shard is peeled.  4+2 x 1 MiB x 1024
    //    stripes 16 / 112 / 1008 B past a line: 0.72 / 0.71 / 0.71 of peak
    //    unpeeled, 0.855 / 0.855 / 0.865 peeled to 1 KiB (0.848 / 0.848 /
    //    0.864 to 128 B; 0.867 line-aligned).  A shard-major recovery run that
    //    starts at group 2 M + 1 (rs_decode_groups_shard_major_dev) 0.674 ->
    //    0.795 (profiles/r4/line_peel_r4p.txt).
    //  * Else 16 B for a batch 8 bytes off (then the 16-byte kernels, not the
    //    8-byte ones).
    // RSAMD_LINE_PEEL (TUNING builds): 0 = no line peel, A = peel to A only.
    const uintptr_t addr = reinterpret_cast<uintptr_t>(g.base + g.col0);
    auto strides_multiple = [&](size_t a) {
        return g.shard_stride % a == 0 && (g.n_stripes == 1 || g.stripe_stride % a == 0);
    };
    size_t peel = 0;
    if (uint64_t(g.n_stripes) * g.len >= kLinePeelMinBytes) {
        const size_t forced = tuning_size("RSAMD_LINE_PEEL", SIZE_MAX);
        const size_t order[2] = {forced != SIZE_MAX ? forced : 1024, forced != SIZE_MAX ? forced : 128};
        for (size_t line : order) {
            if (line == 0 || !strides_multiple(line)) continue;
            if (addr % line == 0) break;  // already on the boundary
            const size_t n = line - addr % line;
            if (n * 1024 <= g.len) {
                peel = n;
                break;
            }
        }
    }
    if (!peel && addr % 16 == 8 && strides_multiple(16) && g.len >= kSmallBytes) peel = 8;
    return peel;
}

}  // namespace

MaskedRecordLayout masked_record_layout(int nin, int mslots) {
    MaskedRecordLayout l;
    l.in_idx = 16;
    l.out_idx = l.in_idx + size_t(nin) * 4;
    l.tabs = (l.out_idx + size_t(mslots) * 4 + 15) / 16 * 16;
    l.bytes = (l.tabs + size_t(nin) * mslots * 20 + 15) / 16 * 16;
    return l;
}

hipError_t launch_gf_masked(const Geometry &g, const MaskedPlan &p, hipStream_t s) {
    if (g.n_stripes == 0 || g.len == 0) return hipSuccess;
    if (p.mslots < 1 || p.mslots > kMaxOut || p.nin < 1) return hipErrorInvalidValue;
    const MaskedRecordLayout l = masked_record_layout(p.nin, p.mslots);
    uint8_t *base = g.base + g.col0;
    // (one stripe: its stripe stride is never used)
    const bool aligned = (reinterpret_cast<uintptr_t>(base) % 16 == 0) && g.shard_stride % 16 == 0 &&
                         (g.n_stripes == 1 || g.stripe_stride % 16 == 0);
    // Patterns per logical stripe: the vector kernels need every 1 KiB chunk
    // inside one pattern (rows of whole 1 KiB chunks, patterns of whole rows
    // or of whole chunks) and the batch's chunk count in 32 bits.
    const size_t chunk_bytes = size_t(kWave) * 16;
    const size_t pb = p.pattern_bytes;
    const bool pat_vec = pb == 0 || (g.col0 == 0 && g.len % chunk_bytes == 0 && pb % chunk_bytes == 0 &&
                                     (pb % g.len == 0 || g.len % pb == 0) &&
                                     g.n_stripes * (g.len / chunk_bytes) <= UINT32_MAX);
    const bool aligned8 = (reinterpret_cast<uintptr_t>(base) % 8 == 0) && g.shard_stride % 8 == 0 &&
                          (g.n_stripes == 1 || g.stripe_stride % 8 == 0);
    // Head peel as launch_gf_tables (per-stripe patterns only: granule
    // patterns are tied to the columns' 1 KiB chunks).
    if (const size_t peel = pb == 0 ? head_peel(g) : 0) {
        hipError_t e = launch_masked_bytes(g, p, l, g.col0, peel, true, s);
        if (e != hipSuccess) return e;
        Geometry rest = g;
        rest.col0 += peel;
        rest.len -= peel;
        MaskedPlan rp = p;
        rp.bad = nullptr;  // counted by the peel's launch
        return launch_gf_masked(rest, rp, s);
    }
    // (the line-owner kernel reads a stripe's outputs off its bitmask: a
    // pattern table, and every pattern's absent shards in one launch group)
    if (aligned8 && !aligned && pb == 0 && p.mask_table && g.total > 0 && p.mslots >= g.total - p.nin &&
        group8_geometry(g, p.nin, p.mslots)) {
        GroupArgs a{};
        a.records = p.records;
        a.rec_stride = p.rec_stride;
        a.plan_ids = p.plan_ids;
        a.mask_table = p.mask_table;
        a.mask_bits = p.mask_bits;
        a.bad = p.bad;
        a.rec_in_idx = uint32_t(l.in_idx);
        a.rec_out_idx = uint32_t(l.out_idx);
        a.rec_tabs = uint32_t(l.tabs);
        return launch_group8<true>(g, a, p.mslots, s);
    }
    if (aligned8 && pb == 0 && (!aligned || small_with_tail8(g.len)) && g.len / 8 <= UINT32_MAX - kWave &&
        masked8_enabled())
        return launch_masked8(g, p, l, s);
    if (!aligned || !pat_vec || g.len / 16 > UINT32_MAX - kWave)
        return launch_masked_bytes(g, p, l, g.col0, g.len, true, s);
    const uint32_t nvec = uint32_t(g.len / 16);
    if (nvec > 0) {
        const uint32_t chunks = (nvec + kWave - 1) / kWave;
        const uint32_t pat_chunks = pb ? uint32_t(pb / chunk_bytes) : 1u;
        const size_t stripes_per_launch = std::max<size_t>(1, kMaxGridBlocks / chunks);
        for (size_t t0 = 0; t0 < g.n_stripes; t0 += stripes_per_launch) {
            const size_t nst = std::min(stripes_per_launch, g.n_stripes - t0);
            const BlockOrder o = block_order(chunks, uint32_t(g.stripe_stride / std::max<size_t>(1, g.shard_stride)),
                                             g.shard_stride, uint32_t(nst * chunks), 0,
                                             masked_lds_pad(p.nin, p.mslots) > 0);
            MaskedArgs a{base + t0 * g.stripe_stride, p.records, p.rec_stride, p.plan_ids + (pb ? 0 : t0),
                         g.stripe_stride, g.shard_stride, nvec, chunks, uint32_t(nst * chunks), o.rot, o.xcd_span,
                         make_fastdiv(chunks), uint32_t(l.in_idx), uint32_t(l.out_idx), uint32_t(l.tabs), p.nin, p.mask_table,
                         p.mask_bits, p.bad, pb ? 1u : 0u, uint32_t(t0 * chunks), make_fastdiv(pat_chunks), pat_chunks};
            hipError_t e = dispatch_masked(a, p.mslots, s);
            if (e != hipSuccess) return e;
        }
    }
    const size_t tail = g.len % 16;
    if (tail) return launch_masked_bytes(g, p, l, g.col0 + size_t(nvec) * 16, tail, false, s);
    return hipSuccess;
}

namespace {

// The table-lookup (v_perm_b32) kernels: any plan, any geometry.
hipError_t launch_vec8(const Geometry &g, const DevPlan &p, Mode mode, int *mismatch, hipStream_t s);

hipError_t launch_gf_tables(const Geometry &g, const DevPlan &p, Mode mode, int *mismatch, hipStream_t s) {
    if (g.n_stripes == 0 || g.len == 0 || p.nout == 0) return hipSuccess;
    if (p.nout > kMaxOut || p.nin < 1) return hipErrorInvalidValue;
    uint8_t *base = g.base + g.col0;
    // (one stripe: its stripe stride is never used)
    const bool aligned = (reinterpret_cast<uintptr_t>(base) % 16 == 0) && g.shard_stride % 16 == 0 &&
                         (g.n_stripes == 1 || g.stripe_stride % 16 == 0);
    const bool aligned8 = (reinterpret_cast<uintptr_t>(base) % 8 == 0) && g.shard_stride % 8 == 0 &&
                          (g.n_stripes == 1 || g.stripe_stride % 8 == 0);
    // Head peel (head_peel): the rest starts on a boundary every shard shares.
    const size_t peel = head_peel(g);
    if (peel) {
        hipError_t e = launch_bytes(g, p, g.col0, peel, mode, mismatch, s);
        if (e != hipSuccess) return e;
        Geometry rest = g;
        rest.col0 += peel;
        rest.len -= peel;
        return launch_gf_tables(rest, p, mode, mismatch, s);
    }
    if (aligned8 && !aligned && mode == Mode::Code && uint64_t(g.n_stripes) * g.len > kSmallBytes &&
        group8_geometry(g, p.nin, p.nout)) {
        GroupArgs a{};
        a.tabs = p.tabs;
        a.in_idx = p.in_idx;
        a.out_idx = p.out_idx;
        return launch_group8<false>(g, a, p.nout, s);
    }
    if (aligned8 && (!aligned || small_with_tail8(g.len)) && uint64_t(g.n_stripes) * g.len > kSmallBytes &&
        g.len / 8 <= UINT32_MAX - kWave && masked8_enabled())
        return launch_vec8(g, p, mode, mismatch, s);
    if (!aligned || g.len / 16 > UINT32_MAX - kWave) return launch_bytes(g, p, g.col0, g.len, mode, mismatch, s);
    // A few KiB of ragged columns: one byte-kernel launch instead of a vector
    // launch plus a tail launch (small host calls are launch-latency bound).
    if (g.len % 16 && uint64_t(g.n_stripes) * g.len <= kSmallBytes)
        return launch_bytes(g, p, g.col0, g.len, mode, mismatch, s);

    const uint32_t nvec = uint32_t(g.len / 16);
    if (nvec > 0) {
        const uint32_t chunks = (nvec + kWave - 1) / kWave;
        // One block per 64 vectors of a stripe; very large batches are split
        // by stripe ranges so the grid stays within kMaxGridBlocks.
        const size_t stripes_per_launch = std::max<size_t>(1, kMaxGridBlocks / chunks);
        for (size_t t0 = 0; t0 < g.n_stripes; t0 += stripes_per_launch) {
            const size_t nst = std::min(stripes_per_launch, g.n_stripes - t0);
            const BlockOrder o = block_order(chunks, uint32_t(g.stripe_stride / std::max<size_t>(1, g.shard_stride)),
                                             g.shard_stride, uint32_t(nst * chunks), mode == Mode::Code ? p.nout : 0,
                                             vec_lds_pad(p.nin, p.nout, mode == Mode::Verify) > 0);
            VecArgs a{base + t0 * g.stripe_stride, p.tabs, p.in_idx, p.out_idx, g.stripe_stride, g.shard_stride,
                      nvec, chunks, uint32_t(nst * chunks), o.rot, o.xcd_span, make_fastdiv(chunks), p.nin,
                      mismatch};
            hipError_t e = dispatch_vec(a, p.nout, mode, s);
            if (e != hipSuccess) return e;
        }
    }
    const size_t tail = g.len % 16;
    if (tail) return launch_bytes(g, p, g.col0 + size_t(nvec) * 16, tail, mode, mismatch, s);
    return hipSuccess;
}

// 8-byte vectors (gf_vec8_kernel), then the < 8-byte tail on the byte kernel.
hipError_t launch_vec8(const Geometry &g, const DevPlan &p, Mode mode, int *mismatch, hipStream_t s) {
    uint8_t *base = g.base + g.col0;
    const Lanes8 n = lanes8(g.len, RSAMD_VEC8_U16);
    if (n.nvec > 0) {
        const uint32_t chunks = (n.nvec + kWave - 1) / kWave;
        const size_t stripes_per_launch = std::max<size_t>(1, kMaxGridBlocks / chunks);
        for (size_t t0 = 0; t0 < g.n_stripes; t0 += stripes_per_launch) {
            const size_t nst = std::min(stripes_per_launch, g.n_stripes - t0);
            const BlockOrder o = block_order(chunks, uint32_t(g.stripe_stride / std::max<size_t>(1, g.shard_stride)),
                                             g.shard_stride, uint32_t(nst * chunks));
            Vec8Args a{{base + t0 * g.stripe_stride, p.tabs, p.in_idx, p.out_idx, g.stripe_stride, g.shard_stride,
                        n.nvec, chunks, uint32_t(nst * chunks), o.rot, o.xcd_span, make_fastdiv(chunks), p.nin,
                        mismatch},
                       n.nfull16};
            hipError_t e = dispatch_vec8(a, p.nout, mode, s);
            if (e != hipSuccess) return e;
        }
    }
    if (n.covered < g.len) return launch_bytes(g, p, g.col0 + n.covered, g.len - n.covered, mode, mismatch, s);
    return hipSuccess;
}

}  // namespace

hipError_t launch_gf(const Geometry &g, const DevPlan &p, Mode mode, int *mismatch, hipStream_t s) {
    return launch_gf_tables(g, p, mode, mismatch, s);
}

namespace {
template <int W, int M>
void launch_direct_t(const DirectArgs &a, unsigned grid, Mode mode, bool pre, hipStream_t s) {
    if (mode == Mode::Verify && pre)
        hipLaunchKernelGGL((gf_direct_kernel<W, M, true, false, true>), dim3(grid), dim3(kThreads), 0, s, a);
    else if (mode == Mode::Verify)
        hipLaunchKernelGGL((gf_direct_kernel<W, M, true, false, false>), dim3(grid), dim3(kThreads), 0, s, a);
    else if (a.tee.file)
        hipLaunchKernelGGL((gf_direct_kernel<W, M, false, true, false>), dim3(grid), dim3(kThreads), 0, s, a);
    else if (pre)
        hipLaunchKernelGGL((gf_direct_kernel<W, M, false, false, true>), dim3(grid), dim3(kThreads), 0, s, a);
    else
        hipLaunchKernelGGL((gf_direct_kernel<W, M, false, false, false>), dim3(grid), dim3(kThreads), 0, s, a);
}
template <int W>
hipError_t dispatch_direct(const DirectArgs &a, int nout, unsigned grid, Mode mode, bool pre, hipStream_t s) {
    switch (nout) {
    case 1: launch_direct_t<W, 1>(a, grid, mode, pre, s); break;
    case 2: launch_direct_t<W, 2>(a, grid, mode, pre, s); break;
    case 3: launch_direct_t<W, 3>(a, grid, mode, pre, s); break;
    case 4: launch_direct_t<W, 4>(a, grid, mode, pre, s); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
}  // namespace

// Blocks of the direct kernel: 256 x 256 threads keep ~1 MiB of loads in
// flight, far more than the link's bandwidth-delay product.  4+2 x 64 MiB
// encode, GiB/s (tools/direct_probe.py, profiles/r3/direct_probe_r3s2f.txt):
//   blocks           64     128    256    512    1024
//   pinned          50.6   51.8   51.7   50.5   44.2
//   anonymous mmap  47.3   51.6   52.4   51.1   47.5
constexpr unsigned kDirectBlocks = 256;

hipError_t launch_gf_direct(const DirectPlan &p, size_t n, Mode mode, int *mismatch, hipStream_t s,
                            const DirectTee *tee, const DirectSignal *sig) {
    if (p.nin < 1 || p.nin > kMaxDirectIn || p.nout < 1 || p.nout > kMaxOut) return hipErrorInvalidValue;
    if (tee && (mode != Mode::Code || !tee->file || tee->blk == 0 || tee->blk % 8 || tee->k < 1 ||
                reinterpret_cast<uintptr_t>(tee->file) % 8 || reinterpret_cast<uintptr_t>(p.in[0]) % 8))
        return hipErrorInvalidValue;  // (the shards share in[0]'s residue: checked below)
    if (sig && (!sig->flag || !sig->ctr || (mode == Mode::Verify && !mismatch))) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;  // (a signalled caller checks for n == 0 first)
    // The widest vector every shard's address agrees on (same residue).
    int W = 16;
    for (int wide : {16, 8}) {
        W = wide;
        const uintptr_t r = reinterpret_cast<uintptr_t>(p.in[0]) % wide;
        bool same = true;
        for (int i = 0; i < p.nin; ++i) same = same && reinterpret_cast<uintptr_t>(p.in[i]) % wide == r;
        for (int q = 0; q < p.nout; ++q) same = same && reinterpret_cast<uintptr_t>(p.out[q]) % wide == r;
        if (same) break;
        W = 0;
    }
    if (W == 0) return hipErrorInvalidValue;  // the caller keeps the staged pipeline
    DirectArgs a{};
    for (int i = 0; i < p.nin; ++i) a.in[i] = p.in[i];
    for (int q = 0; q < p.nout; ++q) a.out[q] = p.out[q];
    a.tabs = p.tabs;
    // The vectors start at the widest power-of-two boundary (up to a 4 KiB
    // page) on which every shard agrees, so a wave's 1 KiB is whole 128-byte
    // lines of one page: numpy arrays (malloc'd 16 bytes past a page start)
    // read 48.5 GiB/s with 16-byte alignment and 52.4 with page alignment, as
    // fast as pinned buffers (tools/direct_probe.py, profiles/r3/
    // direct_probe_r3s2f.txt and r3s2g.txt).
    uintptr_t align = W;
    for (uintptr_t A = 4096; A > uintptr_t(W); A >>= 1) {
        const uintptr_t r = reinterpret_cast<uintptr_t>(p.in[0]) % A;
        bool same = true;
        for (int i = 0; i < p.nin; ++i) same = same && reinterpret_cast<uintptr_t>(p.in[i]) % A == r;
        for (int q = 0; q < p.nout; ++q) same = same && reinterpret_cast<uintptr_t>(p.out[q]) % A == r;
        if (same) {
            align = A;
            break;
        }
    }
    a.head = std::min<uint64_t>(n, (align - reinterpret_cast<uintptr_t>(p.in[0]) % align) % align);
    a.nvec = (n - a.head) / W;
    a.n = n;
    a.nin = p.nin;
    a.mismatch = mismatch;
    if (tee) a.tee = *tee;  // (head % 8 == 0: in[0] is 8-byte aligned and align >= 8)
    if (sig) a.sig = *sig;
    const uint64_t blocks = tuning_size("RSAMD_DIRECT_BLOCKS", kDirectBlocks);  // per call in TUNING builds
    unsigned grid = unsigned(std::max<uint64_t>(1, std::min<uint64_t>(blocks, (a.nvec + kThreads - 1) / kThreads)));
    // The PRE form (inputs loaded eight at a time) for signalled launches of
    // small shards; from 512 KiB the streaming form is as fast or faster
    // (4+2 encode kernel, 1 MiB shards: 131 against 145 us; 256 KiB 39.8 /
    // 39.0; 64 KiB and less PRE 2-5 us faster; profiles/r6/
    // zc_mid_kernels_r6af_r6ag.txt).  Whole calls, PRE at every size / only
    // up to 256 KiB: 512 KiB encode 139-154 / 135-136 us, 768 KiB 198-213 /
    // 194-196 (pre_max_ab_r6ao.txt).  TUNING builds: RSAMD_DIRECT_PRE_MAX.
    static const uint64_t pre_max = tuning_size("RSAMD_DIRECT_PRE_MAX", uint64_t(256) << 10);
    const bool pre = sig && n <= pre_max;
    // The streaming form in mid-size launches: a thread that codes one vector
    // loads, codes and stores once, so a launch's reads all come before its
    // writes and the link's two directions take turns; with several vectors
    // per thread one vector's stores overlap the next one's loads.  At least
    // kDirectIters vectors per thread (not under 32 workgroups): 4+2 x 1 MiB
    // shards, 16 / 32 / 64 / 128 / 256 workgroups: 129 / 112 / 116 / 114 /
    // 131 us per kernel (profiles/r6/direct_grid_r6at.txt).  Large launches
    // keep 256 (kDirectBlocks).  TUNING builds: RSAMD_DIRECT_ITERS (1: off).
    static const uint64_t iters = std::max<uint64_t>(1, tuning_size("RSAMD_DIRECT_ITERS", 8));
    if (!pre && iters > 1) {
        const uint64_t want = (a.nvec + kThreads * iters - 1) / (kThreads * iters);
        grid = unsigned(std::min<uint64_t>(grid, std::max<uint64_t>(want, 32)));
    }
    return W == 16 ? dispatch_direct<16>(a, p.nout, grid, mode, pre, s)
                   : dispatch_direct<8>(a, p.nout, grid, mode, pre, s);
}

hipError_t launch_fill_synthetic(uint8_t *base, int k, size_t n_stripes, size_t shard_len, size_t shard_stride,
                                 size_t stripe_stride, uint64_t seed, uint64_t stripe0, hipStream_t s) {
    if (n_stripes == 0 || shard_len == 0) return hipSuccess;
    if (shard_len % 8 || shard_stride % 8 || stripe_stride % 8 || reinterpret_cast<uintptr_t>(base) % 8)
        return hipErrorInvalidValue;
    const uint64_t wps = shard_len / 8;
    const uint64_t wpst = wps * uint64_t(k);
    const uint64_t n = wpst * n_stripes;
    const unsigned grid = unsigned(std::min<uint64_t>((n + kThreads - 1) / kThreads, 1u << 16));
    hipLaunchKernelGGL(fill_synthetic_kernel, dim3(grid), dim3(kThreads), 0, s, base, wpst, wps, n,
                       uint64_t(shard_stride), uint64_t(stripe_stride), seed, stripe0);
    return hipGetLastError();
}

hipError_t launch_copy(uint8_t *dst, const uint8_t *src, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    size_t head = 0;
    if (reinterpret_cast<uintptr_t>(dst) % 16 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0) {
        const uint64_t nvec = n / 16;
        for (uint64_t v0 = 0; v0 < nvec;) {  // one-shot grids of at most kMaxGridBlocks blocks
            const uint64_t nv = std::min<uint64_t>(nvec - v0, uint64_t(kMaxGridBlocks) * kWave);
            hipLaunchKernelGGL(copy_kernel, dim3(unsigned((nv + kWave - 1) / kWave)), dim3(kWave),
                               tuning_size("RSAMD_COPY_LDS_PAD", 0), s,
                               dst + v0 * 16, src + v0 * 16, nv);
            v0 += nv;
        }
        head = nvec * 16;
    }
    const uint64_t rest = n - head;
    if (rest) {
        const unsigned grid = unsigned((rest + kThreads - 1) / kThreads);
        hipLaunchKernelGGL(copy_tail_kernel, dim3(grid), dim3(kThreads), 0, s, dst + head, src + head, rest);
    }
    return hipGetLastError();
}

}  // namespace rsamd

RSAMD_BOUNDS_TU(kernels)
