// layout.hip -- the client's file <-> shard layout fused into the codec kernels
// (SURVEY.md section 8 row f1).
//
// Reference layout (ReedSolomonEncoder.java:56-85, ReedSolomonDecoder.java:62-103,
// ConfigVariables.java:4-9): the file is zero-padded to a multiple of k*block;
// block b (block bytes) goes to data shard b % k at offset (b / k) * block, so a
// shard is S = padded / k bytes; the decoder merges the blocks back and trims
// to the file size.  Equivalently, shard column c = r*block + w of data shard i
// holds file byte (r*k + i)*block + w.
//
// The fused kernels read the file (or write it) directly:
//   file_encode_kernel<K,M>: file -> K data shards + M parity shards, one pass,
//     traffic k*S read + (k+m)*S written (instead of split + encode: (3k+m)*S).
//   file_decode_kernel<K,E>: K survivors -> file, the E missing data shards
//     computed in registers, traffic k*S read + file_size written.
// block % 8 == 0 (the DFS uses 1000), so every 8-byte half of a lane's 16-byte
// column vector maps to one contiguous 8-byte run of the file.  Any other
// block size, alignment or k uses the generic split / merge kernels plus the
// stripe kernels of kernels.hip.  Global accesses go through RSAMD_G
// (bounds.hpp: the identity in the product build).
#define RSAMD_TU_ID 2
#include "layout.hpp"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <vector>

#include "gf_device.hpp"
#include "tuning.hpp"

namespace rsamd {
namespace {

using namespace dev;

constexpr int kWave = 64;
constexpr int kThreads = 256;

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

struct FileArgs {
    const uint8_t *file;  // encode: source file
    uint8_t *file_out;    // decode: destination file
    uint64_t file_len;    // encode: unpadded length; decode: trimmed file size
    uint8_t *shards;
    uint64_t shard_stride;
    uint64_t S;           // shard length (a multiple of block)
    uint32_t block;
    uint32_t nvec;        // ceil(S / 16)
    const uint32_t *tabs; // [K][M or E][5]
    const int32_t *in_idx;  // decode: survivor shard indices [K]
    const int32_t *dsrc;    // decode: data shard i -> survivor position (>= 0) or -(row + 1)
    uint32_t xcd_span;      // block order (file_block)
};

// How the fused kernels touch the FILE side (the shard side is always 16-byte
// non-temporal): IO_NT8 = 8-byte non-temporal, IO_PLAIN8 = 8-byte plain (the
// two halves of a 16-byte column vector meet in L2), IO_PAIR16 = one 16-byte
// access when both halves fall in the same block row (8-byte aligned), else
// two 8-byte accesses.  Chosen at launch (RSAMD_LAYOUT_IO); default
// IO_PLAIN8, measured best (profiles/r1/layout_io_sweep.txt: file encode 0.78 /
// decode 0.50 of HBM peak vs 0.68 / 0.38 non-temporal and 0.77 / 0.47 paired).
// Round 5, 1000-byte blocks, one process and one set of buffers: encode 0.745
// plain 8-byte against 0.637 paired, 0.633 paired non-temporal -- every other
// block row starts 8 bytes off a 16-byte boundary, and a 16-byte load there
// costs far more than two 8-byte ones (tools/file_io_ab.py,
// profiles/r5/file_io_ab_r6i.txt; the non-temporal form was deleted).
enum FileIo { IO_NT8 = 0, IO_PLAIN8 = 1, IO_PAIR16 = 2 };

// File byte runs of 8: [f, f+8) clipped to len, zero beyond (the padding).
template <int IO>
__device__ __forceinline__ u32x2 load8(const uint8_t *file, uint64_t len, uint64_t f, uint32_t line = __builtin_LINE()) {
    if (f + 8 <= len)
        return IO == IO_NT8 ? __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(RSAMD_GL(file + f, 8, line)))
                            : *reinterpret_cast<const u32x2 *>(RSAMD_GL(file + f, 8, line));
    uint64_t v = 0;
    for (uint64_t b = f; b < len && b < f + 8; ++b) v |= uint64_t(*RSAMD_GL(file + b, 1, line)) << (8 * (b - f));
    return u32x2{uint32_t(v), uint32_t(v >> 32)};
}

template <int IO>
__device__ __forceinline__ void store8(uint8_t *file, uint64_t len, uint64_t f, u32x2 v, uint32_t line = __builtin_LINE()) {
    if (f + 8 <= len) {
        if (IO == IO_NT8)
            __builtin_nontemporal_store(v, reinterpret_cast<u32x2 *>(RSAMD_GL(file + f, 8, line)));
        else
            *reinterpret_cast<u32x2 *>(RSAMD_GL(file + f, 8, line)) = v;
        return;
    }
    const uint64_t x = uint64_t(v[0]) | uint64_t(v[1]) << 32;
    for (uint64_t b = f; b < len && b < f + 8; ++b) *RSAMD_GL(file + b, 1, line) = uint8_t(x >> (8 * (b - f)));
}

// 16 file bytes [f, f+16) when both halves are contiguous (same block row),
// f 8-byte aligned: one dwordx4 access (the hardware splits it if needed).
struct alignas(8) u32x4_a8 {
    uint32_t v[4];
};
__device__ __forceinline__ u32x4 load16_a8(const uint8_t *p) {
    const u32x4_a8 t = *reinterpret_cast<const u32x4_a8 *>(RSAMD_G(p, 16));
    return u32x4{t.v[0], t.v[1], t.v[2], t.v[3]};
}
__device__ __forceinline__ void store16_a8(uint8_t *p, const u32x4 &v) {
    *reinterpret_cast<u32x4_a8 *>(RSAMD_G(p, 16)) = u32x4_a8{{v[0], v[1], v[2], v[3]}};
}

// Row r and in-row offset w of shard column cc = c0 + d, given the
// block-uniform (r0, w0) of c0 and 0 <= d < 1024.
__device__ __forceinline__ void row_of(uint64_t r0, uint32_t w0, uint32_t d, uint32_t block, uint64_t &r,
                                       uint32_t &w) {
    r = r0;
    w = w0 + d;
    while (w >= block) {
        w -= block;
        ++r;
    }
}

// Block order of the file kernels: with xcd_span != 0, XCD x (which gets
// every 8th block) walks blocks [x * xcd_span, (x+1) * xcd_span), one
// contiguous range per XCD (kernels.hip block_item; measured in
// profiles/r1/block_order_sweep.txt for the stripe kernels).
__device__ __forceinline__ uint32_t file_block(uint32_t xcd_span) {
    uint32_t b = blockIdx.x;
    if (xcd_span && b < 8u * xcd_span) b = (b % 8u) * xcd_span + b / 8u;
    return b;
}

template <int K, int M, int IO>
__global__ void __launch_bounds__(kWave) file_encode_kernel(FileArgs a) {
    const uint32_t blk = file_block(a.xcd_span);
    const uint32_t v = blk * kWave + threadIdx.x;
    const uint64_t c0 = uint64_t(blk) * kWave * 16;  // block-uniform first column
    const uint64_t r0 = c0 / a.block;
    const uint32_t w0 = uint32_t(c0 - r0 * a.block);
    if (v >= a.nvec) return;
    const uint64_t c = uint64_t(v) * 16;
    const bool hi = c + 16 <= a.S;  // the last vector of a shard may be a single 8-byte half
    uint64_t rr[2];
    uint32_t ww[2];
    row_of(r0, w0, threadIdx.x * 16, a.block, rr[0], ww[0]);
    row_of(r0, w0, threadIdx.x * 16 + 8, a.block, rr[1], ww[1]);

    // Tables first: read before any store, so they stay scalar loads.
    uint32_t T[M > 0 ? M : 1][K][5];
#pragma unroll
    for (int p = 0; p < M; ++p)
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) T[p][i][j] = *RSAMD_G(a.tabs + ((i * M + p) * 5 + j), 4);
    u32x4 x[K];
    const bool pair = IO == IO_PAIR16 && hi && rr[0] == rr[1];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const uint64_t f0 = (rr[0] * K + i) * a.block + ww[0];
        if (pair && f0 + 16 <= a.file_len) {
            x[i] = load16_a8(a.file + f0);
        } else {
            const u32x2 lo = load8<IO>(a.file, a.file_len, f0);
            const u32x2 up = hi ? load8<IO>(a.file, a.file_len, (rr[1] * K + i) * a.block + ww[1]) : u32x2{0, 0};
            x[i] = u32x4{lo[0], lo[1], up[0], up[1]};
        }
    }
    uint8_t *col = a.shards + c;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        uint8_t *dst = col + uint64_t(i) * a.shard_stride;
        if (hi)
            __builtin_nontemporal_store(x[i], reinterpret_cast<u32x4 *>(RSAMD_G(dst, 16)));
        else
            __builtin_nontemporal_store(u32x2{x[i][0], x[i][1]}, reinterpret_cast<u32x2 *>(RSAMD_G(dst, 8)));
    }
    if (M == 0) return;
    u32x4 acc[M > 0 ? M : 1];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        Sel s[K];
#pragma unroll
        for (int i = 0; i < K; ++i) s[i] = selectors(x[i][w]);
#pragma unroll
        for (int p = 0; p < M; ++p) acc[p][w] = dot_dword<K>(T[p], s);
    }
#pragma unroll
    for (int p = 0; p < M; ++p) {
        uint8_t *dst = col + uint64_t(K + p) * a.shard_stride;
        if (hi)
            __builtin_nontemporal_store(acc[p], reinterpret_cast<u32x4 *>(RSAMD_G(dst, 16)));
        else
            __builtin_nontemporal_store(u32x2{acc[p][0], acc[p][1]}, reinterpret_cast<u32x2 *>(RSAMD_G(dst, 8)));
    }
}

// Data shard held by register vector j of a decode (j < K: survivor j, else
// rebuilt vector j - K), or -1: the inverse of the uniform dsrc map by scalar
// selects.  Kernels scatter each vector to its data shard instead of
// gathering x[dsrc[i]]: a run-time index into a register array (even as a
// select chain, which the compiler folds back into one) puts it in scratch.
template <int K>
__device__ __forceinline__ int data_row(const int (&dsrc)[K], int j) {
    int row = -1;
#pragma unroll
    for (int i = 0; i < K; ++i)
        if (dsrc[i] == (j < K ? j : K - 1 - j)) row = i;
    return row;
}

template <int K, int E, int IO>
__global__ void __launch_bounds__(kWave) file_decode_kernel(FileArgs a) {
    const uint32_t blk = file_block(a.xcd_span);
    const uint32_t v = blk * kWave + threadIdx.x;
    const uint64_t c0 = uint64_t(blk) * kWave * 16;
    const uint64_t r0 = c0 / a.block;
    const uint32_t w0 = uint32_t(c0 - r0 * a.block);
    int dsrc[K];
#pragma unroll
    for (int i = 0; i < K; ++i) dsrc[i] = *RSAMD_G(a.dsrc + i, 4);
    if (v >= a.nvec) return;
    const uint64_t c = uint64_t(v) * 16;
    const bool hi = c + 16 <= a.S;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const uint8_t *src = a.shards + uint64_t(*RSAMD_G(a.in_idx + j, 4)) * a.shard_stride + c;
        if (hi) {
            x[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(RSAMD_G(src, 16)));
        } else {
            const u32x2 h = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(RSAMD_G(src, 8)));
            x[j] = u32x4{h[0], h[1], 0, 0};
        }
    }
    u32x4 y[E > 0 ? E : 1];
    if (E > 0) {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            Sel s[K];
#pragma unroll
            for (int j = 0; j < K; ++j) s[j] = selectors(x[j][w]);
#pragma unroll
            for (int e = 0; e < E; ++e) {
                uint32_t T[K][5];
#pragma unroll
                for (int j = 0; j < K; ++j)
#pragma unroll
                    for (int q = 0; q < 5; ++q) T[j][q] = *RSAMD_G(a.tabs + ((j * E + e) * 5 + q), 4);
                y[e][w] = dot_dword<K>(T, s);
            }
        }
    }
    uint64_t rr[2];
    uint32_t ww[2];
    row_of(r0, w0, threadIdx.x * 16, a.block, rr[0], ww[0]);
    row_of(r0, w0, threadIdx.x * 16 + 8, a.block, rr[1], ww[1]);
#pragma unroll
    for (int j = 0; j < K + E; ++j) {
        const int i = data_row<K>(dsrc, j);
        if (i < 0) continue;
        const u32x4 d = j < K ? x[j] : y[j < K ? 0 : j - K];
        const uint64_t f0 = (rr[0] * K + i) * a.block + ww[0];
        if (IO == IO_PAIR16 && hi && rr[0] == rr[1] && f0 + 16 <= a.file_len) {
            store16_a8(a.file_out + f0, d);
        } else {
            store8<IO>(a.file_out, a.file_len, f0, u32x2{d[0], d[1]});
            if (hi) store8<IO>(a.file_out, a.file_len, (rr[1] * K + i) * a.block + ww[1], u32x2{d[2], d[3]});
        }
    }
}

// ---------------------------------------------------------------------------
// Tiled decode-to-file.  A workgroup (THREADS x SLOTS column vectors) owns R
// whole block rows (R * block columns of every shard; R even so every offset
// stays 16-byte aligned).  Phase 1: each thread loads the K survivors' 16-byte
// column vectors, rebuilds the E missing data shards in registers and parks the K
// data vectors in an LDS tile [data shard][R * block].  Phase 2: the tile's
// file bytes are ONE contiguous run [r0*K*block, (r0+R)*K*block) -- written
// as aligned 16-byte stores, each assembled from two 8-byte LDS reads (a
// 16-byte chunk may straddle two blocks when block % 16 == 8).  This replaces
// the per-lane 8-byte file stores of file_decode_kernel (0.49 of HBM peak).
// ---------------------------------------------------------------------------
constexpr int kTileThreads = 256;
constexpr int kTileSlots = 2;  // 16-byte column vectors per thread and shard in phase 1
// The decode tile's default shape: 512 threads x 1 vector (8 rows at block
// 1000, as 256 x 2) measured 0.750-0.755 of peak on {0,5} against 0.737-0.743
// for 256 x 2 (profiles/r1/file_decode_ab/dec_tile_shapes.txt).
constexpr int kDecTileThreads = 512;
constexpr int kDecTileSlots = 1;

struct TileArgs {
    uint8_t *file_out;
    uint64_t file_size;
    const uint8_t *shards;
    uint64_t shard_stride;
    uint64_t n_rows;       // S / block
    uint32_t block;
    uint32_t rows;         // R rows per tile (even)
    uint32_t inv_block;    // floor(2^32 / block) + 1: t / block for t < 2^16
    uint32_t inv_kblock;   // same for K * block
    const uint32_t *tabs;  // [K][E][5]
    const int32_t *in_idx;
    const int32_t *dsrc;
    uint32_t xcd_span;     // block order (file_block)
};

__device__ __forceinline__ uint32_t div_small(uint32_t t, uint32_t inv) {
    return uint32_t((uint64_t(t) * inv) >> 32);
}

// One 16-byte column vector of each survivor (8 bytes at the ragged end).
template <int K>
__device__ __forceinline__ void tile_load(u32x4 (&x)[K], const uint8_t *shards, const uint64_t (&in_off)[K],
                                          uint32_t c, uint32_t span) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const uint8_t *src = shards + in_off[j] + c;
        if (c + 16 <= span) {
            x[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(RSAMD_G(src, 16)));
        } else if (c < span) {
            const u32x2 h = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(RSAMD_G(src, 8)));
            x[j] = u32x4{h[0], h[1], 0, 0};
        }
    }
}

// Rebuild the E missing data vectors from x and park all K data vectors of
// column c in the LDS tile [data shard][pitch].
template <int K, int E>
__device__ __forceinline__ void tile_park(const u32x4 (&x)[K], const uint32_t (&T)[E > 0 ? E : 1][K][5],
                                          const int (&dsrc)[K], uint8_t *tile, uint32_t pitch, uint32_t c,
                                          uint32_t span) {
    if (c >= span) return;
    constexpr int EY = E > 0 ? E : 1;
    u32x4 y[EY];
    if (E > 0) {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            Sel sl[K];
#pragma unroll
            for (int j = 0; j < K; ++j) sl[j] = selectors(x[j][w]);
#pragma unroll
            for (int e = 0; e < E; ++e) y[e][w] = dot_dword<K>(T[e], sl);
        }
    }
#pragma unroll
    for (int j = 0; j < K + E; ++j) {
        const int row = data_row<K>(dsrc, j);
        if (row < 0) continue;
        const u32x4 d = j < K ? x[j] : y[j < K ? 0 : j - K];
        uint8_t *dst = tile + row * pitch + c;
        if (c + 16 <= span)
            *reinterpret_cast<u32x4 *>(dst) = d;
        else
            *reinterpret_cast<u32x2 *>(dst) = u32x2{d[0], d[1]};
    }
}

template <int K, int E, int THREADS, int SLOTS>
__global__ void __launch_bounds__(THREADS) file_decode_tiled_kernel(TileArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
    const uint64_t r0 = uint64_t(file_block(a.xcd_span)) * a.rows;
    const uint32_t rows = uint32_t(min(uint64_t(a.rows), a.n_rows - r0));
    const uint32_t span = rows * a.block;      // columns of this tile (a multiple of 16 unless last)
    const uint32_t pitch = a.rows * a.block;   // LDS bytes per data shard
    const uint64_t col0 = r0 * a.block;
    int dsrc[K];
#pragma unroll
    for (int i = 0; i < K; ++i) dsrc[i] = *RSAMD_G(a.dsrc + i, 4);
    uint32_t T[E > 0 ? E : 1][K][5];
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
            for (int q = 0; q < 5; ++q) T[e][j][q] = *RSAMD_G(a.tabs + ((j * E + e) * 5 + q), 4);
    uint64_t in_off[K];
#pragma unroll
    for (int j = 0; j < K; ++j) in_off[j] = uint64_t(*RSAMD_G(a.in_idx + j, 4)) * a.shard_stride + col0;

    // Phase 1: survivors -> data vectors -> LDS.  span % 8 == 0 (block % 8 == 0)
    // and span <= 2 * 256 * 16: both slots' loads are issued before any
    // compute, then each slot is folded and parked.  One named register array
    // per slot: an x[slot][shard] array indexed through the slot loop stays
    // an alloca and spills the vectors to scratch (2x the HBM traffic).
    const uint32_t c0 = threadIdx.x * 16, c1 = c0 + THREADS * 16;
    u32x4 x0[K], x1[K];
    tile_load<K>(x0, a.shards, in_off, c0, span);
    if constexpr (SLOTS == 2) tile_load<K>(x1, a.shards, in_off, c1, span);
    tile_park<K, E>(x0, T, dsrc, tile, pitch, c0, span);
    if constexpr (SLOTS == 2) tile_park<K, E>(x1, T, dsrc, tile, pitch, c1, span);
    __syncthreads();

    // Phase 2: the tile's contiguous file run, 16-byte aligned chunks.
    const uint32_t kblock = uint32_t(K) * a.block;
    const uint64_t f0 = r0 * kblock;
    const uint32_t run = rows * kblock;
    for (uint32_t t = threadIdx.x * 16; t < run; t += THREADS * 16) {
        const uint64_t f = f0 + t;
        if (f >= a.file_size) break;
        u32x2 half[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t u = t + 8 * h;               // byte of the run
            const uint32_t row = div_small(u, a.inv_kblock);
            const uint32_t rem = u - row * kblock;
            const uint32_t i = div_small(rem, a.inv_block);
            const uint32_t w = rem - i * a.block;
            half[h] = *reinterpret_cast<const u32x2 *>(tile + i * pitch + row * a.block + w);
        }
        const u32x4 v{half[0][0], half[0][1], half[1][0], half[1][1]};
        if (f + 16 <= a.file_size) {
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(RSAMD_G(a.file_out + f, 16)));
        } else {
            for (uint32_t b = 0; b < 16 && f + b < a.file_size; ++b)
                *RSAMD_G(a.file_out + (f + b), 1) = uint8_t(v[b / 4] >> (8 * (b % 4)));
        }
    }
}

// ---------------------------------------------------------------------------
// Tiled file encode, the mirror image of the tiled decode.  A 256-thread
// workgroup owns R whole block rows.  Phase 1: the tile's file bytes -- ONE
// contiguous run [r0*K*block, (r0+R)*K*block), zero past the file end (the
// padding) -- come in as aligned 16-byte loads, all issued up front, and land
// in LDS unchanged.  Phase 2: each thread gathers the K data shards' 16-byte
// column vectors from LDS (two 8-byte reads each: a vector may straddle two
// blocks when block % 16 == 8), computes the M parity vectors and stores all
// K + M with 16-byte non-temporal stores, in place of file_encode_kernel's
// 8-byte file loads (which fetched 1.2x the file at block 1000 before the
// XCD-contiguous block order, and exactly 1.0x since: profiles/pmc_traffic_all.json).
// Needs a 16-byte aligned file.  Opt-in (RSAMD_FILE_ENCODE=1): not faster
// than file_encode_kernel on MI355X.
// ---------------------------------------------------------------------------
struct EncTileArgs {
    const uint8_t *file;
    uint64_t file_len;
    uint8_t *shards;
    uint64_t shard_stride;
    uint64_t n_rows;
    uint32_t block;
    uint32_t rows;
    uint32_t inv_block;
    const uint32_t *tabs;  // [K][M][5]
    uint32_t xcd_span;     // block order (file_block)
};

template <int K, int M, int THREADS, int SLOTS>
__global__ void __launch_bounds__(THREADS) file_encode_tiled_kernel(EncTileArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
    const uint64_t r0 = uint64_t(file_block(a.xcd_span)) * a.rows;
    const uint32_t rows = uint32_t(min(uint64_t(a.rows), a.n_rows - r0));
    const uint32_t span = rows * a.block;
    const uint32_t kblock = uint32_t(K) * a.block;
    const uint32_t run = rows * kblock;  // a multiple of 16 (rows even, or the file's last tile)
    const uint64_t f0 = r0 * kblock;
    uint32_t T[M > 0 ? M : 1][K][5];
#pragma unroll
    for (int p = 0; p < M; ++p)
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) T[p][i][j] = *RSAMD_G(a.tabs + ((i * M + p) * 5 + j), 4);

    // Phase 1: run <= SLOTS * THREADS * 16 * K bytes, so SLOTS * K loads per thread.
    constexpr int NL = SLOTS * K;
    u32x4 v[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
        const uint32_t t = (u * THREADS + threadIdx.x) * 16;
        const uint64_t f = f0 + t;
        v[u] = u32x4{0, 0, 0, 0};
        if (t < run) {
            if (f + 16 <= a.file_len) {
                v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(RSAMD_G(a.file + f, 16)));
            } else if (f < a.file_len) {
                uint32_t w[4] = {0, 0, 0, 0};
                for (uint64_t b = f; b < a.file_len; ++b) w[(b - f) / 4] |= uint32_t(*RSAMD_G(a.file + b, 1)) << (8 * ((b - f) % 4));
                v[u] = u32x4{w[0], w[1], w[2], w[3]};
            }
        }
    }
#pragma unroll
    for (int u = 0; u < NL; ++u) {
        const uint32_t t = (u * THREADS + threadIdx.x) * 16;
        if (t < run) *reinterpret_cast<u32x4 *>(tile + t) = v[u];
    }
    __syncthreads();

    // Phase 2: columns c of the tile's span, SLOTS vectors per thread.
    const uint64_t col0 = r0 * a.block;
#pragma unroll
    for (int u = 0; u < SLOTS; ++u) {
        const uint32_t c = (u * THREADS + threadIdx.x) * 16;
        if (c >= span) continue;
        const bool hi = c + 16 <= span;  // else only the 8-byte half [c, c+8) exists
        u32x4 x[K];
        uint32_t lo_off, hi_off;  // LDS offsets of data shard 0's two halves
        {
            const uint32_t r = div_small(c, a.inv_block);
            lo_off = r * kblock + (c - r * a.block);
            const uint32_t c8 = c + 8;
            const uint32_t r8 = div_small(c8, a.inv_block);
            hi_off = r8 * kblock + (c8 - r8 * a.block);
        }
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const u32x2 l = *reinterpret_cast<const u32x2 *>(tile + lo_off + i * a.block);
            const u32x2 h = hi ? *reinterpret_cast<const u32x2 *>(tile + hi_off + i * a.block) : u32x2{0, 0};
            x[i] = u32x4{l[0], l[1], h[0], h[1]};
        }
        uint8_t *col = a.shards + col0 + c;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            uint8_t *dst = col + uint64_t(i) * a.shard_stride;
            if (hi)
                __builtin_nontemporal_store(x[i], reinterpret_cast<u32x4 *>(RSAMD_G(dst, 16)));
            else
                __builtin_nontemporal_store(u32x2{x[i][0], x[i][1]}, reinterpret_cast<u32x2 *>(RSAMD_G(dst, 8)));
        }
        if (M == 0) continue;
        u32x4 acc[M > 0 ? M : 1];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            Sel sl[K];
#pragma unroll
            for (int i = 0; i < K; ++i) sl[i] = selectors(x[i][w]);
#pragma unroll
            for (int p = 0; p < M; ++p) acc[p][w] = dot_dword<K>(T[p], sl);
        }
#pragma unroll
        for (int p = 0; p < M; ++p) {
            uint8_t *dst = col + uint64_t(K + p) * a.shard_stride;
            if (hi)
                __builtin_nontemporal_store(acc[p], reinterpret_cast<u32x4 *>(RSAMD_G(dst, 16)));
            else
                __builtin_nontemporal_store(u32x2{acc[p][0], acc[p][1]}, reinterpret_cast<u32x2 *>(RSAMD_G(dst, 8)));
        }
    }
}

// ---------------------------------------------------------------------------
// Generic split (file -> k data shards) and merge (k data shards -> file):
// one thread per W-byte word of one shard, W = 8 when block % 8 == 0 and the
// buffers are 8-aligned, else 1.
// ---------------------------------------------------------------------------
struct CopyArgs {
    const uint8_t *file;
    uint8_t *file_out;
    uint64_t file_len;
    uint8_t *shards;
    uint64_t shard_stride;
    uint64_t S;
    uint64_t block;
    uint64_t words_per_shard;  // ceil(S / W)
    uint64_t total;            // k * words_per_shard
    int k;
};

template <int W, bool SPLIT>
__global__ void __launch_bounds__(kThreads) split_merge_kernel(CopyArgs a) {
    const uint64_t step = uint64_t(gridDim.x) * kThreads;
    for (uint64_t idx = uint64_t(blockIdx.x) * kThreads + threadIdx.x; idx < a.total; idx += step) {
        const uint64_t i = idx / a.words_per_shard;
        const uint64_t c = (idx - i * a.words_per_shard) * W;
        const uint64_t r = c / a.block;
        const uint64_t f = (r * a.k + i) * a.block + (c - r * a.block);
        uint8_t *sh = a.shards + i * a.shard_stride + c;
        const uint64_t n = a.S - c < W ? a.S - c : W;  // bytes of this word inside the shard
        if (SPLIT) {
            if (W == 8 && n == 8) {
                *reinterpret_cast<u32x2 *>(RSAMD_G(sh, 8)) = load8<IO_PLAIN8>(a.file, a.file_len, f);
            } else {
                for (uint64_t b = 0; b < n; ++b) *RSAMD_G(sh + b, 1) = f + b < a.file_len ? *RSAMD_G(a.file + (f + b), 1) : 0;
            }
        } else {
            if (W == 8 && n == 8) {
                store8<IO_PLAIN8>(a.file_out, a.file_len, f, *reinterpret_cast<const u32x2 *>(RSAMD_G(sh, 8)));
            } else {
                for (uint64_t b = 0; b < n; ++b)
                    if (f + b < a.file_len) *RSAMD_G(a.file_out + (f + b), 1) = *RSAMD_G(sh + b, 1);
            }
        }
    }
}

int file_io_mode() {
    const char *e = tuning_env("RSAMD_LAYOUT_IO");  // per launch (TUNING builds): A/B in one process
    return e ? std::atoi(e) : int(IO_PLAIN8);
}

// XCD span for a file-kernel grid of n blocks (RSAMD_FILE_XCD=0 turns the
// remap off for A/B runs).
uint32_t file_xcd_span(uint64_t n_blocks) {
    const char *e = tuning_env("RSAMD_FILE_XCD");  // per launch (TUNING builds): sweeps
    const bool on = !(e && e[0] == '0');
    return on ? uint32_t(n_blocks / 8u) : 0u;
}

// Occupancy cap of the untiled file kernels (one-wave workgroups): dynamic
// LDS bytes per wave, 160 KiB / pad waves per CU (as kernels.hip vec_lds_pad).
// The 4 GiB file encode reads 0.775 uncapped and 0.79 at 10240-11520 B
// (tools/occ_sweep2.py --family file, profiles/r3/occ_sweep2_r3zt.txt); the
// tiled decode is best as it is (extra LDS per workgroup: +0 .. -3.5 points).
size_t file_lds_pad(bool encode) { return tuning_size("RSAMD_FILE_LDS_PAD", encode ? 11520 : 0); }

template <int K, int M>
hipError_t launch_enc_t(const FileArgs &a, hipStream_t s) {
    const dim3 grid((a.nvec + kWave - 1) / kWave);
    switch (file_io_mode()) {
    case IO_NT8: hipLaunchKernelGGL((file_encode_kernel<K, M, IO_NT8>), grid, dim3(kWave), file_lds_pad(true), s, a); break;
    case IO_PLAIN8: hipLaunchKernelGGL((file_encode_kernel<K, M, IO_PLAIN8>), grid, dim3(kWave), file_lds_pad(true), s, a); break;
    default: hipLaunchKernelGGL((file_encode_kernel<K, M, IO_PAIR16>), grid, dim3(kWave), file_lds_pad(true), s, a); break;
    }
    return hipGetLastError();
}

template <int K, int E>
hipError_t launch_dec_t(const FileArgs &a, hipStream_t s) {
    const dim3 grid((a.nvec + kWave - 1) / kWave);
    switch (file_io_mode()) {
    case IO_NT8: hipLaunchKernelGGL((file_decode_kernel<K, E, IO_NT8>), grid, dim3(kWave), file_lds_pad(false), s, a); break;
    case IO_PLAIN8: hipLaunchKernelGGL((file_decode_kernel<K, E, IO_PLAIN8>), grid, dim3(kWave), file_lds_pad(false), s, a); break;
    default: hipLaunchKernelGGL((file_decode_kernel<K, E, IO_PAIR16>), grid, dim3(kWave), file_lds_pad(false), s, a); break;
    }
    return hipGetLastError();
}

bool aligned(const void *p, size_t a) { return reinterpret_cast<uintptr_t>(p) % a == 0; }

hipError_t launch_split_merge(const FileGeom &g, bool split, hipStream_t s) {
    const bool w8 = g.block % 8 == 0 && g.S % 8 == 0 && g.shard_stride % 8 == 0 && aligned(g.shards, 8) &&
                    aligned(split ? static_cast<const void *>(g.file) : static_cast<const void *>(g.file_out), 8);
    const int W = w8 ? 8 : 1;
    CopyArgs a{g.file, g.file_out, g.file_len, g.shards, g.shard_stride, g.S, g.block, (g.S + W - 1) / W, 0, g.k};
    a.total = uint64_t(g.k) * a.words_per_shard;
    if (a.total == 0) return hipSuccess;
    const unsigned grid = unsigned(std::min<uint64_t>((a.total + kThreads - 1) / kThreads, 1u << 20));
    if (w8 && split) hipLaunchKernelGGL((split_merge_kernel<8, true>), dim3(grid), dim3(kThreads), 0, s, a);
    if (w8 && !split) hipLaunchKernelGGL((split_merge_kernel<8, false>), dim3(grid), dim3(kThreads), 0, s, a);
    if (!w8 && split) hipLaunchKernelGGL((split_merge_kernel<1, true>), dim3(grid), dim3(kThreads), 0, s, a);
    if (!w8 && !split) hipLaunchKernelGGL((split_merge_kernel<1, false>), dim3(grid), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace

bool file_fusable(const FileGeom &g, bool encode) {
    return g.k == 4 && g.block % 8 == 0 && g.block >= 8 && g.S % g.block == 0 && g.shard_stride % 16 == 0 &&
           aligned(g.shards, 16) &&
           aligned(encode ? static_cast<const void *>(g.file) : static_cast<const void *>(g.file_out), 8) &&
           (g.S + 15) / 16 <= uint64_t(UINT32_MAX) - kWave;  // grid work-items fit 32 bits
}


namespace {

// Tile shape: THREADS x SLOTS 16-byte columns per shard.  TUNING builds read
// "threads,slots" from `env` at each launch (sweeps change it between legs).
struct DecTile {
    int threads, slots;
};

DecTile tile_shape(const char *env, DecTile dflt) {
    const char *e = tuning_env(env);
    if (e) {
        int t = 0, sl = 0;
        if (std::sscanf(e, "%d,%d", &t, &sl) == 2 && (t == 128 || t == 256 || t == 512 || t == 1024) && (sl == 1 || sl == 2))
            return {t, sl};
    }
    return dflt;
}

DecTile dec_tile() { return tile_shape("RSAMD_DEC_TILE", {kDecTileThreads, kDecTileSlots}); }
DecTile enc_tile() { return tile_shape("RSAMD_ENC_TILE", {kTileThreads, kTileSlots}); }

template <int K, int E>
hipError_t launch_tiled_t(const TileArgs &a, uint64_t tiles, DecTile d, hipStream_t s) {
    const size_t lds = size_t(K) * a.rows * a.block + tuning_size("RSAMD_FILE_TILE_LDS_PAD", 0);
    const dim3 grid{unsigned(tiles)}, blk{unsigned(d.threads)};
#define RSAMD_DEC_TILE(T, SL)                                                                   \
    if (d.threads == T && d.slots == SL) {                                                      \
        hipLaunchKernelGGL((file_decode_tiled_kernel<K, E, T, SL>), grid, blk, lds, s, a);      \
        return hipGetLastError();                                                               \
    }
    RSAMD_DEC_TILE(512, 1)
    RSAMD_DEC_TILE(256, 2)
    RSAMD_DEC_TILE(256, 1)
    RSAMD_DEC_TILE(128, 2)
    RSAMD_DEC_TILE(512, 2)
    RSAMD_DEC_TILE(128, 1)
    RSAMD_DEC_TILE(1024, 1)
#undef RSAMD_DEC_TILE
    return hipErrorInvalidValue;
}

template <int K, int M>
hipError_t launch_enc_tiled_t(const EncTileArgs &a, uint64_t tiles, DecTile d, hipStream_t s) {
    const size_t lds = size_t(K) * a.rows * a.block + tuning_size("RSAMD_FILE_TILE_LDS_PAD", 0);
    const dim3 grid{unsigned(tiles)}, blk{unsigned(d.threads)};
#define RSAMD_ENC_TILE(T, SL)                                                                   \
    if (d.threads == T && d.slots == SL) {                                                      \
        hipLaunchKernelGGL((file_encode_tiled_kernel<K, M, T, SL>), grid, blk, lds, s, a);      \
        return hipGetLastError();                                                               \
    }
    RSAMD_ENC_TILE(256, 2)
    RSAMD_ENC_TILE(512, 2)
    RSAMD_ENC_TILE(512, 1)
    RSAMD_ENC_TILE(1024, 1)
#undef RSAMD_ENC_TILE
    return hipErrorInvalidValue;
}

// A tile spans R * block <= slots * threads * 16 columns (R even, >= 2), so
// LDS per workgroup is <= K * 8 KiB = 32 KiB at K = 4 with the default shape.
uint32_t tile_rows(const FileGeom &g, int threads = kTileThreads, int slots = kTileSlots) {
    if (g.block >= (1u << 15)) return 0;
    uint64_t R = uint64_t(slots) * threads * 16 / g.block;
    if (R % 2) --R;
    return R >= 2 ? uint32_t(R) : 0;
}

}  // namespace

hipError_t launch_file_encode_fused(const FileGeom &g, const DevPlan *parity0, hipStream_t s) {
    if (g.S == 0) return hipSuccess;
    // The untiled kernel is the default: both have exact traffic, and the
    // tiled one measured 0.67-0.78 of peak against 0.72-0.78 across boxes
    // (profiles/r1/file_decode_ab/).
    // RSAMD_FILE_ENCODE=1 selects it (A/B).
    const char *mode = tuning_env("RSAMD_FILE_ENCODE");
    const DecTile d = enc_tile();
    uint32_t R = tile_rows(g, d.threads, d.slots);
    if (R && (g.S / g.block + R - 1) / R * uint64_t(d.threads) > UINT32_MAX) R = 0;  // grid > 2^32 work-items
    if (R && aligned(g.file, 16) && mode && mode[0] == '1') {
        EncTileArgs a{g.file, g.file_len, g.shards, g.shard_stride, g.S / g.block, uint32_t(g.block), R,
                      uint32_t((uint64_t(1) << 32) / g.block + 1), parity0 ? parity0->tabs : nullptr, 0};
        const uint64_t tiles = (a.n_rows + R - 1) / R;
        a.xcd_span = file_xcd_span(tiles);
        switch (parity0 ? parity0->nout : 0) {
        case 0: return launch_enc_tiled_t<4, 0>(a, tiles, d, s);
        case 1: return launch_enc_tiled_t<4, 1>(a, tiles, d, s);
        case 2: return launch_enc_tiled_t<4, 2>(a, tiles, d, s);
        case 3: return launch_enc_tiled_t<4, 3>(a, tiles, d, s);
        case 4: return launch_enc_tiled_t<4, 4>(a, tiles, d, s);
        }
        return hipErrorInvalidValue;
    }
    FileArgs a{g.file, nullptr, g.file_len, g.shards, g.shard_stride, g.S, uint32_t(g.block),
               uint32_t((g.S + 15) / 16), parity0 ? parity0->tabs : nullptr, nullptr, nullptr, 0};
    a.xcd_span = file_xcd_span((a.nvec + kWave - 1) / kWave);
    const int m = parity0 ? parity0->nout : 0;
    switch (m) {
    case 0: return launch_enc_t<4, 0>(a, s);
    case 1: return launch_enc_t<4, 1>(a, s);
    case 2: return launch_enc_t<4, 2>(a, s);
    case 3: return launch_enc_t<4, 3>(a, s);
    case 4: return launch_enc_t<4, 4>(a, s);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_file_decode_fused(const FileGeom &g, const FileDecodePlan &p, hipStream_t s) {
    if (g.S == 0 || g.file_len == 0) return hipSuccess;
    const DecTile d = dec_tile();
    uint32_t R = tile_rows(g, d.threads, d.slots);
    if (R && (g.S / g.block + R - 1) / R * uint64_t(d.threads) > UINT32_MAX) R = 0;  // grid > 2^32 work-items
    const char *mode = tuning_env("RSAMD_FILE_DECODE");
    if (R && !(mode && mode[0] == '0')) {  // RSAMD_FILE_DECODE=0 selects the untiled kernel (A/B only)
        TileArgs a{g.file_out, g.file_len, g.shards, g.shard_stride, g.S / g.block, uint32_t(g.block), R,
                   uint32_t((uint64_t(1) << 32) / g.block + 1), uint32_t((uint64_t(1) << 32) / (uint64_t(g.k) * g.block) + 1),
                   p.tabs, p.in_idx, p.dsrc, 0};
        const uint64_t tiles = (a.n_rows + R - 1) / R;
        a.xcd_span = file_xcd_span(tiles);
        switch (p.n_missing_data) {
        case 0: return launch_tiled_t<4, 0>(a, tiles, d, s);
        case 1: return launch_tiled_t<4, 1>(a, tiles, d, s);
        case 2: return launch_tiled_t<4, 2>(a, tiles, d, s);
        case 3: return launch_tiled_t<4, 3>(a, tiles, d, s);
        case 4: return launch_tiled_t<4, 4>(a, tiles, d, s);
        }
        return hipErrorInvalidValue;
    }
    FileArgs a{nullptr, g.file_out, g.file_len, g.shards, g.shard_stride, g.S, uint32_t(g.block),
               uint32_t((g.S + 15) / 16), p.tabs, p.in_idx, p.dsrc, 0};
    a.xcd_span = file_xcd_span((a.nvec + kWave - 1) / kWave);
    switch (p.n_missing_data) {
    case 0: return launch_dec_t<4, 0>(a, s);
    case 1: return launch_dec_t<4, 1>(a, s);
    case 2: return launch_dec_t<4, 2>(a, s);
    case 3: return launch_dec_t<4, 3>(a, s);
    case 4: return launch_dec_t<4, 4>(a, s);
    }
    return hipErrorInvalidValue;
}

namespace {

// ---------------------------------------------------------------------------
// Direct file encode kernel: rs_file_encode (capi.cpp file_encode_direct) on
// page-locked caller buffers, coded in place across the link like kernels.hip
// gf_direct_kernel -- no staging buffers, no copy engine, H2D and D2H at once.
// One thread codes one 8-byte column unit of every shard (block % 8 == 0, so
// a unit never crosses a block and its bytes of data shard i are one 8-byte
// run of the file); runtime k, the output count a template argument, so
// nothing is indexed dynamically in registers: for each data shard i, load its
// file run (zero past file_len: the pad, ReedSolomonEncoder.java:76-85), store
// it to shard i unless the host splits the data shards (out[i] null) and fold
// it into the M parity units, then store those.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t load_run8(const uint8_t *p, uint64_t f, uint64_t len) {
    if (f + 8 <= len) return __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(RSAMD_G(p + f, 8)));
    uint64_t v = 0;
    for (uint64_t b = f; b < len && b < f + 8; ++b) v |= uint64_t(*RSAMD_G(p + b, 1)) << (8 * (b - f));
    return v;
}

__device__ __forceinline__ void fold_unit(const uint32_t *t, uint64_t x, uint32_t &lo, uint32_t &hi) {
    t = RSAMD_G(t, 20);
    uint32_t a, b, c;
    terms(t, selectors(uint32_t(x)), a, b, c);
    lo = xor3(lo, a, b) ^ c;
    terms(t, selectors(uint32_t(x >> 32)), a, b, c);
    hi = xor3(hi, a, b) ^ c;
}

// Unit u codes shard column rot + 8u (mod cols): the shards' runs of a wave
// then start on the widest power-of-two boundary (up to a page) their
// addresses share, so a wave writes whole 128-byte lines (malloc'd arrays sit
// 16 bytes past a page start; see kernels.hip launch_gf_direct).
__device__ __forceinline__ uint64_t rotated_column(uint64_t u, const FileDirect &a) {
    const uint64_t c = u * 8 + a.rot;
    return c >= a.units * 8 ? c - a.units * 8 : c;
}

template <int M>
__device__ __forceinline__ void file_direct_unit(const FileDirect &a, uint64_t c) {
    const uint64_t r = c / a.block, w = c - r * a.block;
    uint32_t lo[M > 0 ? M : 1] = {}, hi[M > 0 ? M : 1] = {};
    for (int i = 0; i < a.k; ++i) {
        const uint64_t x = load_run8(a.file, (r * uint64_t(a.k) + uint64_t(i)) * a.block + w, a.file_len);
        if (a.out[i])  // (null: the caller splits the data shards on the host, capi.cpp file_encode_direct)
            __builtin_nontemporal_store(x, reinterpret_cast<uint64_t *>(RSAMD_G(a.out[i] + c, 8)));
#pragma unroll
        for (int p = 0; p < M; ++p) fold_unit(a.tabs + (i * M + p) * 5, x, lo[p], hi[p]);
    }
#pragma unroll
    for (int p = 0; p < M; ++p)
        __builtin_nontemporal_store(uint64_t(lo[p]) | (uint64_t(hi[p]) << 32),
                                    reinterpret_cast<uint64_t *>(RSAMD_G(a.out[a.k + p] + c, 8)));
}

template <int M>
__global__ void __launch_bounds__(kThreads) file_direct_encode_kernel(FileDirect a) {
    const uint64_t step = uint64_t(gridDim.x) * kThreads;
    for (uint64_t u = uint64_t(blockIdx.x) * kThreads + threadIdx.x; u < a.units; u += step)
        file_direct_unit<M>(a, rotated_column(u, a));
    if (a.sig.flag) signal_done(a.sig.flag, a.sig.ctr, a.sig.seq, nullptr);
}

// Tiled form: a workgroup takes tile_rows block rows, loads their file bytes
// (one contiguous run of tile_rows * k * block bytes, 64-byte aligned when the
// file is) into LDS with coalesced 8-byte loads, then codes the tile's columns
// from LDS and writes each output's tile_rows * block bytes as one run.  Over
// the link every read and write is then whole 64-byte lines: 1000-byte blocks
// had cut the column order's runs at every block edge (44.5 GiB/s against 51
// for 1024-byte blocks, profiles/r5/pfile_block_r5z.txt).  4+2, 256 MiB pinned
// file, 1000-byte blocks: 44.4 -> 51.2-51.7 GiB/s, 0.98 of the link bound
// (profiles/r5/pfile_tiled_r5z.txt).
template <int M>
__global__ void __launch_bounds__(kThreads) file_direct_tiled_kernel(FileDirect a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t tile_bytes[];  // tile_rows * k * block bytes
    uint64_t *tile = reinterpret_cast<uint64_t *>(tile_bytes);
    const uint64_t kb = uint64_t(a.k) * a.block, rows = a.units * 8 / a.block;
    const uint64_t ntiles = (rows + a.tile_rows - 1) / a.tile_rows;
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t r0 = t * a.tile_rows, nr = min(a.tile_rows, rows - r0);
        __syncthreads();  // the previous tile's LDS reads are done
        // (zeros past the file: its padding); eight loads in flight per lane
        // before their LDS stores, so a few workgroups still keep the link busy
        const uint64_t nq = nr * kb / 8;
        for (uint64_t q0 = threadIdx.x; q0 < nq; q0 += 8 * kThreads) {
            uint64_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint64_t q = q0 + uint64_t(j) * kThreads;
                v[j] = q < nq ? load_run8(a.file, r0 * kb + q * 8, a.file_len) : 0;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint64_t q = q0 + uint64_t(j) * kThreads;
                if (q < nq) tile[q] = v[j];
            }
        }
        __syncthreads();
        for (uint64_t u = threadIdx.x; u < nr * a.block / 8; u += kThreads) {
            const uint64_t cl = u * 8, r = cl / a.block, w = cl - r * a.block, c = r0 * a.block + cl;
            uint32_t lo[M > 0 ? M : 1] = {}, hi[M > 0 ? M : 1] = {};
            for (int i = 0; i < a.k; ++i) {
                const uint64_t x = tile[((r * uint64_t(a.k) + uint64_t(i)) * a.block + w) / 8];
                if (a.out[i]) __builtin_nontemporal_store(x, reinterpret_cast<uint64_t *>(RSAMD_G(a.out[i] + c, 8)));
#pragma unroll
                for (int p = 0; p < M; ++p) fold_unit(a.tabs + (i * M + p) * 5, x, lo[p], hi[p]);
            }
#pragma unroll
            for (int p = 0; p < M; ++p)
                __builtin_nontemporal_store(uint64_t(lo[p]) | (uint64_t(hi[p]) << 32),
                                            reinterpret_cast<uint64_t *>(RSAMD_G(a.out[a.k + p] + c, 8)));
        }
    }
    if (a.sig.flag) signal_done(a.sig.flag, a.sig.ctr, a.sig.seq, nullptr);
}

// 128 x 256 threads.  256 MiB file, 4+2, GiB/s (tools/direct_file_probe.py,
// profiles/r3/direct_file_r3s2j.txt; link bound 32.1):
//   blocks                     128    256    512
//   encode numpy / pinned     30.0   29.4   28.8  /  30.1   29.7   29.6
//   decode {0,5}              29.2   29.0   29.1  /  29.2   29.1   29.2
// Before the column rotation, numpy arrays read 27.2 / 27.6 (r3s2i).
constexpr unsigned kFileDirectBlocks = 128;

unsigned file_direct_grid(uint64_t units) {
    const uint64_t blocks = tuning_size("RSAMD_DIRECT_BLOCKS", kFileDirectBlocks);
    return unsigned(std::max<uint64_t>(1, std::min<uint64_t>(blocks, (units + kThreads - 1) / kThreads)));
}

}  // namespace

// Block rows per workgroup of the tiled kernel: as many as fit 64 KiB of LDS,
// rounded down to a multiple that keeps every tile's runs on 64-byte lines
// (1000-byte blocks, k = 4: 16 rows, 64000 bytes); 0 (the column kernel) when
// not one row fits.  TUNING builds: RSAMD_FILE_DIRECT_TILE=0 turns it off.
static uint64_t file_tile_rows(int k, uint64_t block) {
    if (!tuning_size("RSAMD_FILE_DIRECT_TILE", 1)) return 0;
    const uint64_t kb = uint64_t(k) * block, fit = (uint64_t(64) << 10) / kb;
    uint64_t g = 64, b = block;
    while (b) { const uint64_t t = g % b; g = b; b = t; }  // gcd(64, block)
    const uint64_t align = 64 / g;
    return fit >= align ? fit / align * align : fit;
}

bool file_direct_ok(const FileDirect &d) {
    bool ok = d.k >= 1 && d.k <= kMaxDirectIn && d.nout >= 0 && d.nout <= kMaxOut && d.block >= 8 &&
              d.block % 8 == 0 && d.units * 8 % d.block == 0 && aligned(d.file, 8);
    for (int i = 0; ok && i < d.k + d.nout; ++i) ok = aligned(d.out[i], 8);
    return ok;
}

// The rotation of rotated_column: bytes from the first shard's address to the
// widest power-of-two boundary (<= 4 KiB) every shard address agrees on.
static uint64_t file_direct_rot(const FileDirect &d) {
    std::vector<const void *> ptrs;
    for (int i = 0; i < d.k + d.nout; ++i)
        if (d.out[i]) ptrs.push_back(d.out[i]);
    if (ptrs.empty()) return 0;
    for (uintptr_t A = 4096; A > 8; A >>= 1) {
        const uintptr_t r = reinterpret_cast<uintptr_t>(ptrs[0]) % A;
        bool same = true;
        for (const void *p : ptrs) same = same && reinterpret_cast<uintptr_t>(p) % A == r;
        if (same) return ((A - r) % A) % (d.units * 8);
    }
    return 0;
}

hipError_t launch_file_encode_direct(const FileDirect &d0, hipStream_t s) {
    if (!file_direct_ok(d0)) return hipErrorInvalidValue;
    if (d0.units == 0) return hipSuccess;
    FileDirect d = d0;
    d.rot = file_direct_rot(d);
    d.tile_rows = file_tile_rows(d.k, d.block);
    // Few tiles leave most CUs idle: below 32 tiles (2 MiB of a 4+2 file) the
    // column kernel spreads the file over every CU instead.  Small pageable
    // files (the zero-copy split, capi.cpp file_encode_zc_split), encode per
    // call, tiles / columns: 88 KB 45 / 36 us, 256 KiB 51 / 42-44, 1 MiB 90 /
    // 85-86, 3 MiB 175 / 182-187; 256 MiB pinned 51.4-52.0 / 44.4 GiB/s
    // (profiles/r5/host_sizes_tile8_r5zz.txt, pfile_tile8_r5zz.txt; TUNING
    // builds: RSAMD_FILE_TILE_MIN tiles).
    if (d.tile_rows && (d.units * 8 / d.block + d.tile_rows - 1) / d.tile_rows < tuning_size("RSAMD_FILE_TILE_MIN", 32))
        d.tile_rows = 0;
    if (d.tile_rows) {
        const uint64_t rows = d.units * 8 / d.block, ntiles = (rows + d.tile_rows - 1) / d.tile_rows;
        const dim3 grid(unsigned(std::min<uint64_t>(ntiles, tuning_size("RSAMD_FILE_TILE_BLOCKS", 512))));
        const size_t lds = size_t(d.tile_rows * d.k * d.block);
        switch (d.nout) {
        case 0: hipLaunchKernelGGL((file_direct_tiled_kernel<0>), grid, dim3(kThreads), lds, s, d); break;
        case 1: hipLaunchKernelGGL((file_direct_tiled_kernel<1>), grid, dim3(kThreads), lds, s, d); break;
        case 2: hipLaunchKernelGGL((file_direct_tiled_kernel<2>), grid, dim3(kThreads), lds, s, d); break;
        case 3: hipLaunchKernelGGL((file_direct_tiled_kernel<3>), grid, dim3(kThreads), lds, s, d); break;
        default: hipLaunchKernelGGL((file_direct_tiled_kernel<4>), grid, dim3(kThreads), lds, s, d); break;
        }
        return hipGetLastError();
    }
    const dim3 grid(file_direct_grid(d.units));
    switch (d.nout) {
    case 0: hipLaunchKernelGGL((file_direct_encode_kernel<0>), grid, dim3(kThreads), 0, s, d); break;
    case 1: hipLaunchKernelGGL((file_direct_encode_kernel<1>), grid, dim3(kThreads), 0, s, d); break;
    case 2: hipLaunchKernelGGL((file_direct_encode_kernel<2>), grid, dim3(kThreads), 0, s, d); break;
    case 3: hipLaunchKernelGGL((file_direct_encode_kernel<3>), grid, dim3(kThreads), 0, s, d); break;
    default: hipLaunchKernelGGL((file_direct_encode_kernel<4>), grid, dim3(kThreads), 0, s, d); break;
    }
    return hipGetLastError();
}

hipError_t launch_split(const FileGeom &g, hipStream_t s) { return launch_split_merge(g, true, s); }
hipError_t launch_merge(const FileGeom &g, hipStream_t s) { return launch_split_merge(g, false, s); }

}  // namespace rsamd

RSAMD_BOUNDS_TU(layout)
