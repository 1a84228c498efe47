// xornet.hpp -- bitsliced XOR-network kernels, generated per coefficient
// matrix and compiled at run time (hiprtc) for gfx950.
//
// The coding product of CodingLoop.codeSomeShards (CodingLoop.java:79-85)
//     out[p][b] = XOR_i mul(row[p][i], in[i][b])
// is linear over GF(2): with each shard's bytes transposed into 8 bit planes,
// multiplication by a constant c is a fixed 8x8 bit matrix, and a whole
// coefficient matrix becomes a fixed XOR network over 32-bit plane words.  For
// a KNOWN matrix that network needs about 0.5 VALU op per byte per
// (input, output) pair plus 1.5 ops per byte per shard for the two transposes,
// against 1.125 + 1.25/nout for the table-lookup kernels (kernels.hip): for
// 10+4 about 40% fewer VALU ops, and 10+4 is VALU-issue bound.
// So each distinct plan matrix (encode rows, or a fused decode matrix) gets
// its own kernel source with the network unrolled, compiled once per device and
// cached.  Layout and block order match the vector kernels; one lane codes 32
// bytes of every shard (two 16-byte halves 1 KiB apart), one wave a 2 KiB
// column chunk of one stripe.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace rsamd {

constexpr uint32_t kXorChunk = 2048;  // bytes of a shard one wave codes

// Kernel arguments (one struct, passed by value; mirrored in the generated source).
struct XorNetArgs {
    uint8_t *base;           // column 0 of stripe 0
    const int32_t *in_idx;   // shard index of input i inside a stripe
    const int32_t *out_idx;  // shard index of output p
    uint64_t stripe_stride;
    uint64_t shard_stride;
    uint32_t chunks;    // 2 KiB chunks per stripe in this launch
    uint32_t n_items;   // blocks in this launch
    uint32_t cdiv_m, cdiv_s1, cdiv_s2;  // division by chunks (multiply-high)
    uint32_t xcd_span;  // XCD-contiguous block remap span (0 = off)
    uint32_t rot;       // chunk rotation per stripe (0 = off), as the vector kernels' block order
    int *mismatch;      // verify kernels only
};

// Kernel source for out = rows x in (rows: nout x nin, row-major), coding
// (verify = false) or checking into *mismatch (verify = true).  `name` is the
// extern "C" kernel symbol.  `ops`, when given, receives the VALU operation
// count of the network and transposes per 32 columns (for DESIGN.md numbers).
std::string xornet_source(const uint8_t *rows, int nin, int nout, bool verify, const std::string &name,
                          int *ops = nullptr);

// The compiled kernel for a matrix on the calling thread's current device,
// built on first use and cached (thread-safe).  hipSuccess with *fn set, or an
// error with *err describing a compile failure.
hipError_t xornet_function(const uint8_t *rows, int nin, int nout, bool verify, hipFunction_t *fn,
                           std::string *err);

// Launch over `n_items` blocks of one wave each.
hipError_t launch_xornet(hipFunction_t fn, const XorNetArgs &a, hipStream_t s);

// Whether large launches take these kernels by default: the RSAMD_XORNET
// environment variable ("1" = on; off otherwise: measured no faster than the
// table kernels on MI355X, whose wide-code rate is set by the memory access
// pattern -- DESIGN.md 3.5); rs_debug_xornet overrides (kernels.hip).
bool xornet_enabled();

// Number of kernels compiled so far in this process (tests, probes).
int xornet_compiled_count();

}  // namespace rsamd
