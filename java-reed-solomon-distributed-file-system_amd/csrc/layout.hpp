// layout.hpp -- launchers for the file <-> shard layout kernels (layout.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "kernels.hpp"

namespace rsamd {

// A file and its k data shards (+ parity shards after them) in device memory.
// Shard s starts at shards + s * shard_stride; every shard is S bytes.
struct FileGeom {
    const uint8_t *file = nullptr;  // encode source
    uint8_t *file_out = nullptr;    // decode destination
    size_t file_len = 0;            // encode: unpadded length; decode: trimmed size
    size_t block = 0;               // ConfigVariables.BLOCK_SIZE (1000 in the DFS)
    int k = 0;
    size_t S = 0;                   // padded / k
    uint8_t *shards = nullptr;
    size_t shard_stride = 0;
};

// Device image for the fused decode-to-file kernel:
//   uint32 tabs[k][E][5]  rows of the missing data shards over the survivors
//   int32  in_idx[k]      survivor shard indices (first k present)
//   int32  dsrc[k]        data shard i: survivor position (>= 0) or -(row + 1)
struct FileDecodePlan {
    const uint32_t *tabs = nullptr;
    const int32_t *in_idx = nullptr;
    const int32_t *dsrc = nullptr;
    int n_missing_data = 0;
};

// True when the fused kernels apply: k == 4, block % 8 == 0, S % block == 0,
// 16-byte aligned shards and stride, 8-byte aligned file.
bool file_fusable(const FileGeom &g, bool encode);

// file -> k data shards + the first <= 4 parity shards (parity0 may be null for m == 0).
hipError_t launch_file_encode_fused(const FileGeom &g, const DevPlan *parity0, hipStream_t s);
// k survivors -> file (missing data shards computed in registers, nothing else written).
hipError_t launch_file_decode_fused(const FileGeom &g, const FileDecodePlan &p, hipStream_t s);
// The host file encode's direct path: a file and shards in page-locked host
// memory (device addresses from hipHostGetDevicePointer), coded in place
// across the link by one kernel (layout.hip file_direct_encode_kernel).
// Every pointer 8-byte aligned, block % 8 == 0, units = S / 8.  file
// (file_len unpadded bytes) -> out[0 .. k) data shards (each may be null: the
// caller splits them on the host) and out[k .. k + nout) parity shards; tabs =
// the encode plan's [k][nout][5].  (The host file decode rebuilds shards with
// the shard direct kernels and merges on the host: capi.cpp file_decode_pinned.)
struct FileDirect {
    const uint8_t *file = nullptr;
    uint64_t file_len = 0;
    uint64_t units = 0;
    uint64_t block = 0;
    uint8_t *out[kMaxDirectIn + kMaxOut] = {};
    const uint32_t *tabs = nullptr;
    int k = 0, nout = 0;
    uint64_t rot = 0;        // set by the launcher (layout.hip rotated_column)
    uint64_t tile_rows = 0;  // set by the launcher: block rows per workgroup of the tiled kernel
    DirectSignal sig;        // sig.flag == nullptr: no completion signal (capi.cpp file_encode_zc_split)
};
bool file_direct_ok(const FileDirect &d);
hipError_t launch_file_encode_direct(const FileDirect &d, hipStream_t s);
// Generic permutation copies (any k, block, alignment).
hipError_t launch_split(const FileGeom &g, hipStream_t s);
hipError_t launch_merge(const FileGeom &g, hipStream_t s);

}  // namespace rsamd
