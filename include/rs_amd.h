/*
 * rs_amd.h -- C-ABI of the MI355X Reed-Solomon engine (librsamd.so).
 *
 * Drop-in boundary for the reference codec (Backblaze JavaReedSolomon as
 * vendored in /root/reference/src/main/java/edu/cmu/reedsolomon/).  Every
 * byte of shard data is coded on the GPU by hand-written HIP kernels for
 * gfx950; the host code here only validates arguments, builds GF(2^8)
 * matrices (k x k inversions, as the reference does on the host) and moves
 * bytes.  There is no CPU coding path: with no usable GPU every coding call
 * returns RS_E_HIP / RS_E_NO_DEVICE.
 *
 * Conventions
 *  - Return 0 on success or a negative RS_E_* code.  rs_last_error_message()
 *    then holds the text the Java code would have put in its
 *    IllegalArgumentException (thread-local), so a JNI shim can ThrowNew.
 *  - Argument checks run in the reference's order
 *    (ReedSolomon.java:277-302), all before anything is written: nothing is
 *    written on an argument error.  A call that fails later (RS_E_HIP, or a
 *    relocator's failed acquire) returns only once nothing of it is still in
 *    flight, but may have written part of its outputs.
 *  - Host entry points are synchronous and use the calling thread's current
 *    HIP device.  *_dev entry points are asynchronous on `stream` (a
 *    hipStream_t passed as void*, NULL = the null stream).
 *  - A codec handle is immutable after rs_codec_create and safe to share
 *    between threads (the Java codec is one static final instance:
 *    ReedSolomonEncoder.java:17).
 */
#ifndef RS_AMD_H
#define RS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes.  Java exception each one maps to, and its text. */
enum {
    RS_OK = 0,
    RS_E_WRONG_NSHARDS = -1,    /* IAE "wrong number of shards: <n>"          ReedSolomon.java:281 */
    RS_E_SIZE_MISMATCH = -2,    /* IAE "Shards are different sizes"           ReedSolomon.java:288 */
    RS_E_NEG_OFFSET = -3,       /* IAE "offset is negative: <off>"            ReedSolomon.java:294 */
    RS_E_NEG_COUNT = -4,        /* IAE "byteCount is negative: <n>"           ReedSolomon.java:297 */
    RS_E_TOO_SMALL = -5,        /* IAE "buffers to small: <n><off>"           ReedSolomon.java:300 */
    RS_E_NOT_ENOUGH = -6,       /* IAE "Not enough shards present"            ReedSolomon.java:198 */
    RS_E_TOO_MANY_SHARDS = -7,  /* IAE "too many shards - max is 256"         ReedSolomon.java:45  */
    RS_E_SINGULAR = -8,         /* IAE "Matrix is singular"                   Matrix.java:310      */
    RS_E_HIP = -9,              /* HIP runtime failure (message has the HIP error string)          */
    RS_E_INVALID = -10,         /* bad argument the Java API cannot express (NULL, k<1, layout)    */
    RS_E_TEMP_TOO_SMALL = -11,  /* IAE "tempBuffer is not big enough"         ReedSolomon.java:150 */
    RS_E_NO_DEVICE = -12        /* no HIP device visible                                           */
};

#if defined(__GNUC__)
#define RS_API __attribute__((visibility("default")))
#else
#define RS_API
#endif

typedef struct rs_codec rs_codec;

/* ABI version of this header.  It goes up whenever an existing entry point's
 * arguments change, so a dynamic binder (ctypes, JNA, dlsym) can refuse a
 * library it was not written for: bind only if rs_abi_version() equals the
 * RS_AMD_ABI_VERSION the binding was written against.
 *   3: rs_granule_copy_shard takes n_stripes after granule (round 3).
 *   4: rs_abi_version (this), rs_shard_stride_recommended.
 *   5: rs_set_host_register and rs_host_registry_state removed: the library
 *      no longer page-locks caller memory (round 5).
 *   6: rs_host_alloc / rs_host_free (caller-owned pinned buffers).
 *   7: rs_decode_groups_shard_major (the master's recovery on host arrays),
 *      rs_set_relocator (movable caller arrays: one call per JNI call). */
#define RS_AMD_ABI_VERSION 7
RS_API int rs_abi_version(void);

/* ---------------------------------------------------------------------------
 * Codec lifetime -- replaces ReedSolomon.create / the 3-arg constructor
 * (ReedSolomon.java:30-57).  Builds the systematic generator matrix
 * G = vandermonde(k+m, k) * inverse(top k x k) exactly as buildMatrix
 * (ReedSolomon.java:312-343).  No device work happens here.
 * ------------------------------------------------------------------------- */
RS_API int rs_codec_create(int data_shards, int parity_shards, rs_codec **out);
RS_API void rs_codec_destroy(rs_codec *codec);
RS_API int rs_codec_data_shard_count(const rs_codec *codec);   /* getDataShardCount   ReedSolomon.java:62 */
RS_API int rs_codec_parity_shard_count(const rs_codec *codec); /* getParityShardCount ReedSolomon.java:69 */
RS_API int rs_codec_total_shard_count(const rs_codec *codec);  /* getTotalShardCount  ReedSolomon.java:76 */
/* Copy G ((k+m) x k, row-major) to out_rows. */
RS_API int rs_codec_matrix(const rs_codec *codec, uint8_t *out_rows);
/* The single fused decode matrix for a presence pattern (see rs_decode_missing):
 * survivors[k] = first k present shard indices, missing[] = absent indices in
 * ascending order, rows (n_missing x k) maps survivors -> each missing shard. */
RS_API int rs_codec_decode_matrix(const rs_codec *codec, const uint8_t *present, int nshards,
                           int *survivors, int *missing, int *n_missing, uint8_t *rows);

RS_API const char *rs_last_error_message(void);
/* Free the calling thread's device contexts (streams, staging buffers) and the
 * process's idle pooled pinned slots of the pageable-call pipeline (at most
 * four sets, 384 MiB, per device are kept idle between calls). */
RS_API void rs_thread_release(void);
/* Number of visible HIP devices (0 when none). */
RS_API int rs_device_count(void);
/* ---------------------------------------------------------------------------
 * Host-buffer API (JNI-facing).  Shards are caller-owned host arrays,
 * mutated in place.  shard_lens[i] is the Java array length of shards[i]
 * (for the size checks).  The library never page-locks caller memory:
 *  - arrays the caller page-locked itself (hipHostMalloc, hipHostRegister,
 *    pinned tensors) are coded in place across the link by one kernel;
 *  - pageable arrays (JVM heap arrays through JNI) are copied chunk by chunk
 *    into the library's own device-mapped pinned slots, coded there by the
 *    same kernels and copied back, the copies overlapped with the link.
 * ------------------------------------------------------------------------- */

/* ReedSolomon.encodeParity(byte[][] shards, int offset, int byteCount)
 * (ReedSolomon.java:90-104): parity shards k..k+m-1 := G[k..] * data. */
RS_API int rs_encode_parity(const rs_codec *codec, uint8_t *const *shards, int nshards,
                     const int64_t *shard_lens, int32_t offset, int32_t byte_count);

/* ReedSolomon.decodeMissing(byte[][] shards, boolean[] shardPresent, int offset,
 * int byteCount) (ReedSolomon.java:175-272).  present[i] != 0 marks shard i
 * present.  All present -> returns without touching anything (:190-194).
 * Survivors are the first k present shards in index order (:210-223); every
 * missing shard (data and parity) is produced in ONE GPU pass from them with
 * the matrix rs_codec_decode_matrix reports (bit-identical to Java's two
 * passes).  Missing buffers must be allocated; their contents
 * are overwritten. */
RS_API int rs_decode_missing(const rs_codec *codec, uint8_t *const *shards, int nshards,
                      const int64_t *shard_lens, const uint8_t *present,
                      int32_t offset, int32_t byte_count);

/* ReedSolomon.isParityCorrect(shards, firstByte, byteCount[, tempBuffer])
 * (ReedSolomon.java:115-164).  temp may be NULL; when given, temp_len is its
 * length and only its size is checked (the GPU needs no scratch; the Java
 * tempBuffer is scratch and its contents are not part of the contract).
 * *result = 1 when every parity byte matches, else 0. */
RS_API int rs_is_parity_correct(const rs_codec *codec, uint8_t *const *shards, int nshards,
                         const int64_t *shard_lens, int32_t first_byte, int32_t byte_count,
                         const uint8_t *temp, int64_t temp_len, int *result);

/* ReedSolomon.checkBuffersAndSizes (ReedSolomon.java:277-302) alone, on the
 * shard count and lengths: the checks (same order, same error codes and
 * text) every host entry point above starts with.  A JNI shim that stages
 * large calls through its own buffers validates with it
 * before copying anything. */
RS_API int rs_check_buffers_and_sizes(const rs_codec *codec, int nshards, const int64_t *shard_lens,
                                      int64_t offset, int64_t byte_count);

/* The master's recovery loop on HOST arrays (MasterImpl.recoverOfflineChunkserver,
 * MasterImpl.java:733-743, 794-839, with ChunkserverDiskRecoveryMachine.java:
 * 34-48 per chunk group), in the master's own layout: one array per server,
 * the groups back to back -- chunk g of server s at servers[s] + g*chunk_len
 * (server_lens[s] >= n_groups*chunk_len; bytes past that are untouched).
 * present holds n_groups x (k+m) flags, group after group (nonzero: server s
 * answered for group g); every absent chunk of every group is rebuilt in
 * place from the group's first k present chunks (ReedSolomon.java:210-223),
 * present chunks are not written.  The GPU form of the Java loop that calls
 * decodeMissing once per 6 x 1000-B group: the offline set is the same for
 * every group and only grows when a read fails mid-loop, so the groups form a
 * few runs of one pattern, and a run of n groups is ONE decodeMissing of
 * n*chunk_len-byte shards (rs_decode_missing's host paths: pageable arrays
 * through the mirrored pipeline, the library's pinned buffers coded in place).
 * Flags that form many runs (more than one per 128 MiB, at least 8) are
 * decoded in chunks of groups by the per-stripe pattern kernels.  Checks, in
 * this order, before anything is written: nservers != k+m ->
 * RS_E_WRONG_NSHARDS; NULL arrays -> RS_E_INVALID; a server array shorter than
 * n_groups*chunk_len -> RS_E_INVALID; a group with fewer than k present ->
 * RS_E_NOT_ENOUGH ("Not enough shards present"). */
RS_API int rs_decode_groups_shard_major(const rs_codec *codec, uint8_t *const *servers, int nservers,
                                        const int64_t *server_lens, size_t chunk_len, size_t n_groups,
                                        const uint8_t *present);

/* Movable caller arrays (a JVM's heap byte[]s, reached through JNI): the
 * library reads and writes caller memory only in copy batches -- a chunk's
 * inputs into its pinned slots, outputs back, a file's rows split or merged --
 * and never holds a caller address across one.  With a relocator set on the
 * calling thread, every host entry point it calls brackets each batch with
 * acquire(user, base) -- pin every array (GetPrimitiveArrayCritical) and store
 * its current address into base[0..n) -- and release(user, base), and moves
 * every address inside [keys[i], keys[i] + lens[i]] the call was given to the
 * same offset from base[i].  Between batches (while the GPU codes) the arrays
 * are unpinned and may move, so a caller needs no critical region across the
 * call, and one call codes the whole range with no restart of the pipeline.
 * The keys are stand-in addresses that are never dereferenced: pass them (or
 * pointers made from them) as the call's array arguments; they must not
 * overlap any real memory the call uses (non-canonical addresses do not).
 * Caller arrays are never treated as pinned while a relocator is set.  An
 * acquire that returns nonzero skips its batch and the call returns RS_E_INVALID
 * ("relocator: acquire failed"; outputs may then be partly written).  The
 * struct is copied; keys and lens must stay valid until the relocator is
 * cleared with rs_set_relocator(NULL).  RS_E_INVALID for n < 1 or NULL members. */
typedef struct rs_relocator {
    void *user;
    int n;
    const uint8_t *const *keys;
    const int64_t *lens;
    int (*acquire)(void *user, uint8_t **base);
    void (*release)(void *user, uint8_t **base);
} rs_relocator;
RS_API int rs_set_relocator(const rs_relocator *relocator);

/* CodingLoop.codeSomeShards(matrixRows, inputs, inputCount, outputs, outputCount,
 * offset, byteCount) (CodingLoop.java:79-85; default impl
 * InputOutputByteTableCodingLoop.java:12-44): outputs[o][b] =
 * XOR_i mul(matrix_rows[o][i], inputs[i][b]) for b in [offset, offset+byte_count).
 * matrix_rows[o] has input_count entries.  Outputs must not alias inputs. */
RS_API int rs_code_some_shards(const uint8_t *const *matrix_rows, const uint8_t *const *inputs,
                        int input_count, uint8_t *const *outputs, int output_count,
                        int32_t offset, int32_t byte_count);

/* CodingLoop.checkSomeShards(...) (CodingLoop.java:110-117, CodingLoopBase.java:17-41):
 * *result = 1 iff to_check[o][b] equals the product for every o, b. */
RS_API int rs_check_some_shards(const uint8_t *const *matrix_rows, const uint8_t *const *inputs,
                         int input_count, const uint8_t *const *to_check, int check_count,
                         int32_t offset, int32_t byte_count, int *result);

/* ---------------------------------------------------------------------------
 * Device-resident batched API (the benchmark path; no Java counterpart --
 * it is what a stripe-batching caller uses).  Layout: shard s of stripe t
 * starts at dev_base + t*stripe_stride + s*shard_stride; shard_len bytes are
 * coded per shard.  Fast path when dev_base, both strides are multiples of 16
 * (any shard_len); when they are multiples of 8 (the DFS's 1000-byte chunk
 * groups packed back to back), 8-byte-vector kernels; otherwise a
 * byte-granular kernel is used.
 * ------------------------------------------------------------------------- */

/* Encode parity for n_stripes stripes. */
RS_API int rs_encode_batch_dev(const rs_codec *codec, uint8_t *dev_base, size_t n_stripes,
                        size_t shard_len, size_t shard_stride, size_t stripe_stride, void *stream);

/* Reconstruct the shards absent from present[0..k+m) in every stripe (one
 * presence pattern for the whole batch). */
RS_API int rs_decode_batch_dev(const rs_codec *codec, uint8_t *dev_base, const uint8_t *present,
                        size_t n_stripes, size_t shard_len, size_t shard_stride,
                        size_t stripe_stride, void *stream);

/* Reconstruct with a presence pattern PER STRIPE (the
 * master's per-chunk-group recovery, MasterImpl.java:794-839 with
 * ChunkserverDiskRecoveryMachine.java:34-48, and client reads with different
 * missing shards per stripe).  present is a HOST array of n_stripes x (k+m)
 * flags.  One launch per group of <= 4 outputs; each stripe reads its own
 * first-k-present survivors and writes its own absent shards.  Every stripe
 * needs >= k present shards (else RS_E_NOT_ENOUGH before any launch).
 * Asynchronous on stream.  For k+m <= 20 (and at most 65536 decodable
 * patterns) the flags become per-stripe bitmasks looked up in the codec's
 * pattern table (see below); wider codes get per-call records.  The per-call
 * bytes live in one of two per-thread staging slots used in turn: a call
 * waits only for the kernels of the masked call two before it. */
RS_API int rs_decode_batch_masked_dev(const rs_codec *codec, uint8_t *dev_base, const uint8_t *present,
                                      size_t n_stripes, size_t shard_len, size_t shard_stride,
                                      size_t stripe_stride, void *stream);

/* The same with the presence patterns already in HBM: dev_present_bits[t]
 * has bit i set when shard i of stripe t is present (no host work per call,
 * graph-capturable).  The codec's pattern table -- a record for every
 * bitmask with >= k bits set and a 2^(k+m) id table -- is built and uploaded
 * on the first call per device (blocking); RS_E_INVALID when k+m > 20 or the
 * code has more than 65536 decodable patterns.  Stripes with fewer than k
 * present shards (or bits >= 2^(k+m)) are left untouched and, when
 * dev_bad_count is not NULL, counted into that device int32 (atomic adds;
 * the caller zeroes it).  A stripe with every shard present is untouched. */
RS_API int rs_decode_batch_masked_bits_dev(const rs_codec *codec, uint8_t *dev_base,
                                           const uint32_t *dev_present_bits, size_t n_stripes,
                                           size_t shard_len, size_t shard_stride, size_t stripe_stride,
                                           int32_t *dev_bad_count, void *stream);

/* The master's recovery loop batched in its own layout (SURVEY.md 8f row f2;
 * MasterImpl.recoverOfflineChunkserver, MasterImpl.java:733-743, 794-839,
 * with ChunkserverDiskRecoveryMachine.java:34-48 per chunk group).  The
 * master reads chunk group g's chunk from every present chunkserver; a
 * batching master keeps ONE array per server with the groups back to back:
 * chunk g of server s at dev_base + s*server_stride + g*chunk_len (shard-major,
 * [server][group*chunk]).  The offline set is the same for every group and
 * only grows when a read fails mid-loop, so the groups form a few runs of one
 * presence pattern each, and a run of n groups is byte for byte ONE stripe of
 * n*chunk_len-byte shards: one launch at the headline kernels' rate instead
 * of n 1000-byte stripes.  present holds n_groups x (k+m) HOST flags (group g's
 * pattern); every absent chunk of every group is rebuilt in place, survivors
 * the first k present (ReedSolomon.java:210-223).  RS_E_NOT_ENOUGH (nothing
 * enqueued) when any group has fewer than k present; RS_E_INVALID when
 * server_stride < n_groups*chunk_len.  Full rate with dev_base and
 * server_stride 1 KiB aligned; a run that starts mid-line peels its first
 * bytes onto a byte kernel.  Flags that form many runs (more than one per
 * 128 MiB of the batch, at least 8: patterns that change every few groups)
 * are decoded in one launch of the per-stripe pattern kernels instead, the
 * groups read as stripes of chunk_len-byte shards. */
RS_API int rs_decode_groups_shard_major_dev(const rs_codec *codec, uint8_t *dev_base, size_t server_stride,
                                            size_t chunk_len, size_t n_groups, const uint8_t *present,
                                            void *stream);

/* The shard stride a [stripe][shard][stride] batch of total_shards shards of
 * shard_len bytes should use (the stride measured fastest on MI355X for that
 * geometry): shard_len rounded up to 256 bytes, plus a pad
 * where shards a power of two apart contend for the same HBM channels.  Pass
 * it as shard_stride (and total_shards times it as stripe_stride) to the
 * batch entry points.  0 when total_shards < 1 or shard_len == 0. */
RS_API size_t rs_shard_stride_recommended(int total_shards, size_t shard_len);

/* Verify parity of every stripe: dev_mismatch (a device int) is OR-ed with 1
 * when any parity byte differs.  The caller zeroes it first. */
RS_API int rs_verify_batch_dev(const rs_codec *codec, const uint8_t *dev_base, size_t n_stripes,
                        size_t shard_len, size_t shard_stride, size_t stripe_stride,
                        int *dev_mismatch, void *stream);

/* ---------------------------------------------------------------------------
 * Granule layout: an HBM layout for stripe batches (no Java counterpart).
 * Packed, each shard's shard_len bytes are contiguous, so the k+m streams a
 * stripe's coding reads and writes lie shard_len apart (4 MiB for config[3],
 * 4 KiB for config[4]).  The granule layout lines the batch's byte columns up
 * -- stripe t's column c is batch column t*shard_len + c -- and stores them in
 * G-byte granules, granule j of every shard together:
 *     byte c of shard s of stripe t, with x = t*shard_len + c, lives at
 *     dev_base + (x / G)*(nshards*G) + s*G + (x % G),
 * where G divides shard_len (a stripe spans shard_len/G granules) or
 * shard_len divides G (a granule holds G/shard_len stripes), and G divides
 * n_stripes*shard_len.  Byte for byte that is a packed batch of
 * n_stripes*shard_len/G stripes of G-byte shards (shard_stride G,
 * stripe_stride nshards*G).  Coding is per byte column, so every batch entry
 * point above codes a granule batch unchanged through that view: encode,
 * uniform-pattern decode and verify.  Per-stripe presence patterns take
 * the rs_decode_granule_masked*_dev entry points below (one pattern per
 * stripe, as the packed ones).  A stripe's streams now lie G bytes apart, which the
 * HBM serves faster: 10+4 x 4 MiB encode 0.79-0.81 of the 8 TB/s peak at
 * G = 32 KiB against 0.70-0.75 packed, 4+2 x 1 MiB 0.84-0.85 at G = 64 KiB
 * against 0.80-0.83.
 * ------------------------------------------------------------------------- */

/* The granule measured fastest for stripes of total_shards shards: the
 * largest power of two G in [4 KiB, 1 MiB] with total_shards*G <= 512 KiB
 * (4+2: 64 KiB, 10+4: 32 KiB).  0 when total_shards < 1. */
RS_API size_t rs_granule_recommended(int total_shards);

/* rs_decode_batch_masked_dev on a granule batch of n_stripes stripes of
 * shard_len-byte shards (granule G): present holds n_stripes x (k+m) HOST
 * flags, one pattern per stripe, as there.  Each kernel block looks its
 * stripe up from its batch column (stripe = column / shard_len), so the
 * patterns are not repeated per granule row, and stripes sharing a granule
 * row (shard_len < G) may differ.  Fast vector path when shard_len and G are
 * multiples of 1 KiB; other shapes run a byte-granular kernel.  RS_E_INVALID
 * for a G that neither divides nor is divided by shard_len, or that does not
 * divide n_stripes*shard_len. */
RS_API int rs_decode_granule_masked_dev(const rs_codec *codec, uint8_t *dev_base, const uint8_t *present,
                                        size_t n_stripes, size_t shard_len, size_t granule, void *stream);

/* rs_decode_batch_masked_bits_dev on a granule batch: dev_present_bits[t] is
 * stripe t's presence bitmask (one per stripe, in HBM); dev_bad_count counts
 * each undecodable stripe once. */
RS_API int rs_decode_granule_masked_bits_dev(const rs_codec *codec, uint8_t *dev_base,
                                             const uint32_t *dev_present_bits, size_t n_stripes, size_t shard_len,
                                             size_t granule, int32_t *dev_bad_count, void *stream);

/* Move one shard between a contiguous buffer and a granule batch of
 * n_stripes stripes (asynchronous on stream; one 2-D copy of shard_len/G rows
 * when G divides shard_len, one contiguous run otherwise).  to_granules != 0:
 * buf -> shard `shard` of stripe `stripe`; else that shard -> buf.  buf holds
 * shard_len bytes and may be host memory (pinned or pageable) or device
 * memory.  RS_E_INVALID (nothing copied) for NULL pointers, a stripe outside
 * [0, n_stripes), shard_len or granule 0, neither of shard_len and granule
 * dividing the other, or a shard index outside [0, total_shards). */
RS_API int rs_granule_copy_shard(uint8_t *dev_base, int total_shards, size_t n_stripes, size_t shard_len,
                                 size_t granule, size_t stripe, int shard, void *buf, int to_granules, void *stream);

/* ---------------------------------------------------------------------------
 * Client file layout: ReedSolomonEncoder /
 * ReedSolomonDecoder (client/ReedSolomonEncoder.java:56-85,
 * client/ReedSolomonDecoder.java:33-39,62-103, ConfigVariables.java:4-9).
 * The file is zero-padded to a multiple of k*block; file block b goes to data
 * shard b % k at offset (b / k) * block; shard_len = padded / k.  The DFS uses
 * block = 1000, k = 4, m = 2.  For k == 4, block % 8 == 0 and aligned
 * buffers, encode reads the file and decode writes it inside the coding
 * kernels (no separate split / merge pass).
 * ------------------------------------------------------------------------- */

/* pad() geometry (ReedSolomonEncoder.java:76-85): padded length and shard length. */
RS_API int rs_file_layout(const rs_codec *codec, int64_t file_len, int32_t block, int64_t *padded_len,
                          int64_t *shard_len);

/* ReedSolomonEncoder.encode() (ReedSolomonEncoder.java:56-74) on host buffers:
 * pad + split + encodeParity.  shards_out[0..k+m) must each hold shard_len
 * bytes (rs_file_layout); data shards and parity are written. */
RS_API int rs_file_encode(const rs_codec *codec, const uint8_t *file, int64_t file_len, int32_t block,
                          uint8_t *const *shards_out, int nshards, const int64_t *shard_lens);

/* new ReedSolomonDecoder(shards, shardPresent, byteCntInShard, fileSize)
 * (ReedSolomonDecoder.java:33-39): decodeMissing(shards, present, 0,
 * byteCntInShard) -- missing shards are filled in place, as in the Java --
 * then merge the data shards and trim to file_size into file_out.
 * shard_lens[0] % block must be 0 and file_size <= k * shard_lens[0]
 * (the Java would throw ArrayIndexOutOfBounds otherwise): RS_E_INVALID. */
RS_API int rs_file_decode(const rs_codec *codec, uint8_t *const *shards, int nshards, const int64_t *shard_lens,
                          const uint8_t *present, int32_t byte_cnt_in_shard, int32_t block, uint8_t *file_out,
                          int64_t file_size);

/* Device versions.  dev_shards holds k+m shards of shard_len bytes at
 * dev_shards + s*shard_stride.  Encode: file -> all k+m shards.  Decode:
 * survivors -> the trimmed file; with write_missing != 0 the absent shards
 * are also reconstructed in dev_shards.  With write_missing == 0 the absent
 * shard buffers are scratch: the fused k == 4 path leaves them untouched, the
 * generic path reconstructs them in place before merging. */
RS_API int rs_file_encode_dev(const rs_codec *codec, const uint8_t *dev_file, size_t file_len, size_t block,
                              uint8_t *dev_shards, size_t shard_stride, void *stream);
RS_API int rs_file_decode_dev(const rs_codec *codec, uint8_t *dev_shards, size_t shard_len, size_t shard_stride,
                              const uint8_t *present, size_t block, uint8_t *dev_file_out, size_t file_size,
                              int write_missing, void *stream);

/* ---------------------------------------------------------------------------
 * HBM for stripe batches (no Java counterpart).  A service that keeps its
 * stripes resident allocates the pool once.  With contiguous != 0 the bytes
 * are one physically contiguous range (hipExtMallocWithFlags,
 * hipDeviceMallocContiguous): the 4+2 x 1 MiB encode runs at 0.823-0.825 of
 * peak there against 0.809-0.813 on hipMalloc memory (tools/alloc_probe.py).
 * If that fails the call falls back to hipMalloc; *got_contiguous (may be
 * NULL) says which one it got.  Free with rs_dev_free.
 * ------------------------------------------------------------------------- */
RS_API int rs_dev_alloc(void **out, size_t bytes, int contiguous, int *got_contiguous);
RS_API int rs_dev_free(void *ptr);

/* ---------------------------------------------------------------------------
 * Pinned host memory for callers that can keep their shards and files in it
 * (no Java counterpart; a JVM reaches it as direct ByteBuffers,
 * NativeReedSolomon.allocatePinned).  Page-locked, mapped for the device,
 * pages placed by the calling thread's NUMA policy.  Host calls on arrays in
 * it are coded in place across the link with no host copies (DESIGN.md 5.2:
 * 1.00 of the link bound for 4+2 x 64 MiB encodeParity, against 0.86-0.90
 * for pageable arrays).  Free with rs_host_free, which takes only a live
 * rs_host_alloc pointer (a foreign or interior pointer, or a second free, is
 * RS_E_INVALID and frees nothing).  RS_E_NO_DEVICE without a GPU, RS_E_HIP
 * when the allocation fails.
 * ------------------------------------------------------------------------- */
RS_API int rs_host_alloc(void **out, size_t bytes);
RS_API int rs_host_free(void *ptr);

/* ---------------------------------------------------------------------------
 * Benchmark/test support (not part of the reference API).
 * ------------------------------------------------------------------------- */

/* Fill the k data shards of stripes [0, n_stripes) with synthetic bytes:
 * the k*shard_len data bytes of global stripe g = stripe0 + t, read as
 * consecutive little-endian 64-bit words w = 0,1,..., are
 * splitmix64(seed ^ g) outputs 1,2,...  shard_len % 8 == 0. */
RS_API int rs_fill_synthetic_dev(uint8_t *dev_base, int data_shards, size_t n_stripes, size_t shard_len,
                          size_t shard_stride, size_t stripe_stride, uint64_t seed,
                          uint64_t stripe0, void *stream);

/* dst := src, n bytes, with the same 16-byte streaming kernel style (the
 * "measured device copy" the roofline is also quoted against). */
RS_API int rs_copy_dev(uint8_t *dst, const uint8_t *src, size_t n, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* RS_AMD_H */
