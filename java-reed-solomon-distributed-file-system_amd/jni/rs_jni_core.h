/*
 * rs_jni_core.h -- the JNI shim's marshalling, in plain C behind a small
 * environment interface.
 *
 * rs_jni.c implements rsj_env over a JNIEnv and exports the Java natives;
 * tests/jni_mock/ implements it over mock Java arrays, so the marshalling --
 * argument checks and the exceptions they raise, local-reference accounting,
 * per-batch critical-region pinning of movable arrays, the copying fallback -- is compiled
 * and tested without a JDK.
 *
 * Semantics follow the reference Java code the natives replace:
 *   ReedSolomon.encodeParity / decodeMissing / isParityCorrect
 *     (ReedSolomon.java:90-164, 175-272; checks ReedSolomon.java:277-302),
 *   CodingLoop.codeSomeShards / checkSomeShards
 *     (CodingLoop.java:79-117, InputOutputByteTableCodingLoop.java:12-89).
 * Exceptions are the ones the Java code throws: IllegalArgumentException with
 * its text for the checks, ArrayIndexOutOfBoundsException ("Index i out of
 * bounds for length n") where Java indexes past an array, NullPointerException
 * for null arrays, IllegalStateException for a GPU failure.
 */
#ifndef RS_JNI_CORE_H
#define RS_JNI_CORE_H

#include <stddef.h>
#include <stdint.h>

#include "rs_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RSJ_MAX_SHARDS 256
#define RSJ_COMMIT 0 /* JNI release mode: copy back and free */
#define RSJ_ABORT 2  /* JNI_ABORT: free without copying back */

/* A call is ONE library call with the Java arrays movable: pinned
 * (GetPrimitiveArrayCritical) only around each of the library's copy batches
 * (rs_set_relocator).  When the JVM hands out copies instead of pinning,
 * calls are copied through C buffers (Get/SetByteArrayRegion) in slices of
 * this many bytes per shard. */
#define RSJ_SLICE_BYTES (32u << 20)

typedef void *rsj_obj; /* a jobject (jarray) */

typedef struct rsj_env rsj_env;
struct rsj_env {
    void *ctx;
    int (*array_length)(rsj_env *e, rsj_obj arr);
    rsj_obj (*object_element)(rsj_env *e, rsj_obj arr, int i); /* a new local reference, or NULL */
    void (*delete_local)(rsj_env *e, rsj_obj obj);
    int (*ensure_local_capacity)(rsj_env *e, int n);            /* 0, or < 0 with an exception pending */
    uint8_t *(*critical_get)(rsj_env *e, rsj_obj arr, int *is_copy);
    void (*critical_release)(rsj_env *e, rsj_obj arr, uint8_t *p, int mode);
    void (*byte_region_get)(rsj_env *e, rsj_obj arr, int start, int len, uint8_t *dst);
    void (*byte_region_set)(rsj_env *e, rsj_obj arr, int start, int len, const uint8_t *src);
    void (*bool_region_get)(rsj_env *e, rsj_obj arr, int start, int len, uint8_t *dst);
    int (*exception_pending)(rsj_env *e);
    void (*throw_new)(rsj_env *e, const char *cls, const char *msg);
    uint8_t *(*direct_address)(rsj_env *e, rsj_obj buf); /* NULL: not a direct buffer */
    int64_t (*direct_capacity)(rsj_env *e, rsj_obj buf);
    rsj_obj (*new_direct)(rsj_env *e, void *p, int64_t capacity); /* a new local reference, or NULL */
};

/* The coding entry points (librsamd.so's by default; tests substitute fakes). */
typedef struct rsj_backend {
    int (*encode_parity)(const rs_codec *, uint8_t *const *, int, const int64_t *, int32_t, int32_t);
    int (*decode_missing)(const rs_codec *, uint8_t *const *, int, const int64_t *, const uint8_t *, int32_t,
                          int32_t);
    int (*is_parity_correct)(const rs_codec *, uint8_t *const *, int, const int64_t *, int32_t, int32_t,
                             const uint8_t *, int64_t, int *);
    int (*code_some_shards)(const uint8_t *const *, const uint8_t *const *, int, uint8_t *const *, int, int32_t,
                            int32_t);
    int (*check_some_shards)(const uint8_t *const *, const uint8_t *const *, int, const uint8_t *const *, int,
                             int32_t, int32_t, int *);
    int (*check_buffers_and_sizes)(const rs_codec *, int, const int64_t *, int64_t, int64_t);
    int (*total_shards)(const rs_codec *);
    int (*data_shards)(const rs_codec *);
    const char *(*last_error)(void);
    int (*decode_groups_shard_major)(const rs_codec *, uint8_t *, size_t, size_t, size_t, const uint8_t *, void *);
    int (*file_layout)(const rs_codec *, int64_t, int32_t, int64_t *, int64_t *);
    int (*file_encode)(const rs_codec *, const uint8_t *, int64_t, int32_t, uint8_t *const *, int, const int64_t *);
    int (*file_decode)(const rs_codec *, uint8_t *const *, int, const int64_t *, const uint8_t *, int32_t, int32_t,
                       uint8_t *, int64_t);
    int (*host_alloc)(void **, size_t);
    int (*host_free)(void *);
    int (*decode_groups_shard_major_host)(const rs_codec *, uint8_t *const *, int, const int64_t *, size_t, size_t,
                                          const uint8_t *);
    int (*set_relocator)(const rs_relocator *);
} rsj_backend;

const rsj_backend *rsj_librsamd_backend(void);

/* The natives.  Each returns with the Java-visible outcome: results written
 * to the arrays, or an exception pending in `e`. */
void rsj_encode_parity(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, int32_t offset,
                       int32_t count);
void rsj_decode_missing(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, rsj_obj present,
                        int32_t offset, int32_t count);
/* temp may be NULL (the two-argument isParityCorrect). */
int rsj_is_parity_correct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, int32_t first,
                          int32_t count, rsj_obj temp);
void rsj_code_some_shards(rsj_env *e, const rsj_backend *b, rsj_obj rows, rsj_obj inputs, int32_t nin,
                          rsj_obj outputs, int32_t nout, int32_t offset, int32_t count);
int rsj_check_some_shards(rsj_env *e, const rsj_backend *b, rsj_obj rows, rsj_obj inputs, int32_t nin,
                          rsj_obj to_check, int32_t ncheck, int32_t offset, int32_t count);
/* MasterImpl.recoverOfflineChunkserver's loop (MasterImpl.java:794-839) over
 * chunk groups a GPU-side service keeps in HBM in the master's own layout
 * (rs_decode_groups_shard_major_dev): chunk g of server s at
 * dev_base + s*server_stride + g*chunk_len; present is a byte[] of
 * n_groups * total flags, group after group (nonzero = the server answered).
 * The flags are pinned for the call (it only enqueues kernels on `stream`);
 * a failed pin is OutOfMemoryError, as for the shard arrays. */
void rsj_recover_groups_shard_major(rsj_env *e, const rsj_backend *b, const rs_codec *c, int64_t dev_base,
                                    int64_t server_stride, int32_t chunk_len, int64_t n_groups, rsj_obj present,
                                    int64_t stream);

/* The same loop on the master's HOST arrays (rs_decode_groups_shard_major):
 * servers is a byte[][] of k+m arrays, server s's chunks of n_groups groups
 * back to back (chunk g at g * chunk_len); present as above.  Every absent
 * chunk is rebuilt in place.  One library call with the arrays movable
 * (critical regions only around the library's copy batches); argument errors
 * (short arrays, a group with fewer than k present) are thrown before any
 * array is written.  The _direct form takes a ByteBuffer[] of direct buffers
 * (allocatePinned ones are coded in place across the link). */
void rsj_recover_groups_shard_major_host(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj servers,
                                         int32_t chunk_len, int32_t n_groups, rsj_obj present);
void rsj_recover_groups_shard_major_direct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj servers,
                                           int32_t chunk_len, int32_t n_groups, rsj_obj present);

/* The client's file layout (ReedSolomonEncoder.java:56-85,
 * ReedSolomonDecoder.java:33-39, 62-66, 92-103) through rs_file_encode /
 * rs_file_decode, so only coded bytes cross the link and the split / merge
 * runs in the library instead of the Java per-byte loops.
 *   encode: the whole byte[] file, padded with zeros to a multiple of
 *     k * block, split into the data shards and the parity encoded, into
 *     `shards` (k+m byte[] of at least padded / k bytes each; bytes past that
 *     are untouched).
 *   decode: decodeMissing(shards, present, 0, byte_cnt) in place, then the
 *     data shards merged and trimmed to file_size into file_out (a byte[] of
 *     at least file_size bytes).
 * One library call with the file and the shards movable, like the shard
 * calls; when the JVM copies, slices of whole block rows (RSJ_SLICE_BYTES of
 * each shard, rounded down to the block) through C buffers, validated up
 * front, so a later slice never fails after an earlier one was written. */
void rsj_file_encode(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj file, int32_t block, rsj_obj shards);
void rsj_file_decode(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, rsj_obj present,
                     int32_t byte_cnt, int32_t block, rsj_obj file_out, int32_t file_size);

/* Direct ByteBuffers (no Java counterpart): shards and files the caller keeps
 * outside the Java heap, reached by address with no pinning and no slicing.
 * Buffers from rsj_alloc_pinned (rs_host_alloc) are page-locked, so the
 * library codes them in place across the link; other direct buffers
 * (ByteBuffer.allocateDirect) are pageable and take the mirrored pipeline.
 * A buffer's length is its capacity; an element that is not a direct buffer
 * is IllegalArgumentException ("shard i is not a direct buffer"). */
rsj_obj rsj_alloc_pinned(rsj_env *e, const rsj_backend *b, int32_t capacity);
void rsj_free_pinned(rsj_env *e, const rsj_backend *b, rsj_obj buf);
void rsj_encode_parity_direct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, int32_t offset,
                              int32_t count);
void rsj_decode_missing_direct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, rsj_obj present,
                               int32_t offset, int32_t count);
/* file: the first file_len bytes of a direct buffer; file_out receives file_size bytes */
void rsj_file_encode_direct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj file, int32_t file_len,
                            int32_t block, rsj_obj shards);
void rsj_file_decode_direct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, rsj_obj present,
                            int32_t byte_cnt, int32_t block, rsj_obj file_out, int32_t file_size);

#ifdef __cplusplus
}
#endif
#endif /* RS_JNI_CORE_H */
