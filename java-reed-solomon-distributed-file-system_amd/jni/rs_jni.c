/*
 * rs_jni.c -- JNI binding of librsamd.so for the reference's Java codec API.
 *
 * Source-only in this repository: the build container has no JDK (no jni.h,
 * no javac).  Build where a JDK 17 exists:
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *      -I<repo>/include rs_jni.c rs_jni_core.c \
 *      -L<repo>/java-reed-solomon-distributed-file-system_amd/lib \
 *      -lrsamd -Wl,-rpath,'$ORIGIN' -o librsamd_jni.so
 *
 * Java side: jni/java/edu/cmu/reedsolomon/{NativeReedSolomon,GpuCodingLoop}.java.
 * This file only adapts JNIEnv to the rsj_env interface of rs_jni_core.h; the
 * marshalling (argument checks, exceptions, local references, movable arrays
 * pinned around the library's copy batches, the copying fallback) lives in
 * rs_jni_core.c, which tests/test_jni_core.py compiles and exercises against
 * mock Java arrays.  tests/test_jni_adapter.py compiles this file against a
 * declarations-only jni.h written from the JNI specification
 * (tests/jni_spec/jni.h), so its types and calls are checked without a JDK.
 */
#include <jni.h>
#include <stdint.h>

#include "rs_amd.h"
#include "rs_jni_core.h"

typedef struct {
    rsj_env base; /* first: an rsj_env* is a jenv* */
    JNIEnv *env;
} jenv;

static JNIEnv *J(rsj_env *e) { return ((jenv *)e)->env; }

static int j_array_length(rsj_env *e, rsj_obj a) { return (*J(e))->GetArrayLength(J(e), (jarray)a); }
static rsj_obj j_object_element(rsj_env *e, rsj_obj a, int i) {
    return (*J(e))->GetObjectArrayElement(J(e), (jobjectArray)a, i);
}
static void j_delete_local(rsj_env *e, rsj_obj o) { (*J(e))->DeleteLocalRef(J(e), (jobject)o); }
static int j_ensure_local_capacity(rsj_env *e, int n) { return (*J(e))->EnsureLocalCapacity(J(e), n) == 0 ? 0 : -1; }
static uint8_t *j_critical_get(rsj_env *e, rsj_obj a, int *is_copy) {
    jboolean c = JNI_FALSE;
    uint8_t *p = (uint8_t *)(*J(e))->GetPrimitiveArrayCritical(J(e), (jarray)a, &c);
    *is_copy = c == JNI_TRUE;
    return p;
}
static void j_critical_release(rsj_env *e, rsj_obj a, uint8_t *p, int mode) {
    (*J(e))->ReleasePrimitiveArrayCritical(J(e), (jarray)a, p, mode);
}
static void j_byte_region_get(rsj_env *e, rsj_obj a, int start, int len, uint8_t *dst) {
    (*J(e))->GetByteArrayRegion(J(e), (jbyteArray)a, start, len, (jbyte *)dst);
}
static void j_byte_region_set(rsj_env *e, rsj_obj a, int start, int len, const uint8_t *src) {
    (*J(e))->SetByteArrayRegion(J(e), (jbyteArray)a, start, len, (const jbyte *)src);
}
static void j_bool_region_get(rsj_env *e, rsj_obj a, int start, int len, uint8_t *dst) {
    (*J(e))->GetBooleanArrayRegion(J(e), (jbooleanArray)a, start, len, (jboolean *)dst);
}
static int j_exception_pending(rsj_env *e) { return (*J(e))->ExceptionCheck(J(e)) == JNI_TRUE; }
static void j_throw_new(rsj_env *e, const char *cls, const char *msg) {
    jclass c = (*J(e))->FindClass(J(e), cls);
    if (c) (*J(e))->ThrowNew(J(e), c, msg);
}

static uint8_t *j_direct_address(rsj_env *e, rsj_obj b) {
    return (uint8_t *)(*J(e))->GetDirectBufferAddress(J(e), (jobject)b);
}
static int64_t j_direct_capacity(rsj_env *e, rsj_obj b) {
    return (int64_t)(*J(e))->GetDirectBufferCapacity(J(e), (jobject)b);
}
static rsj_obj j_new_direct(rsj_env *e, void *p, int64_t cap) {
    return (*J(e))->NewDirectByteBuffer(J(e), p, (jlong)cap);
}

static rsj_env *wrap(jenv *je, JNIEnv *env) {
    rsj_env base = {NULL,           j_array_length,    j_object_element,   j_delete_local,
                    j_ensure_local_capacity, j_critical_get, j_critical_release, j_byte_region_get,
                    j_byte_region_set, j_bool_region_get, j_exception_pending, j_throw_new,
                    j_direct_address, j_direct_capacity, j_new_direct};
    je->base = base;
    je->env = env;
    return &je->base;
}

#define CODEC(h) ((const rs_codec *)(uintptr_t)(h))

/* ---- NativeReedSolomon: drop-in for ReedSolomon.java ---- */

JNIEXPORT jlong JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeCreate(JNIEnv *env, jclass cls, jint k,
                                                                                jint m) {
    rs_codec *c = NULL;
    int rc = rs_codec_create(k, m, &c);
    if (rc) {
        jclass e = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
        if (e) (*env)->ThrowNew(env, e, rs_last_error_message());
        return 0;
    }
    return (jlong)(uintptr_t)c;
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeDestroy(JNIEnv *env, jclass cls, jlong h) {
    rs_codec_destroy((rs_codec *)(uintptr_t)h);
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeEncodeParity(JNIEnv *env, jclass cls,
                                                                                     jlong h, jobjectArray shards,
                                                                                     jint offset, jint count) {
    jenv je;
    rsj_encode_parity(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), shards, offset, count);
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeDecodeMissing(JNIEnv *env, jclass cls,
                                                                                      jlong h, jobjectArray shards,
                                                                                      jbooleanArray present,
                                                                                      jint offset, jint count) {
    jenv je;
    rsj_decode_missing(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), shards, present, offset, count);
}

JNIEXPORT jboolean JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeIsParityCorrect(
    JNIEnv *env, jclass cls, jlong h, jobjectArray shards, jint first, jint count, jbyteArray temp) {
    jenv je;
    return rsj_is_parity_correct(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), shards, first, count, temp)
               ? JNI_TRUE
               : JNI_FALSE;
}

/* ReedSolomonEncoder.encode() / new ReedSolomonDecoder(shards, shardPresent,
 * byteCntInShard, fileSize) (ReedSolomonEncoder.java:56-85,
 * ReedSolomonDecoder.java:33-39): the split / merge runs in librsamd, so only
 * coded bytes cross the link (rs_file_encode / rs_file_decode). */
JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeEncodeFile(JNIEnv *env, jclass cls, jlong h,
                                                                                   jbyteArray file, jint block,
                                                                                   jobjectArray shards) {
    jenv je;
    rsj_file_encode(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), file, block, shards);
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeDecodeFile(
    JNIEnv *env, jclass cls, jlong h, jobjectArray shards, jbooleanArray present, jint byteCntInShard, jint block,
    jbyteArray fileOut, jint fileSize) {
    jenv je;
    rsj_file_decode(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), shards, present, byteCntInShard, block, fileOut,
                    fileSize);
}

/* Direct ByteBuffers: pinned ones from allocatePinned (rs_host_alloc) are
 * coded in place across the link; any direct buffer is accepted. */
JNIEXPORT jobject JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeAllocatePinned(JNIEnv *env, jclass cls,
                                                                                        jint capacity) {
    jenv je;
    return (jobject)rsj_alloc_pinned(wrap(&je, env), rsj_librsamd_backend(), capacity);
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeFreePinned(JNIEnv *env, jclass cls,
                                                                                 jobject buf) {
    jenv je;
    rsj_free_pinned(wrap(&je, env), rsj_librsamd_backend(), buf);
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeEncodeParityDirect(
    JNIEnv *env, jclass cls, jlong h, jobjectArray shards, jint offset, jint count) {
    jenv je;
    rsj_encode_parity_direct(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), shards, offset, count);
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeDecodeMissingDirect(
    JNIEnv *env, jclass cls, jlong h, jobjectArray shards, jbooleanArray present, jint offset, jint count) {
    jenv je;
    rsj_decode_missing_direct(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), shards, present, offset, count);
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeEncodeFileDirect(
    JNIEnv *env, jclass cls, jlong h, jobject file, jint fileLength, jint block, jobjectArray shards) {
    jenv je;
    rsj_file_encode_direct(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), file, fileLength, block, shards);
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeDecodeFileDirect(
    JNIEnv *env, jclass cls, jlong h, jobjectArray shards, jbooleanArray present, jint byteCntInShard, jint block,
    jobject fileOut, jint fileSize) {
    jenv je;
    rsj_file_decode_direct(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), shards, present, byteCntInShard, block,
                           fileOut, fileSize);
}

/* Frees this thread's device contexts (streams, staging buffers); for worker
 * threads a pool is about to retire. */
JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeThreadRelease(JNIEnv *env, jclass cls) {
    rs_thread_release();
}

/* ---- GpuCodingLoop: drop-in CodingLoop plugin (CodingLoop.java:79-117) ---- */

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_GpuCodingLoop_nativeCodeSomeShards(
    JNIEnv *env, jclass cls, jobjectArray rows, jobjectArray inputs, jint nin, jobjectArray outputs, jint nout,
    jint offset, jint count) {
    jenv je;
    rsj_code_some_shards(wrap(&je, env), rsj_librsamd_backend(), rows, inputs, nin, outputs, nout, offset, count);
}

JNIEXPORT jboolean JNICALL Java_edu_cmu_reedsolomon_GpuCodingLoop_nativeCheckSomeShards(
    JNIEnv *env, jclass cls, jobjectArray rows, jobjectArray inputs, jint nin, jobjectArray toCheck, jint ncheck,
    jint offset, jint count) {
    jenv je;
    return rsj_check_some_shards(wrap(&je, env), rsj_librsamd_backend(), rows, inputs, nin, toCheck, ncheck, offset,
                                 count)
               ? JNI_TRUE
               : JNI_FALSE;
}

/* ---- Device-resident recovery (no Java counterpart): chunk groups kept in HBM
 * by a GPU-side service, one presence bitmask per group (rs_amd.h). ---- */
JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeDecodeMaskedBitsDevice(
        JNIEnv *env, jclass cls, jlong h, jlong devBase, jlong devBits, jlong nStripes, jlong shardLen,
        jlong shardStride, jlong stripeStride, jlong devBad, jlong stream) {
    if (nStripes < 0 || shardLen < 0 || shardStride < 0 || stripeStride < 0) {
        jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
        if (c) (*env)->ThrowNew(env, c, "negative size");
        return;
    }
    int rc = rs_decode_batch_masked_bits_dev(CODEC(h), (uint8_t *)(uintptr_t)devBase,
                                             (const uint32_t *)(uintptr_t)devBits, (size_t)nStripes,
                                             (size_t)shardLen, (size_t)shardStride, (size_t)stripeStride,
                                             (int32_t *)(uintptr_t)devBad, (void *)(uintptr_t)stream);
    if (rc) {
        jclass c = (*env)->FindClass(env, (rc == RS_E_HIP || rc == RS_E_NO_DEVICE) ? "java/lang/IllegalStateException"
                                                                                : "java/lang/IllegalArgumentException");
        if (c) (*env)->ThrowNew(env, c, rs_last_error_message());
    }
}

/* The master's recovery loop over device-resident chunk groups in its own
 * layout, [server][group * chunkLen] (rs_decode_groups_shard_major_dev). */
JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeRecoverGroupsShardMajorDevice(
        JNIEnv *env, jclass cls, jlong h, jlong devBase, jlong serverStride, jint chunkLen, jlong nGroups,
        jbyteArray present, jlong stream) {
    jenv je;
    rsj_recover_groups_shard_major(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), devBase, serverStride, chunkLen,
                                   nGroups, present, stream);
}

/* The master's recovery loop on its host arrays (rs_decode_groups_shard_major):
 * byte[][] (movable, pinned around the library's copy batches) or direct
 * ByteBuffer[] servers. */
JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeRecoverGroupsShardMajor(
        JNIEnv *env, jclass cls, jlong h, jobjectArray servers, jint chunkLen, jint nGroups, jbyteArray present) {
    jenv je;
    rsj_recover_groups_shard_major_host(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), servers, chunkLen, nGroups,
                                        present);
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeRecoverGroupsShardMajorDirect(
        JNIEnv *env, jclass cls, jlong h, jobjectArray servers, jint chunkLen, jint nGroups, jbyteArray present) {
    jenv je;
    rsj_recover_groups_shard_major_direct(wrap(&je, env), rsj_librsamd_backend(), CODEC(h), servers, chunkLen,
                                          nGroups, present);
}
