/*
 * rs_jni.c -- JNI binding of librsamd.so for the reference's Java codec API.
 *
 * Source-only in this repository: the build container has no JDK (no jni.h,
 * no javac).  Build where a JDK 17 exists:
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *      -I<repo>/include rs_jni.c -L<repo>/java-reed-solomon-distributed-file-system_amd/lib \
 *      -lrsamd -Wl,-rpath,'$ORIGIN' -o librsamd_jni.so
 *
 * Java side: jni/java/edu/cmu/reedsolomon/{NativeReedSolomon,GpuCodingLoop}.java.
 * Shards are pinned with GetPrimitiveArrayCritical (zero copy where the JVM
 * allows it) and released with mode 0 when written, JNI_ABORT when only read;
 * every rs_* error becomes java.lang.IllegalArgumentException with the text
 * the reference would have used (rs_last_error_message()), or
 * java.lang.IllegalStateException for a GPU failure.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rs_amd.h"

#define MAX_SHARDS 256

static void throw_rs(JNIEnv *env, int rc) {
    const char *cls = (rc == RS_E_HIP || rc == RS_E_NO_DEVICE) ? "java/lang/IllegalStateException"
                                                               : "java/lang/IllegalArgumentException";
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, rs_last_error_message());
}

/* Pinned view of a byte[][]. */
typedef struct {
    int n;
    jbyteArray arr[MAX_SHARDS];
    uint8_t *ptr[MAX_SHARDS];
    int64_t len[MAX_SHARDS];
} pinned;

/* Collect array refs and lengths first (no JNI calls are allowed while a
 * critical region is open), then pin.  limit >= 0 pins only the first `limit`
 * elements (CodingLoop arrays may carry unused extra buffers, CodingLoop.java:63-73). */
static int pin_n(JNIEnv *env, jobjectArray shards, int limit, pinned *p) {
    memset(p->ptr, 0, sizeof p->ptr);
    p->n = (*env)->GetArrayLength(env, shards);
    if (limit >= 0 && limit < p->n) p->n = limit;
    if (p->n > MAX_SHARDS) p->n = MAX_SHARDS + 1;  /* reported as a wrong shard count */
    int n = p->n > MAX_SHARDS ? MAX_SHARDS : p->n;
    for (int i = 0; i < n; i++) {
        p->arr[i] = (jbyteArray)(*env)->GetObjectArrayElement(env, shards, i);
        if (!p->arr[i]) {
            jclass c = (*env)->FindClass(env, "java/lang/NullPointerException");
            if (c) (*env)->ThrowNew(env, c, "shard is null");
            return -1;
        }
        p->len[i] = (*env)->GetArrayLength(env, p->arr[i]);
    }
    for (int i = 0; i < n; i++) p->ptr[i] = (uint8_t *)(*env)->GetPrimitiveArrayCritical(env, p->arr[i], NULL);
    return 0;
}

static int pin(JNIEnv *env, jobjectArray shards, pinned *p) { return pin_n(env, shards, -1, p); }

static void unpin(JNIEnv *env, pinned *p, jint mode) {
    int n = p->n > MAX_SHARDS ? MAX_SHARDS : p->n;
    for (int i = n - 1; i >= 0; i--)
        if (p->ptr[i]) (*env)->ReleasePrimitiveArrayCritical(env, p->arr[i], p->ptr[i], mode);
}

/* ---- NativeReedSolomon: drop-in for ReedSolomon.java ---- */

JNIEXPORT jlong JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeCreate(JNIEnv *env, jclass cls, jint k,
                                                                                jint m) {
    rs_codec *c = NULL;
    int rc = rs_codec_create(k, m, &c);
    if (rc) {
        throw_rs(env, rc);
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
    pinned p;
    if (pin(env, shards, &p)) return;
    int rc = rs_encode_parity((rs_codec *)(uintptr_t)h, p.ptr, p.n, p.len, offset, count);
    unpin(env, &p, 0);
    if (rc) throw_rs(env, rc);
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeDecodeMissing(JNIEnv *env, jclass cls,
                                                                                      jlong h, jobjectArray shards,
                                                                                      jbooleanArray present,
                                                                                      jint offset, jint count) {
    uint8_t pres[MAX_SHARDS];
    jsize np = (*env)->GetArrayLength(env, present);
    memset(pres, 0, sizeof pres);
    (*env)->GetBooleanArrayRegion(env, present, 0, np > MAX_SHARDS ? MAX_SHARDS : np, (jboolean *)pres);
    pinned p;
    if (pin(env, shards, &p)) return;
    int rc = rs_decode_missing((rs_codec *)(uintptr_t)h, p.ptr, p.n, p.len, pres, offset, count);
    unpin(env, &p, 0);
    if (rc) throw_rs(env, rc);
}

JNIEXPORT jboolean JNICALL Java_edu_cmu_reedsolomon_NativeReedSolomon_nativeIsParityCorrect(
    JNIEnv *env, jclass cls, jlong h, jobjectArray shards, jint first, jint count, jbyteArray temp) {
    int64_t temp_len = temp ? (*env)->GetArrayLength(env, temp) : 0;
    pinned p;
    if (pin(env, shards, &p)) return JNI_FALSE;
    int result = 0;
    /* the GPU path needs no scratch: only the tempBuffer length is checked */
    static const uint8_t dummy = 0;
    int rc = rs_is_parity_correct((rs_codec *)(uintptr_t)h, p.ptr, p.n, p.len, first, count,
                                  temp ? &dummy : NULL, temp_len, &result);
    unpin(env, &p, JNI_ABORT);
    if (rc) {
        throw_rs(env, rc);
        return JNI_FALSE;
    }
    return result ? JNI_TRUE : JNI_FALSE;
}

/* ---- GpuCodingLoop: drop-in CodingLoop plugin (CodingLoop.java:79-117) ---- */

static int rows_to_c(JNIEnv *env, jobjectArray rows, int nrows, int ncols, uint8_t *flat, const uint8_t **ptrs) {
    for (int r = 0; r < nrows; r++) {
        jbyteArray a = (jbyteArray)(*env)->GetObjectArrayElement(env, rows, r);
        if (!a) return -1;
        (*env)->GetByteArrayRegion(env, a, 0, ncols, (jbyte *)(flat + (size_t)r * ncols));
        ptrs[r] = flat + (size_t)r * ncols;
    }
    return 0;
}

JNIEXPORT void JNICALL Java_edu_cmu_reedsolomon_GpuCodingLoop_nativeCodeSomeShards(
    JNIEnv *env, jclass cls, jobjectArray rows, jobjectArray inputs, jint nin, jobjectArray outputs, jint nout,
    jint offset, jint count) {
    if (nout <= 0 || count <= 0) return;
    uint8_t *flat = (uint8_t *)malloc((size_t)nout * nin);
    const uint8_t *rp[MAX_SHARDS];
    if (!flat || nout > MAX_SHARDS || nin > MAX_SHARDS || rows_to_c(env, rows, nout, nin, flat, rp)) {
        free(flat);
        return;
    }
    pinned in, out;
    if (pin_n(env, inputs, nin, &in)) { free(flat); return; }
    if (pin_n(env, outputs, nout, &out)) { unpin(env, &in, JNI_ABORT); free(flat); return; }
    int rc = rs_code_some_shards(rp, (const uint8_t *const *)in.ptr, nin, out.ptr, nout, offset, count);
    unpin(env, &out, 0);
    unpin(env, &in, JNI_ABORT);
    free(flat);
    if (rc) throw_rs(env, rc);
}

JNIEXPORT jboolean JNICALL Java_edu_cmu_reedsolomon_GpuCodingLoop_nativeCheckSomeShards(
    JNIEnv *env, jclass cls, jobjectArray rows, jobjectArray inputs, jint nin, jobjectArray toCheck, jint ncheck,
    jint offset, jint count) {
    if (ncheck <= 0 || count <= 0) return JNI_TRUE;
    uint8_t *flat = (uint8_t *)malloc((size_t)ncheck * nin);
    const uint8_t *rp[MAX_SHARDS];
    if (!flat || ncheck > MAX_SHARDS || nin > MAX_SHARDS || rows_to_c(env, rows, ncheck, nin, flat, rp)) {
        free(flat);
        return JNI_FALSE;
    }
    pinned in, chk;
    if (pin_n(env, inputs, nin, &in)) { free(flat); return JNI_FALSE; }
    if (pin_n(env, toCheck, ncheck, &chk)) { unpin(env, &in, JNI_ABORT); free(flat); return JNI_FALSE; }
    int result = 0;
    int rc = rs_check_some_shards(rp, (const uint8_t *const *)in.ptr, nin, (const uint8_t *const *)chk.ptr, ncheck,
                                  offset, count, &result);
    unpin(env, &chk, JNI_ABORT);
    unpin(env, &in, JNI_ABORT);
    free(flat);
    if (rc) {
        throw_rs(env, rc);
        return JNI_FALSE;
    }
    return result ? JNI_TRUE : JNI_FALSE;
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
    int rc = rs_decode_batch_masked_bits_dev((const rs_codec *)(uintptr_t)h, (uint8_t *)(uintptr_t)devBase,
                                             (const uint32_t *)(uintptr_t)devBits, (size_t)nStripes,
                                             (size_t)shardLen, (size_t)shardStride, (size_t)stripeStride,
                                             (int32_t *)(uintptr_t)devBad, (void *)(uintptr_t)stream);
    if (rc) throw_rs(env, rc);
}
