/*
 * jni.h -- a declarations-only subset of the Java Native Interface header,
 * written for tests/test_jni_adapter.py from the JNI specification (Java SE
 * "JNI Types and Data Structures" and "JNI Functions"), NOT copied from a JDK.
 *
 * It declares the primitive and reference types, the constants and the
 * JNIEnv function-table entries that jni/rs_jni.c uses, with the signatures
 * the specification gives them, so a compiler checks the adapter's names,
 * argument types and return types without a JDK.  Unused table entries are
 * omitted, so the table's layout is NOT the real one: nothing built against
 * this header may run.  Where a JDK exists, build against its own jni.h
 * (INTEGRATION.md).
 */
#ifndef RSAMD_TEST_JNI_SUBSET_H
#define RSAMD_TEST_JNI_SUBSET_H

#include <stdarg.h>
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

/* Primitive types (spec: "Primitive Types") */
typedef uint8_t jboolean;
typedef int8_t jbyte;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef int32_t jint;
typedef int64_t jlong;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

#define JNI_FALSE 0
#define JNI_TRUE 1

/* Reference types (spec: "Reference Types"), as the C binding declares them */
struct _jobject;
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jbooleanArray;
typedef jarray jbyteArray;

/* Release modes of Release<PrimitiveType>ArrayElements / ReleasePrimitiveArrayCritical */
#define JNI_COMMIT 1
#define JNI_ABORT 2

#define JNI_OK 0

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

/* The function-table entries rs_jni.c calls (spec: "JNI Functions"). */
struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv *env, const char *name);
    jint (*ThrowNew)(JNIEnv *env, jclass clazz, const char *message);
    jboolean (*ExceptionCheck)(JNIEnv *env);
    void (*DeleteLocalRef)(JNIEnv *env, jobject localRef);
    jint (*EnsureLocalCapacity)(JNIEnv *env, jint capacity);
    jsize (*GetArrayLength)(JNIEnv *env, jarray array);
    jobject (*GetObjectArrayElement)(JNIEnv *env, jobjectArray array, jsize index);
    void (*GetBooleanArrayRegion)(JNIEnv *env, jbooleanArray array, jsize start, jsize len, jboolean *buf);
    void (*GetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, jbyte *buf);
    void (*SetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, const jbyte *buf);
    void *(*GetPrimitiveArrayCritical)(JNIEnv *env, jarray array, jboolean *isCopy);
    void (*ReleasePrimitiveArrayCritical)(JNIEnv *env, jarray array, void *carray, jint mode);
    jobject (*NewDirectByteBuffer)(JNIEnv *env, void *address, jlong capacity);
    void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);
    jlong (*GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
};

#endif /* RSAMD_TEST_JNI_SUBSET_H */
