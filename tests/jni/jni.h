/*
 * tests/jni/jni.h -- TEST STAND-IN, not the JDK header.
 *
 * This image has no JDK, so ipls-java-api_amd/jni/ipls_jni.c cannot be
 * compiled against the real <jni.h>.  This header declares exactly the JNI
 * types and the JNIEnv entries the shim uses, with the JDK's names and C
 * signatures (JNI specification, "JNI Functions"), so that
 *   - the shim is compiled with -Wall -Wextra -Werror in the CPU suite
 *     (tests/test_jni.py), catching type and signature errors, and
 *   - tests/jni/fake_jvm.c can drive every native through a function table
 *     of its own against the real libipls_agg.so.
 * The table's LAYOUT is not the JDK's (a real JVM's JNIEnv has ~230 slots in
 * a fixed order): a production build uses the JDK's jni.h, never this file.
 */
#ifndef IPLS_TEST_JNI_H
#define IPLS_TEST_JNI_H

#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbooleanArray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jdoubleArray;
typedef jarray jobjectArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
    jclass (JNICALL *FindClass)(JNIEnv *env, const char *name);
    jint (JNICALL *ThrowNew)(JNIEnv *env, jclass clazz, const char *msg);
    jboolean (JNICALL *ExceptionCheck)(JNIEnv *env);
    void (JNICALL *DeleteLocalRef)(JNIEnv *env, jobject obj);
    jsize (JNICALL *GetArrayLength)(JNIEnv *env, jarray array);
    jobject (JNICALL *GetObjectArrayElement)(JNIEnv *env, jobjectArray array, jsize index);
    jbyteArray (JNICALL *NewByteArray)(JNIEnv *env, jsize len);
    jintArray (JNICALL *NewIntArray)(JNIEnv *env, jsize len);
    jbyte *(JNICALL *GetByteArrayElements)(JNIEnv *env, jbyteArray array, jboolean *isCopy);
    jint *(JNICALL *GetIntArrayElements)(JNIEnv *env, jintArray array, jboolean *isCopy);
    jlong *(JNICALL *GetLongArrayElements)(JNIEnv *env, jlongArray array, jboolean *isCopy);
    void (JNICALL *ReleaseByteArrayElements)(JNIEnv *env, jbyteArray array, jbyte *elems, jint mode);
    void (JNICALL *ReleaseIntArrayElements)(JNIEnv *env, jintArray array, jint *elems, jint mode);
    void (JNICALL *ReleaseLongArrayElements)(JNIEnv *env, jlongArray array, jlong *elems, jint mode);
    void (JNICALL *SetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, const jbyte *buf);
    void (JNICALL *SetIntArrayRegion)(JNIEnv *env, jintArray array, jsize start, jsize len, const jint *buf);
    void (JNICALL *SetDoubleArrayRegion)(JNIEnv *env, jdoubleArray array, jsize start, jsize len,
                                         const jdouble *buf);
    void (JNICALL *GetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, jbyte *buf);
    void (JNICALL *GetDoubleArrayRegion)(JNIEnv *env, jdoubleArray array, jsize start, jsize len, jdouble *buf);
    void *(JNICALL *GetPrimitiveArrayCritical)(JNIEnv *env, jarray array, jboolean *isCopy);
    void (JNICALL *ReleasePrimitiveArrayCritical)(JNIEnv *env, jarray array, void *carray, jint mode);
    jobject (JNICALL *NewDirectByteBuffer)(JNIEnv *env, void *address, jlong capacity);
    void *(JNICALL *GetDirectBufferAddress)(JNIEnv *env, jobject buf);
    jlong (JNICALL *GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
    jint (JNICALL *EnsureLocalCapacity)(JNIEnv *env, jint capacity);
};

#endif /* IPLS_TEST_JNI_H */
