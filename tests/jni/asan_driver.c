/* asan_driver.c -- the JNI shim's host-side paths under AddressSanitizer and
 * UndefinedBehaviorSanitizer (tests/test_jni.py::test_shim_under_asan).
 *
 * Built as one executable with tests/jni/fake_jvm.c and the shim
 * (ipls-java-api_amd/jni/ipls_jni.c), both instrumented, and linked to the
 * uninstrumented libipls_agg.so.  It drives the natives whose work before
 * (or instead of) the library call is the shim's own: Java array pinning and
 * release, length and direct-buffer checks, local-reference reservation for
 * text/file arrays, the error -> exception mapping (null handle, no GPU).
 * Exit status 0 = every expectation held; the sanitizers abort on a memory or
 * UB error.  No device compute (a GPU-less open fails as the test expects;
 * with a GPU present the handle is opened and closed again).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

/* fake JVM (tests/jni/fake_jvm.c) */
JNIEnv *fj_env(void);
jobject fj_new_bytes(const void *src, jsize n);
jobject fj_new_ints(const void *src, jsize n);
jobject fj_new_longs(const void *src, jsize n);
jobject fj_new_doubles(const void *src, jsize n);
jobject fj_new_objects(const jobject *src, jsize n);
jobject fj_new_direct(void *addr, jlong cap);
void *fj_data(jobject o);
jsize fj_len(jobject o);
void fj_free(jobject o);
const char *fj_exception(void);
void fj_clear(void);
int fj_violations(void);
const char *fj_last_violation(void);
void fj_reset_violations(void);

/* the natives exercised (signatures as in ipls_jni.c) */
jlong Java_NativeAggregator_open(JNIEnv *, jclass, jlong, jint, jint, jint, jint, jint);
void Java_NativeAggregator_close(JNIEnv *, jclass, jlong);
jintArray Java_NativeAggregator_shardPlan(JNIEnv *, jclass, jint, jint);
void Java_NativeAggregator_loadModel(JNIEnv *, jclass, jlong, jdoubleArray);
void Java_NativeAggregator_updateGradient(JNIEnv *, jclass, jlong, jdoubleArray, jintArray);
void Java_NativeAggregator_updateGradientDirect(JNIEnv *, jclass, jlong, jobject, jint, jlong, jintArray);
void Java_NativeAggregator_accumulate(JNIEnv *, jclass, jlong, jint, jint, jdoubleArray);
void Java_NativeAggregator_accumulateDirect(JNIEnv *, jclass, jlong, jint, jint, jobject, jint, jlong, jint);
void Java_NativeAggregator_updateIndirect(JNIEnv *, jclass, jlong, jint, jint, jobject, jint, jlong);
jint Java_NativeAggregator_ingestTexts(JNIEnv *, jclass, jlong, jint, jobjectArray, jint, jintArray, jintArray);
void Java_NativeAggregator_finalizePartition(JNIEnv *, jclass, jlong, jint, jbyteArray);
void Java_NativeAggregator_getPartitions(JNIEnv *, jclass, jlong, jdoubleArray);
void Java_NativeAggregator_aggregateRound(JNIEnv *, jclass, jlong, jint, jint, jdoubleArray);
void Java_NativeAggregator_promoteFuture(JNIEnv *, jclass, jlong, jintArray);
jint Java_NativeAggregator_collectReplicas(JNIEnv *, jclass, jlong, jintArray);
jbyteArray Java_NativeAggregator_mergeFiles(JNIEnv *, jclass, jlong, jobjectArray, jboolean);
void Java_NativeAggregator_getPartitionsWire(JNIEnv *, jclass, jlong, jobject, jint, jlong);
jbyteArray Java_NativeAggregator_publishPartial(JNIEnv *, jclass, jlong, jint, jint, jint, jint, jshort, jbyteArray);

static int fails = 0;

/* the pending exception class is the expected one (want == NULL: none) */
static int exc_matches(const char *got, const char *want) {
    if (!want) return got == NULL;
    return got != NULL && strcmp(got, want) == 0;
}

/* one native frame: reset the fake JVM's per-call state, run, then check the
 * JNI rules and the pending exception class (NULL = none expected) */
#define CALL(expect_cls, stmt)                                                                  \
    do {                                                                                        \
        fj_clear();                                                                             \
        fj_reset_violations();                                                                  \
        stmt;                                                                                   \
        const char *got_ = fj_exception();                                                      \
        if (fj_violations()) {                                                                  \
            fprintf(stderr, "line %d: JNI rule broken: %s\n", __LINE__, fj_last_violation());  \
            ++fails;                                                                            \
        }                                                                                       \
        if (!exc_matches(got_, (expect_cls))) {                                                 \
            fprintf(stderr, "line %d: exception %s, expected %s\n", __LINE__, got_ ? got_ : "none", \
                    (expect_cls) ? (expect_cls) : "none");                                      \
            ++fails;                                                                            \
        }                                                                                       \
    } while (0)

static const char *IAE = "java/lang/IllegalArgumentException";

int main(void) {
    JNIEnv *env = fj_env();

    /* shardPlan: a fresh int[] filled by SetIntArrayRegion */
    jintArray plan = NULL;
    CALL(NULL, plan = Java_NativeAggregator_shardPlan(env, NULL, 10, 4));
    static const int want[10] = {0, 0, 0, 1, 1, 1, 2, 2, 2, 3};
    if (!plan || fj_len(plan) != 10 || memcmp(fj_data(plan), want, sizeof want) != 0) {
        fprintf(stderr, "shardPlan(10, 4) wrong\n");
        ++fails;
    }
    fj_free(plan);
    CALL(IAE, Java_NativeAggregator_shardPlan(env, NULL, 10, 0));
    CALL(IAE, Java_NativeAggregator_shardPlan(env, NULL, 0, 4));

    /* Java arrays pinned, the library rejects the null handle, arrays released */
    double g[7] = {1, 2, 3, 4, 5, 6, 1};
    int owned[3] = {0, 1, 2};
    jobject dg = fj_new_doubles(g, 7), io = fj_new_ints(owned, 3);
    jobject b64 = fj_new_bytes(NULL, 64), one_int = fj_new_ints(NULL, 1), ints3 = fj_new_ints(NULL, 3);
    CALL(IAE, Java_NativeAggregator_loadModel(env, NULL, 0, dg));
    CALL(IAE, Java_NativeAggregator_updateGradient(env, NULL, 0, dg, io));
    CALL(IAE, Java_NativeAggregator_accumulate(env, NULL, 0, 0, 0, dg));
    CALL(IAE, Java_NativeAggregator_finalizePartition(env, NULL, 0, 0, b64));
    CALL(IAE, Java_NativeAggregator_getPartitions(env, NULL, 0, dg));
    CALL(IAE, Java_NativeAggregator_aggregateRound(env, NULL, 0, 0, 1, dg));
    CALL(IAE, Java_NativeAggregator_promoteFuture(env, NULL, 0, io));
    CALL(IAE, Java_NativeAggregator_collectReplicas(env, NULL, 0, ints3));
    CALL(IAE, Java_NativeAggregator_publishPartial(env, NULL, 0, 0, 0, 1, 2, 3, b64));

    /* direct buffers: heap buffer (no address), windows outside the capacity */
    unsigned char mem[64] = {0};
    jobject heap = fj_new_direct(NULL, -1), dir = fj_new_direct(mem, 64);
    CALL(IAE, Java_NativeAggregator_accumulateDirect(env, NULL, 0, 0, 0, heap, 0, 4, 1));
    CALL(IAE, Java_NativeAggregator_accumulateDirect(env, NULL, 0, 0, 0, dir, 40, 4, 1));   /* 40 + 32 > 64 */
    CALL(IAE, Java_NativeAggregator_accumulateDirect(env, NULL, 0, 0, 0, dir, -8, 1, 1));
    CALL(IAE, Java_NativeAggregator_accumulateDirect(env, NULL, 0, 0, 0, dir, 0, -1, 1));
    CALL(IAE, Java_NativeAggregator_updateIndirect(env, NULL, 0, 0, 0, dir, 8, 57));
    CALL(IAE, Java_NativeAggregator_updateGradientDirect(env, NULL, 0, heap, 0, 1, io));
    CALL(IAE, Java_NativeAggregator_updateGradientDirect(env, NULL, 0, dir, 8, 8, io));    /* 8 + 64 > 64 */
    CALL(IAE, Java_NativeAggregator_updateGradientDirect(env, NULL, 0, dir, 0, 8, io));    /* in range: null handle */
    CALL(IAE, Java_NativeAggregator_getPartitionsWire(env, NULL, 0, heap, 0, 8));
    CALL(IAE, Java_NativeAggregator_getPartitionsWire(env, NULL, 0, dir, 60, 8));
    CALL(IAE, Java_NativeAggregator_accumulateDirect(env, NULL, 0, 0, 0, dir, 0, 8, 1));     /* in range: null handle */

    /* many texts / files: one local reference per element, reserved first */
    jobject texts[40], files[24];
    for (int i = 0; i < 40; ++i) texts[i] = fj_new_bytes("AAAA", 4);
    for (int i = 0; i < 24; ++i) files[i] = fj_new_bytes(NULL, 16);
    jobject tarr = fj_new_objects(texts, 40), farr = fj_new_objects(files, 24);
    jobject parts_short = fj_new_ints(NULL, 3), status = fj_new_ints(NULL, 40);
    CALL(IAE, Java_NativeAggregator_ingestTexts(env, NULL, 0, 0, tarr, 2, NULL, NULL));
    CALL(IAE, Java_NativeAggregator_ingestTexts(env, NULL, 0, 0, tarr, 2, parts_short, status));  /* parts too short */
    CALL(IAE, Java_NativeAggregator_mergeFiles(env, NULL, 0, farr, 0));

    /* open: no GPU here -> RuntimeException; with one, open and close */
    jlong h = 0;
    fj_clear();
    fj_reset_violations();
    h = Java_NativeAggregator_open(env, NULL, 443610, 3, 3, 0, 0, 0);
    if (h) {
        CALL(NULL, Java_NativeAggregator_close(env, NULL, h));
    } else if (!fj_exception() || strcmp(fj_exception(), "java/lang/RuntimeException") != 0) {
        fprintf(stderr, "open without a GPU: exception %s\n", fj_exception() ? fj_exception() : "none");
        ++fails;
    }

    for (int i = 0; i < 40; ++i) fj_free(texts[i]);
    for (int i = 0; i < 24; ++i) fj_free(files[i]);
    fj_free(tarr);
    fj_free(farr);
    fj_free(parts_short);
    fj_free(status);
    fj_free(heap);
    fj_free(dir);
    fj_free(dg);
    fj_free(io);
    fj_free(b64);
    fj_free(one_int);
    fj_free(ints3);
    printf("asan driver: %d failure(s)\n", fails);
    return fails ? 1 : 0;
}
