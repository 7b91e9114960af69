/*
 * ipls_jni.c -- JNI half of NativeAggregator (ipls-java-api_amd/java/).
 * A 1:1 map onto include/ipls_agg.h: no arithmetic here.  Negative return
 * codes become the Java exception the reference would have thrown.
 *
 * Built only where a JDK exists (make -C ipls-java-api_amd jni); this image
 * has none, so it is compiled on the Java side's build host.
 */
#include <jni.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ipls_agg.h"

static void throw_for(JNIEnv *env, int rc, ipls_agg *h) {
    const char *cls = "java/lang/RuntimeException";
    switch (rc) {
        case IPLS_E_RANGE: cls = "java/lang/ArrayIndexOutOfBoundsException"; break;
        case IPLS_E_NEGSIZE: cls = "java/lang/NegativeArraySizeException"; break;
        case IPLS_E_FORMAT: cls = "java/nio/BufferUnderflowException"; break;
        case IPLS_E_INVAL: cls = "java/lang/IllegalArgumentException"; break;
        case IPLS_E_NOMEM: cls = "java/lang/OutOfMemoryError"; break;
        default: break;
    }
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, ipls_agg_last_error(h));
}

#define H(x) ((ipls_agg *)(intptr_t)(x))
#define CHECK(rc, h) do { int rc_ = (rc); if (rc_ < 0) { throw_for(env, rc_, (h)); } } while (0)

JNIEXPORT jlong JNICALL Java_NativeAggregator_open(JNIEnv *env, jclass c, jlong m, jint pa, jint n,
                                                     jint aggr, jint secure, jint dev) {
    (void)c;
    ipls_agg_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.model_size = m; cfg.n_partitions = pa; cfg.max_peers = n;
    cfg.partial_aggregation = aggr; cfg.secure = secure; cfg.device = dev;
    ipls_agg *h = NULL;
    int rc = ipls_agg_open(&cfg, &h);
    if (rc < 0) { throw_for(env, rc, NULL); return 0; }
    return (jlong)(intptr_t)h;
}

JNIEXPORT void JNICALL Java_NativeAggregator_close(JNIEnv *env, jclass c, jlong h) {
    (void)env; (void)c;
    ipls_agg_close(H(h));
}

JNIEXPORT jlong JNICALL Java_NativeAggregator_partitionLen(JNIEnv *env, jclass c, jlong h, jint p) {
    (void)c;
    int64_t L = 0;
    CHECK(ipls_agg_partition_len(H(h), p, &L), H(h));
    return (jlong)L;
}

JNIEXPORT void JNICALL Java_NativeAggregator_loadModel(JNIEnv *env, jclass c, jlong h, jdoubleArray a) {
    (void)c;
    jsize n = (*env)->GetArrayLength(env, a);
    void *p = (*env)->GetPrimitiveArrayCritical(env, a, NULL);
    int rc = ipls_agg_load_model(H(h), p, n, IPLS_HOST_F64);
    (*env)->ReleasePrimitiveArrayCritical(env, a, p, JNI_ABORT);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_split(JNIEnv *env, jclass c, jlong h, jdoubleArray flat, jint part,
                                                     jdoubleArray out) {
    (void)c;
    jsize n = (*env)->GetArrayLength(env, flat);
    void *src = (*env)->GetPrimitiveArrayCritical(env, flat, NULL);
    void *dst = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
    int rc = ipls_agg_split(H(h), src, n, IPLS_HOST_F64, part, dst, IPLS_HOST_F64);
    (*env)->ReleasePrimitiveArrayCritical(env, out, dst, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, flat, src, JNI_ABORT);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_updateGradient(JNIEnv *env, jclass c, jlong h, jdoubleArray flat,
                                                              jintArray owned) {
    (void)c;
    jsize n = (*env)->GetArrayLength(env, flat), no = (*env)->GetArrayLength(env, owned);
    void *src = (*env)->GetPrimitiveArrayCritical(env, flat, NULL);
    void *own = (*env)->GetPrimitiveArrayCritical(env, owned, NULL);
    int rc = ipls_agg_update_gradient(H(h), src, n, IPLS_HOST_F64, (const int32_t *)own, no);
    (*env)->ReleasePrimitiveArrayCritical(env, owned, own, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, flat, src, JNI_ABORT);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_accumulate(JNIEnv *env, jclass c, jlong h, jint p, jint tgt,
                                                          jdoubleArray g) {
    (void)c;
    jsize n = (*env)->GetArrayLength(env, g);
    void *src = (*env)->GetPrimitiveArrayCritical(env, g, NULL);
    int rc = ipls_agg_accumulate(H(h), p, tgt, src, n, IPLS_HOST_F64);
    (*env)->ReleasePrimitiveArrayCritical(env, g, src, JNI_ABORT);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_accumulateDirect(JNIEnv *env, jclass c, jlong h, jint p, jint tgt,
                                                                jobject buf, jlong n, jint kind) {
    (void)c;
    void *src = (*env)->GetDirectBufferAddress(env, buf);
    CHECK(ipls_agg_accumulate(H(h), p, tgt, src, n, kind), H(h));
}

JNIEXPORT jlong JNICALL Java_NativeAggregator_accumulateAsyncDirect(JNIEnv *env, jclass c, jlong h, jint p,
                                                                      jint tgt, jobject buf, jlong n, jint kind) {
    (void)c;
    void *src = (*env)->GetDirectBufferAddress(env, buf);
    uint64_t t = 0;
    CHECK(ipls_agg_accumulate_async(H(h), p, tgt, src, n, kind, &t), H(h));
    return (jlong)t;
}

JNIEXPORT void JNICALL Java_NativeAggregator_waitTicket(JNIEnv *env, jclass c, jlong h, jlong ticket) {
    (void)c;
    CHECK(ipls_agg_wait(H(h), (uint64_t)ticket), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_flushQueued(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    CHECK(ipls_agg_flush(H(h)), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_updateIndirect(JNIEnv *env, jclass c, jlong h, jint p, jint tgt,
                                                              jobject buf, jlong nBytes) {
    (void)c;
    void *src = (*env)->GetDirectBufferAddress(env, buf);
    CHECK(ipls_agg_update_indirect(H(h), p, tgt, src, nBytes), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_accumulateFrame(JNIEnv *env, jclass c, jlong h, jint p, jint tgt,
                                                               jbyteArray frame) {
    (void)c;
    jsize n = (*env)->GetArrayLength(env, frame);
    void *src = (*env)->GetPrimitiveArrayCritical(env, frame, NULL);
    int rc = ipls_agg_accumulate(H(h), p, tgt, src, n, IPLS_HOST_FRAME);
    (*env)->ReleasePrimitiveArrayCritical(env, frame, src, JNI_ABORT);
    CHECK(rc, H(h));
}

/* ThreadReceiver: a batch of pubsub texts.  The local refs are taken before
 * any critical region opens (no other JNI call is allowed inside one); the
 * texts stay pinned by the JVM for the call (the library copies them to the
 * GPU before returning). */
JNIEXPORT jint JNICALL Java_NativeAggregator_ingestTexts(JNIEnv *env, jclass c, jlong h, jint tgt,
                                                         jobjectArray msgs, jint layers, jintArray parts,
                                                         jintArray status) {
    (void)c;
    const jsize n = msgs ? (*env)->GetArrayLength(env, msgs) : 0;
    jbyteArray *arr = calloc((size_t)n + 1, sizeof *arr);
    const uint8_t **ptr = calloc((size_t)n + 1, sizeof *ptr);
    int64_t *len = calloc((size_t)n + 1, sizeof *len);
    int32_t *st = calloc((size_t)n + 1, sizeof *st);
    jint *pp = NULL;
    int rc = IPLS_E_NOMEM;
    if (!arr || !ptr || !len || !st) goto out;
    for (jsize i = 0; i < n; ++i) {
        arr[i] = (jbyteArray)(*env)->GetObjectArrayElement(env, msgs, i);
        len[i] = arr[i] ? (*env)->GetArrayLength(env, arr[i]) : 0;
    }
    if (parts) pp = (*env)->GetIntArrayElements(env, parts, NULL);
    for (jsize i = 0; i < n; ++i)
        ptr[i] = arr[i] ? (*env)->GetPrimitiveArrayCritical(env, arr[i], NULL) : NULL;
    rc = ipls_agg_ingest_pubsub(H(h), tgt, ptr, len, n, layers, (const int32_t *)pp, st);
    for (jsize i = n; i-- > 0;)
        if (ptr[i]) (*env)->ReleasePrimitiveArrayCritical(env, arr[i], (void *)ptr[i], JNI_ABORT);
    if (pp) (*env)->ReleaseIntArrayElements(env, parts, pp, JNI_ABORT);
    if (status && rc >= 0) (*env)->SetIntArrayRegion(env, status, 0, n, (const jint *)st);
    for (jsize i = 0; i < n; ++i)
        if (arr[i]) (*env)->DeleteLocalRef(env, arr[i]);
out:
    free(arr);
    free(ptr);
    free(len);
    free(st);
    CHECK(rc, H(h));
    return rc;
}

JNIEXPORT void JNICALL Java_NativeAggregator_finalizePartition(JNIEnv *env, jclass c, jlong h, jint p,
                                                                 jbyteArray sum) {
    (void)c;
    void *dst = (*env)->GetPrimitiveArrayCritical(env, sum, NULL);
    int rc = ipls_agg_finalize(H(h), p, dst, IPLS_HOST_BE, NULL);
    (*env)->ReleasePrimitiveArrayCritical(env, sum, dst, 0);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_finalizePartitionDirect(JNIEnv *env, jclass c, jlong h, jint p,
                                                                       jobject sum) {
    (void)c;
    CHECK(ipls_agg_finalize(H(h), p, (*env)->GetDirectBufferAddress(env, sum), IPLS_HOST_BE, NULL), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_setWeightsDirect(JNIEnv *env, jclass c, jlong h, jint p, jobject buf,
                                                                jlong n) {
    (void)c;
    CHECK(ipls_agg_set_weights(H(h), p, (*env)->GetDirectBufferAddress(env, buf), n, IPLS_HOST_BE), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_setWeightsFrame(JNIEnv *env, jclass c, jlong h, jint p,
                                                               jbyteArray frame) {
    (void)c;
    jsize n = (*env)->GetArrayLength(env, frame);
    void *src = (*env)->GetPrimitiveArrayCritical(env, frame, NULL);
    int rc = ipls_agg_set_weights(H(h), p, src, n, IPLS_HOST_FRAME);
    (*env)->ReleasePrimitiveArrayCritical(env, frame, src, JNI_ABORT);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_getPartitions(JNIEnv *env, jclass c, jlong h, jdoubleArray out) {
    (void)c;
    jsize n = (*env)->GetArrayLength(env, out);
    void *dst = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
    int rc = ipls_agg_get_partitions(H(h), dst, n, IPLS_HOST_F64);
    (*env)->ReleasePrimitiveArrayCritical(env, out, dst, 0);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_aggregateRound(JNIEnv *env, jclass c, jlong h, jint p0, jint np,
                                                              jdoubleArray out) {
    (void)c;
    void *dst = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
    int rc = ipls_agg_aggregate_round(H(h), p0, np, NULL, 0, IPLS_DEV_F64, dst, IPLS_HOST_F64);
    (*env)->ReleasePrimitiveArrayCritical(env, out, dst, 0);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_promoteFuture(JNIEnv *env, jclass c, jlong h, jintArray parts) {
    (void)c;
    jsize n = (*env)->GetArrayLength(env, parts);
    jint *ps = (*env)->GetIntArrayElements(env, parts, NULL);
    int rc = ipls_agg_promote_future(H(h), (const int32_t *)ps, n);
    (*env)->ReleaseIntArrayElements(env, parts, ps, JNI_ABORT);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_otherReplicaDirect(JNIEnv *env, jclass c, jlong h, jint p, jint a,
                                                                  jobject buf, jlong n) {
    (void)c;
    CHECK(ipls_agg_other_replica(H(h), p, a, (*env)->GetDirectBufferAddress(env, buf), n, IPLS_HOST_BE), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_collectReplicas(JNIEnv *env, jclass c, jlong h, jintArray out) {
    (void)c;
    jint *ps = (*env)->GetIntArrayElements(env, out, NULL);
    int rc = ipls_agg_collect_replicas(H(h), (int32_t *)ps);
    (*env)->ReleaseIntArrayElements(env, out, ps, 0);
    CHECK(rc, H(h));
}

JNIEXPORT jlong JNICALL Java_NativeAggregator_commitPartialLen(JNIEnv *env, jclass c, jlong h, jint p, jint w) {
    (void)c;
    int64_t n = ipls_agg_commit_partial(H(h), p, w, NULL, 0);
    if (n < 0) { throw_for(env, (int)n, H(h)); return 0; }
    return (jlong)n;
}

JNIEXPORT void JNICALL Java_NativeAggregator_commitPartial(JNIEnv *env, jclass c, jlong h, jint p, jint w,
                                                             jbyteArray out) {
    (void)c;
    jsize n = (*env)->GetArrayLength(env, out);
    void *dst = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
    int64_t rc = ipls_agg_commit_partial(H(h), p, w, (uint8_t *)dst, n);
    (*env)->ReleasePrimitiveArrayCritical(env, out, dst, 0);
    if (rc < 0) throw_for(env, (int)rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_accumulatePair(JNIEnv *env, jclass c, jlong h, jint p, jint tgt,
                                                              jbyteArray file) {
    (void)c;
    jsize n = (*env)->GetArrayLength(env, file);
    void *src = (*env)->GetPrimitiveArrayCritical(env, file, NULL);
    int rc = ipls_agg_accumulate(H(h), p, tgt, src, n, IPLS_HOST_PAIR);
    (*env)->ReleasePrimitiveArrayCritical(env, file, src, JNI_ABORT);
    CHECK(rc, H(h));
}

JNIEXPORT jbyteArray JNICALL Java_NativeAggregator_mergeFiles(JNIEnv *env, jclass c, jlong h, jobjectArray files,
                                                                jboolean partial) {
    (void)c;
    jsize k = (*env)->GetArrayLength(env, files);
    if (k < 1) { throw_for(env, IPLS_E_INVAL, H(h)); return NULL; }
    jbyteArray *arr = (jbyteArray *)calloc((size_t)k, sizeof(jbyteArray));
    const uint8_t **ptrs = (const uint8_t **)calloc((size_t)k, sizeof(uint8_t *));
    int64_t *lens = (int64_t *)calloc((size_t)k, sizeof(int64_t));
    jbyteArray res = NULL;
    for (jsize i = 0; i < k; ++i) {   /* copies: several arrays cannot be held critical across a JNI call */
        arr[i] = (jbyteArray)(*env)->GetObjectArrayElement(env, files, i);
        lens[i] = (*env)->GetArrayLength(env, arr[i]);
        ptrs[i] = (const uint8_t *)(*env)->GetByteArrayElements(env, arr[i], NULL);
    }
    int64_t cap = 8 * (lens[0] / 8);
    if (partial) {
        int32_t w; int64_t off;
        int64_t n0 = ipls_pair_parse(ptrs[0], lens[0], &w, &off);
        cap = n0 < 0 ? 0 : 8 * n0;
    }
    uint8_t *out = (uint8_t *)malloc((size_t)(cap > 0 ? cap : 1));
    int64_t nb = ipls_agg_merge_files(H(h), ptrs, lens, k, partial ? IPLS_HOST_PAIR : IPLS_HOST_BE, out, cap);
    for (jsize i = 0; i < k; ++i) (*env)->ReleaseByteArrayElements(env, arr[i], (jbyte *)ptrs[i], JNI_ABORT);
    if (nb < 0) {
        throw_for(env, (int)nb, H(h));
    } else {
        res = (*env)->NewByteArray(env, (jsize)nb);
        if (res) (*env)->SetByteArrayRegion(env, res, 0, (jsize)nb, (const jbyte *)out);
    }
    free(out); free(lens); free(ptrs); free(arr);
    return res;
}

JNIEXPORT void JNICALL Java_NativeAggregator_getPartitionsWire(JNIEnv *env, jclass c, jlong h, jobject buf) {
    (void)c;
    jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
    CHECK(ipls_agg_get_partitions(H(h), (*env)->GetDirectBufferAddress(env, buf), cap / 8, IPLS_HOST_BE_CANON),
          H(h));
}

JNIEXPORT jobject JNICALL Java_NativeAggregator_hostAllocDirect(JNIEnv *env, jclass c, jint bytes) {
    (void)c;
    void *p = NULL;
    int rc = ipls_host_alloc((size_t)bytes, &p);
    if (rc < 0) { throw_for(env, rc, NULL); return NULL; }
    return (*env)->NewDirectByteBuffer(env, p, bytes);
}
