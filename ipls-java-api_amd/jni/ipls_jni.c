/*
 * ipls_jni.c -- JNI half of NativeAggregator (ipls-java-api_amd/java/).
 * A 1:1 map onto include/ipls_agg.h: no arithmetic here.  Negative return
 * codes become the Java exception the reference would have thrown
 * (throw_for); every array or buffer the library writes is checked against
 * what it will write BEFORE the call, so a wrong size from the Java side is
 * an IllegalArgumentException and never a write past a Java array.
 *
 * Direct ByteBuffers: GetDirectBufferAddress ignores position() and returns
 * NULL for a heap buffer, so the Java wrappers pass position() and the byte
 * count, and the shim adds the position and checks both against capacity.
 *
 * Heap arrays are never held in a critical region across a library call.
 * GetPrimitiveArrayCritical would hand the library the Java heap itself, but
 * the region then spans the call -- host copies, a device fold, a wait on the
 * GPU -- and a JVM blocks its garbage collector for as long as a critical
 * region is open.  So every heap array (double[], byte[], byte[][]) is
 * copied out with Get<T>ArrayRegion into a per-thread staging buffer before
 * the call, and outputs are written there and copied back with
 * Set<T>ArrayRegion after it: one host memcpy, no GC stall.  The zero-copy
 * route is the direct-ByteBuffer natives (hostAlloc memory), which the hot
 * paths use.  Every library call goes through LIB(): a
 * test build (-DIPLS_JNI_CALL_HOOK=fj_library_call) reports each one to the
 * fake JVM, which fails the test if a critical region is open at that point.
 *
 * The one critical region the shim opens is critical_copy(): inside a chunk
 * callback of the three heap-array natives (accumulate(double[]),
 * finalizePartition(byte[]), getPartitions(double[])), around one memcpy of
 * one ring chunk (4 MiB) between the array and the library's pinned ring,
 * split over a few helper threads -- no JNI call and no library call inside,
 * ~0.1 ms.  That is the time HotSpot's own Get/Set<T>ArrayRegion of the same
 * chunk keeps the thread from a safepoint, and one CPU thread's memcpy is
 * what held these natives to 33 / 21 GB/s against PCIe's 56 (VERDICT r5
 * item 4).
 *
 * Built against the JDK's <jni.h> on the Java side's build host (make -C
 * ipls-java-api_amd jni).  This image has no JDK: tests/test_jni.py compiles
 * it with -Wall -Wextra -Werror against tests/jni/jni.h and drives every
 * native through tests/jni/fake_jvm.c.
 */
#define _POSIX_C_SOURCE 200809L
#include <jni.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ipls_agg.h"

static void throw_msg(JNIEnv *env, const char *cls, const char *msg) {
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, msg);
}

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
    (void)h;
    throw_msg(env, cls, ipls_agg_last_error(NULL));   /* this thread's failure */
}

static void throw_iae(JNIEnv *env, const char *what) {
    throw_msg(env, "java/lang/IllegalArgumentException", what);
}

#ifdef IPLS_JNI_CALL_HOOK
void IPLS_JNI_CALL_HOOK(const char *call);
#define LIB(x) (IPLS_JNI_CALL_HOOK(#x), (x))
#else
#define LIB(x) (x)
#endif

#define H(x) ((ipls_agg *)(intptr_t)(x))

/* ---- per-thread staging for heap arrays ----
 * Two slots per thread, each grown to the largest array that thread has
 * passed so far and kept for reuse (no allocation and no page faults per
 * call); freed when the thread ends.  The two hot heap-array natives,
 * accumulate(double[]) and finalizePartition(byte[]), need no staging here:
 * the library calls back into the shim for each chunk
 * (ipls_agg_accumulate_chunked / ipls_agg_finalize_chunked), which copies it
 * between the Java array and the library's pinned ring while the previous
 * chunk is on the bus -- one library call per Java call, so the whole
 * arrival (or AggregatePartition plus its bytes) is one ordered unit. */
struct stage { void *p[2]; size_t cap[2]; };
static pthread_key_t g_stage_key;
static pthread_once_t g_stage_once = PTHREAD_ONCE_INIT;
static void stage_free(void *v) {
    struct stage *st = (struct stage *)v;
    free(st->p[0]);
    free(st->p[1]);
    free(st);
}
static void stage_init(void) { (void)pthread_key_create(&g_stage_key, stage_free); }

/* Staging slot `slot` (0 or 1) of at least `bytes` bytes, or NULL with an
 * OutOfMemoryError pending. */
static void *stage(JNIEnv *env, int slot, size_t bytes) {
    (void)pthread_once(&g_stage_once, stage_init);
    struct stage *st = (struct stage *)pthread_getspecific(g_stage_key);
    if (!st) {
        st = (struct stage *)calloc(1, sizeof *st);
        if (!st || pthread_setspecific(g_stage_key, st) != 0) {
            free(st);
            throw_msg(env, "java/lang/OutOfMemoryError", "JNI staging buffer");
            return NULL;
        }
    }
    if (bytes == 0) bytes = 1;
    if (st->cap[slot] < bytes) {
        void *q = realloc(st->p[slot], bytes);
        if (!q) { throw_msg(env, "java/lang/OutOfMemoryError", "JNI staging buffer"); return NULL; }
        st->p[slot] = q;
        st->cap[slot] = bytes;
    }
    return st->p[slot];
}

/* Values per chunk of the chunked natives, from the sweep of
 * tools/jni_heap_probe.py over chunk size x copy threads on one 4M-double
 * partition (profiles/r06/d): the heap -> ring direction (accumulate) runs
 * best at 16 MiB chunks (51 GB/s vs 44.5 at 4 MiB: fewer, longer H2D
 * transfers), the ring -> heap direction (finalizePartition, getPartitions)
 * at 4 MiB (40-41 GB/s; 16 MiB: 38.5).  IPLS_JNI_RING_CHUNK (values, even,
 * 2^16 .. 2^26) sets both, for sweeps. */
static jsize g_in_chunk = (jsize)1 << 21, g_out_chunk = (jsize)1 << 19;
static pthread_once_t g_ring_once = PTHREAD_ONCE_INIT;
static void ring_init(void) {
    const char *e = getenv("IPLS_JNI_RING_CHUNK");
    const long v = e ? atol(e) : 0;
    if (v >= (1L << 16) && v <= (1L << 26) && !(v & 1)) g_in_chunk = g_out_chunk = (jsize)v;
}
static jsize ring_chunk(int in) {
    (void)pthread_once(&g_ring_once, ring_init);
    return in ? g_in_chunk : g_out_chunk;
}
#define IN_CHUNK ring_chunk(1)    /* heap -> library: accumulate(double[]) */
#define RING_CHUNK ring_chunk(0)  /* library -> heap: finalizePartition, getPartitions */

/* ---- parallel copies between a Java array and the library's pinned ring ----
 * One memcpy thread moves 21-30 GB/s between pageable and pinned host memory
 * (tools/pinned_read_probe.hip, profiles/r05/h), half of what PCIe carries.
 * A chunk of at least PAR_MIN bytes is split over IPLS_JNI_COPY_THREADS
 * threads (default 6, the calling thread included: the ring -> heap copies
 * of finalizePartition / getPartitions gain 1.5-2 GB/s from 4 to 6, the
 * heap -> ring direction is flat, profiles/r06/d and h): a pool of helpers
 * created on first use, woken per chunk.  One caller at a time uses the pool; a
 * caller that finds it busy (another Java thread in the same native) copies
 * alone. */
#define PAR_MIN ((size_t)1 << 20)
#define PAR_MAX_THREADS 16
static struct {
    pthread_mutex_t use;          /* held by the caller whose chunk the helpers copy */
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    unsigned gen;                 /* chunk generation: helpers wake on a change */
    int helpers, pending;
    char *dst;
    const char *src;
    size_t bytes, part;
} g_pool = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER,
            PTHREAD_COND_INITIALIZER, 0, 0, 0, NULL, NULL, 0, 0};
static pthread_once_t g_pool_once = PTHREAD_ONCE_INIT;

static void *copy_helper(void *arg) {
    const size_t i = (size_t)(intptr_t)arg;   /* part i; the caller copies part 0 */
    unsigned seen = 0;
    pthread_mutex_lock(&g_pool.mu);
    for (;;) {
        while (g_pool.gen == seen) pthread_cond_wait(&g_pool.go, &g_pool.mu);
        seen = g_pool.gen;
        char *d = g_pool.dst;
        const char *s = g_pool.src;
        const size_t b = g_pool.bytes, part = g_pool.part;
        pthread_mutex_unlock(&g_pool.mu);
        const size_t lo = part * i;
        if (lo < b) memcpy(d + lo, s + lo, b - lo < part ? b - lo : part);
        pthread_mutex_lock(&g_pool.mu);
        if (--g_pool.pending == 0) pthread_cond_signal(&g_pool.done);
    }
    return NULL;
}

static void pool_init(void) {
    const char *e = getenv("IPLS_JNI_COPY_THREADS");
    int t = e ? atoi(e) : 6;
    if (t < 1) t = 1;
    if (t > PAR_MAX_THREADS) t = PAR_MAX_THREADS;
    int made = 0;
    for (int i = 1; i < t; ++i) {
        pthread_t th;
        pthread_attr_t at;
        pthread_attr_init(&at);
        pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
        if (pthread_create(&th, &at, copy_helper, (void *)(intptr_t)i) == 0) ++made;
        pthread_attr_destroy(&at);
        if (made != i) break;   /* parts are numbered 1..made */
    }
    g_pool.helpers = made;
}

/* memcpy(dst, src, bytes), split over the pool when it is large and free. */
static void par_copy(void *dst, const void *src, size_t bytes) {
    (void)pthread_once(&g_pool_once, pool_init);
    if (bytes < PAR_MIN || g_pool.helpers == 0 || pthread_mutex_trylock(&g_pool.use) != 0) {
        memcpy(dst, src, bytes);
        return;
    }
    const size_t t = (size_t)g_pool.helpers + 1;
    const size_t part = ((bytes + t - 1) / t + 4095) / 4096 * 4096;
    pthread_mutex_lock(&g_pool.mu);
    g_pool.dst = (char *)dst;
    g_pool.src = (const char *)src;
    g_pool.bytes = bytes;
    g_pool.part = part;
    g_pool.pending = g_pool.helpers;
    ++g_pool.gen;
    pthread_cond_broadcast(&g_pool.go);
    pthread_mutex_unlock(&g_pool.mu);
    memcpy(dst, src, bytes < part ? bytes : part);
    pthread_mutex_lock(&g_pool.mu);
    while (g_pool.pending > 0) pthread_cond_wait(&g_pool.done, &g_pool.mu);
    pthread_mutex_unlock(&g_pool.mu);
    pthread_mutex_unlock(&g_pool.use);
}

/* Copy `bytes` at byte offset `off` of a primitive array to (to_array == 0)
 * or from (to_array == 1) `ring`, inside ONE short critical region (see the
 * file comment); no JNI or library call happens while it is open.  Returns 0,
 * or 1 when the JVM could not give the array (OutOfMemoryError pending) or
 * gave a copy of it -- the caller then uses Get/Set<T>ArrayRegion instead. */
static int critical_copy(JNIEnv *env, jarray a, size_t off, void *ring, size_t bytes, int to_array) {
    jboolean is_copy = JNI_FALSE;
    char *p = (char *)(*env)->GetPrimitiveArrayCritical(env, a, &is_copy);
    if (!p) return 1;
    if (is_copy) {   /* a whole-array copy per chunk would be quadratic */
        (*env)->ReleasePrimitiveArrayCritical(env, a, p, JNI_ABORT);
        return 1;
    }
    if (to_array) par_copy(p + off, ring, bytes);
    else par_copy(ring, p + off, bytes);
    (*env)->ReleasePrimitiveArrayCritical(env, a, p, to_array ? 0 : JNI_ABORT);
    return 0;
}

/* A copy of the whole double[] / byte[] in staging slot `slot`. */
static void *copy_doubles(JNIEnv *env, jdoubleArray a, jsize n, int slot) {
    double *d = (double *)stage(env, slot, (size_t)n * 8);
    if (d && n > 0) (*env)->GetDoubleArrayRegion(env, a, 0, n, d);
    return d;
}
static void *copy_bytes(JNIEnv *env, jbyteArray a, jsize n, int slot) {
    jbyte *d = (jbyte *)stage(env, slot, (size_t)n);
    if (d && n > 0) (*env)->GetByteArrayRegion(env, a, 0, n, d);
    return d;
}
#define CHECK(rc, h) do { int rc_ = (rc); if (rc_ < 0) { throw_for(env, rc_, (h)); } } while (0)

/* The bytes [pos, pos + count * elem) of a direct buffer, or NULL with an
 * IllegalArgumentException pending. */
static void *direct_span(JNIEnv *env, jobject buf, jint pos, jlong count, jlong elem) {
    if (!buf) { throw_iae(env, "null buffer"); return NULL; }
    char *a = (char *)(*env)->GetDirectBufferAddress(env, buf);
    const jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
    if (!a || cap < 0) { throw_iae(env, "not a direct ByteBuffer (allocate it with hostAlloc)"); return NULL; }
    /* count elements of elem bytes from byte pos: checked before any
     * multiplication, so a huge count from Java cannot overflow */
    if (pos < 0 || (jlong)pos > cap || count < 0 || count > (cap - (jlong)pos) / elem) {
        throw_iae(env, "position/length outside the buffer");
        return NULL;
    }
    return a + pos;
}

/* L_p (or -1 with the exception pending). */
static int64_t part_len(JNIEnv *env, jlong h, jint p) {
    int64_t L = 0;
    int rc = LIB(ipls_agg_partition_len(H(h), p, &L));
    if (rc < 0) { throw_for(env, rc, H(h)); return -1; }
    return L;
}

/* Java array length >= need, else an IllegalArgumentException. */
static int need_len(JNIEnv *env, jarray a, int64_t need, const char *what) {
    if (!a) { throw_iae(env, what); return 0; }
    if ((int64_t)(*env)->GetArrayLength(env, a) < need) {
        char m[160];
        snprintf(m, sizeof m, "%s: array shorter than the %lld elements the library writes", what, (long long)need);
        throw_iae(env, m);
        return 0;
    }
    return 1;
}

static jlong open_cfg(JNIEnv *env, ipls_agg_cfg *cfg) {
    ipls_agg *h = NULL;
    int rc = LIB(ipls_agg_open(cfg, &h));
    if (rc < 0) { throw_for(env, rc, NULL); return 0; }
    return (jlong)(intptr_t)h;
}

JNIEXPORT jlong JNICALL Java_NativeAggregator_open(JNIEnv *env, jclass c, jlong m, jint pa, jint n,
                                                     jint aggr, jint secure, jint dev) {
    (void)c;
    ipls_agg_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.model_size = m; cfg.n_partitions = pa; cfg.max_peers = n;
    cfg.partial_aggregation = aggr; cfg.secure = secure; cfg.device = dev;
    return open_cfg(env, &cfg);
}

/* The same over several GPUs: -pa partitions in contiguous blocks over devices[]. */
JNIEXPORT jlong JNICALL Java_NativeAggregator_openDevices(JNIEnv *env, jclass c, jlong m, jint pa, jint n,
                                                            jint aggr, jint secure, jintArray devices) {
    (void)c;
    if (!devices || (*env)->GetArrayLength(env, devices) < 1) { throw_iae(env, "need at least one device"); return 0; }
    ipls_agg_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.model_size = m; cfg.n_partitions = pa; cfg.max_peers = n;
    cfg.partial_aggregation = aggr; cfg.secure = secure;
    cfg.n_devices = (*env)->GetArrayLength(env, devices);
    jint *d = (*env)->GetIntArrayElements(env, devices, NULL);
    cfg.devices = (const int32_t *)d;
    cfg.device = d ? d[0] : 0;
    jlong h = d ? open_cfg(env, &cfg) : 0;   /* the list is copied by ipls_agg_open */
    if (d) (*env)->ReleaseIntArrayElements(env, devices, d, JNI_ABORT);
    return h;
}

JNIEXPORT void JNICALL Java_NativeAggregator_close(JNIEnv *env, jclass c, jlong h) {
    (void)env; (void)c;
    LIB(ipls_agg_close(H(h)));
}

JNIEXPORT jlong JNICALL Java_NativeAggregator_partitionLen(JNIEnv *env, jclass c, jlong h, jint p) {
    (void)c;
    return (jlong)part_len(env, h, p);
}

JNIEXPORT jlong JNICALL Java_NativeAggregator_partitionOffset(JNIEnv *env, jclass c, jlong h, jint p) {
    (void)c;
    int64_t off = 0;
    CHECK(LIB(ipls_agg_partition_offset(H(h), p, &off)), H(h));
    return (jlong)off;
}

JNIEXPORT jint JNICALL Java_NativeAggregator_partitionDevice(JNIEnv *env, jclass c, jlong h, jint p) {
    (void)c;
    int32_t d = -1;
    CHECK(LIB(ipls_agg_partition_device(H(h), p, &d, NULL)), H(h));
    return d;
}

JNIEXPORT jintArray JNICALL Java_NativeAggregator_shardPlan(JNIEnv *env, jclass c, jint partitions, jint shards) {
    (void)c;
    if (partitions <= 0) { throw_iae(env, "partitions must be > 0"); return NULL; }
    int32_t *o = (int32_t *)malloc(sizeof(int32_t) * (size_t)partitions);
    if (!o) { throw_msg(env, "java/lang/OutOfMemoryError", "shard plan"); return NULL; }
    int rc = LIB(ipls_shard_plan(partitions, shards, o));
    jintArray res = NULL;
    if (rc < 0) {
        throw_for(env, rc, NULL);
    } else {
        res = (*env)->NewIntArray(env, partitions);
        if (res) (*env)->SetIntArrayRegion(env, res, 0, partitions, (const jint *)o);
    }
    free(o);
    return res;
}

JNIEXPORT void JNICALL Java_NativeAggregator_loadModel(JNIEnv *env, jclass c, jlong h, jdoubleArray a) {
    (void)c;
    if (!a) { throw_iae(env, "null model"); return; }
    jsize n = (*env)->GetArrayLength(env, a);
    void *p = copy_doubles(env, a, n, 0);
    if (!p) return;
    CHECK(LIB(ipls_agg_load_model(H(h), p, n, IPLS_HOST_F64)), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_split(JNIEnv *env, jclass c, jlong h, jdoubleArray flat, jint part,
                                                     jdoubleArray out) {
    (void)c;
    const int64_t L = part_len(env, h, part);
    if (L < 0 || !need_len(env, out, L, "split output") || !need_len(env, flat, 0, "null gradients")) return;
    jsize n = (*env)->GetArrayLength(env, flat);
    void *src = copy_doubles(env, flat, n, 0);
    double *dst = src ? (double *)stage(env, 1, (size_t)L * 8) : NULL;
    if (!dst) return;
    int rc = LIB(ipls_agg_split(H(h), src, n, IPLS_HOST_F64, part, dst, IPLS_HOST_F64));
    if (rc >= 0) (*env)->SetDoubleArrayRegion(env, out, 0, (jsize)L, dst);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_updateGradient(JNIEnv *env, jclass c, jlong h, jdoubleArray flat,
                                                              jintArray owned) {
    (void)c;
    if (!flat) return;   /* Gradients == null: no-op (IPLS.java:1738) */
    if (!owned) { throw_iae(env, "null auth list"); return; }
    jsize n = (*env)->GetArrayLength(env, flat), no = (*env)->GetArrayLength(env, owned);
    double *src = (double *)stage(env, 0, (size_t)n * 8);
    if (!src) return;
    jint *own = (*env)->GetIntArrayElements(env, owned, NULL);
    if (!own) return;   /* OutOfMemoryError pending */
    /* Only the owned partitions' values leave the heap: ipls_agg_update_gradient
     * checks the length against every partition (OrganizeGradients) but reads
     * only the owned partitions' slices [off, off + L - 1) of the vector
     * (engine.hip dev_update_gradient), so the rest of the staging copy would
     * never be looked at.  An owned index the library rejects copies nothing. */
    for (jsize i = 0; i < no; ++i) {
        int64_t off = 0, L = 0;
        if (LIB(ipls_agg_partition_offset(H(h), own[i], &off)) < 0 || LIB(ipls_agg_partition_len(H(h), own[i], &L)) < 0)
            continue;
        const int64_t hi = off + (L - 1) < (int64_t)n ? off + (L - 1) : (int64_t)n;
        if (hi > off) (*env)->GetDoubleArrayRegion(env, flat, (jsize)off, (jsize)(hi - off), src + off);
        if ((*env)->ExceptionCheck(env)) {
            (*env)->ReleaseIntArrayElements(env, owned, own, JNI_ABORT);
            return;
        }
    }
    int rc = LIB(ipls_agg_update_gradient(H(h), src, n, IPLS_HOST_F64, (const int32_t *)own, no));
    (*env)->ReleaseIntArrayElements(env, owned, own, JNI_ABORT);
    CHECK(rc, H(h));
}

/* Middleware task 2 without the List<Double>: the update's big-endian bytes
 * in a direct buffer (as read off the socket) folded into the owned
 * partitions (ipls_agg_update_gradient, HOST_BE: the byte swap fused into
 * the fold, only the owned partitions' bytes cross PCIe). */
JNIEXPORT void JNICALL Java_NativeAggregator_updateGradientDirect(JNIEnv *env, jclass c, jlong h, jobject buf,
                                                                    jint pos, jlong n, jintArray owned) {
    (void)c;
    void *src = direct_span(env, buf, pos, n, 8);
    if (!src) return;
    if (!owned) { throw_iae(env, "null auth list"); return; }
    const jsize no = (*env)->GetArrayLength(env, owned);
    jint *own = (*env)->GetIntArrayElements(env, owned, NULL);
    if (!own) return;   /* OutOfMemoryError pending */
    int rc = LIB(ipls_agg_update_gradient(H(h), src, n, IPLS_HOST_BE, (const int32_t *)own, no));
    (*env)->ReleaseIntArrayElements(env, owned, own, JNI_ABORT);
    CHECK(rc, H(h));
}

/* The chunk source of accumulate(double[]): the library asks for the
 * bucket's values [off, off + n) and the shim copies them out of the heap. */
struct heap_source { JNIEnv *env; jdoubleArray a; };
static int heap_source_fn(void *ctx, void *dst, int64_t off, int64_t n) {
    struct heap_source *s = (struct heap_source *)ctx;
    /* [off, off + n) lies inside the array: the library asks only for values
     * below L_p, and it refused an array shorter than L_p before any chunk */
    if ((size_t)n * 8 >= PAR_MIN && critical_copy(s->env, s->a, (size_t)off * 8, dst, (size_t)n * 8, 0) == 0) return 0;
    if ((*s->env)->ExceptionCheck(s->env)) return 1;
    (*s->env)->GetDoubleArrayRegion(s->env, s->a, (jsize)off, (jsize)n, (jdouble *)dst);
    return (*s->env)->ExceptionCheck(s->env) ? 1 : 0;
}

JNIEXPORT void JNICALL Java_NativeAggregator_accumulate(JNIEnv *env, jclass c, jlong h, jint p, jint tgt,
                                                          jdoubleArray g) {
    (void)c;
    if (!g) return;   /* Gradient == null: the Updater loops do nothing (Updater.java:115) */
    /* One call for the whole arrival (Updater._Update under PeerData.mtx,
     * Updater.java:72-149): the library pulls the bucket's first L values
     * chunk by chunk through heap_source_fn (critical_copy into its pinned
     * ring) while the previous chunk crosses PCIe, then folds the bucket in
     * one launch.  The arrival takes effect as one unit once its last chunk
     * has landed (the GPU shard is not held while the chunks are copied: no
     * other caller waits for this thread's heap copies), a short array is
     * ArrayIndexOutOfBoundsException before any copy, and a failed copy
     * folds nothing. */
    struct heap_source hs = {env, g};
    const jsize n = (*env)->GetArrayLength(env, g);
    const int rc = LIB(ipls_agg_accumulate_chunked(H(h), p, tgt, n, IPLS_HOST_F64, IN_CHUNK, heap_source_fn, &hs));
    if (rc < 0 && !(*env)->ExceptionCheck(env)) throw_for(env, rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_accumulateDirect(JNIEnv *env, jclass c, jlong h, jint p, jint tgt,
                                                                jobject buf, jint pos, jlong n, jint kind) {
    (void)c;
    void *src = direct_span(env, buf, pos, n, 8);
    if (!src) return;
    CHECK(LIB(ipls_agg_accumulate(H(h), p, tgt, src, n, kind)), H(h));
}

JNIEXPORT jlong JNICALL Java_NativeAggregator_accumulateAsyncDirect(JNIEnv *env, jclass c, jlong h, jint p,
                                                                      jint tgt, jobject buf, jint pos, jlong n,
                                                                      jint kind) {
    (void)c;
    void *src = direct_span(env, buf, pos, n, 8);
    if (!src) return 0;
    uint64_t t = 0;
    CHECK(LIB(ipls_agg_accumulate_async(H(h), p, tgt, src, n, kind, &t)), H(h));
    return (jlong)t;
}

JNIEXPORT void JNICALL Java_NativeAggregator_waitTicket(JNIEnv *env, jclass c, jlong h, jlong ticket) {
    (void)c;
    CHECK(LIB(ipls_agg_wait(H(h), (uint64_t)ticket)), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_flushQueued(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    CHECK(LIB(ipls_agg_flush(H(h))), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_updateIndirect(JNIEnv *env, jclass c, jlong h, jint p, jint tgt,
                                                              jobject buf, jint pos, jlong nBytes) {
    (void)c;
    void *src = direct_span(env, buf, pos, nBytes, 1);
    if (!src) return;
    CHECK(LIB(ipls_agg_update_indirect(H(h), p, tgt, src, nBytes)), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_accumulateFrame(JNIEnv *env, jclass c, jlong h, jint p, jint tgt,
                                                               jbyteArray frame) {
    (void)c;
    if (!frame) { throw_iae(env, "null frame"); return; }
    jsize n = (*env)->GetArrayLength(env, frame);
    void *src = copy_bytes(env, frame, n, 0);
    if (!src) return;
    CHECK(LIB(ipls_agg_accumulate(H(h), p, tgt, src, n, IPLS_HOST_FRAME)), H(h));
}

/* ThreadReceiver: a batch of pubsub texts.  The texts are copied into one
 * staging arena (GetByteArrayRegion: no critical region, so the JVM's GC
 * keeps running while the library copies them to the GPU and folds them). */
JNIEXPORT jint JNICALL Java_NativeAggregator_ingestTexts(JNIEnv *env, jclass c, jlong h, jint tgt,
                                                         jobjectArray msgs, jint layers, jintArray parts,
                                                         jintArray status) {
    (void)c;
    const jsize n = msgs ? (*env)->GetArrayLength(env, msgs) : 0;
    if (parts && (*env)->GetArrayLength(env, parts) < n) { throw_iae(env, "partitions shorter than the texts"); return 0; }
    if (status && (*env)->GetArrayLength(env, status) < n) { throw_iae(env, "status shorter than the texts"); return 0; }
    const uint8_t **ptr = calloc((size_t)n + 1, sizeof *ptr);
    int64_t *len = calloc((size_t)n + 1, sizeof *len);
    int64_t *off = calloc((size_t)n + 1, sizeof *off);
    int32_t *st = calloc((size_t)n + 1, sizeof *st);
    jint *pp = NULL;
    int rc = IPLS_E_NOMEM;
    if (!ptr || !len || !off || !st) { throw_msg(env, "java/lang/OutOfMemoryError", "ingestTexts"); goto out; }
    /* pass 1: lengths and arena offsets (one local ref at a time) */
    int64_t total = 0;
    for (jsize i = 0; i < n; ++i) {
        jbyteArray t = (jbyteArray)(*env)->GetObjectArrayElement(env, msgs, i);
        len[i] = t ? (*env)->GetArrayLength(env, t) : 0;
        off[i] = t ? total : -1;
        total += (len[i] + 63) / 64 * 64;
        if (t) (*env)->DeleteLocalRef(env, t);
    }
    uint8_t *arena = (uint8_t *)stage(env, 0, (size_t)total);
    if (!arena) goto out;
    /* pass 2: the copies */
    for (jsize i = 0; i < n; ++i) {
        if (off[i] < 0) continue;
        jbyteArray t = (jbyteArray)(*env)->GetObjectArrayElement(env, msgs, i);
        if (len[i] > 0) (*env)->GetByteArrayRegion(env, t, 0, (jsize)len[i], (jbyte *)(arena + off[i]));
        (*env)->DeleteLocalRef(env, t);
        if ((*env)->ExceptionCheck(env)) goto out;   /* the array changed under us (AIOOBE pending) */
        ptr[i] = arena + off[i];
    }
    if (parts) {
        pp = (*env)->GetIntArrayElements(env, parts, NULL);
        if (!pp) goto out;   /* OutOfMemoryError pending */
    }
    rc = LIB(ipls_agg_ingest_pubsub(H(h), tgt, ptr, len, n, layers, (const int32_t *)pp, st));
    if (pp) (*env)->ReleaseIntArrayElements(env, parts, pp, JNI_ABORT);
    if (status && rc >= 0) (*env)->SetIntArrayRegion(env, status, 0, n, (const jint *)st);
    CHECK(rc, H(h));
out:
    free(ptr);
    free(len);
    free(off);
    free(st);
    return rc;
}

/* The chunk sink of finalizePartition(byte[]): the commit_update bytes of
 * values [off, off + n) straight from the library's pinned ring into the array. */
struct bytes_sink { JNIEnv *env; jbyteArray out; };
static int bytes_sink_fn(void *ctx, const double *values, int64_t off, int64_t n) {
    struct bytes_sink *b = (struct bytes_sink *)ctx;
    /* the array holds 8 * L_p bytes (need_len before the call) */
    if ((size_t)n * 8 >= PAR_MIN && critical_copy(b->env, b->out, (size_t)off * 8, (void *)values, (size_t)n * 8, 1) == 0)
        return 0;
    if ((*b->env)->ExceptionCheck(b->env)) return 1;
    (*b->env)->SetByteArrayRegion(b->env, b->out, (jsize)(8 * off), (jsize)(8 * n), (const jbyte *)values);
    return (*b->env)->ExceptionCheck(b->env) ? 1 : 0;
}

JNIEXPORT void JNICALL Java_NativeAggregator_finalizePartition(JNIEnv *env, jclass c, jlong h, jint p,
                                                                 jbyteArray sum) {
    (void)c;
    if (!sum) {
        CHECK(LIB(ipls_agg_finalize(H(h), p, NULL, IPLS_HOST_BE, NULL)), H(h));
        return;
    }
    const int64_t L = part_len(env, h, p);
    if (L < 0 || !need_len(env, sum, 8 * L, "commit_update bytes")) return;
    /* One call: AggregatePartition on the device, then W's big-endian bytes
     * come back chunk by chunk through the library's pinned ring, each
     * copied into the byte[] while the next is in flight.  The bytes are a
     * snapshot of this call's W: a set_weights or finalize of another thread
     * meanwhile neither waits for the copies nor tears the bytes. */
    struct bytes_sink bs = {env, sum};
    const int rc = LIB(ipls_agg_finalize_chunked(H(h), p, IPLS_HOST_BE, RING_CHUNK, bytes_sink_fn, &bs));
    if (rc < 0 && !(*env)->ExceptionCheck(env)) throw_for(env, rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_finalizePartitionDirect(JNIEnv *env, jclass c, jlong h, jint p,
                                                                       jobject sum, jint pos) {
    (void)c;
    const int64_t L = part_len(env, h, p);
    if (L < 0) return;
    void *dst = direct_span(env, sum, pos, L, 8);
    if (!dst) return;
    CHECK(LIB(ipls_agg_finalize(H(h), p, dst, IPLS_HOST_BE, NULL)), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_setWeightsDirect(JNIEnv *env, jclass c, jlong h, jint p, jobject buf,
                                                                jint pos, jlong n) {
    (void)c;
    void *src = direct_span(env, buf, pos, n, 8);
    if (!src) return;
    CHECK(LIB(ipls_agg_set_weights(H(h), p, src, n, IPLS_HOST_BE)), H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_setWeightsFrame(JNIEnv *env, jclass c, jlong h, jint p,
                                                               jbyteArray frame) {
    (void)c;
    if (!frame) { throw_iae(env, "null frame"); return; }
    jsize n = (*env)->GetArrayLength(env, frame);
    void *src = copy_bytes(env, frame, n, 0);
    if (!src) return;
    CHECK(LIB(ipls_agg_set_weights(H(h), p, src, n, IPLS_HOST_FRAME)), H(h));
}

/* The chunk sink of getPartitions: each chunk of the model straight from
 * the library's pinned ring into the Java array. */
struct model_sink { JNIEnv *env; jdoubleArray out; };
static int model_sink_fn(void *ctx, const double *values, int64_t off, int64_t n) {
    struct model_sink *m = (struct model_sink *)ctx;
    /* off + n <= M <= the array's length (checked before the call) */
    if ((size_t)n * 8 >= PAR_MIN && critical_copy(m->env, m->out, (size_t)off * 8, (void *)values, (size_t)n * 8, 1) == 0)
        return 0;
    if ((*m->env)->ExceptionCheck(m->env)) return 1;
    (*m->env)->SetDoubleArrayRegion(m->env, m->out, (jsize)off, (jsize)n, values);
    return (*m->env)->ExceptionCheck(m->env) ? 1 : 0;
}

JNIEXPORT void JNICALL Java_NativeAggregator_getPartitions(JNIEnv *env, jclass c, jlong h, jdoubleArray out) {
    (void)c;
    if (!out) { throw_iae(env, "null output"); return; }
    jsize n = (*env)->GetArrayLength(env, out);   /* the library checks n against the model size */
    /* the library writes the model's first M values; only those go back into
     * the array (elements past the model keep theirs), so nothing is copied in */
    int64_t M = 0;
    int rc = LIB(ipls_agg_flat_size(H(h), &M));
    if (rc < 0) { throw_for(env, rc, H(h)); return; }
    if (M >= 2 * RING_CHUNK && M <= n) {
        /* Pipelined: the divide once on the GPU, then the model comes back in
         * ring-sized chunks, each copied into the array while the next is in
         * flight (ipls_agg_get_partitions_chunked). */
        struct model_sink ms = {env, out};
        rc = LIB(ipls_agg_get_partitions_chunked(H(h), RING_CHUNK, model_sink_fn, &ms));
        if (rc < 0 && !(*env)->ExceptionCheck(env)) throw_for(env, rc, H(h));
        return;
    }
    double *dst = (double *)stage(env, 0, (size_t)n * 8);
    if (!dst) return;
    rc = LIB(ipls_agg_get_partitions(H(h), dst, n, IPLS_HOST_F64));
    if (rc >= 0) (*env)->SetDoubleArrayRegion(env, out, 0, (jsize)(M < (int64_t)n ? M : (int64_t)n), dst);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_aggregateRound(JNIEnv *env, jclass c, jlong h, jint p0, jint np,
                                                              jdoubleArray out) {
    (void)c;
    /* the averages of [p0, p0+np): flat offsets off[p0] .. off[p_last] + L_last - 1 */
    int64_t o0 = 0, ol = 0, Ll = 0;
    int rc = np > 0 ? LIB(ipls_agg_partition_offset(H(h), p0, &o0)) : IPLS_E_RANGE;
    if (rc >= 0) rc = LIB(ipls_agg_partition_offset(H(h), p0 + np - 1, &ol));
    if (rc >= 0) rc = LIB(ipls_agg_partition_len(H(h), p0 + np - 1, &Ll));
    if (rc < 0) { throw_for(env, rc, H(h)); return; }
    if (out && !need_len(env, out, ol + Ll - 1 - o0, "averages")) return;
    const int64_t na = ol + Ll - 1 - o0;
    double *dst = out ? (double *)stage(env, 0, (size_t)na * 8) : NULL;
    if (out && !dst) return;
    rc = LIB(ipls_agg_aggregate_round(H(h), p0, np, NULL, 0, IPLS_DEV_F64, dst, IPLS_HOST_F64));
    if (out && rc >= 0) (*env)->SetDoubleArrayRegion(env, out, 0, (jsize)na, dst);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_promoteFuture(JNIEnv *env, jclass c, jlong h, jintArray parts) {
    (void)c;
    if (!parts) { throw_iae(env, "null partition list"); return; }
    jsize n = (*env)->GetArrayLength(env, parts);
    jint *ps = (*env)->GetIntArrayElements(env, parts, NULL);
    int rc = LIB(ipls_agg_promote_future(H(h), (const int32_t *)ps, n));
    (*env)->ReleaseIntArrayElements(env, parts, ps, JNI_ABORT);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_otherReplicaDirect(JNIEnv *env, jclass c, jlong h, jint p, jint a,
                                                                  jint keyHash, jobject buf, jint pos, jlong n) {
    (void)c;
    void *src = direct_span(env, buf, pos, n, 8);
    if (!src) return;
    CHECK(LIB(ipls_agg_other_replica_keyed(H(h), p, a, keyHash, src, n, IPLS_HOST_BE)), H(h));
}

JNIEXPORT jboolean JNICALL Java_NativeAggregator_otherReplicaDrop(JNIEnv *env, jclass c, jlong h, jint p, jint a) {
    (void)c;
    const int rc = LIB(ipls_agg_other_replica_drop(H(h), p, a));
    if (rc < 0) {
        throw_for(env, rc, H(h));
        return JNI_FALSE;
    }
    return rc == 1 ? JNI_TRUE : JNI_FALSE;
}

/* The library's Collect_Replicas order as {p0, a0, p1, a1, ...} (a check of
 * its HashMap model against the JVM's own keySet() order). */
JNIEXPORT jintArray JNICALL Java_NativeAggregator_replicaKeyOrder(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    int room = LIB(ipls_agg_replica_order(H(h), NULL, 0, NULL)), n;
    if (room < 0) { throw_for(env, room, H(h)); return NULL; }
    int32_t *pairs = NULL;
    for (;;) {   /* keys stored by another thread in between: ask again with more room */
        free(pairs);
        pairs = (int32_t *)malloc((size_t)(room > 0 ? 2 * (size_t)room : 2) * sizeof(int32_t));
        if (!pairs) { throw_msg(env, "java/lang/OutOfMemoryError", "replicaKeyOrder"); return NULL; }
        n = LIB(ipls_agg_replica_order(H(h), pairs, room, NULL));
        if (n <= room) break;
        room = n;
    }
    jintArray res = NULL;
    if (n < 0) {
        throw_for(env, n, H(h));
    } else {
        res = (*env)->NewIntArray(env, 2 * n);
        if (res) (*env)->SetIntArrayRegion(env, res, 0, 2 * n, (const jint *)pairs);
    }
    free(pairs);
    return res;
}

JNIEXPORT jint JNICALL Java_NativeAggregator_collectReplicas(JNIEnv *env, jclass c, jlong h, jintArray out) {
    (void)c;
    /* the library writes one count per partition: out.length >= P, i.e.
     * partition out.length must NOT exist */
    if (out) {
        int64_t L;
        const jsize n = (*env)->GetArrayLength(env, out);
        if (n == 0 || LIB(ipls_agg_partition_len(H(h), n, &L)) == IPLS_OK) {
            throw_iae(env, "participants array shorter than the number of partitions");
            return 0;
        }
    }
    jint *ps = out ? (*env)->GetIntArrayElements(env, out, NULL) : NULL;
    int rc = LIB(ipls_agg_collect_replicas(H(h), (int32_t *)ps));
    if (ps) (*env)->ReleaseIntArrayElements(env, out, ps, 0);
    CHECK(rc, H(h));
    return rc;
}

JNIEXPORT jlong JNICALL Java_NativeAggregator_commitPartialLen(JNIEnv *env, jclass c, jlong h, jint p, jint w) {
    (void)c;
    int64_t n = LIB(ipls_agg_commit_partial(H(h), p, w, NULL, 0));
    if (n < 0) { throw_for(env, (int)n, H(h)); return 0; }
    return (jlong)n;
}

JNIEXPORT void JNICALL Java_NativeAggregator_commitPartial(JNIEnv *env, jclass c, jlong h, jint p, jint w,
                                                             jbyteArray out) {
    (void)c;
    if (!out) { throw_iae(env, "null output"); return; }
    jsize n = (*env)->GetArrayLength(env, out);   /* passed as the capacity: the library checks it */
    jbyte *dst = (jbyte *)stage(env, 0, (size_t)n);
    if (!dst) return;
    int64_t rc = LIB(ipls_agg_commit_partial(H(h), p, w, (uint8_t *)dst, n));
    if (rc < 0) throw_for(env, (int)rc, H(h));
    else (*env)->SetByteArrayRegion(env, out, 0, (jsize)rc, dst);
}

JNIEXPORT void JNICALL Java_NativeAggregator_accumulatePair(JNIEnv *env, jclass c, jlong h, jint p, jint tgt,
                                                              jbyteArray file) {
    (void)c;
    if (!file) { throw_iae(env, "null file"); return; }
    jsize n = (*env)->GetArrayLength(env, file);
    void *src = copy_bytes(env, file, n, 0);
    if (!src) return;
    CHECK(LIB(ipls_agg_accumulate(H(h), p, tgt, src, n, IPLS_HOST_PAIR)), H(h));
}

JNIEXPORT jbyteArray JNICALL Java_NativeAggregator_mergeFiles(JNIEnv *env, jclass c, jlong h, jobjectArray files,
                                                                jboolean partial) {
    (void)c;
    jsize k = files ? (*env)->GetArrayLength(env, files) : 0;
    if (k < 1) { throw_iae(env, "need at least one file"); return NULL; }
    const uint8_t **ptrs = (const uint8_t **)calloc((size_t)k, sizeof(uint8_t *));
    int64_t *lens = (int64_t *)calloc((size_t)k, sizeof(int64_t));
    int64_t *offs = (int64_t *)calloc((size_t)k, sizeof(int64_t));
    jbyteArray res = NULL;
    uint8_t *out = NULL;
    if (!ptrs || !lens || !offs) { throw_msg(env, "java/lang/OutOfMemoryError", "mergeFiles"); goto done; }
    int64_t total = 0;
    for (jsize i = 0; i < k; ++i) {   /* lengths first, one local ref at a time */
        jbyteArray a = (jbyteArray)(*env)->GetObjectArrayElement(env, files, i);
        if (!a) { throw_iae(env, "null file"); goto done; }
        lens[i] = (*env)->GetArrayLength(env, a);
        offs[i] = total;
        total += (lens[i] + 63) / 64 * 64;
        (*env)->DeleteLocalRef(env, a);
    }
    uint8_t *arena = (uint8_t *)stage(env, 0, (size_t)total);
    if (!arena) goto done;
    for (jsize i = 0; i < k; ++i) {   /* copies (GetByteArrayRegion): no array stays pinned across the merge */
        jbyteArray a = (jbyteArray)(*env)->GetObjectArrayElement(env, files, i);
        if (lens[i] > 0) (*env)->GetByteArrayRegion(env, a, 0, (jsize)lens[i], (jbyte *)(arena + offs[i]));
        (*env)->DeleteLocalRef(env, a);
        if ((*env)->ExceptionCheck(env)) goto done;   /* the array changed under us (AIOOBE pending) */
        ptrs[i] = arena + offs[i];
    }
    int64_t cap = 8 * (lens[0] / 8);
    if (partial) {
        int32_t w; int64_t off;
        int64_t n0 = LIB(ipls_pair_parse(ptrs[0], lens[0], &w, &off));
        cap = n0 < 0 ? 0 : 8 * n0;
    }
    out = (uint8_t *)malloc((size_t)(cap > 0 ? cap : 1));
    if (!out) { throw_msg(env, "java/lang/OutOfMemoryError", "mergeFiles"); goto done; }
    int64_t nb = LIB(ipls_agg_merge_files(H(h), ptrs, lens, k, partial ? IPLS_HOST_PAIR : IPLS_HOST_BE, out, cap));
    if (nb < 0) {
        throw_for(env, (int)nb, H(h));
    } else {
        res = (*env)->NewByteArray(env, (jsize)nb);
        if (res) (*env)->SetByteArrayRegion(env, res, 0, (jsize)nb, (const jbyte *)out);
    }
done:
    free(out); free(offs); free(lens); free(ptrs);
    return res;
}

JNIEXPORT void JNICALL Java_NativeAggregator_getPartitionsWire(JNIEnv *env, jclass c, jlong h, jobject buf,
                                                                 jint pos, jlong nBytes) {
    (void)c;
    void *dst = direct_span(env, buf, pos, nBytes, 1);
    if (!dst) return;
    CHECK(LIB(ipls_agg_get_partitions(H(h), dst, nBytes / 8, IPLS_HOST_BE_CANON)), H(h));
}

JNIEXPORT jobject JNICALL Java_NativeAggregator_hostAllocDirect(JNIEnv *env, jclass c, jint bytes) {
    (void)c;
    if (bytes < 0) { throw_iae(env, "negative size"); return NULL; }
    void *p = NULL;
    int rc = LIB(ipls_host_alloc((size_t)bytes, &p));
    if (rc < 0) { throw_for(env, rc, NULL); return NULL; }
    return (*env)->NewDirectByteBuffer(env, p, bytes);
}

/* ---- device-resident batches (ipls_agg_reduce_batch / reduce_partial) ----
 * ptrs holds n_parts * k device addresses (long), partition-major. */
static const void *const *dev_ptrs(JNIEnv *env, jlongArray ptrs, jint np, jint k, jlong **held) {
    *held = NULL;
    if (np <= 0 || k < 0) { throw_iae(env, "bad batch shape"); return NULL; }
    if (!need_len(env, ptrs, (int64_t)np * k, "device pointers")) return NULL;
    *held = (*env)->GetLongArrayElements(env, ptrs, NULL);
    if (!*held) { throw_msg(env, "java/lang/OutOfMemoryError", "device pointers"); return NULL; }
    return (const void *const *)*held;   /* jlong and void* are both 64-bit here */
}

JNIEXPORT void JNICALL Java_NativeAggregator_reduceBatchDevice(JNIEnv *env, jclass c, jlong h, jint p0, jint np,
                                                                 jlongArray ptrs, jint k, jint kind, jint start,
                                                                 jint target) {
    (void)c;
    jlong *held;
    const void *const *b = dev_ptrs(env, ptrs, np, k, &held);
    if (!b) return;
    int rc = LIB(ipls_agg_reduce_batch(H(h), p0, np, b, k, kind, start, target));
    (*env)->ReleaseLongArrayElements(env, ptrs, held, JNI_ABORT);
    CHECK(rc, H(h));
}

JNIEXPORT void JNICALL Java_NativeAggregator_reducePartialDevice(JNIEnv *env, jclass c, jlong h, jint slot, jint p0,
                                                                   jint np, jlongArray ptrs, jint k, jint kind,
                                                                   jint start) {
    (void)c;
    jlong *held;
    const void *const *b = dev_ptrs(env, ptrs, np, k, &held);
    if (!b) return;
    int rc = LIB(ipls_agg_reduce_partial(H(h), slot, p0, np, b, k, kind, start));
    (*env)->ReleaseLongArrayElements(env, ptrs, held, JNI_ABORT);
    CHECK(rc, H(h));
}

JNIEXPORT jint JNICALL Java_NativeAggregator_combinePartials(JNIEnv *env, jclass c, jlong h, jint p0, jint np) {
    (void)c;
    int rc = LIB(ipls_agg_combine_partials(H(h), p0, np));
    CHECK(rc, H(h));
    return rc;
}

/* Marshall_Packet(target[p], origin, a, b, pid) as the Base64.getUrlEncoder
 * text (MyIPFSClass.java:990-1016), encoded on the GPU. */
JNIEXPORT jbyteArray JNICALL Java_NativeAggregator_publishPartial(JNIEnv *env, jclass c, jlong h, jint p, jint tgt,
                                                                    jint a, jint b, jshort pid, jbyteArray origin) {
    (void)c;
    jsize ol = origin ? (*env)->GetArrayLength(env, origin) : 0;
    jbyte *o = origin ? (*env)->GetByteArrayElements(env, origin, NULL) : NULL;
    jbyteArray res = NULL;
    int64_t n = LIB(ipls_agg_publish_partial(H(h), p, tgt, a, b, pid, (const uint8_t *)o, ol, NULL, 0, IPLS_HOST_TEXT));
    uint8_t *text = n >= 0 ? (uint8_t *)malloc((size_t)(n > 0 ? n : 1)) : NULL;
    if (n >= 0 && !text) {
        throw_msg(env, "java/lang/OutOfMemoryError", "publish text");
    } else if (n >= 0) {
        n = LIB(ipls_agg_publish_partial(H(h), p, tgt, a, b, pid, (const uint8_t *)o, ol, text, n, IPLS_HOST_TEXT));
    }
    if (o) (*env)->ReleaseByteArrayElements(env, origin, o, JNI_ABORT);
    if (n < 0) {
        throw_for(env, (int)n, H(h));
    } else if (text) {
        res = (*env)->NewByteArray(env, (jsize)n);
        if (res) (*env)->SetByteArrayRegion(env, res, 0, (jsize)n, (const jbyte *)text);
    }
    free(text);
    return res;
}

/* ipls_agg_publish_partials layout: total bytes; lens/offs of every text. */
JNIEXPORT jlong JNICALL Java_NativeAggregator_publishPartialsLayout(JNIEnv *env, jclass c, jlong h, jintArray parts,
                                                                    jint originLen, jlongArray lens, jlongArray offs) {
    (void)c;
    if (!parts) { throw_iae(env, "null partition list"); return -1; }
    const jsize n = (*env)->GetArrayLength(env, parts);
    if (!need_len(env, lens, n, "lens") || !need_len(env, offs, n, "offs")) return -1;
    jint *pp = (*env)->GetIntArrayElements(env, parts, NULL);
    jlong *l = (*env)->GetLongArrayElements(env, lens, NULL);
    jlong *o = (*env)->GetLongArrayElements(env, offs, NULL);
    int64_t total = -1;
    if (pp && l && o)
        total = LIB(ipls_agg_publish_partials(H(h), (const int32_t *)pp, n, IPLS_TGT_AGG, 0, NULL, 3, NULL, originLen, NULL,
                                          0, IPLS_HOST_TEXT, (int64_t *)l, (int64_t *)o));
    if (o) (*env)->ReleaseLongArrayElements(env, offs, o, 0);
    if (l) (*env)->ReleaseLongArrayElements(env, lens, l, 0);
    if (pp) (*env)->ReleaseIntArrayElements(env, parts, pp, JNI_ABORT);
    if (total < 0) throw_for(env, (int)total, H(h));
    return (jlong)total;
}

/* The publish loop over Auth_List (IPLS.java:1423-1431) in one launch per
 * GPU: every text into the direct buffer at the layout's offsets. */
JNIEXPORT void JNICALL Java_NativeAggregator_publishPartialsDirect(JNIEnv *env, jclass c, jlong h, jintArray parts,
                                                                   jint tgt, jint a, jintArray b, jshort pid,
                                                                   jbyteArray origin, jobject buf, jint pos,
                                                                   jlong cap) {
    (void)c;
    if (!parts) { throw_iae(env, "null partition list"); return; }
    const jsize n = (*env)->GetArrayLength(env, parts);
    if (!need_len(env, b, n, "b (one value per partition)")) return;
    void *dst = direct_span(env, buf, pos, cap, 1);
    if (!dst) return;
    const jsize ol = origin ? (*env)->GetArrayLength(env, origin) : 0;
    jint *pp = (*env)->GetIntArrayElements(env, parts, NULL);
    jint *bb = (*env)->GetIntArrayElements(env, b, NULL);
    jbyte *o = origin ? (*env)->GetByteArrayElements(env, origin, NULL) : NULL;
    int64_t rc = IPLS_E_NOMEM;
    if (pp && bb && (o || !origin))
        rc = LIB(ipls_agg_publish_partials(H(h), (const int32_t *)pp, n, tgt, a, (const int32_t *)bb, pid,
                                       (const uint8_t *)o, ol, dst, cap, IPLS_HOST_TEXT, NULL, NULL));
    if (o) (*env)->ReleaseByteArrayElements(env, origin, o, JNI_ABORT);
    if (bb) (*env)->ReleaseIntArrayElements(env, b, bb, JNI_ABORT);
    if (pp) (*env)->ReleaseIntArrayElements(env, parts, pp, JNI_ABORT);
    if (rc < 0) throw_for(env, (int)rc, H(h));
}
