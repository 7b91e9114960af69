/*
 * tests/jni/fake_jvm.c -- a minimal stand-in for the JVM side of JNI, so the
 * shim ipls-java-api_amd/jni/ipls_jni.c can be exercised without a JDK
 * (TEST INFRASTRUCTURE; see tests/jni/jni.h).
 *
 * Java objects are heap records: primitive arrays (byte/int/long/double),
 * object arrays, direct ByteBuffers (address + capacity; a NULL address
 * models a heap ByteBuffer, for which GetDirectBufferAddress returns NULL and
 * GetDirectBufferCapacity -1) and classes.  ThrowNew records the pending
 * exception.  The JNI rules the shim must keep are checked and counted as
 * violations:
 *   - no JNI call other than Get/ReleasePrimitiveArrayCritical while a
 *     critical region is open,
 *   - no call other than the release / DeleteLocalRef / ExceptionCheck family
 *     while an exception is pending,
 *   - every Get*ArrayElements / GetPrimitiveArrayCritical released,
 *   - no *ArrayRegion access past the array's end,
 *   - no critical region open when the shim calls into libipls_agg (the shim,
 *     built with -DIPLS_JNI_CALL_HOOK=fj_library_call, reports every library
 *     call here): such a call may wait on the GPU, and a real JVM cannot
 *     collect garbage while a critical region is held.
 * It can also start a second "Java thread" in the middle of a native
 * (fj_inject): a library call on the same handle made between two chunks of
 * a chunked native, to show whether the native's work is one ordered unit.
 * tests/test_jni.py drives it through ctypes.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ipls_agg.h"
#include "jni.h"

enum { K_BYTES = 1, K_INTS, K_LONGS, K_DOUBLES, K_OBJECTS, K_DIRECT, K_CLASS };

struct _jobject {
    int kind;
    jsize n;          /* elements (arrays) */
    void *data;       /* array storage / direct address */
    jlong cap;        /* direct buffer capacity */
    char name[96];    /* class name */
};

static char g_exc_class[96];
static char g_exc_msg[512];
static int g_exc;
static int g_critical;
static int g_pinned;      /* Get*Elements not released yet */
static int g_violations;
static char g_last_violation[160];
static jint g_local_cap = 16;   /* the JNI spec guarantees 16 local refs per native frame */
static jint g_locals;              /* object-array element refs live (DeleteLocalRef releases) */

static void violation(const char *what) {
    ++g_violations;
    snprintf(g_last_violation, sizeof g_last_violation, "%s", what);
}

static void plain_call(const char *fn) {
    if (g_critical) violation(fn);
}

static void guarded_call(const char *fn) {   /* not allowed with an exception pending */
    plain_call(fn);
    if (g_exc) violation(fn);
}

static size_t esize(int kind) {
    switch (kind) {
        case K_BYTES: return 1;
        case K_INTS: return 4;
        case K_LONGS: return 8;
        case K_DOUBLES: return 8;
        case K_OBJECTS: return sizeof(jobject);
        default: return 1;
    }
}

static jobject new_array(int kind, jsize n) {
    jobject o = (jobject)calloc(1, sizeof *o);
    o->kind = kind;
    o->n = n;
    o->data = calloc((size_t)(n > 0 ? n : 1), esize(kind));
    return o;
}

/* ---- the JNIEnv functions ---- */
static jclass JNICALL FindClass(JNIEnv *env, const char *name) {
    (void)env;
    guarded_call("FindClass");
    jobject o = (jobject)calloc(1, sizeof *o);
    o->kind = K_CLASS;
    snprintf(o->name, sizeof o->name, "%s", name);
    return o;
}

static jint JNICALL ThrowNew(JNIEnv *env, jclass c, const char *msg) {
    (void)env;
    guarded_call("ThrowNew");
    snprintf(g_exc_class, sizeof g_exc_class, "%s", c->name);
    snprintf(g_exc_msg, sizeof g_exc_msg, "%s", msg ? msg : "");
    g_exc = 1;
    free(c);   /* the class record is not referenced again */
    return 0;
}

static jboolean JNICALL ExceptionCheck(JNIEnv *env) {
    (void)env;
    plain_call("ExceptionCheck");
    return g_exc ? JNI_TRUE : JNI_FALSE;
}

static void JNICALL DeleteLocalRef(JNIEnv *env, jobject o) {
    (void)env; (void)o;
    plain_call("DeleteLocalRef");   /* local refs of object-array elements: the array owns them */
    if (g_locals > 0) --g_locals;
}

static jsize JNICALL GetArrayLength(JNIEnv *env, jarray a) {
    (void)env;
    guarded_call("GetArrayLength");
    return a->n;
}

static jint JNICALL EnsureLocalCapacity(JNIEnv *env, jint cap) {
    (void)env;
    guarded_call("EnsureLocalCapacity");
    if (cap > g_local_cap) g_local_cap = cap;
    return 0;
}

static jobject JNICALL GetObjectArrayElement(JNIEnv *env, jobjectArray a, jsize i) {
    (void)env;
    guarded_call("GetObjectArrayElement");
    if (a->kind != K_OBJECTS || i < 0 || i >= a->n) { violation("GetObjectArrayElement index"); return NULL; }
    if (++g_locals > g_local_cap) violation("local references beyond EnsureLocalCapacity");
    return ((jobject *)a->data)[i];
}

static jbyteArray JNICALL NewByteArray(JNIEnv *env, jsize n) {
    (void)env;
    guarded_call("NewByteArray");
    return new_array(K_BYTES, n);
}

static jintArray JNICALL NewIntArray(JNIEnv *env, jsize n) {
    (void)env;
    guarded_call("NewIntArray");
    return new_array(K_INTS, n);
}

static void *elems(jarray a, int kind, const char *fn) {
    guarded_call(fn);
    if (!a || a->kind != kind) { violation(fn); return NULL; }
    ++g_pinned;
    return a->data;
}

static void release(jarray a, int kind, const char *fn) {
    plain_call(fn);
    if (!a || a->kind != kind) violation(fn);
    --g_pinned;
}

static jbyte *JNICALL GetByteArrayElements(JNIEnv *env, jbyteArray a, jboolean *c) {
    (void)env;
    if (c) *c = JNI_FALSE;
    return (jbyte *)elems(a, K_BYTES, "GetByteArrayElements");
}
static jint *JNICALL GetIntArrayElements(JNIEnv *env, jintArray a, jboolean *c) {
    (void)env;
    if (c) *c = JNI_FALSE;
    return (jint *)elems(a, K_INTS, "GetIntArrayElements");
}
static jlong *JNICALL GetLongArrayElements(JNIEnv *env, jlongArray a, jboolean *c) {
    (void)env;
    if (c) *c = JNI_FALSE;
    return (jlong *)elems(a, K_LONGS, "GetLongArrayElements");
}
static void JNICALL ReleaseByteArrayElements(JNIEnv *env, jbyteArray a, jbyte *e, jint m) {
    (void)env; (void)e; (void)m;
    release(a, K_BYTES, "ReleaseByteArrayElements");
}
static void JNICALL ReleaseIntArrayElements(JNIEnv *env, jintArray a, jint *e, jint m) {
    (void)env; (void)e; (void)m;
    release(a, K_INTS, "ReleaseIntArrayElements");
}
static void JNICALL ReleaseLongArrayElements(JNIEnv *env, jlongArray a, jlong *e, jint m) {
    (void)env; (void)e; (void)m;
    release(a, K_LONGS, "ReleaseLongArrayElements");
}

static void inject_tick(void);

static void region(jarray a, int kind, jsize start, jsize len, const void *buf, const char *fn) {
    guarded_call(fn);
    inject_tick();
    if (!a || a->kind != kind || start < 0 || len < 0 || start + len > a->n) {
        violation(fn);   /* a JVM throws ArrayIndexOutOfBoundsException here */
        return;
    }
    memcpy((char *)a->data + (size_t)start * esize(kind), buf, (size_t)len * esize(kind));
}
static void JNICALL SetByteArrayRegion(JNIEnv *env, jbyteArray a, jsize s, jsize l, const jbyte *b) {
    (void)env;
    region(a, K_BYTES, s, l, b, "SetByteArrayRegion");
}
static void JNICALL SetIntArrayRegion(JNIEnv *env, jintArray a, jsize s, jsize l, const jint *b) {
    (void)env;
    region(a, K_INTS, s, l, b, "SetIntArrayRegion");
}
static void JNICALL SetDoubleArrayRegion(JNIEnv *env, jdoubleArray a, jsize s, jsize l, const jdouble *b) {
    (void)env;
    region(a, K_DOUBLES, s, l, b, "SetDoubleArrayRegion");
}

static void region_out(jarray a, int kind, jsize start, jsize len, void *buf, const char *fn) {
    guarded_call(fn);
    inject_tick();
    if (!a || a->kind != kind || start < 0 || len < 0 || start + len > a->n) {
        violation(fn);   /* a JVM throws ArrayIndexOutOfBoundsException here */
        return;
    }
    memcpy(buf, (char *)a->data + (size_t)start * esize(kind), (size_t)len * esize(kind));
}
static void JNICALL GetByteArrayRegion(JNIEnv *env, jbyteArray a, jsize s, jsize l, jbyte *b) {
    (void)env;
    region_out(a, K_BYTES, s, l, b, "GetByteArrayRegion");
}
static void JNICALL GetDoubleArrayRegion(JNIEnv *env, jdoubleArray a, jsize s, jsize l, jdouble *b) {
    (void)env;
    region_out(a, K_DOUBLES, s, l, b, "GetDoubleArrayRegion");
}

/* ---- a second Java thread inside a native ----
 * fj_inject arms a one-shot.  At the `after`-th array access (a
 * Get/Set<T>ArrayRegion copy, or a GetPrimitiveArrayCritical: the shim's
 * chunk copies use either) from then on -- inside a chunked native, that is
 * between two chunks of its library call -- a second thread calls the
 * library on the same handle by itself:
 *   op 0: ipls_agg_accumulate(h, p, tgt, src, n, IPLS_HOST_F64)
 *         (another Updater arrival into the same partition),
 *   op 1: ipls_agg_set_weights(h, p, src, n, IPLS_HOST_F64)
 *         (Download_Scheduler.cache_partition on the same partition).
 * The copy that triggered it waits until the thread has started and then
 * `window_ms` more before it returns to the shim.  fj_inject_state: 0 not
 * triggered, 1 the thread's call had returned inside the window (it ran in
 * the middle of the native's work), 2 it was still waiting at the end of
 * the window (ordered after the native's call).  fj_inject_join waits for
 * the thread and returns its library return code.  src stays the caller's. */
struct inject {
    int armed, after, ticks, op, window_ms, state;
    ipls_agg *h;
    int p, tgt;
    const double *src;
    int64_t n;
    pthread_t th;
    int started_th;
    volatile int started, done, rc;
};
static struct inject g_inj;

static void *inject_run(void *arg) {
    struct inject *j = (struct inject *)arg;
    __atomic_store_n(&j->started, 1, __ATOMIC_SEQ_CST);
    int rc = j->op == 0 ? ipls_agg_accumulate(j->h, j->p, j->tgt, j->src, j->n, IPLS_HOST_F64)
                        : ipls_agg_set_weights(j->h, j->p, j->src, j->n, IPLS_HOST_F64);
    j->rc = rc;
    __atomic_store_n(&j->done, 1, __ATOMIC_SEQ_CST);
    return NULL;
}

static void sleep_ms(int ms) {
    struct timespec t = {ms / 1000, (long)(ms % 1000) * 1000000L};
    while (nanosleep(&t, &t) != 0) {}
}

static void inject_tick(void) {
    if (!g_inj.armed || ++g_inj.ticks < g_inj.after) return;
    g_inj.armed = 0;
    if (pthread_create(&g_inj.th, NULL, inject_run, &g_inj) != 0) {
        violation("fj_inject: pthread_create failed");
        return;
    }
    g_inj.started_th = 1;
    while (!__atomic_load_n(&g_inj.started, __ATOMIC_SEQ_CST)) sleep_ms(1);
    sleep_ms(g_inj.window_ms);
    g_inj.state = __atomic_load_n(&g_inj.done, __ATOMIC_SEQ_CST) ? 1 : 2;
}

JNIEXPORT void fj_inject(int op, int after, int window_ms, jlong h, int p, int tgt, const double *src, int64_t n) {
    memset(&g_inj, 0, sizeof g_inj);
    g_inj.op = op;
    g_inj.after = after;
    g_inj.window_ms = window_ms;
    g_inj.h = (ipls_agg *)(intptr_t)h;
    g_inj.p = p;
    g_inj.tgt = tgt;
    g_inj.src = src;
    g_inj.n = n;
    g_inj.armed = 1;
}
JNIEXPORT int fj_inject_state(void) { return g_inj.state; }
JNIEXPORT int fj_inject_join(void) {
    if (!g_inj.started_th) return 1;   /* never triggered */
    pthread_join(g_inj.th, NULL);
    g_inj.started_th = 0;
    return g_inj.rc;
}

/* The shim's report of a call into libipls_agg (IPLS_JNI_CALL_HOOK). */
static int g_library_calls;
JNIEXPORT void fj_library_call(const char *call) {
    ++g_library_calls;
    if (g_critical) {
        char m[160];
        snprintf(m, sizeof m, "critical region held across a library call: %.100s", call);
        violation(m);
    }
}
JNIEXPORT int fj_library_calls(void) { return g_library_calls; }

static void *JNICALL GetPrimitiveArrayCritical(JNIEnv *env, jarray a, jboolean *c) {
    (void)env;
    if (g_critical) violation("GetPrimitiveArrayCritical inside a critical region");
    inject_tick();   /* an array access, like the region copies */
    if (g_exc) violation("GetPrimitiveArrayCritical with an exception pending");
    if (c) *c = JNI_FALSE;
    if (!a || a->kind == K_OBJECTS || a->kind == K_DIRECT || a->kind == K_CLASS) {
        violation("GetPrimitiveArrayCritical on a non-primitive array");
        return NULL;
    }
    ++g_critical;
    return a->data;
}

static void JNICALL ReleasePrimitiveArrayCritical(JNIEnv *env, jarray a, void *p, jint m) {
    (void)env; (void)m;
    if (!a || p != a->data || g_critical <= 0) violation("ReleasePrimitiveArrayCritical");
    --g_critical;
}

static jobject JNICALL NewDirectByteBuffer(JNIEnv *env, void *addr, jlong cap) {
    (void)env;
    guarded_call("NewDirectByteBuffer");
    jobject o = (jobject)calloc(1, sizeof *o);
    o->kind = K_DIRECT;
    o->data = addr;
    o->cap = cap;
    return o;
}

static void *JNICALL GetDirectBufferAddress(JNIEnv *env, jobject b) {
    (void)env;
    guarded_call("GetDirectBufferAddress");
    return (b && b->kind == K_DIRECT) ? b->data : NULL;
}

static jlong JNICALL GetDirectBufferCapacity(JNIEnv *env, jobject b) {
    (void)env;
    guarded_call("GetDirectBufferCapacity");
    return (b && b->kind == K_DIRECT && b->data) ? b->cap : -1;
}

static const struct JNINativeInterface_ g_table = {
    FindClass, ThrowNew, ExceptionCheck, DeleteLocalRef, GetArrayLength, GetObjectArrayElement,
    NewByteArray, NewIntArray, GetByteArrayElements, GetIntArrayElements, GetLongArrayElements,
    ReleaseByteArrayElements, ReleaseIntArrayElements, ReleaseLongArrayElements, SetByteArrayRegion,
    SetIntArrayRegion, SetDoubleArrayRegion, GetByteArrayRegion, GetDoubleArrayRegion, GetPrimitiveArrayCritical,
    ReleasePrimitiveArrayCritical, NewDirectByteBuffer,
    GetDirectBufferAddress, GetDirectBufferCapacity, EnsureLocalCapacity,
};
static JNIEnv g_env = &g_table;

/* ---- the test's side (ctypes) ---- */
JNIEXPORT JNIEnv *fj_env(void) { return &g_env; }

static jobject fj_new(int kind, const void *src, jsize n) {
    jobject o = new_array(kind, n);
    if (src && n > 0) memcpy(o->data, src, (size_t)n * esize(kind));
    return o;
}
JNIEXPORT jobject fj_new_bytes(const void *src, jsize n) { return fj_new(K_BYTES, src, n); }
JNIEXPORT jobject fj_new_ints(const void *src, jsize n) { return fj_new(K_INTS, src, n); }
JNIEXPORT jobject fj_new_longs(const void *src, jsize n) { return fj_new(K_LONGS, src, n); }
JNIEXPORT jobject fj_new_doubles(const void *src, jsize n) { return fj_new(K_DOUBLES, src, n); }
JNIEXPORT jobject fj_new_objects(const jobject *src, jsize n) { return fj_new(K_OBJECTS, src, n); }
JNIEXPORT jobject fj_new_direct(void *addr, jlong cap) {
    jobject o = (jobject)calloc(1, sizeof *o);
    o->kind = K_DIRECT;
    o->data = addr;
    o->cap = cap;
    return o;
}
JNIEXPORT void *fj_data(jobject o) { return o ? o->data : NULL; }
JNIEXPORT jsize fj_len(jobject o) { return o ? o->n : -1; }
JNIEXPORT void fj_free(jobject o) {
    if (!o) return;
    if (o->kind != K_DIRECT && o->kind != K_CLASS) free(o->data);
    free(o);
}
JNIEXPORT const char *fj_exception(void) { return g_exc ? g_exc_class : NULL; }
JNIEXPORT const char *fj_exception_msg(void) { return g_exc_msg; }
JNIEXPORT void fj_clear(void) { g_exc = 0; g_exc_class[0] = 0; g_exc_msg[0] = 0; }
/* rule breaks since the last call, plus regions/elements left open */
JNIEXPORT int fj_violations(void) { return g_violations + (g_critical != 0) + (g_pinned != 0); }
JNIEXPORT const char *fj_last_violation(void) { return g_last_violation; }
JNIEXPORT void fj_reset_violations(void) {
    g_violations = 0; g_critical = 0; g_pinned = 0; g_last_violation[0] = 0;
    g_local_cap = 16; g_locals = 0;   /* a new native frame */
}

/* The critical-region rule itself: a library call reported while a region
 * is open must count as a violation (tests/test_jni.py checks the rule can
 * fire, so its silence on the shim means something).  Returns the
 * violations it recorded. */
JNIEXPORT int fj_selftest_critical_rule(void) {
    jobject a = fj_new_doubles(NULL, 4);
    fj_reset_violations();
    void *p = GetPrimitiveArrayCritical(&g_env, a, NULL);
    fj_library_call("ipls_agg_accumulate(...)");
    ReleasePrimitiveArrayCritical(&g_env, a, p, JNI_ABORT);
    const int v = g_violations;
    fj_reset_violations();
    fj_free(a);
    return v;
}

