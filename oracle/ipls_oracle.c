/*
 * ipls_oracle.c -- CPU restatement of the IPLS aggregation path (TEST
 * INFRASTRUCTURE ONLY; see ipls_oracle.h for the parity status: "parity
 * unpinned" for arithmetic, codec pinned against ETHModel).
 *
 * Build: oracle/Makefile  (gcc -O2 -fno-fast-math -ffp-contract=off -fopenmp)
 */
#include "ipls_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* IPLS.java:1019  int chunk_size = (int)(PeerData._MODEL_SIZE/PeerData._PARTITIONS) + 1;
 * _MODEL_SIZE is a long, _PARTITIONS an int: long division, then (int). */
int64_t ipls_oracle_chunk(int64_t model_size, int32_t n_partitions) {
    return (int64_t)(int32_t)(model_size / n_partitions) + 1;
}

/* IPLS.java:1023-1028 */
int64_t ipls_oracle_partition_len(int64_t model_size, int32_t n_partitions, int32_t i) {
    int64_t c = ipls_oracle_chunk(model_size, n_partitions);
    if ((int64_t)(i + 1) * c > model_size)
        return model_size - (int64_t)i * c + 1;
    return c + 1;
}

/* IPLS.java:1018-1040 */
int ipls_oracle_organize(const double *flat, int64_t n, int64_t model_size,
                         int32_t n_partitions, int32_t i, double *out) {
    int64_t c = ipls_oracle_chunk(model_size, n_partitions);
    int64_t len = ipls_oracle_partition_len(model_size, n_partitions, i);
    int64_t j;
    if (len < 0) return -1;                         /* NegativeArraySizeException */
    for (j = 0; j < len; j++) out[j] = 0.0;         /* new double[] is zeroed */
    for (j = (int64_t)i * c; j < (int64_t)(i + 1) * c && j < n; j++) {
        if (j - (int64_t)i * c >= len) return -1;   /* ArrayIndexOutOfBounds */
        out[j - (int64_t)i * c] = flat[j];          /* Gradients.get(j) (line 1030) */
    }
    if (j - (int64_t)i * c >= len) return -1;       /* count-slot store out of range */
    out[j - (int64_t)i * c] = 1;                    /* line 1033 */
    return 0;
}

/* Updater.java:115-117 -- Aggregated[p][i] = Aggregated[p][i] + Gradient[i] */
void ipls_oracle_fold(double *acc, const double *g, int64_t L) {
    for (int64_t i = 0; i < L; i++) acc[i] = acc[i] + g[i];
}

void ipls_oracle_reduce(double *out, const double *const *bufs, int k, int64_t L, int start_mode) {
    int first = 0;
    if (start_mode == 1) {                           /* fresh accumulator: +0.0 (IPLS.java:1888) */
        for (int64_t i = 0; i < L; i++) out[i] = 0.0;
    } else if (start_mode == 2) {                    /* Aggregation = GetParameters(h0) (DSR:240) */
        if (k <= 0) return;
        memcpy(out, bufs[0], (size_t)L * sizeof(double));
        first = 1;
    }
    for (int j = first; j < k; j++) ipls_oracle_fold(out, bufs[j], L);   /* DSR:242-246 */
}

/* IPLS.java:1255-1270 (secure_ipls == false branch) */
void ipls_oracle_aggregate_partition(double *agg, double *rep, double *w, double *wa, int64_t L) {
    for (int64_t i = 0; i < L; i++) w[i] = agg[i] + rep[i];      /* 1255-1257 */
    for (int64_t i = 0; i < L; i++) {                            /* 1259-1270 */
        wa[i] = w[i];
        agg[i] = 0.0;
        rep[i] = 0.0;
    }
}

/* IPLS.java:1159-1174 */
void ipls_oracle_divide(const double *w, int64_t L, int secure, double *out) {
    double cnt = w[L - 1];
    for (int64_t j = 0; j < L - 1; j++) {
        if (cnt == 0.0) out[j] = w[j];                            /* 1162-1163 */
        else if (secure) out[j] = w[j] / (pow(10, 12) * cnt);     /* 1166-1167 */
        else out[j] = w[j] / cnt;                                 /* 1169-1170 */
    }
}

/* Middleware.java:196-210 */
void ipls_oracle_encode_secure(const double *in, int64_t n, double *out) {
    for (int64_t i = 0; i < n; i++) {
        if (in[i] > 10.0) out[i] = 10 * pow(10, 12);
        else if (in[i] < -10.0) out[i] = -10 * pow(10, 12);
        else out[i] = in[i] * pow(10, 12);
    }
}

static uint64_t load_be64(const uint8_t *b) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | b[i];
    return v;
}
static void store_be64(uint8_t *b, uint64_t v) {
    for (int i = 7; i >= 0; i--) { b[i] = (uint8_t)v; v >>= 8; }
}
static uint32_t load_be32(const uint8_t *b) {
    return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}
static void store_be32(uint8_t *b, uint32_t v) {
    b[0] = (uint8_t)(v >> 24); b[1] = (uint8_t)(v >> 16); b[2] = (uint8_t)(v >> 8); b[3] = (uint8_t)v;
}

/* MyIPFSClass.java:449-452  arr[i] = buff.getDouble() */
void ipls_oracle_be_decode(const uint8_t *bytes, int64_t n, double *out) {
    for (int64_t i = 0; i < n; i++) {
        uint64_t v = load_be64(bytes + 8 * i);
        memcpy(&out[i], &v, 8);
    }
}

/* MyIPFSClass.java:107-109  writeBuffer.putDouble(Weights[i])  (raw bits) */
void ipls_oracle_be_encode(const double *in, int64_t n, uint8_t *bytes) {
    for (int64_t i = 0; i < n; i++) {
        uint64_t v;
        memcpy(&v, &in[i], 8);
        store_be64(bytes + 8 * i, v);
    }
}

/* Middleware.java:167-169  out.writeDouble(updates.get(i)) -> doubleToLongBits */
void ipls_oracle_be_encode_canonical(const double *in, int64_t n, uint8_t *bytes) {
    for (int64_t i = 0; i < n; i++) {
        uint64_t v;
        if (in[i] != in[i]) v = 0x7ff8000000000000ULL;
        else memcpy(&v, &in[i], 8);
        store_be64(bytes + 8 * i, v);
    }
}

/* MyIPFSClass.java:990-1017 */
int64_t ipls_oracle_frame_encode(const double *g, int32_t n, int32_t a, int32_t b,
                                 int16_t pid, const uint8_t *origin, int32_t origin_len,
                                 uint8_t *out) {
    out[0] = (uint8_t)((uint16_t)pid >> 8);
    out[1] = (uint8_t)pid;                               /* putShort(0,pid)      996 */
    store_be32(out + 2, (uint32_t)n);                    /* putInt(2, n)         997 */
    store_be32(out + 6, (uint32_t)a);                    /* putInt(6, Partition) 998 */
    store_be32(out + 10, (uint32_t)b);                   /* putInt(10, iteration) 999 */
    ipls_oracle_be_encode(g, n, out + 14);               /* putDouble(14+8i)  1000-1002 */
    memcpy(out + 14 + 8 * (int64_t)n, origin, (size_t)origin_len);   /* 1006-1013 */
    return 14 + 8 * (int64_t)n + origin_len;
}

/* MyIPFSClass.java:1016 Base64.getUrlEncoder().encodeToString: every 3 input
 * bytes -> 4 chars of A-Z a-z 0-9 - _, the last group padded with '=' */
int64_t ipls_oracle_b64url_encode(const uint8_t *in, int64_t n, uint8_t *out) {
    static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
    int64_t o = 0;
    for (int64_t i = 0; i < n; i += 3) {
        const int64_t r = n - i < 3 ? n - i : 3;
        uint32_t v = (uint32_t)in[i] << 16;
        if (r > 1) v |= (uint32_t)in[i + 1] << 8;
        if (r > 2) v |= in[i + 2];
        out[o++] = (uint8_t)A[(v >> 18) & 63];
        out[o++] = (uint8_t)A[(v >> 12) & 63];
        out[o++] = r > 1 ? (uint8_t)A[(v >> 6) & 63] : '=';
        out[o++] = r > 2 ? (uint8_t)A[v & 63] : '=';
    }
    return o;
}

/* MyIPFSClass.java:1437-1459 (GET_GRADIENTS) / 1462-1481 (Get_Replica_Model) */
int32_t ipls_oracle_frame_decode(const uint8_t *frame, int64_t len, int16_t *pid,
                                 int32_t *a, int32_t *b, double *g,
                                 int64_t *origin_off) {
    if (len < 14) return -1;
    *pid = (int16_t)(((uint16_t)frame[0] << 8) | frame[1]);   /* IPLS.java:405 getShort */
    int32_t n = (int32_t)load_be32(frame + 2);
    *a = (int32_t)load_be32(frame + 6);
    *b = (int32_t)load_be32(frame + 10);
    if (n < 0 || 14 + 8 * (int64_t)n > len) return -1;       /* BufferUnderflowException */
    if (g) ipls_oracle_be_decode(frame + 14, n, g);
    if (origin_off) *origin_off = 14 + 8 * (int64_t)n;
    return n;
}

/* ---- synthetic workload: SURVEY.md §8(d) ---- */
uint64_t ipls_oracle_splitmix64(uint64_t v) {
    uint64_t z = v + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

double ipls_oracle_synth_value(uint64_t seed, int32_t p, int32_t k, int64_t i) {
    uint64_t key = seed ^ ((uint64_t)(uint32_t)p << 40) ^ ((uint64_t)(uint32_t)k << 32) ^ (uint64_t)i;
    double u = (double)(ipls_oracle_splitmix64(key) >> 11) * 0x1.0p-53;
    double t = 2.0 * u;
    t = t - 1.0;
    return t * 1e-2;
}

void ipls_oracle_synth_fill(double *out, int64_t L, uint64_t seed, int32_t p, int32_t k) {
    for (int64_t i = 0; i + 1 < L; i++) out[i] = ipls_oracle_synth_value(seed, p, k, i);
    if (L > 0) out[L - 1] = 1.0;
}

static inline uint64_t checksum_term(double x, int64_t i) {
    uint64_t b;
    memcpy(&b, &x, 8);
    return ipls_oracle_splitmix64(b + (uint64_t)i * 0x9E3779B97F4A7C15ULL);
}

uint64_t ipls_oracle_checksum(const double *x, int64_t n) {
    uint64_t s = 0;
    for (int64_t i = 0; i < n; i++) s += checksum_term(x[i], i);
    return s;
}

uint64_t ipls_oracle_synth_sum_checksum(uint64_t seed, int32_t p, int32_t k, int64_t L) {
    uint64_t s = 0;
#pragma omp parallel for reduction(+ : s) schedule(static)
    for (int64_t i = 0; i < L; i++) {
        double acc = 0.0;                                    /* ZERO start */
        for (int32_t j = 0; j < k; j++) {
            double g = (i == L - 1) ? 1.0 : ipls_oracle_synth_value(seed, p, j, i);
            acc = acc + g;                                   /* Updater.java:116 */
        }
        s += checksum_term(acc, i);
    }
    return s;
}

/* Checksum of W = AGG + REP when partition p's k peers are split over two
 * aggregators: the owner folds peers [0, k_own) into Aggregated_Gradients
 * (Updater.java:115-117), the replica folds peers [k_own, k) into its own
 * partial, which lands in the owner's fresh Replicas_Gradients
 * (Updater.java:40-44: +0.0 + R), and AggregatePartition adds the two
 * (IPLS.java:1256). */
uint64_t ipls_oracle_synth_replica_checksum(uint64_t seed, int32_t p, int32_t k, int32_t k_own, int64_t L) {
    uint64_t s = 0;
#pragma omp parallel for reduction(+ : s) schedule(static)
    for (int64_t i = 0; i < L; i++) {
        double own = 0.0, part = 0.0;
        for (int32_t j = 0; j < k; j++) {
            double g = (i == L - 1) ? 1.0 : ipls_oracle_synth_value(seed, p, j, i);
            if (j < k_own) own = own + g;
            else part = part + g;
        }
        double rep = 0.0;
        rep = rep + part;
        s += checksum_term(own + rep, i);
    }
    return s;
}

/* Checksum of the averaged output of the same fold (GetPartitions divide,
 * IPLS.java:1159-1174) over i < L-1, element index i: cnt = S[L-1] (the fold
 * of k count slots), out = cnt == 0 ? S[i] : S[i] / (secure ? 1e12*cnt : cnt). */
uint64_t ipls_oracle_synth_avg_checksum(uint64_t seed, int32_t p, int32_t k, int64_t L, int32_t secure) {
    double cnt = 0.0;
    for (int32_t j = 0; j < k; j++) cnt = cnt + 1.0;
    const double den = secure ? 1e12 * cnt : cnt;
    uint64_t s = 0;
#pragma omp parallel for reduction(+ : s) schedule(static)
    for (int64_t i = 0; i < L - 1; i++) {
        double acc = 0.0;
        for (int32_t j = 0; j < k; j++) acc = acc + ipls_oracle_synth_value(seed, p, j, i);
        s += checksum_term(cnt == 0.0 ? acc : acc / den, i);
    }
    return s;
}

/* Updater.run + _Update for k indirect-mode buckets (Updater.java:162-187,
 * 115-117): decode into the reused buffer, then fold. */
void ipls_oracle_updater_loop(double *agg, const uint8_t *const *be_bufs, int k,
                              int64_t L, double *scratch) {
    for (int j = 0; j < k; j++) {
        ipls_oracle_be_decode(be_bufs[j], L, scratch);       /* GetParameters(Hash,Gradient_Buff) */
        for (int64_t i = 0; i < L; i++) agg[i] = agg[i] + scratch[i];
    }
}

/* Partition-parallel variant of the Updater loop (CPU baseline, N threads):
 * n_parts independent partitions, each folded by one thread exactly as the
 * single-thread loop does (own accumulator + reused decode buffer).  All
 * partitions read the same k BE buckets (a bounded input sample).  Returns
 * the number of threads used. */
int ipls_oracle_updater_loop_parts(int n_parts, const uint8_t *const *be_bufs, int k, int64_t L,
                                   double *agg0) {
    int threads = 1;
#pragma omp parallel
    {
#ifdef _OPENMP
#pragma omp single
        threads = omp_get_num_threads();
#endif
        double *agg = (double *)malloc((size_t)L * sizeof(double));
        double *scratch = (double *)malloc((size_t)L * sizeof(double));
#pragma omp for schedule(dynamic, 1)
        for (int q = 0; q < n_parts; q++) {
            memset(agg, 0, (size_t)L * sizeof(double));
            ipls_oracle_updater_loop(agg, be_bufs, k, L, scratch);
            if (q == 0 && agg0) memcpy(agg0, agg, (size_t)L * sizeof(double));
        }
        free(scratch);
        free(agg);
    }
    return threads;
}

/* BE byte images (the update_file / `ipfs cat` format) of the synthetic
 * buckets (p, j), p < n_parts, j < k: outs[p*k + j] receives 8*L bytes.
 * Element values as ipls_oracle_synth_fill; OpenMP over the buckets. */
void ipls_oracle_synth_be_buckets(uint8_t *const *outs, int n_parts, int k, int64_t L, uint64_t seed) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int b = 0; b < n_parts * k; b++) {
        const int p = b / k, j = b % k;
        uint8_t *o = outs[b];
        for (int64_t i = 0; i < L; i++) {
            const double x = (i == L - 1) ? 1.0 : ipls_oracle_synth_value(seed, p, j, i);
            uint64_t u;
            memcpy(&u, &x, 8);
            for (int c = 0; c < 8; c++) o[8 * i + c] = (uint8_t)(u >> (56 - 8 * c));
        }
    }
}

/* CPU baseline, N threads: n_parts partitions, each with
 * its OWN k buckets (be_bufs[p*k + j]), each folded by one thread exactly as
 * the single Updater thread folds (decode into a reused buffer, then
 * Agg[i] = Agg[i] + g[i]; Updater.java:162-187, 115-117), `passes` times.
 * threads > 0 sets the team size.  Returns the threads used; agg0 (nullable)
 * receives partition 0's sum. */
int ipls_oracle_updater_loop_partitions(int n_parts, const uint8_t *const *be_bufs, int k, int64_t L, int passes,
                                        int threads, double *agg0) {
    int used = 1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
    {
#ifdef _OPENMP
#pragma omp single
        used = omp_get_num_threads();
#endif
        double *agg = (double *)malloc((size_t)L * sizeof(double));
        double *scratch = (double *)malloc((size_t)L * sizeof(double));
        for (int r = 0; r < passes; r++) {
#pragma omp for schedule(dynamic, 1)
            for (int q = 0; q < n_parts; q++) {
                memset(agg, 0, (size_t)L * sizeof(double));
                ipls_oracle_updater_loop(agg, be_bufs + (size_t)q * k, k, L, scratch);
                if (q == 0 && r == 0 && agg0) memcpy(agg0, agg, (size_t)L * sizeof(double));
            }
        }
        free(scratch);
        free(agg);
    }
    return used;
}
