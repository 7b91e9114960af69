/*
 * ipls_oracle.h -- CPU restatement of the IPLS aggregation path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (ipls-java-api_amd/) may
 * include, link or call this.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, as the checker / CPU baseline.
 *
 * PARITY STATUS: "parity unpinned" for the arithmetic.  The reference is Java
 * with no JDK in this image and ships no test, fixture or golden vector for
 * this path.  Every function below restates the Java
 * loop it cites line by line; Java `double` + and / are IEEE-754 binary64
 * round-to-nearest (JLS §15.17/15.18, SSE2 on x86-64), which C `double` on
 * x86-64 with -ffp-contract=off -fno-fast-math reproduces bit for bit.  The
 * byte codecs are pinned against MNIST_Partitioned_Dataset/ETHModel, a file
 * Java wrote with DataOutputStream.writeDouble (big-endian).
 *
 * All citations are relative to the reference root.
 */
#ifndef IPLS_ORACLE_H
#define IPLS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* chunk_size = (int)(MODEL_SIZE / PARTITIONS) + 1      IPLS.java:1019 */
int64_t ipls_oracle_chunk(int64_t model_size, int32_t n_partitions);

/* Length of partition i incl. the count slot (IPLS.java:1023-1028).
 * Returns a value < 1 when Java would throw NegativeArraySizeException (or
 * allocate a 0-length array and then throw on the count-slot store). */
int64_t ipls_oracle_partition_len(int64_t model_size, int32_t n_partitions, int32_t i);

/* OrganizeGradients (IPLS.java:1018-1040) for one partition: copies
 * flat[i*chunk .. min((i+1)*chunk, n)) and stores 1.0 at the index the loop
 * stopped at.  out must hold partition_len doubles; unwritten slots are 0.0
 * (Java zero-initialises new double[]).  Returns 0 or -1 on Java exception. */
int ipls_oracle_organize(const double *flat, int64_t n, int64_t model_size,
                         int32_t n_partitions, int32_t i, double *out);

/* acc[j] = acc[j] + g[j], j < L   (Updater.java:115-117, IPLS.java:1740,
 * Updater.java:43, IPLS.java:1227, Download_Scheduler.java:258) */
void ipls_oracle_fold(double *acc, const double *g, int64_t L);

/* Fixed-order fold of k buckets into out, start mode:
 *   0 ACCUM: out keeps its value and each bucket is folded in (Updater arrival order)
 *   1 ZERO : out = +0.0 first (fresh accumulator, IPLS.java:1888,1896,1268)
 *   2 FIRST: out = b0, then b1.. folded (Decentralized_Storage_Receiver.java:240-246,
 *            Download_Scheduler.java:262-265)                                    */
void ipls_oracle_reduce(double *out, const double *const *bufs, int k, int64_t L, int start_mode);

/* AggregatePartition (IPLS.java:1248-1274), non-secure branch:
 *   W[i] = AGG[i] + REP[i]; WA[i] = W[i]; AGG[i] = REP[i] = 0.0            */
void ipls_oracle_aggregate_partition(double *agg, double *rep, double *w, double *wa, int64_t L);

/* GetPartitions divide (IPLS.java:1159-1174) for one partition of length L:
 *   out[j] = W[L-1] == 0.0 ? W[j] : W[j] / W[L-1]         (j < L-1)
 *   secure: W[j] / (Math.pow(10,12) * W[L-1])                             */
void ipls_oracle_divide(const double *w, int64_t L, int secure, double *out);

/* Middleware.Encode (Middleware.java:196-210): clip to +-10, scale by 1e12. */
void ipls_oracle_encode_secure(const double *in, int64_t n, double *out);

/* ByteBuffer.getDouble loop (MyIPFSClass.java:444-455): n BE doubles. */
void ipls_oracle_be_decode(const uint8_t *bytes, int64_t n, double *out);

/* ByteBuffer.putDouble loop (MyIPFSClass.java:105-116): raw bits, BE. */
void ipls_oracle_be_encode(const double *in, int64_t n, uint8_t *bytes);

/* DataOutputStream.writeDouble loop (Middleware.java:164-170): BE with NaN
 * canonicalised to 0x7ff8000000000000 (Double.doubleToLongBits).          */
void ipls_oracle_be_encode_canonical(const double *in, int64_t n, uint8_t *bytes);

/* Marshall_Packet(double[],origin,partition,iteration,pid) before base64
 * (MyIPFSClass.java:990-1017).  Frame = [i16 pid][i32 n][i32 a][i32 b]
 * [n f64 BE][origin bytes].  Returns bytes written (14 + 8n + origin_len). */
int64_t ipls_oracle_frame_encode(const double *g, int32_t n, int32_t a, int32_t b,
                                 int16_t pid, const uint8_t *origin, int32_t origin_len,
                                 uint8_t *out);

/* java.util.Base64.getUrlEncoder().encodeToString(in) (MyIPFSClass.java:
 * 1016): RFC 4648 URL-safe alphabet, '=' padding.  Returns chars written
 * (4 * ceil(n / 3)). */
int64_t ipls_oracle_b64url_encode(const uint8_t *in, int64_t n, uint8_t *out);

/* GET_GRADIENTS / Get_Replica_Model after the pid short (MyIPFSClass.java:
 * 1437-1481).  Parses header, decodes n doubles into g (may be NULL).
 * Returns n, or -1 on a short buffer (BufferUnderflowException). */
int32_t ipls_oracle_frame_decode(const uint8_t *frame, int64_t len, int16_t *pid,
                                 int32_t *a, int32_t *b, double *g,
                                 int64_t *origin_off);

/* ---- synthetic workload ---- */
uint64_t ipls_oracle_splitmix64(uint64_t v);
/* x = (2u-1)*1e-2, u = (splitmix64(seed ^ p<<40 ^ k<<32 ^ i) >> 11) * 2^-53;
 * element L-1 is the count slot 1.0. */
double ipls_oracle_synth_value(uint64_t seed, int32_t p, int32_t k, int64_t i);
void ipls_oracle_synth_fill(double *out, int64_t L, uint64_t seed, int32_t p, int32_t k);

/* Order-independent checksum of a double vector:
 *   sum_i splitmix64(bits(x_i) + i * 0x9E3779B97F4A7C15)  (mod 2^64)       */
uint64_t ipls_oracle_checksum(const double *x, int64_t n);

/* Full-size property: per-partition checksum of the ZERO-start fixed-order
 * sum of k synthetic buckets of length L, generated on the fly (no input
 * memory).  Multi-threaded over elements (OpenMP) -- the per-element fold
 * order is unchanged, so this is still the reference's arithmetic. */
uint64_t ipls_oracle_synth_sum_checksum(uint64_t seed, int32_t p, int32_t k, int64_t L);
uint64_t ipls_oracle_synth_avg_checksum(uint64_t seed, int32_t p, int32_t k, int64_t L, int32_t secure);
/* W = AGG(peers [0,k_own)) + (+0.0 + partial(peers [k_own,k))): one replica
 * aggregator's partial folded into the owner's REP, then AggregatePartition. */
uint64_t ipls_oracle_synth_replica_checksum(uint64_t seed, int32_t p, int32_t k, int32_t k_own, int64_t L);

/* CPU baseline: the reference's Updater loop over k BE byte buckets,
 * 1 thread: decode each bucket into a reused double[] (Updater.java:162,177
 * + MyIPFSClass.java:444-455), then Agg[i] = Agg[i] + g[i] (115-117). */
void ipls_oracle_updater_loop(double *agg, const uint8_t *const *be_bufs, int k,
                              int64_t L, double *scratch);

/* N-thread, partition-parallel variant (OpenMP); returns threads used. */
int ipls_oracle_updater_loop_parts(int n_parts, const uint8_t *const *be_bufs, int k, int64_t L,
                                   double *agg0);
/* BE images of the synthetic buckets (p, j) for p < n_parts, j < k. */
void ipls_oracle_synth_be_buckets(uint8_t *const *outs, int n_parts, int k, int64_t L, uint64_t seed);
/* N-thread baseline over n_parts partitions with their own k buckets each. */
int ipls_oracle_updater_loop_partitions(int n_parts, const uint8_t *const *be_bufs, int k, int64_t L, int passes,
                                        int threads, double *agg0);

#ifdef __cplusplus
}
#endif
#endif
