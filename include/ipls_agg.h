/*
 * ipls_agg.h -- C-ABI of the MI355X-native IPLS gradient-partition aggregator.
 *
 * Drop-in boundary for the reference's aggregation path.
 * The reference has no FFI: its reduce loops are inlined into static-state
 * Java methods.  Each entry point below replaces the body of one of those
 * loops; the Java callers keep their signatures and call through the JNI
 * shim shown in INTEGRATION.md (1:1 mapping, no torch / HIP types here).
 *
 * Reference citations are relative to /root/reference/src/main/java/.
 *
 * Conventions
 *  - Every function returns IPLS_OK (0) or a negative IPLS_E_* code and never
 *    aborts; ipls_agg_last_error() gives the message (Java code catches and
 *    prints exceptions at the same places, e.g. Updater.java:213-215).
 *  - The caller owns host buffers for the duration of the call only: a call
 *    that reads or writes host memory has finished with it when it returns.
 *  - Calls with only device-resident operands are stream-ordered on the
 *    handle's HIP stream and may return before the GPU finishes; use
 *    ipls_agg_sync() before reading device results from another stream.
 *    The handle's stream is non-blocking: device operands written on another
 *    stream (the null stream included) must be complete, or ordered before
 *    the call by an event the handle's stream waits on (ipls_agg_stream /
 *    ipls_agg_partition_device give the stream).
 *  - A handle is internally serialised (one mutex per GPU shard): it may be
 *    called from the Updater thread and the daemon thread concurrently, as the
 *    Java code does under PeerData.mtx (PeerData.java:27).  Each CALL is one
 *    ordered unit: calls on one partition take effect in call order -- the
 *    reference's arrival order.  A SEQUENCE of calls is not a unit: another
 *    thread's call may land between two calls of one thread.  So what one
 *    Java-side step must do atomically is one call here: a whole arriving
 *    bucket (ipls_agg_accumulate, or ipls_agg_accumulate_chunked for a
 *    caller that produces the bucket chunk by chunk), AggregatePartition plus
 *    its commit_update bytes (ipls_agg_finalize, ipls_agg_finalize_chunked).
 *    A chunked call takes effect, as one unit, at one instant: an
 *    accumulate_chunked when its last chunk has landed on the GPU (as
 *    Middleware's Deserialize reads the whole stream before UpdateModel takes
 *    PeerData.mtx, Middleware.java:224, 246), a finalize_chunked /
 *    get_partitions(_wire)_chunked when it takes its snapshot, before the
 *    first chunk is delivered.  No shard lock is held while the caller's
 *    source or sink runs, so a blocking one (a socket) holds up nobody else.
 *    ipls_agg_accumulate_range / ipls_agg_read_range are single calls too:
 *    a caller that splits one arrival into ranges holds its own lock across
 *    them (PeerData.mtx, Updater.java:72-149) or gets a mixed order.
 *  - Every ipls_agg_* call returns with the calling thread's current HIP
 *    device unchanged, whichever GPUs the handle's shards live on.
 *  - Arithmetic is IEEE binary64 with no contraction and no reassociation:
 *    each element is folded over the peers in the order given, starting from
 *    +0.0 (or from the first bucket), so results are bit-identical to the
 *    Java loops on the same inputs.
 */
#ifndef IPLS_AGG_H
#define IPLS_AGG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IPLS_AGG_ABI_VERSION 4

/* ---- error codes (Java exception the reference would raise) ---- */
#define IPLS_OK           0
#define IPLS_E_INVAL     -1  /* bad argument / null handle                         */
#define IPLS_E_RANGE     -2  /* partition index or length out of range
                                (ArrayIndexOutOfBoundsException, Updater.java:115) */
#define IPLS_E_NEGSIZE   -3  /* chunk rule gives a partition of length < 1
                                (NegativeArraySizeException, IPLS.java:1024,1863)  */
#define IPLS_E_NOMEM     -4  /* device or pinned-host allocation failed             */
#define IPLS_E_DEVICE    -5  /* HIP runtime / kernel launch error                   */
#define IPLS_E_FORMAT    -6  /* malformed frame or byte length
                                (BufferUnderflowException, MyIPFSClass.java:1444)  */
#define IPLS_E_NODEV     -7  /* no usable GPU                                       */

/* ---- accumulator targets (PeerData.java:137,144,149,189) ---- */
#define IPLS_TGT_AGG      0  /* PeerData.Aggregated_Gradients[p]  */
#define IPLS_TGT_REP      1  /* PeerData.Replicas_Gradients[p]    */
#define IPLS_TGT_WEIGHTS  2  /* PeerData.Weights[p]               */
#define IPLS_TGT_WADDR    3  /* PeerData.Weight_Address[p]        */
#define IPLS_TGT_FUTURE   4  /* PeerData.Aggregated_Gradients_from_future[p]
                                (Updater.java:99-101: a client's bucket for a
                                later iteration) */

/* ---- operand kinds ---- */
#define IPLS_HOST_F64     0  /* host double[] (native byte order)                          */
#define IPLS_HOST_BE      1  /* host byte[] of big-endian doubles: update_file / GetParameters
                                format (MyIPFSClass.java:105-116, 444-455); n = #doubles     */
#define IPLS_HOST_FRAME   2  /* host byte[] pubsub frame after base64 (Marshall_Packet,
                                MyIPFSClass.java:990-1017); n = frame byte length           */
#define IPLS_DEV_F64      3  /* device double*                                               */
#define IPLS_DEV_BE       4  /* device bytes, big-endian doubles, 8-byte aligned             */
#define IPLS_HOST_BE_CANON 5 /* output only: BE with NaN canonicalised, DataOutputStream
                                .writeDouble (Middleware.java:164-170)                      */
#define IPLS_HOST_PAIR    6  /* host byte[] of a Java-serialised org.javatuples.Pair<Integer,
                                double[]> partial update (MyIPFSClass.java:160-166, read by
                                Download_Partial_Updates :326-338); n = byte length         */
#define IPLS_HOST_TEXT    7  /* output only: host bytes of a base64url pubsub text
                                (Marshall_Packet's String, MyIPFSClass.java:1016)           */
#define IPLS_DEV_TEXT     8  /* output only: the same text in device memory                  */

/* ---- fold start modes ---- */
#define IPLS_START_ACCUM  0  /* fold into the target's current value (Updater arrival fold)     */
#define IPLS_START_ZERO   1  /* target = +0.0 first (fresh accumulator, IPLS.java:1888,1268)    */
#define IPLS_START_FIRST  2  /* target = bucket 0, then fold the rest
                                (Decentralized_Storage_Receiver.java:240-246)                   */

#define IPLS_ALL_PARTITIONS (-1)

typedef struct ipls_agg ipls_agg;

typedef struct ipls_agg_cfg {
    int64_t model_size;          /* PeerData._MODEL_SIZE; > 0 selects the reference chunk rule   */
    int32_t n_partitions;        /* -pa  (Middleware.java:35, PeerData._PARTITIONS)              */
    int32_t max_peers;           /* -n   (Middleware.java:44); sizes host staging, may be 0       */
    int32_t partial_aggregation; /* -aggr (Middleware.java:57); informational                     */
    int32_t secure;              /* PeerData.secure_ipls (PeerData.java:62): /1e12 in the divide  */
    int32_t device;              /* HIP device ordinal                                           */
    int32_t flags;               /* reserved, must be 0                                          */
    int64_t bucket_len;          /* model_size == 0: every partition has this length incl. the
                                    count slot (synthetic configs, SURVEY.md §8 notation)        */
    /* ABI 2: the devices of a multi-GPU handle (SURVEY.md §8(b) "device ids", §8(e)).
     * n_devices == 0 (or devices == NULL): one device, `device`.  Otherwise the
     * -pa partitions are sharded over devices[0..n_devices) in contiguous blocks,
     * partition p on shard p / ceil(P / n_devices) (ipls_shard_plan), each shard
     * with its own HIP stream and accumulator arena on its device; a device may
     * appear more than once (shards sharing one GPU).  The list is copied. */
    const int32_t *devices;
    int32_t n_devices;
    int32_t reserved;            /* must be 0 */
} ipls_agg_cfg;

/* Caller callbacks of the chunked calls (ipls_agg_get_partitions_chunked,
 * ipls_agg_finalize_chunked: sink; ipls_agg_accumulate_chunked: source).
 * They run on the calling thread, inside the call, with no library lock held:
 * they may block (a socket recv/send -- bound it with a timeout, the call
 * waits for its callback) and may call into the same handle. */
typedef int (*ipls_chunk_sink)(void *ctx, const double *values, int64_t offset, int64_t n);
typedef int (*ipls_chunk_source)(void *ctx, void *dst, int64_t offset, int64_t n);

/* ABI version of the loaded library (IPLS_AGG_ABI_VERSION). */
int ipls_agg_abi_version(void);

/* Allocate the per-partition accumulators on the device, all zero.
 * Replaces IPLS.init's InitializeWeights() (IPLS.java:1860-1878). */
int ipls_agg_open(const ipls_agg_cfg *cfg, ipls_agg **out);

/* Free everything.  NULL is accepted. */
int ipls_agg_close(ipls_agg *h);

/* Message of the last failure on h (h == NULL: last failure of this thread).
 * Right after a call fails, ipls_agg_last_error(NULL) is that call's message
 * even while other threads use the same handle.  The string belongs to the
 * calling thread and stays valid until its next ipls_agg_last_error call. */
const char *ipls_agg_last_error(const ipls_agg *h);

/* Partition length incl. the count slot: IPLS.java:1019-1028. */
int ipls_agg_partition_len(const ipls_agg *h, int p, int64_t *len);

/* Offset of partition p's first value in the flat model (p * chunk). */
int ipls_agg_partition_offset(const ipls_agg *h, int p, int64_t *off);
/* Values of the flat model: model_size (sum of L_p - 1), what GetPartitions
 * writes and OrganizeGradients reads. */
int ipls_agg_flat_size(const ipls_agg *h, int64_t *n);

/* InitializeWeights(List<Double> Model), IPLS.java:1880-1901: Weights and
 * Weight_Address get the model values with count slot 0.0; AGG, REP = 0.
 * src: HOST_F64 / HOST_BE (read_file format, IPLS.java:2000-2008) / DEV_*. */
int ipls_agg_load_model(ipls_agg *h, const void *src, int64_t n, int src_kind);

/* OrganizeGradients (IPLS.java:1018-1040) for partition p: dst gets
 * double[L_p] with the count slot 1.0.  dst_kind: HOST_F64, HOST_BE, DEV_F64,
 * DEV_BE.  n is the length of the flat gradient vector. */
int ipls_agg_split(ipls_agg *h, const void *flat, int64_t n, int src_kind,
                   int p, void *dst, int dst_kind);

/* UpdateGradient's own-partition accumulate (IPLS.java:1737-1743):
 * for every p in owned[0..n_owned): AGG[p] = AGG[p] + OrganizeGradients(flat)[p].
 * flat == NULL is the "did not train in time" case (Gradients == null): no-op. */
int ipls_agg_update_gradient(ipls_agg *h, const void *flat, int64_t n, int src_kind,
                             const int32_t *owned, int n_owned);

/* Updater._Update for one arriving bucket (Updater.java:36-48 REP branch,
 * 74-137 AGG branches): target[p][i] = target[p][i] + g[i], i < L_p.
 * n = #doubles (F64/BE kinds) or frame byte length (FRAME kind; the frame's
 * n field must be >= L_p; PAIR kind: its double[] must be >= L_p).  Returns IPLS_E_RANGE when the bucket is shorter
 * than L_p.  Also Collect_Replicas (IPLS.java:1217-1241) with target REP. */
int ipls_agg_accumulate(ipls_agg *h, int p, int target, const void *src, int64_t n,
                        int src_kind);

/* Asynchronous form of ipls_agg_accumulate (Updater._Update without waiting,
 * Updater.java:115-117); returns at once with *ticket.
 *  - DEV_F64 / DEV_BE (8-B aligned): the bucket is queued, not read.  Each
 *    partition's queued buckets are folded together in one launch, in call
 *    order (bit-identical to folding them one by one), when the queues fill
 *    (ipls_agg_set_coalesce, default 32), at ipls_agg_wait, or at the first
 *    other call on the handle.
 *  - pinned host memory (ipls_host_alloc, 16-B aligned, HOST_F64/HOST_BE):
 *    the fold is queued at once and reads the bucket over PCIe, so the next
 *    `ipfs cat` can fill another buffer meanwhile.
 *  - other sources run synchronously (ticket already done).
 * The caller keeps the bucket untouched (and allocated) until
 * ipls_agg_wait(h, ticket) -- or any other call on the handle -- returns.
 * Folds apply in call order. */
int ipls_agg_accumulate_async(ipls_agg *h, int p, int target, const void *src, int64_t n,
                              int src_kind, uint64_t *ticket);

/* One range of one arrival, asynchronous: src[0..n) is folded into
 * target[offset .. offset+n) of partition p (Agg[i] = Agg[i] + g[i],
 * Updater.java:115-117, for those i), reading pinned host memory
 * (ipls_host_alloc; HOST_F64 or HOST_BE) over PCIe with no staging copy.
 * offset must be even and src 16-B aligned.  A bucket folded as any set of
 * ranges that covers [0, L_p) once gets the bits of the whole-bucket fold:
 * every element is added once, in call order.  This lets a caller that must
 * first copy the bucket (the JNI shim's double[] natives) overlap that copy
 * with the fold, chunk by chunk.  Keep src untouched until
 * ipls_agg_wait(h, *ticket) returns.  IPLS_E_RANGE outside [0, L_p);
 * IPLS_E_INVAL for other memory or a misaligned range.
 * Each range is its own call: another thread's fold into the same target
 * can land between two ranges of one arrival, and the elements of the
 * earlier ranges then see a different order than those of the later ones.
 * Hold a lock across the ranges, or use ipls_agg_accumulate_chunked. */
int ipls_agg_accumulate_range(ipls_agg *h, int p, int target, const void *src, int64_t offset, int64_t n,
                              int src_kind, uint64_t *ticket);

/* One arriving bucket that the caller produces chunk by chunk, as ONE call
 * (Updater._Update's whole-bucket fold under PeerData.mtx, Updater.java:72-149,
 * 115-117): the library calls source(ctx, dst, offset, n) on the calling
 * thread for consecutive chunks of `chunk` values (even, >= 2) covering
 * [0, L_p); the source writes the bucket's values [offset, offset + n) into
 * dst -- 8 * n bytes of pinned staging owned by the library, native doubles
 * (HOST_F64) or big-endian bytes (HOST_BE) -- and returns 0.  Each chunk is
 * sent to the GPU while the source fills the next one; once every chunk has
 * landed, the bucket is folded into target[p] in one launch.
 *  - n is the caller's bucket length: n < L_p is IPLS_E_RANGE before any
 *    source call (the ArrayIndexOutOfBoundsException of Updater.java:115);
 *    values past L_p are never asked for.
 *  - All or nothing: a non-zero source return stops the call with
 *    IPLS_E_INVAL and nothing folded.
 *  - The chunks land in staging of this call's own, with no lock held; the
 *    shard's lock is taken once every chunk has landed, for the fold alone.
 *    So the bucket takes effect as one unit at that instant (a fold another
 *    thread makes into the same target while the source is still producing
 *    lands before it): the bits are those of ipls_agg_accumulate on the whole
 *    bucket at that point of the call order.  A slow source holds up no other
 *    caller of the shard.
 * The JNI shim's accumulate(double[]) source is GetDoubleArrayRegion; the
 * Middleware servers' is a socket recv. */
int ipls_agg_accumulate_chunked(ipls_agg *h, int p, int target, int64_t n, int src_kind, int64_t chunk,
                                ipls_chunk_source source, void *ctx);

/* The reverse of a ranged fold, asynchronous: target[offset .. offset+n) of
 * partition p is copied into pinned host memory dst (ipls_host_alloc), as
 * doubles (HOST_F64) or as big-endian bytes (HOST_BE: putDouble order, what
 * update_file writes, MyIPFSClass.java:105-116).  dst is complete when
 * ipls_agg_wait(h, *ticket) returns.  With ipls_agg_finalize(h, p, NULL, ...)
 * first, reading IPLS_TGT_WEIGHTS in ranges gives the commit_update bytes
 * chunk by chunk -- but as separate calls, so a set_weights or a finalize
 * from another thread between them tears the bytes: ipls_agg_finalize_chunked
 * is the one-call form.  IPLS_E_RANGE outside [0, L_p); IPLS_E_INVAL for
 * other memory. */
int ipls_agg_read_range(ipls_agg *h, int p, int target, void *dst, int64_t offset, int64_t n, int dst_kind,
                        uint64_t *ticket);

/* Wait until fold `ticket` (and every fold queued before it) has finished. */
int ipls_agg_wait(ipls_agg *h, uint64_t ticket);

/* Launch the folds of every queued asynchronous device bucket now, without
 * waiting for them (for example when the Updater's queue runs dry). */
int ipls_agg_flush(ipls_agg *h);

/* Coalescing group g (>= 1; 1 = fold each arrival at once) of asynchronous
 * device buckets: the queues are flushed when they average g buckets per
 * partition or one of them holds 2g.  Device traffic per element is
 * (g + 2) * 8 bytes for a group of g buckets, against 24 * g one by one. */
int ipls_agg_set_coalesce(ipls_agg *h, int max_group);

/* Updater.run's indirect request (Updater.java:176-187): the queue item holds
 * only a hash, so the bucket is `ipfs cat` bytes read into the Updater's one
 * reusable Gradient_Buff of (int)M/P + 2 doubles (Updater.java:162, zeroed
 * once) by GetParameters(hash, Gradient_Buff) (MyIPFSClass.java:444-455), and
 * _Update folds Gradient_Buff[0..L_p) into target[p].  Exactly as in Java, a
 * file shorter than L_p leaves the tail of the previous request in the buffer
 * and that tail is folded; a file longer than the buffer overwrites the
 * buffer, folds nothing and returns IPLS_E_RANGE (the AIOOBE).  The handle
 * owns the buffer (one per handle, like one Updater thread per peer). */
int ipls_agg_update_indirect(ipls_agg *h, int p, int target, const void *bytes, int64_t n_bytes);

/* ---- PeerData.Other_Replica_Gradients (PeerData.java:140-141) ----
 * The downloads of OTHER aggregators' buckets of partition p, kept per key
 * (p, aggregator) in a java.util.HashMap<Pair<Integer,String>, double[]>.
 *
 * The aggregator index contract.  The reference key is the aggregator's
 * peer-ID String.  Here `aggregator` is any int32 the caller maps 1:1 from
 * that String (e.g. its index in the Java side's table of known peers, or an
 * interned ID): two keys are the same key exactly when (p, aggregator) are
 * equal.  `key_hash` is the reference key's hashCode,
 *     new org.javatuples.Pair<>(p, peerId).hashCode()
 * (Java computes it directly; ipls_java_pair_hash computes it from the ID's
 * UTF-8 bytes).  It fixes where the key sits in the HashMap, and so the order
 * in which Collect_Replicas folds the stored arrays: floating-point addition
 * does not associate, so that order decides the bits of REP[p] once a
 * partition has two or more stored arrays.  ipls_agg_other_replica (no hash)
 * takes the peer ID to be Integer.toString(aggregator). */

/* new Pair<Integer,String>(p, id).hashCode() (javatuples 1.2, pom.xml:66-68) of a
 * peer ID given as UTF-8 bytes: 31 + 31*(31 + p) + id.hashCode() in wrapping
 * int32 arithmetic, String.hashCode over the ID's UTF-16 units.  IPLS_E_FORMAT
 * for malformed UTF-8.  No handle, no GPU. */
int ipls_java_pair_hash(int32_t p, const uint8_t *id, int64_t len, int32_t *hash);

/* Download_Scheduler.download_gradients, a bucket of ANOTHER aggregator of
 * partition p (Download_Scheduler.java:245-268): kept per (p, aggregator) in
 * Other_Replica_Gradients -- the first download becomes the stored array
 * (its own length n, -0.0 kept) and the key is put into the map model with
 * key_hash; later ones fold into it for j < n and leave its position as it
 * is (a later call with another key_hash for a stored key: IPLS_E_INVAL).  A
 * later download longer than the stored array returns IPLS_E_RANGE, nothing
 * folded.  Other_Replica_Gradients_Received counts the downloads. */
int ipls_agg_other_replica_keyed(ipls_agg *h, int p, int32_t aggregator, int32_t key_hash, const void *src,
                                 int64_t n, int src_kind);
/* The same with the peer ID Integer.toString(aggregator). */
int ipls_agg_other_replica(ipls_agg *h, int p, int32_t aggregator, const void *src, int64_t n,
                           int src_kind);

/* Other_Replica_Gradients.remove(new Pair<>(p, aggregator)) and the same
 * remove on Other_Replica_Gradients_Received: the stored array and its
 * download count are discarded (the HashMap keeps its capacity).  Returns 1
 * if the key was stored, 0 if not (no-op).  The reference removes the key when
 * that aggregator's own partial sum has arrived, so its downloaded buckets
 * are not counted twice: Download_Scheduler.java:215-217 (already in
 * Received_Replicas), :329-332 and :438-440 (its partial-update file
 * downloaded).  GlobalGradientPool.java:90-93 builds its key from the
 * frame's List<String> of origins, which never equals a stored
 * Pair<Integer,String>: that remove is a no-op in the reference
 * (INTEGRATION.md §2). */
int ipls_agg_other_replica_drop(ipls_agg *h, int p, int32_t aggregator);

/* Collect_Replicas (IPLS.java:1217-1241): REP[p][j] = REP[p][j] + Other[(p,a)][j]
 * for every stored key, in the order of new ArrayList<>(keySet()) of the JDK
 * HashMap (ascending bin of the key hashes under the map's capacity, then
 * insertion order within a bin), then clears the store
 * (Other_Replica_Gradients = new HashMap<>(): capacity reset).
 * participants (nullable, P ints) receives, per partition, what the reference
 * adds to PeerData.Participants[p]: its put / replace sits inside the element
 * loop (IPLS.java:1229-1234), so every stored key adds its download count
 * (Other_Replica_Gradients_Received) once per element -- received * length,
 * wrapping like Java int.  The Java side adds a nonzero entry to its map
 * (put if absent, else +=).  Returns the number of stored arrays folded, or
 * IPLS_E_RANGE (nothing folded) if one is longer than its partition. */
int ipls_agg_collect_replicas(ipls_agg *h, int32_t *participants);

/* The order Collect_Replicas would fold the stored keys in right now, as
 * (partition, aggregator) pairs: pairs[2i], pairs[2i+1].  Returns the number
 * of stored keys and writes the first min(that, max_pairs) of them (pairs may
 * be NULL with max_pairs 0 to ask for the count); a return above max_pairs
 * means the list was cut -- another thread may have stored keys since the
 * count was asked for -- and the caller asks again with more room.
 * A diagnostic for a Java caller to check the library's HashMap model against
 * its own `new ArrayList<>(Other_Replica_Gradients.keySet())`.  *capacity
 * (nullable) receives the model's table capacity (0 after new HashMap<>()). */
int ipls_agg_replica_order(ipls_agg *h, int32_t *pairs, int max_pairs, int32_t *capacity);

/* Batched fixed-order fold, ONE kernel launch for n_parts partitions:
 *   for q in [0,n_parts): target[p_first+q] = fold(start_mode; bufs[q*k + 0..k-1])
 * bufs are device pointers (DEV_F64 or DEV_BE), each at least L_p long.
 * This is the benchmarked kernel. */
int ipls_agg_reduce_batch(ipls_agg *h, int p_first, int n_parts,
                          const void *const *bufs, int k, int src_kind,
                          int start_mode, int target);

/* The same batched fold written to caller device buffers, one per partition
 * (dst[q], at least L_p doubles / 8*L_p bytes): dst_kind DEV_BE fuses the
 * double->byte pack of update_file (MyIPFSClass.java:105-116) into the fold,
 * src_kind DEV_BE the byte->double unpack of GetParameters (:444-455).  With
 * START_FIRST this is the storage node's `-aggr 1` merge
 * (Decentralized_Storage_Receiver.java:239-258: S = g0; S += g_i; write the
 * `_partial_aggregation` file).  ACCUM reads dst in dst_kind's byte order. */
int ipls_agg_reduce_batch_out(ipls_agg *h, int p_first, int n_parts,
                              const void *const *bufs, int k, int src_kind,
                              int start_mode, void *const *dst, int dst_kind);

/* Pubsub ingest on the device (ThreadReceiver.run/process, IPLS.java:851-866,
 * 399-465; Utils.getRawMessage, Utils.java:8-17).  msgs[i] / lens[i] are the
 * JSON "data" texts of n_msgs pubsub messages: `layers` (1 or 2) rounds of
 * java.util.Base64 URL encoding of a Marshall_Packet frame
 * (MyIPFSClass.java:990-1017).  They are copied to the device, decoded there
 * (alphabet and '=' rules of Base64.getUrlDecoder), parsed as GET_GRADIENTS
 * frames (MyIPFSClass.java:1437-1459), and each payload is folded (BE decode
 * fused) into target[p] in message order.  p = parts[i], or the frame's
 * partition field when parts is NULL.  A bad message is dropped and reported,
 * as the Java receiver drops it after printing the exception:
 * status[i] = 0 folded, 1 null gradient (n == 0, no fold), IPLS_E_FORMAT
 * (bad base64 / short frame), IPLS_E_RANGE (partition out of range or
 * payload shorter than L_p).  Returns the number of messages folded.
 * The texts are copied by IPLS_INGEST_COPY_THREADS (default 2) short-lived
 * host threads, each on its own stream, while the device decodes the texts
 * that have already landed; msgs must stay valid until the call returns. */
int ipls_agg_ingest_pubsub(ipls_agg *h, int target, const uint8_t *const *msgs,
                           const int64_t *lens, int n_msgs, int layers,
                           const int32_t *parts, int32_t *status);

/* Variants (-async true / leaving peers):
 *   blend: target[p][i] = a*target[p][i] + b*g[i]  (products rounded, then the sum)
 *     async replica fold  a = 0.75, b = 1        Updater.java:57-59
 *     leaving-peer blend  a = 0.6,  b = 1 - 0.6  Updater.java:65-69
 *   scale: dst[p][i] = c * src[p][i]             Updater.java:197-199 (0.25 * W) */
int ipls_agg_blend(ipls_agg *h, int p, int target, const void *src, int64_t n, int src_kind,
                   double a, double b);
int ipls_agg_scale(ipls_agg *h, int p, int dst_target, int src_target, double c);

/* AggregatePartition (IPLS.java:1248-1274): W = AGG + REP, Weight_Address = W,
 * AGG = REP = 0.  p may be IPLS_ALL_PARTITIONS.  Optional host outputs for one
 * partition: sum_out (the commit_update file bytes, IPLS_Comm.java:27-37 ->
 * update_file, when sum_kind == HOST_BE; or doubles, HOST_F64) and avg_out
 * (L_p - 1 averaged values, the GetPartitions divide).  Either may be NULL. */
int ipls_agg_finalize(ipls_agg *h, int p, void *sum_out, int sum_kind, double *avg_out);

/* ipls_agg_finalize of one partition with its sum handed to a sink chunk by
 * chunk, as ONE call: AggregatePartition (IPLS.java:1248-1274), then W[p]
 * comes back through a pinned ring (three slots) in chunks of `chunk` values
 * (even, >= 2), sink(ctx, values, offset, n) on the calling thread for
 * consecutive ranges of [0, L_p), so the sink's copy of one chunk overlaps
 * the transfer of the next.  values: n 8-byte values, doubles (HOST_F64) or
 * the commit_update file bytes (HOST_BE, update_file's putDouble order,
 * MyIPFSClass.java:105-116), valid during the sink call only.  Under the
 * shard's lock the call runs AggregatePartition and snapshots W (or its
 * bytes) into staging of its own; the lock is released before the first sink
 * call.  So the bytes are this call's W whatever set_weights, fold or
 * finalize another thread makes meanwhile (never torn), and a slow sink
 * holds up nobody.  A non-zero sink return stops the delivery with
 * IPLS_E_INVAL; the round is consumed either way (W is written, AGG = REP =
 * 0), as after a failed update_file.  The JNI shim's finalizePartition(byte[])
 * sink is SetByteArrayRegion. */
int ipls_agg_finalize_chunked(ipls_agg *h, int p, int sum_kind, int64_t chunk, ipls_chunk_sink sink, void *ctx);

/* A whole aggregation round for partitions [p_first, p_first+n_parts) in ONE
 * kernel launch (one pass over the buckets):
 *   AGG[p]   = AGG[p] + b_0 + ... + b_{k-1}     Updater._Update folds (Updater.java:115-117)
 *   W[p]     = AGG[p] + REP[p]; AGG = REP = 0   AggregatePartition (IPLS.java:1248-1274)
 *   avg_out  = W[p][j] / W[p][L_p-1]            GetPartitions divide (IPLS.java:1159-1174)
 * AGG is never stored: its final value only feeds W.  Results are bit-identical
 * to reduce_batch(ACCUM) + finalize + get_partitions.  bufs: n_parts*k device
 * buckets (DEV_F64/DEV_BE, k may be 0).  avg_out (or NULL) receives the
 * averaged values of the partitions, partition p at flat offset
 * partition_offset(p) - partition_offset(p_first) -- for all partitions the
 * GetPartitions model; avg_kind DEV_F64 or HOST_F64. */
int ipls_agg_aggregate_round(ipls_agg *h, int p_first, int n_parts,
                             const void *const *bufs, int k, int src_kind,
                             void *avg_out, int avg_kind);

/* Download_Scheduler.cache_partition (Download_Scheduler.java:752-792):
 * Weight_Address[p] = GetParameters(hash) -- the downloaded updated partition
 * (n doubles, F64/BE host or device kinds).  src_kind HOST_FRAME (n = frame
 * bytes) is the pid-4 ACK of ThreadReceiver (IPLS.java:491-498): the frame's
 * first L_p payload doubles become Weight_Address[p]. */
int ipls_agg_set_weights(ipls_agg *h, int p, const void *src, int64_t n, int src_kind);

/* GetPartitions (IPLS.java:1140-1174): Weights = Weight_Address, then the
 * flat model with every partition divided by its count slot (count 0.0 ->
 * values unchanged; secure -> / (1e12 * count)).  out holds model_size
 * doubles; out_kind HOST_F64, HOST_BE_CANON (Middleware task-3 stream), DEV_F64. */
int ipls_agg_get_partitions(ipls_agg *h, void *out, int64_t n, int out_kind);

/* GetPartitions (IPLS.java:1159-1174) delivered in chunks of `chunk` doubles
 * (even, >= 2) to sink(ctx, values, offset, n) on the calling thread, in
 * model order: the divide runs once on the GPU into staging of this call's
 * own -- every shard's, each under its shard lock for that launch only,
 * before any chunk is delivered, so the whole model is one snapshot -- then
 * each chunk comes back through a pinned ring (three slots) with no lock held, so
 * the sink's copy of chunk k overlaps the transfer of chunk k + 1 (the JNI
 * getPartitions(double[]) copies each chunk into the Java array with
 * SetDoubleArrayRegion).  `values` is valid only during the sink call.  A
 * non-zero sink return stops the transfer: the call returns IPLS_E_INVAL and
 * no further chunk is delivered.  Replaces the same loop as
 * ipls_agg_get_partitions. */
int ipls_agg_get_partitions_chunked(ipls_agg *h, int64_t chunk, ipls_chunk_sink sink, void *ctx);

/* The same delivery as Middleware task 3's reply (Serialize, Middleware.java:
 * 164-170): each chunk is n values of the writeDouble stream -- big-endian
 * bytes, NaN canonicalised, written by the divide kernel -- so a socket sink
 * sends chunk k while chunk k + 1 comes back over PCIe (ipls.middleware's
 * loopback server).  Rules as ipls_agg_get_partitions_chunked. */
int ipls_agg_get_partitions_wire_chunked(ipls_agg *h, int64_t chunk, ipls_chunk_sink sink, void *ctx);

/* Copy an accumulator out (tests, replica publish IPLS.java:1423-1431).
 * dst_kind HOST_F64, HOST_BE, DEV_F64, DEV_BE; n >= L_p. */
int ipls_agg_read(ipls_agg *h, int p, int target, void *dst, int64_t n, int dst_kind);

/* End of IPLS.Update_Client_WaitAck_List (IPLS.java:1556-1562): for every p
 * in parts[0..n_parts): AGG[p] = FUTURE[p]; FUTURE[p] = 0.  O(1) per partition
 * (the two accumulators swap storage), so an address from ipls_agg_device_ptr
 * for AGG or FUTURE of such a p is stale afterwards. */
int ipls_agg_promote_future(ipls_agg *h, const int32_t *parts, int n_parts);

/* Zero AGG[p] and REP[p] (IPLS.java:1268-1269); p may be IPLS_ALL_PARTITIONS. */
int ipls_agg_reset(ipls_agg *h, int p);

/* Device address of an accumulator (for RCCL send/recv of replica partials).
 * Work the caller orders on the handle's stream sees the folds of every call
 * made so far -- except device buckets still queued by
 * ipls_agg_accumulate_async: call ipls_agg_flush (or any other entry point)
 * before reading the accumulator through this address. */
int ipls_agg_device_ptr(ipls_agg *h, int p, int target, void **ptr);

/* The handle's HIP stream (hipStream_t as void*) and a host wait on it
 * (ipls_agg_sync also folds queued device buckets first). */
void *ipls_agg_stream(ipls_agg *h);
int ipls_agg_sync(ipls_agg *h);

/* Order-independent checksum of partition p of a target:
 *   sum_i splitmix64(bits(x_i) + i*0x9E3779B97F4A7C15) mod 2^64
 * computed on the device (wave DPP + LDS reduction, exact integer sum). */
int ipls_agg_checksum(ipls_agg *h, int p, int target, uint64_t *out);

/* ---- multi-GPU (cfg.devices) ----
 * A partition's accumulators live on its owner shard.  Its contributors may
 * span GPUs the way the reference's replica aggregators of one partition do
 * (IPLS.java:1402-1468: each aggregator folds the buckets it received, the
 * partials are published at :1423-1431, the owner adds them in
 * Collect_Replicas :1449 / the Updater replica branch, Updater.java:40-44,
 * and AggregatePartition :1462-1468 forms W = AGG + REP).  Here a replica
 * aggregator is a SLOT: a shard other than the owner folds the buckets
 * resident on its GPU into the slot's partial sum of p
 * (ipls_agg_reduce_partial), and ipls_agg_combine_partials pulls the partials
 * of every other slot over xGMI (peer loads in the owner's fold kernel) and
 * folds them into REP[p] in ascending slot order:
 *     REP[p] = ((REP[p] + R_s1) + R_s2) + ...     (REP starts at +0.0)
 * which is the reference's expression for aggregators s1 < s2 < ...  */

/* Owner shard of partition p: its HIP device ordinal and stream (hipStream_t
 * as void*; work on p's device pointers is ordered on that stream).  Either
 * output may be NULL. */
int ipls_agg_partition_device(ipls_agg *h, int p, int32_t *device, void **stream);

/* The contiguous-block shard plan of cfg.devices, without a handle (no GPU
 * needed): owner[p] = p / ceil(n_partitions / n_shards) for every p. */
int ipls_shard_plan(int32_t n_partitions, int32_t n_shards, int32_t *owner);

/* Replica slot `slot` (a shard index, not the owner of any partition in
 * range) folds k device buckets per partition -- resident on that slot's
 * device -- into its partial sums of partitions [p_first, p_first+n_parts):
 *     R_slot[p] = fold(start_mode; bufs[q*k + 0..k-1])
 * with the same kernels and order as ipls_agg_reduce_batch.  ACCUM folds on
 * top of the slot's current partial (+0.0 after a combine). */
int ipls_agg_reduce_partial(ipls_agg *h, int slot, int p_first, int n_parts, const void *const *bufs, int k,
                            int src_kind, int start_mode);

/* For every partition of [p_first, p_first+n_parts): REP[p] += the partial of
 * every slot that folded into p since the last combine, slots ascending, in
 * one launch per owner shard that reads the partials over xGMI (partitions
 * with the same number of live slots share a launch whichever GPUs hold their
 * partials, so an owner reads over all its links at once); the partials are
 * then logically +0.0 again.  Returns the number of partials folded.
 * A pair of devices without peer access is not an error: such a partial is
 * first copied into an owner-side buffer (hipMemcpyPeerAsync on the SLOT's
 * stream, after the slot's folds, so copies from different GPUs run at once;
 * the partial's `ready` event is then re-recorded on that stream and the
 * owner waits on it) and the same fold reads that copy, in the same slot
 * order, so the result is bit-identical.  Memory: each such owner-side
 * buffer is L_p doubles per (slot, partition) pair that was ever staged,
 * allocated on the owner at the first staged combine and kept until
 * ipls_agg_close -- up to (G-1) extra copies of every partition an owner
 * holds on a node without peer access; it is not reserved at open, so an
 * out-of-memory shows up as IPLS_E_NOMEM from this call.  Setting
 * IPLS_PEER_STAGED=1 in the environment before ipls_agg_open forces this
 * path for every cross-shard read (the combine and the Gradient_Buff of
 * ipls_agg_update_indirect) -- a test switch; ipls_launch_info.staged counts
 * the staged partials.  The staged path has run only with shards sharing one
 * GPU (a copy within one device); between two distinct GPUs it is unmeasured
 * on hardware. */
int ipls_agg_combine_partials(ipls_agg *h, int p_first, int n_parts);

/* ---- publish-side codec (a9) ----
 * Marshall_Packet(target[p], origin, a, b, pid) (MyIPFSClass.java:990-1016),
 * as the aggregator publishes its partial sum every round
 * (IPLS.java:1429-1430: a = middleware_iteration, b = workers + 1, pid = 3):
 * the frame [i16 pid][i32 L_p][i32 a][i32 b][L_p x f64 BE][origin] encoded
 * with Base64.getUrlEncoder ('=' padding), produced on the device straight
 * from the accumulator (k_b64url_encode_frame).  origin = the bytes of
 * OriginPeer.getBytes() the frame carries (String.length() of them).
 * out_kind IPLS_HOST_TEXT (copied back, call complete on return) or
 * IPLS_DEV_TEXT (device buffer, stream-ordered).  Returns the text length
 * 4*ceil((14 + 8*L_p + origin_len)/3); out == NULL: the length only. */
int64_t ipls_agg_publish_partial(ipls_agg *h, int p, int target, int32_t a, int32_t b, int16_t pid,
                                 const uint8_t *origin, int32_t origin_len, void *out, int64_t out_cap,
                                 int out_kind);

/* The same for several partitions in one launch per GPU: the publish loop
 * over Auth_List (IPLS.java:1423-1431), text i = Marshall_Packet(target[
 * parts[i]], origin, a, b[i], pid) base64url-encoded.  Text i lands at
 * out + offs[i] (offs are 64-byte multiples, texts in list order), lens[i]
 * bytes.  lens/offs (n_parts entries, either may be NULL) are filled even
 * when out == NULL.  Returns the bytes the buffer needs (offs[n-1] +
 * lens[n-1]); b and origin may be NULL when out is (origin_len still counts).  IPLS_DEV_TEXT with partitions on several GPUs: out must be
 * memory every owner device can write (its own or a peer's). */
int64_t ipls_agg_publish_partials(ipls_agg *h, const int32_t *parts, int n_parts, int target, int32_t a,
                                  const int32_t *b, int16_t pid, const uint8_t *origin, int32_t origin_len,
                                  void *out, int64_t out_cap, int out_kind, int64_t *lens, int64_t *offs);

/* ---- observability ----
 * What the last fold launch of a handle (of p's shard for multi-GPU handles:
 * the shard of the last call) ran: the kernel, the tile shape chosen by the
 * dispatch, lanes per workgroup, 16-B vectors per lane per
 * tile, the SEQ schedule code, the block->tile map and the grid. */
#define IPLS_KERNEL_REDUCE        1  /* k_reduce        */
#define IPLS_KERNEL_ROUND         2  /* k_round (fused) */
#define IPLS_KERNEL_FOLD1         3  /* k_fold1         */
#define IPLS_KERNEL_REDUCE_SCALAR 4  /* k_reduce_scalar */
#define IPLS_SHAPE_BIG    1
#define IPLS_SHAPE_MID    2
#define IPLS_SHAPE_SMALL  3
#define IPLS_SHAPE_HALF   4  /* 512 lanes x 16 vectors: native doubles, few partitions */
typedef struct ipls_launch_info {
    int32_t kernel, shape, block, vectors, seqf, map;
    int64_t grid;
    int32_t be_in, be_out, start;
    int32_t staged;   /* partials the handle's last ipls_agg_combine_partials copied to the owner
                         first (no xGMI peer access, or IPLS_PEER_STAGED=1) instead of peer loads */
} ipls_launch_info;
int ipls_agg_last_launch(ipls_agg *h, ipls_launch_info *out);

/* ---- host memory ---- */

/* Pinned host memory for IPFS byte buffers / the Middleware stream (the Java
 * side wraps it with JNI NewDirectByteBuffer).  Host operands that live in
 * such memory are DMA'd to the device directly, without a staging copy. */
int ipls_host_alloc(size_t bytes, void **ptr);
/* (Such buffers are also valid DEV_F64 / DEV_BE bucket pointers for
 * ipls_agg_reduce_batch: the fold kernel then reads them over PCIe directly,
 * zero copy.  ipls_agg_accumulate does this by itself for pinned sources.) */
int ipls_host_free(void *ptr);

/* ---- device utilities (no handle) -- stream may be NULL (default stream) ---- */

/* Fill a device bucket with the synthetic workload of SURVEY.md §8(d):
 * x_i = (2u-1)*1e-2, u = (splitmix64(seed ^ p<<40 ^ k<<32 ^ i) >> 11) * 2^-53,
 * x_{L-1} = 1.0 (count slot).  dst_kind DEV_F64 or DEV_BE. */
int ipls_synth_fill(void *dst, int64_t len, uint64_t seed, int p, int k, int dst_kind,
                    void *stream);

/* Checksum (as above) of n device doubles (DEV_F64) or BE doubles (DEV_BE). */
int ipls_checksum_dev(const void *src, int64_t n, int src_kind, uint64_t *out, void *stream);

/* Middleware.Encode (secure mode, Middleware.java:196-210) on n device
 * doubles: clip to +-10 then scale by 1e12 (dst may equal src). */
int ipls_encode_secure(const void *src, void *dst, int64_t n, int src_kind, int dst_kind,
                       void *stream);

/* Pubsub frame header parse (MyIPFSClass.java:1437-1446 / 1462-1469).
 * Returns the number of doubles n, or IPLS_E_FORMAT. */
int64_t ipls_frame_parse(const uint8_t *frame, int64_t len, int16_t *pid, int32_t *a,
                         int32_t *b, int64_t *payload_off, int64_t *origin_off);

/* Frame encode (MyIPFSClass.java:990-1017) of n device or host doubles into a
 * host byte buffer of 14 + 8n + origin_len bytes.  Returns bytes written. */
int64_t ipls_frame_encode(const double *g, int64_t n, int g_kind, int32_t a, int32_t b,
                          int16_t pid, const uint8_t *origin, int32_t origin_len,
                          uint8_t *out, int64_t out_cap);

/* ---- the partial-update object: Java-serialised Pair<Integer, double[]> ----
 * IPLS_Comm.commit_partial_update (IPLS_Comm.java:51-61) and
 * DStorage_Client.sendPartition(..., mod 1) (DStorage_Client.java:152-154,
 * `-i 1`) write new Pair<>(workers, Aggregated_Gradients[p]) with
 * ObjectOutputStream; Download_Scheduler (:324-325) and the storage merge
 * (Decentralized_Storage_Receiver.java:249-256) read it back. */

/* Parse such a stream: returns the number of doubles (the payload is that
 * many big-endian doubles at byte *payload_off) and the Integer in *workers,
 * or IPLS_E_FORMAT (not a Pair<Integer,double[]> object stream, or truncated). */
int64_t ipls_pair_parse(const uint8_t *buf, int64_t len, int32_t *workers, int64_t *payload_off);

/* The exact bytes ObjectOutputStream.writeObject(new Pair<>(workers, g)) writes
 * for n doubles (g_kind HOST_F64 or HOST_BE).  Returns the byte count; with
 * out == NULL only the count; IPLS_E_RANGE if out_cap is too small. */
int64_t ipls_pair_encode(int32_t workers, const void *g, int64_t n, int g_kind, uint8_t *out,
                         int64_t out_cap);

/* commit_partial_update's file bytes for AGG[p] (IPLS.java:1423-1425):
 * Pair<>(workers, Aggregated_Gradients[p]) with the payload packed on the
 * device.  Returns the byte count (out == NULL: count only). */
int64_t ipls_agg_commit_partial(ipls_agg *h, int p, int32_t workers, uint8_t *out, int64_t out_cap);

/* The storage node's merge (Decentralized_Storage_Receiver.java:239-258) of k
 * downloaded files: status 0 -> raw BE files (file_kind HOST_BE), status != 0
 * -> Pair partial updates (HOST_PAIR).  Aggregation = the first file's doubles;
 * then Aggregation[j] += g[j] for j < g.length, file by file; the result is
 * written to out as the `<p>_partial_aggregation` file bytes (update_file: BE).
 * Returns the byte count; IPLS_E_RANGE when a later file is longer than the
 * first (the reference's ArrayIndexOutOfBoundsException) or out_cap is short. */
int64_t ipls_agg_merge_files(ipls_agg *h, const uint8_t *const *files, const int64_t *lens, int k,
                             int file_kind, uint8_t *out, int64_t out_cap);

#ifdef __cplusplus
}
#endif
#endif /* IPLS_AGG_H */
