// NativeAggregator.java -- Java side of the JNI binding of libipls_agg
// (include/ipls_agg.h).  A Java IPLS maintainer drops this class into
// src/main/java/ next to IPLS.java and calls it from the patched loops listed
// in INTEGRATION.md.  Not compiled in this image (no JDK); the C half is
// ipls-java-api_amd/jni/ipls_jni.c.
//
// Arrays are passed as primitive arrays (the shim copies them with
// Get/Set<T>ArrayRegion: never pinned across a library call, so the GC keeps
// running) or as direct ByteBuffers (zero copy; allocate them with hostAlloc()
// so the library DMA's straight from them).

import java.nio.ByteBuffer;

import org.javatuples.Pair;

public final class NativeAggregator implements AutoCloseable {
    static { System.loadLibrary("ipls_jni"); }   // links libipls_agg.so

    // include/ipls_agg.h constants
    public static final int TGT_AGG = 0, TGT_REP = 1, TGT_WEIGHTS = 2, TGT_WADDR = 3, TGT_FUTURE = 4;
    public static final int START_ACCUM = 0, START_ZERO = 1, START_FIRST = 2;
    public static final int ALL_PARTITIONS = -1;

    private long handle;
    private final int partitions;

    /** IPLS.init -> InitializeWeights(): -pa, -n, -aggr from Middleware.parse_arguments. */
    public NativeAggregator(long modelSize, int partitions, int minPeers, boolean partialAggregation,
                            boolean secure, int device) {
        handle = open(modelSize, partitions, minPeers, partialAggregation ? 1 : 0, secure ? 1 : 0, device);
        this.partitions = partitions;
    }

    /** The same over several GPUs of one node: the -pa partitions are sharded over
     *  `devices` in contiguous blocks (partition p on devices[p / ceil(P/G)]). */
    public NativeAggregator(long modelSize, int partitions, int minPeers, boolean partialAggregation,
                            boolean secure, int[] devices) {
        handle = openDevices(modelSize, partitions, minPeers, partialAggregation ? 1 : 0, secure ? 1 : 0, devices);
        this.partitions = partitions;
    }

    /** HIP device that owns partition p (allocate p's device buckets there). */
    public int partitionDevice(int p) { return partitionDevice(handle, p); }

    /** The contiguous-block plan: owner shard of every partition. */
    public static int[] shards(int partitions, int nShards) { return shardPlan(partitions, nShards); }

    public int partitionLength(int p) { return (int) partitionLen(handle, p); }

    /** InitializeWeights(List<Double> Model) (IPLS.java:1880-1901). */
    public void initializeWeights(double[] model) { loadModel(handle, model); }

    /** UpdateGradient own accumulate (IPLS.java:1737-1743); gradients == null is a no-op. */
    public void updateGradient(double[] gradients, int[] authList) {
        if (gradients != null) updateGradient(handle, gradients, authList);
    }

    /** Middleware task 2 (Deserialize, Middleware.java:156-160) + UpdateModel's
     *  own accumulate, without the List&lt;Double&gt;: the update's model_size
     *  big-endian doubles, as read off the socket into a hostAlloc direct buffer
     *  (e.g. Channels.newChannel(in).read(buf) until full), folded from there
     *  (the byte swap is fused into the fold; only the owned partitions' bytes
     *  cross PCIe). */
    public void updateGradientWire(ByteBuffer direct, int[] authList) {
        updateGradientDirect(handle, direct, direct.position(), direct.remaining() / 8, authList);
    }

    /** OrganizeGradients (IPLS.java:1018-1040) for partition p (count slot 1.0). */
    public double[] organize(double[] gradients, int p) {
        double[] out = new double[partitionLength(p)];
        split(handle, gradients, p, out);
        return out;
    }

    /** Updater._Update: client buckets -> TGT_AGG, replica partials -> TGT_REP.
     *  One library call for the whole bucket (ipls_agg_accumulate_chunked: the
     *  array is copied out chunk by chunk inside it, with no GPU lock held), and
     *  the bucket takes effect as one unit once its last chunk has landed: no
     *  other thread's fold lands between two of its chunks -- the whole-bucket
     *  fold the Updater does under PeerData.mtx (Updater.java:72-149) -- and no
     *  other thread waits for its heap copies.  A failed copy folds nothing. */
    public void update(double[] gradient, int p, boolean fromClients) {
        if (gradient != null) accumulate(handle, p, fromClients ? TGT_AGG : TGT_REP, gradient);
    }

    /** Updater indirect mode (Updater.java:176-187): the `ipfs cat` bytes of a
     *  gradient file go through the handle's Gradient_Buff, as GetParameters(hash,
     *  Gradient_Buff) + _Update do (short files fold the previous file's tail). */
    public void updateFromFile(ByteBuffer catBytes, int p, boolean fromClients) {
        updateIndirect(handle, p, fromClients ? TGT_AGG : TGT_REP, catBytes, catBytes.position(), catBytes.remaining());
    }

    /** A bucket already decoded to exactly L_p big-endian doubles (no Gradient_Buff). */
    public void updateFromBytes(ByteBuffer beDoubles, int p, boolean fromClients) {
        accumulateDirect(handle, p, fromClients ? TGT_AGG : TGT_REP, beDoubles, beDoubles.position(),
                         beDoubles.remaining() / 8, 1);
    }

    /** The same fold without waiting (one call per queue.take(), Updater.java:169-211):
     *  beDoubles is a direct buffer from hostAllocDirect (pinned), folded over PCIe
     *  while the next `ipfs cat` fills another buffer.  Keep it until await(ticket). */
    public long updateFromBytesAsync(ByteBuffer beDoubles, int p, boolean fromClients) {
        return accumulateAsyncDirect(handle, p, fromClients ? TGT_AGG : TGT_REP, beDoubles, beDoubles.position(),
                                     beDoubles.remaining() / 8, 1);
    }

    /** Block until fold `ticket` (and every fold queued before it) has finished. */
    public void await(long ticket) {
        waitTicket(handle, ticket);
    }

    /** Start the folds of queued device buckets now (Updater.run when queue.isEmpty()). */
    public void flush() {
        flushQueued(handle);
    }

    /** Updater.java:99-101: a client's bucket for a later iteration. */
    public void updateFromFuture(double[] gradient, int p) {
        if (gradient != null) accumulate(handle, p, TGT_FUTURE, gradient);
    }

    /** Download_Scheduler.download_gradients (:254-266): another aggregator's
     *  bucket for partition p, kept per (p, aggregator) until collectReplicas().
     *  aggregator: an int mapped 1:1 from the aggregator's peer-ID String (e.g.
     *  its index in a peer table); aggregatorId: that String, whose
     *  new Pair<>(p, aggregatorId).hashCode() places the key in the native
     *  model of the HashMap Other_Replica_Gradients (PeerData.java:140) and so
     *  fixes the Collect_Replicas fold order (IPLS.java:1218). */
    public void otherReplica(int p, int aggregator, String aggregatorId, ByteBuffer catBytes) {
        otherReplicaDirect(handle, p, aggregator, new Pair<Integer, String>(p, aggregatorId).hashCode(), catBytes,
                           catBytes.position(), catBytes.remaining() / 8);
    }

    /** Other_Replica_Gradients.remove(new Pair<>(p, aggregatorId)) together with
     *  Other_Replica_Gradients_Received.remove: that aggregator's partial sum
     *  arrived (Download_Scheduler.java:215-217, 329-332, 438-440).  Returns
     *  whether the key was stored. */
    public boolean dropOtherReplica(int p, int aggregator) {
        return otherReplicaDrop(handle, p, aggregator);
    }

    /** The (partition, aggregator) order collectReplicas() would fold in now,
     *  {p0, a0, p1, a1, ...}: compare it with the keys of
     *  new ArrayList<>(PeerData.Other_Replica_Gradients.keySet()) mapped to
     *  aggregator indices to check the native HashMap model in a real JVM. */
    public int[] replicaKeyOrder() {
        return replicaKeyOrder(handle);
    }

    /** IPLS.Collect_Replicas (IPLS.java:1217-1241); returns, per partition, what the
     *  reference adds to PeerData.Participants (received x length per key: its
     *  put/replace runs once per element, :1229-1234).  The caller applies a
     *  nonzero entry with Participants.merge(p, v, Integer::sum). */
    public int[] collectReplicas() {
        int[] participants = new int[partitions];
        collectReplicas(handle, participants);
        return participants;
    }

    /** IPLS_Comm.commit_partial_update (IPLS_Comm.java:51-61): the Pair<Integer,double[]> file bytes. */
    public byte[] commitPartial(int p, int workers) {
        byte[] out = new byte[(int) commitPartialLen(handle, p, workers)];
        commitPartial(handle, p, workers, out);
        return out;
    }

    /** Download_Scheduler.java:324: a replica's Pair partial update, folded into REP. */
    public void updateFromPartial(byte[] catBytes, int p) { accumulatePair(handle, p, TGT_REP, catBytes); }

    /** Decentralized_Storage_Receiver.java:239-258: merge of downloaded files
     *  (raw BE gradient files, or Pair partial updates when status != 0). */
    public byte[] mergeFiles(byte[][] files, boolean partialUpdates) {
        return mergeFiles(handle, files, partialUpdates);
    }

    /** Tail of Update_Client_WaitAck_List (IPLS.java:1556-1562). */
    public void promoteFuture(int[] authList) { promoteFuture(handle, authList); }

    /** ThreadReceiver pid 3: a decoded (base64) pubsub frame. */
    public void updateFromFrame(byte[] frame, int p, boolean fromClients) {
        accumulateFrame(handle, p, fromClients ? TGT_AGG : TGT_REP, frame);
    }

    /** ThreadReceiver.run/process (IPLS.java:851-866, 453-465): pubsub 'data' texts
     *  (base64url x layers of Marshall_Packet frames) decoded, parsed and folded on the
     *  GPU in message order; partitions may be null (the frame's own field is used).
     *  status[i]: 0 folded, 1 null gradient, negative = the dropped message's exception
     *  (include/ipls_agg.h).  Returns the number of messages folded. */
    public int ingestPubsub(byte[][] texts, int layers, int[] partitions, boolean fromClients, int[] status) {
        return ingestTexts(handle, fromClients ? TGT_AGG : TGT_REP, texts, layers, partitions, status);
    }

    /** AggregatePartition (IPLS.java:1248-1274); returns the commit_update file bytes.
     *  One library call (ipls_agg_finalize_chunked): the bytes are a snapshot of
     *  this call's sum, so a cache_partition or fold of another thread neither
     *  tears them nor waits for their copy into the array. */
    public byte[] aggregatePartition(int p) {
        byte[] sum = new byte[8 * partitionLength(p)];
        finalizePartition(handle, p, sum);
        return sum;
    }

    /** AggregatePartition into a direct buffer from hostAlloc (pinned): the sum's
     *  D2H runs at the PCIe rate; a heap byte[] costs 10-15 % of a round. */
    public void aggregatePartition(int p, ByteBuffer directOut) {
        if (!directOut.isDirect() || directOut.remaining() < 8L * partitionLength(p))
            throw new IllegalArgumentException("need a direct buffer of 8*L_p bytes");
        finalizePartitionDirect(handle, p, directOut, directOut.position());
    }

    /** Download_Scheduler.cache_partition: Weight_Address[p] = GetParameters(hash). */
    public void cachePartition(int p, ByteBuffer beDoubles) {
        setWeightsDirect(handle, p, beDoubles, beDoubles.position(), beDoubles.remaining() / 8);
    }

    /** ThreadReceiver pid 4 (IPLS.java:491-498): the ACK frame's payload becomes Weight_Address[p]. */
    public void cachePartitionFrame(int p, byte[] frame) { setWeightsFrame(handle, p, frame); }

    /** GetPartitions (IPLS.java:1140-1174). */
    public double[] getPartitions(int modelSize) {
        double[] out = new double[modelSize];
        getPartitions(handle, out);
        return out;
    }

    /** AggregatePartition for partitions [pFirst, pFirst+nParts) and their
     *  GetPartitions averages in one fused launch (ipls_agg_aggregate_round);
     *  the result is sized here from the partition geometry. */
    public double[] aggregateRound(int pFirst, int nParts) {
        long first = offsetOf(pFirst), last = offsetOf(pFirst + nParts - 1) + partitionLength(pFirst + nParts - 1) - 1;
        double[] out = new double[(int) (last - first)];
        aggregateRound(handle, pFirst, nParts, out);
        return out;
    }

    private long offsetOf(int p) { return partitionOffset(handle, p); }   // p * chunk (IPLS.java:1019-1028)

    /** Middleware task 3: the writeDouble stream in one bulk write. */
    public void getPartitionsWire(ByteBuffer direct) {
        getPartitionsWire(handle, direct, direct.position(), direct.remaining());
    }

    /** The aggregator's partial sum published every round (IPLS.java:1429-1430):
     *  ipfsClass.send(topic, publishPartial(p, iteration, workers + 1, id)) --
     *  Marshall_Packet + Base64.getUrlEncoder, encoded on the GPU. */
    public String publishPartial(int p, int iteration, int workersPlusOne, String originPeer) {
        byte[] o = java.util.Arrays.copyOf(originPeer.getBytes(), originPeer.length());   // finalbarr's origin bytes
        return new String(publishPartial(handle, p, TGT_AGG, iteration, workersPlusOne, (short) 3, o),
                          java.nio.charset.StandardCharsets.US_ASCII);
    }

    /** The whole publish loop of a round (IPLS.java:1423-1431) in one launch per GPU:
     *  text i = Marshall_Packet(Aggregated_Gradients[parts[i]], id, iteration,
     *  workersPlusOne[i], 3) base64url-encoded. */
    public String[] publishPartials(int[] parts, int iteration, int[] workersPlusOne, String originPeer) {
        byte[] o = java.util.Arrays.copyOf(originPeer.getBytes(), originPeer.length());
        long[] lens = new long[parts.length], offs = new long[parts.length];
        long total = publishPartialsLayout(handle, parts, o.length, lens, offs);
        ByteBuffer buf = ByteBuffer.allocateDirect((int) Math.max(1, total));
        publishPartialsDirect(handle, parts, TGT_AGG, iteration, workersPlusOne, (short) 3, o, buf, 0, total);
        String[] out = new String[parts.length];
        for (int i = 0; i < parts.length; ++i) {
            byte[] t = new byte[(int) lens[i]];
            buf.position((int) offs[i]);
            buf.get(t);
            out[i] = new String(t, java.nio.charset.StandardCharsets.US_ASCII);
        }
        return out;
    }

    /** Device-resident batches: n_parts x k device addresses, partition-major. */
    public void reduceBatch(int pFirst, int nParts, long[] devPtrs, int k, boolean bigEndian, int start, int target) {
        reduceBatchDevice(handle, pFirst, nParts, devPtrs, k, bigEndian ? 4 : 3, start, target);
    }

    /** A replica slot (another GPU of this handle) folds its buckets of partitions it
     *  does not own; combinePartials adds every slot's partial to REP in slot order. */
    public void reducePartial(int slot, int pFirst, int nParts, long[] devPtrs, int k, boolean bigEndian, int start) {
        reducePartialDevice(handle, slot, pFirst, nParts, devPtrs, k, bigEndian ? 4 : 3, start);
    }

    public int combinePartials(int pFirst, int nParts) { return combinePartials(handle, pFirst, nParts); }

    public static ByteBuffer hostAlloc(int bytes) { return hostAllocDirect(bytes); }

    @Override public void close() { if (handle != 0) { close(handle); handle = 0; } }

    // ---- natives (ipls_jni.c) ----
    private static native long open(long modelSize, int partitions, int maxPeers, int aggr, int secure, int device);
    private static native long openDevices(long modelSize, int partitions, int maxPeers, int aggr, int secure,
                                           int[] devices);
    private static native int partitionDevice(long h, int p);
    private static native int[] shardPlan(int partitions, int shards);
    private static native void reduceBatchDevice(long h, int pFirst, int nParts, long[] ptrs, int k, int kind,
                                                 int start, int target);
    private static native void reducePartialDevice(long h, int slot, int pFirst, int nParts, long[] ptrs, int k,
                                                   int kind, int start);
    private static native int combinePartials(long h, int pFirst, int nParts);
    private static native byte[] publishPartial(long h, int p, int target, int a, int b, short pid, byte[] origin);
    private static native long publishPartialsLayout(long h, int[] parts, int originLen, long[] lens, long[] offs);
    private static native void publishPartialsDirect(long h, int[] parts, int target, int a, int[] b, short pid,
                                                     byte[] origin, ByteBuffer out, int pos, long cap);
    private static native void close(long h);
    private static native long partitionLen(long h, int p);
    private static native long partitionOffset(long h, int p);
    private static native void loadModel(long h, double[] model);
    private static native void split(long h, double[] flat, int p, double[] out);
    private static native void updateGradient(long h, double[] flat, int[] owned);
    private static native void updateGradientDirect(long h, ByteBuffer buf, int pos, long n, int[] owned);
    private static native void accumulate(long h, int p, int target, double[] g);
    private static native void accumulateDirect(long h, int p, int target, ByteBuffer buf, int pos, long n, int kind);
    private static native long accumulateAsyncDirect(long h, int p, int target, ByteBuffer buf, int pos, long n,
                                                     int kind);
    private static native void waitTicket(long h, long ticket);
    private static native void flushQueued(long h);
    private static native int ingestTexts(long h, int target, byte[][] msgs, int layers, int[] parts, int[] status);
    private static native void accumulateFrame(long h, int p, int target, byte[] frame);
    private static native void updateIndirect(long h, int p, int target, ByteBuffer buf, int pos, long nBytes);
    private static native void finalizePartition(long h, int p, byte[] sumOut);
    private static native void finalizePartitionDirect(long h, int p, ByteBuffer sumOut, int pos);
    private static native void setWeightsDirect(long h, int p, ByteBuffer buf, int pos, long n);
    private static native void setWeightsFrame(long h, int p, byte[] frame);
    private static native void getPartitions(long h, double[] out);
    private static native void aggregateRound(long h, int pFirst, int nParts, double[] avgOut);
    private static native void promoteFuture(long h, int[] parts);
    private static native long commitPartialLen(long h, int p, int workers);
    private static native void commitPartial(long h, int p, int workers, byte[] out);
    private static native void accumulatePair(long h, int p, int target, byte[] file);
    private static native byte[] mergeFiles(long h, byte[][] files, boolean partialUpdates);
    private static native void otherReplicaDirect(long h, int p, int aggregator, int keyHash, ByteBuffer buf, int pos,
                                                  long n);
    private static native boolean otherReplicaDrop(long h, int p, int aggregator);
    private static native int[] replicaKeyOrder(long h);
    private static native int collectReplicas(long h, int[] participants);
    private static native void getPartitionsWire(long h, ByteBuffer direct, int pos, long nBytes);
    private static native ByteBuffer hostAllocDirect(int bytes);
}
