"""GPU parity of the multi-GPU handle (cfg.devices) and of the publish-side
codec, through the C-ABI.

The box has one MI355X, so the sharded handle runs with device lists like
[0, 0] or [0, 0, 0]: every shard is its own engine (own stream, own arena),
partitions are routed by the same contiguous-block plan as on eight GPUs, and
the replica-slot combine runs the same cross-shard event ordering and the
same owner-side fold kernel over the slots' partials -- only the xGMI hop is
missing (peer access is enabled between distinct devices at open).  It is
"unmeasured on hardware" beyond one GPU until the driver's 8-GPU run.

References: IPLS.java:1402-1468 (replica aggregators' partials, Collect_Replicas,
AggregatePartition), Updater.java:40-44 (REP fold), MyIPFSClass.java:990-1016
(Marshall_Packet), IPLS.java:1429-1430 (the publish call), IPLS.java:851-866
(ThreadReceiver decode).
"""
import numpy as np
import pytest

from conftest import assert_bits_equal

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ipls():
    if not torch.cuda.is_available():
        pytest.fail("-m gpu run without a visible GPU")
    import ipls as m
    return m


@pytest.fixture(scope="module")
def O():
    from oracle import oracle as o   # checker only
    return o


def dev_buckets(ipls, P, L, K, p0=0, k0=0, be=False, seed=None):
    from oracle import oracle as O
    t = torch.empty(P * K * (L + 2), dtype=torch.float64, device="cuda")
    base = (int(t.data_ptr()) + 15) // 16 * 16
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * (L + 2), L, big_endian=be) for k in range(K)]
            for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], p0 + q, k0 + k, O.SEED if seed is None else seed)
    torch.cuda.synchronize()
    return t, rows


def test_sharded_handle_routes_like_one_engine(ipls, O):
    """A model-geometry handle (M = 1,000,003, -pa 5) over shards [0, 0]
    (partitions 0-2 | 3-4) against the one-shard handle on the same calls:
    InitializeWeights, UpdateGradient over every shard, arrivals from host
    and device, a reduce_batch spanning both shards, AggregatePartition(all),
    GetPartitions (doubles, the Middleware wire stream, device), and the
    fused round with host averages."""
    M, P, K = 1_000_003, 5, 4
    one = ipls.Aggregator(M, P, max_peers=K)
    two = ipls.Aggregator(M, P, max_peers=K, devices=[0, 0])
    assert [two.partition_device(p)[0] for p in range(P)] == [0] * P
    assert ipls.shard_plan(P, 2) == [0, 0, 0, 1, 1]
    assert two.partition_device(0)[1] != two.partition_device(4)[1]   # one stream per shard
    model = O.synth_bucket(M, 9, 9)
    peers = [O.synth_bucket(M, 7, k) for k in range(K)]
    for agg in (one, two):
        agg.InitializeWeights(model)
        agg.UpdateGradient(peers[0], auth_list=[4, 0, 3, 1, 2])
        for k in (1, 2):
            parts = O.organize_gradients(peers[k], M, P)
            for p in range(P):
                agg.Update(O.be_encode(parts[p]) if k == 1 else parts[p], p)
    keep, rows = [], []
    parts3 = O.organize_gradients(peers[3], M, P)
    for p in range(P):
        t = torch.from_numpy(parts3[p]).to("cuda")
        keep.append(t)
        rows.append([ipls.DeviceBuffer.from_tensor(t)])
    for agg in (one, two):
        # rows have one bucket per partition but ragged lengths: one call per partition
        for p in range(P):
            agg.reduce_batch(p, [rows[p]], start_mode=ipls.START_ACCUM)
    for p in range(P):
        assert_bits_equal(two.read(p), one.read(p), f"AGG[{p}]")
        assert_bits_equal(two.read(p), O.reduce([O.organize_gradients(g, M, P)[p] for g in peers], one.lengths[p]),
                          f"oracle AGG[{p}]")
    for agg in (one, two):
        agg.AggregatePartition(ipls.ALL_PARTITIONS)
    assert_bits_equal(two.GetPartitions(), one.GetPartitions(), "GetPartitions")
    assert two.GetPartitions(wire=True) == one.GetPartitions(wire=True)
    flat = torch.empty(M, dtype=torch.float64, device="cuda")
    two.GetPartitions(out=ipls.DeviceBuffer.from_tensor(flat))
    two.sync()
    assert_bits_equal(flat.cpu().numpy(), one.GetPartitions(), "GetPartitions device")
    # fused round across both shards, host averages (one thread per shard)
    L = 50_001
    one2, two2 = ipls.Aggregator(n_partitions=4, bucket_len=L), ipls.Aggregator(n_partitions=4, bucket_len=L,
                                                                                devices=[0, 0])
    t, rws = dev_buckets(ipls, 4, L, 6)
    a1 = one2.aggregate_round(0, rws)
    a2 = two2.aggregate_round(0, rws)
    assert_bits_equal(a2, a1, "fused round averages")
    a3 = two2.aggregate_round(1, rws[1:3])        # a sub-range that straddles the shard boundary
    assert_bits_equal(a3, one2.aggregate_round(1, rws[1:3]), "straddling round")
    for agg in (one, two, one2, two2):
        agg.close()


def test_replica_slots_combine_in_slot_order(ipls, O):
    """Contributors of a partition spanning GPUs: the owner
    folds peers [0, 4), the other shard -- a replica aggregator of the same
    partitions -- folds peers [4, 8) into its partials; the combine adds the
    partial to REP and AggregatePartition gives W = AGG + (+0.0 + R), the
    oracle's replica checksum (IPLS.java:1256, Updater.java:40-44)."""
    P, L, K, kh = 4, 1_000_003, 8, 4
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, devices=[0, 0])
    t, rows = dev_buckets(ipls, P, L, K)
    own = [r[:kh] for r in rows]
    far = [r[kh:] for r in rows]
    agg.reduce_batch(0, own, start_mode=ipls.START_ZERO)
    # shard 1 is the replica of partitions 0-1, shard 0 of partitions 2-3
    agg.reduce_partial(1, 0, far[0:2])
    agg.reduce_partial(0, 2, far[2:4])
    with pytest.raises(ipls.IplsError):
        agg.reduce_partial(0, 0, far[0:1])        # shard 0 owns partition 0
    assert agg.combine_partials() == P
    assert agg.combine_partials() == 0           # consumed
    agg.AggregatePartition(ipls.ALL_PARTITIONS)
    for p in range(P):
        assert agg.checksum(p, ipls.TGT_WEIGHTS) == O.c_synth_replica_checksum(L, p, K, kh), p
    # the partial of a second round starts from +0.0 again
    agg.reduce_batch(0, own, start_mode=ipls.START_ZERO)
    agg.reduce_partial(1, 0, far[0:2])
    agg.reduce_partial(0, 2, far[2:4])
    agg.combine_partials(0, 4)
    agg.AggregatePartition(ipls.ALL_PARTITIONS)
    assert [agg.checksum(p, ipls.TGT_WEIGHTS) for p in range(P)] == \
        [O.c_synth_replica_checksum(L, p, K, kh) for p in range(P)]
    agg.close()


def test_three_slots_fold_order_and_accum(ipls, O):
    """Three shards, every partition with two remote slots: REP = ((+0.0 +
    R_a) + R_b) with a < b, on top of a REP that already holds a replica
    bucket; the partial of one slot built by two reduce_partial calls
    (ZERO, then ACCUM); BE buckets in one slot."""
    P, L = 3, 200_003
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, devices=[0, 0, 0])
    t, rows = dev_buckets(ipls, P, L, 6)
    tb, rows_be = dev_buckets(ipls, P, L, 6, be=True)
    b = [[O.synth_bucket(L, q, k) for k in range(6)] for q in range(P)]
    pre = [O.synth_bucket(L, 50 + q, 0) for q in range(P)]
    for q in range(P):
        agg.reduce_batch(q, [rows[q][0:2]], start_mode=ipls.START_ZERO)
        agg.Update(pre[q], q, from_clients=False)
        slots = [s for s in range(3) if s != q]
        agg.reduce_partial(slots[0], q, [rows[q][2:3]], start_mode=ipls.START_ZERO)
        agg.reduce_partial(slots[0], q, [rows[q][3:4]], start_mode=ipls.START_ACCUM)
        agg.reduce_partial(slots[1], q, [rows_be[q][4:6]], big_endian=True)
    assert agg.combine_partials() == 2 * P
    for q in range(P):
        agg_own = O.reduce(b[q][0:2], L)
        ra = O.reduce(b[q][2:4], L)
        rb = O.reduce(b[q][4:6], L)
        rep = ((0.0 + pre[q]) + ra) + rb
        assert_bits_equal(agg.read(q, ipls.TGT_REP), rep, f"REP[{q}]")
        s, _ = agg.AggregatePartition(q, with_sum=True, sum_big_endian=False)
        assert_bits_equal(s, agg_own + rep, f"W[{q}]")
    agg.close()


def test_sharded_ingest_indirect_async_and_replicas(ipls, O):
    """The rest of the surface on shards [0, 0]: pubsub ingest routed by the
    frame's partition field, hash-only requests through the handle's ONE
    Gradient_Buff (a short file folds the previous file's tail even when the
    two requests land on different shards), queued device arrivals with
    handle-wide tickets, Other_Replica_Gradients + Collect_Replicas with the
    Participants counts, and the promotion of future gradients."""
    M, P = 100_003, 4
    one = ipls.Aggregator(M, P, max_peers=4)
    two = ipls.Aggregator(M, P, max_peers=4, devices=[0, 0])
    Ls = one.lengths
    msgs = []
    for k in range(3):
        g = O.organize_gradients(O.synth_bucket(M, 3, k), M, P)
        for p in (3, 0, 2, 1):
            msgs.append(O.pubsub_message(O.frame_encode(g[p], p, 5, 3, b"QmX")))
    msgs.append(b"not base64!")                               # dropped: FORMAT
    msgs.append(O.pubsub_message(O.frame_encode(np.ones(9), 7, 5, 3, b"QmX")))   # partition 7: RANGE
    r1, r2 = one.ingest_pubsub(msgs), two.ingest_pubsub(msgs)
    assert r1 == r2 and r1[0] == 12 and r1[1][-2:] == [-6, -2]   # FORMAT, RANGE
    # hash-only requests, alternating shards, short files reuse the stale tail
    for p, n in ((3, Ls[3]), (0, Ls[0] - 50), (2, 10), (1, 0)):
        data = O.be_encode(O.synth_bucket(n, p, 11))
        one.UpdateIndirect(data, p)
        two.UpdateIndirect(data, p)
    # queued device arrivals on both shards
    t, rows = dev_buckets(ipls, P, max(Ls), 2)
    tickets = []
    for k in range(2):
        for p in range(P):
            b = ipls.DeviceBuffer(rows[p][k].ptr, Ls[p])
            one.UpdateAsync(b, p)
            tickets.append(two.UpdateAsync(b, p))
    two.Wait(tickets[-1])
    # Other_Replica_Gradients on both shards
    for agg in (one, two):
        for p, a in ((0, 7), (3, 2), (3, 9), (1, 2)):
            agg.OtherReplicaGradients(p, a, O.synth_bucket(Ls[p], p, a))
            agg.OtherReplicaGradients(p, a, O.synth_bucket(Ls[p] - 3, p, a + 1))
    c1, c2 = one.Collect_Replicas(), two.Collect_Replicas()
    # Participants increments: received x stored length per key (IPLS.java:1229-1234)
    assert c1 == c2 and c1[0] == 4 and c1[1] == [2 * Ls[0], 2 * Ls[1], 0, 4 * Ls[3]]
    for p in range(P):
        assert_bits_equal(two.read(p), one.read(p), f"AGG[{p}]")
        assert_bits_equal(two.read(p, ipls.TGT_REP), one.read(p, ipls.TGT_REP), f"REP[{p}]")
    # from-future fold and promotion on a subset spanning both shards
    for agg in (one, two):
        for p in range(P):
            agg.Update(O.synth_bucket(Ls[p], p, 33), p, from_future=True)
        agg.PromoteFuture([1, 3])
    for p in range(P):
        assert_bits_equal(two.read(p), one.read(p), f"promoted AGG[{p}]")
    one.close()
    two.close()


def test_staged_combine_and_indirect_without_peer_access(ipls, O, monkeypatch):
    """a device pair without xGMI peer access is not an
    error.  IPLS_PEER_STAGED=1 (read at open) forces the fallback on [0, 0, 0]:
    every remote partial is copied into an owner-side buffer on the owner's
    stream and the SAME fold reads it in the same slot order -- bit-identical
    to the oracle's replica expression; the hash-only requests' Gradient_Buff
    (on shard 0) is staged into the other shards the same way.  Two rounds, so
    the staging buffers are reused behind the `consumed` ordering."""
    monkeypatch.setenv("IPLS_PEER_STAGED", "1")
    P, L, K, kh = 3, 600_007, 6, 2
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, devices=[0, 0, 0])
    monkeypatch.delenv("IPLS_PEER_STAGED")
    t, rows = dev_buckets(ipls, P, L, K)
    for rnd in range(2):
        agg.reduce_batch(0, [r[:kh] for r in rows], start_mode=ipls.START_ZERO)
        for q in range(P):
            a, b = [s for s in range(3) if s != q]
            agg.reduce_partial(a, q, [rows[q][kh:kh + 2]])
            agg.reduce_partial(b, q, [rows[q][kh + 2:]])
        assert agg.combine_partials() == 2 * P
        assert agg.last_launch()["staged"] == 2 * P, rnd
        agg.AggregatePartition(ipls.ALL_PARTITIONS)
        for q in range(P):
            b = [O.synth_bucket(L, q, k) for k in range(K)]
            own = O.reduce(b[:kh], L)
            rep = (0.0 + O.reduce(b[kh:kh + 2], L)) + O.reduce(b[kh + 2:], L)
            assert_bits_equal(agg.read(q, ipls.TGT_WEIGHTS), own + rep, f"round {rnd} W[{q}]")
    # without the switch the same handle shape uses peer loads (nothing staged)
    plain = ipls.Aggregator(n_partitions=P, bucket_len=L, devices=[0, 0, 0])
    plain.reduce_partial(1, 0, [rows[0][kh:kh + 2]])
    assert plain.combine_partials() == 1 and plain.last_launch()["staged"] == 0
    plain.close()
    # hash-only requests through the staged Gradient_Buff vs a one-shard handle
    M = 300_001
    one = ipls.Aggregator(M, P)
    monkeypatch.setenv("IPLS_PEER_STAGED", "1")
    three = ipls.Aggregator(M, P, devices=[0, 0, 0])
    monkeypatch.delenv("IPLS_PEER_STAGED")
    Ls = one.lengths
    for p, n in ((2, Ls[2]), (0, Ls[0] - 70), (1, 33), (2, 5), (1, Ls[1])):
        data = O.be_encode(O.synth_bucket(n, p, 17))
        one.UpdateIndirect(data, p)
        three.UpdateIndirect(data, p)
    for p in range(P):
        assert_bits_equal(three.read(p), one.read(p), f"indirect AGG[{p}]")
    one.close()
    three.close()
    agg.close()


@pytest.mark.parametrize("staged", [False, True])
def test_combine_one_launch_per_owner_across_slots(ipls, O, monkeypatch, staged):
    """The spread replica plan (every owner pulls from all G-1 other GPUs):
    the partitions of one owner have their partials on DIFFERENT slots, one
    each.  The combine folds them in one launch per owner (per-partition
    pointer table), so on 8 GPUs an owner reads over all its links at once;
    here [0]*4, 3 partitions per owner of 4M (the half shape: 256 tiles per
    partition, so one launch over all three has a grid of 768).  Bit-exact against the
    oracle's replica expression, with peer loads and with staged copies."""
    if staged:
        monkeypatch.setenv("IPLS_PEER_STAGED", "1")
    G, Pg, L, K, kh = 4, 3, 4_194_304, 4, 2
    P = G * Pg
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, devices=[0] * G)
    monkeypatch.delenv("IPLS_PEER_STAGED", raising=False)
    t, rows = dev_buckets(ipls, P, L, K)
    slot = {o * Pg + q: (o + 1 + q % (G - 1)) % G for o in range(G) for q in range(Pg)}
    assert len({slot[q] for q in range(Pg)}) == Pg            # owner 0's partitions: three different slots
    agg.reduce_batch(0, [r[:kh] for r in rows], start_mode=ipls.START_ZERO)
    for p in range(P):
        agg.reduce_partial(slot[p], p, [rows[p][kh:]])
    assert agg.combine_partials() == P
    li = agg.last_launch()
    # the last owner's 3 partitions in one launch: 3 x 256 half tiles (one partition alone: 256)
    assert (li["kernel"], li["shape"], li["grid"]) == (ipls.KERNEL_REDUCE, ipls.SHAPE_HALF, Pg * 256), li
    assert li["staged"] == (P if staged else 0)
    agg.AggregatePartition(ipls.ALL_PARTITIONS)
    for p in range(P):
        assert agg.checksum(p, ipls.TGT_WEIGHTS) == O.c_synth_replica_checksum(L, p, K, kh), p
    agg.close()


def test_indirect_requests_from_two_threads_on_two_shards(ipls, O):
    """the handle's ONE Gradient_Buff lives on shard 0, so a
    hash-only request for a partition of shard 1 loads it there and folds it
    over on shard 1.  Two threads feed different files to a partition of each
    shard at once; each partition must receive exactly its own files (the
    load -> fold -> hand-back sequence is one critical section for every
    shard, shard 0 included).  Files are full length, so every partition's
    result is its own thread's fixed-order fold, whatever the interleaving."""
    import threading
    M, P, n_req = 400_004, 4, 24
    agg = ipls.Aggregator(M, P, devices=[0, 0])
    Ls = agg.lengths
    files = {p: [O.be_encode(O.synth_bucket(Ls[p], p, 100 + i)) for i in range(n_req)] for p in (0, 3)}
    errs = []

    def feed(p):
        try:
            for f in files[p]:
                agg.UpdateIndirect(f, p)
        except Exception as e:   # noqa: BLE001
            errs.append(e)
    th = [threading.Thread(target=feed, args=(p,)) for p in (0, 3)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    for p in (0, 3):
        want = O.reduce([np.frombuffer(f, dtype=">f8").astype(np.float64) for f in files[p]], Ls[p])
        assert_bits_equal(agg.read(p), want, f"AGG[{p}]")
    agg.close()


# ---------------------------------------------------------------------------
# a9: Marshall_Packet + Base64.getUrlEncoder on the device
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("L,origin", [(7, b""), (7, b"Q"), (7, b"Qm"),
                                      (100_000, b"QmPeerOrigin46charsxxxxxxxxxxxxxxxxxxxxxxxxxxx"),
                                      (1_048_581, b"QmY"), (1_048_580, b"QmY"),
                                      (13_000_001, b"QmZ")])   # > 16384 blocks: grid-stride
def test_publish_partial_matches_marshall_packet(ipls, O, L, origin):
    """ipls_agg_publish_partial = Base64.getUrlEncoder().encodeToString(frame)
    for the frame Marshall_Packet builds from Aggregated_Gradients[p]
    (MyIPFSClass.java:990-1016), as IPLS.java:1429-1430 calls it (a = the
    iteration, b = workers + 1, pid 3): every '=' padding case (frame length
    mod 3), the header-only and tail lanes, a logically-zero accumulator, and
    device output; and the round trip through the GPU ingest."""
    agg = ipls.Aggregator(n_partitions=2, bucket_len=L)
    # logically +0.0 accumulator (src == null path)
    z = agg.publish_partial(0, 12, 4, origin=origin)
    assert z == O.java_b64url_encode(O.frame_encode(np.zeros(L), 12, 4, 3, origin))
    vals = O.synth_bucket(L, 1, 2)
    vals[:3] = [-0.0, np.inf, 5e-324]
    agg.Update(vals, 1)
    text = agg.publish_partial(1, 12, 4, origin=origin)
    want = O.java_b64url_encode(O.frame_encode(agg.read(1), 12, 4, 3, origin))
    assert len(text) == len(want) and text == want
    # device text
    buf = torch.empty(len(want) + 16, dtype=torch.uint8, device="cuda")
    n = agg.publish_partial(1, 12, 4, origin=origin, out=int(buf.data_ptr()), out_cap=buf.numel())
    agg.sync()
    assert n == len(want) and bytes(buf[:n].cpu().numpy()) == want
    # an undersized device buffer is refused before anything is written:
    # a DeviceBuffer's size is its own, a raw address needs its capacity
    small = torch.full((len(want) + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    with pytest.raises(ValueError):
        agg.publish_partial(1, 12, 4, origin=origin, out=ipls.DeviceBuffer(int(small.data_ptr()), (len(want) - 1) // 8))
    with pytest.raises(ValueError):
        agg.publish_partial(1, 12, 4, origin=origin, out=int(small.data_ptr()))
    with pytest.raises(ValueError):
        agg.publish_partial(1, 12, 4, origin=origin, out=int(small.data_ptr()), out_cap=len(want) - 1)
    with pytest.raises(ValueError):
        agg.publish_partials([1], 12, [4], origin=origin, out=int(small.data_ptr()), out_cap=len(want) - 1)
    agg.sync()
    assert bool((small == 0xAB).all())
    # round trip: the IPFS daemon wraps the text once more (IPLS.java:855-859)
    rx = ipls.Aggregator(n_partitions=13, bucket_len=L)
    k, st = rx.ingest_pubsub([O.java_b64url_encode(text)], layers=2)   # routed by field a = 12
    assert (k, st) == (1, [0])
    assert_bits_equal(rx.read(12), 0.0 + agg.read(1), "round trip")
    k, st = rx.ingest_pubsub([text], layers=1, partitions=[0])
    assert (k, st) == (1, [0])
    assert_bits_equal(rx.read(0), 0.0 + agg.read(1), "round trip, one layer")
    rx.close()
    agg.close()


def test_publish_partial_rejects_bad_arguments(ipls):
    agg = ipls.Aggregator(n_partitions=1, bucket_len=10)
    with pytest.raises(ipls.IplsError):
        agg.publish_partial(1, 0, 0)
    import ctypes
    from ipls import _native as N
    lib = N.lib()
    need = lib.ipls_agg_publish_partial(agg.handle, 0, N.TGT_AGG, 0, 0, 3, None, 0, None, 0, N.HOST_TEXT)
    buf = (ctypes.c_uint8 * need)()
    out = ctypes.addressof(buf)
    assert need == 4 * -(-(14 + 8 * 10) // 3)
    assert lib.ipls_agg_publish_partial(agg.handle, 0, N.TGT_AGG, 0, 0, 3, None, 0, out, need - 1,
                                        N.HOST_TEXT) == N.IPLS_E_RANGE
    assert lib.ipls_agg_publish_partial(agg.handle, 0, N.TGT_AGG, 0, 0, 3, None, 0, out, need,
                                        N.HOST_F64) == N.IPLS_E_INVAL
    # device text into pageable host memory: rejected before any launch
    assert lib.ipls_agg_publish_partial(agg.handle, 0, N.TGT_AGG, 0, 0, 3, None, 0, out, need,
                                        N.DEV_TEXT) == N.IPLS_E_INVAL
    import numpy as _np
    parts, bs = _np.zeros(1, dtype=_np.int32), _np.ones(1, dtype=_np.int32)
    assert lib.ipls_agg_publish_partials(agg.handle, parts.ctypes.data, 1, N.TGT_AGG, 0, bs.ctypes.data, 3, None, 0,
                                         out, need, N.DEV_TEXT, None, None) == N.IPLS_E_INVAL
    agg.close()


# ---------------------------------------------------------------------------
# Full-size BASELINE geometries through the multi-device handle
# ---------------------------------------------------------------------------
def test_config_e_geometry_full_size(ipls, O):
    """Config E: -pa 64 sharded 16 per GPU over a
    four-entry device list ([0, 0, 0, 0] on this one-GPU box), 4M doubles,
    K = 32.  Round 1 (reduce_batch over all 64 partitions in one call, the
    launch split over the four shards): per-partition checksums against the
    C oracle at every shard boundary.  Round 2 (the replica exchange of
    config E, IPLS.java:1402-1468): the owner folds peers [0, 16), the next
    shard -- a replica aggregator of the same partitions -- folds peers
    [16, 32) into its partials, the combine adds them to REP over the
    cross-shard path, and W = AGG + (+0.0 + R) matches the oracle's replica
    checksum (Updater.java:40-44, IPLS.java:1256)."""
    P, L, K, G = 64, 4_194_304, 32, 4
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, devices=[0] * G)
    assert ipls.shard_plan(P, G) == [p // 16 for p in range(P)]
    t, rows = dev_buckets(ipls, P, L, K)
    check = [0, 15, 16, 31, 32, 47, 48, 63]
    agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
    for p in check:
        assert agg.checksum(p) == O.c_synth_sum_checksum(L, p, K), p
    kh = K // 2
    agg.reduce_batch(0, [r[:kh] for r in rows], start_mode=ipls.START_ZERO)
    for s in range(G):                        # shard s replicates shard (s-1)'s partitions
        o = (s - 1) % G
        agg.reduce_partial(s, 16 * o, [r[kh:] for r in rows[16 * o:16 * o + 16]])
    assert agg.combine_partials() == P
    agg.AggregatePartition(ipls.ALL_PARTITIONS)
    for p in check:
        assert agg.checksum(p, ipls.TGT_WEIGHTS) == O.c_synth_replica_checksum(L, p, K, kh), p
    agg.close()
    del t


def test_config_f_slice_full_size(ipls, O):
    """One GPU's slice of config F: 16 partitions x 8M doubles x 64 peers
    (69.8 GB of buckets resident), one reduce_batch, checksums of the first,
    a middle and the last partition against the C oracle."""
    P, L, K = 16, 8_388_608, 64
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    t, rows = dev_buckets(ipls, P, L, K)
    agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
    for p in (0, 7, 15):
        assert agg.checksum(p) == O.c_synth_sum_checksum(L, p, K), p
    agg.close()
    del t


def test_publish_partials_batch_matches_single(ipls, O):
    """ipls_agg_publish_partials: the publish loop over Auth_List
    (IPLS.java:1423-1431) in one launch per GPU.  Model geometry with a short
    last partition, partitions on both shards of [0, 0] in a mixed order, one
    partition logically +0.0, a distinct b per text; every text equals the
    single-partition call and Base64.getUrlEncoder(Marshall_Packet(...)), in
    host memory, pinned memory and device memory (64-B aligned offsets)."""
    M, P = 1_000_003, 5
    agg = ipls.Aggregator(M, P, devices=[0, 0])
    g = O.synth_bucket(M, 3, 1)
    agg.UpdateGradient(g, auth_list=[0, 1, 3, 4])          # partition 2 stays logically +0.0
    parts, bs = [4, 0, 2, 3, 1], [9, 2, 5, 7, 3]
    origin = b"QmBatchOrigin"
    texts = agg.publish_partials(parts, 12, bs, origin=origin)
    for p, b, t in zip(parts, bs, texts):
        want = O.java_b64url_encode(O.frame_encode(agg.read(p), 12, b, 3, origin))
        assert t == want, p
        assert t == agg.publish_partial(p, 12, b, origin=origin), p
    lens = [len(t) for t in texts]
    offs, pos = [], 0
    for n in lens:
        pos = (pos + 63) // 64 * 64
        offs.append(pos)
        pos += n
    # device memory
    dev = torch.zeros(pos + 64, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()   # torch's stream; the handle's stream does not order after it
    assert agg.publish_partials(parts, 12, bs, origin=origin, out=int(dev.data_ptr()),
                                out_cap=dev.numel()) == (lens, offs)
    agg.sync()
    host = dev.cpu().numpy().tobytes()
    for i, t in enumerate(texts):
        assert host[offs[i]:offs[i] + lens[i]] == t, parts[i]
    # pinned host memory
    pb = ipls.PinnedBuffer(pos)
    assert agg.publish_partials(parts, 12, bs, origin=origin, out=pb) == (lens, offs)
    v = pb.view()
    for i, t in enumerate(texts):
        assert v[offs[i]:offs[i] + lens[i]].tobytes() == t, parts[i]
    pb.close()
    # errors: a partition out of range, a buffer one byte short
    with pytest.raises(ipls.IplsError):
        agg.publish_partials([0, P], 1, [1, 1])
    from ipls import _native as N
    lib = N.lib()
    pa = np.array(parts, dtype=np.int32)
    ba = np.array(bs, dtype=np.int32)
    buf = np.empty(pos, dtype=np.uint8)
    assert lib.ipls_agg_publish_partials(agg.handle, pa.ctypes.data, len(parts), N.TGT_AGG, 12, ba.ctypes.data, 3,
                                         None, 0, buf.ctypes.data, 10, N.HOST_TEXT, None, None) == N.IPLS_E_RANGE
    agg.close()


def test_calls_keep_the_callers_current_device(ipls, O):
    """Every C-ABI call returns with the caller's current HIP device as it
    found it (include/ipls_agg.h conventions): a handle whose shards live on
    other GPUs must not switch a torch caller's device.  On a one-GPU box the
    handle runs over [0, 0] (shards still switch devices internally); with
    two or more GPUs the handle lives on the last device while the caller
    stays on device 0."""
    n = torch.cuda.device_count()
    devs = [0, 0] if n < 2 else [n - 1, n - 1]
    torch.cuda.set_device(0)
    before = torch.cuda.current_device()
    P, L, K = 4, 5003, 3
    with ipls.Aggregator(n_partitions=P, bucket_len=L, devices=devs) as agg:
        assert torch.cuda.current_device() == before
        g = O.synth_bucket(L, 0, 0)
        agg.Update(g, 0, from_clients=True)
        agg.Update(O.be_encode(g), P - 1, from_clients=True)
        agg.AggregatePartition(ipls.ALL_PARTITIONS)
        avg = agg.GetPartitions()
        agg.sync()
        assert torch.cuda.current_device() == before
    assert torch.cuda.current_device() == before
    ref = O.get_partitions([O.reduce([g], L) if p in (0, P - 1) else np.zeros(L) for p in range(P)])
    assert_bits_equal(avg, ref, "model")
