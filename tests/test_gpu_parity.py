"""GPU parity: the HIP path (through the C-ABI) against the oracle and the
committed golden fixtures.  Bit-exact for every element (NaN == NaN; payloads
unspecified by Java).  Parity status of the oracle itself: unpinned
 -- see oracle/__init__.py.
"""
import ctypes
import hashlib

import numpy as np
import pytest

from conftest import assert_bits_equal

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ipls():
    if not torch.cuda.is_available():
        pytest.fail("-m gpu run without a visible GPU")
    import ipls as _ipls
    return _ipls


@pytest.fixture(scope="module")
def O():
    from oracle import oracle
    return oracle


def dev(a: np.ndarray):
    """Host doubles -> device tensor (keeps the tensor alive) + DeviceBuffer."""
    import ipls
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to("cuda")
    return t, ipls.DeviceBuffer.from_tensor(t)


def dev_be(a: np.ndarray):
    import ipls
    raw = np.frombuffer(np.asarray(a, dtype=np.float64).astype(">f8").tobytes(), dtype=np.uint8).copy()
    t = torch.from_numpy(raw).to("cuda")
    return t, ipls.DeviceBuffer(int(t.data_ptr()), raw.size // 8, big_endian=True)


# ---------------------------------------------------------------------------
# synthetic buckets: device generator == oracle generator
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("L,p,k", [(1, 0, 0), (2, 1, 3), (1031, 3, 7), (70001, 15, 63)])
def test_synth_fill_matches_oracle(ipls, O, L, p, k):
    t = torch.empty(L, dtype=torch.float64, device="cuda")
    ipls.synth_fill(ipls.DeviceBuffer.from_tensor(t), p, k, O.SEED)
    torch.cuda.synchronize()
    assert_bits_equal(t.cpu().numpy(), O.synth_bucket(L, p, k), "synth")
    tb = torch.empty(8 * L, dtype=torch.uint8, device="cuda")
    ipls.synth_fill(ipls.DeviceBuffer(int(tb.data_ptr()), L, big_endian=True), p, k, O.SEED)
    torch.cuda.synchronize()
    assert bytes(tb.cpu().numpy()) == O.be_encode(O.synth_bucket(L, p, k))


def test_checksum_kernel_matches_oracle(ipls, O):
    rng = np.random.default_rng(7)
    for n in (0, 1, 63, 64, 65, 1000, 262147):
        x = rng.standard_normal(n)
        t, b = dev(x)
        assert ipls.checksum_dev(b) == O.checksum(x)
        tb, bb = dev_be(x)
        assert ipls.checksum_dev(bb) == O.checksum(x)


# ---------------------------------------------------------------------------
# batched reduce (the benchmarked kernel) vs golden synthetic cases
# ---------------------------------------------------------------------------
SMALL = [(3, 1, 2), (2, 2, 1), (4, 1031, 8), (2, 4096, 5), (1, 517, 33), (2, 70001, 3), (1, 262147, 12)]


@pytest.mark.parametrize("P,L,K", SMALL)
@pytest.mark.parametrize("be", [False, True])
def test_reduce_batch_synth(ipls, O, golden, golden_meta, P, L, K, be):
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    keep, rows = [], []
    for p in range(P):
        row = []
        for k in range(K):
            t, b = (dev_be if be else dev)(O.synth_bucket(L, p, k))
            keep.append(t)
            row.append(b)
        rows.append(row)
    for mode, name in [(ipls.START_ZERO, "zero"), (ipls.START_FIRST, "first")]:
        agg.reduce_batch(0, rows, start_mode=mode, big_endian=be)
        for p in range(P):
            got = agg.read(p)
            key = f"synth_P{P}_L{L}_K{K}_p{p}_{name}"
            if key in golden:
                assert_bits_equal(got, golden[key], key)
            else:
                assert O.checksum(got) == golden_meta["synth_checksum"][key], key
                assert agg.checksum(p) == golden_meta["synth_checksum"][key], key
    agg.close()


def test_reduce_batch_unaligned_buckets(ipls, O):
    """8-byte aligned (not 16) bucket views take the scalar kernel."""
    L, K = 3001, 4
    bufs = [O.synth_bucket(L, 0, k) for k in range(K)]
    big = torch.from_numpy(np.concatenate([np.zeros(1)] + [np.concatenate([b, [0.0]]) for b in bufs])).to("cuda")
    base = int(big.data_ptr()) + 8
    ptrs = [base + 8 * (L + 1) * k for k in range(K)]
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L)
    agg.reduce_batch(0, [ptrs], start_mode=ipls.START_ZERO)
    assert_bits_equal(agg.read(0), O.reduce(bufs, L), "unaligned")
    agg.close()


# ---------------------------------------------------------------------------
# edge cases: signed zero, cancellation order, subnormals, inf/NaN
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("case", ["szero", "cancel", "special"])
def test_edge_fold_host_and_device(ipls, O, golden, case):
    bufs = golden[f"{case}_bufs"]
    L = bufs.shape[1]
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L)
    # host arrivals one by one (Updater._Update), accumulator starts at +0.0
    for b in bufs:
        agg.Update(b, 0, from_clients=True)
    assert_bits_equal(agg.read(0), golden[f"{case}_zero"], f"{case} host")
    # device batch, ZERO and FIRST
    keep = [dev(b) for b in bufs]
    agg.reduce_batch(0, [[d for _, d in keep]], start_mode=ipls.START_ZERO)
    assert_bits_equal(agg.read(0), golden[f"{case}_zero"], f"{case} dev zero")
    if f"{case}_first" in golden:
        agg.reduce_batch(0, [[d for _, d in keep]], start_mode=ipls.START_FIRST)
        assert_bits_equal(agg.read(0), golden[f"{case}_first"], f"{case} dev first")
    # big-endian file bytes (GetParameters input)
    agg.reset(0)
    for b in bufs:
        agg.Update(O.be_encode(b), 0)
    assert_bits_equal(agg.read(0), golden[f"{case}_zero"], f"{case} BE")
    agg.close()


def test_accumulate_equals_batch(ipls, O):
    """K arrivals via accumulate (ACCUM) == one ZERO batch == oracle."""
    L, K = 9001, 11
    bufs = [O.synth_bucket(L, 2, k) for k in range(K)]
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L)
    keep = [dev(b) for b in bufs]
    for _, d in keep:
        agg.Update(d, 0)
    a1 = agg.read(0)
    agg.reduce_batch(0, [[d for _, d in keep]], start_mode=ipls.START_ZERO)
    a2 = agg.read(0)
    ref = O.reduce(bufs, L)
    assert_bits_equal(a1, ref, "accum")
    assert_bits_equal(a2, ref, "batch")
    # ACCUM on top of an existing value
    agg.reduce_batch(0, [[d for _, d in keep[:3]]], start_mode=ipls.START_ACCUM)
    assert_bits_equal(agg.read(0), O.reduce(bufs[:3], L, O.START_ACCUM, acc=ref), "accum2")
    agg.close()


def test_frame_update(ipls, O, golden):
    """Pubsub frame (MyIPFSClass.java:990-1017) decoded and folded."""
    fr = bytes(golden["frame_bytes"])
    g = golden["frame_g"]
    assert ipls.frame_encode(g, 7, 42, 3, b"QmPeerOrigin") == fr
    pid, n, a, b, po, oo = ipls.frame_parse(fr)
    assert (pid, n, a, b, po, oo) == (3, 4, 7, 42, 14, 14 + 32)
    agg = ipls.Aggregator(n_partitions=1, bucket_len=4)
    agg.Update(fr, 0, frame=True)
    agg.Update(fr, 0, frame=True)
    assert_bits_equal(agg.read(0), O.reduce([g, g], 4), "frame fold")
    # empty frame -> null gradient -> no-op (MyIPFSClass.java:1449-1451)
    agg.Update(O.frame_encode(None, 7, 42, 3, b"x"), 0, frame=True)
    assert_bits_equal(agg.read(0), O.reduce([g, g], 4), "empty frame")
    with pytest.raises(ipls.IplsError) as e:
        agg.Update(fr[:20], 0, frame=True)
    assert e.value.java_name == "BufferUnderflow"
    agg.close()


# ---------------------------------------------------------------------------
# divide / finalize / GetPartitions
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("case,secure", [("div", False), ("div_zero", False), ("div_nzero", False),
                                         ("div_secure", True)])
def test_divide(ipls, golden, case, secure):
    w = golden[f"{case}_w"]
    L = len(w)
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L, secure=secure)
    agg.cache_partition(0, w)
    assert_bits_equal(agg.GetPartitions(), golden[f"{case}_out"], case)
    agg.close()


def test_finalize_with_replicas(ipls, O):
    """W = AGG + REP (IPLS.java:1256), Weight_Address = W, then zeroed."""
    L = 5003
    own = [O.synth_bucket(L, 1, k) for k in range(4)]
    reps = [O.synth_bucket(L, 9, k) for k in range(3)]
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L)
    for b in own:
        agg.Update(b, 0, from_clients=True)
    for r in reps:
        agg.Update(r, 0, from_clients=False)
    s, a = agg.AggregatePartition(0, with_sum=True, sum_big_endian=True, with_average=True)
    S = O.reduce(own, L) + O.reduce(reps, L)
    assert bytes(s) == O.be_encode(S)
    assert_bits_equal(a, O.divide(S), "avg")
    assert_bits_equal(agg.read(0, ipls.TGT_WEIGHTS), S, "weights")
    assert_bits_equal(agg.read(0, ipls.TGT_WADDR), S, "weight_address")
    assert not agg.read(0, ipls.TGT_AGG).any() and not agg.read(0, ipls.TGT_REP).any()
    # next round starts from +0.0
    agg.Update(own[0], 0)
    assert_bits_equal(agg.read(0), O.reduce(own[:1], L), "next round")
    agg.close()


def test_config_a_ethmodel(ipls, O, ethmodel, golden_meta):
    """BASELINE configs[0]: ETHModel, -pa 3 -n 3, three peers, full API flow."""
    meta = golden_meta["config_a"]
    M = meta["model_size"]
    peers = [ethmodel + O.synth_bucket(M + 1, 0, k)[:M] for k in range(3)]
    agg = ipls.Aggregator(M, 3, max_peers=3)
    assert agg.lengths == meta["partition_len"]
    agg.InitializeWeights(ethmodel)
    # before any aggregation the count slot is 0.0 -> model passes through
    assert_bits_equal(agg.GetPartitions(), ethmodel, "initial model")
    # peer 0 is this aggregator (UpdateGradient own-accumulate); 1, 2 arrive
    agg.UpdateGradient(peers[0], auth_list=[0, 1, 2])
    for k in (1, 2):
        parts = agg.OrganizeGradients(peers[k], big_endian_out=(k == 2))
        for p in range(3):
            agg.Update(parts[p], p, from_clients=True)
    for p in range(3):
        s, _ = agg.AggregatePartition(p, with_sum=True)
        assert hashlib.sha256(bytes(s)).hexdigest() == meta["sum_sha256"][p]
    avg = agg.GetPartitions()
    assert hashlib.sha256(avg.astype(">f8").tobytes()).hexdigest() == meta["avg_sha256"]
    wire = agg.GetPartitions(wire=True)
    assert hashlib.sha256(wire).hexdigest() == meta["wire_sha256"]
    agg.close()


def test_organize_gradients_geometry(ipls, O, golden):
    for M, P, tag in [(10, 4, "org10x4"), (12, 4, "org12x4")]:
        flat = np.arange(1.0, M + 1.0)
        agg = ipls.Aggregator(M, P)
        parts = agg.OrganizeGradients(flat)
        for p in range(P):
            assert_bits_equal(parts[p], golden[f"{tag}_p{p}"], f"{tag} p{p}")
        agg.close()


def test_split_device_and_be(ipls, O):
    M, P = 100003, 7
    flat = O.synth_bucket(M, 4, 4)
    ref = O.organize_gradients(flat, M, P)
    agg = ipls.Aggregator(M, P)
    t, d = dev(flat)
    for p in range(P):
        L = agg.lengths[p]
        out = torch.empty(L, dtype=torch.float64, device="cuda")
        import ctypes
        ipls.lib().ipls_agg_split(agg.handle, d.ptr, M, ipls.DEV_F64, p, ctypes.c_void_p(out.data_ptr()),
                                  ipls.DEV_F64)
        agg.sync()
        assert_bits_equal(out.cpu().numpy(), ref[p], f"dev split {p}")
    be = agg.OrganizeGradients(flat.astype(">f8"), big_endian_out=True)
    for p in range(P):
        assert bytes(be[p]) == O.be_encode(ref[p])
    agg.close()


@pytest.mark.parametrize("devices", [None, [0, 0], [0, 0, 0]])
def test_get_partitions_chunked(ipls, O, devices):
    """ipls_agg_get_partitions_chunked: GetPartitions (IPLS.java:1159-1174)
    delivered to a sink chunk by chunk, in model order, on the calling thread;
    the chunks tile [0, M) exactly and carry the bits of the oracle's model,
    for chunks of 2 doubles, an odd chunk count, and one chunk larger than the
    model, on one- and multi-shard handles (shard segments in order).  A sink
    that returns non-zero stops the transfer; an odd chunk is refused."""
    from ipls import _native as N
    M, P = 300007, 3
    agg = ipls.Aggregator(M, P, devices=devices)
    lib, h = agg._lib, agg._h
    flats = [O.synth_bucket(M, 6, k) for k in range(2)]
    for g in flats:
        agg.UpdateGradient(g, range(P))
    for p in range(P):
        agg.AggregatePartition(p)
    parts = [O.organize_gradients(g, M, P) for g in flats]
    want = O.get_partitions([O.reduce([pt[p] for pt in parts], agg.lengths[p]) + 0.0 for p in range(P)])
    for chunk in (65536, 2, 100002, 1 << 22):
        got = np.full(M, np.nan)
        seen = []

        @N.CHUNK_SINK
        def sink(ctx, vals, off, n):
            got[off:off + n] = np.ctypeslib.as_array(vals, shape=(n,))
            seen.append((off, n))
            return 0
        if chunk == 2:                            # 150,004 sink calls: check a slice only
            got_small = []

            @N.CHUNK_SINK
            def sink(ctx, vals, off, n):          # noqa: F811
                if off < 1000:
                    got_small.append((off, vals[0], vals[1]))
                seen.append((off, n))
                return 0
            assert lib.ipls_agg_get_partitions_chunked(h, chunk, sink, None) == 0
            assert [o for o, _ in seen] == sorted(o for o, _ in seen) and sum(n for _, n in seen) == M
            assert all(want[o] == a and want[o + 1] == b for o, a, b in got_small)
            continue
        assert lib.ipls_agg_get_partitions_chunked(h, chunk, sink, None) == 0
        assert [o for o, _ in seen] == sorted(o for o, _ in seen)
        assert sum(n for _, n in seen) == M and all(n <= chunk for _, n in seen)
        assert_bits_equal(got, want, f"chunk {chunk}")
    calls = []

    @N.CHUNK_SINK
    def stop(ctx, vals, off, n):
        calls.append(off)
        return 1 if len(calls) == 2 else 0
    assert lib.ipls_agg_get_partitions_chunked(h, 65536, stop, None) == N.IPLS_E_INVAL
    assert calls == [0, 65536]
    assert lib.ipls_agg_get_partitions_chunked(h, 65537, stop, None) == N.IPLS_E_INVAL
    assert_bits_equal(agg.GetPartitions(), want, "model after a stopped transfer")
    agg.close()


@pytest.mark.parametrize("M,P,devices", [(443610, 3, None), (50001, 5, None), (10, 4, None), (100003, 7, [0, 0, 0]),
                                         (7, 8, [0, 0])])
def test_flat_size_and_offsets(ipls, O, M, P, devices):
    """ipls_agg_flat_size (what the JNI getPartitions copies back) is the
    model size, and partition_offset / partition_len follow the chunk rule
    (IPLS.java:1019-1029), on one- and multi-shard handles; in (7, 8) the
    last partition holds only its count slot (L_p = 1)."""
    agg = ipls.Aggregator(M, P, devices=devices)
    n = ctypes.c_int64()
    assert agg._lib.ipls_agg_flat_size(agg._h, ctypes.byref(n)) == 0
    assert n.value == agg.flat_size == M
    c = O.chunk_size(M, P)
    assert agg.offsets == [p * c for p in range(P)]
    assert agg.lengths == [O.partition_len(M, P, p) for p in range(P)]
    agg.close()


def test_update_gradient_owned_subset(ipls, O):
    M, P = 50001, 5
    g1, g2 = O.synth_bucket(M, 0, 1), O.synth_bucket(M, 0, 2)
    agg = ipls.Aggregator(M, P)
    agg.UpdateGradient(g1, [1, 3])
    agg.UpdateGradient(None, [1, 3])      # did not train in time: no-op
    agg.UpdateGradient(g2, [3])
    r1, r2 = O.organize_gradients(g1, M, P), O.organize_gradients(g2, M, P)
    assert_bits_equal(agg.read(1), O.reduce([r1[1]], agg.lengths[1]), "p1")
    assert_bits_equal(agg.read(3), O.reduce([r1[3], r2[3]], agg.lengths[3]), "p3")
    assert not agg.read(0).any()
    agg.close()


def test_merge_first_start(ipls, O, golden):
    """Storage-node merge starts from g0 (keeps -0.0), returns BE file bytes."""
    bufs = golden["szero_bufs"]
    st = ipls.Aggregator(n_partitions=1, bucket_len=bufs.shape[1])
    keep = [dev_be(b) for b in bufs]
    out = st.Merge(0, [d for _, d in keep])
    assert out == O.be_encode(golden["szero_first"])
    st.close()


# ---------------------------------------------------------------------------
# errors (the reference's exceptions)
# ---------------------------------------------------------------------------
def test_errors(ipls, O):
    with pytest.raises(ipls.IplsError) as e:
        ipls.Aggregator(10, 7)          # chunk 2, partition 6 length -1
    assert e.value.java_name == "NegativeArraySize"
    agg = ipls.Aggregator(n_partitions=2, bucket_len=100)
    with pytest.raises(ipls.IplsError) as e:
        agg.Update(np.zeros(99), 0)
    assert e.value.java_name == "ArrayIndexOutOfBounds"
    with pytest.raises(ipls.IplsError):
        agg.Update(np.zeros(100), 2)
    with pytest.raises(ipls.IplsError):
        agg.cache_partition(0, np.zeros(101))
    t = torch.empty(2 * 100 + 2, dtype=torch.float64, device="cuda")
    with pytest.raises(ipls.IplsError):   # device outputs must be 8-B aligned
        agg.GetPartitions(out=ipls.DeviceBuffer(int(t.data_ptr()) + 4, 2 * 99))
    agg.Update(np.ones(100), 1)            # still usable after errors
    assert agg.read(1).sum() == 100.0
    agg.close()


def test_invalid_arguments_rejected_before_launch(ipls, O):
    """Bad arguments at every C-ABI entry come back as negative codes before
    any device work (so no kernel ever sees them), and the handle keeps its
    state: the reference's exceptions leave PeerData intact too."""
    import ctypes
    from ipls import _native as N
    lib = ipls.lib()
    L = 1000
    agg = ipls.Aggregator(n_partitions=2, bucket_len=L)
    h = agg.handle
    g = O.synth_bucket(L, 0, 1)
    agg.Update(g, 0)
    t = torch.from_numpy(np.asarray(g)).to("cuda")
    torch.cuda.synchronize()
    d = int(t.data_ptr())
    P = ctypes.c_void_p
    tab = (P * 2)(d, d)
    nul = (P * 2)(d, None)
    mis = (P * 2)(d, d + 4)
    tk = ctypes.c_uint64()
    out = np.zeros(2 * L)
    msg = np.frombuffer(O.pubsub_message(O.frame_encode(g, 0, 1, 3, b"Qm")), dtype=np.uint8)
    mp = (P * 1)(msg.ctypes.data)
    ml = (ctypes.c_int64 * 1)(msg.size)
    cases = {
        "reduce_batch p_first -1": lambda: lib.ipls_agg_reduce_batch(h, -1, 1, tab, 2, N.DEV_F64, N.START_ACCUM, N.TGT_AGG),
        "reduce_batch past P": lambda: lib.ipls_agg_reduce_batch(h, 1, 2, tab, 1, N.DEV_F64, N.START_ACCUM, N.TGT_AGG),
        "reduce_batch host kind": lambda: lib.ipls_agg_reduce_batch(h, 0, 1, tab, 2, N.HOST_F64, N.START_ACCUM, N.TGT_AGG),
        "reduce_batch start 7": lambda: lib.ipls_agg_reduce_batch(h, 0, 1, tab, 2, N.DEV_F64, 7, N.TGT_AGG),
        "reduce_batch target 9": lambda: lib.ipls_agg_reduce_batch(h, 0, 1, tab, 2, N.DEV_F64, N.START_ACCUM, 9),
        "reduce_batch k -1": lambda: lib.ipls_agg_reduce_batch(h, 0, 1, tab, -1, N.DEV_F64, N.START_ACCUM, N.TGT_AGG),
        "reduce_batch NULL table": lambda: lib.ipls_agg_reduce_batch(h, 0, 1, None, 2, N.DEV_F64, N.START_ACCUM, N.TGT_AGG),
        "reduce_batch NULL bucket": lambda: lib.ipls_agg_reduce_batch(h, 0, 1, nul, 2, N.DEV_F64, N.START_ACCUM, N.TGT_AGG),
        "reduce_batch 4-B aligned": lambda: lib.ipls_agg_reduce_batch(h, 0, 1, mis, 2, N.DEV_F64, N.START_ACCUM, N.TGT_AGG),
        "accumulate p 2": lambda: lib.ipls_agg_accumulate(h, 2, N.TGT_AGG, d, L, N.DEV_F64),
        "accumulate target 9": lambda: lib.ipls_agg_accumulate(h, 0, 9, d, L, N.DEV_F64),
        "accumulate kind 99": lambda: lib.ipls_agg_accumulate(h, 0, N.TGT_AGG, d, L, 99),
        "accumulate short": lambda: lib.ipls_agg_accumulate(h, 0, N.TGT_AGG, d, L - 1, N.DEV_F64),
        "async 4-B aligned": lambda: lib.ipls_agg_accumulate_async(h, 0, N.TGT_AGG, d + 4, L, N.DEV_F64, ctypes.byref(tk)),
        "async short": lambda: lib.ipls_agg_accumulate_async(h, 0, N.TGT_AGG, d, L - 1, N.DEV_F64, ctypes.byref(tk)),
        "async NULL ticket": lambda: lib.ipls_agg_accumulate_async(h, 0, N.TGT_AGG, d, L, N.DEV_F64, None),
        "async p -1": lambda: lib.ipls_agg_accumulate_async(h, -1, N.TGT_AGG, d, L, N.DEV_F64, ctypes.byref(tk)),
        "wait unissued": lambda: lib.ipls_agg_wait(h, 1 << 40),
        "finalize p 5": lambda: lib.ipls_agg_finalize(h, 5, None, N.HOST_BE, None),
        "read kind 99": lambda: lib.ipls_agg_read(h, 0, N.TGT_AGG, out.ctypes.data, L, 99),
        "read p 2": lambda: lib.ipls_agg_read(h, 2, N.TGT_AGG, out.ctypes.data, L, N.HOST_F64),
        "ingest layers 3": lambda: lib.ipls_agg_ingest_pubsub(h, N.TGT_AGG, mp, ml, 1, 3, None, None),
        "ingest n -1": lambda: lib.ipls_agg_ingest_pubsub(h, N.TGT_AGG, mp, ml, -1, 2, None, None),
        "ingest target 9": lambda: lib.ipls_agg_ingest_pubsub(h, 9, mp, ml, 1, 2, None, None),
        "blend target 9": lambda: lib.ipls_agg_blend(h, 0, 9, d, L, N.DEV_F64, 0.5, 0.5),
        "promote p 4": lambda: lib.ipls_agg_promote_future(h, (ctypes.c_int32 * 1)(4), 1),
        "reset p 3": lambda: lib.ipls_agg_reset(h, 3),
    }
    for name, call in cases.items():
        rc = call()
        assert rc < 0, f"{name}: rc {rc}"
    for bad in (dict(n_partitions=0, bucket_len=10), dict(n_partitions=2, bucket_len=-5)):
        with pytest.raises(ipls.IplsError):
            ipls.Aggregator(**bad)
    with pytest.raises(ipls.IplsError) as e:
        ipls.Aggregator(n_partitions=1, bucket_len=1 << 46)    # 512 TiB arena
    assert e.value.code == N.IPLS_E_NOMEM
    agg.Update(g, 0)                          # state intact: exactly the two good folds
    assert_bits_equal(agg.read(0), O.reduce([g, g], L), "after rejected calls")
    agg.close()


# ---------------------------------------------------------------------------
# full-size configs: size-independent property (checksum of the fixed-order
# sum, computed by the C oracle from the counter formula at build time)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("cfg", ["B", "C"])
def test_full_size_checksums(ipls, golden_meta, cfg):
    m = golden_meta["full"][cfg]
    P, L, K = m["partitions"], m["bucket_len"], m["peers"]
    arena = torch.empty(P * K * L, dtype=torch.float64, device="cuda")
    base = int(arena.data_ptr())
    rows = []
    for p in range(P):
        row = []
        for k in range(K):
            b = ipls.DeviceBuffer(base + 8 * (p * K + k) * L, L)
            ipls.synth_fill(b, p, k, golden_meta["seed"])
            row.append(b)
        rows.append(row)
    torch.cuda.synchronize()
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
    li = agg.last_launch()
    # the launch the bench measures: C's 2048 big tiles; B's 512 run the half shape (512 lanes)
    assert (li["shape"], li["block"], li["vectors"], li["map"]) == \
        ((ipls.SHAPE_HALF, 512, 16, 0) if cfg == "B" else (ipls.SHAPE_BIG, 1024, 16, 0)), li
    got = [agg.checksum(p) for p in range(P)]
    assert got == m["sum_checksum"]
    agg.close()
    del arena
    torch.cuda.empty_cache()


def test_big_shape_with_partial_tile(ipls, O):
    """Batches large enough for the 64-KiB-per-block shape, with an odd
    length: full tiles + 512-element vector steps + a scalar remainder."""
    P, L, K = 4, 4200001, 3
    arena = torch.empty(P * K * (L + 1), dtype=torch.float64, device="cuda")
    base = int(arena.data_ptr())
    rows = [[ipls.DeviceBuffer(base + 8 * (p * K + k) * (L + 1), L) for k in range(K)] for p in range(P)]
    for p in range(P):
        for k in range(K):
            ipls.synth_fill(rows[p][k], p, k, O.SEED)
    torch.cuda.synchronize()
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
    assert [agg.checksum(p) for p in range(P)] == [O.c_synth_sum_checksum(L, p, K) for p in range(P)]
    # ACCUM on top: S + S (fold of the same buckets again) vs oracle on one partition
    agg.reduce_batch(0, rows, start_mode=ipls.START_ACCUM)
    s0 = agg.read(0)
    ref = O.reduce([O.synth_bucket(L, 0, k) for k in range(K)], L)
    ref2 = O.reduce([O.synth_bucket(L, 0, k) for k in range(K)], L, O.START_ACCUM, acc=ref)
    assert_bits_equal(s0, ref2, "accum twice")
    agg.close()
    del arena
    torch.cuda.empty_cache()


def test_reduce_batch_out_fused_pack(ipls, O):
    """BE buckets in, BE sum bytes out (config D's pack/unpack) and the
    storage-node merge (FIRST start) into caller buffers."""
    P, L, K = 3, 20001, 5
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    keep, rows, outs = [], [], []
    for p in range(P):
        row = []
        for k in range(K):
            t, b = dev_be(O.synth_bucket(L, p, k))
            keep.append(t)
            row.append(b)
        rows.append(row)
        o = torch.empty(8 * L, dtype=torch.uint8, device="cuda")
        outs.append(o)
    for mode in (ipls.START_ZERO, ipls.START_FIRST):
        agg.reduce_batch_out(0, rows, [int(o.data_ptr()) for o in outs], start_mode=mode,
                             big_endian_in=True, big_endian_out=True)
        agg.sync()
        for p in range(P):
            ref = O.reduce([O.synth_bucket(L, p, k) for k in range(K)], L, mode)
            assert bytes(outs[p].cpu().numpy()) == O.be_encode(ref)
    # native doubles out, ACCUM on top of the previous FIRST result
    o64 = [torch.from_numpy(O.reduce([O.synth_bucket(L, p, k) for k in range(K)], L)).to("cuda") for p in range(P)]
    agg.reduce_batch_out(0, rows, [int(o.data_ptr()) for o in o64], start_mode=ipls.START_ACCUM,
                         big_endian_in=True)
    agg.sync()
    for p in range(P):
        s = O.reduce([O.synth_bucket(L, p, k) for k in range(K)], L)
        assert_bits_equal(o64[p].cpu().numpy(), O.reduce([O.synth_bucket(L, p, k) for k in range(K)], L,
                                                         O.START_ACCUM, acc=s), "accum out")
    agg.close()


def test_pinned_host_operands(ipls, O):
    """Host buckets in pinned memory (ipls_host_alloc) take the direct DMA path."""
    L, K = 300007, 4                       # > 1 MiB per bucket
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L)
    bufs = []
    for k in range(K):
        pb = ipls.PinnedBuffer(8 * L)
        pb.view()[:] = np.frombuffer(O.be_encode(O.synth_bucket(L, 0, k)), dtype=np.uint8)
        bufs.append(pb)
    for pb in bufs:
        agg.Update(pb.view(), 0)
        pb.view()[:] = 0                     # caller may reuse the buffer at once
    assert_bits_equal(agg.read(0), O.reduce([O.synth_bucket(L, 0, k) for k in range(K)], L), "pinned")
    for pb in bufs:
        pb.close()
    agg.close()


def test_pinned_zero_copy_long_bucket_and_pinned_sum(ipls, O):
    """Zero-copy single-bucket folds from pinned memory run on 128 workgroups:
    a 2,000,003-double bucket takes several grid-stride passes plus the odd
    tail.  The BE sum is written into a caller PinnedBuffer (sum_out)."""
    L = 2000003
    vals = [O.synth_bucket(L, 9, k) for k in range(3)]
    bufs = []
    for v in vals:
        pb = ipls.PinnedBuffer(8 * L)
        pb.view()[:] = np.frombuffer(O.be_encode(v), dtype=np.uint8)
        bufs.append(pb)
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L)
    agg.Update(bufs[0].view(), 0)                   # synchronous zero copy
    t = agg.UpdateAsync(bufs[1], 0)                 # queued zero copy
    agg.Update(bufs[2].view(), 0)
    agg.Wait(t)
    out = ipls.PinnedBuffer(8 * L)
    s, _ = agg.AggregatePartition(0, sum_out=out)
    ref = O.reduce(vals, L)
    assert s.nbytes == 8 * L
    assert bytes(s) == O.be_encode(ref)
    assert_bits_equal(np.frombuffer(bytes(out.view()), dtype=">f8").astype(np.float64), ref, "pinned sum_out")
    with pytest.raises(ValueError):
        agg.AggregatePartition(0, sum_out=ipls.PinnedBuffer(8))
    agg.close()
    for pb in [*bufs, out]:
        pb.close()


def test_export_import_partial(ipls, O):
    """The GPU half of the replica exchange: a replica's partial leaves through
    export_partial (AGG -> device tensor) and the owner folds it into REP;
    finalize gives AGG_own + ((+0.0 + R1) + R2) (IPLS.java:1256)."""
    L = 70003
    owner = ipls.Aggregator(n_partitions=1, bucket_len=L)
    reps = [ipls.Aggregator(n_partitions=1, bucket_len=L) for _ in range(2)]
    own_b = [O.synth_bucket(L, 5, k) for k in range(3)]
    rep_b = [[O.synth_bucket(L, 6 + r, k) for k in range(2)] for r in range(2)]
    for b in own_b:
        owner.Update(b, 0)
    partials = []
    for r, agg in enumerate(reps):
        for b in rep_b[r]:
            agg.Update(b, 0)
        t = torch.empty(L, dtype=torch.float64, device="cuda")
        agg.export_partial(0, t)
        partials.append(t)
    for t in partials:
        owner.import_partial(0, t)
    s, _ = owner.AggregatePartition(0, with_sum=True, sum_big_endian=False)
    R = [O.reduce(rb, L) for rb in rep_b]
    assert_bits_equal(s, O.reduce(own_b, L) + O.reduce(R, L), "replica combine")
    # replace_agg: the partial becomes AGG exactly (FIRST start keeps -0.0)
    neg = torch.full((L,), -0.0, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()   # torch's stream; the handle's stream does not order after it
    owner.import_partial(0, neg, replace_agg=True)
    assert np.signbit(owner.read(0)).all()
    for a in [owner, *reps]:
        a.close()


def test_concurrent_threads_one_handle(ipls, O):
    """The Updater thread and the daemon thread share one handle (PeerData.mtx
    in the reference): concurrent Update calls on different partitions and
    own-accumulates must give the sequential result per partition."""
    import threading
    M, P = 40003, 4
    agg = ipls.Aggregator(M, P)
    peers = [O.synth_bucket(M, 9, k) for k in range(6)]
    parts = [O.organize_gradients(g, M, P) for g in peers]
    errs = []

    def arrivals(p):
        try:
            for k in range(6):
                agg.Update(parts[k][p], p)
        except Exception as e:   # pragma: no cover
            errs.append(e)

    ths = [threading.Thread(target=arrivals, args=(p,)) for p in range(P)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs
    for p in range(P):
        assert_bits_equal(agg.read(p), O.reduce([parts[k][p] for k in range(6)], agg.lengths[p]), f"p{p}")
    agg.close()


def test_degenerate_batches(ipls, O):
    L = 1001
    agg = ipls.Aggregator(n_partitions=2, bucket_len=L)
    t, d = dev(O.synth_bucket(L, 0, 0))
    agg.Update(np.ones(L), 0)
    agg.reduce_batch(0, [[], []], start_mode=ipls.START_ACCUM)          # k=0 ACCUM: unchanged
    assert (agg.read(0) == 1.0).all()
    agg.reduce_batch(0, [[], []], start_mode=ipls.START_ZERO)           # k=0 ZERO: +0.0
    assert not agg.read(0).any() and not np.signbit(agg.read(0)).any()
    agg.reduce_batch(1, [[d]], start_mode=ipls.START_FIRST)             # k=1 FIRST: exact copy
    assert_bits_equal(agg.read(1), O.synth_bucket(L, 0, 0), "first k=1")
    agg.reset()
    assert not agg.read(1).any()
    # GetPartitions before any aggregation: all-zero weights, count 0.0 -> zeros
    assert not agg.GetPartitions().any()
    agg.close()


def test_many_partitions_small_buckets(ipls, O):
    """-pa much larger than the GPU: 300 partitions of an odd model size in
    one batch launch (small shape), vs the oracle."""
    M, P, K = 100003, 300, 3
    agg = ipls.Aggregator(M, P)
    flats = [O.synth_bucket(M, 1, k) for k in range(K)]
    for k in range(K):
        agg.UpdateGradient(flats[k], range(P))
    ref = [O.organize_gradients(f, M, P) for f in flats]
    for p in (0, 1, 150, P - 1):
        assert_bits_equal(agg.read(p), O.reduce([ref[k][p] for k in range(K)], agg.lengths[p]), f"p{p}")
    for p in range(P):
        agg.AggregatePartition(p)
    got = agg.GetPartitions()
    exp = O.get_partitions([O.reduce([ref[k][p] for k in range(K)], agg.lengths[p]) for p in range(P)])
    assert_bits_equal(got, exp, "average")
    agg.close()


def test_ingest_pubsub_double_base64(ipls, O):
    """ThreadReceiver path on the GPU: pubsub 'data' texts (base64url of the
    base64url of a Marshall_Packet frame) decoded, parsed and folded, routed
    by the frame's partition field, in message order."""
    M, P, K = 30011, 3, 4
    agg = ipls.Aggregator(M, P)
    peers = [O.synth_bucket(M, 2, k) for k in range(K)]
    parts = [O.organize_gradients(g, M, P) for g in peers]
    msgs = []
    for k in range(K):
        for p in range(P):
            fr = O.frame_encode(parts[k][p], p, 17, 3, f"QmPeer{k}".encode())
            m = O.pubsub_message(fr)
            if k % 2:
                m = m.rstrip(b"=")             # Java accepts unpadded text too
            msgs.append(m)
    n, st = agg.ingest_pubsub(msgs)
    assert n == K * P and st == [0] * (K * P)
    for p in range(P):
        assert_bits_equal(agg.read(p), O.reduce([parts[k][p] for k in range(K)], agg.lengths[p]), f"p{p}")
    agg.close()


def test_ingest_pubsub_errors_dropped(ipls, O):
    M, P = 1000, 2
    agg = ipls.Aggregator(M, P)
    L0 = agg.lengths[0]
    g = O.synth_bucket(L0, 0, 0)
    good = O.pubsub_message(O.frame_encode(g, 0, 1, 3, b"QmA"))
    bad_char = good[:10] + b"+" + good[11:]                    # '+' is not in the URL alphabet
    bad_pad = good.rstrip(b"=") + b"="                          # wrong '=' tail (if it was unpadded)
    inner = O.java_b64url_encode(O.frame_encode(g, 0, 1, 3, b"QmA"))
    bad_inner = O.java_b64url_encode(inner[:5] + b"*" + inner[6:])
    short = O.pubsub_message(O.frame_encode(g[:10], 0, 1, 3, b"QmA"))     # n < L_p
    null = O.pubsub_message(O.frame_encode(None, 0, 1, 3, b"QmA"))         # arr_len 0 -> null
    wrong_p = O.pubsub_message(O.frame_encode(g, 7, 1, 3, b"QmA"))         # partition 7 of 2
    trunc = O.pubsub_message(O.frame_encode(g, 0, 1, 3, b"QmA")[:20])      # n says more than it holds
    msgs = [good, bad_char, bad_inner, short, null, wrong_p, trunc, good]
    exp_ok = []
    for m in msgs:
        try:
            fr = O.pubsub_decode(m)
            pid, nn, a, b, gg, origin = O.frame_decode(fr)
            exp_ok.append(gg is not None and 0 <= a < P and nn >= agg.lengths[a])
        except ValueError:
            exp_ok.append(False)
    n, st = agg.ingest_pubsub(msgs)
    assert n == 2 and [s == 0 for s in st] == exp_ok
    assert st[1] == -6 and st[2] == -6 and st[3] == -2 and st[4] == 1 and st[5] == -2 and st[6] == -6
    assert_bits_equal(agg.read(0), O.reduce([g, g], L0), "two good")
    # bad_pad only differs when the text had no padding to begin with
    n2, st2 = agg.ingest_pubsub([bad_pad])
    try:
        O.pubsub_decode(bad_pad)
        assert st2 == [0]
    except ValueError:
        assert st2 == [-6] and n2 == 0
    agg.close()


def _ingest_expected(O, m, layers, P, lengths, part=None):
    """Status the ingest must report for one text, from the oracle's Java
    restatement: -6 IllegalArgument/BufferUnderflow, 1 null gradient, -2 out
    of range (GET_GRADIENTS, MyIPFSClass.java:1437-1459), 0 folded."""
    try:
        fr = O.pubsub_decode(m) if layers == 2 else O.java_b64url_decode(m)
        pid, nn, a, b, gg, origin = O.frame_decode(fr)
    except ValueError:
        return -6, None
    if gg is None:
        return 1, None
    p = a if part is None else part
    if not 0 <= p < P or nn < lengths[p]:
        return -2, None
    return 0, (p, gg)


def test_ingest_pubsub_inner_padding(ipls, O):
    """The inner text's '=' rules count the WHOLE inner text's data chars,
    not those of the few chars the host decodes at its end (found by
    tools/fuzz_ingest.py): inner 'xx=' / 'x==' / '===' endings are
    IllegalArgumentException (-6), 'xx==' / 'xxx=' / unpadded fold."""
    M, P = 9001, 3
    agg = ipls.Aggregator(M, P)
    L0 = int(agg.lengths[0])
    msgs, exp = [], []
    for extra in range(3):                 # frame length % 3 = 0, 1, 2 across the origins
        for origin in (b"Qm", b"QmM", b"QmM1"):
            g = O.synth_bucket(L0 + extra, 4, 7)
            inner = O.java_b64url_encode(O.frame_encode(g, 0, 3, 3, origin))
            variants = [inner, inner.rstrip(b"="), inner[:-1], inner.rstrip(b"=") + b"=",
                        inner.rstrip(b"=") + b"==", inner.rstrip(b"=") + b"==="]
            for v in variants:
                m = O.java_b64url_encode(v)
                msgs.append(m)
                exp.append(_ingest_expected(O, m, 2, P, agg.lengths)[0])
    assert -6 in exp and 0 in exp
    n, st = agg.ingest_pubsub(msgs, layers=2)
    assert st == exp
    assert n == exp.count(0)
    agg.close()


@pytest.mark.parametrize("layers,override", [(1, False), (2, False), (2, True)])
def test_ingest_pubsub_mutations(ipls, O, layers, override, seed=None, n_msgs=120):
    """Every status the pipelined ingest reports (host-read text ends, device-
    checked bodies) against the oracle: invalid chars in the header, body or
    tail of either base64 layer, '=' in the middle, truncations, wrong
    partition or n, and combinations (an invalid body char beats a bad route)."""
    rng = np.random.default_rng(11 + layers if seed is None else seed)
    M, P = 9001, 3
    agg = ipls.Aggregator(M, P)
    L = agg.lengths
    enc = (lambda fr: O.pubsub_message(fr)) if layers == 2 else (lambda fr: O.java_b64url_encode(fr))
    bad_chars = b"+/=*\n.\x80 "
    msgs = []
    for t in range(n_msgs):
        p = int(rng.integers(0, P))
        g = O.synth_bucket(int(L[p]) + int(rng.integers(0, 3)), 4, t)
        fr = bytearray(O.frame_encode(g, p, 3, 3, b"QmM%d" % t))
        kind = t % 10
        if kind == 1:                                  # wrong partition field
            fr[6:10] = int(rng.choice([P, 7, -1])).to_bytes(4, "big", signed=True)
        elif kind == 2:                                # n too big / negative / short
            fr[2:6] = int(rng.choice([len(g) + 5, -3, 10])).to_bytes(4, "big", signed=True)
        elif kind == 3:
            fr = fr[:int(rng.integers(0, 40))]         # truncated frame (header cut too)
        elif kind == 4:
            fr[2:6] = (0).to_bytes(4, "big")           # null gradient
        m = bytearray(enc(bytes(fr)))
        if kind in (5, 6, 7) and len(m) > 4:
            # one bad char in the outer text: first 28 chars (header), body, last 8 (tail)
            pos = {5: int(rng.integers(0, min(28, len(m)))),
                   6: int(rng.integers(0, len(m))),
                   7: max(0, len(m) - 1 - int(rng.integers(0, 8)))}[kind]
            m[pos] = bad_chars[int(rng.integers(0, len(bad_chars)))]
        elif kind == 8 and layers == 2:                # bad char in the inner text, re-encoded
            inner = bytearray(O.java_b64url_encode(bytes(fr)))
            pos = int(rng.choice([0, 5, 19, len(inner) // 2, len(inner) - 1, len(inner) - 3]))
            inner[pos] = bad_chars[int(rng.integers(0, len(bad_chars)))]
            m = bytearray(O.java_b64url_encode(bytes(inner)))
        elif kind == 9:
            m = m[:len(m) - int(rng.integers(1, 6))]   # truncated text
            if t % 20 == 9:
                m[len(m) // 2] = ord("+")               # and a bad body char
        if t % 7 == 0:
            m = m.rstrip(b"=")                          # Java accepts unpadded text
        if t % 11 == 0 and kind == 1 and len(m) > 40:
            m[len(m) // 2] = ord("*")                   # bad route AND bad body char -> -6
        msgs.append(bytes(m))
    # override: the caller routes each text (Download_Scheduler's known partition), -1 and P out of range
    parts = [int(x) for x in rng.integers(-1, P + 1, size=len(msgs))] if override else None
    exp = [_ingest_expected(O, m, layers, P, L, None if parts is None else parts[i]) for i, m in enumerate(msgs)]
    n, st = agg.ingest_pubsub(msgs, layers=layers, partitions=parts)
    bad = [(i, msgs[i][:48], len(msgs[i]), e[0], st[i]) for i, e in enumerate(exp) if st[i] != e[0]]
    assert not bad, f"(index, text head, text len, expected, got): {bad}"
    assert n == sum(1 for e in exp if e[0] == 0)
    assert len(set(st)) >= 4 or seed is not None, st
    for p in range(P):
        gs = [e[1][1] for e in exp if e[0] == 0 and e[1][0] == p]
        assert gs or seed is not None or override, p       # the fixed-seed cases fold into every partition
        assert_bits_equal(agg.read(p), O.reduce(gs, L[p]), f"p{p}")
    agg.close()


def test_ingest_pubsub_single_layer_large(ipls, O):
    """One base64 layer (Marshall_Packet text as published), 1M-double
    payloads (vector decode path), replica frames routed by caller partitions."""
    L = 1 << 20
    agg = ipls.Aggregator(n_partitions=2, bucket_len=L)
    bufs = [O.synth_bucket(L, 1, k) for k in range(3)]
    msgs = [O.java_b64url_encode(O.frame_encode(b, 5, 2, 3, b"QmRep")) for b in bufs]
    n, st = agg.ingest_pubsub(msgs, layers=1, partitions=[1, 1, 1], from_clients=False)
    assert n == 3
    assert_bits_equal(agg.read(1, ipls.TGT_REP), O.reduce(bufs, L), "replica frames")
    agg.close()


def test_async_variants(ipls, O):
    """-async true branches: W = 0.75*W + g, leaving-peer W = 0.6*W + (1-0.6)*w,
    and the 0.25*W publish scale -- each product rounded, then the sum."""
    L = 20011
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L)
    w0 = O.synth_bucket(L, 3, 0) * 37.0
    agg.cache_partition(0, w0)
    g1, g2 = O.synth_bucket(L, 3, 1), O.synth_bucket(L, 3, 2)
    agg.UpdateAsyncReplica(g1, 0)
    agg.UpdateLeavingPeer(O.be_encode(g2), 0)
    w = O.blend(O.blend(w0, g1, 0.75, 1.0), g2, 0.6, 1 - 0.6)
    assert_bits_equal(agg.read(0, ipls.TGT_WEIGHTS), w, "blends")
    agg.AsyncPublishScale(0)
    assert_bits_equal(agg.read(0, ipls.TGT_AGG), O.scale(w, 0.25), "scale")
    agg.close()


@pytest.mark.parametrize("L", [1, 2047, 2048, 2049, 6149, 20011])
def test_elementwise_kernels_both_shapes(ipls, O, L):
    """k_blend, k_scale, k_encode_secure and k_fold_n take a 16-B tile shape
    (2,048 elements per block) when every operand is 16-B aligned and an 8-B
    grid-stride loop otherwise.  Device operands at a 16-B boundary and at
    8 mod 16, at lengths around the tile (one element, one short of a tile,
    a tile, one over, three tiles and a tail): the bits equal the oracle's
    either way, native and big-endian."""
    pool = torch.empty(4 * L + 8, dtype=torch.float64, device="cuda")
    pool_be = torch.empty(8 * (4 * L + 8), dtype=torch.uint8, device="cuda")
    assert pool.data_ptr() % 16 == 0 and pool_be.data_ptr() % 16 == 0

    def dev_at(x, shift, be=False):       # x placed at a 16-B boundary (shift 0) or 8 mod 16 (shift 1)
        if be:
            b = np.frombuffer(O.be_encode(x), dtype=np.uint8)
            pool_be[8 * shift:8 * shift + b.size].copy_(torch.from_numpy(b.copy()))
            return ipls.DeviceBuffer(int(pool_be.data_ptr()) + 8 * shift, len(x), big_endian=True)
        pool[shift:shift + len(x)].copy_(torch.from_numpy(x))
        return ipls.DeviceBuffer(int(pool.data_ptr()) + 8 * shift, len(x))

    for shift in (0, 1):
        agg = ipls.Aggregator(n_partitions=1, bucket_len=L)
        w0 = O.synth_bucket(L, 4, shift) * 37.0
        agg.cache_partition(0, w0)
        g1, g2 = O.synth_bucket(L, 4, 10 + shift), O.synth_bucket(L, 4, 20 + shift)
        agg.UpdateAsyncReplica(dev_at(g1, shift), 0)                  # k_blend, native
        torch.cuda.synchronize()
        agg.UpdateLeavingPeer(dev_at(g2, shift, be=True), 0)          # k_blend, big-endian
        w = O.blend(O.blend(w0, g1, 0.75, 1.0), g2, 0.6, 1 - 0.6)
        assert_bits_equal(agg.read(0, ipls.TGT_WEIGHTS), w, f"blends L={L} shift={shift}")
        agg.AsyncPublishScale(0)                                        # k_scale (arena: aligned)
        assert_bits_equal(agg.read(0, ipls.TGT_AGG), O.scale(w, 0.25), f"scale L={L}")
        # k_fold_n: stored download (FIRST), a second one folded in, then the collect into REP
        store = O.ReplicaStore()
        for k, be in ((30, False), (31, True)):
            gk = O.synth_bucket(L, 4, k + shift) * 1e3
            agg.OtherReplicaGradients(0, 7, dev_at(gk, shift, be=be))
            torch.cuda.synchronize()
            O.other_replica_add(store, 0, 7, gk)
        rep = [np.zeros(L)]
        O.collect_replicas(rep, store, [0])
        agg.Collect_Replicas()
        assert_bits_equal(agg.read(0, ipls.TGT_REP), rep[0], f"replica fold L={L} shift={shift}")
        # k_bswap64: REP read out as big-endian bytes into a device buffer, and
        # Weights set from big-endian device bytes (cache_partition)
        from ipls import _native as N
        out = torch.zeros(8 * (L + 2), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()              # torch's fill runs on its own stream, not the handle's
        agg._chk(agg._lib.ipls_agg_read(agg._h, 0, ipls.TGT_REP, int(out.data_ptr()) + 8 * shift, L, N.DEV_BE))
        torch.cuda.synchronize()
        assert bytes(out[8 * shift:8 * (shift + L)].cpu().numpy()) == O.be_encode(rep[0]), f"BE read L={L}"
        w3 = O.synth_bucket(L, 4, 40 + shift)
        agg.cache_partition(0, dev_at(w3, shift, be=True))
        assert_bits_equal(agg.read(0, ipls.TGT_WEIGHTS), w3, f"BE weights L={L} shift={shift}")
        agg.close()
        # k_encode_secure between device buffers, every byte-order pairing
        x = O.synth_bucket(L, 5, shift) * 3000.0
        x[::7] = 11.0
        x[1::7] = -11.0
        want = O.encode_secure(x)
        src = dev_at(x, shift)
        for bo in (False, True):
            out = torch.zeros(8 * (L + 2), dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            dst = ipls.DeviceBuffer(int(out.data_ptr()) + 8 * shift, L, big_endian=bo)
            ipls.encode_secure(src, dst)
            torch.cuda.synchronize()
            got = bytes(out[8 * shift:8 * (shift + L)].cpu().numpy())
            assert got == (O.be_encode(want) if bo else want.tobytes()), f"encode_secure L={L} shift={shift} be={bo}"


@pytest.mark.parametrize("M,P", [(20481, 4), (443610, 3), (65536, 5)])
def test_update_gradient_both_shapes(ipls, O, M, P):
    """IPLS.UpdateGradient's own accumulate (IPLS.java:1737-1743) through
    k_split: partitions whose segment of the flat vector starts 16-B aligned
    take the tile shape, the others one element per lane; a logically-zero
    AGG is written as +0.0 + v without a memset (MODE 2), later steps fold
    (MODE 1).  Host input and device input at a 16-B boundary and at 8 mod
    16; big-endian device input; -0.0 values show the +0.0 start."""
    owned = list(range(P))
    for kind in ("host", "dev0", "dev1", "be1"):
        agg = ipls.Aggregator(M, P)
        acc = {p: np.zeros(agg.lengths[p]) for p in owned}
        keep = []
        for step in range(3):
            g = O.synth_bucket(M, 7, 10 * step + len(kind))
            g[::97] = -0.0
            if kind == "host":
                src = g
            else:
                shift = 0 if kind == "dev0" else 1
                be = kind == "be1"
                raw = np.frombuffer(O.be_encode(g) if be else g.tobytes(), dtype=np.uint8)
                t = torch.zeros(raw.size + 16, dtype=torch.uint8, device="cuda")
                t[8 * shift:8 * shift + raw.size] = torch.from_numpy(raw.copy()).to("cuda")
                torch.cuda.synchronize()
                keep.append(t)
                src = ipls.DeviceBuffer(int(t.data_ptr()) + 8 * shift, M, big_endian=be)
            agg.UpdateGradient(src, owned)
            parts = O.organize_gradients(g, M, P)
            for p in owned:
                acc[p] = O.fold(acc[p], parts[p])
        for p in owned:
            assert_bits_equal(agg.read(p, ipls.TGT_AGG), acc[p], f"AGG[{p}] M={M} {kind}")
        agg.close()


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_accumulate_range(ipls, O, devices):
    """ipls_agg_accumulate_range: one arrival folded as ranges of pinned host
    memory gets the bits of the whole-bucket fold, into a logically-zero
    target and a live one, native and big-endian; misuse is refused before
    anything is folded.  devices=[0, 0]: partition 1 lives on the second
    shard (the front's ticket bookkeeping)."""
    from ipls import _native as N
    L = 300007
    agg = ipls.Aggregator(n_partitions=2, bucket_len=L, devices=devices)
    lib, h = agg._lib, agg._h
    pin = ipls.PinnedBuffer(8 * L + 64)
    view = pin.view()
    t = ctypes.c_uint64()
    want = np.zeros(L)
    for k, (be, cuts) in enumerate(((False, [0, 2048, 150000, L]), (True, [0, 100000, 100002, L]), (False, [0, L]))):
        g = O.synth_bucket(L, 1, 60 + k) * 10.0 ** k
        raw = np.frombuffer(O.be_encode(g) if be else g.tobytes(), dtype=np.uint8)
        view[:raw.size] = raw
        kind = N.HOST_BE if be else N.HOST_F64
        for a, b in zip(cuts[:-1], cuts[1:]):
            assert lib.ipls_agg_accumulate_range(h, 1, ipls.TGT_AGG, pin.ptr + 8 * a, a, b - a, kind, ctypes.byref(t)) == 0
        assert lib.ipls_agg_wait(h, t.value) == 0
        want = O.fold(want, g)
        assert_bits_equal(agg.read(1, ipls.TGT_AGG), want, f"ranges {cuts}")
    host = np.zeros(L + 2)
    bad = [(pin.ptr + 8, 1, 10, N.IPLS_E_INVAL),                 # odd start
           (pin.ptr + 8, 0, 10, N.IPLS_E_INVAL),                 # bytes at 8 mod 16
           (host.ctypes.data, 0, 10, N.IPLS_E_INVAL),            # not pinned memory
           (pin.ptr, L - 2, 4, N.IPLS_E_RANGE),                  # past the partition
           (pin.ptr, -2, 4, N.IPLS_E_RANGE)]
    for ptr, off, n, code in bad:
        assert lib.ipls_agg_accumulate_range(h, 1, ipls.TGT_AGG, ptr, off, n, N.HOST_F64, ctypes.byref(t)) == code
    assert lib.ipls_agg_accumulate_range(h, 1, ipls.TGT_AGG, pin.ptr, 0, 4, N.DEV_F64, ctypes.byref(t)) == N.IPLS_E_INVAL
    assert_bits_equal(agg.read(1, ipls.TGT_AGG), want, "refused ranges folded nothing")
    assert_bits_equal(agg.read(0, ipls.TGT_AGG), np.zeros(L), "partition 0 untouched")
    agg.close()
    pin.close()


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_read_range(ipls, O, devices):
    """ipls_agg_read_range: a target read in ranges into pinned memory, native
    and big-endian, equals the whole read; after ipls_agg_finalize with no
    output, Weights in big-endian ranges are the commit_update bytes; misuse
    is refused."""
    from ipls import _native as N
    L = 200003
    agg = ipls.Aggregator(n_partitions=2, bucket_len=L, devices=devices)
    lib, h = agg._lib, agg._h
    a, r = O.synth_bucket(L, 1, 1), O.synth_bucket(L, 1, 2) * 3.0
    agg.Update(a, 1)
    agg.Update(r, 1, from_clients=False)
    pin = ipls.PinnedBuffer(8 * L)
    t = ctypes.c_uint64()
    for kind, want in ((N.HOST_F64, a.tobytes()), (N.HOST_BE, O.be_encode(a))):
        for lo, hi in ((0, 65536), (65536, 65538), (65538, L)):
            assert lib.ipls_agg_read_range(h, 1, ipls.TGT_AGG, pin.ptr + 8 * lo, lo, hi - lo, kind, ctypes.byref(t)) == 0
        assert lib.ipls_agg_wait(h, t.value) == 0
        assert pin.view()[:8 * L].tobytes() == want, f"kind {kind}"
    assert lib.ipls_agg_finalize(h, 1, None, N.HOST_BE, None) == 0
    for lo, hi in ((0, 100000), (100000, L)):
        assert lib.ipls_agg_read_range(h, 1, ipls.TGT_WEIGHTS, pin.ptr + 8 * lo, lo, hi - lo, N.HOST_BE, ctypes.byref(t)) == 0
    assert lib.ipls_agg_wait(h, t.value) == 0
    assert pin.view()[:8 * L].tobytes() == O.be_encode(a + r), "commit_update bytes"
    host = np.zeros(8)
    assert lib.ipls_agg_read_range(h, 1, ipls.TGT_AGG, host.ctypes.data, 0, 4, N.HOST_F64, ctypes.byref(t)) == N.IPLS_E_INVAL
    assert lib.ipls_agg_read_range(h, 1, ipls.TGT_AGG, pin.ptr, L - 1, 2, N.HOST_F64, ctypes.byref(t)) == N.IPLS_E_RANGE
    assert lib.ipls_agg_read_range(h, 1, ipls.TGT_AGG, pin.ptr, 0, 2, N.DEV_F64, ctypes.byref(t)) == N.IPLS_E_INVAL
    agg.close()
    pin.close()


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_accumulate_chunked(ipls, O, devices):
    """ipls_agg_accumulate_chunked: one arrival pulled from a caller source
    chunk by chunk, as one call (Updater._Update's whole-bucket fold,
    Updater.java:115-117).  The source is asked for consecutive ranges that
    tile [0, L) exactly (never past L, even when the caller's bucket is
    longer), and the bits equal the oracle's whole-bucket folds: native and
    big-endian values, a logically-zero target and a live one, AGG and REP,
    chunks of 2 values, an odd chunk count and one chunk larger than L.  A
    short bucket is IPLS_E_RANGE before any source call; a source that stops
    folds nothing (all or nothing); an odd chunk is refused."""
    from ipls import _native as N
    L = 300007
    agg = ipls.Aggregator(n_partitions=2, bucket_len=L, devices=devices)
    lib, h = agg._lib, agg._h
    acc = {0: np.zeros(L), 1: np.zeros(L)}
    for k, (tgt, be, chunk, extra) in enumerate(((0, False, 65536, 0), (0, True, 100002, 9), (1, False, 1 << 22, 0),
                                                   (1, True, 65536, 0), (0, False, 2, 0))):
        g = O.synth_bucket(L + extra, 1, 70 + k) * 10.0 ** (k - 2)
        g[::997] = -0.0
        raw = np.frombuffer(O.be_encode(g) if be else g.tobytes(), dtype=np.uint8)
        seen = []

        @N.CHUNK_SOURCE
        def src(ctx, dst, off, n):
            seen.append((off, n))
            ctypes.memmove(dst, raw.ctypes.data + 8 * off, 8 * n)
            return 0
        kind = N.HOST_BE if be else N.HOST_F64
        assert lib.ipls_agg_accumulate_chunked(h, 1, tgt, L + extra, kind, chunk, src, None) == 0
        assert [o for o, _ in seen] == list(range(0, L, min(chunk, L))), "consecutive chunks"
        assert sum(n for _, n in seen) == L and all(n <= chunk for _, n in seen)
        acc[tgt] = O.fold(acc[tgt], g[:L])
        assert_bits_equal(agg.read(1, tgt), acc[tgt], f"chunked fold {k}")
    calls = []

    @N.CHUNK_SOURCE
    def stop(ctx, dst, off, n):
        calls.append(off)
        ctypes.memset(dst, 0x7F, 8 * n)            # garbage that must never be folded
        return 1 if len(calls) == 3 else 0
    assert lib.ipls_agg_accumulate_chunked(h, 1, 0, L, N.HOST_F64, 65536, stop, None) == N.IPLS_E_INVAL
    assert calls == [0, 65536, 131072]
    calls.clear()
    assert lib.ipls_agg_accumulate_chunked(h, 0, 0, L, N.HOST_F64, 65536, stop, None) == N.IPLS_E_INVAL
    calls.clear()
    assert lib.ipls_agg_accumulate_chunked(h, 1, 0, L - 1, N.HOST_F64, 65536, stop, None) == N.IPLS_E_RANGE
    assert lib.ipls_agg_accumulate_chunked(h, 1, 0, L, N.HOST_F64, 65537, stop, None) == N.IPLS_E_INVAL
    assert lib.ipls_agg_accumulate_chunked(h, 1, 0, L, N.DEV_F64, 65536, stop, None) == N.IPLS_E_INVAL
    assert calls == [], "refused before any source call"
    assert_bits_equal(agg.read(1, 0), acc[0], "a stopped source folded nothing")
    assert_bits_equal(agg.read(0, 0), np.zeros(L), "partition 0 untouched (logically zero)")
    agg.Update(np.ones(L), 0)                       # partition 0 is still a +0.0 start
    assert_bits_equal(agg.read(0, 0), O.fold(np.zeros(L), np.ones(L)), "p0 after the stopped source")
    agg.close()


@pytest.mark.parametrize("devices", [None, [0, 0, 0]])
def test_chunked_calls_tiny_partitions_and_wire(ipls, O, devices):
    """The chunked calls at the smallest shapes: partitions of 1 value (the
    count slot alone) and 3 values, every target (AGG, REP, FUTURE, Weights)
    through ipls_agg_accumulate_chunked, finalize_chunked of both, and
    ipls_agg_get_partitions_wire_chunked over a three-shard handle equal to
    the whole-model wire bytes of ipls_agg_get_partitions (and the oracle)."""
    from ipls import _native as N
    for L in (1, 3):
        agg = ipls.Aggregator(n_partitions=3, bucket_len=L, devices=devices)
        lib, h = agg._lib, agg._h
        want = {}
        for p in range(3):
            for tgt in (N.TGT_AGG, N.TGT_REP, N.TGT_FUTURE):
                g = O.synth_bucket(L, p, 40 + tgt) * (2.0 + tgt)

                @N.CHUNK_SOURCE
                def src(ctx, dst, off, n, g=g):
                    ctypes.memmove(dst, g.ctypes.data + 8 * off, 8 * n)
                    return 0
                assert lib.ipls_agg_accumulate_chunked(h, p, tgt, L, N.HOST_F64, 2, src, None) == 0
                want[(p, tgt)] = O.fold(np.zeros(L), g)
                assert_bits_equal(agg.read(p, tgt), want[(p, tgt)], f"L={L} p={p} tgt={tgt}")
        for p in range(3):
            out = bytearray(8 * L)

            @N.CHUNK_SINK
            def sink(ctx, vals, off, n, out=out):
                out[8 * off:8 * (off + n)] = ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n)
                return 0
            assert lib.ipls_agg_finalize_chunked(h, p, N.HOST_BE, 2, sink, None) == 0
            w = want[(p, N.TGT_AGG)] + want[(p, N.TGT_REP)]
            assert bytes(out) == O.be_encode(w), f"L={L} W[{p}]"
        whole = agg.GetPartitions(wire=True)
        got = bytearray()

        @N.CHUNK_SINK
        def wsink(ctx, vals, off, n):
            got.extend(ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n))
            return 0
        assert lib.ipls_agg_get_partitions_wire_chunked(h, 2, wsink, None) == 0
        assert bytes(got) == whole
        ws = [want[(p, N.TGT_AGG)] + want[(p, N.TGT_REP)] for p in range(3)]
        assert whole == O.be_encode_canonical(O.get_partitions(ws))
        agg.close()


@pytest.mark.parametrize("case", ["szero", "cancel", "special"])
def test_chunked_calls_golden_edge_values(ipls, O, golden, case):
    """The golden edge buckets (signed zeros, cancellation order, NaN / inf /
    -0.0 / subnormals, the count slot among them) through the chunked calls
    with two-value chunks, so neighbouring special values cross PCIe in
    different chunks, ring slots and copy streams, alternately big-endian
    and native: AGG equals the golden fold from +0.0 bit for bit, the
    commit_update bytes are W's (AggregatePartition, IPLS.java:1248-1274),
    and the task-3 stream is the oracle's writeDouble bytes of the divide
    (NaN canonical, Middleware.java:164-170)."""
    from ipls import _native as N
    bufs = golden[f"{case}_bufs"]
    L = bufs.shape[1]
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L)
    lib, h = agg._lib, agg._h
    for k, g in enumerate(bufs):
        be = k % 2 == 0
        raw = O.be_encode(g) if be else np.ascontiguousarray(g).tobytes()

        @N.CHUNK_SOURCE
        def src(ctx, dst, off, n, raw=raw):
            ctypes.memmove(dst, ctypes.c_char_p(raw[8 * off:8 * (off + n)]), 8 * n)
            return 0
        assert lib.ipls_agg_accumulate_chunked(h, 0, N.TGT_AGG, L, N.HOST_BE if be else N.HOST_F64, 2, src,
                                               None) == 0
    assert_bits_equal(agg.read(0, N.TGT_AGG), golden[f"{case}_zero"], f"{case}: AGG")
    W = golden[f"{case}_zero"] + 0.0
    out = bytearray(8 * L)

    @N.CHUNK_SINK
    def sink(ctx, vals, off, n):
        out[8 * off:8 * (off + n)] = ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n)
        return 0
    assert lib.ipls_agg_finalize_chunked(h, 0, N.HOST_BE, 2, sink, None) == 0
    # putDouble keeps a NaN's payload, which Java does not specify: compared as values, NaN meeting NaN
    assert_bits_equal(np.frombuffer(bytes(out), dtype=">f8").astype(np.float64), W, f"{case}: commit_update bytes")
    got = bytearray()

    @N.CHUNK_SINK
    def wsink(ctx, vals, off, n):
        got.extend(ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n))
        return 0
    assert lib.ipls_agg_get_partitions_wire_chunked(h, 2, wsink, None) == 0
    assert bytes(got) == O.be_encode_canonical(O.get_partitions([W])), f"{case}: task-3 stream"
    agg.close()


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_accumulate_chunked_threads_serialise(ipls, O, devices):
    """Four threads fold four buckets into the same partition, each as one
    ipls_agg_accumulate_chunked call whose source sleeps between chunks (so
    that, were the calls not units, they would interleave).  Each call takes
    effect as a whole when its last chunk has landed (the shard lock is held
    for the fold only), so the target equals the oracle's fold of the four
    whole buckets in ONE serial order, bit for bit -- normally the order in
    which the sources delivered their last chunks; two calls whose last
    chunks land within the same instant may take the lock in either order,
    so every order is tried and exactly one must match.  A fifth thread keeps
    folding into another partition of the same shard meanwhile."""
    import itertools
    import threading
    import time
    from ipls import _native as N
    L = 262147
    agg = ipls.Aggregator(n_partitions=2, bucket_len=L, devices=devices)
    lib, h = agg._lib, agg._h
    gs = [O.synth_bucket(L, 1, 300 + i) * (1.0 + i) for i in range(4)]
    base = O.synth_bucket(L, 1, 299)   # a non-zero start: (0 + a) + b == (0 + b) + a would hide an order
    agg.Update(base, 1)
    last, lock = [], threading.Lock()
    errs = []

    def worker(i):
        raw = gs[i].tobytes()

        @N.CHUNK_SOURCE
        def src(ctx, dst, off, n):
            ctypes.memmove(dst, ctypes.c_char_p(raw[8 * off:8 * (off + n)]), 8 * n)
            if off + n == L:
                with lock:
                    last.append(i)
            else:
                time.sleep(0.002 * (1 + i))
            return 0
        rc = lib.ipls_agg_accumulate_chunked(h, 1, ipls.TGT_AGG, L, N.HOST_F64, 32768, src, None)
        if rc != 0:
            errs.append(rc)

    other = O.synth_bucket(L, 0, 9)

    def side():
        for _ in range(20):
            agg.Update(other, 0)
    ths = [threading.Thread(target=worker, args=(i,)) for i in range(4)] + [threading.Thread(target=side)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    assert not errs and sorted(last) == [0, 1, 2, 3]
    got = agg.read(1, ipls.TGT_AGG).view(np.uint64)

    def serial(order):
        want = O.fold(np.zeros(L), base)
        for i in order:
            want = O.fold(want, gs[i])
        return want
    matches = [o for o in itertools.permutations(range(4)) if np.array_equal(serial(o).view(np.uint64), got)]
    assert len(matches) == 1, f"{len(matches)} serial orders match (last-chunk order {last})"
    side_want = np.zeros(L)
    for _ in range(20):
        side_want = O.fold(side_want, other)
    assert_bits_equal(agg.read(0, ipls.TGT_AGG), side_want, "the other partition")
    agg.close()


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_chunked_io_holds_no_shard_lock(ipls, O, devices):
    """a chunked call's source or sink -- in the
    Middleware servers a blocking socket recv/send -- runs with no shard lock
    held, so a stalled peer freezes nothing else (the reference deserialises
    the whole stream before UpdateModel takes PeerData.mtx, and writes the
    reply after Get_Partitions returned, Middleware.java:224, 246, 254).

    1. Thread A's accumulate_chunked into partition 1 blocks in its source
       after the first chunk, for 500 ms.  Meanwhile a fold into partition 0
       (same shard) and one into partition 1 itself both return, and so does
       a GetPartitions.  A then completes; it takes effect when its last chunk
       has landed: p1 = (base + B) + A and p0 = +0.0 + B0, bit for bit.
    2. finalize_chunked of partition 1 whose sink blocks after the first
       chunk: an Update into partition 1 and a set_weights of partition 1
       return meanwhile.  The bytes delivered are the commit_update bytes of
       this call's AggregatePartition (a snapshot: not torn), AGG then holds
       the new arrival and W the new weights.
    3. get_partitions_wire_chunked whose sink blocks: set_weights of every
       partition returns meanwhile; the stream is the pre-call model's."""
    import threading
    import time
    from ipls import _native as N
    L = 300007
    agg = ipls.Aggregator(n_partitions=4, bucket_len=L, devices=devices)
    lib, h = agg._lib, agg._h
    a, b, b0, base = (O.synth_bucket(L, 1, 610 + i) * (1.0 + 2 * i) for i in range(4))
    agg.Update(base, 1)   # a non-zero start, so that (base + B) + A and (base + A) + B differ
    blocked, release = threading.Event(), threading.Event()
    res = {}

    def run_a():
        raw = a.tobytes()

        @N.CHUNK_SOURCE
        def src(ctx, dst, off, n):
            ctypes.memmove(dst, ctypes.c_char_p(raw[8 * off:8 * (off + n)]), 8 * n)
            if off == 0:
                blocked.set()
                release.wait(10)
            return 0
        res["a"] = lib.ipls_agg_accumulate_chunked(h, 1, ipls.TGT_AGG, L, N.HOST_F64, 65536, src, None)
    ta = threading.Thread(target=run_a)
    ta.start()
    assert blocked.wait(30)
    t0 = time.perf_counter()
    agg.Update(b0, 0)
    agg.Update(b, 1)
    whole = agg.GetPartitions(wire=True)
    inside = time.perf_counter() - t0
    time.sleep(max(0.0, 0.5 - inside))
    assert not res, "A finished while its source was blocked"
    release.set()
    ta.join(30)
    assert res["a"] == 0
    assert inside < 0.5, f"the other calls waited {inside:.3f} s behind a blocked source"
    assert len(whole) == 8 * 4 * (L - 1)
    assert_bits_equal(agg.read(0, ipls.TGT_AGG), O.fold(np.zeros(L), b0), "p0")
    p1 = O.fold(O.fold(O.fold(np.zeros(L), base), b), a)
    assert not np.array_equal(p1.view(np.uint64), O.fold(O.fold(O.fold(np.zeros(L), base), a), b).view(np.uint64))
    assert_bits_equal(agg.read(1, ipls.TGT_AGG), p1, "p1 = (base + B) + A")

    # 2. a blocked finalize sink
    r = O.synth_bucket(L, 1, 620) * 3.0
    agg.Update(r, 1, from_clients=False)
    w_round = p1 + O.fold(np.zeros(L), r)
    nxt, w_new = O.synth_bucket(L, 1, 621), O.synth_bucket(L, 1, 622)
    blocked.clear()
    release.clear()
    out = bytearray(8 * L)

    def run_f():
        @N.CHUNK_SINK
        def sink(ctx, vals, off, n):
            out[8 * off:8 * (off + n)] = ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n)
            if off == 0:
                blocked.set()
                release.wait(10)
            return 0
        res["f"] = lib.ipls_agg_finalize_chunked(h, 1, N.HOST_BE, 65536, sink, None)
    tf = threading.Thread(target=run_f)
    tf.start()
    assert blocked.wait(30)
    t0 = time.perf_counter()
    agg.Update(nxt, 1)
    assert lib.ipls_agg_set_weights(h, 1, w_new.ctypes.data, L, N.HOST_F64) == 0
    inside = time.perf_counter() - t0
    assert "f" not in res
    release.set()
    tf.join(30)
    assert res["f"] == 0 and inside < 0.5, inside
    assert bytes(out) == O.be_encode(w_round), "commit_update bytes: this call's snapshot"
    assert_bits_equal(agg.read(1, ipls.TGT_AGG), O.fold(np.zeros(L), nxt), "AGG: the arrival after the round")
    assert_bits_equal(agg.read(1, ipls.TGT_WEIGHTS), w_new, "W: the later set_weights")

    # 3. a blocked GetPartitions sink
    ws = [agg.read(p, ipls.TGT_WEIGHTS) for p in range(4)]
    want = O.be_encode_canonical(O.get_partitions(ws))
    blocked.clear()
    release.clear()
    got = bytearray()

    def run_g():
        @N.CHUNK_SINK
        def sink(ctx, vals, off, n):
            got.extend(ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n))
            if len(got) == 8 * n:
                blocked.set()
                release.wait(10)
            return 0
        res["g"] = lib.ipls_agg_get_partitions_wire_chunked(h, 65536, sink, None)
    tg = threading.Thread(target=run_g)
    tg.start()
    assert blocked.wait(30)
    t0 = time.perf_counter()
    for p in range(4):
        assert lib.ipls_agg_set_weights(h, p, w_new.ctypes.data, L, N.HOST_F64) == 0
    inside = time.perf_counter() - t0
    assert "g" not in res
    release.set()
    tg.join(30)
    assert res["g"] == 0 and inside < 0.5, inside
    assert bytes(got) == want, "the wire stream is the model at the call"
    agg.close()


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_chunked_stage_pool_under_concurrency(ipls, O, devices):
    """The per-call staging of the chunked calls (a pool of stages per shard,
    each regrown only by the call that owns it): six threads, one partition
    each (three per shard on a [0, 0] handle), run random sequences of
    accumulate_chunked (chunk sizes from 2 Ki to 1 Mi values, so stages are
    regrown both ways), sources that stop mid-bucket (nothing folded),
    finalize_chunked (the commit_update bytes) and get_partitions_chunked
    (every partition's snapshot; each thread checks its own slice).  Every
    result is bit-exact against the oracle replaying that thread's sequence."""
    import threading
    from ipls import _native as N
    P, L = 6, 200003
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, devices=devices)
    lib, h = agg._lib, agg._h
    chunks = (2048, 65536, 100002, 1 << 20)
    errs = []

    def worker(p):
        try:
            rng = np.random.default_rng(100 + p)
            acc, w = np.zeros(L), np.zeros(L)
            for i in range(14):
                op = rng.choice(["acc", "acc", "stop", "fin", "getp"])
                chunk = int(rng.choice(chunks))
                if op in ("acc", "stop"):
                    g = O.synth_bucket(L, p, 1000 + i) * (1.0 + i)
                    raw = g.tobytes()
                    stop_at = int(rng.integers(0, (L + chunk - 1) // chunk)) if op == "stop" else -1

                    @N.CHUNK_SOURCE
                    def src(ctx, dst, off, n, raw=raw, stop_at=stop_at, chunk=chunk):
                        ctypes.memmove(dst, ctypes.c_char_p(raw[8 * off:8 * (off + n)]), 8 * n)
                        return 1 if off // chunk == stop_at else 0
                    rc = lib.ipls_agg_accumulate_chunked(h, p, ipls.TGT_AGG, L, N.HOST_F64, chunk, src, None)
                    if op == "acc":
                        assert rc == 0, (p, i, rc)
                        acc = O.fold(acc, g)
                    else:
                        assert rc == N.IPLS_E_INVAL, (p, i, rc)
                elif op == "fin":
                    out = bytearray(8 * L)

                    @N.CHUNK_SINK
                    def sink(ctx, vals, off, n, out=out):
                        out[8 * off:8 * (off + n)] = ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n)
                        return 0
                    assert lib.ipls_agg_finalize_chunked(h, p, N.HOST_BE, chunk, sink, None) == 0
                    w = acc + 0.0
                    assert bytes(out) == O.be_encode(w), (p, i, "commit_update bytes")
                    acc = np.zeros(L)
                else:
                    got = bytearray()
                    lo, hi = 8 * p * (L - 1), 8 * (p + 1) * (L - 1)

                    @N.CHUNK_SINK
                    def gsink(ctx, vals, off, n, got=got):
                        a, b = 8 * off, 8 * (off + n)
                        if b > lo and a < hi:
                            v = ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n)
                            got.extend(v[max(lo - a, 0):min(hi, b) - a])
                        return 0
                    assert lib.ipls_agg_get_partitions_chunked(h, chunk, gsink, None) == 0
                    assert bytes(got) == O.get_partitions([w]).tobytes(), (p, i, "GetPartitions slice")
            assert_bits_equal(agg.read(p, ipls.TGT_AGG), acc, f"partition {p}")
        except BaseException as e:   # noqa: BLE001 -- reported by the main thread
            errs.append((p, repr(e)))
    ths = [threading.Thread(target=worker, args=(p,)) for p in range(P)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    assert not errs, errs
    agg.close()


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_finalize_chunked(ipls, O, devices):
    """ipls_agg_finalize_chunked: AggregatePartition (W = AGG + REP,
    IPLS.java:1248-1274) with W handed to a sink chunk by chunk, as one call:
    the commit_update bytes (big-endian) or doubles equal the oracle's, for
    several chunk sizes; a sink that stops gets IPLS_E_INVAL after the round
    is consumed; an odd chunk or a bad kind is refused with the round left in
    place."""
    from ipls import _native as N
    L = 200003
    agg = ipls.Aggregator(n_partitions=2, bucket_len=L, devices=devices)
    lib, h = agg._lib, agg._h
    for k, (kind, chunk) in enumerate(((N.HOST_BE, 65536), (N.HOST_F64, 100002), (N.HOST_BE, 1 << 22), (N.HOST_BE, 2))):
        a, r = O.synth_bucket(L, 1, 80 + k), O.synth_bucket(L, 1, 90 + k) * 3.0
        agg.Update(a, 1)
        agg.Update(r, 1, from_clients=False)
        if k == 0:   # refused calls leave the round in place
            assert lib.ipls_agg_finalize_chunked(h, 1, N.HOST_BE, 65537, N.CHUNK_SINK(lambda *x: 0), None) == N.IPLS_E_INVAL
            assert lib.ipls_agg_finalize_chunked(h, 1, N.DEV_F64, 65536, N.CHUNK_SINK(lambda *x: 0), None) == N.IPLS_E_INVAL
            assert lib.ipls_agg_finalize_chunked(h, 2, N.HOST_BE, 65536, N.CHUNK_SINK(lambda *x: 0), None) == N.IPLS_E_RANGE
        out = bytearray(8 * L)
        seen = []

        @N.CHUNK_SINK
        def sink(ctx, vals, off, n):
            seen.append((off, n))
            out[8 * off:8 * (off + n)] = ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n)
            return 0
        if chunk == 2:                                   # 100,002 sink calls: keep them cheap
            @N.CHUNK_SINK
            def sink(ctx, vals, off, n):                 # noqa: F811
                seen.append((off, n))
                if off < 4096 or off > L - 4096:
                    out[8 * off:8 * (off + n)] = ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n)
                return 0
        assert lib.ipls_agg_finalize_chunked(h, 1, kind, chunk, sink, None) == 0
        assert [o for o, _ in seen] == list(range(0, L, min(chunk, L))) and sum(n for _, n in seen) == L
        w = O.fold(np.zeros(L), a) + O.fold(np.zeros(L), r)
        want = O.be_encode(w) if kind == N.HOST_BE else w.tobytes()
        if chunk == 2:
            assert out[:8 * 4096] == want[:8 * 4096] and out[-8 * 4000:] == want[-8 * 4000:]
        else:
            assert bytes(out) == want, f"finalize chunked {k}"
        assert_bits_equal(agg.read(1, ipls.TGT_AGG), np.zeros(L), "AGG zeroed")
    a = O.synth_bucket(L, 1, 99)
    agg.Update(a, 1)
    calls = []

    @N.CHUNK_SINK
    def stop(ctx, vals, off, n):
        calls.append(off)
        return 1
    assert lib.ipls_agg_finalize_chunked(h, 1, N.HOST_BE, 65536, stop, None) == N.IPLS_E_INVAL
    assert calls == [0]
    assert_bits_equal(agg.read(1, ipls.TGT_WEIGHTS), O.fold(np.zeros(L), a) + 0.0, "the round is consumed")
    agg.close()


def test_encode_secure_device(ipls, O, golden):
    x = golden["enc_in"]
    t, d = dev(x)
    o = torch.empty(8 * len(x), dtype=torch.uint8, device="cuda")
    ipls.encode_secure(d, ipls.DeviceBuffer(int(o.data_ptr()), len(x), big_endian=True))
    torch.cuda.synchronize()
    assert bytes(o.cpu().numpy()) == O.be_encode(golden["enc_out"])


# ---------------------------------------------------------------------------
# fused round: folds + AggregatePartition + GetPartitions divide in one launch
# ---------------------------------------------------------------------------
def _round_oracle(O, own_prev, rounds_buckets, reps, secure=False):
    """AGG = fold(prev arrivals) then fold(batch); W = AGG + REP; avg = divide(W)."""
    out_w, out_avg = [], []
    for prev, batch, rep in zip(own_prev, rounds_buckets, reps):
        L = len(batch[0]) if batch else len(prev[0]) if prev else len(rep[0])
        a = O.reduce(prev, L) if prev else np.zeros(L)
        a = O.reduce(batch, L, O.START_ACCUM, acc=a) if batch else a
        r = O.reduce(rep, L) if rep else np.zeros(L)
        w = a + r
        out_w.append(w)
        out_avg.append(O.divide(w, secure))
    return out_w, np.concatenate(out_avg)


@pytest.mark.parametrize("be", [False, True])
@pytest.mark.parametrize("secure", [False, True])
def test_aggregate_round_model_geometry(ipls, O, be, secure):
    """Ragged -pa geometry; partition 0 has earlier arrivals in AGG (ACCUM
    start), partition 1 has replicas in REP, partition 2 starts from zero."""
    M, P, K = 300007, 3, 5
    agg = ipls.Aggregator(M, P, max_peers=K, secure=secure)
    Ls = agg.lengths
    prev = [[O.synth_bucket(Ls[0], 0, 90 + j) for j in range(2)], [], []]
    reps = [[], [O.synth_bucket(Ls[1], 1, 80 + j) for j in range(3)], []]
    batch = [[O.synth_bucket(Ls[p], p, k) for k in range(K)] for p in range(P)]
    for b in prev[0]:
        agg.Update(b, 0, from_clients=True)
    for r in reps[1]:
        agg.Update(r, 1, from_clients=False)
    keep, rows = [], []
    for p in range(P):
        row = []
        for b in batch[p]:
            t, d = dev_be(b) if be else dev(b)
            keep.append(t)
            row.append(d)
        rows.append(row)
    avg = agg.aggregate_round(0, rows, big_endian=be)
    ref_w, ref_avg = _round_oracle(O, prev, batch, reps, secure)
    assert_bits_equal(avg, ref_avg, "avg")
    for p in range(P):
        assert_bits_equal(agg.read(p, ipls.TGT_WEIGHTS), ref_w[p], f"W[{p}]")
        assert not agg.read(p, ipls.TGT_AGG).any() and not agg.read(p, ipls.TGT_REP).any()
    # the unfused sequence gives the same model
    assert_bits_equal(agg.GetPartitions(), ref_avg, "GetPartitions after round")
    # next round starts from +0.0
    agg.aggregate_round(0, [rows[0][:1]], big_endian=be, with_average=False)
    assert_bits_equal(agg.read(0, ipls.TGT_WEIGHTS), O.reduce(batch[0][:1], Ls[0]) + 0.0, "next round")
    agg.close()


@pytest.mark.parametrize("shift", [0, 1])
def test_aggregate_round_big_shape_device_out(ipls, O, shift):
    """The fused round's half shape (4 x 64 big tiles: 512 lanes) with a
    partial tile; averages into a device buffer that is 16-B aligned (shift
    0) or 8 mod 16 (shift 1: lane-pair stores)."""
    P, L, K = 4, 2100001, 3
    arena = torch.empty(P * K * (L + 1), dtype=torch.float64, device="cuda")
    base = int(arena.data_ptr())
    rows = [[ipls.DeviceBuffer(base + 8 * (p * K + k) * (L + 1), L) for k in range(K)] for p in range(P)]
    for p in range(P):
        for k in range(K):
            ipls.synth_fill(rows[p][k], p, k, O.SEED)
    out = torch.full((P * (L - 1) + 2,), 7.0, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()   # fills and the poison ran on the null stream; the handle's is non-blocking
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    agg.Update(O.synth_bucket(L, 3, 77), 3, from_clients=False)    # one partition with REP
    # undersized operands are refused before any launch (bare pointers at the C-ABI)
    with pytest.raises(ValueError, match="averages"):
        agg.aggregate_round(0, rows, out=ipls.DeviceBuffer(int(out.data_ptr()) + 8 * shift, P * (L - 1) - 1))
    with pytest.raises(ValueError, match="needs buckets"):
        agg.aggregate_round(0, rows[:3] + [rows[3][:2] + [ipls.DeviceBuffer(rows[3][2].ptr, L - 1)]],
                            out=ipls.DeviceBuffer(int(out.data_ptr()) + 8 * shift, P * (L - 1)))
    agg.aggregate_round(0, rows, out=ipls.DeviceBuffer(int(out.data_ptr()) + 8 * shift, P * (L - 1)))
    torch.cuda.synchronize()
    full = out.cpu().numpy()
    got = full[shift:shift + P * (L - 1)]
    assert full[:shift].tolist() == [7.0] * shift and full[shift + P * (L - 1):].tolist() == [7.0] * (2 - shift)
    for p in (0, 3):
        S = O.reduce([O.synth_bucket(L, p, k) for k in range(K)], L)
        S = S + (O.synth_bucket(L, 3, 77) if p == 3 else 0.0)
        assert_bits_equal(agg.read(p, ipls.TGT_WEIGHTS), S, f"W[{p}]")
        assert_bits_equal(got[p * (L - 1):(p + 1) * (L - 1)], O.divide(S), f"avg[{p}]")
    assert [agg.checksum(p, ipls.TGT_WEIGHTS) for p in (1, 2)] == \
        [O.c_synth_sum_checksum(L, p, K) for p in (1, 2)]
    agg.close()
    del arena, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("P", [16, 4])
@pytest.mark.parametrize("shift,accum,secure", [(0, False, False), (1, True, False), (0, True, True),
                                                (1, False, False)])
def test_aggregate_round_whole_tiles(ipls, O, shift, accum, secure, P):
    """Partitions of whole 1024-lane tiles (config C's shape class, no
    partial tile anywhere) through the fused round's big shape: every
    partition's W and averages compared in full (odd and even partitions,
    averages buffer 16-B aligned or 8 mod 16, i.e. both store paths of the
    averages-before-W epilogue), with AGG started from a previous arrival
    (ACCUM) or zero, and the secure divide.  16 partitions of 2M run the big
    shape (1024 big tiles); 4 run the half shape from zero and the big R = 8
    shape on top of AGG (ACCUM)."""
    L, K = 2097152, 3
    arena = torch.empty(P * K * (L + 32), dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = [[ipls.DeviceBuffer(base + 8 * (p * K + k) * (L + 32), L) for k in range(K)] for p in range(P)]
    for p in range(P):
        for k in range(K):
            ipls.synth_fill(rows[p][k], p, k, O.SEED)
    out = torch.full((P * (L - 1) + 2,), 7.0, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, secure=secure)
    first = [O.synth_bucket(L, p, 50) for p in range(P)]
    if accum:
        for p in range(P):
            agg.Update(first[p], p, from_clients=True)
    agg.aggregate_round(0, rows, out=ipls.DeviceBuffer(int(out.data_ptr()) + 8 * shift, P * (L - 1)))
    li = agg.last_launch()
    want = ipls.SHAPE_BIG if (P == 16 or accum) else ipls.SHAPE_HALF
    assert li["kernel"] == ipls.KERNEL_ROUND and li["shape"] == want and li["map"] != 3, li
    torch.cuda.synchronize()
    full = out.cpu().numpy()
    got = full[shift:shift + P * (L - 1)]
    assert full[:shift].tolist() == [7.0] * shift and full[shift + P * (L - 1):].tolist() == [7.0] * (2 - shift)
    for p in range(P):
        bk = [O.synth_bucket(L, p, k) for k in range(K)]
        S = O.reduce(bk, L, ipls.START_ACCUM, acc=first[p]) if accum else O.reduce(bk, L)
        S = S + 0.0
        assert_bits_equal(agg.read(p, ipls.TGT_WEIGHTS), S, f"W[{p}]")
        assert_bits_equal(got[p * (L - 1):(p + 1) * (L - 1)], O.divide(S, secure=secure), f"avg[{p}]")
    agg.close()
    del arena, out
    torch.cuda.empty_cache()


def test_aggregate_round_edges(ipls, O, golden):
    """k = 0 (W = AGG + REP), a zero count slot (values pass through),
    special values, a sub-range of partitions, 8-B aligned buckets (unfused
    fallback)."""
    L = 1031
    agg = ipls.Aggregator(n_partitions=4, bucket_len=L)
    b = O.synth_bucket(L, 0, 0)
    agg.Update(b, 1, from_clients=True)
    avg = agg.aggregate_round(1, [[]])
    assert_bits_equal(avg, O.divide(b + 0.0), "k=0")
    assert_bits_equal(agg.read(1, ipls.TGT_WEIGHTS), b + 0.0, "k=0 W")
    # count slot 0 -> pass through; specials from the golden edge cases
    z = O.synth_bucket(L, 2, 0)
    z[-1] = 0.0
    t1, d1 = dev(z)
    avg = agg.aggregate_round(2, [[d1]])
    assert_bits_equal(avg, O.divide(z + 0.0), "cnt 0")
    # 8-B aligned buckets -> unfused path, same results
    raw = torch.empty(2 * L + 1, dtype=torch.float64, device="cuda")
    x = [O.synth_bucket(L, 3, k) for k in range(2)]
    raw[1:L + 1] = torch.from_numpy(x[0]).cuda()
    raw[L + 1:] = torch.from_numpy(x[1]).cuda()
    base = int(raw.data_ptr())
    avg = agg.aggregate_round(3, [[ipls.DeviceBuffer(base + 8, L), ipls.DeviceBuffer(base + 8 * (L + 1), L)]])
    S = O.reduce(x, L)
    assert_bits_equal(avg, O.divide(S), "unaligned")
    assert_bits_equal(agg.read(3, ipls.TGT_WEIGHTS), S, "unaligned W")
    agg.close()
    # NaN / inf / -0.0 / subnormal buckets (golden), the count slot among them
    sb = golden["special_bufs"]
    agg = ipls.Aggregator(n_partitions=1, bucket_len=sb.shape[1])
    keep = [dev(r) for r in sb]
    avg = agg.aggregate_round(0, [[d for _, d in keep]])
    W = golden["special_zero"] + 0.0
    assert_bits_equal(agg.read(0, ipls.TGT_WEIGHTS), W, "special W")
    assert_bits_equal(avg, O.divide(W), "special avg")
    agg.close()


def test_future_accumulator_and_promotion(ipls, O):
    """Updater.java:99-101 folds a bucket for a later iteration into
    Aggregated_Gradients_from_future; Update_Client_WaitAck_List
    (IPLS.java:1556-1562) then makes it the new AGG and zeroes it."""
    M, P = 200003, 4
    agg = ipls.Aggregator(M, P, max_peers=4)
    Ls = agg.lengths
    now = [[O.synth_bucket(Ls[p], p, k) for k in range(2)] for p in range(P)]
    fut = [[O.synth_bucket(Ls[p], p, 10 + k) for k in range(3)] for p in range(P)]
    for p in range(P):
        for b in now[p]:
            agg.Update(b, p)
        for b in fut[p]:
            agg.Update(O.be_encode(b), p, from_future=True)       # BE file bytes
    # this round sees only the current-iteration buckets
    for p in range(P):
        assert_bits_equal(agg.read(p), O.reduce(now[p], Ls[p]), f"AGG[{p}]")
        assert_bits_equal(agg.read(p, ipls.TGT_FUTURE), O.reduce(fut[p], Ls[p]), f"FUT[{p}]")
    avg = agg.aggregate_round(0, [[] for _ in range(P)])
    assert_bits_equal(avg, O.get_partitions([O.reduce(now[p], Ls[p]) for p in range(P)]), "round 1")
    # promotion for the Auth_List {1, 3}; 0 and 2 keep an empty AGG and their FUT
    agg.PromoteFuture([1, 3])
    ref_agg = [np.zeros(L) for L in Ls]
    ref_fut = [O.reduce(fut[p], Ls[p]) for p in range(P)]
    for p in (1, 3):
        O.promote_future(ref_agg[p], ref_fut[p])
    for p in range(P):
        assert_bits_equal(agg.read(p), ref_agg[p], f"AGG after promote [{p}]")
        assert_bits_equal(agg.read(p, ipls.TGT_FUTURE), ref_fut[p], f"FUT after promote [{p}]")
    # the next iteration's arrivals fold on top of the promoted sums
    extra = O.synth_bucket(Ls[1], 1, 99)
    agg.Update(extra, 1)
    assert_bits_equal(agg.read(1), O.reduce([extra], Ls[1], O.START_ACCUM, acc=ref_agg[1].copy()), "fold after")
    agg.Update(extra, 1, from_future=True)
    assert_bits_equal(agg.read(1, ipls.TGT_FUTURE), O.reduce([extra], Ls[1]), "FUT refills from +0.0")
    with pytest.raises(ipls.IplsError):
        agg.PromoteFuture([P])
    agg.close()


def test_update_indirect_gradient_buff(ipls, O):
    """Updater.run indirect requests (Updater.java:162-187): every file goes
    through the one reusable Gradient_Buff, so a short file folds the previous
    file's tail and an over-long one raises after overwriting the buffer."""
    M, P = 100003, 3
    agg = ipls.Aggregator(M, P, max_peers=3)
    Ls = agg.lengths
    G = O.gradient_buff_len(M, P)
    assert G >= max(Ls)
    buff = np.zeros(G)
    acc = [np.zeros(L) for L in Ls]

    def step(p, vals, pinned=False, fut=False):
        data = O.be_encode(vals)
        if pinned:
            pb = ipls.PinnedBuffer(len(data))
            pb.view()[:] = np.frombuffer(data, dtype=np.uint8)
            src = pb
        else:
            src = data
        try:
            O.get_parameters_into(buff, data)
        except IndexError:
            with pytest.raises(ipls.IplsError):
                agg.UpdateIndirect(src, p)
            return
        agg.UpdateIndirect(src, p, from_future=fut)
        if not fut:
            acc[p][:] = O.reduce([buff[:Ls[p]]], Ls[p], O.START_ACCUM, acc=acc[p])

    step(0, O.synth_bucket(Ls[0], 0, 1), pinned=True)     # whole partition, zero-copy source
    step(1, O.synth_bucket(Ls[1] - 100, 1, 1))             # short: 100 stale values from the last file
    step(2, O.synth_bucket(Ls[2], 2, 1))                   # last partition (2 shorter than G)
    step(0, O.synth_bucket(G + 5, 0, 2))                   # too long: AIOOBE, buffer overwritten
    step(0, O.synth_bucket(10, 0, 3))                      # 10 new values + the long file's tail
    step(1, O.synth_bucket(Ls[1], 1, 4), pinned=True)
    step(2, np.zeros(0))                                   # empty file: all stale
    for p in range(P):
        assert_bits_equal(agg.read(p), acc[p], f"AGG[{p}]")
    agg.close()


def test_other_replica_gradients_and_collect(ipls, O):
    """Download_Scheduler.java:245-268 + IPLS.Collect_Replicas (:1217-1241):
    per-(partition, aggregator) arrays, FIRST-started (so -0.0 survives), folded
    into REP in the JDK HashMap's key order after what REP already holds."""
    M, P = 80001, 2
    agg = ipls.Aggregator(M, P, max_peers=4)
    Ls = agg.lengths
    rep = [np.zeros(L) for L in Ls]
    store = O.ReplicaStore()
    own_rep = O.synth_bucket(Ls[0], 0, 50)
    agg.Update(own_rep, 0, from_clients=False)                 # a replica that did answer
    rep[0] = O.reduce([own_rep], Ls[0])
    negz = O.synth_bucket(Ls[0], 0, 60)
    negz[::7] = -0.0
    downloads = [(0, 7, negz), (0, 3, O.synth_bucket(Ls[0], 0, 61)), (0, 7, O.synth_bucket(Ls[0], 0, 62)),
                 (1, 5, O.synth_bucket(Ls[1], 1, 63)), (1, 5, O.synth_bucket(Ls[1] - 1000, 1, 64))]
    for i, (p, a, g) in enumerate(downloads):
        O.other_replica_add(store, p, a, g)
        agg.OtherReplicaGradients(p, a, O.be_encode(g) if i % 2 else g)   # BE file bytes or doubles
    with pytest.raises(ipls.IplsError):                         # longer than the stored array
        agg.OtherReplicaGradients(1, 5, O.synth_bucket(Ls[1] + 3, 1, 65))
    parts_ref = [0] * P
    n_ref = O.collect_replicas(rep, store, parts_ref)
    n, parts = agg.Collect_Replicas()
    assert (n, parts) == (n_ref, parts_ref) == (3, [3 * Ls[0], 2 * Ls[1]])   # received x length (IPLS.java:1229-1234)
    for p in range(P):
        assert_bits_equal(agg.read(p, ipls.TGT_REP), rep[p], f"REP[{p}]")
    assert agg.Collect_Replicas() == (0, [0, 0])               # the store was cleared
    agg.close()


def test_replica_drop_when_its_partial_arrives(ipls, O):
    """VERDICT r3 next 2 (Download_Scheduler.java:215-217, 329-332, 438-440):
    buckets of two other aggregators of one partition are downloaded; one of
    them then publishes its partial sum, which the Updater's replica branch
    folds into REP (Updater.java:40-44), and its stored downloads are removed,
    so Collect_Replicas folds only the other aggregator's -- nothing counted
    twice.  Bit-exact vs the oracle; the drop of an absent key is a no-op."""
    L, P = 70001, 2
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    store = O.ReplicaStore()
    rep = [np.zeros(L) for _ in range(P)]
    ids = {11: "12D3KooWAggregatorB", 12: "12D3KooWAggregatorC"}
    for a, ks in ((11, (70, 71)), (12, (72, 73, 74))):
        for k in ks:
            g = O.synth_bucket(L, 0, k)
            kh = ipls.java_pair_hash(0, ids[a])
            assert kh == O.java_pair_hash(0, ids[a])
            agg.OtherReplicaGradients(0, a, g, key_hash=kh)
            O.other_replica_add(store, 0, a, g, key_hash=kh)
    partial_b = O.reduce([O.synth_bucket(L, 0, k) for k in (70, 71, 75)], L)   # B's own published partial
    agg.Update(partial_b, 0, from_clients=False)                                 # replica branch -> REP
    rep[0] = rep[0] + partial_b
    assert agg.OtherReplicaDrop(0, 11) is True and O.other_replica_drop(store, 0, 11)
    assert agg.OtherReplicaDrop(0, 11) is False                                  # already gone
    assert agg.OtherReplicaDrop(1, 12) is False                                  # never stored for p 1
    parts_ref = [0] * P
    n_ref = O.collect_replicas(rep, store, parts_ref)
    n, parts = agg.Collect_Replicas()
    assert (n, parts) == (n_ref, parts_ref) == (1, [3 * L, 0])                   # only C's 3 downloads (x L, per element)
    assert_bits_equal(agg.read(0, ipls.TGT_REP), rep[0], "REP[0] after drop + collect")
    # without the drop B's downloads would have been folded as well
    twice = partial_b + O.reduce([O.synth_bucket(L, 0, k) for k in (70, 71)], L, ipls.START_FIRST) \
        + O.reduce([O.synth_bucket(L, 0, k) for k in (72, 73, 74)], L, ipls.START_FIRST)
    assert not np.array_equal(twice.view(np.uint64), rep[0].view(np.uint64))
    agg.close()


def test_replica_store_argument_errors(ipls, O):
    """The keyed store refuses what would desynchronise it from Java's map:
    a second key hash for a stored key (IPLS_E_INVAL, nothing folded), an
    out-of-range partition (ArrayIndexOutOfBounds); a failed call leaves the
    store and its order as they were."""
    from ipls import _native as N
    L, P = 1001, 2
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    g = O.synth_bucket(L, 0, 1)
    kh = O.java_pair_hash(0, "12D3KooWA")
    agg.OtherReplicaGradients(0, 4, g, key_hash=kh)
    before = agg.replica_order()
    with pytest.raises(ipls.IplsError) as e:
        agg.OtherReplicaGradients(0, 4, g, key_hash=kh + 1)
    assert e.value.code == N.IPLS_E_INVAL
    with pytest.raises(ipls.IplsError) as e:
        agg.OtherReplicaGradients(P, 4, g, key_hash=kh)
    assert e.value.code == N.IPLS_E_RANGE
    with pytest.raises(ipls.IplsError):
        agg.OtherReplicaDrop(-1, 4)
    assert agg.replica_order() == before
    # a buffer with less room than there are keys: the full count comes back,
    # only max_pairs pairs are written (the callers ask again with more room)
    agg.OtherReplicaGradients(1, 5, O.synth_bucket(L, 1, 2), key_hash=O.java_pair_hash(1, "12D3KooWB"))
    keys, _ = agg.replica_order()
    buf = (ctypes.c_int32 * 4)(*([-7] * 4))
    assert agg._lib.ipls_agg_replica_order(agg._h, buf, 1, None) == 2
    assert list(buf) == [keys[0][0], keys[0][1], -7, -7]
    assert agg.OtherReplicaDrop(1, 5) is True
    n, parts = agg.Collect_Replicas()
    assert (n, parts) == (1, [L, 0])
    assert_bits_equal(agg.read(0, ipls.TGT_REP), 0.0 + g, "REP[0]")    # folded once, not twice
    assert agg.replica_order() == ([], 0)                             # new HashMap<>()
    agg.close()


def _ids_with_non_ascending_order(O, p, n):
    """n peer IDs whose Pair(p, id) hashes fall in bins 13, 7, 2 of a 16-bin
    HashMap: stored in that order, they iterate in reverse -- neither
    ascending index nor insertion order."""
    ids, i = [], 0
    for target in (13, 7, 2)[:n]:
        while True:
            cand = f"QmPeer{i:04d}"
            i += 1
            if O.JavaHashMap.spread(O.java_pair_hash(p, cand)) & 15 == target:
                ids.append(cand)
                break
    return ids


def test_collect_replicas_in_java_hashmap_order(ipls, O):
    """VERDICT r3 next 3 (IPLS.java:1218-1227, PeerData.java:140): three stored
    arrays on partition 0 and two on partition 1 (whose REP already holds a
    replica's partial), keyed by peer IDs whose HashMap order differs from
    both ascending index and insertion order.  The GPU result matches the
    oracle's table simulation bit for bit, and differs from the ascending
    order's bits (so the order is what the test checks)."""
    L, P = 60007, 2
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    store = O.ReplicaStore()
    rep = [np.zeros(L) for _ in range(P)]
    scale = [1e16, 1.0, -1e16]                 # cancellation: any other order changes the bits
    pre = O.synth_bucket(L, 1, 90) * 3.0
    agg.Update(pre, 1, from_clients=False)
    rep[1] = rep[1] + pre
    plan = {0: _ids_with_non_ascending_order(O, 0, 3), 1: _ids_with_non_ascending_order(O, 1, 2)}
    arrays = {}
    for p, ids in plan.items():
        for a, pid in enumerate(ids):
            g = O.synth_bucket(L, p, 80 + a) * scale[a]
            kh = O.java_pair_hash(p, pid)
            agg.OtherReplicaGradients(p, a, g, key_hash=kh)
            O.other_replica_add(store, p, a, g, key_hash=kh)
            arrays[(p, a)] = g
    order = store.map.keys()
    assert order != sorted(order)
    asc = [r.copy() for r in rep]
    for (p, a) in sorted(arrays):
        asc[p] = asc[p] + arrays[(p, a)]
    n_ref = O.collect_replicas(rep, store, [0] * P)
    n, parts = agg.Collect_Replicas()
    assert n == n_ref == 5 and parts == [3 * L, 2 * L]
    for p in range(P):
        assert_bits_equal(agg.read(p, ipls.TGT_REP), rep[p], f"REP[{p}] (HashMap order)")
    assert any(not np.array_equal(asc[p].view(np.uint64), rep[p].view(np.uint64)) for p in range(P))
    agg.close()


def test_collect_replicas_order_after_resize_and_drops(ipls, O):
    """Enough keys to resize the map (13 keys > 0.75 x 16, 25 > 0.75 x 32),
    drops in between (the capacity stays), keys re-stored after a drop (they go
    to the tail of their bin), and a collect that resets the map: every REP
    matches the oracle's JDK table simulation bit for bit."""
    L, P = 4099, 4
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    store = O.ReplicaStore()
    rep = [np.zeros(L) for _ in range(P)]
    rng = np.random.default_rng(5)
    for rnd in range(2):
        for i in range(60):
            p, a = int(rng.integers(0, P)), int(rng.integers(0, 9))
            if rng.integers(0, 5) == 0:
                assert agg.OtherReplicaDrop(p, a) == O.other_replica_drop(store, p, a)
                continue
            g = O.synth_bucket(L, p, i) * float(10.0 ** rng.integers(-8, 9))
            kh = O.java_pair_hash(p, f"12D3KooW{a}{'x' * a}")
            agg.OtherReplicaGradients(p, a, g, key_hash=kh)
            O.other_replica_add(store, p, a, g, key_hash=kh)
            if i % 10 == 9:                       # the library's model vs the simulated JDK table
                assert agg.replica_order() == (store.map.keys(), len(store.map.table) if store.map.table else 0)
        assert len(store.map.table) >= 32 and not store.map.tree_bin
        exp_parts = [0] * P
        n_ref = O.collect_replicas(rep, store, exp_parts)
        assert agg.Collect_Replicas() == (n_ref, exp_parts)
        for p in range(P):
            assert_bits_equal(agg.read(p, ipls.TGT_REP), rep[p], f"round {rnd} REP[{p}]")
    agg.close()


def test_collect_replicas_order_through_a_tree_bin(ipls, O):
    """A HashMap bin that becomes a red-black tree (HashMap.treeifyBin at 9
    keys and >= 64 bins): 14 keys whose hashes share the low 8 bits go to one
    bin, drops unlink tree nodes (removeTreeNode), and more keys resize the
    table so TreeNode.split cuts the tree into a half that stays a tree and
    a half of at most 6 keys that becomes a chain again (untreeify).  The library's order model and the oracle's
    JDK simulation agree on the key order at every step, and the collect
    folds in that order bit for bit, with cancelling magnitudes so a
    different order changes the bits."""
    L, P = 2053, 3
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    store = O.ReplicaStore()
    rep = [np.zeros(L) for _ in range(P)]
    scale = [1e16, 1.0, -1e16, 3.0, -1.0, 1e-3]
    coll = [(j % P, j) for j in range(14)]              # hashes 0x1A + 64 j: spread(h) = h
    for i, (p, a) in enumerate(coll):
        g = O.synth_bucket(L, p, 300 + i) * scale[i % len(scale)]
        kh = 0x1A + 64 * i
        agg.OtherReplicaGradients(p, a, g, key_hash=kh)
        O.other_replica_add(store, p, a, g, key_hash=kh)
    assert store.map.tree_bin and len(store.map.table) == 64
    assert agg.replica_order() == (store.map.keys(), 64)
    for p, a in (coll[1], coll[7], coll[11]):
        assert agg.OtherReplicaDrop(p, a) == O.other_replica_drop(store, p, a) == 1
    assert agg.replica_order() == (store.map.keys(), 64)
    for j in range(60):                                  # 71 keys > 0.75 x 64: 128 bins
        p, a = j % P, 100 + j
        g = O.synth_bucket(L, p, 400 + j) * scale[j % len(scale)]
        kh = O.java_pair_hash(p, f"12D3KooWFill{j}")
        agg.OtherReplicaGradients(p, a, g, key_hash=kh)
        O.other_replica_add(store, p, a, g, key_hash=kh)
    tab = store.map.table
    assert len(tab) == 128 and not store.map.nondeterministic
    assert tab[0x1A] is not None and tab[0x1A].tree                # even j (and fill keys): still a tree
    assert tab[0x1A + 64] is not None and not tab[0x1A + 64].tree  # odd j: a chain again
    assert agg.replica_order() == (store.map.keys(), 128)
    exp_parts = [0] * P
    n_ref = O.collect_replicas(rep, store, exp_parts)
    assert agg.Collect_Replicas() == (n_ref, exp_parts)
    for p in range(P):
        assert_bits_equal(agg.read(p, ipls.TGT_REP), rep[p], f"REP[{p}] (tree bin)")
    agg.close()


def test_collect_replicas_many_keys(ipls, O):
    """A store of ~1,500 keys (64 partitions x up to 40 aggregators, real
    Pair hashes of peer-ID strings; the map grows to 2,048 bins), with drops:
    the library's order equals the JDK simulation's, and the collect folds
    every key into REP bit for bit with the reference's Participants."""
    L, P, A = 33, 64, 40
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    store = O.ReplicaStore()
    rep = [np.zeros(L) for _ in range(P)]
    rng = np.random.default_rng(17)
    for i in range(2600):
        p, a = int(rng.integers(0, P)), int(rng.integers(0, A))
        if rng.integers(0, 10) == 0:
            assert agg.OtherReplicaDrop(p, a) == O.other_replica_drop(store, p, a)
            continue
        g = O.synth_bucket(L, p, i) * float(10.0 ** rng.integers(-6, 7))
        kh = O.java_pair_hash(p, f"QmPeer{a:03d}")
        agg.OtherReplicaGradients(p, a, g, key_hash=kh)
        O.other_replica_add(store, p, a, g, key_hash=kh)
    assert len(store.map) > 1200 and len(store.map.table) >= 2048
    assert agg.replica_order() == (store.map.keys(), len(store.map.table))
    exp_parts = [0] * P
    n_ref = O.collect_replicas(rep, store, exp_parts)
    assert agg.Collect_Replicas() == (n_ref, exp_parts)
    for p in range(P):
        assert_bits_equal(agg.read(p, ipls.TGT_REP), rep[p], f"REP[{p}] (many keys)")
    assert agg.replica_order() == ([], 0)
    agg.close()


def test_ack_frame_sets_weight_address(ipls, O):
    """ThreadReceiver pid 4 (IPLS.java:491-498): the ACK frame's payload becomes
    Weight_Address[p]; GetPartitions then divides it."""
    M, P = 30001, 2
    agg = ipls.Aggregator(M, P)
    Ls = agg.lengths
    ws = [O.synth_bucket(Ls[p], p, 3) for p in range(P)]
    for p in range(P):
        fr = O.frame_encode(np.concatenate([ws[p], [7.0, 8.0]]), p, 12, 4, b"QmServer")   # longer payload is fine
        agg.cache_partition(p, fr, frame=True)
        assert_bits_equal(agg.read(p, ipls.TGT_WADDR), ws[p], f"WADDR[{p}]")
    assert_bits_equal(agg.GetPartitions(), O.get_partitions(ws), "model")
    with pytest.raises(ipls.IplsError):
        agg.cache_partition(0, O.frame_encode(ws[0][:-1], 0, 12, 4, b"Qm"), frame=True)    # short payload
    agg.close()


def _free_hbm():
    free, _ = torch.cuda.mem_get_info()
    return free


@pytest.mark.parametrize("P,L,K", [(1, 2**31 - 3, 2), (3, 2**30 + 1, 2)])
def test_maximum_sizes(ipls, O, P, L, K):
    """Java's largest double[] (HotSpot: Integer.MAX_VALUE - 2) as one
    partition, and flat model offsets past 2^31 elements: byte offsets past
    2^34, through the fold, the fused round and the checksums."""
    need = 8 * L * (P * K + 4 * P + P) + (1 << 30)      # buckets + AGG/REP/W/FUT + averages
    if _free_hbm() < need:
        pytest.skip(f"needs {need / 2**30:.0f} GiB of free HBM")
    stride = L + (L & 1)                                  # keep every bucket 16-B aligned
    arena = torch.empty(P * K * stride, dtype=torch.float64, device="cuda")
    base = int(arena.data_ptr())
    rows = [[ipls.DeviceBuffer(base + 8 * (p * K + k) * stride, L) for k in range(K)] for p in range(P)]
    for p in range(P):
        for k in range(K):
            ipls.synth_fill(rows[p][k], p, k, O.SEED)
    # the fills ran on the null stream; the handle's stream is non-blocking
    torch.cuda.synchronize()
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
    ref = [O.c_synth_sum_checksum(L, p, K) for p in range(P)]
    assert [agg.checksum(p) for p in range(P)] == ref
    agg.reset(ipls.ALL_PARTITIONS)
    avg = torch.empty(P * (L - 1), dtype=torch.float64, device="cuda")
    agg.aggregate_round(0, rows, out=ipls.DeviceBuffer.from_tensor(avg))
    assert [agg.checksum(p, ipls.TGT_WEIGHTS) for p in range(P)] == ref
    for p in range(P):
        part = ipls.DeviceBuffer(int(avg.data_ptr()) + 8 * p * (L - 1), L - 1)
        assert ipls.checksum_dev(part) == O.c_synth_avg_checksum(L, p, K), f"avg[{p}]"
    agg.close()
    del arena, avg
    torch.cuda.empty_cache()


def test_maximum_sizes_elementwise(ipls, O):
    """The elementwise kernels in their 16-B tile shape on Java's largest
    partition (L = Integer.MAX_VALUE - 2, byte offsets up to 2^34):
    UpdateGradient's own accumulate into a logically-zero AGG and then a live
    one (k_split, IPLS.java:1737-1743), AggregatePartition, the async replica
    fold and the leaving-peer blend (k_blend, Updater.java:57-59,65-69) and the
    publish scale (k_scale, Updater.java:197-199), and a ranged fold and
    ranged read (the JNI ring's) near the partition's end.  Each state is checked by
    its position-keyed checksum against the same IEEE operations in torch fp64
    on the device (one rounding per multiply and per add, as the kernels do:
    -ffp-contract=off); the oracle's Python loops would take minutes here."""
    L = 2**31 - 3
    M = L - 1
    need = 8 * L * 10 + (1 << 30)        # AGG/REP/W/FUT + v + two expected states + temporaries
    if _free_hbm() < need:
        pytest.skip(f"needs {need / 2**30:.0f} GiB of free HBM")
    v = torch.empty(L, dtype=torch.float64, device="cuda")
    ipls.synth_fill(ipls.DeviceBuffer.from_tensor(v), 0, 3, O.SEED)
    torch.cuda.synchronize()
    v[M] = 1.0                           # OrganizeGradients' count slot (IPLS.java:1033)
    torch.cuda.synchronize()             # torch's stream; the handle's stream does not wait on it
    flat = ipls.DeviceBuffer(int(v.data_ptr()), M)
    agg = ipls.Aggregator(M, 1)
    assert agg.lengths == [L]

    def same(target, want, what):
        torch.cuda.synchronize()
        assert agg.checksum(0, target) == ipls.checksum_dev(ipls.DeviceBuffer.from_tensor(want)), what

    agg.UpdateGradient(flat, [0])
    exp = v + 0.0
    same(ipls.TGT_AGG, exp, "own accumulate into a logically-zero AGG")
    agg.UpdateGradient(flat, [0])
    exp = exp + v
    same(ipls.TGT_AGG, exp, "own accumulate into a live AGG")
    agg.AggregatePartition(0)
    w = exp + 0.0
    del exp
    same(ipls.TGT_WEIGHTS, w, "AggregatePartition")
    agg.UpdateAsyncReplica(ipls.DeviceBuffer.from_tensor(v), 0)
    w = w * 0.75 + v * 1.0
    same(ipls.TGT_WEIGHTS, w, "async replica fold")
    a = agg.LEAVING_A
    agg.UpdateLeavingPeer(ipls.DeviceBuffer.from_tensor(v), 0)
    w = w * a + v * (1 - a)
    same(ipls.TGT_WEIGHTS, w, "leaving-peer blend")
    agg.AsyncPublishScale(0)
    same(ipls.TGT_AGG, w * 0.25, "publish scale")
    del w
    # the JNI ring's ranged fold and read at element offsets past 2^31 - 2^20
    from ipls import _native as N
    n = 1 << 20
    off = (L - n - 1) & ~1
    chunk = O.synth_bucket(n, 5, 1)
    pin = ipls.PinnedBuffer(8 * n)
    pin.view()[:] = np.frombuffer(chunk.tobytes(), dtype=np.uint8)
    t = ctypes.c_uint64()
    assert agg._lib.ipls_agg_accumulate_range(agg._h, 0, ipls.TGT_REP, pin.ptr, off, n, N.HOST_F64,
                                              ctypes.byref(t)) == 0
    assert agg._lib.ipls_agg_wait(agg._h, t.value) == 0
    assert agg._lib.ipls_agg_read_range(agg._h, 0, ipls.TGT_REP, pin.ptr, off, n, N.HOST_BE, ctypes.byref(t)) == 0
    assert agg._lib.ipls_agg_wait(agg._h, t.value) == 0
    assert pin.view()[:8 * n].tobytes() == O.be_encode(chunk + 0.0), "ranged fold, then ranged read"
    rep = torch.zeros(L, dtype=torch.float64, device="cuda")
    rep[off:off + n] = torch.from_numpy(chunk + 0.0).to("cuda")
    same(ipls.TGT_REP, rep, "ranged fold into a logically-zero REP")
    pin.close()
    agg.close()
    del v, rep
    torch.cuda.empty_cache()


def test_async_pinned_arrivals(ipls, O):
    """ipls_agg_accumulate_async: queued zero-copy folds give the same bits as
    synchronous Updates, in call order, across more folds than the ticket ring."""
    L, K = 70001, 80
    bufs = []
    vals = [O.synth_bucket(L, 4, k) for k in range(8)]
    for k in range(8):
        pb = ipls.PinnedBuffer(8 * L)
        pb.view()[:] = np.frombuffer(O.be_encode(vals[k]), dtype=np.uint8)
        bufs.append(pb)
    agg = ipls.Aggregator(n_partitions=2, bucket_len=L)
    ref = np.zeros(L)
    tickets = []
    for j in range(K):                       # 80 folds > the 64-entry ring
        tickets.append(agg.UpdateAsync(bufs[j % 8], 0))
        ref = O.reduce([vals[j % 8]], L, O.START_ACCUM, acc=ref)
    assert tickets == sorted(tickets) and len(set(tickets)) == K
    agg.Wait(tickets[3])                     # an old ticket, long overwritten in the ring
    agg.Wait(tickets[-1])
    assert_bits_equal(agg.read(0), ref, "async folds")
    t = agg.UpdateAsync(bufs[0], 1, from_clients=False)
    agg.Wait(t)
    assert_bits_equal(agg.read(1, ipls.TGT_REP), O.reduce([vals[0]], L), "REP")
    with pytest.raises(ipls.IplsError):
        agg.Wait(tickets[-1] + 100)          # never issued
    agg.close()
    for pb in bufs:
        pb.close()


@pytest.mark.parametrize("group", [1, 3, 8, 32])
def test_async_device_coalesced(ipls, O, group):
    """Queued device arrivals (ipls_agg_accumulate_async, DEV_F64/DEV_BE) fold
    in call order with the same bits as one-by-one Updates, whatever flushes
    the queues: the group size, a byte-order change, a synchronous Update, a
    pinned-host async fold, a read, Wait.  Ragged queues across partitions,
    an odd length, an 8-B (not 16-B) aligned bucket, both targets."""
    P, L = 5, 70001
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    agg.set_coalesce(group)
    vals = [O.synth_bucket(L + 1, 6, k)[:L] for k in range(12)]
    keep = []

    def devbuf(k, be=False, shift=False):
        raw = O.be_encode(vals[k]) if be else np.asarray(vals[k]).tobytes()
        t = torch.zeros(len(raw) + 16, dtype=torch.uint8, device="cuda")
        off = 8 if shift else 0
        t[off:off + len(raw)] = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to("cuda")
        keep.append(t)
        torch.cuda.synchronize()          # the handle's stream does not order after torch's
        return ipls.DeviceBuffer(int(t.data_ptr()) + off, L, big_endian=be)

    ref = {(tg, p): None for tg in (ipls.TGT_AGG, ipls.TGT_REP) for p in range(P)}

    def fold(tg, p, k):
        acc = ref[(tg, p)]
        ref[(tg, p)] = O.reduce([vals[k]], L) if acc is None else O.reduce([vals[k]], L, O.START_ACCUM, acc=acc)

    pb = ipls.PinnedBuffer(8 * L)
    pb.view()[:] = np.frombuffer(O.be_encode(vals[11]), dtype=np.uint8)
    tickets = []
    rng = np.random.default_rng(group)
    for j in range(90):
        p = int(rng.integers(0, P)) if j % 3 else j % P
        tg = ipls.TGT_REP if j % 7 == 3 else ipls.TGT_AGG
        k = j % 11
        if j == 40:
            agg.Update(vals[k], p, from_clients=tg == ipls.TGT_AGG)     # synchronous host fold
        elif j == 55:
            tickets.append(agg.UpdateAsync(pb, p, from_clients=tg == ipls.TGT_AGG))   # pinned, zero copy
            k = 11
        elif j == 70:
            assert_bits_equal(agg.read(0), ref[(ipls.TGT_AGG, 0)], "mid-stream read")
            continue
        else:
            b = devbuf(k, be=(j // 9) % 2 == 1, shift=j % 13 == 5)
            tickets.append(agg.UpdateAsync(b, p, from_clients=tg == ipls.TGT_AGG))
        fold(tg, p, k)
    assert tickets == sorted(tickets) and len(set(tickets)) == len(tickets)
    agg.Wait(tickets[len(tickets) // 2])
    agg.Wait(tickets[-1])
    for (tg, p), r in ref.items():
        if r is not None:
            assert_bits_equal(agg.read(p, tg), r, f"target {tg} p{p}")
    with pytest.raises(ipls.IplsError):
        agg.UpdateAsync(ipls.DeviceBuffer(int(keep[0].data_ptr()) + 4, L), 0)   # not 8-B aligned
    with pytest.raises(ipls.IplsError):
        agg.UpdateAsync(ipls.DeviceBuffer(int(keep[0].data_ptr()), L - 1), 0)   # shorter than L_p
    agg.close()
    pb.close()


def test_concurrent_failures_keep_their_messages(ipls, O):
    """Two threads fail on one handle over and over with different errors (a
    bucket shorter than its partition, Updater.java:115; an out-of-range
    partition), a third folds correctly in between.  Each exception must carry
    its own call's message (the failing thread's, include/ipls_agg.h), never
    the other thread's, and the good folds must still be exact."""
    import threading
    P, L = 4, 4099
    with ipls.Aggregator(n_partitions=P, bucket_len=L, devices=[0, 0]) as agg:
        short = O.synth_bucket(L, 1, 0)[:L - 7]
        good = O.synth_bucket(L, 1, 1)
        wrong = []

        def short_bucket():
            for _ in range(300):
                try:
                    agg.Update(short, 1, from_clients=True)
                    wrong.append("short bucket accepted")
                except ipls.IplsError as e:
                    if "shorter than partition length" not in str(e):
                        wrong.append(f"short: {e}")

        def bad_partition():
            for _ in range(300):
                try:
                    agg.checksum(P + 3)
                    wrong.append("partition P+3 read")
                except ipls.IplsError as e:
                    if "out of range" not in str(e) or "shorter" in str(e):
                        wrong.append(f"range: {e}")

        def folds():
            for _ in range(50):
                agg.Update(good, 3, from_clients=True)

        th = [threading.Thread(target=f) for f in (short_bucket, bad_partition, folds)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not wrong, wrong[:5]
        assert_bits_equal(agg.read(3), O.reduce([good] * 50, L), "partition 3 after 50 folds")
        assert_bits_equal(agg.read(1), np.zeros(L), "partition 1 untouched by rejected buckets")


@pytest.mark.parametrize("devices", [None, [0, 0, 0]])
def test_concurrent_callers_one_handle(ipls, O, devices):
    """The reference's producer threads, Updater thread and daemon thread all
    reach the accumulators (serialised by PeerData.mtx, PeerData.java:27).
    Four Python threads (ctypes drops the GIL) share one handle, each owning
    its own partitions so the per-partition order is fixed: synchronous host
    and device folds, queued device folds, pubsub ingest, hash-only requests
    through the handle's one Gradient_Buff, and reads interleave.  Every
    partition must end bit-identical to the oracle's fold in that thread's
    order.  ``devices=[0, 0, 0]``: the same over a three-shard handle (the
    persistent shard workers, the Gradient_Buff sequence lock, handle-wide
    tickets)."""
    import threading
    P, L, T = 8, 30011, 4
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, devices=devices)
    agg.set_coalesce(3)
    vals = [O.synth_bucket(L, 7, k) for k in range(6)]
    dev = []
    for v in vals:
        t = torch.from_numpy(np.asarray(v)).to("cuda")
        dev.append((t, ipls.DeviceBuffer.from_tensor(t)))
    torch.cuda.synchronize()
    msgs = [O.pubsub_message(O.frame_encode(v, 0, 1, 3, b"QmT")) for v in vals]
    files = [O.be_encode(v) for v in vals]          # full-length `ipfs cat` files (hash-only requests)
    plans = {}
    errors = []

    def worker(w):
        rng = np.random.default_rng(100 + w)
        mine = [p for p in range(P) if p % T == w]
        seq = []
        try:
            for j in range(60):
                p = mine[j % len(mine)]
                k = int(rng.integers(0, len(vals)))
                how = int(rng.integers(0, 5))
                if how == 0:
                    agg.Update(vals[k], p)
                elif how == 1:
                    agg.Update(dev[k][1], p)
                elif how == 2:
                    t = agg.UpdateAsync(dev[k][1], p)
                    if j % 5 == 0:
                        agg.Wait(t)            # host waits run with the handle's lock released
                elif how == 3:
                    n, st = agg.ingest_pubsub([msgs[k]], partitions=[p])
                    assert n == 1 and st == [0]
                else:                          # through the handle's one Gradient_Buff (on shard 0)
                    agg.UpdateIndirect(files[k], p)
                seq.append((p, k))
                if j % 17 == 0:
                    agg.read(p)
                if j % 23 == 0:
                    agg.sync()
            plans[w] = seq
        except Exception as e:   # surfaced below
            errors.append(e)

    ths = [threading.Thread(target=worker, args=(w,)) for w in range(T)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors
    for w, seq in plans.items():
        for p in {p for p, _ in seq}:
            ks = [k for q, k in seq if q == p]
            assert_bits_equal(agg.read(p), O.reduce([vals[k] for k in ks], L), f"thread {w} p{p}")
    agg.close()


@pytest.mark.parametrize("devices", [None, [0, 0, 0]])
def test_concurrent_replica_store(ipls, O, devices):
    """Download_Scheduler threads store and drop other aggregators' downloads
    concurrently (Download_Scheduler.java:215-268, 329-332 under com_mtx).
    Four threads, each on its own partitions: the store never loses or
    mixes an array, the reported key order (the HashMap model) is ascending
    in bin under its capacity, and Collect_Replicas folds exactly that order,
    bit-exact."""
    import threading
    P, L, T = 8, 20011, 4
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, devices=devices)
    ids = [f"12D3KooWConc{a}" for a in range(6)]
    live = [dict() for _ in range(T)]          # per thread: (p, a) -> stored array
    errors = []

    def worker(w):
        rng = np.random.default_rng(700 + w)
        mine = [p for p in range(P) if p % T == w]
        try:
            for j in range(50):
                p, a = mine[j % len(mine)], int(rng.integers(0, len(ids)))
                if rng.integers(0, 4) == 0:
                    assert agg.OtherReplicaDrop(p, a) == ((p, a) in live[w])
                    live[w].pop((p, a), None)
                    continue
                g = O.synth_bucket(L, p, 100 * w + j) * float(10.0 ** rng.integers(-6, 7))
                agg.OtherReplicaGradients(p, a, g, key_hash=O.java_pair_hash(p, ids[a]))
                if (p, a) in live[w]:
                    live[w][(p, a)] = live[w][(p, a)] + g
                else:
                    live[w][(p, a)] = g.copy()
        except Exception as e:   # surfaced below
            errors.append(e)

    ths = [threading.Thread(target=worker, args=(w,)) for w in range(T)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors
    stored = {k: v for d in live for k, v in d.items()}
    order, cap = agg.replica_order()
    assert sorted(order) == sorted(stored)
    bins = [O.JavaHashMap.spread(O.java_pair_hash(p, ids[a])) & (cap - 1) for p, a in order]
    assert bins == sorted(bins)
    rep = [np.zeros(L) for _ in range(P)]
    for p, a in order:
        rep[p] = rep[p] + stored[(p, a)]
    n, _ = agg.Collect_Replicas()
    assert n == len(stored)
    for p in range(P):
        assert_bits_equal(agg.read(p, ipls.TGT_REP), rep[p], f"REP[{p}]")
    agg.close()


def test_partial_update_pair_files(ipls, O):
    """-i 1 partial updates: commit_partial_update's Pair<Integer,double[]>
    bytes (IPLS_Comm.java:51-61) from AGG on the device; a replica's Pair
    folded into REP (Download_Scheduler.java:324); the storage merge of Pair
    and raw BE files (Decentralized_Storage_Receiver.java:239-258)."""
    from oracle import javaser as J
    M, P = 40003, 2
    agg = ipls.Aggregator(M, P, max_peers=4)
    Ls = agg.lengths
    own = [O.synth_bucket(Ls[0], 0, k) for k in range(3)]
    for b in own:
        agg.Update(b, 0)
    S = O.reduce(own, Ls[0])
    file0 = agg.commit_partial_update(0, workers=3)
    assert file0 == J.encode_pair(3, S)
    assert agg.commit_partial_update(1, workers=1) == J.encode_pair(1, np.zeros(Ls[1]))   # empty AGG
    # a replica's partial update arrives as a Pair file -> REP
    rep = O.synth_bucket(Ls[0], 0, 40)
    agg.Update(J.encode_pair(2, rep), 0, from_clients=False, pair=True)
    assert_bits_equal(agg.read(0, ipls.TGT_REP), O.reduce([rep], Ls[0]), "REP from Pair")
    with pytest.raises(ipls.IplsError):
        agg.Update(J.encode_pair(2, rep[:-1]), 0, from_clients=False, pair=True)        # shorter than L_p
    with pytest.raises(ipls.IplsError):
        agg.Update(file0[:-3], 0, pair=True)                                             # truncated stream
    # storage merge: first file as is (-0.0 kept), later files folded, prefix rule
    g = [O.synth_bucket(5000, 1, k) for k in range(4)]
    g[0][::5] = -0.0
    g[2] = g[2][:4000]
    ref = O.storage_merge(g)
    assert agg.merge_files([O.be_encode(x) for x in g]) == O.be_encode(ref)
    assert agg.merge_files([J.encode_pair(k, x) for k, x in enumerate(g)], partial_updates=True) == O.be_encode(ref)
    with pytest.raises(ipls.IplsError):
        agg.merge_files([O.be_encode(g[2]), O.be_encode(g[1])])                          # later file longer
    agg.close()


def test_full_ipls_round_four_peers(ipls, O):
    """One synchronous IPLS round across 4 simulated peers on one GPU, every
    transport of the path in play, checked end to end against the oracle:
      * partition p is aggregated by A = p and by the replica B = p+1 (mod 4);
      * each aggregator folds its own gradient (UpdateGradient, IPLS.java:1737),
        A receives the others as pubsub texts (ThreadReceiver, double base64),
        B as `ipfs cat` files through Gradient_Buff (Updater.run indirect);
      * partials cross as -i 1 Pair<Integer,double[]> files (commit_partial_update
        -> Download_Partial_Updates -> REP), except that the replica of
        partition 3 stays silent and its aggregator folds the bucket it had
        downloaded for it instead (Other_Replica_Gradients + Collect_Replicas);
      * A commits W (AggregatePartition -> update_file bytes), every peer
        caches every partition it does not aggregate (cache_partition) and
        GetPartitions gives the model, identical on all peers."""
    from oracle import javaser as J
    M, P, NP = 100003, 4, 4
    grads = [O.synth_bucket(M, 9, k) for k in range(NP)]           # flat List<Double> per peer
    parts = [O.organize_gradients(g, M, P) for g in grads]
    Ls = [O.partition_len(M, P, p) for p in range(P)]
    A = lambda p: p                                                 # noqa: E731
    B = lambda p: (p + 1) % NP                                      # noqa: E731
    peers = [ipls.Aggregator(M, P, max_peers=NP) for _ in range(NP)]
    auth = [[k, (k - 1) % P] for k in range(NP)]                   # own partition + the one it replicates
    # ---- device: gradients to the aggregators ----
    for k, agg in enumerate(peers):
        agg.UpdateGradient(grads[k], auth_list=auth[k])
    for p in range(P):
        msgs = [O.pubsub_message(O.frame_encode(parts[k][p], p, 0, 3, f"QmPeer{k}".encode()))
                for k in range(NP) if k != A(p)]
        n_ok, st = peers[A(p)].ingest_pubsub(msgs, partitions=[p] * len(msgs))
        assert n_ok == len(msgs) and st == [0] * len(msgs)
        for k in range(NP):
            if k != B(p):
                peers[B(p)].UpdateIndirect(O.be_encode(parts[k][p]), p)
    # ---- partial exchange ----
    for p in range(P):
        if p != 3:                                                  # replica answers with its partial
            f = peers[B(p)].commit_partial_update(p, workers=NP)
            peers[A(p)].Update(f, p, from_clients=False, pair=True)
        else:                                                       # silent replica: use what A downloaded for it
            peers[A(p)].OtherReplicaGradients(p, B(p), parts[B(p)][p])
    for k in range(NP):
        peers[k].Collect_Replicas()
    # ---- commit and distribute ----
    files = {}
    for p in range(P):
        s, _ = peers[A(p)].AggregatePartition(p, with_sum=True, sum_big_endian=True)
        files[p] = bytes(s)
    for k, agg in enumerate(peers):
        for p in range(P):
            if A(p) != k:
                agg.cache_partition(p, files[p])
    models = [agg.GetPartitions() for agg in peers]
    # ---- oracle ----
    W = []
    for p in range(P):
        own_a = [parts[A(p)][p]] + [parts[k][p] for k in range(NP) if k != A(p)]
        agg_a = O.reduce(own_a, Ls[p])
        if p != 3:
            own_b = [parts[B(p)][p]] + [parts[k][p] for k in range(NP) if k != B(p)]
            partial = J.parse_pair(J.encode_pair(NP, O.reduce(own_b, Ls[p])))[1]
            rep = O.reduce([partial], Ls[p])
        else:
            rep = O.reduce([parts[B(p)][p]], Ls[p])
        W.append(agg_a + rep)
        assert files[p] == O.be_encode(W[p]), f"update_file of partition {p}"
    ref = O.get_partitions(W)
    for k in range(NP):
        assert_bits_equal(models[k], ref, f"model on peer {k}")
    for agg in peers:
        agg.close()


@pytest.mark.parametrize("seed,group,devices", [(1, 1, None), (2, 4, None), (3, 32, None), (4, 2, None), (5, 8, None),
                                                (6, 4, [0, 0]), (7, 32, [0, 0, 0])])
def test_stateful_random_sequence(ipls, O, seed, group, devices, P=4, L=5003, steps=300, shapes=None, prefix=()):
    """A random sequence over the whole accumulator surface, checked step by
    step against a numpy model of the Java state (Aggregated_Gradients,
    Replicas_Gradients, Aggregated_Gradients_from_future, Weights): host and
    device folds, queued folds (coalescing group 1/4/32), batched folds with
    every start mode and byte order, AggregatePartition, resets, promotion of
    future gradients, the async blend, cache_partition, the fused round,
    GetPartitions, the ranged folds and reads from pinned memory
    (ipls_agg_accumulate_range / ipls_agg_read_range at random even cuts), and
    the chunked calls (accumulate_chunked with a source that sometimes stops,
    finalize_chunked, get_partitions_wire_chunked at random even chunk
    sizes).  Buckets include -0.0, subnormals and huge values so the
    start-value and grouping rules show in the bits.  ``devices``: the same
    sequence through a multi-device handle (shards [0,2) | [2,4), and a
    three-entry list whose last shard owns no partition), so the front's
    routing of every call is checked against the same model.  ``shapes``: a
    set that collects the (kernel, shape, map, big-endian, start) of every
    batched launch, for callers that must show which production shapes a
    sequence reached.  ``prefix``: scripted steps run before the random ones,
    each a dict fixing some of a step's draws (op, p, n, kk, mode, be, tg);
    the draws it does not fix come from the rng as usual."""
    rng = np.random.default_rng(seed)
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, devices=devices)
    agg.set_coalesce(group)
    pool = []
    for k in range(10):
        g = O.synth_bucket(L, 9, k) * (10.0 ** rng.integers(-3, 4))
        g[rng.integers(0, L, 40)] = -0.0
        g[rng.integers(0, L, 10)] = 5e-324
        g[rng.integers(0, L, 5)] = rng.choice([1e300, -1e300, 1e16])
        g[-1] = 1.0
        pool.append(g)
    dev = [torch.from_numpy(g).to("cuda") for g in pool]
    dev_be = [torch.from_numpy(np.frombuffer(O.be_encode(g), dtype=np.uint8).copy()).to("cuda") for g in pool]
    torch.cuda.synchronize()
    D = [ipls.DeviceBuffer.from_tensor(t) for t in dev]
    DB = [ipls.DeviceBuffer(int(t.data_ptr()), L, big_endian=True) for t in dev_be]
    T = {ipls.TGT_AGG: "agg", ipls.TGT_REP: "rep", ipls.TGT_FUTURE: "fut", ipls.TGT_WEIGHTS: "w"}
    M = {name: [np.zeros(L) for _ in range(P)] for name in T.values()}

    def check(p, tg, what):
        assert_bits_equal(agg.read(p, tg), M[T[tg]][p], f"step {what}: p{p} {T[tg]}")

    gbuf = np.zeros(L)          # the Updater's one Gradient_Buff (synthetic geometry: L doubles)
    store = O.ReplicaStore()    # Other_Replica_Gradients
    # aggregator peer IDs: odd seeds pass the Pair hash of a real-looking ID
    # (ipls_agg_other_replica_keyed), even seeds the index-as-ID default
    peer_ids = [f"12D3KooW{seed}x{i}{'Q' * (i % 3)}" for i in range(5)]
    # seeds 2 mod 3: keyed hashes that share their low 6 bits (one HashMap bin
    # up to 64 bins), more store traffic and rare collects, so the store's
    # map resizes through treeifyBin and grows red-black tree bins
    collide = seed % 3 == 2
    msgs = [O.pubsub_message(O.frame_encode(g, 0, 1, 3, b"QmS")) for g in pool]
    from ipls import _native as N
    lib, h = agg._lib, agg._h
    pin = ipls.PinnedBuffer(8 * L + 64)          # the JNI shim's pinned ring, one slot of a whole bucket
    tk = ctypes.c_uint64()

    def cuts():                                  # even cut points: the ranges a chunked copy folds / reads
        return sorted({0, L, *(2 * int(x) for x in rng.integers(0, L // 2 + 1, int(rng.integers(0, 4))))})
    script = list(prefix)
    for step in range(len(script) + steps):
        fixed = script[step] if step < len(script) else {}

        def draw(key, fn):
            return fixed[key] if key in fixed else fn()
        op = draw("op", lambda: int(rng.integers(0, 22)))
        if collide and op in (8, 16) and "op" not in fixed:
            op = 14
        if op == 21 and L > (1 << 20) and "op" not in fixed and rng.integers(0, 3):
            op = 11                                         # the whole-model check costs ~1 s at production lengths
        p = draw("p", lambda: int(rng.integers(0, P)))
        k = int(rng.integers(0, len(pool)))
        g = pool[k]
        if op == 0:                                         # Updater._Update from host bytes/doubles
            tg = [ipls.TGT_AGG, ipls.TGT_REP][int(rng.integers(0, 2))]
            if rng.integers(0, 2):
                agg.Update(g, p, from_clients=tg == ipls.TGT_AGG)
            else:
                agg.Update(O.be_encode(g), p, from_clients=tg == ipls.TGT_AGG)
            M[T[tg]][p] = M[T[tg]][p] + g
        elif op == 1:                                       # from the future
            agg.Update(g, p, from_future=True)
            M["fut"][p] = M["fut"][p] + g
        elif op in (2, 3):                                  # queued device folds
            tg = [ipls.TGT_AGG, ipls.TGT_REP][op - 2]
            agg.UpdateAsync(DB[k] if rng.integers(0, 3) == 0 else D[k], p, from_clients=tg == ipls.TGT_AGG)
            M[T[tg]][p] = M[T[tg]][p] + g
        elif op == 4:                                       # batched folds, any start mode
            n = draw("n", lambda: int(rng.integers(1, P - p + 1)))
            kk = draw("kk", lambda: int(rng.integers(1, 4)))
            ks = [[int(x) for x in rng.integers(0, len(pool), kk)] for _ in range(n)]
            mode = draw("mode", lambda: [ipls.START_ZERO, ipls.START_ACCUM, ipls.START_FIRST][int(rng.integers(0, 3))])
            be = draw("be", lambda: bool(rng.integers(0, 2)))
            tg = draw("tg", lambda: [ipls.TGT_AGG, ipls.TGT_REP][int(rng.integers(0, 2))])
            agg.reduce_batch(p, [[(DB if be else D)[j] for j in row] for row in ks], start_mode=mode, target=tg,
                             big_endian=be)
            if shapes is not None:
                li = agg.last_launch()
                shapes.add((li["kernel"], li["shape"], li["map"], be, mode))
            for q, row in enumerate(ks):
                bufs = [pool[j] for j in row]
                M[T[tg]][p + q] = O.reduce(bufs, L, mode, acc=M[T[tg]][p + q])
        elif op == 5:                                       # AggregatePartition
            agg.AggregatePartition(p)
            M["w"][p] = M["agg"][p] + M["rep"][p]
            M["agg"][p] = np.zeros(L)
            M["rep"][p] = np.zeros(L)
        elif op == 6:                                       # reset one / all
            if rng.integers(0, 3) == 0:
                agg.reset()
                qs = range(P)
            else:
                agg.reset(p)
                qs = [p]
            for q in qs:
                M["agg"][q] = np.zeros(L)
                M["rep"][q] = np.zeros(L)
        elif op == 7:                                       # Update_Client_WaitAck_List
            qs = sorted({int(x) for x in rng.integers(0, P, 2)})
            agg.PromoteFuture(qs)
            for q in qs:
                M["agg"][q] = M["fut"][q]
                M["fut"][q] = np.zeros(L)
        elif op == 8:                                       # -async replica fold W = 0.75 W + g
            agg.UpdateAsyncReplica(g, p)
            M["w"][p] = O.blend(M["w"][p], g, 0.75, 1.0)
        elif op == 9:                                       # cache_partition: GetParameters into W
            n = int(rng.integers(1, L + 1))
            agg.cache_partition(p, O.be_encode(g[:n]))
            M["w"][p][:n] = g[:n]
        elif op == 10:                                      # fused round over a range
            n = draw("n", lambda: int(rng.integers(1, P - p + 1)))
            kk = draw("kk", lambda: int(rng.integers(0, 3)))
            ks = [[int(x) for x in rng.integers(0, len(pool), kk)] for _ in range(n)]
            avg = agg.aggregate_round(p, [[D[j] for j in row] for row in ks])
            if shapes is not None and kk:
                li = agg.last_launch()
                shapes.add((li["kernel"], li["shape"], li["map"], False, -1))
            exp = []
            for q, row in enumerate(ks):
                a = O.reduce([pool[j] for j in row], L, ipls.START_ACCUM, acc=M["agg"][p + q]) if row \
                    else M["agg"][p + q]
                M["w"][p + q] = a + M["rep"][p + q]
                M["agg"][p + q] = np.zeros(L)
                M["rep"][p + q] = np.zeros(L)
                exp.append(O.divide(M["w"][p + q]))
            assert_bits_equal(avg, np.concatenate(exp), f"step {step}: fused round")
        elif op == 12:                                      # ThreadReceiver: pubsub text -> frame -> fold
            n, st = agg.ingest_pubsub([msgs[k]], partitions=[p])
            assert n == 1 and st == [0]
            M["agg"][p] = M["agg"][p] + g
        elif op == 13:                                      # Updater.run, hash-only: GetParameters(hash, Gradient_Buff)
            n = int(rng.integers(1, L + 1))
            agg.UpdateIndirect(O.be_encode(g[:n]), p)
            gbuf[:n] = g[:n]
            M["agg"][p] = M["agg"][p] + gbuf
        elif op == 14:                                      # Download_Scheduler: another aggregator's bucket
            a = int(rng.integers(0, 12 if collide else 5))
            if rng.integers(0, 4) == 0:                     # its partial arrived: Other_Replica_Gradients.remove
                assert agg.OtherReplicaDrop(p, a) == O.other_replica_drop(store, p, a)
            else:
                if collide:
                    kh = 0x1A + 64 * (p * 12 + a)
                else:
                    kh = O.java_pair_hash(p, peer_ids[a]) if seed % 2 else None
                agg.OtherReplicaGradients(p, a, g, key_hash=kh)
                O.other_replica_add(store, p, a, g, key_hash=kh)
            if collide:                                     # the library's model vs the JDK simulation
                assert agg.replica_order()[0] == store.map.keys(), f"step {step}: replica order"
                if shapes is not None and store.map.tree_bin:
                    shapes.add(("replica store", "tree bin", "", False, -1))
        elif op == 17:                                      # a heap double[] through the ring: ranged folds
            tg = [ipls.TGT_AGG, ipls.TGT_REP, ipls.TGT_FUTURE][int(rng.integers(0, 3))]
            be = bool(rng.integers(0, 2))
            raw = np.frombuffer(O.be_encode(g) if be else g.tobytes(), dtype=np.uint8)
            pin.view()[:raw.size] = raw
            for a, b in _pairs(cuts()):
                assert lib.ipls_agg_accumulate_range(h, p, tg, pin.ptr + 8 * a, a, b - a,
                                                     N.HOST_BE if be else N.HOST_F64, ctypes.byref(tk)) == 0
            assert lib.ipls_agg_wait(h, tk.value) == 0
            M[T[tg]][p] = M[T[tg]][p] + g
        elif op == 18:                                      # a byte[] / double[] output through the ring
            tg = list(T)[int(rng.integers(0, len(T)))]
            be = bool(rng.integers(0, 2))
            for a, b in _pairs(cuts()):
                assert lib.ipls_agg_read_range(h, p, tg, pin.ptr + 8 * a, a, b - a,
                                               N.HOST_BE if be else N.HOST_F64, ctypes.byref(tk)) == 0
            assert lib.ipls_agg_wait(h, tk.value) == 0
            want = O.be_encode(M[T[tg]][p]) if be else M[T[tg]][p].tobytes()
            assert pin.view()[:8 * L].tobytes() == want, f"step {step}: read_range p{p} {T[tg]} be={be}"
        elif op == 19:                                      # one arrival pulled chunk by chunk, as one call
            tg = [ipls.TGT_AGG, ipls.TGT_REP, ipls.TGT_FUTURE][int(rng.integers(0, 3))]
            be = bool(rng.integers(0, 2))
            raw = np.frombuffer(O.be_encode(g) if be else g.tobytes(), dtype=np.uint8)
            ch = 2 * int(rng.integers(max(1, L // 4096), L // 2 + 2))
            stop_at = int(rng.integers(0, 4)) if rng.integers(0, 5) == 0 else -1   # a failing source folds nothing
            calls = []

            @N.CHUNK_SOURCE
            def src(ctx, dst, off, n, raw=raw, calls=calls, stop_at=stop_at):
                calls.append(off)
                if len(calls) - 1 == stop_at:
                    return 1
                ctypes.memmove(dst, raw.ctypes.data + 8 * off, 8 * n)
                return 0
            rc = lib.ipls_agg_accumulate_chunked(h, p, tg, L, N.HOST_BE if be else N.HOST_F64, ch, src, None)
            if 0 <= stop_at < -(-L // min(ch, L)):
                assert rc == N.IPLS_E_INVAL, f"step {step}: stopped source"
            else:
                assert rc == 0, f"step {step}: accumulate_chunked"
                M[T[tg]][p] = M[T[tg]][p] + g
        elif op == 20:                                      # AggregatePartition, its bytes handed over in chunks
            be = bool(rng.integers(0, 2))
            ch = 2 * int(rng.integers(max(1, L // 4096), L // 2 + 2))
            out = bytearray(8 * L)

            @N.CHUNK_SINK
            def sink(ctx, vals, off, n, out=out):
                out[8 * off:8 * (off + n)] = ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n)
                return 0
            assert lib.ipls_agg_finalize_chunked(h, p, N.HOST_BE if be else N.HOST_F64, ch, sink, None) == 0
            M["w"][p] = M["agg"][p] + M["rep"][p]
            M["agg"][p] = np.zeros(L)
            M["rep"][p] = np.zeros(L)
            want = O.be_encode(M["w"][p]) if be else M["w"][p].tobytes()
            assert bytes(out) == want, f"step {step}: finalize_chunked p{p}"
        elif op == 21:                                      # Middleware task 3, chunk by chunk
            ch = 2 * int(rng.integers(max(1, P * L // 4096), P * L // 2 + 2))
            got = bytearray()

            @N.CHUNK_SINK
            def wsink(ctx, vals, off, n, got=got):
                got.extend(ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n))
                return 0
            assert lib.ipls_agg_get_partitions_wire_chunked(h, ch, wsink, None) == 0
            assert bytes(got) == O.be_encode_canonical(O.get_partitions(M["w"])), f"step {step}: wire chunked"
        elif op == 15 and collide and rng.integers(0, 6):  # (collide: most collects skipped)
            pass
        elif op == 15:                                      # Collect_Replicas
            n, part = agg.Collect_Replicas()
            exp_part = [0] * P
            assert n == O.collect_replicas(M["rep"], store, exp_part)
            assert part == exp_part
        else:                                               # -async publish / leaving peer
            if rng.integers(0, 2):
                agg.AsyncPublishScale(p)
                M["agg"][p] = O.scale(M["w"][p], 0.25)
            else:
                agg.UpdateLeavingPeer(g, p)
                M["w"][p] = O.blend(M["w"][p], g, 0.6, 1 - 0.6)
        if op == 11 or step % 25 == 24:                     # reads
            for tg in T:
                check(p, tg, step)
        if step % 40 == 39:
            assert_bits_equal(agg.GetPartitions(), O.get_partitions(M["w"]), f"step {step}: GetPartitions")
    for p in range(P):
        for tg in T:
            check(p, tg, "end")
    agg.close()
    pin.close()


def _pairs(c):
    return list(zip(c[:-1], c[1:]))


def production_prefix(ipls, P):
    """Scripted steps that reach every production launch shape whatever the
    seed: a batched fold over all P partitions (the big 1024-lane tiles when
    P = 4) and over one partition (the 256-lane mid shape), for each byte order
    and each start mode, then the fused round over all P and over one.  Each
    fused round and AggregatePartition in between keeps the state moving."""
    steps = []
    for be in (False, True):
        for mode in (ipls.START_ZERO, ipls.START_FIRST, ipls.START_ACCUM):
            for p, n in ((0, P), (P - 1, 1)):
                steps.append({"op": 4, "p": p, "n": n, "kk": 2, "mode": mode, "be": be, "tg": ipls.TGT_AGG})
            steps.append({"op": 5, "p": 0})
    steps.append({"op": 10, "p": 0, "n": P, "kk": 2})
    steps.append({"op": 10, "p": P - 1, "n": 1, "kk": 2})
    return steps


@pytest.mark.parametrize("seed,P,L", [(21, 4, 8 * 1048576 + 5), (22, 4, 8 * 1048576 + 5), (23, 4, 8 * 1048576 + 5),
                                      (22, 1, 4 * 1048576 + 3)])
def test_stateful_random_sequence_production_shapes(ipls, O, seed, P, L):
    """The random sequence at production bucket lengths (ragged, so every
    batch ends in a partial tile), so that its batched folds and fused rounds
    run the production launch shapes interleaved with every other call on the
    same state: the big 1024-lane tiles (4 partitions of 8M: 1024 big tiles;
    big-endian input on the R = 16 SEQ schedule, ACCUM at R = 8) and the
    512-lane half shape (one partition), every start mode.  A scripted prefix (production_prefix) reaches every (shape, byte
    order, start mode) and the fused round's shapes first, so the coverage
    does not depend on the seed (seed 21 alone never reached the
    big shape); the random steps follow.  With one partition of 4M only the
    half shape exists."""
    shapes = set()
    test_stateful_random_sequence(ipls, O, seed, 32, None, P=P, L=L, steps=300, shapes=shapes,
                                  prefix=production_prefix(ipls, P))
    reduce_shapes = {(s, be, mode) for k, s, _, be, mode in shapes if k == ipls.KERNEL_REDUCE}
    want = []
    for mode in (ipls.START_ZERO, ipls.START_FIRST):
        want.append((ipls.SHAPE_HALF, False, mode))            # one partition
        want.append((ipls.SHAPE_HALF, True, mode))
    if P == 4:
        for mode in (ipls.START_ZERO, ipls.START_FIRST, ipls.START_ACCUM):
            want.append((ipls.SHAPE_BIG, True, mode))          # 4 partitions of 8M
            want.append((ipls.SHAPE_BIG, False, mode))
    for be in (False, True):
        want.append((ipls.SHAPE_HALF, be, ipls.START_ACCUM))   # one partition, ACCUM at R = 16
    for w in want:
        assert w in reduce_shapes, (w, sorted(reduce_shapes))
    round_shapes = {s for k, s, _, _, _ in shapes if k == ipls.KERNEL_ROUND}
    for shape in ((ipls.SHAPE_BIG, ipls.SHAPE_HALF) if P == 4 else (ipls.SHAPE_HALF,)):
        assert shape in round_shapes, (shape, sorted(round_shapes))


def test_update_async_many_is_the_per_arrival_calls(ipls, O):
    """Aggregator.UpdateAsyncMany (ipls._fast.accumulate_async_many: one
    Python -> C transition for a list of arrivals) folds
    exactly what one UpdateAsync per arrival folds, in the same order: queued
    device buckets (native and big-endian) and pinned host buckets over three
    partitions and both targets, through _fast and through ctypes, equal to
    the oracle.  A bad arrival in the middle raises; the ones before it are
    queued, as after the same UpdateAsync calls."""
    from ipls import _native as N
    P, L = 3, 40003
    vals = [O.synth_bucket(L, 11, k) for k in range(5)]
    dv = [dev(v) for v in vals[:3]]
    bt, bb = dev_be(vals[3])
    pb = ipls.PinnedBuffer(8 * L)
    pb.view()[:] = np.frombuffer(O.be_encode(vals[4]), dtype=np.uint8)
    torch.cuda.synchronize()
    arrivals = [(dv[k][1], p) for k in range(3) for p in range(P)] + [(bb, 1), (pb, 2)]
    for library in (None, N.load(N.LIB_PATH)):
        agg = ipls.Aggregator(n_partitions=P, bucket_len=L, library=library)
        agg.set_coalesce(4)
        assert (agg._fast is not None) == (library is None)
        t = agg.UpdateAsyncMany(arrivals)
        t2 = agg.UpdateAsyncMany([(dv[2][1], 0)], from_clients=False)
        assert t2 > t > 0 and agg.UpdateAsyncMany([]) == 0
        agg.Wait(t2)
        ref = [O.reduce(vals[:3], L), O.reduce(vals[:4], L), O.reduce(vals[:3] + [vals[4]], L)]
        for p in range(P):
            assert_bits_equal(agg.read(p, ipls.TGT_AGG), ref[p], f"p{p} fast={agg._fast is not None}")
        assert_bits_equal(agg.read(0, ipls.TGT_REP), O.reduce([vals[2]], L))
        agg.reset()
        with pytest.raises(ipls.IplsError):
            agg.UpdateAsyncMany([(dv[0][1], 0), (dv[1][1], P), (dv[2][1], 1)])   # partition P out of range
        agg.sync()
        assert_bits_equal(agg.read(0, ipls.TGT_AGG), O.reduce([vals[0]], L), "the arrival before the bad one")
        assert_bits_equal(agg.read(1, ipls.TGT_AGG), np.zeros(L), "nothing after it")
        agg.close()
    pb.close()


def test_fast_extension_and_ctypes_give_the_same_bits(ipls, O):
    """A default Aggregator takes the per-arrival calls through ipls._fast
    (csrc/pyfast.c); one bound to another ctypes mapping of the same library
    (library=...) takes ctypes.  The same arrivals -- queued device buckets
    (native and big-endian), pinned host buckets, synchronous host and device
    Updates, both targets -- give the same bits through either, equal to the
    oracle; errors come back the same way."""
    from ipls import _native as N
    P, L = 3, 40003
    vals = [O.synth_bucket(L, 9, k) for k in range(6)]
    dv = [dev(v) for v in vals[:3]]
    bt, bb = dev_be(vals[3])
    pb = ipls.PinnedBuffer(8 * L)
    pb.view()[:] = np.frombuffer(O.be_encode(vals[4]), dtype=np.uint8)
    torch.cuda.synchronize()
    fast = ipls.Aggregator(n_partitions=P, bucket_len=L)
    slow = ipls.Aggregator(n_partitions=P, bucket_len=L, library=N.load(N.LIB_PATH))
    assert fast._fast is not None and fast._fast is N.fast() and slow._fast is None
    for agg in (fast, slow):
        agg.set_coalesce(4)
        t = [agg.UpdateAsync(dv[k][1], p) for p in range(P) for k in range(3)]
        t.append(agg.UpdateAsync(bb, 1))
        t.append(agg.UpdateAsync(pb, 2))
        t.append(agg.UpdateAsync(dv[0][1], 0, from_clients=False))
        assert t == sorted(t) and len(set(t)) == len(t)
        agg.Wait(t[-1])
        agg.Update(vals[5], 0)                                      # host doubles
        agg.Update(np.frombuffer(O.be_encode(vals[5]), dtype=np.uint8), 2)  # host BE bytes
        agg.Update(dv[1][1], 1, from_clients=False)                 # device, REP
        with pytest.raises(ipls.IplsError):
            agg.Update(vals[5], P)                                  # partition out of range
        with pytest.raises(ipls.IplsError):
            agg.UpdateAsync(dv[0][1], -1)
        agg.sync()
    ref_agg = [O.reduce([vals[0], vals[1], vals[2]] + extra, L) for extra in ([vals[5]], [vals[3]], [vals[4], vals[5]])]
    ref_rep = [vals[0], vals[1], None]
    for p in range(P):
        a, b = fast.read(p, ipls.TGT_AGG), slow.read(p, ipls.TGT_AGG)
        assert_bits_equal(a, b)
        assert_bits_equal(a, ref_agg[p])
        if ref_rep[p] is not None:
            assert_bits_equal(fast.read(p, ipls.TGT_REP), slow.read(p, ipls.TGT_REP))
            assert_bits_equal(fast.read(p, ipls.TGT_REP), O.reduce([ref_rep[p]], L))
    fast.close()
    slow.close()
    pb.close()
    with pytest.raises(ipls.IplsError):
        fast.Update(vals[0], 0)                                     # closed handle: null, not a crash
