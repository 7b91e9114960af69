"""GPU parity of the launch shapes the production sizes take.

The fold kernel's dispatch picks a tile shape by how many tiles a batch fills
(engine.hip launch_reduce_v: big = 1024 lanes x 16 vectors, half = 512 lanes
x 16 vectors (fewer than 1024 whole big tiles, ZERO/FIRST start), mid = 256
lanes x 16 vectors (8 for big-endian input), small = 256 lanes x 8 peers in
flight).
Big-endian input at R = 16 runs the hand-fenced SEQ schedule (SEQF = 3),
START_ACCUM runs R = 8,
partial last tiles run map 3.  Every case below asserts through
ipls_agg_last_launch that it reached the shape it was written for, then
compares with the oracle: bit for bit on whole partitions (C oracle,
oracle/ipls_oracle.c) and by per-partition checksums of the counter
workload (tests/golden/golden.json "full", config D = 64 x 4M x 32 in full).
References: MyIPFSClass.java:444-455 (GetParameters BE decode),
:105-116 (update_file BE encode), Decentralized_Storage_Receiver.java:239-257
(FIRST-start merge), Updater.java:115-117 (the fold), IPLS.java:1248-1274 and
1159-1174 (the fused round).
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


class Pool:
    """P x K synthetic device buckets of L doubles (BE bytes when `be`), with
    a 256-B pad between buckets as the bench lays them out, plus one output
    buffer per partition."""

    def __init__(self, ipls, P, L, K, be, seed, p0=0, out=True):
        elem = (L + 32 + 31) // 32 * 32
        self.arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
        base = (int(self.arena.data_ptr()) + 255) // 256 * 256
        self.rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L, big_endian=be) for k in range(K)]
                     for q in range(P)]
        for q in range(P):
            for k in range(K):
                ipls.synth_fill(self.rows[q][k], p0 + q, k, seed)
        self.outs = None
        if out:
            self.out_arena = torch.empty(P * elem + 32, dtype=torch.float64, device="cuda")
            ob = (int(self.out_arena.data_ptr()) + 255) // 256 * 256
            self.outs = [ob + 8 * q * elem for q in range(P)]
        torch.cuda.synchronize()

    def out_host(self, q, L, be):
        off = self.outs[q] - int(self.out_arena.data_ptr())
        a = self.out_arena.view(torch.uint8)[off:off + 8 * L].cpu().numpy()
        return np.frombuffer(a.tobytes(), dtype=">f8" if be else "<f8").astype(np.float64)

    def free(self):
        del self.arena
        self.rows = None
        if self.outs is not None:
            del self.out_arena
        torch.cuda.empty_cache()


def ref_sum(O, L, p, K, start=None, acc=None):
    bufs = [O.c_synth_bucket(L, p, k) for k in range(K)]
    if start is None:
        start = O.START_ZERO
    return O.c_reduce(bufs, L, start, acc)


def expect(li, ipls, kernel, shape, vectors, seqf, be_in, be_out, mapping=None):
    got = (li["kernel"], li["shape"], li["vectors"], li["seqf"], li["be_in"], li["be_out"])
    assert got == (kernel, shape, vectors, seqf, int(be_in), int(be_out)), li
    if mapping is not None:
        assert li["map"] == mapping, li


def test_config_d_full_size_be_in_out(ipls, O, golden_meta):
    """Config D exactly: 64 partitions x 4,194,304 BE doubles x 32 peers, BE
    sum bytes out -- the shipped big shape with the SEQF = 3 schedule
    (8192 tiles, no partial tile: partition-major order), ZERO and FIRST start; then BE in with
    native doubles out into the accumulators, and ACCUM (R = 8) on top."""
    m = golden_meta["full"]["D"]
    P, L, K = m["partitions"], m["bucket_len"], m["peers"]
    pool = Pool(ipls, P, L, K, True, golden_meta["seed"])
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    want = m["sum_checksum"]
    for start in (ipls.START_ZERO, ipls.START_FIRST):
        agg.reduce_batch_out(0, pool.rows, pool.outs, start_mode=start, big_endian_in=True, big_endian_out=True)
        li = agg.last_launch()
        expect(li, ipls, ipls.KERNEL_REDUCE, ipls.SHAPE_BIG, 16, 3, True, True, mapping=0)
        assert li["block"] == 1024 and li["grid"] == P * L // (1024 * 2 * 16)
        agg.sync()
        got = [ipls.checksum_dev(ipls.DeviceBuffer(o, L, big_endian=True)) for o in pool.outs]
        assert got == want, f"start {start}: partitions {[q for q in range(P) if got[q] != want[q]]} differ"
    # whole partitions bit for bit (first and last of the batch)
    for q in (0, P - 1):
        assert_bits_equal(pool.out_host(q, L, True), ref_sum(O, L, q, K), f"D partition {q}")
    # BE in, native doubles into AGG (GetParameters decode fused, Updater fold)
    agg.reduce_batch(0, pool.rows, start_mode=ipls.START_ZERO, big_endian=True)
    expect(agg.last_launch(), ipls, ipls.KERNEL_REDUCE, ipls.SHAPE_BIG, 16, 3, True, False)
    assert [agg.checksum(q) for q in range(P)] == want
    # ACCUM: S + fold again, BE out (R = 8, compiler schedule)
    agg.reduce_batch_out(0, pool.rows, pool.outs, start_mode=ipls.START_ACCUM, big_endian_in=True,
                         big_endian_out=True)
    expect(agg.last_launch(), ipls, ipls.KERNEL_REDUCE, ipls.SHAPE_BIG, 8, 0, True, True)
    agg.sync()
    for q in (0, 37):
        s = ref_sum(O, L, q, K)
        assert_bits_equal(pool.out_host(q, L, True), ref_sum(O, L, q, K, O.START_ACCUM, s), f"D accum {q}")
    agg.close()
    pool.free()


def test_be_big_shape_xcd_order(ipls, O):
    """Big-endian input on a grid of at most 4096 whole tiles runs the big
    shape XCD-chunked (map 2): 8 x 4M x 8 = 1024 tiles (fewer would take the
    half shape), the fold with BE bytes out and the fused round, against the
    oracle."""
    P, L, K = 8, 4_194_304, 8
    pool = Pool(ipls, P, L, K, True, O.SEED)
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    refs = [ref_sum(O, L, q, K) for q in range(P)]
    agg.reduce_batch_out(0, pool.rows, pool.outs, start_mode=ipls.START_ZERO, big_endian_in=True,
                         big_endian_out=True)
    li = agg.last_launch()
    expect(li, ipls, ipls.KERNEL_REDUCE, ipls.SHAPE_BIG, 16, 3, True, True, mapping=2)
    assert li["grid"] == P * L // (1024 * 2 * 16), li
    agg.sync()
    for q in range(P):
        assert_bits_equal(pool.out_host(q, L, True), refs[q], f"map 2 partition {q}")
    out = agg.aggregate_round(0, pool.rows, big_endian=True)
    expect(agg.last_launch(), ipls, ipls.KERNEL_ROUND, ipls.SHAPE_BIG, 16, 3, True, False, mapping=2)
    for q in range(P):
        assert_bits_equal(agg.read(q, ipls.TGT_WEIGHTS), refs[q] + 0.0, f"map 2 W[{q}]")
        assert_bits_equal(out[q * (L - 1):(q + 1) * (L - 1)], O.c_divide(refs[q] + 0.0), f"map 2 avg[{q}]")
    agg.close()
    pool.free()


@pytest.mark.parametrize("be_out", [True, False])
def test_be_big_shape_partial_tile(ipls, O, be_out):
    """>= 1024 whole big tiles with a partial last tile (map 3): 8 x 4,200,001 x 8."""
    P, L, K = 8, 4_200_001, 8
    pool = Pool(ipls, P, L, K, True, O.SEED)
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    want = [O.c_synth_sum_checksum(L, q, K) for q in range(P)]
    for start in (ipls.START_ZERO, ipls.START_FIRST):
        agg.reduce_batch_out(0, pool.rows, pool.outs, start_mode=start, big_endian_in=True, big_endian_out=be_out)
        expect(agg.last_launch(), ipls, ipls.KERNEL_REDUCE, ipls.SHAPE_BIG, 16, 3, True, be_out, mapping=3)
        agg.sync()
        assert [ipls.checksum_dev(ipls.DeviceBuffer(o, L, big_endian=be_out)) for o in pool.outs] == want
    assert_bits_equal(pool.out_host(P - 1, L, be_out), ref_sum(O, L, P - 1, K), "partial-tile partition")
    agg.reduce_batch_out(0, pool.rows, pool.outs, start_mode=ipls.START_ACCUM, big_endian_in=True,
                         big_endian_out=be_out)
    expect(agg.last_launch(), ipls, ipls.KERNEL_REDUCE, ipls.SHAPE_BIG, 8, 0, True, be_out, mapping=3)
    agg.sync()
    s = ref_sum(O, L, 2, K)
    assert_bits_equal(pool.out_host(2, L, be_out), ref_sum(O, L, 2, K, O.START_ACCUM, s), "accum partial tile")
    agg.close()
    pool.free()


@pytest.mark.parametrize("P,L", [(1, 2_100_003), (2, 1_050_003)])
def test_be_mid_shape(ipls, O, P, L):
    """One or two partitions too short for 256 whole half tiles: the 256-lane
    mid shape (8 vectors per lane on hipcc's schedule for BE input) with a
    partial last tile."""
    K = 32
    pool = Pool(ipls, P, L, K, True, O.SEED)
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    refs = [ref_sum(O, L, q, K) for q in range(P)]
    for start in (ipls.START_ZERO, ipls.START_FIRST):
        agg.reduce_batch_out(0, pool.rows, pool.outs, start_mode=start, big_endian_in=True, big_endian_out=True)
        li = agg.last_launch()
        expect(li, ipls, ipls.KERNEL_REDUCE, ipls.SHAPE_MID, 8, 0, True, True, mapping=3)
        assert li["block"] == 256
        agg.sync()
        for q in range(P):
            assert_bits_equal(pool.out_host(q, L, True), refs[q], f"mid start {start} partition {q}")
    agg.reduce_batch_out(0, pool.rows, pool.outs, start_mode=ipls.START_ACCUM, big_endian_in=True,
                         big_endian_out=True)
    li = agg.last_launch()
    assert (li["kernel"], li["vectors"], li["be_in"]) == (ipls.KERNEL_REDUCE, 8, 1), li
    agg.sync()
    for q in range(P):
        assert_bits_equal(pool.out_host(q, L, True), O.c_reduce([O.c_synth_bucket(L, q, k) for k in range(K)], L,
                                                                O.START_ACCUM, refs[q]), f"mid accum {q}")
    agg.close()
    pool.free()


def test_be_fused_round_config_c(ipls, O, golden_meta):
    """The fused round (k_round: fold + W = AGG + REP + GetPartitions divide)
    on config C's shape with BE buckets: big shape, SEQF = 3; W and the
    averages against the oracle's checksums."""
    m = golden_meta["full"]["C"]
    P, L, K = m["partitions"], m["bucket_len"], m["peers"]
    pool = Pool(ipls, P, L, K, True, golden_meta["seed"], out=False)
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    avg = torch.empty(P * (L - 1), dtype=torch.float64, device="cuda")
    agg.aggregate_round(0, pool.rows, big_endian=True, out=ipls.DeviceBuffer.from_tensor(avg))
    expect(agg.last_launch(), ipls, ipls.KERNEL_ROUND, ipls.SHAPE_BIG, 16, 3, True, False)
    agg.sync()
    assert [agg.checksum(q, ipls.TGT_WEIGHTS) for q in range(P)] == m["sum_checksum"]
    base = int(avg.data_ptr())
    got = [ipls.checksum_dev(ipls.DeviceBuffer(base + 8 * q * (L - 1), L - 1)) for q in range(P)]
    assert got == m["avg_checksum"]
    # partition 1 in full (its averages start 8 mod 16: the shuffled-pair store path)
    w = agg.read(1, ipls.TGT_WEIGHTS)
    ref = ref_sum(O, L, 1, K)
    assert_bits_equal(w, ref, "W[1]")
    assert_bits_equal(avg[(L - 1):2 * (L - 1)].cpu().numpy(), O.c_divide(ref), "avg[1]")
    agg.close()
    del avg
    pool.free()


@pytest.mark.parametrize("P,L,K,shape", [(8, 4_200_001, 8, "big"), (1, 4_194_304 + 4099, 16, "half"),
                                         (1, 2_100_003, 8, "mid")])
def test_be_fused_round_partial_and_mid(ipls, O, P, L, K, shape):
    """The fused round's big (SEQF = 3), half (512 lanes, hipcc's schedule)
    and mid (R = 8) shapes, each with a partial tile, on BE buckets, on top
    of a REP accumulator that is not zero."""
    pool = Pool(ipls, P, L, K, True, O.SEED, out=False)
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    rep = [O.c_synth_bucket(L, 100 + q, 0) for q in range(P)]
    for q in range(P):
        agg.Update(rep[q], q, from_clients=False)          # Replicas_Gradients = +0.0 + R
    out = agg.aggregate_round(0, pool.rows, big_endian=True)
    li = agg.last_launch()
    want = {"big": (ipls.SHAPE_BIG, 1024, 16, 3), "half": (ipls.SHAPE_HALF, 512, 16, 0),
            "mid": (ipls.SHAPE_MID, 256, 8, 0)}[shape]
    assert (li["kernel"], li["be_in"], li["map"]) == (ipls.KERNEL_ROUND, 1, 3), li
    assert (li["shape"], li["block"], li["vectors"], li["seqf"]) == want, li
    for q in range(P):
        s = ref_sum(O, L, q, K)
        w = s + (0.0 + rep[q])                             # AggregatePartition, IPLS.java:1256
        assert_bits_equal(agg.read(q, ipls.TGT_WEIGHTS), w, f"W[{q}]")
        assert_bits_equal(out[q * (L - 1):(q + 1) * (L - 1)], O.c_divide(w), f"avg[{q}]")
    agg.close()
    pool.free()


@pytest.mark.parametrize("be", [False, True])
@pytest.mark.parametrize("P,L,K", [(1, 4_194_304, 32), (3, 4_194_304, 8), (5, 4_194_304 + 4099, 6),
                                   (7, 2_097_152 + 5, 4), (16, 1_048_576, 8)])
def test_half_shape(ipls, O, P, L, K, be):
    """Round 3's half shape (512 lanes x 16 vectors, ZERO / FIRST / ACCUM
    start, fewer than 1024 whole big tiles; big-endian input on hipcc's schedule):
    one to seven partitions, whole and partial last tiles (map 3), config B's
    geometry; into the accumulators, into caller buffers as doubles and as BE
    bytes (the update_file image); checked bit for bit on the first and last
    partition and by checksum on every one."""
    pool = Pool(ipls, P, L, K, be, O.SEED)
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    partial = L % (512 * 2 * 16) != 0
    for start in (ipls.START_ZERO, ipls.START_FIRST):
        agg.reduce_batch(0, pool.rows, start_mode=start, big_endian=be)
        li = agg.last_launch()
        assert (li["kernel"], li["shape"], li["block"], li["vectors"], li["seqf"], li["map"]) == \
            (ipls.KERNEL_REDUCE, ipls.SHAPE_HALF, 512, 16, 0, 3 if partial else 0), li
        for q in (0, P - 1):
            ref = ref_sum(O, L, q, K, O.START_ZERO if start == ipls.START_ZERO else O.START_FIRST)
            assert_bits_equal(agg.read(q), ref, f"start {start} partition {q}")
        if start == ipls.START_ZERO:
            assert [agg.checksum(q) for q in range(P)] == [O.c_synth_sum_checksum(L, q, K) for q in range(P)]
    for be_out in (False, True):
        agg.reduce_batch_out(0, pool.rows, pool.outs, start_mode=ipls.START_ZERO, big_endian_in=be,
                             big_endian_out=be_out)
        li = agg.last_launch()
        assert (li["shape"], li["be_in"], li["be_out"]) == (ipls.SHAPE_HALF, int(be), int(be_out)), li
        agg.sync()
        assert_bits_equal(pool.out_host(P - 1, L, be_out), ref_sum(O, L, P - 1, K), f"out be={be_out}")
    # ACCUM on top of the last fold: the half shape at R = 16 as well
    agg.reduce_batch(0, pool.rows, start_mode=ipls.START_ZERO, big_endian=be)
    agg.reduce_batch(0, pool.rows, start_mode=ipls.START_ACCUM, big_endian=be)
    li = agg.last_launch()
    assert (li["shape"], li["block"], li["vectors"], li["start"]) == \
        (ipls.SHAPE_HALF, 512, 16, ipls.START_ACCUM), li
    for q in (0, P - 1):
        s = ref_sum(O, L, q, K)
        assert_bits_equal(agg.read(q), ref_sum(O, L, q, K, O.START_ACCUM, s), f"accum partition {q}")
    agg.close()
    pool.free()


@pytest.mark.parametrize("start", ["ZERO", "ACCUM"])
def test_half_shape_ragged_model_geometry(ipls, O, start):
    """The half shape over a model geometry whose partitions differ in length
    (IPLS.java:1019-1028: chunk = ceil(M / P), the last partition short):
    partitions 0-1 are 256 whole half tiles (map 0, no partial tile in the
    grid's plan) and the last stops 2 doubles short, so its last tile is
    partial inside a whole-tile grid; every partition compared in full with
    the oracle, ZERO start and ACCUM on top of an arrival."""
    M, P, K = 3 * 4_194_303 - 2, 3, 5
    agg = ipls.Aggregator(M, P, max_peers=K)
    Ls = agg.lengths
    assert Ls[-1] < Ls[0]
    t = torch.empty(P * K * (max(Ls) + 32), dtype=torch.float64, device="cuda")
    base = (int(t.data_ptr()) + 255) // 256 * 256
    stride = (max(Ls) + 31) // 32 * 32
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * stride, Ls[q]) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], q, k, O.SEED)
    torch.cuda.synchronize()
    first = [O.synth_bucket(Ls[q], q, 40) for q in range(P)]
    if start == "ACCUM":
        for q in range(P):
            agg.Update(first[q], q)
    agg.reduce_batch(0, rows, start_mode=ipls.START_ACCUM if start == "ACCUM" else ipls.START_ZERO)
    li = agg.last_launch()
    assert (li["shape"], li["block"], li["vectors"], li["map"]) == (ipls.SHAPE_HALF, 512, 16, 0), li
    assert Ls == [4_194_304, 4_194_304, 4_194_302], Ls
    for q in range(P):
        bk = [O.c_synth_bucket(Ls[q], q, k) for k in range(K)]
        ref = O.c_reduce(bk, Ls[q], O.START_ACCUM, 0.0 + first[q]) if start == "ACCUM" else O.c_reduce(bk, Ls[q])
        assert_bits_equal(agg.read(q), ref, f"partition {q} (L={Ls[q]})")
    agg.close()
    del t
    torch.cuda.empty_cache()


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_chunked_calls_at_production_partitions(ipls, O, devices):
    """The chunked calls (round 6: per-call stages, two copy streams, chunk k
    on stream k mod 2) at config C's partition length, L = 4,194,304, with the
    chunk sizes the JNI shim and the Middleware servers use (2^19 and 2^21
    values) and one that leaves a short last chunk: three arrivals into AGG
    and one into REP of partition 1 through accumulate_chunked (big-endian and
    native), then finalize_chunked's commit_update bytes and
    get_partitions_wire_chunked's stream over both partitions -- bit for bit
    against the oracle (Updater.java:115-117, IPLS.java:1248-1274, 1159-1174,
    Middleware.java:164-170)."""
    import ctypes
    from ipls import _native as N
    L, P = 4_194_304, 2
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, devices=devices)
    lib, h = agg._lib, agg._h
    gs = [O.synth_bucket(L, 1, 700 + k) * (1.0 + k) for k in range(4)]
    for g in gs:
        g[-1] = 1.0                                    # each arrival's count slot
    for k, (g, chunk, be, tgt) in enumerate(((gs[0], 1 << 19, True, N.TGT_AGG), (gs[1], 1 << 21, False, N.TGT_AGG),
                                             (gs[2], 1_000_002, True, N.TGT_AGG), (gs[3], 1 << 19, True, N.TGT_REP))):
        raw = O.be_encode(g) if be else g.tobytes()

        @N.CHUNK_SOURCE
        def src(ctx, dst, off, n, raw=raw):
            ctypes.memmove(dst, ctypes.c_char_p(raw[8 * off:8 * (off + n)]), 8 * n)
            return 0
        assert lib.ipls_agg_accumulate_chunked(h, 1, tgt, L, N.HOST_BE if be else N.HOST_F64, chunk, src, None) == 0
    agg_want = O.fold(O.fold(O.fold(np.zeros(L), gs[0]), gs[1]), gs[2])
    assert_bits_equal(agg.read(1, N.TGT_AGG), agg_want, "AGG[1]")
    w = agg_want + O.fold(np.zeros(L), gs[3])
    out = bytearray(8 * L)

    @N.CHUNK_SINK
    def sink(ctx, vals, off, n):
        out[8 * off:8 * (off + n)] = ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n)
        return 0
    assert lib.ipls_agg_finalize_chunked(h, 1, N.HOST_BE, 1 << 19, sink, None) == 0
    assert bytes(out) == O.be_encode(w), "commit_update bytes of W[1]"
    got = bytearray()

    @N.CHUNK_SINK
    def wsink(ctx, vals, off, n):
        got.extend(ctypes.string_at(ctypes.cast(vals, ctypes.c_void_p), 8 * n))
        return 0
    assert lib.ipls_agg_get_partitions_wire_chunked(h, 1 << 19, wsink, None) == 0
    assert bytes(got) == O.be_encode_canonical(O.get_partitions([np.zeros(L), w])), "task-3 stream"
    agg.close()
