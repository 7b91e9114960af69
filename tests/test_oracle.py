"""CPU-only: the oracle (C and Python restatements) against the committed
golden fixtures and against each other, plus reference-format pins.

Parity status: unpinned -- the reference ships no golden vectors for this path
and cannot run here (no JDK).  The ETHModel fixture pins the byte order (a
Java-written BE double array) and the partition geometry of config A.
"""
import gzip
import struct

import numpy as np
import pytest

from conftest import GOLDEN, assert_bits_equal
from oracle import oracle as O


def test_partition_geometry_config_a():
    # ETHModel M=443,610, -pa 3 -> 147,872 / 147,872 / 147,869
    assert O.chunk_size(443610, 3) == 147871
    assert [O.partition_len(443610, 3, i) for i in range(3)] == [147872, 147872, 147869]
    lib = O.c_oracle()
    assert [lib.ipls_oracle_partition_len(443610, 3, i) for i in range(3)] == [147872, 147872, 147869]


@pytest.mark.parametrize("M,P", [(10, 4), (12, 4), (443610, 3), (1000003, 16), (7, 3), (5, 1)])
def test_organize_python_vs_c(M, P):
    flat = O.synth_bucket(M, 1, 1)
    py = O.organize_gradients(flat, M, P)
    lib = O.c_oracle()
    for p in range(P):
        L = O.partition_len(M, P, p)
        out = np.empty(L)
        assert lib.ipls_oracle_organize(O._dp(flat), M, M, P, p, O._dp(out)) == 0
        assert_bits_equal(out, py[p], f"M={M} P={P} p={p}")
        assert py[p][-1] == 1.0 or L == 0


def test_organize_negative_size():
    with pytest.raises(ValueError, match="NegativeArraySize"):
        O.organize_gradients(np.zeros(10), 10, 7)
    # M=7, P=7: partition 4 has length 0, the count-slot store overruns it
    with pytest.raises(ValueError, match="ArrayIndexOutOfBounds"):
        O.organize_gradients(np.zeros(7), 7, 7)


def test_golden_organize(golden):
    for M, P, tag in [(10, 4, "org10x4"), (12, 4, "org12x4")]:
        got = O.organize_gradients(np.arange(1.0, M + 1.0), M, P)
        for p in range(P):
            assert_bits_equal(got[p], golden[f"{tag}_p{p}"], tag)
    # the M=12, P=4 last partition is the count slot alone
    assert list(golden["org12x4_p3"]) == [1.0]


@pytest.mark.parametrize("case", ["szero", "cancel", "special"])
def test_golden_edge_folds(golden, case):
    bufs = list(golden[f"{case}_bufs"])
    L = len(bufs[0])
    assert_bits_equal(O.reduce(bufs, L, O.START_ZERO), golden[f"{case}_zero"], case)
    assert_bits_equal(O.c_reduce(bufs, L, O.START_ZERO), golden[f"{case}_zero"], case + " C")
    if f"{case}_first" in golden:
        assert_bits_equal(O.c_reduce(bufs, L, O.START_FIRST), golden[f"{case}_first"], case + " first")


def test_fold_semantics_pinned(golden):
    # ZERO start turns -0.0 into +0.0, FIRST start keeps -0.0
    assert np.all(np.signbit(golden["szero_first"]))
    assert not np.any(np.signbit(golden["szero_zero"]))
    # fixed order: ((0 + 1e16) + 1) + -1e16 == 0.0, not 1.0
    assert golden["cancel_zero"][0] == 0.0
    assert golden["cancel_zero"][1] == 0.0


def test_golden_divide(golden):
    for case, sec in [("div", False), ("div_zero", False), ("div_nzero", False), ("div_secure", True)]:
        assert_bits_equal(O.divide(golden[f"{case}_w"], sec), golden[f"{case}_out"], case)
        lib_out = np.empty(len(golden[f"{case}_w"]) - 1)
        O.c_oracle().ipls_oracle_divide(O._dp(np.ascontiguousarray(golden[f"{case}_w"])),
                                        len(golden[f"{case}_w"]), int(sec), O._dp(lib_out))
        assert_bits_equal(lib_out, golden[f"{case}_out"], case + " C")
    # count 0.0 and -0.0 both pass values through (Java 0.0 == -0.0)
    assert list(golden["div_nzero_out"]) == [3.0, -6.0]


def test_golden_encode(golden):
    assert_bits_equal(O.encode_secure(golden["enc_in"]), golden["enc_out"], "encode")
    assert golden["enc_out"][0] == -1e13 and golden["enc_out"][4] == 1e13


def test_codecs(golden):
    raw = bytes(golden["be_raw"])
    canon = bytes(golden["be_canon"])
    assert raw == O.be_encode(golden["be_in"])
    assert canon == O.be_encode_canonical(golden["be_in"])
    assert canon[8:16] == bytes.fromhex("7ff8000000000000")      # doubleToLongBits
    assert raw[16:24] == bytes.fromhex("fff0000000000001")       # putDouble keeps raw bits
    # C codec agrees
    x = np.ascontiguousarray(golden["be_in"])
    buf = np.empty(8 * len(x), dtype=np.uint8)
    O.c_oracle().ipls_oracle_be_encode(O._dp(x), len(x), buf.ctypes.data_as(O.ctypes.POINTER(O.ctypes.c_uint8)))
    assert bytes(buf) == raw
    assert_bits_equal(O.be_decode(raw)[:1], x[:1], "decode")


def test_frame_layout(golden):
    fr = bytes(golden["frame_bytes"])
    pid, n, a, b = struct.unpack(">hiii", fr[:14])
    assert (pid, n, a, b) == (3, 4, 7, 42)
    assert fr[14 + 32:] == b"QmPeerOrigin"
    pid, n, a, b, g, origin = O.frame_decode(fr)
    assert_bits_equal(g, golden["frame_g"], "frame")
    assert O.frame_decode(O.frame_encode(None, 1, 2, 3, b"x"))[4] is None
    with pytest.raises(ValueError):
        O.frame_decode(fr[:20])


def test_synth_python_vs_c():
    for L, p, k in [(1, 0, 0), (5, 3, 9), (4097, 15, 63)]:
        assert_bits_equal(O.synth_bucket(L, p, k), O.c_synth_bucket(L, p, k), "synth")


def test_golden_synth_small(golden, golden_meta):
    for key, val in golden.items():
        if not key.startswith("synth_"):
            continue
        _, P, L, K, p, mode = key.split("_")
        L, K, p = int(L[1:]), int(K[1:]), int(p[1:])
        bufs = [O.synth_bucket(L, p, k) for k in range(K)]
        m = O.START_ZERO if mode == "zero" else O.START_FIRST
        assert_bits_equal(O.c_reduce(bufs, L, m), val, key)
    for key, cs in golden_meta["synth_checksum"].items():
        _, P, L, K, p, mode = key.split("_")
        L, K, p = int(L[1:]), int(K[1:]), int(p[1:])
        if L > 100000:
            continue
        bufs = [O.synth_bucket(L, p, k) for k in range(K)]
        m = O.START_ZERO if mode == "zero" else O.START_FIRST
        assert O.checksum(O.reduce(bufs, L, m)) == cs, key


def test_full_size_checksum_spot(golden_meta):
    """One partition of config B via the on-the-fly C oracle (OpenMP)."""
    m = golden_meta["full"]["B"]
    assert O.c_synth_sum_checksum(m["bucket_len"], 5, m["peers"]) == m["sum_checksum"][5]


def test_ethmodel_fixture(ethmodel, golden_meta):
    assert ethmodel.shape == (443610,)
    assert np.isfinite(ethmodel).all()
    ref = O.ethmodel_path()
    if ref is not None:       # build container: fixture == the reference file's [D payload
        assert_bits_equal(O.parse_ethmodel(ref.read_bytes()), ethmodel, "ETHModel")


def test_config_a_oracle(ethmodel, golden_meta):
    import hashlib
    meta = golden_meta["config_a"]
    M = meta["model_size"]
    peers = [ethmodel + O.synth_bucket(M + 1, 0, k)[:M] for k in range(3)]
    parts = [O.organize_gradients(g, M, 3) for g in peers]
    sums = [O.c_reduce([parts[k][p] for k in range(3)], O.partition_len(M, 3, p)) for p in range(3)]
    for p in range(3):
        assert hashlib.sha256(sums[p].astype(">f8").tobytes()).hexdigest() == meta["sum_sha256"][p]
    avg = O.get_partitions(sums)
    assert hashlib.sha256(avg.astype(">f8").tobytes()).hexdigest() == meta["avg_sha256"]


def test_updater_loop_baseline_matches_reduce():
    L, K = 4099, 6
    bufs = [O.synth_bucket(L, 1, k) for k in range(K)]
    be = [np.frombuffer(O.be_encode(b), dtype=np.uint8).copy() for b in bufs]
    assert_bits_equal(O.c_updater_loop(be, L), O.reduce(bufs, L), "updater loop")


def test_promote_future_oracle():
    """IPLS.java:1557-1562: AGG takes FUTURE's values (bits, incl. -0.0/NaN), FUTURE -> +0.0."""
    from oracle import oracle as O
    fut = np.array([1.5, -0.0, np.nan, 5e-324])
    agg = np.array([9.0, 9.0, 9.0, 9.0])
    ref = fut.copy()
    O.promote_future(agg, fut)
    assert agg.view(np.uint64).tolist() == ref.view(np.uint64).tolist()
    assert fut.view(np.uint64).tolist() == [0, 0, 0, 0]


@pytest.mark.parametrize("secure", [False, True])
def test_c_synth_avg_checksum_matches_numpy(secure):
    """The large-size GPU tests check averages through this C checksum."""
    L, p, k = 5003, 2, 3
    S = O.reduce([O.synth_bucket(L, p, j) for j in range(k)], L)
    assert O.c_synth_avg_checksum(L, p, k, secure) == O.checksum(O.divide(S, secure))


@pytest.mark.parametrize("k,k_own", [(6, 3), (5, 1), (4, 4)])
def test_c_synth_replica_checksum_matches_numpy(k, k_own):
    """The bench's cross-GPU replica leg checks W = AGG + (+0.0 + R) through this."""
    L, p = 4099, 3
    own = O.reduce([O.synth_bucket(L, p, j) for j in range(k_own)], L)
    part = O.reduce([O.synth_bucket(L, p, j) for j in range(k_own, k)], L)
    W = own + O.reduce([part], L)
    assert O.c_synth_replica_checksum(L, p, k, k_own) == O.checksum(W)


def test_c_b64url_encoder_matches_python_and_frames():
    """The C oracle's Base64.getUrlEncoder restatement (MyIPFSClass.java:1016)
    against Python's RFC 4648 urlsafe encoder (an independent implementation
    of the same alphabet and '=' padding) over every length mod 3, and over
    whole Marshall_Packet frames."""
    import ctypes
    lib = O.c_oracle()
    lib.ipls_oracle_b64url_encode.restype = ctypes.c_int64
    lib.ipls_oracle_b64url_encode.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    rng = np.random.default_rng(7)
    cases = [bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in (0, 1, 2, 3, 4, 5, 1000, 1001, 1002)]
    cases += [O.frame_encode(O.synth_bucket(L, 1, 2), 7, 33, 3, origin)
              for L, origin in ((5, b""), (6, b"Q"), (1001, b"QmOrigin"))]
    for data in cases:
        src = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, dtype=np.uint8)
        out = np.zeros(4 * ((len(data) + 2) // 3) + 1, dtype=np.uint8)
        n = lib.ipls_oracle_b64url_encode(src.ctypes.data, len(data), out.ctypes.data)
        assert out[:n].tobytes() == O.java_b64url_encode(data), len(data)
