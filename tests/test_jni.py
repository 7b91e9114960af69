"""The JNI shim (ipls-java-api_amd/jni/ipls_jni.c), compiled and driven
without a JDK (ADVICE r1 JNI items).

tests/jni/jni.h declares exactly the JNI types and JNIEnv entries the shim
uses; tests/jni/fake_jvm.c implements them (Java arrays, direct ByteBuffers,
pending exceptions) and counts breaks of the JNI rules (calls inside a
critical region, calls with an exception pending, unreleased elements,
region writes past an array).  The shim is built with -Wall -Wextra -Werror
into one test library with the fake JVM and linked to the real
libipls_agg.so.  CPU tests cover the argument checks the shim does before
the library is called; -m gpu tests run whole Java-API sequences through the
natives against the oracle, including the exception mapping and the
guarantee that a rejected call leaves the accumulators unchanged.

The shim's ring chunk is pinned to 512 Ki values in both directions here
(IPLS_JNI_RING_CHUNK, read once per process), so that the partitions of
about 1M doubles below are multi-chunk calls whose chunk edges the tests
name; its defaults (16 MiB in, 4 MiB out, profiles/r06/d) only change how
many chunks a call takes.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, assert_bits_equal

os.environ["IPLS_JNI_RING_CHUNK"] = "524288"

BUILD = ROOT / "tests" / "jni" / "build"
LIB = BUILD / "libfakejni.so"
AGG = ROOT / "ipls-java-api_amd" / "lib"

_j = None


def build():
    BUILD.mkdir(parents=True, exist_ok=True)
    subprocess.run(["gcc", "-std=c11", "-O1", "-g", "-Wall", "-Wextra", "-Werror", "-fPIC", "-shared",
                    "-DIPLS_JNI_CALL_HOOK=fj_library_call",
                    f"-I{ROOT / 'tests' / 'jni'}", f"-I{ROOT / 'include'}",
                    str(ROOT / "tests" / "jni" / "fake_jvm.c"), str(ROOT / "ipls-java-api_amd" / "jni" / "ipls_jni.c"),
                    f"-L{AGG}", "-lipls_agg", f"-Wl,-rpath,{AGG}", "-o", str(LIB)], check=True)


class JVM:
    """ctypes view of the fake JVM + the natives of NativeAggregator."""

    def __init__(self):
        build()
        L = ctypes.CDLL(str(LIB))
        vp = ctypes.c_void_p
        for name, res, args in [
            ("fj_env", vp, []), ("fj_new_bytes", vp, [vp, ctypes.c_int32]), ("fj_new_ints", vp, [vp, ctypes.c_int32]),
            ("fj_new_longs", vp, [vp, ctypes.c_int32]), ("fj_new_doubles", vp, [vp, ctypes.c_int32]),
            ("fj_new_objects", vp, [vp, ctypes.c_int32]), ("fj_new_direct", vp, [vp, ctypes.c_int64]),
            ("fj_data", vp, [vp]), ("fj_len", ctypes.c_int32, [vp]), ("fj_free", None, [vp]),
            ("fj_exception", ctypes.c_char_p, []), ("fj_exception_msg", ctypes.c_char_p, []), ("fj_clear", None, []),
            ("fj_violations", ctypes.c_int, []), ("fj_last_violation", ctypes.c_char_p, []),
            ("fj_reset_violations", None, []), ("fj_library_calls", ctypes.c_int, []),
            ("fj_selftest_critical_rule", ctypes.c_int, []),
            ("fj_inject", None, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                 vp, ctypes.c_int64]),
            ("fj_inject_state", ctypes.c_int, []), ("fj_inject_join", ctypes.c_int, [])]:
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        self.L = L
        self.env = ctypes.c_void_p(L.fj_env())
        self.keep = []

    # ---- Java objects ----
    def doubles(self, a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        return ctypes.c_void_p(self.L.fj_new_doubles(a.ctypes.data, a.size))

    def bytes_(self, b):
        a = np.frombuffer(bytes(b), dtype=np.uint8)
        return ctypes.c_void_p(self.L.fj_new_bytes(a.ctypes.data if a.size else None, a.size))

    def ints(self, a):
        a = np.ascontiguousarray(a, dtype=np.int32)
        return ctypes.c_void_p(self.L.fj_new_ints(a.ctypes.data if a.size else None, a.size))

    def longs(self, a):
        a = np.ascontiguousarray(a, dtype=np.int64)
        return ctypes.c_void_p(self.L.fj_new_longs(a.ctypes.data if a.size else None, a.size))

    def objects(self, objs):
        arr = (ctypes.c_void_p * max(1, len(objs)))(*[o.value for o in objs])
        return ctypes.c_void_p(self.L.fj_new_objects(arr, len(objs)))

    def direct(self, nbytes=None, heap=False):
        """A direct ByteBuffer over host memory this object keeps alive
        (heap=True: a heap ByteBuffer, no address)."""
        if heap:
            return ctypes.c_void_p(self.L.fj_new_direct(None, -1)), None
        mem = np.zeros(nbytes, dtype=np.uint8)
        self.keep.append(mem)
        return ctypes.c_void_p(self.L.fj_new_direct(mem.ctypes.data, nbytes)), mem

    def data(self, obj, dtype, n=None):
        n = self.L.fj_len(obj) if n is None else n
        size = np.dtype(dtype).itemsize * n
        buf = (ctypes.c_char * size).from_address(self.L.fj_data(obj))
        return np.frombuffer(buf, dtype=dtype).copy()

    # ---- calls ----
    def call(self, name, *args, res=None):
        f = getattr(self.L, "Java_NativeAggregator_" + name)
        f.restype = res
        self.L.fj_clear()
        self.L.fj_reset_violations()
        conv = []
        for a in args:
            if isinstance(a, float):
                conv.append(ctypes.c_double(a))
            elif isinstance(a, int):
                assert abs(a) < 2 ** 31, "pass jlong arguments as ctypes.c_int64"
                conv.append(ctypes.c_int32(a))
            elif a is None:
                conv.append(ctypes.c_void_p(None))
            else:
                conv.append(a)
        r = f(self.env, None, *conv)
        v = self.L.fj_violations()
        assert v == 0, f"{name}: JNI rule broken: {self.L.fj_last_violation()}"
        exc = self.L.fj_exception()
        return r, (exc.decode() if exc else None)


@pytest.fixture(scope="module")
def jvm():
    global _j
    if _j is None:
        _j = JVM()
    return _j


L64 = ctypes.c_int64


def test_shim_builds_with_werror_and_exports_every_native(jvm):
    import re
    java = (ROOT / "ipls-java-api_amd" / "java" / "NativeAggregator.java").read_text()
    natives = set(re.findall(r"\bnative\s+[\w\[\]<>.]+\s+(\w+)\s*\(", java))
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"Java_NativeAggregator_(\w+)", out))
    assert natives == exported, natives ^ exported


def test_no_critical_region_across_a_library_call(jvm):
    """the shim never holds a GetPrimitiveArrayCritical
    region while it calls into the library (a call that may wait on the GPU
    would block a real JVM's GC for that long).  The fake JVM fails any call
    made with a region open (JVM.call checks fj_violations after every
    native, and that no region is left open); this checks the rule can fire
    and that the shim reports its library calls.  The shim's one critical
    region is critical_copy's: one memcpy of one ring
    chunk inside a chunk callback, opened and released in that function with
    no JNI or library call in between -- checked here on the source text."""
    import re
    assert jvm.L.fj_selftest_critical_rule() >= 1
    before = jvm.L.fj_library_calls()
    r, exc = jvm.call("shardPlan", 4, 2, res=ctypes.c_void_p)
    assert exc is None and jvm.L.fj_library_calls() > before
    shim = (ROOT / "ipls-java-api_amd" / "jni" / "ipls_jni.c").read_text()
    code = "\n".join(ln for ln in shim.splitlines() if not ln.lstrip().startswith(("*", "/*")))
    assert code.count("GetPrimitiveArrayCritical") == 1 and code.count("ReleasePrimitiveArrayCritical") == 2
    body = code[code.index("static int critical_copy("):]
    body = body[:body.index("\n}\n")]
    assert "GetPrimitiveArrayCritical" in body and body.count("ReleasePrimitiveArrayCritical") == 2
    end = body.rindex("ReleasePrimitiveArrayCritical") + len("ReleasePrimitiveArrayCritical")
    inside = body[body.index("GetPrimitiveArrayCritical"):end]
    assert not re.search(r"\(\*env\)->(?!ReleasePrimitiveArrayCritical)|LIB\(|ipls_agg_", inside), inside


def test_shard_plan_native(jvm):
    r, exc = jvm.call("shardPlan", 10, 4, res=ctypes.c_void_p)
    assert exc is None
    assert list(jvm.data(r, np.int32)) == [0, 0, 0, 1, 1, 1, 2, 2, 2, 3]
    r, exc = jvm.call("shardPlan", 10, 0, res=ctypes.c_void_p)
    assert r is None and exc == "java/lang/IllegalArgumentException"


def test_direct_buffer_checks_before_the_library(jvm):
    """a heap ByteBuffer (no address) or a position/length outside
    the buffer is an IllegalArgumentException, never a silent no-op or a read
    of the wrong bytes -- checked before the handle is even looked at."""
    heap, _ = jvm.direct(heap=True)
    buf, _ = jvm.direct(64)
    for name, args in [("accumulateDirect", (L64(0), 0, 0, heap, 0, L64(4), 1)),
                       ("accumulateDirect", (L64(0), 0, 0, buf, 40, L64(4), 1)),      # 40 + 32 > 64
                       ("accumulateDirect", (L64(0), 0, 0, buf, -8, L64(1), 1)),
                       ("accumulateAsyncDirect", (L64(0), 0, 0, heap, 0, L64(1), 1)),
                       ("updateIndirect", (L64(0), 0, 0, buf, 8, L64(57))),
                       ("setWeightsDirect", (L64(0), 0, heap, 0, L64(1))),
                       ("otherReplicaDirect", (L64(0), 0, 1, 0, buf, 0, L64(9))),
                       ("getPartitionsWire", (L64(0), heap, 0, L64(8))),
                       # counts whose byte size overflows a jlong (8 * n wraps to a small or
                       # negative value) are rejected before any multiplication
                       ("accumulateDirect", (L64(0), 0, 0, buf, 0, L64(1 << 61), 1)),
                       ("accumulateDirect", (L64(0), 0, 0, buf, 8, L64((1 << 63) - 1), 1)),
                       ("accumulateAsyncDirect", (L64(0), 0, 0, buf, 0, L64((1 << 61) + 1), 1)),
                       ("setWeightsDirect", (L64(0), 0, buf, 0, L64(1 << 62))),
                       ("otherReplicaDirect", (L64(0), 0, 1, 0, buf, 0, L64(1 << 61))),
                       ("updateIndirect", (L64(0), 0, 0, buf, 65, L64(0))),           # pos past the end
                       ("updateGradientDirect", (L64(0), heap, 0, L64(1), jvm.ints([0]))),
                       ("updateGradientDirect", (L64(0), buf, 8, L64(8), jvm.ints([0])))]:   # 8 + 64 > 64
        _, exc = jvm.call(name, *args)
        assert exc == "java/lang/IllegalArgumentException", (name, exc)


def test_many_texts_and_files_reserve_local_refs(jvm):
    """A native frame is guaranteed 16 local references; ingestTexts and
    mergeFiles hold one per element at once, so they reserve the rest with
    EnsureLocalCapacity first (the fake JVM counts live element refs against
    the reserved capacity).  A null handle makes the library call fail after
    the refs are taken, so this runs without a GPU."""
    texts = jvm.objects([jvm.bytes_(b"AAAA")] * 40)
    _, exc = jvm.call("ingestTexts", L64(0), 0, texts, 2, None, None, res=ctypes.c_int32)
    assert exc == "java/lang/IllegalArgumentException"
    files = jvm.objects([jvm.bytes_(b"\0" * 16)] * 24)
    _, exc = jvm.call("mergeFiles", L64(0), files, 0, res=ctypes.c_void_p)
    assert exc == "java/lang/IllegalArgumentException"


def test_open_without_gpu_throws(jvm):
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h, exc = jvm.call("open", L64(443610), 3, 3, 0, 0, 0, res=ctypes.c_int64)
    assert h == 0 and exc == "java/lang/RuntimeException"
    assert b"device" in jvm.L.fj_exception_msg().lower()


# ---------------------------------------------------------------------------
# on the GPU: Java-API sequences through the natives
# ---------------------------------------------------------------------------
@pytest.fixture
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("-m gpu run without a visible GPU")


@pytest.fixture(scope="module")
def O():
    from oracle import oracle as o   # checker only
    return o


def _open(jvm, M, P, devices=None):
    if devices is None:
        h, exc = jvm.call("open", L64(M), P, 3, 0, 0, 0, res=ctypes.c_int64)
    else:
        h, exc = jvm.call("openDevices", L64(M), P, 3, 0, 0, jvm.ints(devices), res=ctypes.c_int64)
    assert exc is None and h
    return L64(h)


@pytest.mark.gpu
def test_jni_round_against_oracle(jvm, gpu, O):
    """IPLS round through the natives: updateGradient (own partitions),
    accumulate (heap double[]), updateFromBytes (direct buffer at a non-zero
    position), finalizePartition (commit_update bytes), aggregateRound,
    getPartitions and the Middleware wire stream."""
    M, P, K = 30011, 3, 4
    h = _open(jvm, M, P)
    peers = [O.synth_bucket(M, 4, k) for k in range(K)]
    parts = [O.organize_gradients(g, M, P) for g in peers]
    _, exc = jvm.call("updateGradient", h, jvm.doubles(peers[0]), jvm.ints([0, 1, 2]))
    assert exc is None
    for p in range(P):
        _, exc = jvm.call("accumulate", h, p, 0, jvm.doubles(parts[1][p]))
        assert exc is None
        # a direct buffer with position 16: the bucket starts 16 bytes in
        be = O.be_encode(parts[2][p])
        buf, mem = jvm.direct(16 + len(be) + 8)
        mem[16:16 + len(be)] = np.frombuffer(be, dtype=np.uint8)
        _, exc = jvm.call("accumulateDirect", h, p, 0, buf, 16, L64(len(be) // 8), 1)
        assert exc is None
        split_out = jvm.doubles(np.zeros(len(parts[3][p])))
        _, exc = jvm.call("split", h, jvm.doubles(peers[3]), p, split_out)
        assert exc is None
        assert_bits_equal(jvm.data(split_out, np.float64), parts[3][p], "split")
        _, exc = jvm.call("accumulate", h, p, 0, split_out)
        assert exc is None
    sums = []
    for p in range(P):
        s = O.reduce([parts[k][p] for k in range(K)], len(parts[0][p]))
        sums.append(s)
        out = jvm.bytes_(b"\0" * (8 * len(s)))
        _, exc = jvm.call("finalizePartition", h, p, out)
        assert exc is None
        assert jvm.data(out, np.uint8).tobytes() == O.be_encode(s)
    avg = O.get_partitions(sums)
    got = jvm.doubles(np.zeros(M))
    _, exc = jvm.call("getPartitions", h, got)
    assert exc is None
    assert_bits_equal(jvm.data(got, np.float64), avg, "getPartitions")
    wire, mem = jvm.direct(8 * M + 24)
    _, exc = jvm.call("getPartitionsWire", h, wire, 24, L64(8 * M))
    assert exc is None and mem[24:].tobytes() == O.be_encode_canonical(avg)
    jvm.call("close", h)


@pytest.mark.gpu
def test_jni_heap_accumulate_pipelined(jvm, gpu, O):
    """accumulate(double[]) for partitions of >= 2 chunks (2 x 512 Ki doubles)
    goes chunk by chunk through the library's pinned ring
    (ipls_agg_accumulate_chunked pulling from the heap array with
    GetDoubleArrayRegion), each chunk sent while the next is copied: the bits
    equal the oracle's whole-bucket folds.  An odd partition length (the last
    chunk short and odd), a logically-zero AGG and then a live one, REP as
    the target, and an array longer than the partition (Java reads only the
    first L, Updater.java:115-117); a short array still raises
    ArrayIndexOutOfBoundsException with nothing folded."""
    M, P = 2 * 1048576 + 4099, 2                 # L = 1,050,627 / 1,050,626: 2.004 chunks each
    h = _open(jvm, M, P)
    lens = [O.partition_len(M, P, p) for p in range(P)]
    assert min(lens) >= 2 * 524288 and lens[0] % 2 == 1
    acc = {(p, t): np.zeros(lens[p]) for p in range(P) for t in (0, 1)}
    for k in range(3):
        for p in range(P):
            for t in (0, 1):                         # AGG, REP
                g = O.synth_bucket(lens[p] + (5 if k == 2 else 0), p, 10 * k + t) * (10.0 ** (k - 1))
                g[::1009] = -0.0
                _, exc = jvm.call("accumulate", h, p, t, jvm.doubles(g))
                assert exc is None
                acc[(p, t)] = O.fold(acc[(p, t)], g)
    _, exc = jvm.call("accumulate", h, 0, 0, jvm.doubles(np.ones(lens[0] - 1)))
    assert exc == "java/lang/ArrayIndexOutOfBoundsException"
    for p in range(P):   # AggregatePartition: W = AGG + REP (IPLS.java:1256), as commit_update bytes
        out = jvm.bytes_(b"\0" * (8 * lens[p]))
        _, exc = jvm.call("finalizePartition", h, p, out)
        assert exc is None
        assert jvm.data(out, np.uint8).tobytes() == O.be_encode(acc[(p, 0)] + acc[(p, 1)]), f"W[{p}]"
    jvm.call("close", h)


@pytest.mark.gpu
def test_jni_heap_natives_are_one_ordered_unit(jvm, gpu, O):
    """a second thread's call on the same
    partition, started in the middle of a heap-array native, lands before or
    after the native's whole work, never inside it -- and it does not wait for
    the native's Java-side copies (no shard lock is held across them).

    accumulate(double[]) of bucket A (3 chunks): the fake JVM starts a second
    thread's ipls_agg_accumulate of bucket B into the same (p, target) at the
    native's 2nd GetDoubleArrayRegion -- after chunk 0 was handed to the
    library -- and gives it 300 ms.  It returns inside that window
    (fj_inject_state 1), and the target holds one serial order, (acc + B) + A:
    the native's bucket takes effect when its last chunk has landed, bit for
    bit against the oracle (Updater.java:72-149: whole-bucket folds under
    PeerData.mtx; Middleware.java:224, 246: the whole bucket is read before
    the fold).  The per-range library calls the round-4 shim used do
    interleave under the same schedule (chunk 0 of A, then B, then the rest
    of A), and those bits differ from every serial order: the check can tell.

    finalizePartition(byte[]): a second thread's set_weights on the same
    partition (Download_Scheduler.cache_partition) started at the native's 2nd
    SetByteArrayRegion returns inside the window too; the bytes are exactly
    this call's AGG + REP (a snapshot, not torn), and W holds the new weights
    after the join."""
    from ipls import _native as N
    lib = N.lib()
    M, P = 2 * 1048576 + 4099, 2
    h = _open(jvm, M, P)
    L = O.partition_len(M, P, 1)
    assert L > 2 * 524288
    a = O.synth_bucket(L, 1, 501)
    b = O.synth_bucket(L, 1, 502) * 7.0
    base = O.synth_bucket(L, 1, 500)
    _, exc = jvm.call("accumulate", h, 1, 0, jvm.doubles(base))
    assert exc is None
    jvm.L.fj_inject(0, 2, 300, h.value, 1, 0, b.ctypes.data, L)
    _, exc = jvm.call("accumulate", h, 1, 0, jvm.doubles(a))
    assert exc is None
    assert jvm.L.fj_inject_state() == 1, "the second thread's fold waited for accumulate(double[])'s heap copies"
    assert jvm.L.fj_inject_join() == 0
    serial = O.fold(O.fold(O.fold(np.zeros(L), base), b), a)
    got = np.zeros(L)
    assert lib.ipls_agg_sync(ctypes.c_void_p(h.value)) == 0
    assert lib.ipls_agg_read(ctypes.c_void_p(h.value), 1, N.TGT_AGG, got.ctypes.data, L, N.HOST_F64) == 0
    assert_bits_equal(got, serial, "one serial order: (base + B) + A")
    # the round-4 pattern under the same schedule: per-range calls interleave
    c = 524288
    mixed = O.fold(np.zeros(L), base)
    mixed[:c] = mixed[:c] + a[:c]
    mixed = mixed + b
    mixed[c:] = mixed[c:] + a[c:]
    other = O.fold(O.fold(O.fold(np.zeros(L), base), a), b)
    assert not np.array_equal(mixed.view(np.uint64), serial.view(np.uint64))
    assert not np.array_equal(mixed.view(np.uint64), other.view(np.uint64))
    hv = ctypes.c_void_p(h.value)
    from ipls import PinnedBuffer
    pb = PinnedBuffer(8 * L)
    pv = pb.view()
    t = ctypes.c_uint64()
    assert lib.ipls_agg_reset(hv, 1) == 0
    _, exc = jvm.call("accumulate", h, 1, 0, jvm.doubles(base))
    assert exc is None
    pv[:8 * L] = np.frombuffer(a.tobytes(), dtype=np.uint8)
    assert lib.ipls_agg_accumulate_range(hv, 1, N.TGT_AGG, pb.ptr, 0, c, N.HOST_F64, ctypes.byref(t)) == 0
    assert lib.ipls_agg_wait(hv, t.value) == 0
    assert lib.ipls_agg_accumulate(hv, 1, N.TGT_AGG, b.ctypes.data, L, N.HOST_F64) == 0
    assert lib.ipls_agg_accumulate_range(hv, 1, N.TGT_AGG, pb.ptr + 8 * c, c, L - c, N.HOST_F64, ctypes.byref(t)) == 0
    assert lib.ipls_agg_wait(hv, t.value) == 0
    assert lib.ipls_agg_read(hv, 1, N.TGT_AGG, got.ctypes.data, L, N.HOST_F64) == 0
    assert_bits_equal(got, mixed, "per-range calls with a fold in between: the mixed order")
    pb.close()
    # finalizePartition(byte[]) against a concurrent set_weights
    assert lib.ipls_agg_reset(hv, 1) == 0
    r = O.synth_bucket(L, 1, 503) * 3.0
    for t_, g in ((0, a), (1, r)):
        _, exc = jvm.call("accumulate", h, 1, t_, jvm.doubles(g))
        assert exc is None
    w_new = O.synth_bucket(L, 1, 504)
    jvm.L.fj_inject(1, 2, 300, h.value, 1, 0, w_new.ctypes.data, L)
    out = jvm.bytes_(b"\0" * (8 * L))
    _, exc = jvm.call("finalizePartition", h, 1, out)
    assert exc is None
    assert jvm.L.fj_inject_state() == 1, "set_weights waited for finalizePartition(byte[])'s heap copies"
    assert jvm.L.fj_inject_join() == 0
    w = O.fold(np.zeros(L), a) + O.fold(np.zeros(L), r)
    assert jvm.data(out, np.uint8).tobytes() == O.be_encode(w), "commit_update bytes not torn"
    assert lib.ipls_agg_read(hv, 1, N.TGT_WEIGHTS, got.ctypes.data, L, N.HOST_F64) == 0
    assert_bits_equal(got, w_new, "W after the second thread's set_weights")
    jvm.call("close", h)


@pytest.mark.gpu
def test_jni_update_gradient_owned_subset(jvm, gpu, O):
    """updateGradient(double[], owned) copies only the owned partitions'
    slices out of the heap (the library reads nothing else): owned {1, 3} of
    4 folds exactly those partitions' values, and leaves 0 and 2 at zero; the
    second update arrives as Middleware task 2's big-endian bytes in a direct
    buffer (updateGradientDirect); a vector one value too long is still
    ArrayIndexOutOfBoundsException for the whole call (OrganizeGradients
    checks every partition)."""
    M, P = 40009, 4
    h = _open(jvm, M, P)
    flats = [O.synth_bucket(M, 9, k) for k in range(2)]
    _, exc = jvm.call("updateGradient", h, jvm.doubles(flats[0]), jvm.ints([1, 3]))
    assert exc is None
    # Middleware task 2 without the List<Double>: the second update's BE bytes
    # in a direct buffer at position 8 (updateGradientDirect, HOST_BE)
    be = O.be_encode(flats[1])
    buf, mem = jvm.direct(8 + len(be))
    mem[8:] = np.frombuffer(be, dtype=np.uint8)
    _, exc = jvm.call("updateGradientDirect", h, buf, 8, L64(M), jvm.ints([1, 3]))
    assert exc is None
    _, exc = jvm.call("updateGradient", h, jvm.doubles(np.ones(M + 1)), jvm.ints([1, 3]))
    assert exc == "java/lang/ArrayIndexOutOfBoundsException"
    _, exc = jvm.call("updateGradientDirect", h, buf, 8, L64(M + 1), jvm.ints([1, 3]))
    assert exc == "java/lang/IllegalArgumentException"          # past the buffer: refused by the shim
    parts = [O.organize_gradients(g, M, P) for g in flats]
    for p in range(P):
        L = O.partition_len(M, P, p)
        want = np.zeros(L)
        if p in (1, 3):
            for pt in parts:
                want = O.fold(want, pt[p])
        out = jvm.bytes_(b"\0" * (8 * L))
        _, exc = jvm.call("finalizePartition", h, p, out)
        assert exc is None
        assert jvm.data(out, np.uint8).tobytes() == O.be_encode(want + 0.0), f"W[{p}]"
    jvm.call("close", h)


@pytest.mark.gpu
def test_jni_get_partitions_longer_array(jvm, gpu, O):
    """getPartitions(double[]) into an array longer than the model: the first
    M values are GetPartitions' (IPLS.java:1159-1174), the rest keep what the
    array held (the shim copies nothing in, and back only the model)."""
    M, P = 30011, 3
    h = _open(jvm, M, P)
    w = [O.synth_bucket(O.partition_len(M, P, p), p, 5) for p in range(P)]
    for p in range(P):
        w[p][-1] = float(p + 2)                  # the count slot
    # weights through a round: p's W = its one bucket (count slot included)
    for p in range(P):
        _, exc = jvm.call("accumulate", h, p, 0, jvm.doubles(w[p]))
        assert exc is None
        _, exc = jvm.call("finalizePartition", h, p, None)
        assert exc is None
    arr = jvm.doubles(np.full(M + 3, 7.0))
    _, exc = jvm.call("getPartitions", h, arr)
    assert exc is None
    got = jvm.data(arr, np.float64)
    assert_bits_equal(got[:M], O.get_partitions([0.0 + x for x in w]), "model")
    assert (got[M:] == 7.0).all()
    jvm.call("close", h)


@pytest.mark.gpu
def test_jni_get_partitions_pipelined(jvm, gpu, O):
    """getPartitions(double[]) for a model of >= 2 ring chunks goes through
    ipls_agg_get_partitions_chunked: each chunk is copied into the Java array
    (SetDoubleArrayRegion, from the library's pinned ring) while the next is
    in flight.  The model's bits equal the oracle's, elements past the model
    keep their values, and a short array is still
    ArrayIndexOutOfBoundsException with the array untouched."""
    M, P = 2 * 1048576 + 4099, 2
    h = _open(jvm, M, P)
    g = O.synth_bucket(M, 8, 1)
    _, exc = jvm.call("updateGradient", h, jvm.doubles(g), jvm.ints([0, 1]))
    assert exc is None
    for p in range(P):
        _, exc = jvm.call("finalizePartition", h, p, None)
        assert exc is None
    parts = O.organize_gradients(g, M, P)
    want = O.get_partitions([O.reduce([parts[p]], O.partition_len(M, P, p)) + 0.0 for p in range(P)])
    arr = jvm.doubles(np.full(M + 3, 7.0))
    _, exc = jvm.call("getPartitions", h, arr)
    assert exc is None
    got = jvm.data(arr, np.float64)
    assert_bits_equal(got[:M], want, "model")
    assert (got[M:] == 7.0).all()
    short = jvm.doubles(np.full(M - 1, 5.0))
    _, exc = jvm.call("getPartitions", h, short)
    assert exc == "java/lang/ArrayIndexOutOfBoundsException"
    assert (jvm.data(short, np.float64) == 5.0).all()
    jvm.call("close", h)


@pytest.mark.gpu
def test_jni_exceptions_leave_state_unchanged(jvm, gpu, O):
    """A short bucket is ArrayIndexOutOfBoundsException with nothing folded
    (Updater.java:115-117 would throw mid-loop; the library rejects it first,
    DESIGN.md §1); wrong output sizes are IllegalArgumentException before the
    library writes anything; a bad frame is BufferUnderflowException."""
    M, P = 20003, 2
    h = _open(jvm, M, P)
    g = O.organize_gradients(O.synth_bucket(M, 1, 1), M, P)
    _, exc = jvm.call("accumulate", h, 0, 0, jvm.doubles(g[0]))
    assert exc is None
    _, exc = jvm.call("accumulate", h, 0, 0, jvm.doubles(g[0][:-1]))     # one short
    assert exc == "java/lang/ArrayIndexOutOfBoundsException"
    _, exc = jvm.call("accumulate", h, 5, 0, jvm.doubles(g[0]))          # no partition 5
    assert exc == "java/lang/ArrayIndexOutOfBoundsException"
    _, exc = jvm.call("accumulateFrame", h, 0, 0, jvm.bytes_(b"\0\3\0\0"))
    assert exc == "java/nio/BufferUnderflowException"
    L0 = len(g[0])
    _, exc = jvm.call("finalizePartition", h, 0, jvm.bytes_(b"\0" * (8 * L0 - 1)))
    assert exc == "java/lang/IllegalArgumentException"
    _, exc = jvm.call("aggregateRound", h, 0, P, jvm.doubles(np.zeros(M - 1)))
    assert exc == "java/lang/IllegalArgumentException"
    _, exc = jvm.call("collectReplicas", h, jvm.ints([0]), res=ctypes.c_int32)
    assert exc == "java/lang/IllegalArgumentException"
    _, exc = jvm.call("split", h, jvm.doubles(np.zeros(M)), 1, jvm.doubles(np.zeros(3)))
    assert exc == "java/lang/IllegalArgumentException"
    texts = jvm.objects([jvm.bytes_(O.pubsub_message(O.frame_encode(g[0], 0, 1, 3, b"Q")))] * 2)
    _, exc = jvm.call("ingestTexts", h, 0, texts, 2, None, jvm.ints([0]), res=ctypes.c_int32)
    assert exc == "java/lang/IllegalArgumentException"
    # none of the rejected calls touched AGG[0]: finalize gives exactly the one good fold
    out = jvm.bytes_(b"\0" * (8 * L0))
    _, exc = jvm.call("finalizePartition", h, 0, out)
    assert exc is None and jvm.data(out, np.uint8).tobytes() == O.be_encode(0.0 + g[0])
    # the ingest itself, statuses into a right-sized array
    st = jvm.ints([9, 9])
    n, exc = jvm.call("ingestTexts", h, 0, texts, 2, None, st, res=ctypes.c_int32)
    assert exc is None and n == 2 and list(jvm.data(st, np.int32)) == [0, 0]
    parts_ok = jvm.ints([0, 0])
    n, exc = jvm.call("collectReplicas", h, parts_ok, res=ctypes.c_int32)
    assert exc is None and n == 0
    jvm.call("close", h)


@pytest.mark.gpu
def test_jni_replica_store_drop_and_hashmap_order(jvm, gpu, O):
    """otherReplicaDirect with the Pair hash the Java side computes
    (NativeAggregator.otherReplica), otherReplicaDrop when an aggregator's
    partial arrived, collectReplicas in the HashMap order: REP equals the
    oracle's bit for bit and the counts are the Participants."""
    M, P = 30002, 2
    h = _open(jvm, M, P)
    L = O.partition_len(M, P, 0)
    store = O.ReplicaStore()
    ids = ["12D3KooWQmAlpha", "12D3KooWQmBeta", "12D3KooWQmGamma"]
    for i, (a, k) in enumerate([(0, 1), (1, 2), (2, 3), (0, 4), (2, 5)]):
        g = O.synth_bucket(L, 0, k) * (1e15 if a == 1 else 1.0)
        buf, mem = jvm.direct(8 * L)
        mem[:] = np.frombuffer(O.be_encode(g), dtype=np.uint8)
        kh = O.java_pair_hash(0, ids[a])
        _, exc = jvm.call("otherReplicaDirect", h, 0, a, kh, buf, 0, L64(L))
        assert exc is None
        O.other_replica_add(store, 0, a, g, key_hash=kh)
    r, exc = jvm.call("replicaKeyOrder", h, res=ctypes.c_void_p)
    assert exc is None and [tuple(x) for x in jvm.data(r, np.int32).reshape(-1, 2)] == store.map.keys()
    r, exc = jvm.call("otherReplicaDrop", h, 0, 2, res=ctypes.c_bool)
    assert exc is None and r is True and O.other_replica_drop(store, 0, 2)
    r, exc = jvm.call("otherReplicaDrop", h, 1, 2, res=ctypes.c_bool)
    assert exc is None and r is False
    r, exc = jvm.call("otherReplicaDrop", h, 9, 2, res=ctypes.c_bool)
    assert exc == "java/lang/ArrayIndexOutOfBoundsException"
    rep = [np.zeros(O.partition_len(M, P, p)) for p in range(P)]
    exp = [0, 0]
    n_ref = O.collect_replicas(rep, store, exp)
    parts = jvm.ints([0, 0])
    n, exc = jvm.call("collectReplicas", h, parts, res=ctypes.c_int32)
    assert exc is None and n == n_ref == 2 and list(jvm.data(parts, np.int32)) == exp == [3 * L, 0]
    out = jvm.bytes_(b"\0" * (8 * L))
    _, exc = jvm.call("finalizePartition", h, 0, out)              # W = AGG (+0.0) + REP
    assert exc is None and jvm.data(out, np.uint8).tobytes() == O.be_encode(0.0 + rep[0])
    jvm.call("close", h)


@pytest.mark.gpu
def test_jni_devices_publish_and_device_batches(jvm, gpu, O):
    """openDevices over two shards of one GPU, partitionDevice, the device
    batch natives (reduceBatchDevice / reducePartialDevice / combinePartials)
    and publishPartial == Base64.getUrlEncoder(Marshall_Packet frame)."""
    import torch
    import ipls
    L, P, K = 10_001, 4, 4
    M = P * (L - 1)
    h = _open(jvm, M, P, devices=[0, 0])
    assert [jvm.call("partitionDevice", h, p, res=ctypes.c_int32)[0] for p in range(P)] == [0] * P
    Ls = [jvm.call("partitionLen", h, p, res=ctypes.c_int64)[0] for p in range(P)]
    t = torch.empty(P * K * (max(Ls) + 2), dtype=torch.float64, device="cuda")
    base = (int(t.data_ptr()) + 15) // 16 * 16
    ptr = [[base + 8 * (q * K + k) * (max(Ls) + 2) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(ipls.DeviceBuffer(ptr[q][k], Ls[q]), q, k, O.SEED)
    torch.cuda.synchronize()
    own = [x for q in range(P) for x in ptr[q][:2]]
    _, exc = jvm.call("reduceBatchDevice", h, 0, P, jvm.longs(own), 2, 3, 1, 0)
    assert exc is None
    # slot 1 replicates partitions 0-1, slot 0 partitions 2-3
    _, exc = jvm.call("reducePartialDevice", h, 1, 0, 2, jvm.longs([x for q in (0, 1) for x in ptr[q][2:]]), 2, 3, 1)
    assert exc is None
    _, exc = jvm.call("reducePartialDevice", h, 0, 2, 2, jvm.longs([x for q in (2, 3) for x in ptr[q][2:]]), 2, 3, 1)
    assert exc is None
    n, exc = jvm.call("combinePartials", h, 0, P, res=ctypes.c_int32)
    assert exc is None and n == P
    for q in range(P):
        b = [O.synth_bucket(Ls[q], q, k) for k in range(K)]
        w = O.reduce(b[:2], Ls[q]) + (0.0 + O.reduce(b[2:], Ls[q]))
        text, exc = jvm.call("publishPartial", h, q, 1, 7, 3, 3, jvm.bytes_(b"QmOrigin"), res=ctypes.c_void_p)
        assert exc is None
        assert jvm.data(text, np.uint8).tobytes() == O.java_b64url_encode(
            O.frame_encode(0.0 + O.reduce(b[2:], Ls[q]), 7, 3, 3, b"QmOrigin"))   # REP = +0.0 + R
        out = jvm.bytes_(b"\0" * (8 * Ls[q]))
        _, exc = jvm.call("finalizePartition", h, q, out)
        assert exc is None and jvm.data(out, np.uint8).tobytes() == O.be_encode(w)
    # the round's publish loop in one call (publishPartials): layout, then the
    # texts into a direct buffer; target Weights (what finalize left)
    parts, bs = [3, 0, 2], [5, 9, 1]
    lens, offs = jvm.longs([0] * 3), jvm.longs([0] * 3)
    total, exc = jvm.call("publishPartialsLayout", h, jvm.ints(parts), 8, lens, offs, res=ctypes.c_int64)
    assert exc is None
    L_, O_ = jvm.data(lens, np.int64), jvm.data(offs, np.int64)
    assert total == O_[-1] + L_[-1] and all(o % 64 == 0 for o in O_)
    buf, mem = jvm.direct(int(total))
    _, exc = jvm.call("publishPartialsDirect", h, jvm.ints(parts), 2, 7, jvm.ints(bs), 3, jvm.bytes_(b"QmOrigin"),
                      buf, 0, ctypes.c_int64(int(total)))
    assert exc is None
    for i, q in enumerate(parts):
        single, exc = jvm.call("publishPartial", h, q, 2, 7, bs[i], 3, jvm.bytes_(b"QmOrigin"), res=ctypes.c_void_p)
        assert exc is None
        assert mem[O_[i]:O_[i] + L_[i]].tobytes() == jvm.data(single, np.uint8).tobytes(), q
    # a b[] shorter than the partition list, a buffer too small
    _, exc = jvm.call("publishPartialsDirect", h, jvm.ints(parts), 2, 7, jvm.ints(bs[:2]), 3, None, buf, 0,
                      ctypes.c_int64(int(total)))
    assert exc == "java/lang/IllegalArgumentException"
    small, _ = jvm.direct(16)
    _, exc = jvm.call("publishPartialsDirect", h, jvm.ints(parts), 2, 7, jvm.ints(bs), 3, None, small, 0,
                      ctypes.c_int64(16))
    assert exc == "java/lang/ArrayIndexOutOfBoundsException"
    jvm.call("close", h)
    del t


# Java parameter / return type -> the JNI C type the shim must declare
JNI_TYPES = {"void": "void", "boolean": "jboolean", "byte": "jbyte", "char": "jchar", "short": "jshort",
             "int": "jint", "long": "jlong", "float": "jfloat", "double": "jdouble",
             "boolean[]": "jbooleanArray", "byte[]": "jbyteArray", "short[]": "jshortArray", "int[]": "jintArray",
             "long[]": "jlongArray", "float[]": "jfloatArray", "double[]": "jdoubleArray",
             "String": "jstring", "Class": "jclass"}


def _jni_type(t):
    t = t.strip()
    if t in JNI_TYPES:
        return JNI_TYPES[t]
    return "jobjectArray" if t.endswith("[]") else "jobject"   # byte[][], ByteBuffer, any other object


def test_natives_match_the_shim_signatures():
    """Every `native` of NativeAggregator.java has a C definition in the shim
    with the JNI types a JVM will pass: (JNIEnv*, jclass) for a static native,
    then one C parameter per Java parameter of the matching JNI type, and the
    matching return type.  A JVM binds non-overloaded natives by name only, so
    a type mismatch here would not be caught at link time -- it would read
    the wrong registers at run time."""
    import re
    java = (ROOT / "ipls-java-api_amd" / "java" / "NativeAggregator.java").read_text()
    shim = (ROOT / "ipls-java-api_amd" / "jni" / "ipls_jni.c").read_text()
    decls = re.findall(r"private\s+static\s+native\s+([\w\[\]<>.]+)\s+(\w+)\s*\(([^)]*)\)\s*;", java)
    assert len(decls) == len(set(re.findall(r"\bnative\s+[\w\[\]<>.]+\s+(\w+)\s*\(", java))), "unparsed natives"
    defs = {m.group(2): (m.group(1), m.group(3)) for m in
            re.finditer(r"JNIEXPORT\s+(\w+)\s+JNICALL\s+Java_NativeAggregator_(\w+)\s*\(([^)]*)\)", shim)}
    bad = []
    for ret, name, params in decls:
        if name not in defs:
            bad.append(f"{name}: no C definition")
            continue
        cret, cparams = defs[name]
        cps = [" ".join(p.split()) for p in cparams.split(",")]
        if cret != _jni_type(ret):
            bad.append(f"{name}: returns {cret}, Java {ret} needs {_jni_type(ret)}")
        if len(cps) < 2 or not cps[0].startswith("JNIEnv *") or not cps[1].startswith("jclass"):
            bad.append(f"{name}: must start (JNIEnv *env, jclass cls), has {cps[:2]}")
            continue
        jps = [p for p in (x.strip() for x in params.split(",")) if p]
        if len(jps) != len(cps) - 2:
            bad.append(f"{name}: {len(jps)} Java parameters, {len(cps) - 2} C parameters")
            continue
        for jp, cp in zip(jps, cps[2:]):
            jt = jp.rsplit(None, 1)[0]
            ct = cp.rsplit(None, 1)[0].replace(" *", "*")
            if ct != _jni_type(jt):
                bad.append(f"{name}: Java '{jp}' passed as C '{cp}' (needs {_jni_type(jt)})")
    assert not bad, bad


def test_shim_under_asan():
    """The shim's own host work (array pinning and release, length and
    direct-buffer checks, local-reference reservation, exception mapping)
    under AddressSanitizer + UndefinedBehaviorSanitizer: tests/jni/asan_driver.c
    with the fake JVM and the shim instrumented, linked to the uninstrumented
    libipls_agg.so (host code only: no device compute, a GPU-less open fails
    as expected)."""
    import os
    BUILD.mkdir(parents=True, exist_ok=True)
    exe = BUILD / "asan_driver"
    subprocess.run(["gcc", "-std=c11", "-O1", "-g", "-Wall", "-Wextra", "-Werror",
                    "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all",
                    "-DIPLS_JNI_CALL_HOOK=fj_library_call",
                    f"-I{ROOT / 'tests' / 'jni'}", f"-I{ROOT / 'include'}",
                    str(ROOT / "tests" / "jni" / "asan_driver.c"), str(ROOT / "tests" / "jni" / "fake_jvm.c"),
                    str(ROOT / "ipls-java-api_amd" / "jni" / "ipls_jni.c"),
                    f"-L{AGG}", "-lipls_agg", f"-Wl,-rpath,{AGG}", "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "0 failure(s)" in r.stdout, r.stdout + r.stderr[-2000:]
