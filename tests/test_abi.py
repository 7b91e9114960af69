"""CPU-only: the C-ABI library builds, loads, and exports every symbol that
include/ipls_agg.h declares (no device compute here), plus the host-only
frame codec entry points and the no-GPU error path."""
import ctypes
import re

import numpy as np
import pytest

from conftest import ROOT


def declared_symbols():
    text = (ROOT / "include" / "ipls_agg.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ipls_\w+)\s*\(", text)))


def test_header_declares_expected_surface():
    syms = declared_symbols()
    for s in ["ipls_agg_open", "ipls_agg_close", "ipls_agg_reduce_batch", "ipls_agg_accumulate",
              "ipls_agg_finalize", "ipls_agg_get_partitions", "ipls_agg_last_error"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    import ipls
    from ipls import _native as N
    L = ipls.lib()
    for s in declared_symbols():
        assert hasattr(L, s), f"{s} declared in include/ipls_agg.h but not exported"
        assert s in N.SIGNATURES, f"{s} has no ctypes signature"
    assert L.ipls_agg_abi_version() == N.ABI_VERSION == 4


def test_header_constants_match_binding():
    from ipls import _native as N
    text = (ROOT / "include" / "ipls_agg.h").read_text()
    defs = dict((m.group(1), int(m.group(2))) for m in re.finditer(r"#define\s+(IPLS_\w+)\s+\(?(-?\d+)\)?", text))
    assert defs["IPLS_TGT_AGG"] == N.TGT_AGG and defs["IPLS_TGT_REP"] == N.TGT_REP
    assert defs["IPLS_HOST_F64"] == N.HOST_F64 and defs["IPLS_HOST_BE"] == N.HOST_BE
    assert defs["IPLS_HOST_FRAME"] == N.HOST_FRAME and defs["IPLS_DEV_F64"] == N.DEV_F64
    assert defs["IPLS_DEV_BE"] == N.DEV_BE and defs["IPLS_HOST_BE_CANON"] == N.HOST_BE_CANON
    assert defs["IPLS_START_ZERO"] == N.START_ZERO and defs["IPLS_START_FIRST"] == N.START_FIRST
    assert defs["IPLS_E_RANGE"] == N.IPLS_E_RANGE and defs["IPLS_E_NODEV"] == N.IPLS_E_NODEV
    assert defs["IPLS_ALL_PARTITIONS"] == N.ALL_PARTITIONS
    assert ctypes.sizeof(N.AggCfg) == 56
    assert ctypes.sizeof(N.LaunchInfo) == 48
    assert defs["IPLS_HOST_TEXT"] == N.HOST_TEXT and defs["IPLS_DEV_TEXT"] == N.DEV_TEXT
    assert defs["IPLS_SHAPE_BIG"] == N.SHAPE_BIG and defs["IPLS_KERNEL_ROUND"] == N.KERNEL_ROUND
    for nm in ("SHAPE_MID", "SHAPE_SMALL", "SHAPE_HALF", "KERNEL_REDUCE", "KERNEL_FOLD1", "KERNEL_REDUCE_SCALAR"):
        assert defs["IPLS_" + nm] == getattr(N, nm), nm
    # ipls_launch_info: the last int32 is `staged` (was `reserved`), layout unchanged
    assert [f for f, _ in N.LaunchInfo._fields_][-1] == "staged"
    assert re.search(r"int32_t\s+staged;", text)


def test_library_is_gfx950_code_object():
    """The .so carries a gfx950 device code object (hipcc cross-compiled)."""
    from ipls import _native as N
    data = N.LIB_PATH.read_bytes()
    assert b"gfx950" in data


def test_frame_codec_host_entry_points():
    import ipls
    from oracle import oracle as O
    g = np.array([1.5, -2.25, 3.0])
    fr = ipls.frame_encode(g, 5, 9, 3, b"QmOrigin")
    assert fr == O.frame_encode(g, 5, 9, 3, b"QmOrigin")
    assert ipls.frame_parse(fr) == (3, 3, 5, 9, 14, 38)
    with pytest.raises(ipls.IplsError) as e:
        ipls.frame_parse(fr[:13])
    assert e.value.java_name == "BufferUnderflow"
    with pytest.raises(ipls.IplsError):
        ipls.frame_parse(fr[:30])


def test_open_without_gpu_fails_loudly():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import ipls
    with pytest.raises(ipls.IplsError) as e:
        ipls.Aggregator(443610, 3)
    assert e.value.java_name == "NoDevice"


def test_jni_shim_matches_java_natives():
    """The JNI shim against NativeAggregator.java (every native has its
    Java_NativeAggregator_* function and no function is orphaned) and
    include/ipls_agg.h (every ipls_* it calls is declared).  tests/test_jni.py
    compiles and drives it."""
    import re
    pkg = ROOT / "ipls-java-api_amd"
    java = (pkg / "java" / "NativeAggregator.java").read_text()
    jni = (pkg / "jni" / "ipls_jni.c").read_text()
    natives = set(re.findall(r"\bnative\s+[\w\[\]<>.]+\s+(\w+)\s*\(", java))
    exported = set(re.findall(r"JNICALL\s+Java_NativeAggregator_(\w+)\s*\(", jni))
    assert natives and natives == exported, (natives ^ exported)
    header = (ROOT / "include" / "ipls_agg.h").read_text()
    declared = set(re.findall(r"\b(ipls_\w+)\s*\(", header))
    called = set(re.findall(r"\b(ipls_\w+)\s*\(", jni))
    assert called <= declared, called - declared


def test_null_handle_fails_cleanly():
    """Every entry point that takes a handle returns a negative code for a
    NULL one (the Java caller's closed/never-opened aggregator), without
    touching a GPU or crashing."""
    import ipls
    from ipls import _native as N
    L = ipls.lib()
    skipped = {"ipls_agg_open", "ipls_agg_abi_version", "ipls_agg_close", "ipls_agg_last_error", "ipls_agg_stream",
               "ipls_host_alloc", "ipls_host_free", "ipls_synth_fill", "ipls_checksum_dev", "ipls_encode_secure",
               "ipls_frame_parse", "ipls_frame_encode", "ipls_pair_parse", "ipls_pair_encode"}
    checked = 0
    for name, (res, args) in N.SIGNATURES.items():
        if name in skipped or not args or args[0] is not ctypes.c_void_p:
            continue
        vals = [None] + [t() if isinstance(t, type) and issubclass(t, ctypes._SimpleCData) else None for t in args[1:]]
        rc = getattr(L, name)(*vals)
        assert rc < 0, f"{name}(NULL, ...) returned {rc}"
        checked += 1
    assert checked >= 25
    assert L.ipls_agg_close(None) == 0                     # closing nothing is a no-op


@pytest.mark.parametrize("P,G", [(16, 1), (64, 4), (128, 8), (3, 8), (17, 4), (5, 2)])
def test_shard_plan_contiguous_blocks(P, G):
    """-pa segments map to devices in contiguous blocks,
    partition p on shard p / ceil(P/G) (no GPU needed)."""
    import ipls
    per = -(-P // G)
    owner = ipls.shard_plan(P, G)
    assert owner == [p // per for p in range(P)]
    assert owner == sorted(owner) and max(owner) < G
    if P % G == 0:
        assert all(owner.count(s) == P // G for s in range(G))   # 16/GPU in configs E and F


def test_shard_plan_rejects_bad_arguments():
    import ipls
    with pytest.raises(ipls.IplsError):
        ipls.shard_plan(0, 2)
    with pytest.raises(ipls.IplsError):
        ipls.shard_plan(4, 0)


def _prototypes():
    """name -> (return C type, [parameter C types]) of every function include/ipls_agg.h declares."""
    text = (ROOT / "include" / "ipls_agg.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"#.*", "", text)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(ipls_\w+)\s*\(([^)]*)\)\s*;", text):
        ret = " ".join(m.group(1).split())
        params = [" ".join(p.split()) for p in m.group(3).split(",")]
        params = [] if params == ["void"] else params
        out[m.group(2)] = (ret, params)
    return out


def _ctype_of(c, N):
    """The ctypes type a C type must be bound with (pointers: None = any pointer type is checked separately)."""
    c = c.replace("const ", "").strip()
    scalars = {"int": ctypes.c_int, "int32_t": ctypes.c_int32, "int64_t": ctypes.c_int64, "uint64_t": ctypes.c_uint64,
               "int16_t": ctypes.c_int16, "size_t": ctypes.c_size_t, "double": ctypes.c_double}
    if "*" not in c:
        return scalars[c]
    return None


def _pointee(c):
    c = c.replace("const", " ")
    base, stars = c.split("*", 1)[0].strip(), c.count("*")
    return base.split()[-1] if base else base, stars


def test_ctypes_signatures_match_the_header():
    """Every prototype in include/ipls_agg.h against its ctypes binding in
    ipls/_native.py: same parameter count, the same scalar types (an int64_t
    bound as c_int would truncate lengths above 2^31), pointers bound as
    pointers of the right element type, and the same return type."""
    from ipls import _native as N
    protos = _prototypes()
    assert set(protos) == set(N.SIGNATURES), set(protos) ^ set(N.SIGNATURES)
    elem = {"double": ctypes.c_double, "int32_t": ctypes.c_int32, "int64_t": ctypes.c_int64,
            "uint64_t": ctypes.c_uint64, "int16_t": ctypes.c_int16, "ipls_agg_cfg": N.AggCfg,
            "ipls_launch_info": N.LaunchInfo}
    bad = []
    for name, (ret, params) in sorted(protos.items()):
        res, args = N.SIGNATURES[name]
        # return type
        if "*" in ret:
            want = ctypes.c_char_p if "char" in ret else ctypes.c_void_p
            if res is not want:
                bad.append(f"{name}: returns {ret}, bound {res}")
        elif res is not _ctype_of(ret, N):
            bad.append(f"{name}: returns {ret}, bound {res}")
        if len(args) != len(params):
            bad.append(f"{name}: {len(params)} parameters, {len(args)} bound")
            continue
        for i, (c, a) in enumerate(zip(params, args)):
            ctype = re.sub(r"\b\w+$", "", c).strip() if re.search(r"[*\s]\w+$", c) else c   # drop the name
            if ctype in ("ipls_chunk_sink", "ipls_chunk_source"):   # a function pointer: travels as void*
                if a is not ctypes.c_void_p:
                    bad.append(f"{name} arg {i}: C '{c}' bound {a}")
                continue
            if "*" not in ctype:
                if a is not _ctype_of(ctype, N):
                    bad.append(f"{name} arg {i}: C '{c}' bound {a.__name__}")
                continue
            base, stars = _pointee(ctype)
            if a in (ctypes.c_void_p, ctypes.c_char_p):
                continue                                    # any pointer may travel as void*
            inner = getattr(a, "_type_", None)
            if inner is None:
                bad.append(f"{name} arg {i}: C '{c}' bound {a}")
            elif stars >= 2:
                if inner not in (ctypes.c_void_p, ctypes.c_char_p):
                    bad.append(f"{name} arg {i}: C '{c}' (pointer to pointer) bound POINTER({inner.__name__})")
            elif base in elem and inner is not elem[base]:
                bad.append(f"{name} arg {i}: C '{c}' bound POINTER({inner.__name__})")
    assert not bad, bad


def test_fast_extension_calls_the_bound_library():
    """ipls._fast (csrc/pyfast.c): the per-arrival accumulate calls without
    ctypes.  It is linked against the in-tree library, and ipls uses it only
    when its entry points are the ones ipls._native bound (one mapping of one
    file); a null handle comes back as the library's error code and message,
    bad arguments as Python exceptions before any library call."""
    from ipls import _native as N
    fast = N.fast()
    assert fast is not None, "ipls._fast not built (make -C ipls-java-api_amd)"
    L = N.lib()
    assert fast.entry_points() == (ctypes.cast(L.ipls_agg_accumulate_async, ctypes.c_void_p).value,
                                   ctypes.cast(L.ipls_agg_accumulate, ctypes.c_void_p).value)
    for call in (fast.accumulate_async, fast.accumulate):
        rc = call(None, 0, N.TGT_AGG, 0, 0, N.DEV_F64)
        assert rc == N.IPLS_E_INVAL and "null" in N.last_error(None)
        with pytest.raises(TypeError):
            call(None, 0, N.TGT_AGG, 0, 0)
        with pytest.raises(OverflowError):
            call(None, 2 ** 40, N.TGT_AGG, 0, 0, N.DEV_F64)
        with pytest.raises(TypeError):
            call(None, 0, N.TGT_AGG, "not an address", 0, N.DEV_F64)
