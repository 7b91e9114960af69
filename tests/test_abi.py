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
    assert L.ipls_agg_abi_version() == N.ABI_VERSION == 2


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
