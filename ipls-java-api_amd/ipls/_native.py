"""ctypes binding of libipls_agg.so (include/ipls_agg.h).

This is the Python twin of the JNI shim in INTEGRATION.md: one Python call
per C entry point, plain pointers and sizes.  There is no fallback: if the
library is missing or a call fails, an exception is raised (the product path
never computes on the CPU).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent          # ipls-java-api_amd/
LIB_PATH = Path(os.environ.get("IPLS_AGG_LIB", PKG_ROOT / "lib" / "libipls_agg.so"))
HEADER = PKG_ROOT.parent / "include" / "ipls_agg.h"

# ---- constants (mirrors include/ipls_agg.h) ----
IPLS_OK = 0
IPLS_E_INVAL, IPLS_E_RANGE, IPLS_E_NEGSIZE, IPLS_E_NOMEM = -1, -2, -3, -4
IPLS_E_DEVICE, IPLS_E_FORMAT, IPLS_E_NODEV = -5, -6, -7

TGT_AGG, TGT_REP, TGT_WEIGHTS, TGT_WADDR, TGT_FUTURE = 0, 1, 2, 3, 4
HOST_F64, HOST_BE, HOST_FRAME, DEV_F64, DEV_BE, HOST_BE_CANON, HOST_PAIR = 0, 1, 2, 3, 4, 5, 6
HOST_TEXT, DEV_TEXT = 7, 8
KERNEL_REDUCE, KERNEL_ROUND, KERNEL_FOLD1, KERNEL_REDUCE_SCALAR = 1, 2, 3, 4
SHAPE_BIG, SHAPE_MID, SHAPE_SMALL, SHAPE_HALF = 1, 2, 3, 4
ABI_VERSION = 4
START_ACCUM, START_ZERO, START_FIRST = 0, 1, 2
ALL_PARTITIONS = -1

# ipls_chunk_sink: int (*)(void *ctx, const double *values, int64_t offset, int64_t n)
CHUNK_SINK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int64,
                              ctypes.c_int64)
# ipls_chunk_source: int (*)(void *ctx, void *dst, int64_t offset, int64_t n)
CHUNK_SOURCE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64)

ERROR_NAMES = {
    IPLS_E_INVAL: "IllegalArgument",
    IPLS_E_RANGE: "ArrayIndexOutOfBounds",
    IPLS_E_NEGSIZE: "NegativeArraySize",
    IPLS_E_NOMEM: "OutOfMemory",
    IPLS_E_DEVICE: "DeviceError",
    IPLS_E_FORMAT: "BufferUnderflow",
    IPLS_E_NODEV: "NoDevice",
}


class IplsError(RuntimeError):
    """A negative return code from the C-ABI (the Java exception it stands for
    is in ``java_name``)."""

    def __init__(self, code: int, msg: str):
        self.code = code
        self.java_name = ERROR_NAMES.get(code, "Error")
        super().__init__(f"[{code} {self.java_name}] {msg}")


class AggCfg(ctypes.Structure):
    _fields_ = [
        ("model_size", ctypes.c_int64),
        ("n_partitions", ctypes.c_int32),
        ("max_peers", ctypes.c_int32),
        ("partial_aggregation", ctypes.c_int32),
        ("secure", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("bucket_len", ctypes.c_int64),
        ("devices", ctypes.POINTER(ctypes.c_int32)),
        ("n_devices", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class LaunchInfo(ctypes.Structure):
    _fields_ = [
        ("kernel", ctypes.c_int32), ("shape", ctypes.c_int32), ("block", ctypes.c_int32),
        ("vectors", ctypes.c_int32), ("seqf", ctypes.c_int32), ("map", ctypes.c_int32),
        ("grid", ctypes.c_int64),
        ("be_in", ctypes.c_int32), ("be_out", ctypes.c_int32), ("start", ctypes.c_int32),
        ("staged", ctypes.c_int32),
    ]


# name -> (restype, argtypes); every symbol declared in include/ipls_agg.h
_vp, _i, _i64, _u64, _i32, _i16 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int16
_P = ctypes.POINTER
SIGNATURES = {
    "ipls_agg_abi_version": (_i, []),
    "ipls_agg_open": (_i, [_P(AggCfg), _P(_vp)]),
    "ipls_agg_close": (_i, [_vp]),
    "ipls_agg_last_error": (ctypes.c_char_p, [_vp]),
    "ipls_agg_partition_len": (_i, [_vp, _i, _P(_i64)]),
    "ipls_agg_partition_offset": (_i, [_vp, _i, _P(_i64)]),
    "ipls_agg_load_model": (_i, [_vp, _vp, _i64, _i]),
    "ipls_agg_split": (_i, [_vp, _vp, _i64, _i, _i, _vp, _i]),
    "ipls_agg_update_gradient": (_i, [_vp, _vp, _i64, _i, _P(_i32), _i]),
    "ipls_agg_accumulate": (_i, [_vp, _i, _i, _vp, _i64, _i]),
    "ipls_agg_reduce_batch": (_i, [_vp, _i, _i, _P(_vp), _i, _i, _i, _i]),
    "ipls_agg_reduce_batch_out": (_i, [_vp, _i, _i, _P(_vp), _i, _i, _i, _P(_vp), _i]),
    "ipls_agg_aggregate_round": (_i, [_vp, _i, _i, _P(_vp), _i, _i, _vp, _i]),
    "ipls_agg_promote_future": (_i, [_vp, _P(ctypes.c_int32), _i]),
    "ipls_agg_update_indirect": (_i, [_vp, _i, _i, _vp, _i64]),
    "ipls_agg_accumulate_async": (_i, [_vp, _i, _i, _vp, _i64, _i, _P(_u64)]),
    "ipls_agg_accumulate_range": (_i, [_vp, _i, _i, _vp, _i64, _i64, _i, _P(_u64)]),
    "ipls_agg_read_range": (_i, [_vp, _i, _i, _vp, _i64, _i64, _i, _P(_u64)]),
    "ipls_agg_flat_size": (_i, [_vp, _P(_i64)]),
    "ipls_agg_get_partitions_chunked": (_i, [_vp, _i64, _vp, _vp]),   # sink: a CHUNK_SINK instance
    "ipls_agg_get_partitions_wire_chunked": (_i, [_vp, _i64, _vp, _vp]),   # sink: a CHUNK_SINK instance
    "ipls_agg_accumulate_chunked": (_i, [_vp, _i, _i, _i64, _i, _i64, _vp, _vp]),   # source: a CHUNK_SOURCE
    "ipls_agg_finalize_chunked": (_i, [_vp, _i, _i, _i64, _vp, _vp]),   # sink: a CHUNK_SINK instance
    "ipls_agg_wait": (_i, [_vp, _u64]),
    "ipls_agg_set_coalesce": (_i, [_vp, _i]),
    "ipls_agg_flush": (_i, [_vp]),
    "ipls_agg_other_replica": (_i, [_vp, _i, _i32, _vp, _i64, _i]),
    "ipls_agg_other_replica_keyed": (_i, [_vp, _i, _i32, _i32, _vp, _i64, _i]),
    "ipls_agg_other_replica_drop": (_i, [_vp, _i, _i32]),
    "ipls_java_pair_hash": (_i, [_i32, _vp, _i64, _P(_i32)]),
    "ipls_agg_replica_order": (_i, [_vp, _P(_i32), _i, _P(_i32)]),
    "ipls_agg_collect_replicas": (_i, [_vp, _P(_i32)]),
    "ipls_agg_ingest_pubsub": (_i, [_vp, _i, _P(_vp), _P(_i64), _i, _i, _P(_i32), _P(_i32)]),
    "ipls_agg_blend": (_i, [_vp, _i, _i, _vp, _i64, _i, ctypes.c_double, ctypes.c_double]),
    "ipls_agg_scale": (_i, [_vp, _i, _i, _i, ctypes.c_double]),
    "ipls_agg_finalize": (_i, [_vp, _i, _vp, _i, _P(ctypes.c_double)]),
    "ipls_agg_set_weights": (_i, [_vp, _i, _vp, _i64, _i]),
    "ipls_agg_get_partitions": (_i, [_vp, _vp, _i64, _i]),
    "ipls_agg_read": (_i, [_vp, _i, _i, _vp, _i64, _i]),
    "ipls_agg_reset": (_i, [_vp, _i]),
    "ipls_agg_device_ptr": (_i, [_vp, _i, _i, _P(_vp)]),
    "ipls_agg_stream": (_vp, [_vp]),
    "ipls_agg_sync": (_i, [_vp]),
    "ipls_agg_checksum": (_i, [_vp, _i, _i, _P(_u64)]),
    "ipls_host_alloc": (_i, [ctypes.c_size_t, _P(_vp)]),
    "ipls_host_free": (_i, [_vp]),
    "ipls_synth_fill": (_i, [_vp, _i64, _u64, _i, _i, _i, _vp]),
    "ipls_checksum_dev": (_i, [_vp, _i64, _i, _P(_u64), _vp]),
    "ipls_encode_secure": (_i, [_vp, _vp, _i64, _i, _i, _vp]),
    "ipls_frame_parse": (_i64, [_vp, _i64, _P(_i16), _P(_i32), _P(_i32), _P(_i64), _P(_i64)]),
    "ipls_frame_encode": (_i64, [_vp, _i64, _i, _i32, _i32, _i16, _vp, _i32, _vp, _i64]),
    "ipls_pair_parse": (_i64, [_vp, _i64, _P(_i32), _P(_i64)]),
    "ipls_pair_encode": (_i64, [_i32, _vp, _i64, _i, _vp, _i64]),
    "ipls_agg_commit_partial": (_i64, [_vp, _i, _i32, _vp, _i64]),
    "ipls_agg_merge_files": (_i64, [_vp, _P(_vp), _P(_i64), _i, _i, _vp, _i64]),
    "ipls_agg_partition_device": (_i, [_vp, _i, _P(_i32), _P(_vp)]),
    "ipls_shard_plan": (_i, [_i32, _i32, _P(_i32)]),
    "ipls_agg_reduce_partial": (_i, [_vp, _i, _i, _i, _P(_vp), _i, _i, _i]),
    "ipls_agg_combine_partials": (_i, [_vp, _i, _i]),
    "ipls_agg_publish_partial": (_i64, [_vp, _i, _i, _i32, _i32, _i16, _vp, _i32, _vp, _i64, _i]),
    "ipls_agg_publish_partials": (_i64, [_vp, _vp, _i, _i, _i32, _vp, _i16, _vp, _i32, _vp, _i64, _i, _vp, _vp]),
    "ipls_agg_last_launch": (_i, [_vp, _P(LaunchInfo)]),
}

_lib = None


def load(path) -> ctypes.CDLL:
    """Load and bind one build of the library (every symbol of the header)."""
    if not Path(path).exists():
        raise ImportError(
            f"{path} not found: build it with `make -C ipls-java-api_amd` "
            "(or __graft_entry__.build()); the aggregator has no CPU fallback")
    L = ctypes.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib() -> ctypes.CDLL:
    """Load the in-tree HIP library.  Raises if it has not been built --
    there is deliberately no CPU path behind this package."""
    global _lib
    if _lib is None:
        # Load order with torch: a process that uses torch as well
        # must import torch BEFORE the first call that loads this library --
        # torch's bundled HIP runtime has to be the process's runtime before
        # the library's link to /opt/rocm's is resolved; in the other order the
        # library finds "no HIP device available" (tools/jni_open_probe.py,
        # profiles/r04/i/).  The entry points that mix the two do so
        # (tests/conftest.py, bench.py, the tools); a caller without torch
        # pays no torch import here.
        _lib = load(LIB_PATH)
    return _lib


_fast = None


def fast():
    """ipls._fast (csrc/pyfast.c: the per-arrival accumulate calls without
    ctypes) when it calls the very library lib() bound -- the in-tree build,
    one mapping of one file, checked by comparing entry-point addresses --
    else None, and the callers use the ctypes binding of the same library."""
    global _fast
    if _fast is None:
        _fast = False
        if LIB_PATH == PKG_ROOT / "lib" / "libipls_agg.so":
            try:
                from . import _fast as m
            except ImportError:
                m = None
            if m is not None:
                L = lib()
                mine = (ctypes.cast(L.ipls_agg_accumulate_async, ctypes.c_void_p).value,
                        ctypes.cast(L.ipls_agg_accumulate, ctypes.c_void_p).value)
                if m.entry_points() == mine:
                    _fast = m
    return _fast or None


def build_info() -> dict:
    """Provenance of the library this process loads: its sha256 now, and the
    build stamp written next to it at link time (tools/build_stamp.py: git
    revision, whether the library's sources differed from it, kernel-source
    sha256).  `stamp_matches_so` is False when the .so was replaced after the
    stamp was written."""
    import hashlib
    import json
    h = hashlib.sha256()
    with open(LIB_PATH, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    info = {"so": LIB_PATH.name, "so_sha256": h.hexdigest()}
    stamp = LIB_PATH.with_name(LIB_PATH.name + ".buildinfo.json")
    try:
        rec = json.loads(stamp.read_text())
    except (OSError, ValueError):
        rec = None
    if rec is None:
        info.update(git_rev=None, sources_dirty=None, kernel_src_sha256=None, stamp_matches_so=None)
    else:
        info.update(git_rev=rec.get("git_rev"), sources_dirty=rec.get("sources_dirty"),
                    kernel_src_sha256=rec.get("kernel_src_sha256"), built_utc=rec.get("built_utc"),
                    stamp_matches_so=rec.get("so_sha256") == info["so_sha256"])
        # the library's sources travel with the tree: recompute their hash here
        # and compare it with the one recorded at link time
        try:
            import importlib.util
            root = LIB_PATH.resolve().parent.parent.parent
            spec = importlib.util.spec_from_file_location("_ipls_build_stamp", root / "tools" / "build_stamp.py")
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            now = mod.lib_src_sha256(root)
            info["lib_src_sha256"] = rec.get("lib_src_sha256")
            info["device_code_sha256"] = mod.device_code_sha256(LIB_PATH)
            info["sources_match"] = rec.get("lib_src_sha256") == now if rec.get("lib_src_sha256") else None
        except Exception as e:   # noqa: BLE001 -- provenance never costs the caller
            info["sources_match"] = None
            info["sources_match_error"] = f"{type(e).__name__}: {e}"
    return info


def last_error(h=None) -> str:
    msg = lib().ipls_agg_last_error(h)
    return msg.decode(errors="replace") if msg else ""


def check(rc: int, h=None) -> int:
    if rc < 0:
        # this thread's failure: another thread may already have failed on h since
        raise IplsError(rc, last_error(None))
    return rc
