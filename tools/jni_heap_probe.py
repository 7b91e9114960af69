"""Dev probe: what a heap-array native costs against the direct-buffer one,
through the JNI shim and the fake JVM (tests/jni/fake_jvm.c) on the GPU box.
One partition of L doubles (one bucket per call, as the Updater folds):
  accumulate(double[])         -- one ipls_agg_accumulate_chunked call: the library
                                  pulls the array chunk by chunk (the shim's
                                  GetDoubleArrayRegion source) into its pinned ring,
                                  each chunk sent while the next is copied, one fold
  accumulateDirect(ByteBuffer) -- a hostAlloc direct buffer, zero copy
  finalizePartition(byte[])    -- one ipls_agg_finalize_chunked call:
                                  AggregatePartition, then the BE sum back in ring
                                  chunks, each copied into the byte[] (the shim's
                                  SetByteArrayRegion sink) while the next arrives
  finalizePartitionDirect      -- the BE sum straight into a direct buffer
  getPartitions(double[])      -- GetPartitions (the divide) into a heap double[]
  getPartitionsWire(ByteBuffer)-- the same as Middleware's big-endian stream into
                                  a pinned direct buffer
GB/s = bytes of the Java-side array / wall time per call (median of reps).
Usage: jni_heap_probe.py [L] [reps] [--ab-slots=2,3,4]
(--ab-slots: the stage ring depth, one handle per value, interleaved in one process)"""
import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd"), str(ROOT / "tests")]
_ring = os.environ.get("IPLS_JNI_RING_CHUNK")   # a sweep's value; test_jni pins its own on import
import test_jni as TJ  # noqa: E402
if _ring is None:
    os.environ.pop("IPLS_JNI_RING_CHUNK", None)   # the shim's defaults (read at its first chunked native)
else:
    os.environ["IPLS_JNI_RING_CHUNK"] = _ring

_pos = [a for a in sys.argv[1:] if not a.startswith("--")]
L = int(_pos[0]) if len(_pos) > 0 else 4194304
reps = int(_pos[1]) if len(_pos) > 1 else 20
_ab = next((a.split("=", 1)[1].split(",") for a in sys.argv[1:] if a.startswith("--ab-slots=")), None)
jvm = TJ.JVM()
L64 = ctypes.c_int64
# one partition of L doubles: model_size = L - 1 (the chunk rule gives L_0 = M + 1)
h, exc = jvm.call("open", L64(L - 1), 1, 3, 0, 0, 0, res=ctypes.c_int64)
assert exc is None and h
h = L64(h)
g = np.random.default_rng(1).standard_normal(L)
arr = jvm.doubles(g)
buf, mem = jvm.direct(8 * L)
mem[:] = np.frombuffer(g.astype(">f8").tobytes(), dtype=np.uint8)
out_heap = jvm.bytes_(b"\0" * (8 * L))
pin_obj, _ = jvm.call("hostAllocDirect", 8 * L, res=ctypes.c_void_p)
pin_obj = ctypes.c_void_p(pin_obj)


def timed(fn):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


if _ab:
    # the stage ring depth, A/B in ONE process: a handle per IPLS_STAGE_SLOTS
    # value (a stage reads it when it is made, at the handle's first chunked
    # call), the heap natives timed rep by rep in turn on each
    model = jvm.doubles(np.zeros(L - 1))
    hs = {}
    for v in _ab:
        os.environ["IPLS_STAGE_SLOTS"] = v
        hv, exc = jvm.call("open", L64(L - 1), 1, 3, 0, 0, 0, res=ctypes.c_int64)
        assert exc is None and hv
        hs[v] = L64(hv)
        for name, args in (("accumulate", (hs[v], 0, 0, arr)), ("finalizePartition", (hs[v], 0, out_heap)),
                           ("getPartitions", (hs[v], model))):
            assert jvm.call(name, *args)[1] is None
    # accumulate(double[]) is not timed here: it returns once its fold is
    # queued, so one handle's copies would run under the other's timed call
    ops = {"finalize_heap_byte[]": lambda hv: jvm.call("finalizePartition", hv, 0, out_heap),
           "getPartitions_heap_double[]": lambda hv: jvm.call("getPartitions", hv, model)}
    out = {"L": L, "reps": reps, "mode": "ab-slots, interleaved in one process"}
    for name, fn in ops.items():
        ts = {v: [] for v in _ab}
        for _ in range(reps):
            for v in _ab:
                t0 = time.perf_counter()
                fn(hs[v])
                ts[v].append(time.perf_counter() - t0)
        out[name] = {f"slots_{v}": round(8 * L / float(np.median(t)) / 1e9, 2) for v, t in ts.items()}
    for hv in hs.values():
        jvm.call("close", hv)
    jvm.call("close", h)
    print(json.dumps(out))
    sys.exit(0)

res = {}
res["accumulate_heap_double[]"] = timed(lambda: jvm.call("accumulate", h, 0, 0, arr))
res["accumulateDirect_pinned_BE"] = timed(lambda: jvm.call("accumulateDirect", h, 0, 0, pin_obj, 0, L64(L), 1))
res["finalize_heap_byte[]"] = timed(lambda: jvm.call("finalizePartition", h, 0, out_heap))
res["finalizeDirect_pinned"] = timed(lambda: jvm.call("finalizePartitionDirect", h, 0, pin_obj, 0))
model = jvm.doubles(np.zeros(L - 1))
res["getPartitions_heap_double[]"] = timed(lambda: jvm.call("getPartitions", h, model))
res["getPartitionsWire_pinned"] = timed(lambda: jvm.call("getPartitionsWire", h, pin_obj, 0, L64(8 * (L - 1))))
jvm.call("close", h)
print(json.dumps({"L": L, "bytes_per_call": 8 * L, "reps": reps,
                  "copy_threads": os.environ.get("IPLS_JNI_COPY_THREADS", "6 (default)"),
                  "ring_chunk": os.environ.get("IPLS_JNI_RING_CHUNK", "default: 2097152 in, 524288 out"),
                  **{k: {"ms": round(v * 1e3, 3), "GBps": round(8 * L / v / 1e9, 2)} for k, v in res.items()}}))
