#!/usr/bin/env python3
"""Dev probe: what the chunked calls' pipeline itself moves, with a caller
that does (almost) nothing -- so the JNI heap natives' rates (DESIGN.md
§5.2) can be split into the library's staging pipeline and the caller's
copies.  One partition of L doubles:
  accumulate_chunked   source returns at once (the ring slot's old bytes are
                       folded: only the H2D pipeline and the fold are timed)
  finalize_chunked     sink returns at once (AggregatePartition, the snapshot
                       and the D2H pipeline)
  get_partitions_wire_chunked  the same for the divide's stream
each at chunk sizes 2^19 .. 2^22 values, and the direct (pinned) forms beside
them.  GB/s = 8 L / wall time per call, median of reps.
Usage: chunk_probe.py [L] [reps] [--ab]   (--ab: one vs two copy streams, interleaved)"""
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "ipls-java-api_amd")]
import ipls  # noqa: E402
from ipls import _native as N  # noqa: E402

_args = [a for a in sys.argv[1:] if not a.startswith("--")]
L = int(_args[0]) if len(_args) > 0 else 4194304
reps = int(_args[1]) if len(_args) > 1 else 20


def timed(fn):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def ab():
    """One vs two copy streams per stage in ONE process, interleaved rep by
    rep (a stage reads IPLS_STAGE_STREAMS when it is first used): two
    handles, the first's stages with one stream, the second's with two."""
    import os
    src = N.CHUNK_SOURCE(lambda ctx, dst, off, n: 0)
    sink = N.CHUNK_SINK(lambda ctx, vals, off, n: 0)
    hs = {}
    for s in ("1", "2"):
        os.environ["IPLS_STAGE_STREAMS"] = s
        a = ipls.Aggregator(n_partitions=1, bucket_len=L)
        assert a._lib.ipls_agg_finalize_chunked(a._h, 0, N.HOST_BE, 1 << 19, sink, None) == 0   # its stage
        hs[s] = a
    out = {"L": L, "reps": reps, "mode": "ab, interleaved in one process"}
    for chunk in (1 << 19, 1 << 20, 1 << 21):
        ops = {
            "accumulate_chunked": lambda a: (a._lib.ipls_agg_accumulate_chunked(a._h, 0, N.TGT_AGG, L, N.HOST_F64,
                                                                                chunk, src, None), a.sync()),
            "finalize_chunked": lambda a: a._lib.ipls_agg_finalize_chunked(a._h, 0, N.HOST_BE, chunk, sink, None),
            "get_partitions_wire_chunked": lambda a: a._lib.ipls_agg_get_partitions_wire_chunked(a._h, chunk, sink,
                                                                                                None),
        }
        row = {}
        for name, fn in ops.items():
            ts = {"1": [], "2": []}
            for _ in range(reps):
                for s in ("1", "2"):
                    t0 = time.perf_counter()
                    fn(hs[s])
                    ts[s].append(time.perf_counter() - t0)
            row[name] = {f"streams_{s}": round(8 * L / float(np.median(v)) / 1e9, 2) for s, v in ts.items()}
        out[f"chunk_{chunk}"] = row
    for a in hs.values():
        a.close()
    print(json.dumps(out))


def main():
    if "--ab" in sys.argv:
        return ab()
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L)
    lib, h = agg._lib, agg._h
    src = N.CHUNK_SOURCE(lambda ctx, dst, off, n: 0)
    sink = N.CHUNK_SINK(lambda ctx, vals, off, n: 0)
    pin = ipls.PinnedBuffer(8 * L)
    pin.view()[:] = 0
    out = {"L": L, "reps": reps}
    for chunk in (1 << 19, 1 << 20, 1 << 21, 1 << 22):
        row = {}

        def acc():
            assert lib.ipls_agg_accumulate_chunked(h, 0, N.TGT_AGG, L, N.HOST_F64, chunk, src, None) == 0
            agg.sync()
        row["accumulate_chunked"] = timed(acc)

        def fin():
            assert lib.ipls_agg_finalize_chunked(h, 0, N.HOST_BE, chunk, sink, None) == 0
        row["finalize_chunked"] = timed(fin)

        def gp():
            assert lib.ipls_agg_get_partitions_wire_chunked(h, chunk, sink, None) == 0
        row["get_partitions_wire_chunked"] = timed(gp)
        out[f"chunk_{chunk}"] = {k: round(8 * L / v / 1e9, 2) for k, v in row.items()}

    def acc_direct():
        assert lib.ipls_agg_accumulate(h, 0, N.TGT_AGG, pin.ptr, L, N.HOST_BE) == 0
        agg.sync()

    def fin_direct():
        assert lib.ipls_agg_finalize(h, 0, ctypes.c_void_p(pin.ptr), N.HOST_BE, None) == 0
    out["direct"] = {"accumulate_pinned": round(8 * L / timed(acc_direct) / 1e9, 2),
                     "finalize_pinned": round(8 * L / timed(fin_direct) / 1e9, 2)}
    pin.close()
    agg.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
