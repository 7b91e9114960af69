#!/usr/bin/env python3
"""Fused round (ipls_agg_aggregate_round, k_round) on few partitions: the
fused round on its big/mid shapes (the IPLS_HALF_ROUND=0 build) against the
512-lane half shape (the shipped library), same process, same buckets,
interleaved; averages into device memory; bit-identity of W and the
averages checked between the two.  Algorithmic bytes (K+2)*L*8 per partition
(K buckets read, W and the averages written).
Usage: half_round_probe.py [REPS]   (needs make -C ipls-java-api_amd variants)"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ipls  # noqa: E402
from ipls import _native as N  # noqa: E402


def run(P, L, K, be, reps):
    elem = (L + 1) // 2 * 2 + 32      # every bucket 16-B aligned (the vector path)
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L, big_endian=be) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], q, k, ipls.SEED)
    torch.cuda.synchronize()
    libs = {"big_mid_round": N.load(N.PKG_ROOT / "lib" / "ab" / "libipls_agg_nohalfround.so"), "half_round": None}
    aggs = {nm: ipls.Aggregator(n_partitions=P, bucket_len=L, library=lb) for nm, lb in libs.items()}
    outs = {nm: torch.empty(P * (L - 1) + 2, dtype=torch.float64, device="cuda") for nm in libs}
    ms = {nm: [] for nm in libs}
    shape = {}
    for r in range(reps):
        for nm, agg in aggs.items():
            st = torch.cuda.ExternalStream(agg.stream)
            ob = ipls.DeviceBuffer.from_tensor(outs[nm])
            agg.aggregate_round(0, rows, big_endian=be, out=ob)
            agg.sync()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(5):
                agg.aggregate_round(0, rows, big_endian=be, out=ob)
            e1.record(st)
            agg.sync()
            ms[nm].append(e0.elapsed_time(e1) / 5)
            shape[nm] = agg.last_launch()["shape"]
    same = bool(torch.equal(outs["big_mid_round"].view(torch.int64), outs["half_round"].view(torch.int64))) and all(
        np.array_equal(aggs["big_mid_round"].read(q, ipls.TGT_WEIGHTS).view(np.uint64),
                       aggs["half_round"].read(q, ipls.TGT_WEIGHTS).view(np.uint64)) for q in (0, P - 1))
    nbytes = P * (K + 2) * L * 8
    res = {"P": P, "L": L, "K": K, "be": be, "bit_identical": same}
    for nm in libs:
        m = float(np.median(ms[nm]))
        res[nm] = {"ms": round(m, 4), "frac": round(nbytes / m / 1e6 / 8000, 4), "shape": shape[nm]}
        aggs[nm].close()
    del arena, outs
    torch.cuda.empty_cache()
    return res


if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    for P, L, be in ((1, 4194304, False), (2, 4194304, False), (3, 4194304, False), (5, 4194304, False),
                     (7, 4194304 + 5, False), (3, 4194304, True), (16, 1048576, False)):
        print(json.dumps(run(P, L, 32 if L > 2 * 1048576 else 8, be, reps)), flush=True)
