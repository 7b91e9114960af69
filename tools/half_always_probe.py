#!/usr/bin/env python3
"""Where the big shape still ships (config C's fold, its fused round, ACCUM
on C, config F's fold), is the 512-lane half shape better?  The shipped
library against the IPLS_HALF_ALWAYS=1 build (every grid that fills takes
the half shape), same process, same buckets, interleaved rounds, HIP events
on each handle's stream; results compared bit for bit.
Usage: half_always_probe.py [ROUNDS]   (needs make -C ipls-java-api_amd variants)"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ipls  # noqa: E402
from ipls import _native as N  # noqa: E402


def run(P, L, K, what, rounds):
    elem = L + 32
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], q, k, ipls.SEED)
    torch.cuda.synchronize()
    libs = {"shipped": None, "half_always": N.load(N.PKG_ROOT / "lib" / "ab" / "libipls_agg_halfalways.so")}
    aggs = {nm: ipls.Aggregator(n_partitions=P, bucket_len=L, library=lb) for nm, lb in libs.items()}
    outs = {nm: torch.empty(P * (L - 1) + 2, dtype=torch.float64, device="cuda") for nm in libs}

    def step(nm):
        a = aggs[nm]
        if what == "reduce":
            a.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
        elif what == "accum":
            a.reduce_batch(0, rows, start_mode=ipls.START_ACCUM)
        else:
            a.aggregate_round(0, rows, out=ipls.DeviceBuffer.from_tensor(outs[nm]))
    ms = {nm: [] for nm in libs}
    shape = {}
    for _ in range(rounds):
        for nm, a in aggs.items():
            if what == "accum":
                a.reduce_batch(0, rows, start_mode=ipls.START_ZERO)   # AGG live, same value for both
            st = torch.cuda.ExternalStream(a.stream)
            step(nm)
            a.sync()
            if what == "accum":
                a.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(5):
                step(nm)
            e1.record(st)
            a.sync()
            ms[nm].append(e0.elapsed_time(e1) / 5)
            shape[nm] = a.last_launch()["shape"]
    same = all(np.array_equal(aggs["shipped"].read(q, t).view(np.uint64), aggs["half_always"].read(q, t).view(np.uint64))
               for q in (0, P - 1) for t in (ipls.TGT_AGG, ipls.TGT_WEIGHTS))
    nbytes = P * L * 8 * (K + (2 if what != "reduce" else 1))
    res = {"what": what, "P": P, "L": L, "K": K, "bit_identical": same}
    for nm in libs:
        m = float(np.median(ms[nm]))
        res[nm] = {"ms": round(m, 4), "frac": round(nbytes / m / 1e6 / 8000, 4), "shape": shape[nm]}
        aggs[nm].close()
    del arena, outs
    torch.cuda.empty_cache()
    return res


if __name__ == "__main__":
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    for P, L, K, what in ((16, 4194304, 32, "reduce"), (16, 4194304, 32, "round"), (16, 4194304, 32, "accum"),
                          (16, 8388608, 64, "reduce")):
        print(json.dumps(run(P, L, K, what, rounds)), flush=True)
