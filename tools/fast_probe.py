#!/usr/bin/env python3
"""Per-arrival calls from Python: ipls._fast (CPython extension) against the
ctypes binding of the same library, interleaved in one process on the bench's
per_arrival workload (config C, 16 partitions x 4M doubles x 32 peers, peer-
major, queued device folds).  Per repetition: the host time of the 512-call
loop (perf_counter) and the time from the first call to the folds' end (HIP
events on the handle's stream, as bench.py's per_arrival leg), both paths.
Usage: fast_probe.py [REPS]   Dev tool."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ipls  # noqa: E402
from ipls import _native as N  # noqa: E402


def main(reps=10, P=16, L=4194304, K=32):
    elem = L + 32
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], q, k, ipls.SEED)
    torch.cuda.synchronize()
    aggs = {"fast": ipls.Aggregator(n_partitions=P, bucket_len=L),
            "ctypes": ipls.Aggregator(n_partitions=P, bucket_len=L, library=N.load(N.LIB_PATH))}
    assert aggs["fast"]._fast is not None and aggs["ctypes"]._fast is None
    res = {nm: {"host_us_per_call": [], "ms": []} for nm in aggs}
    sums = {}
    for r in range(reps + 1):
        for nm, agg in aggs.items():
            st = torch.cuda.ExternalStream(agg.stream)
            agg.reset()
            agg.sync()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            t0 = time.perf_counter()
            t = 0
            for k in range(K):
                for q in range(P):
                    t = agg.UpdateAsync(rows[q][k], q)
            host = time.perf_counter() - t0
            agg.Wait(t)
            e1.record(st)
            agg.sync()
            if r:                                   # the first repetition warms both paths
                res[nm]["host_us_per_call"].append(host / (K * P) * 1e6)
                res[nm]["ms"].append(e0.elapsed_time(e1))
            sums[nm] = agg.checksum(0)
    nbytes = P * (K + 1) * L * 8
    out = {"workload": f"{P} x {L} x {K}, peer-major, queued device folds", "reps": reps,
           "same_sum_p0": sums["fast"] == sums["ctypes"]}
    for nm, v in res.items():
        ms = float(np.median(v["ms"]))
        out[nm] = {"host_us_per_call_median": round(float(np.median(v["host_us_per_call"])), 3),
                   "host_us_per_call_min": round(float(np.min(v["host_us_per_call"])), 3),
                   "ms_median": round(ms, 4), "ms_min": round(float(np.min(v["ms"])), 4),
                   "frac_median": round(nbytes / ms / 1e6 / 8000, 4)}
    print(json.dumps(out), flush=True)
    for agg in aggs.values():
        agg.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
