#!/usr/bin/env python3
"""Per-call overhead of the multi-shard front's host fan-out (VERDICT r2
next-4): ipls_agg_sync, get_partitions into host memory and into device
memory, and collect_replicas on a handle over an 8-entry device list
([0]*8 on a one-GPU box: eight engines, eight streams, the same host code as
eight GPUs).  Every call is one the front spreads over the shards with
par_shards; round 2 spawned and joined a std::thread per shard per call, the
shipped front hands the parts to persistent per-shard workers.
Usage: [IPLS_AGG_LIB=lib.so] shard_pool_probe.py [N_CALLS] [SHARDS]
Run once per library (same box) and compare the medians."""
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ipls  # noqa: E402
from ipls import _native as N  # noqa: E402


def timed(fn, n):
    fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return {"median_us": round(statistics.median(ts) * 1e6, 2), "p10_us": round(np.percentile(ts, 10) * 1e6, 2),
            "p90_us": round(np.percentile(ts, 90) * 1e6, 2)}


def main(n=2000, shards=8):
    M, P = 8 * 4096, 8                      # small partitions: the call overhead, not the copies
    agg = ipls.Aggregator(M, P, devices=[0] * shards)
    lib, h = N.lib(), agg.handle
    host = np.zeros(M + 8)
    dev = torch.zeros(M + 8, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    dptr = int(dev.data_ptr())
    parts = (ipls._native.ctypes.c_int32 * P)()

    def sync():
        N.check(lib.ipls_agg_sync(h))

    def get_host():
        N.check(lib.ipls_agg_get_partitions(h, host.ctypes.data, host.size, N.HOST_F64))

    def get_dev():
        N.check(lib.ipls_agg_get_partitions(h, dptr, host.size, N.DEV_F64))
        N.check(lib.ipls_agg_sync(h))

    def collect():
        N.check(lib.ipls_agg_collect_replicas(h, parts))

    out = {"lib": str(N.LIB_PATH.name), "build": ipls.build_info(), "shards": shards, "calls": n,
           "sync": timed(sync, n), "get_partitions_host": timed(get_host, n),
           "get_partitions_dev_plus_sync": timed(get_dev, n), "collect_replicas": timed(collect, n)}
    one = ipls.Aggregator(M, P)
    lib1, h1 = N.lib(), one.handle
    out["one_shard_sync"] = timed(lambda: N.check(lib1.ipls_agg_sync(h1)), n)
    one.close()
    agg.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:3]])
