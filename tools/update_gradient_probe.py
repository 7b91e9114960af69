#!/usr/bin/env python3
"""Dev probe (round 4): IPLS.UpdateGradient (IPLS.java:1703-1743) from a host
double[] of the whole model, M = 16 x 4,194,303 (config C's partitions), with
1, 4 and 16 owned partitions.  Only the owned partitions' values cross PCIe;
the wall time per call is reported with the bytes that had to move and the
AGG bits checked against the oracle for the last call.
Usage: update_gradient_probe.py [REPS]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime first)
import ipls  # noqa: E402
from oracle import oracle as O  # noqa: E402  (checker only)

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
P = 16
M = P * 4194303
flat = np.random.default_rng(7).standard_normal(M)
out = {"M": M, "partitions": P, "reps": reps}
for owned_n in (1, 4, 16):
    agg = ipls.Aggregator(M, P)
    owned = list(range(owned_n))
    agg.UpdateGradient(flat, owned)          # warm (scratch, pages)
    agg.sync()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        agg.UpdateGradient(flat, owned)
        agg.sync()
        ts.append(time.perf_counter() - t0)
    ms = float(np.median(ts)) * 1e3
    moved = sum(O.partition_len(M, P, p) - 1 for p in owned) * 8
    parts = O.organize_gradients(flat, M, P)
    acc = parts[0].copy() * 0.0
    for _ in range(reps + 1):
        acc = O.fold(acc, parts[0])
    ok = np.array_equal(agg.read(0, ipls.TGT_AGG).view(np.uint64), acc.view(np.uint64))
    out[f"owned_{owned_n}"] = {"ms": round(ms, 3), "host_bytes_moved": moved,
                               "GBps_moved": round(moved / ms / 1e6, 1), "agg0_bit_exact": ok}
    agg.close()
print(json.dumps(out))
