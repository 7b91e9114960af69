#!/usr/bin/env python3
"""Config D (64 x 4,194,304 x 32) with the bucket layout held fixed: the same
68.7 GB arena filled with big-endian bytes (the BASELINE configs[2] workload:
BE in, BE sum out) and then with native doubles (same bits, no byte swap),
alternating three times in one process.  VERDICT r5 item 2: if the two read
the same, the fused v_perm byte swap costs nothing and the gap of D's
bench leg to config C is the memory system (bucket count and layout,
DESIGN.md §5.3), not the kernel's issue.  Each arm: 5 back-to-back launches
between two HIP events on the handle's stream, after one untimed launch.
Prints one JSON line."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ipls-java-api_amd"))
import ipls  # noqa: E402

P, L, K = 64, 4194304, 32
STEPS, ALTERNATIONS = 5, 3


def main():
    elem = L + 32
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    out_arena = torch.empty(P * elem + 32, dtype=torch.float64, device="cuda")
    obase = (int(out_arena.data_ptr()) + 255) // 256 * 256
    dsts = [obase + 8 * q * elem for q in range(P)]
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    stream = torch.cuda.ExternalStream(agg.stream)
    nbytes = P * (K + 1) * L * 8
    res = {"be": [], "native": []}
    for _ in range(ALTERNATIONS):
        for be in (True, False):
            rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L, big_endian=be) for k in range(K)]
                    for q in range(P)]
            for q in range(P):
                for k in range(K):
                    ipls.synth_fill(rows[q][k], q, k, ipls.SEED)
            torch.cuda.synchronize()

            def step():
                agg.reduce_batch_out(0, rows, dsts, start_mode=ipls.START_ZERO, big_endian_in=be, big_endian_out=be)
            step()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(stream)
            for _ in range(STEPS):
                step()
            ev1.record(stream)
            agg.sync()
            ms = ev0.elapsed_time(ev1) / STEPS
            res["be" if be else "native"].append(round(ms, 4))
            print(f"[d_be_probe] {'be' if be else 'native'} {ms:.4f} ms", file=sys.stderr, flush=True)
    out = {"workload": "D: 64 x 4194304 x 32, one arena, BE and native alternating",
           "launch": agg.last_launch()}
    for k, v in res.items():
        ms = float(np.median(v))
        out[k] = {"ms": v, "median_ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1),
                  "frac_of_8TBps": round(nbytes / ms / 1e6 / 8000.0, 4)}
    out["be_over_native"] = round(out["be"]["median_ms"] / out["native"]["median_ms"], 4)
    agg.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
