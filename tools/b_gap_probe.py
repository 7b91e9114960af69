#!/usr/bin/env python3
"""Config B's line vs its kernel, one process, the same
buckets (16 partitions x 1,048,576 doubles x 8 peers, 1.21 GB per launch):

  events_each   50 launches, a HIP event recorded after every launch (what
                bench.py's config_leg times: kernel + boundary per launch)
  events_ends   50 launches between two events only (back to back, no
                event packets in between)
  host_us       host time per reduce_batch call (Python -> C-ABI -> launch),
                to see whether the GPU ever waits on the host
  out_ends      as events_ends, but reduce_batch_out into caller buffers
                (what bench.py's config_leg launches)

`IPLS_PROBE_CONFIG=C` runs the headline shape instead (16 x 4,194,304 x 32,
17.7 GB per launch): whether an event packet between launches changes the
kernel's own duration, not only the gap.

Run it under `rocprofv3 --kernel-trace` and feed the trace to
tools/gap_split.py for the kernel-only time and the gap between launches.
Prints one JSON line.
"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ipls-java-api_amd"))
import ipls  # noqa: E402

CFG = os.environ.get("IPLS_PROBE_CONFIG", "B")
P, L, K = {"B": (16, 1048576, 8), "C": (16, 4194304, 32)}[CFG]
N, ROUNDS = (50, 6) if CFG == "B" else (20, 3)


def main():
    elem = L + 32
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], q, k, ipls.SEED)
    torch.cuda.synchronize()
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    stream = torch.cuda.ExternalStream(agg.stream)

    out_arena = torch.empty(P * elem + 32, dtype=torch.float64, device="cuda")
    obase = (int(out_arena.data_ptr()) + 255) // 256 * 256
    dsts = [obase + 8 * q * elem for q in range(P)]

    def step():
        agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)

    def step_out():
        agg.reduce_batch_out(0, rows, dsts, start_mode=ipls.START_ZERO)
    for _ in range(20):
        step()
        step_out()
    agg.sync()
    nbytes = P * (K + 1) * L * 8
    each, ends, host, outs = [], [], [], []
    for _ in range(ROUNDS):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(N + 1)]
        ev[0].record(stream)
        for i in range(N):
            step()
            ev[i + 1].record(stream)
        agg.sync()
        each.append(float(np.mean([ev[i].elapsed_time(ev[i + 1]) for i in range(N)])))
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        t0 = time.perf_counter()
        for i in range(N):
            step()
        t1 = time.perf_counter()
        b.record(stream)
        agg.sync()
        ends.append(a.elapsed_time(b) / N)
        host.append((t1 - t0) / N * 1e6)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for i in range(N):
            step_out()
        b.record(stream)
        agg.sync()
        outs.append(a.elapsed_time(b) / N)
    me, mn = float(np.median(each)), float(np.median(ends))
    out = {"workload": f"{CFG}: {P} x {L} x {K}, {nbytes} B per launch", "launches_per_round": N, "rounds": ROUNDS,
           "events_each_ms": round(me, 5), "events_each_frac": round(nbytes / me / 8e9, 4),
           "events_ends_ms": round(mn, 5), "events_ends_frac": round(nbytes / mn / 8e9, 4),
           "out_ends_ms": round(float(np.median(outs)), 5),
           "out_ends_frac": round(nbytes / float(np.median(outs)) / 8e9, 4),
           "host_us_per_call": round(float(np.median(host)), 2), "launch": agg.last_launch(),
           "per_round_each_ms": [round(x, 5) for x in each], "per_round_ends_ms": [round(x, 5) for x in ends]}
    agg.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
