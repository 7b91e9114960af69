"""Per-arrival folds: the config-C workload (16
partitions x 4M doubles x 32 peers) folded one bucket per call, the way
Updater._Update folds each queue item (Updater.java:115-117), instead of one
reduce_batch launch.  Two arrival orders: partition-major (all peers of p0,
then p1, ...) and peer-major (peer 0's 16 buckets, then peer 1's ...).  The
GPU time of the K*P folds comes from HIP events on the handle's stream after
the calls are queued back to back; run it under rocprofv3 --kernel-trace
--stats for per-kernel numbers.  Rates are the batch's algorithmic bytes
P*(K+1)*L*8 over that time.  Dev tool."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd")]
import torch  # noqa: E402
import ipls  # noqa: E402


def main(P=16, L=4194304, K=32, reps=3):
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
    algo = P * (K + 1) * L * 8
    from oracle import oracle as O
    want = O.c_synth_sum_checksum(L, 0, K)
    for mode in ("Update", "UpdateAsync"):
        for order in ("partition-major", "peer-major"):
            seq = [(q, k) for q in range(P) for k in range(K)] if order == "partition-major" else \
                  [(q, k) for k in range(K) for q in range(P)]
            best = None
            for _ in range(reps):
                agg.reset()
                # the first fold of each partition starts from +0.0 (logically-zero flag)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                if mode == "Update":          # one fold launch per arrival
                    for q, k in seq:
                        agg.Update(rows[q][k], q)
                else:                         # queued, folded in groups (ipls_agg_set_coalesce)
                    t = 0
                    for q, k in seq:
                        t = agg.UpdateAsync(rows[q][k], q)
                    agg.Wait(t)
                e1.record(stream)
                agg.sync()
                ms = e0.elapsed_time(e1)
                best = ms if best is None else min(best, ms)
            ok = agg.checksum(0) == want
            print(f"per-arrival {mode} {order}: {P}x{K} folds of {L} doubles in {best:.3f} ms (best of {reps}) = "
                  f"{algo / best / 1e6:.1f} GB/s algorithmic ({algo / best / 1e6 / 8000 * 100:.1f} % of 8 TB/s), "
                  f"checksum p0 {'ok' if ok else 'MISMATCH'}")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    agg.reduce_batch(0, rows)
    e0.record(stream)
    agg.reduce_batch(0, rows)
    e1.record(stream)
    agg.sync()
    ms = e0.elapsed_time(e1)
    print(f"batched (one reduce_batch): {ms:.3f} ms = {algo / ms / 1e6:.1f} GB/s")
    agg.close()


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
