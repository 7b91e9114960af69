"""Time the fused round (ipls_agg_aggregate_round) against the plain fold on
config-C-sized batches: with / without the averaged output, and with a
bucket length whose flat offsets keep the averages 16-B aligned or not."""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd")]
import ipls  # noqa: E402


def run(P, L, K, reps=10, align=16):
    a = align // 8
    elem = (L + a - 1) // a * a + 32  # every bucket `align`-B aligned
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], q, k, ipls.SEED)
    out = torch.empty(P * (L - 1) + 2, dtype=torch.float64, device="cuda")
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    st = torch.cuda.ExternalStream(agg.stream)
    res = {}
    for name, fn in [
        ("reduce", lambda: agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)),
        ("round_noavg", lambda: agg.aggregate_round(0, rows, with_average=False)),
        ("round_avg", lambda: agg.aggregate_round(0, rows, out=ipls.DeviceBuffer.from_tensor(out))),
        ("round_avg_shift8", lambda: agg.aggregate_round(
            0, rows, out=ipls.DeviceBuffer(int(out.data_ptr()) + 8, P * (L - 1)))),
    ]:
        fn()
        agg.sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        agg.sync()
        res[name] = round(e0.elapsed_time(e1) / reps, 4)
    agg.close()
    del arena, out
    torch.cuda.empty_cache()
    return res


if __name__ == "__main__":
    for L, align in ((4194304, 16), (4194305, 16), (4194305, 256), (4194306, 16)):
        print(f"P=16 L={L} K=32 bucket alignment {align} B", run(16, L, 32, align=align), flush=True)
