"""Time the rest of an aggregation round on config C's geometry, REPS times
each (HIP events on the handle's stream): AggregatePartition(all)
(k_finalize, 16 B/element) and GetPartitions into a device buffer
(k_divide, 16 B/element).  Dev tool."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd")]
import ipls  # noqa: E402


def main(P=16, L=4194304, reps=10):
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L)
    st = torch.cuda.ExternalStream(agg.stream)
    buck = torch.empty(L + 32, dtype=torch.float64, device="cuda")
    b = ipls.DeviceBuffer(int(buck.data_ptr()), L)      # torch allocations are 512-B aligned
    ipls.synth_fill(b, 0, 0, ipls.SEED)
    rows = [[b] for _ in range(P)]
    flat = torch.empty(P * (L - 1), dtype=torch.float64, device="cuda")
    fb = ipls.DeviceBuffer.from_tensor(flat)
    fin, div = [], []
    for r in range(reps + 1):
        agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record(st)
        agg.AggregatePartition(ipls.ALL_PARTITIONS)
        e[1].record(st)
        agg.GetPartitions(out=fb)
        e[2].record(st)
        agg.sync()
        if r:
            fin.append(e[0].elapsed_time(e[1]))
            div.append(e[1].elapsed_time(e[2]))
    n = P * L
    fm, dm = float(np.median(fin)), float(np.median(div))
    print(f"P={P} L={L}: finalize median {fm:.4f} ms = {16 * n / fm / 1e6:.1f} GB/s "
          f"({16 * n / fm / 8e7:.1f}% of 8 TB/s); divide median {dm:.4f} ms = "
          f"{16 * (n - P) / dm / 1e6:.1f} GB/s ({16 * (n - P) / dm / 8e7:.1f}%)")
    agg.close()


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
