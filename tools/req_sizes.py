#!/usr/bin/env python3
"""L2 -> fabric read requests by size per kernel, from rocprofv3 --pmc passes
of tools/copy_sweep.hip (tools/gpu_r05o.sh): TCC_EA0_RDREQ (all), _32B,
_64B, _128B, _DRAM and TCC_BUBBLE, each summed over the XCDs and instances.
Bytes = 32 n32 + 64 n64 + 128 n128, against the kernel's W bytes, beside
FETCH_SIZE's own expression (BUBBLE*128 + (RDREQ-BUBBLE-32B)*64 + 32B*32) and
that doubled (the gfx950 correction for wide streaming reads).
Usage: req_sizes.py DIR [W_BYTES]     (DIR holds p1/ p2/ p3/)
"""
import collections
import csv
import sys
from pathlib import Path


def load(path):
    out = collections.defaultdict(lambda: collections.defaultdict(dict))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        c = r["Counter_Name"].replace("_sum", "")
        d = out[k][r["Dispatch_Id"]]
        d[c] = d.get(c, 0.0) + float(r["Counter_Value"])
    return out


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2] if xs else float("nan")


def main():
    root = Path(sys.argv[1])
    W = float(sys.argv[2]) if len(sys.argv) > 2 else 16 * 4194304 * 8
    per = collections.defaultdict(dict)
    for p in ("p1", "p2", "p3"):
        for k, disp in load(root / p / "run_counter_collection.csv").items():
            for c in next(iter(disp.values())):
                per[k][c] = med([d[c] for d in disp.values()])
    print("# kernel: requests by size (median dispatch), bytes / W; FETCH_SIZE expr / W and x2")
    for k, c in per.items():
        if "divide" not in k and "finalize" not in k:
            continue
        n, n32, n64, n128 = c["TCC_EA0_RDREQ"], c["TCC_EA0_RDREQ_32B"], c["TCC_EA0_RDREQ_64B"], c["TCC_EA0_RDREQ_128B"]
        by = 32 * n32 + 64 * n64 + 128 * n128
        fs = c["TCC_BUBBLE"] * 128 + (n - c["TCC_BUBBLE"] - n32) * 64 + n32 * 32
        print(f"{k}: req {n:.0f} = 32B {n32:.0f} + 64B {n64:.0f} + 128B {n128:.0f} (sum {n32 + n64 + n128:.0f}); "
              f"DRAM {c['TCC_EA0_RDREQ_DRAM']:.0f}; bytes/W {by / W:.4f}; FETCH_SIZE/W {fs / W:.4f}, x2 {2 * fs / W:.4f}")


if __name__ == "__main__":
    main()
