#!/usr/bin/env python3
"""Split a run of back-to-back launches into kernel time and the gaps between
them, from a rocprofv3 --kernel-trace CSV (Start_Timestamp / End_Timestamp
in ns).  VERDICT r4 next 6: config B's bench line (HIP events around 50
launches of 0.18 ms) reads lower than the kernel's rocprof mean; this says
how much of each step is the kernel and how much the boundary to the next.

    python3 tools/gap_split.py kernel_trace.csv --kernel k_reduce --bytes 1207959552 [--min-run 20]

Only launches of the named kernel that follow another launch of it with no
other kernel in between count (the timed loop); a gap is the next launch's
start minus this launch's end.  Output: one JSON object.
"""
import argparse
import csv
import json
import statistics


def runs_of(rows, name):
    """Maximal runs of consecutive dispatches (in start order, one queue) of `name`."""
    rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
    run, out = [], []
    for r in rows:
        if name in r["Kernel_Name"]:
            run.append(r)
        else:
            if run:
                out.append(run)
            run = []
    if run:
        out.append(run)
    return out


def split(path, name, nbytes, min_run=20, peak_gbs=8000.0):
    with open(path, newline="") as f:
        rows = list(csv.DictReader(f))
    runs = [r for r in runs_of(rows, name) if len(r) >= min_run]
    if not runs:
        raise SystemExit(f"no run of >= {min_run} consecutive {name} launches in {path}")
    kern, gaps = [], []
    for run in runs:
        for a, b in zip(run, run[1:]):
            kern.append(int(a["End_Timestamp"]) - int(a["Start_Timestamp"]))
            gaps.append(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]))
    k_ns, g_ns = statistics.mean(kern), statistics.mean(gaps)
    gs = sorted(gaps)
    step = k_ns + g_ns
    return {
        "trace": path, "kernel": name, "runs": len(runs), "launches_counted": len(kern),
        "kernel_ns_mean": round(k_ns, 1), "kernel_ns_median": statistics.median(kern),
        "gap_ns_mean": round(g_ns, 1), "gap_ns_median": statistics.median(gaps),
        "gap_ns_p10": gs[len(gs) // 10], "gap_ns_p90": gs[(9 * len(gs)) // 10],
        "gap_share_of_step": round(g_ns / step, 4),
        "kernel_only_frac": round(nbytes / k_ns / peak_gbs, 4) if nbytes else None,
        "back_to_back_frac": round(nbytes / step / peak_gbs, 4) if nbytes else None,
        "algorithmic_bytes_per_launch": nbytes,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_reduce")
    ap.add_argument("--bytes", type=int, default=0)
    ap.add_argument("--min-run", type=int, default=20)
    a = ap.parse_args()
    print(json.dumps(split(a.trace, a.kernel, a.bytes, a.min_run)))


if __name__ == "__main__":
    main()
