#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per
launch of ipls::k_reduce (MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7):
  * counters are in KiB;
  * on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide (16 B per
    lane) coalesced streaming read -> doubled;
  * WRITE_SIZE is exact for 16-B streaming stores.
Usage: pmc_traffic.py WORKLOAD FETCH_CSV WRITE_CSV ALGO_BYTES [OUT_JSON] [KERNEL]
(KERNEL defaults to k_reduce; k_round for the fused round.)
"""
import csv
import json
import statistics
import sys
from pathlib import Path


def per_dispatch(path, counter, kernel="k_reduce"):
    vals = {}
    for r in csv.DictReader(open(path)):
        base = r.get("Kernel_Name", "").split("<")[0].split("(")[0].strip()
        if base.split("::")[-1] != kernel:       # k_round, not k_round_counts
            continue
        if r.get("Counter_Name") != counter:
            continue
        vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    wl, fcsv, wcsv, algo = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    out = Path(sys.argv[5]) if len(sys.argv) > 5 and sys.argv[5] != "-" else \
        Path(__file__).resolve().parent.parent / "profiles" / "pmc_traffic.json"
    kernel = sys.argv[6] if len(sys.argv) > 6 else "k_reduce"
    f = per_dispatch(fcsv, "FETCH_SIZE", kernel)
    w = per_dispatch(wcsv, "WRITE_SIZE", kernel)
    fetch = statistics.median(f) * 1024 * 2      # gfx950: FETCH_SIZE = 1/2 of wide streaming reads
    write = statistics.median(w) * 1024
    d = json.loads(out.read_text()) if out.exists() else {}
    d[wl] = {"hbm_bytes_per_launch": int(fetch + write), "read_bytes": int(fetch), "write_bytes": int(write),
             "algorithmic_bytes_per_launch": algo, "traffic_over_algorithmic": round((fetch + write) / algo, 4),
             "kernel": kernel, "dispatches": [len(f), len(w)],
             "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                       "KiB*1024, FETCH_SIZE doubled (gfx950 half-count of wide streaming reads)"}
    out.write_text(json.dumps(d, indent=1) + "\n")
    print(json.dumps(d[wl]))


if __name__ == "__main__":
    main()
