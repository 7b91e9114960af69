#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per
launch of ipls::k_reduce (MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7):
  * counters are in KiB;
  * on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide (16 B per
    lane) coalesced streaming read -> doubled;
  * WRITE_SIZE is exact for 16-B streaming stores.
Usage: pmc_traffic.py WORKLOAD FETCH_CSV WRITE_CSV ALGO_BYTES [OUT_JSON] [KERNEL] [--bench-log LOG ...] [--source S]
(KERNEL defaults to k_reduce; k_round for the fused round.)
--bench-log: the stdout of the profiled bench.py processes (the PMC passes);
their JSON line's "build" record (ipls.build_info(): .so sha256, git revision,
kernel-source sha256) is stored with the entry, and bench.py reports the
entry's traffic only for the same build.  Both passes must agree on it.
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


def build_of(log):
    """The build record in a bench.py stdout log (its JSON line)."""
    rec = None
    for ln in Path(log).read_text(errors="replace").splitlines():
        ln = ln.strip()
        if ln.startswith("{") and '"build"' in ln:
            try:
                rec = json.loads(ln).get("build")
            except ValueError:
                pass
    if rec is None:
        sys.exit(f"{log}: no bench JSON line with a build record")
    return rec


def main():
    argv, logs, source = [], [], None
    it = iter(sys.argv[1:])
    for a in it:
        if a == "--bench-log":
            logs.append(next(it))
        elif a == "--source":
            source = next(it)
        else:
            argv.append(a)
    wl, fcsv, wcsv, algo = argv[0], argv[1], argv[2], int(argv[3])
    out = Path(argv[4]) if len(argv) > 4 and argv[4] != "-" else \
        Path(__file__).resolve().parent.parent / "profiles" / "pmc_traffic.json"
    kernel = argv[5] if len(argv) > 5 else "k_reduce"
    builds = [build_of(x) for x in logs]
    if any(b.get("so_sha256") != builds[0].get("so_sha256") for b in builds):
        sys.exit("the PMC passes ran on different builds of the library")
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
    if builds:
        d[wl]["build"] = {k: builds[0].get(k) for k in ("so_sha256", "kernel_src_sha256", "device_code_sha256",
                                                         "git_rev", "sources_dirty")}
    if source:
        d[wl]["source"] = source
    if builds:
        out.write_text(json.dumps(d, indent=1) + "\n")
    else:   # an entry without a build record would hide its traffic from every bench line: report only
        print("not stored: no --bench-log, so no build record", file=sys.stderr)
    print(json.dumps(d[wl]))


if __name__ == "__main__":
    main()
