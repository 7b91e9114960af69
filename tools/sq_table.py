#!/usr/bin/env python3
"""Occupancy / stall table of k_reduce from rocprofv3 --pmc passes
(tools/gpu_r06a.sh): per workload, the mean over the last three k_reduce
dispatches of each counter, and the derived rates.  VERDICT r5 item 2: which
limit binds config D's big-endian fold against native config C.

Units (MI355X_MICROARCH.md, SQ PMC): SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* / SQ_BUSY_CYCLES count quad-cycles (summed over waves for
the WAVE/WAIT/ACTIVE ones); GRBM_GUI_ACTIVE counts cycles summed over the 8
XCDs; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES.

Usage: sq_table.py DIR OUT_PREFIX   (DIR holds <wl>_P1/ <wl>_P2/ run_counter_collection.csv)
Writes OUT_PREFIX.md (the table), OUT_PREFIX.json, and OUT_PREFIX_k_reduce.csv
(the k_reduce rows of every pass, the rest of the process dropped)."""
import csv
import json
import statistics
import sys
from pathlib import Path

CUS = 256
WORKLOADS = {   # name: (algorithmic bytes per launch, description)
    "Dbe": (64 * 33 * 4194304 * 8, "D: 64 x 4M x 32, big-endian in + out"),
    "C": (16 * 33 * 4194304 * 8, "C: 16 x 4M x 32, native doubles"),
}


def load(d: Path, wl: str, rows_out: list):
    per = {}
    for pas in ("P1", "P2"):
        f = d / f"{wl}_{pas}" / "run_counter_collection.csv"
        if not f.exists():
            continue
        disp = {}
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].split("<")[0].split("(")[0].strip().split("::")[-1] != "k_reduce":
                continue
            rows_out.append({"workload": wl, "pass": pas, **r})
            x = disp.setdefault(int(r["Dispatch_Id"]), {"dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                        "vgpr": r["VGPR_Count"], "grid": int(r["Grid_Size"]),
                                                        "wg": int(r["Workgroup_Size"])})
            x[r["Counter_Name"]] = x.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        last = [disp[k] for k in sorted(disp)[-3:]]
        for k in last[0]:
            if k == "vgpr":
                per[k] = last[0][k]
            else:
                per.setdefault(k, []).extend(v[k] for v in last)
    return {k: (statistics.mean(v) if isinstance(v, list) else v) for k, v in per.items()}


def derive(c: dict, algo: int) -> dict:
    dur = c["dur_ns"] * 1e-9
    clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / dur
    wc = c.get("SQ_WAVE_CYCLES", 0)
    out = {
        "dispatch_ms (under PMC)": dur * 1e3,
        "GB/s": algo / dur / 1e9,
        "frac_of_8TBps": algo / dur / 8e12,
        "clock_GHz": clk / 1e9,
        "waves": c.get("SQ_WAVES"),
        "mean_waves_per_CU": wc * 4 / (clk * dur) / CUS if clk else None,
        "WAIT_ANY / WAVE_CYCLES": c.get("SQ_WAIT_ANY", 0) / wc if wc else None,
        "WAIT_INST_ANY / WAVE_CYCLES": c.get("SQ_WAIT_INST_ANY", 0) / wc if wc else None,
        "ACTIVE_INST_ANY / WAVE_CYCLES": c.get("SQ_ACTIVE_INST_ANY", 0) / wc if wc else None,
        "VALU insts per VMEM read": c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_VMEM_RD"] if c.get("SQ_INSTS_VMEM_RD") else None,
        "VMEM reads per GB": c.get("SQ_INSTS_VMEM_RD", 0) / (algo / 1e9),
        "INST_LEVEL_VMEM / INSTS_VMEM (quad-cycles in flight per VMEM inst)":
            c.get("SQ_INST_LEVEL_VMEM", 0) / c["SQ_INSTS_VMEM"] if c.get("SQ_INSTS_VMEM") else None,
        "SALU insts per VMEM read": c.get("SQ_INSTS_SALU", 0) / c["SQ_INSTS_VMEM_RD"] if c.get("SQ_INSTS_VMEM_RD") else None,
    }
    return out


def main():
    d, pre = Path(sys.argv[1]), Path(sys.argv[2])
    rows, res = [], {}
    for wl, (algo, desc) in WORKLOADS.items():
        c = load(d, wl, rows)
        if not c:
            continue
        res[wl] = {"desc": desc, "algorithmic_bytes": algo, "raw": c, "derived": derive(c, algo)}
    pre.with_suffix(".json").write_text(json.dumps(res, indent=1))
    keys = list(next(iter(res.values()))["derived"])
    lines = ["| | " + " | ".join(res[w]["desc"] for w in res) + " |", "|---" * (len(res) + 1) + "|"]
    for k in keys:
        vals = []
        for w in res:
            v = res[w]["derived"][k]
            vals.append("—" if v is None else (f"{v:,.0f}" if abs(v) >= 1000 else f"{v:.4g}"))
        lines.append(f"| {k} | " + " | ".join(vals) + " |")
    lines.append(f"| VGPR_Count (rocprof) | " + " | ".join(str(res[w]["raw"].get("vgpr")) for w in res) + " |")
    pre.with_suffix(".md").write_text("\n".join(lines) + "\n")
    with open(str(pre) + "_k_reduce.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
