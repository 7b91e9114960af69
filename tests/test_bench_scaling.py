"""the first N > 1 run must be judgeable against numbers
written before it.  bench.scaling_prediction(N) is the table of DESIGN.md
§6.1, and every N > 1 line carries it (scaling_check.predicted) beside the
measured combine / exchange / value, with the xGMI link peak DESIGN states.
CPU only."""
import json
import re
import subprocess
import sys

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, str(ROOT))
    import bench as b
    return b


def _design_table():
    text = (ROOT / "DESIGN.md").read_text()
    sec = text[text.index("### 6.1"):]
    sec = sec[:sec.index("\n## ")] if "\n## " in sec else sec
    rows = {}
    for ln in sec.splitlines():
        m = re.match(r"\|\s*(\d)\s*\|\s*([\d,]+)–([\d,]+)\s*\|(.*)\|\s*$", ln)
        if m:
            rest = [c.strip() for c in m.group(4).split("|")]
            rows[int(m.group(1))] = (float(m.group(2).replace(",", "")), float(m.group(3).replace(",", "")), rest)
    return sec, rows


def test_design_table_is_the_prediction(bench):
    sec, rows = _design_table()
    assert sorted(rows) == [1, 2, 4, 8]
    assert f"{bench.XGMI_LINK_GBS:.0f} GB/s per direction" in sec
    for n, (lo, hi, rest) in rows.items():
        p = bench.scaling_prediction(n)
        assert (lo, hi) == tuple(p["value_GBps"]), n
        if n == 1:
            continue
        links, busiest, even, peak, frac = rest
        assert int(links) == p["links_per_owner"] and int(busiest) == p["busiest_link_partials"]
        assert float(even) == p["combine_ms_even_links"] and float(peak) == p["combine_ms_at_link_peak"]
        assert float(frac) == p["frac_of_xgmi_if_busiest_link_saturated"]


def test_prediction_follows_the_spread_schedule(bench):
    from ipls.distributed import ReplicaPlan
    for g in (2, 4, 8):
        P = 16
        plan = ReplicaPlan.spread(P * g, g)
        # owner 0's partitions 0..P-1: which rank holds each one's replica partial
        src = {}
        for p, o, others in plan.exchanges():
            if o == 0:
                for r in others:
                    src[r] = src.get(r, 0) + 1
        assert src == bench.spread_sources(0, g, P), g
        p = bench.scaling_prediction(g)
        assert p["busiest_link_partials"] == max(src.values())
        assert p["links_per_owner"] == len(src)


def test_the_n_gt_1_line_carries_frac_of_xgmi_and_the_stated_peak(bench):
    out = {"metric": bench.METRIC, "value": 55000.0, "ms_per_step": 2.57, "n_gpus": 8,
           "c_abi_multi_gpu": {"combine": {"owner_kernel_ms": [0.9] * 8, "frac_of_xgmi": [0.5] * 8,
                                           "frac_of_xgmi_min": 0.5, "xgmi_link_GBps": bench.XGMI_LINK_GBS,
                                           "status": "measured: distinct GPUs over xGMI"}},
           "replica_exchange": {"exchange_ms": 1.2, "exchange_GBps_per_rank_each_way": 447.0},
           "host_inclusive_multi": {"GBps_per_gpu_min": 53.0},
           "verified": True, "verified_partitions": "16/16", "build": {"so_sha256": "x", "sources_match": True}}
    out["scaling_check"] = bench.scaling_check(8, out)
    sc = out["scaling_check"]
    assert sc["predicted"]["link_GBps"] == bench.XGMI_LINK_GBS == 153.0
    assert sc["measured"]["combine_frac_of_xgmi_min"] == 0.5
    assert sc["measured"]["combine_xgmi_link_GBps"] == sc["predicted"]["link_GBps"]
    assert sc["measured"]["replica_exchange_ms"] == 1.2 and sc["measured"]["e2e_GBps_per_gpu_min"] == 53.0
    line = list(bench.proof_last(out))
    # just before the proof keys, so a driver's stdout tail keeps it
    assert line[-4:] == ["scaling_check", "verified", "verified_partitions", "build"]
    assert len(json.dumps(sc)) < 1500


def test_spawned_n2_line_carries_the_prediction():
    import os
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--dist-backend", "gloo", "--plumbing-selftest",
                        "--gpus", "2"], capture_output=True, text=True, timeout=180, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert line["scaling_check"]["predicted"]["links_per_owner"] == 1
    assert line["scaling_check"]["predicted"]["link_GBps"] == 153.0
