"""Provenance of the bench numbers, on the CPU: the build
record of the library (ipls.build_info, tools/build_stamp.py), the rule by
which bench.py reports roofline.traffic only for the build the PMC passes
were taken on, and tools/pmc_traffic.py reading the profiled process's build
from its bench line.  Also the publish wrappers' capacity checks,
which run before any library call."""
import hashlib
import json
import subprocess
import sys

import pytest

from conftest import ROOT


def test_build_info_hashes_the_loaded_library():
    import ipls
    from ipls import _native as N
    info = ipls.build_info()
    assert info["so_sha256"] == hashlib.sha256(N.LIB_PATH.read_bytes()).hexdigest()
    stamp = N.LIB_PATH.with_name(N.LIB_PATH.name + ".buildinfo.json")
    if stamp.exists():                      # written by every `make` of the library
        rec = json.loads(stamp.read_text())
        assert info["stamp_matches_so"] == (rec["so_sha256"] == info["so_sha256"])
        assert info["kernel_src_sha256"] == rec["kernel_src_sha256"]


def test_build_stamp_records_kernel_source_hash(tmp_path):
    sys.path.insert(0, str(ROOT / "tools"))
    import build_stamp
    lib = tmp_path / "libx.so"
    lib.write_bytes(b"not really a library")
    subprocess.run([sys.executable, str(ROOT / "tools" / "build_stamp.py"), str(lib)], check=True,
                   capture_output=True)
    rec = json.loads((tmp_path / "libx.so.buildinfo.json").read_text())
    assert rec["so_sha256"] == hashlib.sha256(b"not really a library").hexdigest()
    assert rec["kernel_src_sha256"] == build_stamp.kernel_src_sha256()
    assert rec["so"] == "libx.so"


@pytest.fixture
def bench(tmp_path, monkeypatch):
    sys.path.insert(0, str(ROOT))
    import bench as b
    prof = tmp_path / "profiles"
    prof.mkdir()
    entry = {"hbm_bytes_per_launch": 123, "build": {"so_sha256": "aa", "kernel_src_sha256": "kk", "git_rev": "r"},
             "source": "profiles/rXX"}
    (prof / "pmc_traffic.json").write_text(json.dumps({"C": entry, "old": {"hbm_bytes_per_launch": 7}}))
    monkeypatch.setattr(b, "ROOT", tmp_path)
    return b


def test_traffic_reported_only_for_the_profiled_build(bench):
    t, p = bench.pmc_traffic("C", {"so_sha256": "aa", "kernel_src_sha256": "zz"})
    assert t == 123 and p["match"] == "so_sha256" and p["traffic_stale"] is False
    t, p = bench.pmc_traffic("C", {"so_sha256": "bb", "kernel_src_sha256": "kk"})
    assert t == 123 and p["match"] == "kernel_src_sha256"          # relinked, same kernels
    t, p = bench.pmc_traffic("C", {"so_sha256": "bb", "kernel_src_sha256": "zz"})
    assert t is None and p["traffic_stale"] is True and p["entry_so_sha256"] == "aa"
    t, p = bench.pmc_traffic("old", {"so_sha256": "aa"})            # an entry without a build record
    assert t is None and p["traffic_stale"] is True
    t, p = bench.pmc_traffic("D-be", {"so_sha256": "aa"})
    assert t is None and "no PMC entry" in p["why"]


def test_pmc_tool_reads_the_build_from_the_bench_line(tmp_path):
    sys.path.insert(0, str(ROOT / "tools"))
    import pmc_traffic
    log = tmp_path / "pmc_fetch.log"
    line = {"metric": "x", "build": {"so_sha256": "aa", "kernel_src_sha256": "kk"}}
    log.write_text("rocprofv3 chatter\n" + json.dumps(line) + "\nmore chatter\n")
    assert pmc_traffic.build_of(log) == line["build"]
    bad = tmp_path / "bad.log"
    bad.write_text("no json here\n")
    with pytest.raises(SystemExit):
        pmc_traffic.build_of(bad)


def test_device_text_capacity_checks():
    import ipls
    out = ipls.Aggregator._device_text_out
    assert out(ipls.DeviceBuffer(4096, 100), None, 800) == (4096, 800)       # capacity = 8 * n
    assert out(ipls.DeviceBuffer(4096, 100), 600, 600) == (4096, 600)       # a smaller explicit cap wins
    with pytest.raises(ValueError):
        out(ipls.DeviceBuffer(4096, 99), None, 800)                         # 792 B < 800 needed
    with pytest.raises(ValueError):
        out(4096, None, 10)                                                 # raw address without a capacity
    with pytest.raises(ValueError):
        out(4096, 9, 10)
    assert out(4096, 10, 10) == (4096, 10)


def test_bucket_table_size_checks():
    """The batched calls' bucket tables carry bare pointers, and the kernels
    read L_p doubles from each: a DeviceBuffer shorter than its partition is
    refused before any call (raw addresses stay the caller's contract)."""
    from ipls.aggregator import _bucket_table
    import ipls
    lengths = [100, 100, 97]
    rows = [[ipls.DeviceBuffer(4096 * (q * 2 + k + 1), lengths[q]) for k in range(2)] for q in range(3)]
    flat, k = _bucket_table(rows, lengths, 0)
    assert k == 2 and flat == [4096 * i for i in range(1, 7)]
    flat, k = _bucket_table([[1, 2], [3, ipls.DeviceBuffer(8, 97)]], lengths, 1)   # raw ints pass through
    assert (flat, k) == ([1, 2, 3, 8], 2)
    with pytest.raises(ValueError, match="partition 1 needs buckets of 100"):
        _bucket_table([[ipls.DeviceBuffer(8, 99)]], lengths, 1)
    with pytest.raises(ValueError, match="same number of buckets"):
        _bucket_table([[1, 2], [3]], lengths, 0)
    assert _bucket_table([], lengths, 0) == ([], 0)
    # a partition out of range is the library's IPLS_E_RANGE, not a size error here
    assert _bucket_table([[ipls.DeviceBuffer(8, 1)]], lengths, 5) == ([8], 1)


def test_committed_pmc_entries_carry_their_build():
    """Every committed PMC entry names the build it was taken on and the
    profile it came from; an entry without them would make bench.py report
    `traffic: null` (tools/pmc_traffic.py stores nothing without --bench-log)."""
    d = json.loads((ROOT / "profiles" / "pmc_traffic.json").read_text())
    for k in ("C", "C-round", "C-finalize", "C-divide", "B", "D-be", "F"):   # the entries bench.py reads
        e = d[k]                                                             # (C_r02 ... are history)
        b = e.get("build") or {}
        assert b.get("so_sha256") and b.get("device_code_sha256"), k
        assert (ROOT / e["source"]).is_dir(), (k, e.get("source"))
        assert 0.99 <= e["traffic_over_algorithmic"] <= 1.1, k


def test_pmc_tool_stores_nothing_without_a_build(tmp_path):
    sys.path.insert(0, str(ROOT / "tools"))
    fetch = tmp_path / "f.csv"
    write = tmp_path / "w.csv"
    hdr = "Dispatch_Id,Kernel_Name,Grid_Size,Workgroup_Size,VGPR_Count,Counter_Name,Counter_Value\n"
    fetch.write_text(hdr + "1,k_reduce,1,1,1,FETCH_SIZE,4.0\n")
    write.write_text(hdr + "1,k_reduce,1,1,1,WRITE_SIZE,8.0\n")
    out = tmp_path / "pmc.json"
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "pmc_traffic.py"), "C", str(fetch), str(write), "16384",
                        str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert not out.exists() and "not stored" in r.stderr


def test_bench_line_ends_with_the_proof(bench):
    """the driver keeps only the tail of stdout, so the
    line's last keys are `verified`, `verified_partitions` and `build`, and
    `build` ends with the library's identity and sources_match -- whatever
    order the legs were added in."""
    line = {"metric": "m", "value": 1.0, "verified": True, "verified_partitions": "16/16",
            "build": {"sources_match": True, "so_sha256": "s", "git_rev": "g", "device_code_sha256": "d",
                      "stamp_matches_so": True, "built_utc": "t", "kernel_src_sha256": "k"},
            "roofline": {"frac": 0.88, "traffic_provenance": {"x": 1}}, "round": {"a": 1}, "few_partitions": {"b": 2}}
    out = bench.proof_last(line)
    assert list(out)[-3:] == ["verified", "verified_partitions", "build"]
    assert list(out["build"])[-5:] == ["so_sha256", "device_code_sha256", "built_utc", "stamp_matches_so",
                                       "sources_match"]
    assert out["roofline"] == line["roofline"] and set(out) == set(line)
    text = json.dumps(out)
    assert text.endswith('"sources_match": true}}')
    assert '"verified_partitions": "16/16"' in text[-600:]
