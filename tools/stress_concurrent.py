"""Stress: tests/test_gpu_parity.py::test_concurrent_callers_one_handle,
::test_concurrent_replica_store and (round 6) the chunked calls' stage pool
under concurrency and their lock scope (::test_chunked_stage_pool_under_
concurrency, ::test_chunked_io_holds_no_shard_lock) repeated N times in one
process (dev tool).
Usage: stress_concurrent.py N [sharded]   (sharded: the three-shard [0, 0, 0] handle;
the chunked tests then run on their two-shard [0, 0] handle)"""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd"), str(ROOT / "tests")]
import ipls
from oracle import oracle as O
import test_gpu_parity as T
t0 = time.time()
devices = [0, 0, 0] if len(sys.argv) > 2 and sys.argv[2] == "sharded" else None
for i in range(int(sys.argv[1])):
    T.test_concurrent_callers_one_handle(ipls, O, devices)
    T.test_concurrent_replica_store(ipls, O, devices)
    T.test_chunked_stage_pool_under_concurrency(ipls, O, devices and [0, 0])
    T.test_chunked_io_holds_no_shard_lock(ipls, O, devices and [0, 0])
    if i % 5 == 4:
        print(f"{i+1} runs ok ({time.time()-t0:.0f} s)", flush=True)
print("stress ok")
