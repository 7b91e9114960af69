"""Stress: tests/test_gpu_parity.py::test_concurrent_callers_one_handle and
::test_concurrent_replica_store repeated N times in one process (dev tool).
Usage: stress_concurrent.py N [sharded]   (sharded: the three-shard [0, 0, 0] handle)"""
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
    if i % 20 == 19:
        print(f"{i+1} runs ok ({time.time()-t0:.0f} s)", flush=True)
print("stress ok")
