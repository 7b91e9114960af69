"""Soak run of tests/test_gpu_parity.py::test_stateful_random_sequence over
many seeds, coalescing groups and device lists (dev tool; one process,
stops at the first mismatch).  Usage: fuzz_stateful.py FIRST_SEED N_SEEDS"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd"), str(ROOT / "tests")]
import ipls  # noqa: E402
from oracle import oracle as O  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def main(first=100, n=200):
    t0 = time.time()
    for seed in range(first, first + n):
        group = [1, 2, 3, 5, 8, 16, 32, 64][seed % 8]
        P = 1 + seed % 5
        L = [2, 3, 17, 1024, 5003, 65537, 262147][seed % 7]
        devices = [None, [0, 0], [0, 0, 0], [0, 0, 0, 0]][(seed // 7) % 4]   # one- and multi-shard handles
        T.test_stateful_random_sequence(ipls, O, seed, group, devices, P=P, L=L)
        if (seed - first) % 20 == 19:
            print(f"seeds {first}..{seed} ok ({time.time() - t0:.0f} s)", flush=True)
    print(f"fuzz ok: {n} seeds x 300 steps", flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
