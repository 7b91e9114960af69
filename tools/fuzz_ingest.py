"""Soak run of tests/test_gpu_parity.py::test_ingest_pubsub_mutations over
many seeds, both base64 layer counts and caller-given routing (dev tool; one process, stops at the
first status or bit mismatch).  Usage: fuzz_ingest.py FIRST_SEED N_SEEDS"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd"), str(ROOT / "tests")]
import ipls  # noqa: E402
from oracle import oracle as O  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def main(first=100, n=100):
    t0 = time.time()
    fails = 0
    for seed in range(first, first + n):
        for layers, override in ((1, False), (2, False), (2, True)):
            try:
                T.test_ingest_pubsub_mutations(ipls, O, layers, override, seed=seed, n_msgs=60)
            except AssertionError as e:
                fails += 1
                print(f"MISMATCH seed {seed} layers {layers} override {override}: {e}", flush=True)
                if fails >= 12:
                    raise SystemExit(1)
        if (seed - first) % 20 == 19:
            print(f"seeds {first}..{seed} ok ({time.time() - t0:.0f} s)", flush=True)
    if fails:
        raise SystemExit(f"{fails} mismatching cases")
    print(f"fuzz ok: {n} seeds x 3 (layers, routing) cases x 60 mutated texts", flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
