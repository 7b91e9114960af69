"""Soak run of tests/test_gpu_parity.py::test_stateful_random_sequence over
many seeds, coalescing groups and device lists (dev tool; one process,
stops at the first mismatch).
Usage: fuzz_stateful.py FIRST_SEED N_SEEDS [big]
  big: bucket lengths of the production launch shapes (1M-4M doubles,
       ragged), so the batched folds and fused rounds run the big and mid
       tiles; the shapes reached are printed per seed."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd"), str(ROOT / "tests")]
import ipls  # noqa: E402
from oracle import oracle as O  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def main(first=100, n=200, mode="small"):
    t0 = time.time()
    collide_seeds = tree_seeds = 0
    big = mode == "big"
    for seed in range(first, first + n):
        group = [1, 2, 3, 5, 8, 16, 32, 64][seed % 8]
        devices = [None, [0, 0], [0, 0, 0], [0, 0, 0, 0]][(seed // 7) % 4]   # one- and multi-shard handles
        if big:
            P = 1 + seed % 4
            L = [4 * 1048576 + 5, 2 * 1048576 + 3, 4 * 1048576, 1048576 + 7][(seed // 4) % 4]
            shapes = set()
            T.test_stateful_random_sequence(ipls, O, seed, group, devices, P=P, L=L, shapes=shapes)
            if seed % 3 == 2:
                collide_seeds += 1
                tree_seeds += any(sh[0] == "replica store" for sh in shapes)
            print(f"seed {seed} ok: P={P} L={L} group={group} devices={devices} "
                  f"(kernel, shape, map, be, start) reached {sorted(shapes, key=repr)} ({time.time() - t0:.0f} s)", flush=True)
            continue
        P = 1 + seed % 5
        L = [2, 3, 17, 1024, 5003, 65537, 262147][seed % 7]
        shapes = set()
        T.test_stateful_random_sequence(ipls, O, seed, group, devices, P=P, L=L, shapes=shapes)
        if seed % 3 == 2:   # the colliding-hash seeds: did the replica store grow a tree bin?
            collide_seeds += 1
            tree_seeds += any(sh[0] == "replica store" for sh in shapes)
        if (seed - first) % 20 == 19:
            print(f"seeds {first}..{seed} ok ({time.time() - t0:.0f} s)", flush=True)
    print(f"fuzz ok: {n} seeds x 300 steps; replica-store tree bins in {tree_seeds} of {collide_seeds} "
          f"colliding-hash seeds", flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(*[int(x) for x in a[:2]], *a[2:3])
