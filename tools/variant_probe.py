#!/usr/bin/env python3
"""The shipped library against an A/B build of the same sources (default the
IPLS_HALF_ALWAYS=1 build: every grid that fills takes the 512-lane half
shape) on the grids the big shape ships for: config C's fold, its fused
round, ACCUM on C, config F's fold, config B's fold, config D's BE in + out
fold.  Same process, same buckets, interleaved rounds, HIP events on each
handle's stream; results compared bit for bit.
Usage: variant_probe.py [ROUNDS] [VARIANT_SO] [CASES]   (needs make -C ipls-java-api_amd variants;
CASES: comma list of C,Cround,Caccum,F,B,D,Dround,Fround,Bround)"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ipls  # noqa: E402
from ipls import _native as N  # noqa: E402


def run(P, L, K, what, rounds, variant="libipls_agg_halfalways.so", be=False):
    elem = L + 32
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L, big_endian=be) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], q, k, ipls.SEED)
    torch.cuda.synchronize()
    libs = {"shipped": None, "variant": N.load(N.PKG_ROOT / "lib" / "ab" / variant)}
    aggs = {nm: ipls.Aggregator(n_partitions=P, bucket_len=L, library=lb) for nm, lb in libs.items()}
    outs = {nm: torch.empty(P * (L - 1) + 2, dtype=torch.float64, device="cuda") for nm in libs}

    dst = torch.empty(P * elem + 32, dtype=torch.float64, device="cuda") if be else None
    dsts = [(int(dst.data_ptr()) + 255) // 256 * 256 + 8 * q * elem for q in range(P)] if be else None

    def step(nm):
        a = aggs[nm]
        if be:
            a.reduce_batch_out(0, rows, dsts, start_mode=ipls.START_ZERO, big_endian_in=True, big_endian_out=True)
        elif what == "reduce":
            a.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
        elif what == "accum":
            a.reduce_batch(0, rows, start_mode=ipls.START_ACCUM)
        else:
            a.aggregate_round(0, rows, out=ipls.DeviceBuffer.from_tensor(outs[nm]))
    ms = {nm: [] for nm in libs}
    shape = {}
    for _ in range(rounds):
        for nm, a in aggs.items():
            if what == "accum":
                a.reduce_batch(0, rows, start_mode=ipls.START_ZERO)   # AGG live, same value for both
            st = torch.cuda.ExternalStream(a.stream)
            step(nm)
            a.sync()
            if what == "accum":
                a.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(5):
                step(nm)
            e1.record(st)
            a.sync()
            ms[nm].append(e0.elapsed_time(e1) / 5)
            shape[nm] = a.last_launch()["shape"]
    same = all(np.array_equal(aggs["shipped"].read(q, t).view(np.uint64), aggs["variant"].read(q, t).view(np.uint64))
               for q in (0, P - 1) for t in (ipls.TGT_AGG, ipls.TGT_WEIGHTS))
    if be:   # both handles wrote the same destinations: the last writer's bytes against the oracle's checksum
        from oracle import oracle as O   # checker only
        same = ipls.checksum_dev(ipls.DeviceBuffer(dsts[0], L, big_endian=True)) == O.c_synth_sum_checksum(L, 0, K)
    nbytes = P * L * 8 * (K + (2 if what != "reduce" else 1))
    res = {"what": what, "P": P, "L": L, "K": K, "be": be, "variant": variant, "bit_identical": same}
    for nm in libs:
        m = float(np.median(ms[nm]))
        res[nm] = {"ms": round(m, 4), "frac": round(nbytes / m / 1e6 / 8000, 4), "shape": shape[nm]}
        aggs[nm].close()
    del arena, outs, dst
    torch.cuda.empty_cache()
    return res


CASES = {"C": (16, 4194304, 32, "reduce", False), "Cround": (16, 4194304, 32, "round", False),
         "Caccum": (16, 4194304, 32, "accum", False), "F": (16, 8388608, 64, "reduce", False),
         "B": (16, 1048576, 8, "reduce", False), "D": (64, 4194304, 32, "reduce", True),
         "Dround": (64, 4194304, 32, "round", False), "Fround": (16, 8388608, 64, "round", False),
         "Bround": (16, 1048576, 8, "round", False)}

if __name__ == "__main__":
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    variant = sys.argv[2] if len(sys.argv) > 2 else "libipls_agg_halfalways.so"
    cases = sys.argv[3].split(",") if len(sys.argv) > 3 else ["C", "Cround", "Caccum", "F"]
    for c in cases:
        P, L, K, what, be = CASES[c]
        print(json.dumps(run(P, L, K, what, rounds, variant, be)), flush=True)
