#!/usr/bin/env python3
"""Generate the committed golden fixtures of tests/golden/ (run in the build
container, where /root/reference exists).

Outputs (all data, no reference source):
  ethmodel.f64be.gz  -- the 443,610 big-endian doubles of the reference's
                        MNIST_Partitioned_Dataset/ETHModel ([D payload of the
                        Java-serialised DoubleArrayAsList, extracted by
                        oracle.parse_ethmodel; nothing in the file is executed)
  golden.npz         -- small explicit cases: inputs and expected outputs
  golden.json        -- metadata, checksums of the full-size synthetic configs,
                        SHA-256 of the config-A outputs

  ref_scheduler.ser  -- the reference's own `Scheduler` file, byte for byte: a
                        Java ObjectOutputStream of an org.javatuples.Pair (data;
                        pins the Pair/Tuple/Object[]/Integer/Number/
                        Arrays$ArrayList descriptors of oracle/javaser.py)
  ref_ethmodel_head.bin -- the first 136 bytes of ETHModel (its stream header,
                        incl. the `[D` descriptor)

Expected values come from the Python restatement (oracle/oracle.py) and are
cross-checked bit for bit against the C restatement (oracle/ipls_oracle.c)
before anything is written.  Parity status: unpinned.
"""
from __future__ import annotations

import gzip
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

from oracle import oracle as O  # noqa: E402

SEED = O.SEED


def bits(x):
    return np.ascontiguousarray(x, dtype=np.float64).view(np.uint64)


def same(a, b):
    return np.array_equal(bits(a), bits(b))


def config_a(model: np.ndarray):
    """Config A (BASELINE configs[0]): ETHModel, -pa 3 -n 3.  Peer k's update
    vector is model + synth noise(p=0,k); one aggregator owns all 3
    partitions, folds the 3 peers' OrganizeGradients buckets in peer order,
    finalizes (REP empty) and GetPartitions divides by the count slot (3.0)."""
    M, P, K = len(model), 3, 3
    peers = [model + O.synth_bucket(M + 1, 0, k)[:M] for k in range(K)]
    parts = [O.organize_gradients(g, M, P) for g in peers]
    sums = []
    for p in range(P):
        L = O.partition_len(M, P, p)
        s = O.reduce([parts[k][p] for k in range(K)], L, O.START_ZERO)
        s_c = O.c_reduce([parts[k][p] for k in range(K)], L, O.START_ZERO)
        assert same(s, s_c)
        agg, rep = s.copy(), np.zeros(L)
        w, wa = np.zeros(L), np.zeros(L)
        O.aggregate_partition(agg, rep, w, wa)
        sums.append(w)
    avg = O.get_partitions(sums)
    for p in range(P):
        assert same(O.divide(sums[p]), O.c_divide(sums[p]))
    return peers, sums, avg


def edge_cases():
    cases = {}
    # signed zero: ZERO start gives +0.0, FIRST start keeps -0.0
    nz = np.full(5, -0.0)
    cases["szero_bufs"] = np.stack([nz, nz])
    cases["szero_zero"] = O.reduce([nz, nz], 5, O.START_ZERO)
    cases["szero_first"] = O.reduce([nz, nz], 5, O.START_FIRST)
    # cancellation: fixed order matters ((0+1e16)+1)-1e16 = 0, not 1
    cb = [np.array([1e16, 1.0, 3.0, 1.0]), np.array([1.0, 1e16, -1e-300, 1.0]),
          np.array([-1e16, -1e16, 5e-324, 1.0])]
    cases["cancel_bufs"] = np.stack(cb)
    cases["cancel_zero"] = O.reduce(cb, 4, O.START_ZERO)
    cases["cancel_first"] = O.reduce(cb, 4, O.START_FIRST)
    # subnormals, infinities, NaN
    sb = [np.array([5e-324, 2.2e-308, -np.inf, np.nan, 1.0, 0.0, 1.0]),
          np.array([5e-324, -2.2e-308, np.inf, 1.0, np.inf, -0.0, 1.0]),
          np.array([-1e-323, 1e-310, 1.0, 2.0, -np.inf, 0.0, 1.0])]
    cases["special_bufs"] = np.stack(sb)
    cases["special_zero"] = O.reduce(sb, 7, O.START_ZERO)
    # divide: count 0 -> passthrough, -0.0 also (Java ==), NaN count -> NaN
    w = np.array([3.0, -6.0, 1e-320, 3.0])
    cases["div_w"] = w
    cases["div_out"] = O.divide(w)
    cases["div_zero_w"] = np.array([3.0, -6.0, 0.0])
    cases["div_zero_out"] = O.divide(cases["div_zero_w"])
    cases["div_nzero_w"] = np.array([3.0, -6.0, -0.0])
    cases["div_nzero_out"] = O.divide(cases["div_nzero_w"])
    cases["div_secure_w"] = np.array([3e12, -6e12, 7.0, 3.0])
    cases["div_secure_out"] = O.divide(cases["div_secure_w"], secure=True)
    # encode (secure mode, Middleware.java:196-210)
    e = np.array([-11.0, -10.0, 0.5, 10.0, 10.5, -0.0])
    cases["enc_in"] = e
    cases["enc_out"] = O.encode_secure(e)
    # OrganizeGradients geometry: M=10, P=4 (chunk 3, last partition 2 long)
    flat = np.arange(1.0, 11.0)
    og = O.organize_gradients(flat, 10, 4)
    for p, v in og.items():
        cases[f"org10x4_p{p}"] = v
    # M=12, P=4: chunk 4; last partition count-slot only (length 1)
    og = O.organize_gradients(np.arange(1.0, 13.0), 12, 4)
    for p, v in og.items():
        cases[f"org12x4_p{p}"] = v
    # frame bytes (Marshall_Packet double[], pid 3) with origin id
    g = np.array([1.5, -0.0, np.inf, 2.0 ** -1074])
    fr = O.frame_encode(g, 7, 42, 3, b"QmPeerOrigin")
    cases["frame_g"] = g
    cases["frame_bytes"] = np.frombuffer(fr, dtype=np.uint8)
    # BE codec: raw NaN bits kept by putDouble, canonicalised by writeDouble
    nanv = np.array([1.0, np.nan, -np.nan]).copy()
    nanv.view(np.uint64)[2] = np.uint64(0xFFF0000000000001)  # signalling NaN pattern
    cases["be_in"] = nanv
    cases["be_raw"] = np.frombuffer(O.be_encode(nanv), dtype=np.uint8)
    cases["be_canon"] = np.frombuffer(O.be_encode_canonical(nanv), dtype=np.uint8)
    return cases


def synth_small(meta):
    """Synthetic reduce cases whose inputs are regenerated from the counter
    formula; outputs stored (odd lengths hit the scalar tail path), or only
    their checksum for the larger ones."""
    out = {}
    meta["synth_checksum"] = {}
    for (P, L, K) in [(3, 1, 2), (2, 2, 1), (4, 1031, 8), (2, 4096, 5), (1, 517, 33), (2, 70001, 3),
                      (1, 262147, 12)]:
        for p in range(P):
            bufs = [O.synth_bucket(L, p, k) for k in range(K)]
            for k in range(K):
                assert same(bufs[k], O.c_synth_bucket(L, p, k))
            for mode, name in [(O.START_ZERO, "zero"), (O.START_FIRST, "first")]:
                s = O.reduce(bufs, L, mode)
                assert same(s, O.c_reduce(bufs, L, mode))
                key = f"synth_P{P}_L{L}_K{K}_p{p}_{name}"
                if L <= 4096:
                    out[key] = s
                else:
                    meta["synth_checksum"][key] = O.checksum(s)
    return out


def main():
    ref = O.ethmodel_path()
    if ref is None:
        sys.exit("reference ETHModel not found; run in the build container")
    model = O.parse_ethmodel(ref.read_bytes())
    assert model.shape == (443610,)
    (HERE / "ethmodel.f64be.gz").write_bytes(gzip.compress(model.astype(">f8").tobytes(), 9, mtime=0))
    (HERE / "ref_ethmodel_head.bin").write_bytes(ref.read_bytes()[:136])
    sched = ref.parent.parent / "Scheduler"            # <reference>/Scheduler, written by Bootstraper_Services
    (HERE / "ref_scheduler.ser").write_bytes(sched.read_bytes())

    meta = {"seed": SEED, "parity": "unpinned (no reference golden vectors; SURVEY.md §8(c))"}
    peers, sums, avg = config_a(model)
    meta["config_a"] = {
        "model_size": 443610, "partitions": 3, "peers": 3,
        "partition_len": [len(s) for s in sums],
        "sum_sha256": [hashlib.sha256(s.astype(">f8").tobytes()).hexdigest() for s in sums],
        "avg_sha256": hashlib.sha256(avg.astype(">f8").tobytes()).hexdigest(),
        "wire_sha256": hashlib.sha256(O.be_encode_canonical(avg)).hexdigest(),
        "sum_checksum": [O.checksum(s) for s in sums],
        "avg_checksum": O.checksum(avg),
    }
    cases = edge_cases()
    cases.update(synth_small(meta))
    np.savez(HERE / "golden.npz", **cases)

    # full-size synthetic configs: per-partition checksum of the ZERO-start
    # fixed-order sum (C oracle, OpenMP over elements, per-element order intact)
    full = {}
    for name, (P, L, K) in {"B": (16, 1048576, 8), "C": (16, 4194304, 32), "D": (64, 4194304, 32)}.items():
        full[name] = {"partitions": P, "bucket_len": L, "peers": K,
                      "sum_checksum": [O.c_synth_sum_checksum(L, p, K) for p in range(P)]}
        print(name, full[name]["sum_checksum"][:2], flush=True)
    # the fused round's averages (GetPartitions divide of the same sums), config C
    full["C"]["avg_checksum"] = [O.c_synth_avg_checksum(4194304, p, 32) for p in range(16)]
    # D's first 16 partitions are C's (the counter formula is keyed by (p, k, i))
    assert full["D"]["sum_checksum"][:16] == full["C"]["sum_checksum"]
    # spot-check the C checksum path against the Python fold on one partition of B
    bufs = [O.synth_bucket(1048576, 3, k) for k in range(8)]
    assert O.checksum(O.reduce(bufs, 1048576)) == full["B"]["sum_checksum"][3]
    meta["full"] = full
    (HERE / "golden.json").write_text(json.dumps(meta, indent=1) + "\n")
    print("wrote", sorted(p.name for p in HERE.iterdir()))


if __name__ == "__main__":
    main()
