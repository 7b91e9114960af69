"""CPU: world-size 2 and 4 `gloo` runs of the partition sharding and the
replica exchange (ipls.distributed).  The exchange code is the product code;
the aggregator behind it is a numpy stand-in built on the oracle (test
infrastructure), because the HIP aggregator needs a GPU.  The GPU half of the
exchange (export/import of partials through the C-ABI) is in
test_gpu_parity.py::test_export_import_partial."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import assert_bits_equal
from oracle import oracle as O


class NumpyAggregator:
    """Stand-in with the Aggregator surface the exchange uses (test only)."""

    def __init__(self, P, L):
        self.lengths = [L] * P
        self.agg = [np.zeros(L) for _ in range(P)]
        self.rep = [np.zeros(L) for _ in range(P)]

    def Update(self, g, p, from_clients=True):
        O.fold(self.agg[p] if from_clients else self.rep[p], np.asarray(g))

    def export_partial(self, p, t):
        t.copy_(torch.from_numpy(self.agg[p]))

    def import_partial(self, p, t, replace_agg=False):
        if replace_agg:
            self.agg[p] = t.numpy().copy()
        else:
            O.fold(self.rep[p], t.numpy())

    def finalize(self, p):
        return self.agg[p] + self.rep[p]

    def sync(self):
        pass


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def bucket(p, k, L):
    x = O.synth_bucket(L, p, k)
    x[0] = [1e16, 1.0, -1e16, 3.0][k % 4]        # order-sensitive element
    return x


def worker(rank, world, port, P, L, K, replicas, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ipls.distributed import ReplicaPlan, combine_replicas, finish_exchange, owner_of, start_exchange
    plan = ReplicaPlan.build(P, world, replicas)
    agg = NumpyAggregator(P, L)

    # each holder of partition p folds its own peers' buckets: holder h gets peers k with k % len == idx
    def fold(owned):
        for p, hs in plan.holders.items():
            if rank in hs and (owner_of(p, P, world) == rank) == owned:
                idx = hs.index(rank)
                for k in range(K):
                    if k % len(hs) == idx:
                        agg.Update(bucket(p, k, L), p)
    if mode == "overlapped":
        # the replica partials first; the owner's own folds run while the
        # exchange is in flight (start_exchange ... finish_exchange)
        fold(owned=False)
        ex = start_exchange(agg, plan, rank, device="cpu")
        fold(owned=True)
        filled = finish_exchange(ex)
    else:
        fold(owned=False)
        fold(owned=True)
        filled = combine_replicas(agg, plan, rank, device="cpu", mode=mode)
    res = {p: agg.finalize(p) for p in filled}
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def expected(P, L, K, world, replicas):
    from ipls.distributed import ReplicaPlan, owner_of
    plan = ReplicaPlan.build(P, world, replicas)
    out = {}
    for p, hs in plan.holders.items():
        if len(hs) == 1:
            continue
        parts = {}
        for idx, h in enumerate(hs):
            parts[h] = O.reduce([bucket(p, k, L) for k in range(K) if k % len(hs) == idx], L)
        own = owner_of(p, P, world)
        rep = O.reduce([parts[r] for r in hs if r != own], L)     # (+0.0 + R1) + R2 ...
        out[p] = parts[own] + rep                                  # AGG + REP (IPLS.java:1256)
    return out


@pytest.mark.parametrize("world,replicas,mode", [
    (2, {0: [1], 3: [0]}, "fixed_order"),
    (4, {0: [1, 2, 3], 5: [0, 3], 6: [1]}, "fixed_order"),
    (4, {0: [1, 2, 3], 5: [0, 3], 6: [1]}, "overlapped"),
])
def test_replica_exchange_fixed_order(world, replicas, mode):
    """fixed_order: combine_replicas after every fold.  overlapped: the
    exchange is started right after the replica partials are folded, the
    owners fold their own buckets while it is in flight, then it finishes --
    the same bits."""
    P, L, K = 8, 1031, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, P, L, K, replicas, mode, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    got = {}
    for _ in range(world):
        rank, res = q.get(timeout=120)
        got.update(res)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    exp = expected(P, L, K, world, replicas)
    assert sorted(got) == sorted(exp)
    for p in exp:
        assert_bits_equal(got[p], exp[p], f"partition {p}")


def shard_worker(rank, world, port, P, L, K, q):
    """The bench's config-E exchange (ReplicaPlan.spread + RankShard): each rank
    owns P partitions, folds their first K/2 peers, and is the replica of P
    other partitions (their last K/2 peers) in a second handle."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ipls.distributed import RankShard, ReplicaPlan, combine_replicas
    plan = ReplicaPlan.spread(P * world, world)
    rep_ids = plan.replicated_on(rank)
    own, rep = NumpyAggregator(P, L), NumpyAggregator(len(rep_ids), L)
    for i in range(P):
        for k in range(K // 2):
            own.Update(bucket(rank * P + i, k, L), i)
    for i, p in enumerate(rep_ids):
        for k in range(K // 2, K):
            rep.Update(bucket(p, k, L), i)
    shard = RankShard(own, rank * P, rep, rep_ids, device="cpu")
    filled = combine_replicas(shard, plan, rank, device="cpu")
    q.put((rank, len(rep_ids), {p: own.finalize(p - rank * P) for p in filled}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_spread_replica_shards(world):
    P, L, K = 6, 515, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=shard_worker, args=(r, world, port, P, L, K, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = {}
    for _ in range(world):
        rank, n_rep, res = q.get(timeout=120)
        assert n_rep == P                        # every rank replicates exactly P partitions
        got.update(res)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert sorted(got) == list(range(P * world))
    for p, w in got.items():
        own = O.reduce([bucket(p, k, L) for k in range(K // 2)], L)
        part = O.reduce([bucket(p, k, L) for k in range(K // 2, K)], L)
        assert_bits_equal(w, own + O.reduce([part], L), f"partition {p}")


def test_spread_plan_uses_every_link():
    from ipls.distributed import ReplicaPlan, owner_of
    for world, P in ((2, 16), (4, 16), (8, 16)):
        plan = ReplicaPlan.spread(P * world, world)
        for r in range(world):
            reps = plan.replicated_on(r)
            assert len(reps) == P
            srcs = {owner_of(p, P * world, world) for p in reps}
            assert srcs == set(range(world)) - {r}


def test_owner_mapping():
    from ipls.distributed import owned_partitions, owner_of
    # config E: 64 partitions on 4 GPUs -> 16 per GPU; F: 128 on 8
    assert [len(owned_partitions(r, 64, 4)) for r in range(4)] == [16] * 4
    assert owner_of(127, 128, 8) == 7 and owner_of(16, 128, 8) == 1
    assert sum(len(owned_partitions(r, 10, 4)) for r in range(4)) == 10


def test_replica_exchange_rccl_reduce_mode_two_ranks():
    """The RCCL-reduce comparison mode (here over gloo): with 2 contributors a
    single add, so it still matches AGG_own + R exactly."""
    P, L, K, world = 4, 257, 4, 2
    replicas = {1: [1]}   # owner of 1 is rank 0 -> rank 1 replica
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, P, L, K, replicas, "rccl_reduce", q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    got = {}
    for _ in range(world):
        rank, res = q.get(timeout=120)
        got.update(res)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    exp = expected(P, L, K, world, replicas)
    for p in exp:
        assert np.array_equal(got[p], exp[p]) or np.allclose(got[p], exp[p], rtol=0, atol=4e-16 * np.abs(exp[p]).max())


def gpu_worker(rank, world, port, P, L, K, replicas, q):
    """Two processes on one GPU: real HIP aggregators, gloo transport with
    host tensors (RCCL needs one GPU per rank)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ipls
    from ipls.distributed import ReplicaPlan, combine_replicas
    plan = ReplicaPlan.build(P, world, replicas)
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, device=0)
    for p, hs in plan.holders.items():
        if rank in hs:
            idx = hs.index(rank)
            for k in range(K):
                if k % len(hs) == idx:
                    agg.Update(bucket(p, k, L), p)
    filled = combine_replicas(agg, plan, rank, device="cpu")
    res = {}
    for p in filled:
        s, _ = agg.AggregatePartition(p, with_sum=True, sum_big_endian=False)
        res[p] = s
    agg.close()
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_replica_exchange_hip_aggregators_two_processes():
    if not torch.cuda.is_available():
        pytest.fail("-m gpu run without a visible GPU")
    P, L, K, world = 4, 20011, 5, 2
    replicas = {0: [1], 3: [0]}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=gpu_worker, args=(r, world, port, P, L, K, replicas, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = {}
    for _ in range(world):
        rank, res = q.get(timeout=300)
        got.update(res)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    exp = expected(P, L, K, world, replicas)
    assert sorted(got) == sorted(exp)
    for p in exp:
        assert_bits_equal(got[p], exp[p], f"partition {p}")


def test_rccl_reduce_rejects_a_caller_group():
    """dist.reduce over a caller-given group would hang the ranks
    outside it; the mode builds its own per-partition groups instead."""
    from ipls.distributed import ReplicaPlan, combine_replicas
    plan = ReplicaPlan.build(4, 2, {1: [1]})
    with pytest.raises(ValueError):
        combine_replicas(NumpyAggregator(4, 8), plan, 0, mode="rccl_reduce", group=object())


def test_ulp_distance_known_pairs():
    from ipls.distributed import ulp_distance
    a = torch.tensor([1.0, -1.0, 0.0, -0.0, 1e16, 5e-324, -5e-324], dtype=torch.float64)
    b = torch.tensor([np.nextafter(1.0, 2.0), np.nextafter(-1.0, -2.0), -0.0, 0.0,
                      np.nextafter(np.nextafter(1e16, 2e16), 2e16), -5e-324, 5e-324], dtype=torch.float64)
    assert ulp_distance(a, b).tolist() == [1, 1, 0, 0, 2, 2, 2]


def test_ulp_distance_saturates_for_far_opposite_signs():
    """opposite signs with |x| >= 2.0 are more than 2^63 - 1 ULP
    apart; the int64 difference must saturate, not wrap to a small or
    negative count."""
    from ipls.distributed import ulp_distance
    big = 2 ** 63 - 1
    a = torch.tensor([3.0, -1e300, 2.0, -2.0, 1.0, np.inf], dtype=torch.float64)
    b = torch.tensor([-3.0, 1e300, -2.0, 2.0, -1.0, -np.inf], dtype=torch.float64)
    d = ulp_distance(a, b).tolist()
    assert d[:4] == [big] * 4
    one = int(np.float64(1.0).view(np.int64))
    assert d[4] == 2 * one                       # 1.0 and -1.0: 2 x 0x3FF0... fits in int64
    assert d[5] == big
    assert all(x >= 0 for x in d)


def ulp_worker(rank, world, port, L, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ipls.distributed import rccl_reduce_ulp
    x = torch.from_numpy(bucket(0, rank, L))
    rep = rccl_reduce_ulp(x, rank, world, keep=True)
    q.put((rank, None if rep is None else {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in rep.items()}))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rccl_reduce_ulp_report(world):
    """the ULP report of the collective's own reduction against
    the fixed-order fold (here gloo's reduce on the CPU; on the GPU box the
    bench's N > 1 line runs it over RCCL).  The fixed order is checked against
    the oracle's fold, the reported distances against a numpy recount."""
    L = 1031
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=ulp_worker, args=(r, world, port, L, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert all(got[r] is None for r in range(1, world))
    rep = got[0]
    exp = np.zeros(L)
    for r in range(world):
        O.fold(exp, bucket(0, r, L))
    assert_bits_equal(rep["fixed"], exp)
    def line(v):
        i = v.view(np.int64)
        return np.where(i >= 0, i, -(i & 0x7FFFFFFFFFFFFFFF))
    d = np.abs(line(rep["sum"]) - line(exp))
    assert rep["max_ulp"] == int(d.max()) and rep["elements_differing"] == int((d != 0).sum())
    assert rep["elements"] == L and rep["contributors"] == world
    mag = sum(np.abs(bucket(0, r, L)) for r in range(world))
    err = np.abs(rep["sum"] - exp) / np.maximum(mag, np.finfo(np.float64).tiny)
    assert rep["max_err_vs_sum_of_magnitudes_u"] == pytest.approx(err.max() * 2.0 ** 53, abs=1e-3)
    assert rep["max_err_vs_sum_of_magnitudes_u"] <= 2 * (world - 1)   # any association: (n-1)u-bounded
    if world == 2:                                  # one add, commutative: no association to choose
        assert rep["bit_identical"] and rep["max_ulp"] == 0
