"""Sharding of `-pa` partitions over the GPUs of a node, and the one exchange
step of the path: the replica combine.

Partitions are independent, so the data path is sharded with no collective:
rank r owns a contiguous block of partitions (``owner_of``), and every bucket
of a partition is folded on its owner's GPU.

The reference has one exchange step. Several aggregators may be responsible
for the same partition (``Replica_holders``). Each folds the buckets it
received into its ``Aggregated_Gradients`` and publishes that partial sum
(``IPLS.java:1423-1431``). Each then folds the other aggregators' partials
into ``Replicas_Gradients`` as they arrive (``Updater.java:40-44``), and
finishes with ``W = AGG + REP`` (``IPLS.java:1256``).

On one node those aggregators are GPUs. The owner pulls each replica's
partial over xGMI with RCCL point-to-point send/recv (``torch.distributed``,
backend "nccl" = RCCL) into a device buffer. It then folds the partials in
ascending replica-rank order on its own GPU:
``S = AGG_own + ((+0.0 + R_1) + R_2 ...)``, which is the reference's grouping
with a fixed arrival order, bit for bit. Only partials move (one L_p vector
per replica); k remote partials arrive on k distinct xGMI links.

``mode="rccl_reduce"`` instead sums all partials with RCCL's own reduction
(``dist.reduce``). It is faster to write but not bit-identical for more than
2 contributors, because RCCL picks the association. It is only for comparison.

The exchange code is written against two methods of the aggregator,
``export_partial`` and ``import_partial``. ``ipls.Aggregator`` implements
them on the GPU; the CPU tests drive this same code over gloo with a
stand-in.
"""
from __future__ import annotations

from dataclasses import dataclass

from . import _native as N


def owner_of(p: int, n_partitions: int, world: int) -> int:
    """Contiguous block mapping of -pa partitions to ranks: dev = p // ceil(P/G)."""
    per = -(-n_partitions // world)
    return p // per


def owned_partitions(rank: int, n_partitions: int, world: int) -> list[int]:
    return [p for p in range(n_partitions) if owner_of(p, n_partitions, world) == rank]


@dataclass(frozen=True)
class ReplicaPlan:
    """Who holds a partial of which partition.

    ``holders[p]`` lists the ranks that aggregated buckets of partition p
    (the owner included) in the order their partials are folded. This is
    ascending rank, the fixed stand-in for the reference's arrival order."""
    n_partitions: int
    world: int
    holders: dict

    @classmethod
    def build(cls, n_partitions: int, world: int, replicas: dict | None = None) -> "ReplicaPlan":
        replicas = replicas or {}
        h = {}
        for p in range(n_partitions):
            o = owner_of(p, n_partitions, world)
            h[p] = sorted({o, *replicas.get(p, ())})
        return cls(n_partitions, world, h)

    def exchanges(self):
        """[(p, owner, [replica ranks in fold order])] for partitions whose
        contributors span GPUs."""
        out = []
        for p, hs in self.holders.items():
            o = owner_of(p, self.n_partitions, self.world)
            others = [r for r in hs if r != o]
            if others:
                out.append((p, o, others))
        return out


def combine_replicas(agg, plan: ReplicaPlan, rank: int, *, device=None, mode: str = "fixed_order",
                     group=None) -> list[int]:
    """Run the replica exchange for this rank. Returns the partitions whose
    REP accumulator this rank filled (the ones it owns that had replicas).

    Every rank calls this with the same plan. Point-to-point operations are
    posted in one global order (partition ascending, replica ascending), so
    every pair of ranks sees its sends and receives in the same order and
    no cycle can deadlock. All receives are posted up front, so the k partials
    of a partition stream in concurrently over their own links. They are then
    folded strictly in replica order as each lands."""
    import torch
    import torch.distributed as dist

    exchanges = plan.exchanges()
    if mode == "rccl_reduce":
        # new_group is collective over the WORLD: every rank creates every group.
        groups = {}
        for p, owner, others in exchanges:
            key = tuple(sorted([owner, *others]))
            if key not in groups:
                groups[key] = dist.new_group(list(key)) if group is None else group
        filled = []
        for p, owner, others in exchanges:
            if rank not in (owner, *others):
                continue
            buf = torch.empty(agg.lengths[p], dtype=torch.float64, device=device)
            agg.export_partial(p, buf)
            dist.reduce(buf, dst=owner, op=dist.ReduceOp.SUM, group=groups[tuple(sorted([owner, *others]))])
            _landed(buf)
            if rank == owner:
                # buf = AGG_own + sum(R) in RCCL's association, stored as the
                # whole partial (REP stays 0) -- NOT bit-exact for > 2 ranks.
                agg.import_partial(p, buf, replace_agg=True)
                filled.append(p)
        return filled

    pending, sends, filled = [], [], []
    for p, owner, others in exchanges:
        L = agg.lengths[p]
        if rank == owner:
            for r in others:
                buf = torch.empty(L, dtype=torch.float64, device=device)
                pending.append((p, buf, dist.irecv(buf, src=r, group=group)))
            filled.append(p)
        elif rank in others:
            buf = torch.empty(L, dtype=torch.float64, device=device)
            agg.export_partial(p, buf)                    # AGG[p] -> the published partial
            sends.append((buf, dist.isend(buf, dst=owner, group=group)))
    for p, buf, work in pending:                          # fold in (partition, replica) order
        work.wait()
        _landed(buf)
        agg.import_partial(p, buf)                        # REP[p] += R_r (Updater.java:40-44)
    for _, work in sends:
        work.wait()
    return filled


def _landed(buf):
    """Make a received device tensor visible to the aggregator's own stream."""
    if getattr(buf, "is_cuda", False):
        import torch
        torch.cuda.current_stream(buf.device).synchronize()


def replica_tags() -> dict:
    """Accumulator targets used by the exchange (documentation aid)."""
    return {"partial_out": N.TGT_AGG, "partials_in": N.TGT_REP}
