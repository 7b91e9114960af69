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
2 contributors, because RCCL picks the association. It is only for comparison;
``rccl_reduce_ulp`` measures how far it lands from the fixed order.

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

    @classmethod
    def spread(cls, n_partitions: int, world: int) -> "ReplicaPlan":
        """Every partition gets one replica aggregator on another GPU, spread
        so that each rank sends to and receives from every other rank: the
        q-th partition of rank o is replicated on ``(o + 1 + q % (G-1)) % G``.
        All G-1 xGMI links of a GPU carry partials at once (config E of
        SURVEY.md §8(d): contributors of a partition span GPUs)."""
        if world < 2:
            return cls.build(n_partitions, world)
        per = -(-n_partitions // world)
        replicas = {}
        for p in range(n_partitions):
            o, q = p // per, p % per
            replicas[p] = [(o + 1 + q % (world - 1)) % world]
        return cls.build(n_partitions, world, replicas)

    def replicated_on(self, rank: int) -> list[int]:
        """Partitions rank holds a replica partial of (it is not their owner)."""
        return [p for p, hs in self.holders.items()
                if rank in hs and owner_of(p, self.n_partitions, self.world) != rank]

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
    no cycle can deadlock. All sends and receives are posted as one batch, so
    the k partials of a partition stream in concurrently over their own links.
    Once the batch has landed they are folded strictly in replica order."""
    import torch
    import torch.distributed as dist

    exchanges = plan.exchanges()
    if mode == "rccl_reduce" and group is not None:
        # dist.reduce is collective over its group: a caller group that does not
        # hold exactly each partition's (owner, replicas) set would hang the
        # ranks outside it
        raise ValueError("rccl_reduce builds one group per (owner, replicas) set; pass group=None")
    if mode == "rccl_reduce":
        # new_group is collective over the WORLD: every rank creates every group.
        groups = {}
        for p, owner, others in exchanges:
            key = tuple(sorted([owner, *others]))
            if key not in groups:
                groups[key] = dist.new_group(list(key))
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

    return finish_exchange(start_exchange(agg, plan, rank, device=device, group=group))


@dataclass
class Exchange:
    """A replica exchange in flight (start_exchange -> finish_exchange)."""
    agg: object
    works: list
    ops: list
    landing: list
    filled: list


def start_exchange(agg, plan: ReplicaPlan, rank: int, *, device=None, group=None) -> Exchange:
    """First half of the fixed-order replica exchange: export this rank's
    replica partials and post every send and receive, without waiting.

    All of this rank's sends and receives go out as ONE batch
    (batch_isend_irecv: one RCCL group), so partials to and from every peer
    GPU move at once, each pair over its own xGMI link.  The ops are listed in
    the global (partition, replica) order on every rank.  The transfers run on
    RCCL's stream: work queued on the aggregator's own stream before
    finish_exchange (the owner's own folds, which the exchange never reads or
    writes) overlaps them."""
    import torch.distributed as dist

    ops, landing, filled = [], [], []
    bufs = getattr(agg, "transport_buffers", None)
    for p, owner, others in plan.exchanges():
        if rank == owner:
            L = agg.lengths[p]
            for r in others:
                buf = bufs(("in", p, r), L) if bufs else _empty(L, device)
                ops.append(dist.P2POp(dist.irecv, buf, r, group=group))
                landing.append((p, buf))
            filled.append(p)
        elif rank in others:
            L = agg.lengths[p]
            buf = bufs(("out", p, rank), L) if bufs else _empty(L, device)
            agg.export_partial(p, buf)                    # AGG[p] -> the published partial
            ops.append(dist.P2POp(dist.isend, buf, owner, group=group))
    works = dist.batch_isend_irecv(ops) if ops else []
    return Exchange(agg, works, ops, landing, filled)


def finish_exchange(ex: Exchange) -> list[int]:
    """Second half: wait for the transfers, then fold the landed partials into
    REP strictly in (partition, replica) order."""
    for work in ex.works:
        work.wait()
    if ex.ops:
        # RCCL's wait() only orders torch's stream after the group: block the
        # host on it, so received partials are visible to the aggregator's
        # stream and a send buffer is not refilled by the next export while
        # the send may still read it (a rank may only send)
        _landed(ex.ops[0].tensor)
    for p, buf in ex.landing:                             # fold in (partition, replica) order
        ex.agg.import_partial(p, buf)                     # REP[p] += R_r (Updater.java:40-44)
    if ex.landing:
        # the folds above are queued on the aggregator's stream and read the
        # transport buffers, which the next round's irecv (on RCCL's stream)
        # overwrites: wait for them before the buffers are handed out again
        ex.agg.sync()
    return ex.filled


def _empty(L, device):
    import torch
    return torch.empty(L, dtype=torch.float64, device=device)


def ulp_distance(a, b):
    """Per-element distance in units in the last place between two float64
    tensors: both bit patterns mapped onto one monotone integer line (a
    negative double -x maps to -(bits of x)), then subtracted.  +0.0 and -0.0
    are 0 apart; NaNs are not expected here (the fold inputs are finite).
    Values of opposite sign far apart (|x| >= 2.0 on both sides) are more
    than 2^63 - 1 ULP apart: the distance saturates there instead of
    wrapping in int64."""
    import torch

    def line(x):
        i = x.contiguous().view(torch.int64)
        return torch.where(i >= 0, i, -(i & 0x7FFFFFFFFFFFFFFF))
    la, lb = line(a), line(b)
    d = la - lb                                              # wraps on overflow
    over = (((la ^ lb) < 0) & ((la ^ d) < 0)) | (d == torch.iinfo(torch.int64).min)
    return torch.where(over, torch.full_like(d, torch.iinfo(torch.int64).max), d.abs())


def rccl_reduce_ulp(partial, rank: int, world: int, *, dst: int = 0, group=None, keep: bool = False) -> dict | None:
    """how far RCCL's own reduction (``ncclReduce(sum)``, here
    ``dist.reduce``) lands from the reference's fixed-order fold.

    Every rank contributes one partial of the same partition.  ``dst``
    receives RCCL's sum, gathers the partials themselves, folds them in rank
    order from +0.0 (``(+0.0 + R_0) + R_1 ...``, Updater.java:40-44 with a
    fixed arrival order) and returns the element-wise ULP distance between
    the two: ``max_ulp``, how many elements differ, and the largest error
    relative to the sum of the partials' magnitudes (in units u = 2^-53).  RCCL picks the
    association, so only 2 contributors are guaranteed 0 ULP (one add,
    commutative).  Collective over ``group``: every rank calls it; only
    ``dst`` gets the report (with both sums as ``sum``/``fixed`` if ``keep``)."""
    import torch
    import torch.distributed as dist

    red = partial.clone()
    dist.reduce(red, dst=dst, op=dist.ReduceOp.SUM, group=group)
    parts = [torch.empty_like(partial) for _ in range(world)] if rank == dst else None
    dist.gather(partial, parts, dst=dst, group=group)
    if rank != dst:
        return None
    fixed = torch.zeros_like(partial)                  # +0.0 start (START_ZERO)
    for r in range(world):                             # ascending rank = the fixed arrival order
        fixed = fixed + parts[r]                       # one IEEE add per element, as the fold does
    d = ulp_distance(red, fixed)
    # ULPs blow up where the partials cancel (a sum near 0 has tiny ULPs): the
    # error is also given against the sum of magnitudes, in units of 2^-53
    mag = torch.zeros_like(partial)
    for r in range(world):
        mag = mag + parts[r].abs()
    err = ((red - fixed).abs() / mag.clamp_min(torch.finfo(torch.float64).tiny)).max().item()
    rep = {"contributors": world, "max_ulp": int(d.max().item()),
           "max_err_vs_sum_of_magnitudes_u": round(err * 2.0 ** 53, 3),
           "elements_differing": int((d != 0).sum().item()), "elements": int(partial.numel()),
           "bit_identical": bool(torch.equal(red.view(torch.int64), fixed.view(torch.int64)))}
    if keep:
        rep.update(sum=red, fixed=fixed)
    return rep


class RankShard:
    """One rank's handles under node-wide partition ids, for combine_replicas.

    ``own`` holds the partitions this GPU owns, ``[first, first + n)`` as local
    ``0..n-1``; ``rep`` holds the partials it aggregates as a replica for other
    GPUs' partitions (``rep_ids[i]`` is local partition ``i``).  Transport
    buffers are allocated once and reused across rounds."""

    def __init__(self, own, first: int, rep=None, rep_ids=(), device=None):
        self.own, self.first, self.rep = own, first, rep
        self.rep_index = {p: i for i, p in enumerate(rep_ids)}
        self.device = device
        self.lengths = {first + i: L for i, L in enumerate(own.lengths)}
        if rep is not None:
            self.lengths.update({p: rep.lengths[i] for p, i in self.rep_index.items()})
        self._bufs = {}

    def transport_buffers(self, key, L):
        import torch
        b = self._bufs.get(key)
        if b is None:
            b = self._bufs[key] = torch.empty(L, dtype=torch.float64, device=self.device)
        return b

    def export_partial(self, p, tensor):
        self.rep.export_partial(self.rep_index[p], tensor)

    def import_partial(self, p, tensor, replace_agg=False):
        self.own.import_partial(p - self.first, tensor, replace_agg=replace_agg)

    def sync(self):
        self.own.sync()
        if self.rep is not None:
            self.rep.sync()


def _landed(buf):
    """Make a received device tensor visible to the aggregator's own stream."""
    if getattr(buf, "is_cuda", False):
        import torch
        torch.cuda.current_stream(buf.device).synchronize()


def replica_tags() -> dict:
    """Accumulator targets used by the exchange (documentation aid)."""
    return {"partial_out": N.TGT_AGG, "partials_in": N.TGT_REP}
