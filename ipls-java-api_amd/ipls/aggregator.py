"""Host-side mirror of the reference's aggregation interface, over the C-ABI.

The reference keeps the aggregator state in static maps (PeerData.java:137-189)
and reduces inside IPLS / Updater methods.  ``Aggregator`` owns the same state
on one GPU (one ``ipls_agg`` handle) and exposes the reference's operations
under the reference's names, with the reference's argument meaning:

=====================================  =========================================
reference (src/main/java/)             here
=====================================  =========================================
IPLS.InitializeWeights(List) 1880      ``InitializeWeights(model)``
IPLS.OrganizeGradients 1018            ``OrganizeGradients(gradients)``
IPLS.UpdateGradient 1703 (1737-1743)   ``UpdateGradient(gradients, auth_list)``
Updater._Update 31 (from_clients)      ``Update(gradient, partition, from_clients)``
Download_Scheduler 245-268             ``OtherReplicaGradients(p, aggregator, g)``
IPLS.Collect_Replicas 1217             ``Collect_Replicas()``
IPLS.Update_Client_WaitAck_List 1556   ``PromoteFuture(auth_list)``
Updater.run indirect 176-187           ``UpdateIndirect(file_bytes, partition)``
Decentralized_Storage_Receiver 239     ``Merge(partition, buckets)``
IPLS.AggregatePartition 1248           ``AggregatePartition(partition)``
Download_Scheduler.cache_partition 752 ``cache_partition(partition, data)``
IPLS.GetPartitions 1080 (1140-1174)    ``GetPartitions()``
=====================================  =========================================

Host buffers are numpy arrays (``float64`` for doubles, ``uint8``/bytes for the
big-endian IPFS file format and pubsub frames).  Device buffers may be passed
as ``DeviceBuffer`` (raw pointer + length) -- e.g. ``torch`` CUDA tensors via
``DeviceBuffer.from_tensor``.  Every call goes to the HIP library; a missing
library raises at construction.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _native as N


@dataclass
class DeviceBuffer:
    """A device-resident operand: address, element count, big-endian or not.

    The handle's HIP stream is non-blocking (include/ipls_agg.h): bytes
    written by torch or the null stream must be complete before the call
    that reads them (``torch.cuda.synchronize()``, or an event the handle's
    stream ``Aggregator.stream`` waits on)."""
    ptr: int
    n: int
    big_endian: bool = False

    @classmethod
    def from_tensor(cls, t, big_endian: bool = False) -> "DeviceBuffer":
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("need a contiguous device tensor")
        return cls(int(t.data_ptr()), t.numel() * t.element_size() // 8, big_endian)

    @property
    def kind(self) -> int:
        return N.DEV_BE if self.big_endian else N.DEV_F64


def _bucket_table(buckets, lengths, p_first: int):
    """(flat pointer list, k) of a batched call's bucket table: ``buckets[q]``
    are the k device buckets of partition ``p_first + q``.  The C-ABI takes
    bare pointers and reads L_p doubles from each (include/ipls_agg.h), so a
    DeviceBuffer shorter than its partition is refused here, before any
    launch could read past it.  Raw integer addresses are the caller's
    contract; partitions out of range are left to the library's range check."""
    n_parts = len(buckets)
    k = len(buckets[0]) if n_parts else 0
    flat = []
    for q, row in enumerate(buckets):
        if len(row) != k:
            raise ValueError("every partition needs the same number of buckets")
        p = p_first + q
        need = lengths[p] if 0 <= p < len(lengths) else 0
        for b in row:
            if isinstance(b, DeviceBuffer):
                if b.n < need:
                    raise ValueError(f"partition {p} needs buckets of {need} doubles, a DeviceBuffer holds {b.n}")
                flat.append(b.ptr)
            else:
                flat.append(int(b))
    return flat, k


def _host_operand(x, big_endian: bool):
    """(pointer, n_doubles, kind, keepalive) for a host operand."""
    if isinstance(x, (bytes, bytearray, memoryview)):
        a = np.frombuffer(x, dtype=np.uint8)
    else:
        a = np.asarray(x)
    if a.dtype == np.uint8:          # raw bytes are always BE doubles (IPFS file format)
        a = np.ascontiguousarray(a)
        return a.ctypes.data, a.nbytes // 8, N.HOST_BE, a
    if a.dtype.byteorder == ">":
        a = np.ascontiguousarray(a)
        return a.ctypes.data, a.size, N.HOST_BE, a
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a.ctypes.data, a.size, N.HOST_F64, a


def _operand(x, big_endian: bool = False):
    if isinstance(x, DeviceBuffer):
        return x.ptr, x.n, x.kind, x
    return _host_operand(x, big_endian)


def _callback(caught: list, fn, *args) -> int:
    """Body of a chunk source/sink called from C: 0 to go on, 1 to stop.  No
    exception may unwind through the library, so any -- a socket's EOFError
    or timeout, a KeyboardInterrupt -- is kept and stops the call; the Python
    caller re-raises it (_reraise) once the library has returned."""
    if caught:
        return 1
    try:
        return 0 if fn(*args) else 1
    except BaseException as e:   # noqa: BLE001 -- re-raised after the library call
        caught.append(e)
        return 1


def _reraise(caught: list) -> None:
    if caught:
        raise caught[0]


class Aggregator:
    """One aggregator's partition accumulators on one MI355X.

    ``model_size``/``n_partitions`` follow Middleware's ``-pa`` semantics and the
    reference chunk rule (IPLS.java:1019-1028).  ``bucket_len`` (with
    model_size=0) selects the synthetic geometry of SURVEY.md §8: every
    partition ``bucket_len`` doubles including the count slot."""

    def __init__(self, model_size: int = 0, n_partitions: int = 1, *, max_peers: int = 0,
                 partial_aggregation: int = 0, secure: bool = False, device: int = 0,
                 bucket_len: int = 0, devices=None, library=None):
        """``devices``: a list of HIP device ordinals shards the partitions over
        several GPUs in contiguous blocks (cfg.devices, ipls_shard_plan); a
        device may repeat (several shards on one GPU).  ``library``: another
        build of the C-ABI (``ipls._native.load(path)``) for same-process A/B
        runs; default the in-tree library."""
        self._lib = library if library is not None else N.lib()
        devs = None if devices is None else (ctypes.c_int32 * len(devices))(*devices)
        cfg = N.AggCfg(model_size=model_size, n_partitions=n_partitions, max_peers=max_peers,
                       partial_aggregation=partial_aggregation, secure=int(bool(secure)),
                       device=device, flags=0, bucket_len=bucket_len,
                       devices=devs, n_devices=0 if devices is None else len(devices), reserved=0)
        h = ctypes.c_void_p()
        N.check(self._lib.ipls_agg_open(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self._hv = h.value                      # the handle's address, for ipls._fast
        self._fast = N.fast() if library is None else None
        self.model_size = model_size
        self.n_partitions = n_partitions
        self.secure = bool(secure)
        self.device = device if devices is None else devices[0]
        self.devices = [device] if devices is None else list(devices)
        self.lengths = [self.partition_len(p) for p in range(n_partitions)]
        self.offsets = [self.partition_offset(p) for p in range(n_partitions)]
        self.flat_size = max(o + L - 1 for o, L in zip(self.offsets, self.lengths))

    # ---- lifetime ----
    def close(self):
        if getattr(self, "_h", None):
            self._hv = None
            self._lib.ipls_agg_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc >= 0:                                # the per-call fast path (UpdateAsync per arrival)
            return rc
        if self._lib is not N.lib():               # a variant build keeps its own error slot
            msg = self._lib.ipls_agg_last_error(None)
            raise N.IplsError(rc, msg.decode(errors="replace") if msg else "")
        return N.check(rc, self._h)

    @property
    def handle(self):
        return self._h

    @property
    def stream(self) -> int:
        return int(self._lib.ipls_agg_stream(self._h) or 0)

    def sync(self):
        self._chk(self._lib.ipls_agg_sync(self._h))

    # ---- geometry (IPLS.java:1019-1028) ----
    def partition_len(self, p: int) -> int:
        v = ctypes.c_int64()
        self._chk(self._lib.ipls_agg_partition_len(self._h, p, ctypes.byref(v)))
        return v.value

    def partition_offset(self, p: int) -> int:
        v = ctypes.c_int64()
        self._chk(self._lib.ipls_agg_partition_offset(self._h, p, ctypes.byref(v)))
        return v.value

    # ---- reference operations ----
    def InitializeWeights(self, model, big_endian: bool = False):
        """IPLS.java:1880-1901 (model = List<Double>, or read_file's raw BE bytes)."""
        ptr, n, kind, keep = _operand(model, big_endian)
        self._chk(self._lib.ipls_agg_load_model(self._h, ptr, n, kind))

    def OrganizeGradients(self, gradients, big_endian_out: bool = False) -> dict[int, np.ndarray]:
        """IPLS.java:1018-1040: {p: double[L_p]} with the count slot 1.0."""
        ptr, n, kind, keep = _operand(gradients)
        out = {}
        for p in range(self.n_partitions):
            L = self.lengths[p]
            if big_endian_out:
                buf = np.empty(8 * L, dtype=np.uint8)
                dk = N.HOST_BE
            else:
                buf = np.empty(L, dtype=np.float64)
                dk = N.HOST_F64
            self._chk(self._lib.ipls_agg_split(self._h, ptr, n, kind, p, buf.ctypes.data, dk))
            out[p] = buf
        return out

    def UpdateGradient(self, gradients, auth_list):
        """Own-partition accumulate of IPLS.UpdateGradient (IPLS.java:1737-1743).
        ``gradients=None`` is the "did not train in time" call (no-op)."""
        owned = np.ascontiguousarray(np.asarray(list(auth_list), dtype=np.int32))
        if gradients is None:
            return
        ptr, n, kind, keep = _operand(gradients)
        self._chk(self._lib.ipls_agg_update_gradient(
            self._h, ptr, n, kind, owned.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(owned)))

    def Update(self, gradient, partition: int, from_clients: bool = True, *, frame: bool = False,
               pair: bool = False, from_future: bool = False):
        """Updater._Update: client buckets fold into Aggregated_Gradients
        (Updater.java:115-117), replica partial sums into Replicas_Gradients
        (Updater.java:40-44), and a client's bucket for a later iteration
        (``from_future=True``) into Aggregated_Gradients_from_future
        (Updater.java:99-101).  ``gradient`` may be doubles, big-endian file
        bytes (GetParameters input), a pubsub frame (``frame=True``) or a
        DeviceBuffer.  ``None`` is a no-op, as in the reference."""
        if gradient is None:
            return
        target = N.TGT_FUTURE if from_future else (N.TGT_AGG if from_clients else N.TGT_REP)
        if frame or pair:       # a pubsub frame / a Java-serialised Pair<Integer,double[]> partial update
            a = np.frombuffer(bytes(gradient), dtype=np.uint8)
            self._chk(self._lib.ipls_agg_accumulate(self._h, partition, target, a.ctypes.data,
                                                    a.size, N.HOST_PAIR if pair else N.HOST_FRAME))
            return
        ptr, n, kind, keep = _operand(gradient)
        if self._fast is not None:
            rc = self._fast.accumulate(self._hv, partition, target, ptr, n, kind)
            if rc < 0:
                self._chk(rc)
            return
        self._chk(self._lib.ipls_agg_accumulate(self._h, partition, target, ptr, n, kind))

    def UpdateAsync(self, gradient, partition: int, from_clients: bool = True, *, big_endian: bool = True) -> int:
        """Updater._Update without waiting.  ``gradient`` is a PinnedBuffer (the
        `ipfs cat` bytes, big-endian unless ``big_endian=False``) that the fold
        reads over PCIe, or a DeviceBuffer that is queued and folded with the
        partition's other queued buckets in one launch (set_coalesce).  Returns
        a ticket; keep the buffer until Wait(ticket)."""
        target = N.TGT_AGG if from_clients else N.TGT_REP
        if self._fast is not None and isinstance(gradient, DeviceBuffer):
            t = self._fast.accumulate_async(self._hv, partition, target, gradient.ptr, gradient.n,
                                            N.DEV_BE if gradient.big_endian else N.DEV_F64)
            if t < 0:
                self._chk(t)
            return t
        t = ctypes.c_uint64()
        if isinstance(gradient, DeviceBuffer):
            rc = self._lib.ipls_agg_accumulate_async(self._h, partition, target, gradient.ptr, gradient.n,
                                                     N.DEV_BE if gradient.big_endian else N.DEV_F64, ctypes.byref(t))
            if rc < 0:
                self._chk(rc)
            return t.value
        if not isinstance(gradient, PinnedBuffer):
            raise TypeError("UpdateAsync takes a PinnedBuffer (ipls_host_alloc memory) or a DeviceBuffer")
        if self._fast is not None:
            t = self._fast.accumulate_async(self._hv, partition, target, gradient.ptr, gradient.nbytes // 8,
                                            N.HOST_BE if big_endian else N.HOST_F64)
            if t < 0:
                self._chk(t)
            return t
        self._chk(self._lib.ipls_agg_accumulate_async(self._h, partition, target, gradient.ptr,
                                                      gradient.nbytes // 8,
                                                      N.HOST_BE if big_endian else N.HOST_F64, ctypes.byref(t)))
        return t.value

    def UpdateAsyncMany(self, arrivals, from_clients: bool = True, *, big_endian: bool = True) -> int:
        """UpdateAsync for several arrivals in order, e.g. every bucket the
        Updater's queue holds at once (one peer's partitions): ``arrivals`` is
        a sequence of (gradient, partition) with DeviceBuffer or PinnedBuffer
        gradients.  Through ipls._fast it is one Python -> C transition for
        the whole list; the folds, their order and their bits are those of
        one UpdateAsync per arrival.  Returns the last ticket (0 for an empty
        list).  An error stops at the failing arrival: the earlier ones are
        queued, as after the same UpdateAsync calls."""
        target = N.TGT_AGG if from_clients else N.TGT_REP
        items = []
        for g, p in arrivals:
            if isinstance(g, DeviceBuffer):
                items.append((p, g.ptr, g.n, N.DEV_BE if g.big_endian else N.DEV_F64))
            elif isinstance(g, PinnedBuffer):
                items.append((p, g.ptr, g.nbytes // 8, N.HOST_BE if big_endian else N.HOST_F64))
            else:
                raise TypeError("UpdateAsyncMany takes DeviceBuffer or PinnedBuffer gradients")
        if not items:
            return 0
        if self._fast is not None:
            t = self._fast.accumulate_async_many(self._hv, target, items)
            if isinstance(t, tuple):
                self._chk(t[0])
            return t
        t = ctypes.c_uint64()
        for p, ptr, n, kind in items:
            self._chk(self._lib.ipls_agg_accumulate_async(self._h, p, target, ptr, n, kind, ctypes.byref(t)))
        return t.value

    def UpdateChunked(self, partition: int, n: int, source, *, big_endian: bool = True, from_clients: bool = True,
                      chunk: int = 1 << 19):
        """Updater._Update of one bucket that the caller produces chunk by
        chunk, as ONE library call (ipls_agg_accumulate_chunked): ``source(dst,
        offset, count)`` writes the bucket's values [offset, offset + count)
        -- 8*count bytes, big-endian unless ``big_endian=False`` -- at the
        address ``dst`` (the library's pinned ring) and returns True; False
        stops the call with nothing folded.  ``n`` is the bucket's length
        (shorter than the partition: ArrayIndexOutOfBounds, before any
        source call)."""
        target = N.TGT_AGG if from_clients else N.TGT_REP
        caught = []

        @N.CHUNK_SOURCE
        def cb(ctx, dst, off, cnt):
            return _callback(caught, source, dst, off, cnt)
        rc = self._lib.ipls_agg_accumulate_chunked(self._h, partition, target, n,
                                                   N.HOST_BE if big_endian else N.HOST_F64, chunk, cb, None)
        _reraise(caught)
        self._chk(rc)

    def GetPartitionsChunked(self, sink, *, wire: bool = False, chunk: int = 1 << 19):
        """GetPartitions (IPLS.java:1159-1174) handed to ``sink(ptr, offset,
        count)`` chunk by chunk in model order (ipls_agg_get_partitions_chunked,
        or with ``wire=True`` the Middleware task-3 writeDouble stream,
        ipls_agg_get_partitions_wire_chunked): 8*count bytes at ``ptr`` in
        the library's pinned ring, valid during the call; the sink returns
        True to go on."""
        caught = []

        @N.CHUNK_SINK
        def cb(ctx, vals, off, cnt):
            return _callback(caught, sink, ctypes.cast(vals, ctypes.c_void_p).value, off, cnt)
        fn = self._lib.ipls_agg_get_partitions_wire_chunked if wire else self._lib.ipls_agg_get_partitions_chunked
        rc = fn(self._h, chunk, cb, None)
        _reraise(caught)
        self._chk(rc)

    def AggregatePartitionChunked(self, partition: int, sink, *, big_endian: bool = True, chunk: int = 1 << 19):
        """AggregatePartition with the committed sum handed to ``sink(ptr,
        offset, count)`` chunk by chunk, as one call (ipls_agg_finalize_chunked:
        no other caller's call lands between the sum and its bytes)."""
        caught = []

        @N.CHUNK_SINK
        def cb(ctx, vals, off, cnt):
            return _callback(caught, sink, ctypes.cast(vals, ctypes.c_void_p).value, off, cnt)
        rc = self._lib.ipls_agg_finalize_chunked(self._h, partition, N.HOST_BE if big_endian else N.HOST_F64,
                                                 chunk, cb, None)
        _reraise(caught)
        self._chk(rc)

    def flush(self):
        """Launch the folds of every queued device bucket now (no wait)."""
        self._chk(self._lib.ipls_agg_flush(self._h))

    def set_coalesce(self, max_group: int):
        """Largest group of queued device buckets folded per partition in one launch."""
        self._chk(self._lib.ipls_agg_set_coalesce(self._h, max_group))

    def Wait(self, ticket: int):
        """Block until the UpdateAsync fold ``ticket`` (and all before it) is done."""
        self._chk(self._lib.ipls_agg_wait(self._h, ticket))

    def UpdateIndirect(self, file_bytes, partition: int, from_clients: bool = True, *,
                       from_future: bool = False):
        """Updater.run for a queue item with only a hash (Updater.java:176-187):
        GetParameters(hash, Gradient_Buff) then _Update(Gradient_Buff, ...),
        with the reference's reusable Gradient_Buff (a short file folds the
        previous request's tail; a file longer than the buffer raises the
        AIOOBE after overwriting it).  ``file_bytes``: the `ipfs cat` bytes."""
        target = N.TGT_FUTURE if from_future else (N.TGT_AGG if from_clients else N.TGT_REP)
        if isinstance(file_bytes, PinnedBuffer):
            ptr, nb = file_bytes.ptr, file_bytes.nbytes
        else:
            a = np.frombuffer(bytes(file_bytes), dtype=np.uint8)
            ptr, nb = (a.ctypes.data if a.size else None), a.size
        self._chk(self._lib.ipls_agg_update_indirect(self._h, partition, target, ptr, nb))

    def PromoteFuture(self, partitions):
        """End of Update_Client_WaitAck_List (IPLS.java:1556-1562): for p in
        ``partitions`` (the Auth_List), Aggregated_Gradients[p] =
        Aggregated_Gradients_from_future[p], and the latter is zeroed."""
        parts = np.ascontiguousarray(list(partitions), dtype=np.int32)
        self._chk(self._lib.ipls_agg_promote_future(
            self._h, parts.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), parts.size))

    def ingest_pubsub(self, messages, *, from_clients: bool = True, layers: int = 2, partitions=None):
        """ThreadReceiver (IPLS.java:851-866, 453-465): a batch of pubsub
        'data' texts -> base64url x layers -> GET_GRADIENTS frame -> fold, all
        on the GPU.  Returns (number folded, per-message status)."""
        msgs = [np.frombuffer(bytes(m), dtype=np.uint8) for m in messages]
        n = len(msgs)
        ptrs = (ctypes.c_void_p * max(1, n))(*[m.ctypes.data if m.size else None for m in msgs])
        lens = (ctypes.c_int64 * max(1, n))(*[m.size for m in msgs])
        st = (ctypes.c_int32 * max(1, n))()
        parts = None
        if partitions is not None:
            parts = (ctypes.c_int32 * max(1, n))(*partitions)
        target = N.TGT_AGG if from_clients else N.TGT_REP
        k = self._chk(self._lib.ipls_agg_ingest_pubsub(self._h, target, ptrs, lens, n, layers, parts, st))
        return k, list(st)[:n]

    # ---- -async true variants (Updater.java:57-69, 197-199) ----
    ASYNC_DECAY = 0.75      # Updater.java:58
    LEAVING_A = 0.6         # Updater.java:17 (field a)

    def UpdateAsyncReplica(self, gradient, partition: int):
        """Async replica fold: W = 0.75*W + g (Updater.java:57-59)."""
        ptr, n, kind, keep = _operand(gradient)
        self._chk(self._lib.ipls_agg_blend(self._h, partition, N.TGT_WEIGHTS, ptr, n, kind, 0.75, 1.0))

    def UpdateLeavingPeer(self, weights, partition: int):
        """Leaving peer's weights: W = a*W + (1-a)*w, a = 0.6 (Updater.java:65-69)."""
        a = self.LEAVING_A
        ptr, n, kind, keep = _operand(weights)
        self._chk(self._lib.ipls_agg_blend(self._h, partition, N.TGT_WEIGHTS, ptr, n, kind, a, 1 - a))

    def AsyncPublishScale(self, partition: int):
        """Aggregated = 0.25*Weights before the async publish (Updater.java:197-199)."""
        self._chk(self._lib.ipls_agg_scale(self._h, partition, N.TGT_AGG, N.TGT_WEIGHTS, 0.25))

    def OtherReplicaGradients(self, partition: int, aggregator: int, gradients, *, key_hash: int | None = None):
        """Download_Scheduler.download_gradients (Download_Scheduler.java:245-268):
        a bucket that another aggregator of ``partition`` will also fold.  The
        first one becomes Other_Replica_Gradients[(p, a)], later ones fold into
        it.  ``aggregator`` is the int the caller maps 1:1 from the aggregator's
        peer-ID String; ``key_hash`` is ``new Pair<>(p, peerId).hashCode()``
        (java_pair_hash), which places the key in the HashMap and so fixes the
        Collect_Replicas order.  Without it the peer ID is str(aggregator)."""
        ptr, n, kind, keep = _operand(gradients)
        if key_hash is None:
            self._chk(self._lib.ipls_agg_other_replica(self._h, partition, aggregator, ptr, n, kind))
        else:
            self._chk(self._lib.ipls_agg_other_replica_keyed(self._h, partition, aggregator,
                                                             ctypes.c_int32(key_hash).value, ptr, n, kind))

    def OtherReplicaDrop(self, partition: int, aggregator: int) -> bool:
        """Other_Replica_Gradients.remove(new Pair<>(p, a)) with its received
        count (Download_Scheduler.java:215-217, 329-332, 438-440): that
        aggregator's own partial arrived, so its downloaded buckets are not
        collected.  True if the key was stored."""
        return self._chk(self._lib.ipls_agg_other_replica_drop(self._h, partition, aggregator)) == 1

    def replica_order(self):
        """(keys, capacity): the (partition, aggregator) order Collect_Replicas
        would fold in now -- the library's model of the JDK HashMap's keySet()
        order -- and the model's table capacity."""
        room = self._chk(self._lib.ipls_agg_replica_order(self._h, None, 0, None))
        cap = ctypes.c_int32()
        while True:   # keys stored by another thread in between: ask again with more room
            buf = (ctypes.c_int32 * max(2, 2 * room))()
            n = self._chk(self._lib.ipls_agg_replica_order(self._h, buf, room, ctypes.byref(cap)))
            if n <= room:
                return [(buf[2 * i], buf[2 * i + 1]) for i in range(n)], cap.value
            room = n

    def Collect_Replicas(self):
        """IPLS.java:1217-1241: fold every stored Other_Replica_Gradients array
        into REP in the JDK HashMap's key-set order and clear the store.
        Returns (arrays folded, per-partition Participants increments: each
        stored key adds received x its length, IPLS.java:1229-1234 updating
        Participants inside the element loop)."""
        part = (ctypes.c_int32 * max(1, self.n_partitions))()
        k = self._chk(self._lib.ipls_agg_collect_replicas(self._h, part))
        return k, list(part)[:self.n_partitions]

    def reduce_batch(self, p_first: int, buckets, *, start_mode: int = N.START_ZERO,
                     target: int = N.TGT_AGG, big_endian: bool = False):
        """One launch over len(buckets) partitions; buckets[q] is the list of
        device pointers (ints or DeviceBuffers) for partition p_first+q."""
        n_parts = len(buckets)
        flat, k = _bucket_table(buckets, self.lengths, p_first)
        arr = (ctypes.c_void_p * max(1, len(flat)))(*flat)
        kind = N.DEV_BE if big_endian else N.DEV_F64
        self._chk(self._lib.ipls_agg_reduce_batch(self._h, p_first, n_parts, arr, k, kind,
                                                  start_mode, target))

    def reduce_batch_out(self, p_first: int, buckets, dsts, *, start_mode: int = N.START_ZERO,
                         big_endian_in: bool = False, big_endian_out: bool = False):
        """Batched fold into caller device buffers ``dsts[q]`` (one per
        partition); ``big_endian_out`` fuses the update_file byte pack."""
        n_parts = len(buckets)
        if len(dsts) != n_parts:
            raise ValueError("need k buckets and one destination per partition")
        flat, k = _bucket_table(buckets, self.lengths, p_first)
        for q, d in enumerate(dsts):
            p = p_first + q
            if isinstance(d, DeviceBuffer) and 0 <= p < self.n_partitions and d.n < self.lengths[p]:
                raise ValueError(f"partition {p} needs a destination of {self.lengths[p]} doubles, "
                                 f"the DeviceBuffer holds {d.n}")
        arr = (ctypes.c_void_p * max(1, len(flat)))(*flat)
        darr = (ctypes.c_void_p * max(1, n_parts))(*[d.ptr if isinstance(d, DeviceBuffer) else int(d) for d in dsts])
        self._chk(self._lib.ipls_agg_reduce_batch_out(
            self._h, p_first, n_parts, arr, k, N.DEV_BE if big_endian_in else N.DEV_F64, start_mode,
            darr, N.DEV_BE if big_endian_out else N.DEV_F64))

    def aggregate_round(self, p_first: int, buckets, *, big_endian: bool = False, with_average: bool = True,
                        out=None):
        """A whole round in one launch: the folds of ``buckets`` (buckets[q] =
        device buckets of partition p_first+q, may be empty lists) into AGG,
        AggregatePartition (IPLS.java:1248-1274) and the GetPartitions divide
        (IPLS.java:1159-1174).  Returns the averaged values of the partitions
        (host array, or ``out`` when a DeviceBuffer is given), or None."""
        n_parts = len(buckets)
        flat, k = _bucket_table(buckets, self.lengths, p_first)
        arr = (ctypes.c_void_p * max(1, len(flat)))(*flat)
        kind = N.DEV_BE if big_endian else N.DEV_F64
        ap, ak, res = None, N.HOST_F64, None
        if isinstance(out, DeviceBuffer):
            if n_parts and 0 <= p_first and p_first + n_parts <= self.n_partitions:
                last = p_first + n_parts - 1
                need = self.offsets[last] + self.lengths[last] - 1 - self.offsets[p_first]
                if out.n < need:
                    raise ValueError(f"the averages of partitions {p_first}..{last} need {need} doubles, "
                                     f"the DeviceBuffer holds {out.n}")
            ap, ak, res = out.ptr, N.DEV_F64, out
        elif with_average:
            last = p_first + n_parts - 1
            n = self.offsets[last] + self.lengths[last] - 1 - self.offsets[p_first]
            res = np.empty(max(0, n))
            ap = res.ctypes.data if res.size else None
        self._chk(self._lib.ipls_agg_aggregate_round(self._h, p_first, n_parts, arr, k, kind, ap, ak))
        return res

    def commit_partial_update(self, partition: int, workers: int) -> bytes:
        """IPLS_Comm.commit_partial_update (IPLS_Comm.java:51-61, called at
        IPLS.java:1423-1425): the Java-serialised new Pair<>(workers,
        Aggregated_Gradients[p]) file bytes, packed on the device."""
        n = self._chk(self._lib.ipls_agg_commit_partial(self._h, partition, workers, None, 0))
        out = np.empty(n, dtype=np.uint8)
        self._chk(self._lib.ipls_agg_commit_partial(self._h, partition, workers, out.ctypes.data, n))
        return out.tobytes()

    def merge_files(self, files, *, partial_updates: bool = False) -> bytes:
        """Storage node merge (Decentralized_Storage_Receiver.java:239-258) of
        downloaded files -- raw BE gradient files (status 0) or Pair partial
        updates (status != 0) -- into the `_partial_aggregation` file bytes."""
        arrs = [np.frombuffer(bytes(f), dtype=np.uint8) for f in files]
        k = len(arrs)
        ptrs = (ctypes.c_void_p * max(1, k))(*[a.ctypes.data if a.size else None for a in arrs])
        lens = (ctypes.c_int64 * max(1, k))(*[a.size for a in arrs])
        kind = N.HOST_PAIR if partial_updates else N.HOST_BE
        if k == 0:
            raise ValueError("need at least one file")
        if partial_updates:
            n0, _, _ = pair_parse(arrs[0])
            cap = 8 * len(n0)
        else:
            cap = 8 * (arrs[0].size // 8)
        out = np.empty(max(1, cap), dtype=np.uint8)
        nb = self._chk(self._lib.ipls_agg_merge_files(self._h, ptrs, lens, k, kind, out.ctypes.data, cap))
        return out[:nb].tobytes()

    def Merge(self, partition: int, buckets, *, big_endian: bool = True, target: int = N.TGT_REP):
        """Storage-node merge (Decentralized_Storage_Receiver.java:239-247):
        S = g0; S += g_i -- a FIRST-start fold (it overwrites ``target``, so call
        it on the storage node's own Aggregator), returned as BE file bytes
        (the ``<p>_partial_aggregation`` file, :258)."""
        self.reduce_batch(partition, [list(buckets)], start_mode=N.START_FIRST, target=target,
                          big_endian=big_endian)
        return self.read(partition, target, big_endian=True)

    def AggregatePartition(self, partition: int, *, with_sum: bool = False, sum_big_endian: bool = True,
                           with_average: bool = False, sum_out=None):
        """IPLS.java:1248-1274.  Optionally returns the committed sum (the
        update_file bytes of IPLS_Comm.commit_update) and the averaged values.
        ``sum_out`` (a PinnedBuffer of at least 8*L_p bytes) receives the sum
        instead of a new pageable array: the D2H then runs at the PCIe rate."""
        L = self.lengths[partition] if partition >= 0 else 0
        s = a = None
        sp, sk = None, N.HOST_F64
        if sum_out is not None:
            if not isinstance(sum_out, PinnedBuffer) or sum_out.nbytes < 8 * L:
                raise ValueError("sum_out must be a PinnedBuffer of at least 8*L_p bytes")
            s = sum_out.view(np.uint8 if sum_big_endian else np.float64)[:8 * L if sum_big_endian else L]
            sp, sk = sum_out.ptr, (N.HOST_BE if sum_big_endian else N.HOST_F64)
        elif with_sum:
            s = np.empty(8 * L, dtype=np.uint8) if sum_big_endian else np.empty(L)
            sp, sk = s.ctypes.data, (N.HOST_BE if sum_big_endian else N.HOST_F64)
        ap = None
        if with_average:
            a = np.empty(max(0, L - 1))
            ap = a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        self._chk(self._lib.ipls_agg_finalize(self._h, partition, sp, sk, ap))
        return s, a

    def cache_partition(self, partition: int, data, *, frame: bool = False):
        """Download_Scheduler.cache_partition: Weight_Address[p] = GetParameters(hash).
        ``frame=True``: the pid-4 ACK frame of ThreadReceiver (IPLS.java:491-498)."""
        if frame:
            a = np.frombuffer(bytes(data), dtype=np.uint8)
            self._chk(self._lib.ipls_agg_set_weights(self._h, partition, a.ctypes.data, a.size, N.HOST_FRAME))
            return
        ptr, n, kind, keep = _operand(data)
        self._chk(self._lib.ipls_agg_set_weights(self._h, partition, ptr, n, kind))

    def GetPartitions(self, *, wire: bool = False, out=None):
        """IPLS.java:1140-1174: the averaged flat model.  ``wire=True`` returns
        the Middleware task-3 byte stream (DataOutputStream.writeDouble);
        with ``out`` a PinnedBuffer it is written there (the D2H at the PCIe
        rate) and a memoryview of those 8*M bytes is returned, ready for
        ``sendall`` without another copy."""
        n = self.flat_size
        if isinstance(out, DeviceBuffer):
            self._chk(self._lib.ipls_agg_get_partitions(self._h, out.ptr, out.n, N.DEV_F64))
            return out
        if isinstance(out, PinnedBuffer):
            if out.nbytes < 8 * n:
                raise ValueError(f"PinnedBuffer of {out.nbytes} bytes < the model's {8 * n}")
            kind = N.HOST_BE_CANON if wire else N.HOST_F64
            self._chk(self._lib.ipls_agg_get_partitions(self._h, out.ptr, n, kind))
            v = out.view()[:8 * n]
            return memoryview(v) if wire else v.view(np.float64)
        if wire:
            buf = np.empty(8 * n, dtype=np.uint8)
            self._chk(self._lib.ipls_agg_get_partitions(self._h, buf.ctypes.data, n, N.HOST_BE_CANON))
            return buf.tobytes()
        buf = np.empty(n)
        self._chk(self._lib.ipls_agg_get_partitions(self._h, buf.ctypes.data, n, N.HOST_F64))
        return buf

    # ---- replica exchange hooks (ipls.distributed) ----
    def export_partial(self, partition: int, tensor):
        """Copy this aggregator's partial sum AGG[p] into a transport tensor
        (the published partial of IPLS.java:1423-1431) and wait for it.  A
        device tensor (RCCL) gets a device-to-device copy, a host tensor
        (gloo) a device-to-host copy."""
        if getattr(tensor, "is_cuda", False):
            d = DeviceBuffer.from_tensor(tensor)
            self._chk(self._lib.ipls_agg_read(self._h, partition, N.TGT_AGG, d.ptr, d.n, N.DEV_F64))
            self.sync()
        else:
            self._chk(self._lib.ipls_agg_read(self._h, partition, N.TGT_AGG, int(tensor.data_ptr()),
                                              tensor.numel(), N.HOST_F64))

    def import_partial(self, partition: int, tensor, *, replace_agg: bool = False):
        """Fold a replica's partial (a transport tensor that has landed) into
        REP[p] (Updater.java:40-44); replace_agg stores it as AGG[p] instead."""
        if not getattr(tensor, "is_cuda", False):
            if not replace_agg:
                self.Update(tensor.numpy(), partition, from_clients=False)
                return
            # exact FIRST-start copy needs a device operand: on the GPU of the
            # shard that owns the partition (the one whose kernel reads it)
            tensor = tensor.to(f"cuda:{self.partition_device(partition)[0]}")
        d = DeviceBuffer.from_tensor(tensor)
        if replace_agg:
            self.reduce_batch(partition, [[d]], start_mode=N.START_FIRST, target=N.TGT_AGG)
        else:
            self.Update(d, partition, from_clients=False)

    # ---- multi-GPU: shards and replica slots (include/ipls_agg.h, cfg.devices) ----
    def partition_device(self, partition: int):
        """(device ordinal, HIP stream) of the shard that owns ``partition``."""
        d, st = ctypes.c_int32(), ctypes.c_void_p()
        self._chk(self._lib.ipls_agg_partition_device(self._h, partition, ctypes.byref(d), ctypes.byref(st)))
        return d.value, int(st.value or 0)

    def reduce_partial(self, slot: int, p_first: int, buckets, *, start_mode: int = N.START_ZERO,
                       big_endian: bool = False):
        """Replica slot ``slot`` (a shard that does not own these partitions)
        folds buckets resident on its GPU into its partial sums (an aggregator
        of the partition other than its owner, IPLS.java:1402-1431)."""
        n_parts = len(buckets)
        flat, k = _bucket_table(buckets, self.lengths, p_first)
        arr = (ctypes.c_void_p * max(1, len(flat)))(*flat)
        self._chk(self._lib.ipls_agg_reduce_partial(self._h, slot, p_first, n_parts, arr, k,
                                                    N.DEV_BE if big_endian else N.DEV_F64, start_mode))

    def combine_partials(self, p_first: int = 0, n_parts: int | None = None) -> int:
        """REP[p] += every slot's partial of p, slots ascending, read over xGMI
        by the owner's fold kernel (Collect_Replicas, IPLS.java:1449).
        Returns the number of partials folded."""
        n = self.n_partitions - p_first if n_parts is None else n_parts
        return self._chk(self._lib.ipls_agg_combine_partials(self._h, p_first, n))

    # ---- publish-side codec (a9) ----
    @staticmethod
    def _device_text_out(out, out_cap, need: int):
        """(address, capacity in bytes) of a device text destination.  A
        DeviceBuffer's capacity is its own size (8 * n); a raw address must come
        with ``out_cap`` -- the library can only bound its writes by what it is
        told, so an undersized buffer is refused here, never written past."""
        if isinstance(out, DeviceBuffer):
            ptr, cap = out.ptr, 8 * out.n
            if out_cap is not None:
                cap = min(cap, int(out_cap))
        else:
            if out_cap is None:
                raise ValueError("a raw device address needs out_cap= (its capacity in bytes)")
            ptr, cap = int(out), int(out_cap)
        if cap < need:
            raise ValueError(f"publish text needs {need} bytes, the device buffer holds {cap}")
        return ptr, cap

    def publish_partial(self, partition: int, a: int, b: int, *, pid: int = 3, origin: bytes = b"",
                        target: int = N.TGT_AGG, out=None, out_cap: int | None = None) -> bytes | int:
        """Marshall_Packet(target[p], origin, a, b, pid) as Base64.getUrlEncoder
        text (MyIPFSClass.java:990-1016; IPLS.java:1429-1430 publishes AGG with
        a = iteration, b = workers + 1, pid 3), encoded on the GPU.  Returns the
        text bytes, or its length when ``out`` is a DeviceBuffer / int address
        with ``out_cap`` bytes (device text, stream-ordered) or a PinnedBuffer
        (host text)."""
        o = np.frombuffer(bytes(origin), dtype=np.uint8)
        op = o.ctypes.data if o.size else None
        n = self._chk(self._lib.ipls_agg_publish_partial(self._h, partition, target, a, b, pid, op, o.size,
                                                         None, 0, N.HOST_TEXT))
        if isinstance(out, PinnedBuffer):   # host text into pinned memory: the D2H runs at the PCIe rate
            if out.nbytes < n:
                raise ValueError(f"publish text needs {n} bytes")
            return self._chk(self._lib.ipls_agg_publish_partial(self._h, partition, target, a, b, pid, op,
                                                                o.size, out.ptr, n, N.HOST_TEXT))
        if out is not None:
            ptr, cap = self._device_text_out(out, out_cap, n)
            return self._chk(self._lib.ipls_agg_publish_partial(self._h, partition, target, a, b, pid, op,
                                                                o.size, ptr, cap, N.DEV_TEXT))
        buf = np.empty(max(1, n), dtype=np.uint8)
        self._chk(self._lib.ipls_agg_publish_partial(self._h, partition, target, a, b, pid, op, o.size,
                                                     buf.ctypes.data, n, N.HOST_TEXT))
        return buf[:n].tobytes()

    def publish_partials(self, partitions, a: int, b, *, pid: int = 3, origin: bytes = b"",
                         target: int = N.TGT_AGG, out=None, out_cap: int | None = None):
        """The publish loop over Auth_List (IPLS.java:1423-1431) in one launch
        per GPU: text i = Marshall_Packet(target[partitions[i]], origin, a,
        b[i], pid) base64url-encoded.  Returns the list of texts (bytes), or,
        when ``out`` is a DeviceBuffer / device address with ``out_cap`` bytes /
        PinnedBuffer, the (lens, offs) of the texts written there (device:
        stream-ordered)."""
        parts = np.ascontiguousarray(list(partitions), dtype=np.int32)
        bb = np.ascontiguousarray(list(b), dtype=np.int32)
        if bb.size != parts.size:
            raise ValueError("one b value per partition")
        o = np.frombuffer(bytes(origin), dtype=np.uint8)
        op = o.ctypes.data if o.size else None
        n = parts.size
        lens = np.zeros(max(1, n), dtype=np.int64)
        offs = np.zeros(max(1, n), dtype=np.int64)
        total = self._chk(self._lib.ipls_agg_publish_partials(
            self._h, parts.ctypes.data, n, target, a, bb.ctypes.data, pid, op, o.size, None, 0, N.HOST_TEXT,
            lens.ctypes.data, offs.ctypes.data))
        if out is not None:
            if isinstance(out, PinnedBuffer):
                ptr, cap, kind = out.ptr, out.nbytes, N.HOST_TEXT
            else:
                (ptr, cap), kind = self._device_text_out(out, out_cap, total), N.DEV_TEXT
            self._chk(self._lib.ipls_agg_publish_partials(
                self._h, parts.ctypes.data, n, target, a, bb.ctypes.data, pid, op, o.size, ptr, cap, kind,
                None, None))
            return lens[:n].tolist(), offs[:n].tolist()
        buf = np.empty(max(1, total), dtype=np.uint8)
        self._chk(self._lib.ipls_agg_publish_partials(
            self._h, parts.ctypes.data, n, target, a, bb.ctypes.data, pid, op, o.size, buf.ctypes.data, total,
            N.HOST_TEXT, None, None))
        return [buf[offs[i]:offs[i] + lens[i]].tobytes() for i in range(n)]

    def last_launch(self) -> dict:
        """What the last fold launch ran (kernel, shape, lanes, vectors, SEQ code, map, grid)."""
        li = N.LaunchInfo()
        self._chk(self._lib.ipls_agg_last_launch(self._h, ctypes.byref(li)))
        return {f: getattr(li, f) for f, _ in N.LaunchInfo._fields_}

    # ---- state access ----
    def read(self, partition: int, target: int = N.TGT_AGG, *, big_endian: bool = False):
        L = self.lengths[partition]
        if big_endian:
            buf = np.empty(8 * L, dtype=np.uint8)
            self._chk(self._lib.ipls_agg_read(self._h, partition, target, buf.ctypes.data, L, N.HOST_BE))
            return buf.tobytes()
        buf = np.empty(L)
        self._chk(self._lib.ipls_agg_read(self._h, partition, target, buf.ctypes.data, L, N.HOST_F64))
        return buf

    def reset(self, partition: int = N.ALL_PARTITIONS):
        self._chk(self._lib.ipls_agg_reset(self._h, partition))

    def device_ptr(self, partition: int, target: int = N.TGT_AGG) -> int:
        p = ctypes.c_void_p()
        self._chk(self._lib.ipls_agg_device_ptr(self._h, partition, target, ctypes.byref(p)))
        return int(p.value)

    def checksum(self, partition: int, target: int = N.TGT_AGG) -> int:
        v = ctypes.c_uint64()
        self._chk(self._lib.ipls_agg_checksum(self._h, partition, target, ctypes.byref(v)))
        return int(v.value)


class PinnedBuffer:
    """Pinned host memory from ipls_host_alloc (what the Java side would wrap
    as a direct ByteBuffer).  Host operands in it are DMA'd without staging."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        N.check(N.lib().ipls_host_alloc(nbytes, ctypes.byref(p)))
        self.ptr = int(p.value or 0)
        self.nbytes = nbytes

    def view(self, dtype=np.uint8) -> np.ndarray:
        buf = (ctypes.c_char * self.nbytes).from_address(self.ptr)
        return np.frombuffer(buf, dtype=np.uint8).view(dtype)

    def close(self):
        if self.ptr:
            N.lib().ipls_host_free(self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- handle-free device utilities ----
def shard_plan(n_partitions: int, n_shards: int) -> list[int]:
    """Owner shard of every partition (contiguous blocks, p / ceil(P/G))."""
    out = (ctypes.c_int32 * max(1, n_partitions))()
    N.check(N.lib().ipls_shard_plan(n_partitions, n_shards, out))
    return list(out)[:n_partitions]


def java_pair_hash(p: int, peer_id: str) -> int:
    """new org.javatuples.Pair<Integer,String>(p, peer_id).hashCode() (the key
    hash of Other_Replica_Gradients, PeerData.java:140), computed by the
    library from the ID's UTF-8 bytes."""
    b = peer_id.encode("utf-8")
    buf = (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(b or b"\0")
    out = ctypes.c_int32()
    N.check(N.lib().ipls_java_pair_hash(p, ctypes.addressof(buf), len(b), ctypes.byref(out)))
    return out.value


def synth_fill(buf: DeviceBuffer, p: int, k: int, seed: int, stream: int = 0):
    N.check(N.lib().ipls_synth_fill(buf.ptr, buf.n, seed, p, k, buf.kind, stream or None))


def checksum_dev(buf: DeviceBuffer, n: int | None = None, stream: int = 0) -> int:
    v = ctypes.c_uint64()
    N.check(N.lib().ipls_checksum_dev(buf.ptr, buf.n if n is None else n, buf.kind,
                                      ctypes.byref(v), stream or None))
    return int(v.value)


def encode_secure(src: DeviceBuffer, dst: DeviceBuffer, stream: int = 0):
    """Middleware.Encode (Middleware.java:196-210) on the device."""
    N.check(N.lib().ipls_encode_secure(src.ptr, dst.ptr, min(src.n, dst.n), src.kind, dst.kind, stream or None))


def frame_parse(frame: bytes):
    """Header of a pubsub frame: (pid, n, a, b, payload_off, origin_off)."""
    a = np.frombuffer(bytes(frame), dtype=np.uint8)
    pid, x, y = ctypes.c_int16(), ctypes.c_int32(), ctypes.c_int32()
    po, oo = ctypes.c_int64(), ctypes.c_int64()
    n = N.check(N.lib().ipls_frame_parse(a.ctypes.data, a.size, ctypes.byref(pid), ctypes.byref(x),
                                         ctypes.byref(y), ctypes.byref(po), ctypes.byref(oo)))
    return pid.value, n, x.value, y.value, po.value, oo.value


def pair_parse(data):
    """Download_Partial_Updates (MyIPFSClass.java:326-338) through the C-ABI:
    (gradients as float64, workers, payload byte offset)."""
    a = np.frombuffer(bytes(data), dtype=np.uint8)
    w, off = ctypes.c_int32(), ctypes.c_int64()
    n = N.check(N.lib().ipls_pair_parse(a.ctypes.data, a.size, ctypes.byref(w), ctypes.byref(off)))
    g = np.frombuffer(a[off.value:off.value + 8 * n].tobytes(), dtype=">f8").astype(np.float64)
    return g, w.value, off.value


def pair_encode(workers: int, gradients) -> bytes:
    """ObjectOutputStream.writeObject(new Pair<>(workers, gradients)), as
    MyIPFSClass.Update_file(String, Pair) writes it (MyIPFSClass.java:160-166)."""
    g = np.ascontiguousarray(gradients, dtype=np.float64)
    n = N.check(N.lib().ipls_pair_encode(workers, g.ctypes.data, g.size, N.HOST_F64, None, 0))
    out = np.empty(n, dtype=np.uint8)
    N.check(N.lib().ipls_pair_encode(workers, g.ctypes.data, g.size, N.HOST_F64, out.ctypes.data, n))
    return out.tobytes()


def frame_encode(gradient, a: int, b: int, pid: int, origin: bytes) -> bytes:
    """Marshall_Packet(double[],...) before base64 (MyIPFSClass.java:990-1017)."""
    if isinstance(gradient, DeviceBuffer):
        ptr, n, kind = gradient.ptr, gradient.n, N.DEV_F64
        keep = None
    else:
        keep = np.ascontiguousarray(np.zeros(0) if gradient is None else gradient, dtype=np.float64)
        ptr, n, kind = keep.ctypes.data, keep.size, N.HOST_F64
    o = np.frombuffer(bytes(origin), dtype=np.uint8)
    out = np.empty(14 + 8 * n + o.size, dtype=np.uint8)
    nb = N.check(N.lib().ipls_frame_encode(ptr, n, kind, a, b, pid, o.ctypes.data if o.size else None,
                                           o.size, out.ctypes.data, out.size))
    return out[:nb].tobytes()
