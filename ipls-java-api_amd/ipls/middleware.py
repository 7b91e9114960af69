"""The Middleware loopback protocol (Middleware.java:26-268): flags, the task
1/2/3 byte stream, and a single-aggregator loopback server.

Wire format (Java DataInput/OutputStream, big-endian):
  task 1  [i16 1][i16 bootstrapper][i16 n]{[i16 len][bytes]}*n [i16 len][path]
          [i16 len][file name][i32 model_size]                (Middleware.java:128-154)
  task 2  [i16 2][model_size x f64]                            (:156-160)
  task 3  [i16 3]  -> reply model_size x f64 (writeDouble)      (:164-170, 253-258)
  ack     writeChar('A') = 00 41                                (:188-194)

MI355X path. Java reads task 2 one ``readDouble`` at a time and writes task 3
one ``writeDouble`` at a time on an unbuffered stream. Here each partition's
slice of task 2 is received chunk by chunk straight into the library's pinned
staging and handed to the GPU still big-endian (the fold kernel does the byte
swap; ``update_from_socket``). The task-3 reply is the bytes produced on the
GPU by the divide kernel, NaN canonicalised as ``writeDouble`` does, sent
chunk by chunk (``reply_to_socket``). Neither holds a library lock while the
socket is read or written, and every connection has a timeout (``serve``).

``LoopbackAggregator`` plays the aggregator of BASELINE configs[0] ("-pa 3
-n 3 loopback: the aggregator averages 3 peers' List<Double>"). Each task 2 is
one peer's update, folded into every partition as an arrival. After ``-n``
updates the round closes: AggregatePartition for every partition. Task 3
returns GetPartitions' averaged model. The IPFS transport, the schedule and
the responsibility protocol are out of scope.
"""
from __future__ import annotations

import ctypes
import socket
import struct
import threading
import time
from dataclasses import dataclass, field

import numpy as np

from ._native import IplsError


class MissingOptionError(SystemExit):
    pass


class MiddlewareTaskError(RuntimeError):
    """A task the server cannot run: task 2 or 3 before any task 1 (Java's
    Middleware dereferences a null ipls_daemon there, Middleware.java:243-246,
    254, and exits)."""


@dataclass
class Options:
    """Middleware.parse_arguments (Middleware.java:26-110)."""
    port: int
    partitions: int                 # -pa   PeerData._PARTITIONS
    min_partitions: int             # -mp   PeerData._MIN_PARTITIONS
    min_peers: int                  # -n    PeerData.Min_Members
    indirect_communication: bool    # -i    > 0
    training: int                   # -training
    partial_aggregation: bool       # -aggr > 0
    ipns: bool = False              # -IPNS "true"
    synchronous: bool = True        # -async "true" -> False
    extra: dict = field(default_factory=dict)


_FLAGS = {  # short, long, required
    "p": ("port_number", True), "pa": ("partitions", True), "mp": ("minimum_partitions", True),
    "n": ("min_peers", True), "i": ("indirect_communication", True), "training": ("training", True),
    "aggr": ("partial_aggregation", True), "IPNS": ("IPNS", False), "async": ("Async", False),
}


def parse_arguments(argv: list[str]) -> Options:
    """Same flags as commons-cli in Middleware.java:30-65 (``-x v`` or
    ``--long v``).  A missing required flag or a non-integer value exits with
    status 1, as Middleware does (:104-109)."""
    vals = {}
    it = iter(argv)
    for a in it:
        if not a.startswith("-"):
            continue
        key = a.lstrip("-")
        short = next((s for s, (lng, _) in _FLAGS.items() if key in (s, lng)), None)
        if short is None:
            raise MissingOptionError(1)
        try:
            vals[short] = next(it)
        except StopIteration:
            raise MissingOptionError(1)
    missing = [s for s, (_, req) in _FLAGS.items() if req and s not in vals]
    if missing:
        raise MissingOptionError(1)
    try:
        return Options(
            port=int(vals["p"]), partitions=int(vals["pa"]), min_partitions=int(vals["mp"]),
            min_peers=int(vals["n"]), indirect_communication=int(vals["i"]) > 0,
            training=int(vals["training"]), partial_aggregation=int(vals["aggr"]) > 0,
            ipns=vals.get("IPNS") == "true", synchronous=vals.get("async") != "true")
    except ValueError:
        raise MissingOptionError(1)


# ---------------------------------------------------------------------------
# task frames
# ---------------------------------------------------------------------------
def _jstr(s: str | bytes) -> bytes:
    b = s.encode() if isinstance(s, str) else bytes(s)
    return struct.pack(">h", len(b)) + b


def encode_init(is_bootstrapper: bool, bootstrappers: list[str], path: str, file_name: str,
                model_size: int) -> bytes:
    out = struct.pack(">hhh", 1, 1 if is_bootstrapper else 0, len(bootstrappers))
    for b in bootstrappers:
        out += _jstr(b)
    return out + _jstr(path) + _jstr(file_name) + struct.pack(">i", model_size)


def encode_update(gradients) -> bytes:
    return struct.pack(">h", 2) + np.asarray(gradients, dtype=np.float64).astype(">f8").tobytes()


def encode_get() -> bytes:
    return struct.pack(">h", 3)


ACK = struct.pack(">H", ord("A"))   # DataOutputStream.writeChar('A')


def _recv_exact(sock: socket.socket, n: int, into=None) -> memoryview:
    buf = into if into is not None else bytearray(n)
    mv = memoryview(buf)[:n]
    got = 0
    while got < n:
        k = sock.recv_into(mv[got:], n - got)
        if k == 0:
            raise EOFError("socket closed mid-message")
        got += k
    return mv


def read_task(sock: socket.socket, model_size: int, payload_buffer=None, task: int | None = None):
    """Deserialize (Middleware.java:121-162).  Returns (task, data): task 1 ->
    dict of the init fields; task 2 -> the model_size*8 BE bytes (a memoryview
    into payload_buffer when one is supplied, e.g. a PinnedBuffer view);
    task 3 -> None.  ``task``: the task short was already read."""
    if task is None:
        (task,) = struct.unpack(">h", _recv_exact(sock, 2))
    if task == 1:
        boot, nb = struct.unpack(">hh", _recv_exact(sock, 4))
        bs = []
        for _ in range(nb):
            (ln,) = struct.unpack(">h", _recv_exact(sock, 2))
            bs.append(bytes(_recv_exact(sock, ln)).decode())
        (ln,) = struct.unpack(">h", _recv_exact(sock, 2))
        path = bytes(_recv_exact(sock, ln)).decode()
        (ln,) = struct.unpack(">h", _recv_exact(sock, 2))
        fname = bytes(_recv_exact(sock, ln)).decode()
        (ms,) = struct.unpack(">i", _recv_exact(sock, 4))
        return 1, {"is_bootstrapper": boot != 0, "bootstrappers": bs, "path": path, "file_name": fname,
                   "model_size": ms}
    if task == 2:
        return 2, _recv_exact(sock, 8 * model_size, payload_buffer)
    return task, None


# ---------------------------------------------------------------------------
# loopback aggregator + server
# ---------------------------------------------------------------------------
class LoopbackAggregator:
    """One aggregator that owns every partition and closes a round after
    ``min_peers`` updates (see module docstring)."""

    def __init__(self, opts: Options, model_size: int, device: int = 0, initial_model=None):
        from .aggregator import Aggregator, PinnedBuffer
        self.opts = opts
        self.model_size = model_size
        self.agg = Aggregator(model_size, opts.partitions, max_peers=opts.min_peers,
                              partial_aggregation=int(opts.partial_aggregation), device=device)
        if initial_model is not None:
            self.agg.InitializeWeights(initial_model)
        self._pinned = PinnedBuffer
        self._staging = None   # whole-payload pinned staging of update_model / get_partitions_wire, on first use
        self.pending = 0
        self.rounds = 0
        self.lock = threading.Lock()
        # host seconds inside the aggregator per task (the rest of a task is the socket)
        self.stats = {"updates": 0, "update_s": 0.0, "replies": 0, "reply_s": 0.0}

    def update_model(self, be_bytes):
        """Task 2: one peer's update vector (BE bytes) folded into every
        partition as an arrival (Updater._Update / UpdateGradient fold)."""
        with self.lock:
            t0 = time.perf_counter()
            flat = np.frombuffer(be_bytes, dtype=np.uint8)
            self.agg.UpdateGradient(flat, range(self.opts.partitions))
            self._close_round_if_due()
            self.agg.sync()
            self.stats["update_s"] += time.perf_counter() - t0
            self.stats["updates"] += 1

    @property
    def staging(self):
        """Pinned staging of one whole payload (8 * model_size bytes)."""
        if self._staging is None:
            self._staging = self._pinned(8 * self.model_size)
        return self._staging

    def _close_round_if_due(self):
        self.pending += 1
        if self.pending >= self.opts.min_peers:
            for p in range(self.opts.partitions):
                self.agg.AggregatePartition(p)
            self.pending = 0
            self.rounds += 1

    def update_from_socket(self, sock: socket.socket):
        """Task 2 streamed off the socket (Deserialize, Middleware.java:156-160,
        then UpdateGradient, IPLS.java:1737-1743): partition p's slice of the
        update -- the next L_p - 1 big-endian doubles of the stream, then its
        count slot 1.0 (OrganizeGradients, IPLS.java:1018-1040) -- is one
        ipls_agg_accumulate_chunked call whose source receives each chunk
        straight into the library's pinned ring; the copy engine sends it to
        the GPU while the next chunk is received, and the partition is folded
        once its slice has landed.  The library takes its shard lock for that
        fold only, never across the recv, so the other callers of the
        aggregator are not held by a slow client (``self.lock`` orders this
        server's own tasks and round count only).  Same bits as update_model on the whole
        payload.  A connection that ends mid-update raises (Java's
        EOFException ends the Middleware, Middleware.java:262-265), with the
        partitions received before it already folded."""
        one = struct.pack(">d", 1.0)
        with self.lock:
            t0 = time.perf_counter()
            for p in range(self.opts.partitions):
                L = self.agg.lengths[p]

                def source(dst, off, n, L=L):
                    wire = min(off + n, L - 1) - off     # values of this chunk that come off the socket
                    if wire > 0:
                        _recv_exact(sock, 8 * wire, (ctypes.c_char * (8 * wire)).from_address(dst))
                    if off + n == L:                     # the count slot
                        ctypes.memmove(dst + 8 * (n - 1), one, 8)
                    return True
                self.agg.UpdateChunked(p, L, source)
            self._close_round_if_due()
            self.agg.sync()
            self.stats["update_s"] += time.perf_counter() - t0
            self.stats["updates"] += 1

    def reply_to_socket(self, sock: socket.socket):
        """Task 3 (Return_Global_model, Middleware.java:178-184): GetPartitions'
        writeDouble stream produced by the divide kernel and sent chunk by
        chunk straight from the library's pinned ring, each chunk on the wire
        while the next crosses PCIe (ipls_agg_get_partitions_wire_chunked)."""
        with self.lock:
            t0 = time.perf_counter()

            def sink(ptr, off, n):
                sock.sendall((ctypes.c_char * (8 * n)).from_address(ptr))
                return True
            self.agg.GetPartitionsChunked(sink, wire=True)
            self.stats["reply_s"] += time.perf_counter() - t0
            self.stats["replies"] += 1

    def get_partitions_wire(self) -> memoryview:
        """Task 3: GetPartitions' writeDouble stream, written by the divide
        kernel's big-endian output (NaN canonicalised) into the pinned staging
        and handed to ``sendall`` from there.  The view is valid until the
        next task 2 lands in the same staging (the server is sequential)."""
        with self.lock:
            t0 = time.perf_counter()
            v = self.agg.GetPartitions(wire=True, out=self.staging)
            self.stats["reply_s"] += time.perf_counter() - t0
            self.stats["replies"] += 1
            return v

    def close(self):
        self.agg.close()
        if self._staging is not None:
            self._staging.close()


def serve(opts: Options, max_connections: int | None = None, device: int = 0, initial_model=None,
          ready: threading.Event | None = None, host: str = "127.0.0.1", on_listen=None, on_daemon=None,
          io_timeout: float | None = 60.0, on_error=None):
    """Middleware.main (Middleware.java:212-268): one connection per task.
    ``opts.port`` 0 binds a free port; ``on_listen(port)`` is told which, and
    ``on_daemon(aggregator)`` gets the LoopbackAggregator task 1 creates.

    Every accepted connection gets ``io_timeout`` seconds per blocking socket
    operation: a client that stalls mid-task fails that task (socket.timeout)
    instead of holding the server.  The library holds no shard lock while the
    socket is read or written (ipls_agg_accumulate_chunked /
    get_partitions_wire_chunked), so other callers of the same aggregator --
    the Updater's folds -- go on meanwhile either way.  A task that fails
    (timeout, connection closed mid-message, a library error) ends that
    connection only; ``on_error(task, exc)`` is told, and the server goes on
    with the next connection.  Java's Middleware exits on any exception
    (:262-265); a server of many peers should not be ended by one bad one.
    A task 2 that fails mid-stream leaves the partitions whose slices fully
    arrived folded, the rest untouched (each partition is one
    all-or-nothing call)."""
    srv = socket.socket()
    srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    srv.bind((host, opts.port))
    srv.listen(16)
    if on_listen is not None:
        on_listen(srv.getsockname()[1])
    if ready is not None:
        ready.set()
    daemon = None
    served = 0
    try:
        while max_connections is None or served < max_connections:
            conn, _ = srv.accept()
            served += 1
            task = None
            with conn:
                conn.settimeout(io_timeout)
                try:
                    (task,) = struct.unpack(">h", _recv_exact(conn, 2))
                    if task == 1:
                        _, data = read_task(conn, 0, task=1)
                        daemon = LoopbackAggregator(opts, data["model_size"], device, initial_model)
                        if on_daemon is not None:
                            on_daemon(daemon)
                        conn.sendall(ACK)
                    elif task in (2, 3) and daemon is None:
                        raise MiddlewareTaskError(f"task {task} before task 1")
                    elif task == 2:
                        daemon.update_from_socket(conn)
                        conn.sendall(ACK)
                    elif task == 3:
                        daemon.reply_to_socket(conn)
                except (OSError, EOFError, IplsError, MiddlewareTaskError) as e:   # socket.timeout is an OSError
                    if daemon is not None:
                        daemon.stats["failed"] = daemon.stats.get("failed", 0) + 1
                    if on_error is not None:
                        on_error(task, e)
    finally:
        srv.close()
        if daemon is not None:
            daemon.close()


def client_call(port: int, payload: bytes, reply_bytes: int, host: str = "127.0.0.1") -> bytes:
    """What the Python IPLS API does per task: connect, send, read the reply."""
    with socket.create_connection((host, port)) as s:
        s.sendall(payload)
        return bytes(_recv_exact(s, reply_bytes)) if reply_bytes else b""
