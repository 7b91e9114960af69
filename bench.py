#!/usr/bin/env python3
"""Benchmark of the IPLS gradient-partition aggregation hot path on MI355X.

Metric (BASELINE.json): "aggregated-gradient GB/s (device-resident), 32
peers x 4M doubles/partition".  Workload = config C of SURVEY.md §8(d): per
GPU, 16 partitions x 4,194,304-double buckets (count slot included) x 32 peers,
synthetic splitmix64 counter data generated on the device before timing.

One step = ONE launch of the batched fixed-order reduce over all of the GPU's
partitions through the C-ABI (ipls_agg_reduce_batch, ZERO start = fresh
Aggregated_Gradients, Updater.java:115-117 semantics), with every bucket
already resident in HBM.  Algorithmic bytes per step = P * (K+1) * L * 8
(read K buckets, write 1 sum).  Multi-GPU: one process per GPU, partitions
sharded 16 per GPU (`-pa` segments mapped to devices), no data-path
collective -> weak scaling; value = all ranks' bytes / max-over-ranks time.

Extra JSON objects: `roofline` (dominant kernel, HIP-event time on the
handle's stream vs 8 TB/s HBM peak; traffic from the committed rocprofv3 PMC
pass when one matches this workload) and `cpu_baseline` (the reference's
single-thread Updater decode+fold loop restated in C, oracle/, timed on this
host on a bounded sample; rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "ipls-java-api_amd"))
sys.path.insert(0, str(ROOT))

METRIC = "aggregated-gradient GB/s (device-resident), 32 peers×4M doubles/partition"
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 153.0       # one xGMI link, per direction (7 links per GPU)
PCIE_GBS = 56.0             # PCIe Gen5 x16 per direction, measured (tools/h2d_bench.hip, profiles/r01/h2d_bench.txt)

CONFIGS = {
    # name: (partitions per GPU, bucket length incl. count slot, peers)
    "B": (16, 1048576, 8),
    "C": (16, 4194304, 32),
    "D": (64, 4194304, 32),
    "F": (16, 8388608, 64),     # per GPU; 69.8 GB of buckets resident in HBM
}


# The 1-GPU numbers the multi-GPU prediction starts from:
# config C's k_reduce on the round-5 library over the round's boxes
# (profiles/r05/q, r05/t and the driver's BENCH_r05: 2.4814-2.5193 ms).
ONE_GPU_C_MS = (2.48, 2.54)


def spread_sources(owner: int, world: int, P: int) -> dict:
    """ReplicaPlan.spread (ipls.distributed) / c_abi_multi_gpu's slot map:
    the q-th partition of `owner` has its replica partial on GPU
    (owner + 1 + q mod (G-1)) mod G.  Returns {source GPU: partials}."""
    cnt = {}
    for q in range(P):
        s = (owner + 1 + q % (world - 1)) % world
        cnt[s] = cnt.get(s, 0) + 1
    return cnt


def scaling_prediction(world: int, P: int = 16, L: int = 4194304, K: int = 32) -> dict:
    """What an N-GPU run of this bench should read, written before any such
    run (the table of DESIGN.md §6.1 is this function's
    output).  Weak scaling: every GPU folds its own config-C slice from its
    own HBM, so the fold time stays the 1-GPU one and the line's value is
    N x the per-GPU rate over the slowest rank's time.  The exchange legs are
    bounded by xGMI: one link per GPU pair, XGMI_LINK_GBS per direction, and
    the spread schedule pulls each owner's P partials (L doubles each) from
    its G-1 peers -- ceil(P / (G-1)) over the busiest link."""
    fold_bytes = P * (K + 1) * L * 8
    lo, hi = ONE_GPU_C_MS
    pred = {"link_GBps": XGMI_LINK_GBS, "fold_ms_per_gpu": [lo, hi],
            "value_GBps": [round(world * fold_bytes / hi / 1e6, 0), round(world * fold_bytes / lo / 1e6, 0)]}
    if world > 1:
        part = L * 8
        busiest = max(spread_sources(0, world, P).values())
        links = min(world - 1, P)
        pred.update({
            "partials_per_owner": P, "partial_bytes": part, "links_per_owner": links,
            "busiest_link_partials": busiest,
            # c_abi_multi_gpu's combine and replica_exchange's RCCL exchange move the same bytes
            "combine_ms_at_link_peak": round(busiest * part / (XGMI_LINK_GBS * 1e9) * 1e3, 3),
            "combine_ms_even_links": round(P * part / (links * XGMI_LINK_GBS * 1e9) * 1e3, 3),
            "frac_of_xgmi_if_busiest_link_saturated": round(P / (links * busiest), 4),
            "e2e_GBps_per_gpu_pcie_bound": PCIE_GBS,
        })
    return pred


def scaling_check(world: int, out: dict) -> dict:
    """The N > 1 line's prediction next to what this run measured, compact
    and near the end of the line (the driver keeps its stdout tail)."""
    m = {"value_GBps": out.get("value"), "ms_per_step": out.get("ms_per_step")}
    ml = out.get("c_abi_multi_gpu") or {}
    cb = ml.get("combine") or {}
    for k in ("owner_kernel_ms", "frac_of_xgmi", "frac_of_xgmi_min", "xgmi_link_GBps", "status"):
        if k in cb:
            m[f"combine_{k}" if not k.startswith("combine") else k] = cb[k]
    rx = out.get("replica_exchange") or {}
    for k in ("exchange_ms", "exchange_GBps_per_rank_each_way"):
        if k in rx:
            m[f"replica_{k}"] = rx[k]
    e2e = out.get("host_inclusive_multi") or {}
    if "GBps_per_gpu_min" in e2e:
        m["e2e_GBps_per_gpu_min"] = e2e["GBps_per_gpu_min"]
    return {"predicted": scaling_prediction(world), "measured": m, "source": "DESIGN.md §6.1"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C", choices=sorted(CONFIGS))
    ap.add_argument("--strong", action="store_true",
                    help="fixed total work: the config's partitions are split over the ranks "
                         "(default: weak scaling, the config per GPU)")
    ap.add_argument("--be", action="store_true",
                    help="buckets are big-endian IPFS bytes and the sum is written as BE bytes "
                         "(fused unpack + pack, config D's timed pack/unpack)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-inclusive (H2D+D2H) leg")
    ap.add_argument("--e2e-reps", type=int, default=4)
    ap.add_argument("--no-middleware", action="store_true",
                    help="N=1: skip the Middleware loopback-socket leg (task 2 x 32 + task 3 at model scale)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-passes", type=int, default=16,
                    help="CPU baseline sample: passes over one partition's K buckets")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="N=1: skip the config-B and config-D (BE in/out) lines measured after the headline")
    ap.add_argument("--no-per-arrival", action="store_true",
                    help="N=1: skip the per-arrival (one call per bucket) leg measured after the headline")
    ap.add_argument("--no-replica-leg", action="store_true",
                    help="N>1: skip the cross-GPU replica exchange measurement (config E)")
    ap.add_argument("--no-strong-leg", action="store_true",
                    help="N>1: skip the fixed-total-work leg (config D split over the ranks)")
    ap.add_argument("--replica-reps", type=int, default=5)
    ap.add_argument("--no-ulp-leg", action="store_true",
                    help="N>1: skip the collective-reduce ULP report (dist.reduce over all ranks vs the fixed order)")
    ap.add_argument("--no-multi-leg", action="store_true",
                    help="N>1: skip the single-handle multi-GPU leg (rank 0 drives all N GPUs through the C-ABI)")
    ap.add_argument("--multi-rehearsal", action="store_true",
                    help="N=1: run the single-handle multi-GPU leg over two shards of GPU 0 (a functional "
                         "rehearsal of the cross-GPU code path; the numbers measure one GPU)")
    ap.add_argument("--replica-timeout", type=float, default=240.0)
    ap.add_argument("--be-schedule-ab", action="store_true",
                    help="N=1: after the headline, A/B config D's big-endian schedules in one process on the same "
                         "buckets (needs make -C ipls-java-api_amd variants)")
    ap.add_argument("--watchdog-selftest", action="store_true",
                    help="CPU only: run the N>1 watchdog over a gloo exchange that never completes "
                         "(tests/test_bench_watchdog.py); exits with Watchdog.EXIT_CODE")
    ap.add_argument("--plumbing-selftest", action="store_true",
                    help="CPU only: the N>1 launch plumbing over gloo (tests/test_bench_spawn.py)")
    ap.add_argument("--selftest-fail-rank", type=int, default=-1,
                    help="with --plumbing-selftest: this rank exits with code 7 after joining the group")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: rehearsal of the N>1 code on one GPU (ranks share cuda:0, partials "
                         "travel through host memory); numbers are not a measurement")
    return ap.parse_args()


def cpu_share() -> tuple[int, dict]:
    """CPUs this process may use: the affinity mask, capped by the cgroup CPU
    quota and by OMP_NUM_THREADS (the GPU box sets both to its per-GPU share)."""
    n = len(os.sched_getaffinity(0))
    info = {"nproc": os.cpu_count(), "affinity": n}
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        if q[0] != "max":
            info["cgroup_quota_cpus"] = round(int(q[0]) / int(q[1]), 2)
            n = min(n, max(1, int(int(q[0]) // int(q[1]))))
    except (OSError, ValueError, IndexError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        info["OMP_NUM_THREADS"] = int(os.environ["OMP_NUM_THREADS"])
        n = min(n, int(os.environ["OMP_NUM_THREADS"]))
    return max(1, n), info


def cpu_baseline(L: int, K: int, passes: int, mt_passes: int = 2) -> dict:
    """Reference Updater loop (Updater.java:162-187 + 115-117, MyIPFSClass.java:
    444-455) restated in C, ONE thread as the reference's single Updater thread:
    per bucket a BE getDouble decode into a reused buffer, then the fold.
    Beside it the N-thread partition-parallel variant of SURVEY.md §8(d): N
    partitions with their OWN K buckets each, one thread per partition, N =
    the CPUs this process may use (cpu_share)."""
    from oracle import oracle as O
    be = []
    for k in range(K):
        b = O.c_synth_bucket(L, 0, k)
        be.append(np.frombuffer(b.astype(">f8").tobytes(), dtype=np.uint8).copy())
    O.c_updater_loop(be, L)                      # warm pages
    t0 = time.perf_counter()
    for _ in range(passes):
        O.c_updater_loop(be, L)
    dt = time.perf_counter() - t0
    nbytes = passes * (K + 1) * L * 8
    del be
    threads, share = cpu_share()
    mt = {}
    try:
        bufs = O.c_synth_be_buckets(threads, K, L)     # threads x K distinct buckets (BE bytes)
        O.c_updater_loop_partitions(bufs, threads, K, L, 1, threads)   # warm pages
        t1 = time.perf_counter()
        _, used = O.c_updater_loop_partitions(bufs, threads, K, L, mt_passes, threads)
        dt_mt = time.perf_counter() - t1
        mt_bytes = mt_passes * threads * (K + 1) * L * 8
        mt = {"value": round(mt_bytes / dt_mt / 1e9, 3), "cores": used,
              "sample": f"{mt_passes} passes x {threads} partitions (one per thread), each with its own {K} BE "
                        f"buckets of {L} doubles ({threads * K * L * 8 / 1e9:.1f} GB of buckets, "
                        f"{mt_bytes / 1e9:.1f} GB algorithmic, {dt_mt:.1f} s)",
              "cpu_share": share,
              "note": "N = the CPUs this process may use (affinity, cgroup quota, OMP_NUM_THREADS): the GPU box "
                      "grants each GPU its share of the host, so N is that share, not nproc"}
        del bufs
    except MemoryError as e:
        mt = {"error": f"MemoryError: {e}"}
    return {"value": round(nbytes / dt / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{passes} passes x 1 partition x {K} peers x {L} doubles "
                      f"({nbytes / 1e9:.1f} GB algorithmic, {dt:.1f} s), BE decode + fold, "
                      f"oracle/ipls_oracle.c ipls_oracle_updater_loop (JDK absent: C restatement)",
            "multi_thread": mt, "host_cpus": os.cpu_count(), "cpu_model": _cpu_model()}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_inclusive(ipls, agg_cls, L: int, K: int, reps: int, device: int) -> dict:
    """Rate including the PCIe copies: K peers' BE byte buckets start in host
    memory (as pulled from IPFS), each arrival is folded (Updater._Update),
    then AggregatePartition writes the BE sum bytes back to host memory
    (commit_update's update_file).  Pinned buffers (ipls_host_alloc, DMA
    straight from them) and pageable numpy buffers (staged) are both timed."""
    import torch
    agg = agg_cls(n_partitions=1, bucket_len=L, device=device)
    pinned = []
    for k in range(K):
        t = torch.empty(8 * L, dtype=torch.uint8, device="cuda")
        ipls.synth_fill(ipls.DeviceBuffer(int(t.data_ptr()), L, big_endian=True), 0, k, ipls.SEED)
        pb = ipls.PinnedBuffer(8 * L)
        pb.view()[:] = t.cpu().numpy()
        pinned.append(pb)
    pageable = [pb.view().copy() for pb in pinned]
    sum_pinned = ipls.PinnedBuffer(8 * L)     # the commit_update bytes land in pinned memory too
    out = {}
    # batched: all K pinned buckets in one launch, read over PCIe (zero copy)
    row = [[ipls.DeviceBuffer(pb.ptr, L, big_endian=True) for pb in pinned]]
    agg.reduce_batch(0, row, start_mode=ipls.START_ZERO, big_endian=True)
    agg.AggregatePartition(0, sum_out=sum_pinned)
    t0 = time.perf_counter()
    for _ in range(reps):
        agg.reduce_batch(0, row, start_mode=ipls.START_ZERO, big_endian=True)
        agg.AggregatePartition(0, sum_out=sum_pinned)
    out["pinned_batched"] = round(reps * (K + 1) * L * 8 / (time.perf_counter() - t0) / 1e9, 2)
    for name, bufs in (("pinned", [pb.view() for pb in pinned]), ("pageable", pageable)):
        so = sum_pinned if name == "pinned" else None   # pageable: a heap byte[] for the sum as well
        for b in bufs:                                   # warm
            agg.Update(b, 0)
        agg.AggregatePartition(0, with_sum=True, sum_out=so)
        t0 = time.perf_counter()
        for _ in range(reps):
            for b in bufs:
                agg.Update(b, 0)
            agg.AggregatePartition(0, with_sum=True, sum_big_endian=True, sum_out=so)
        dt = time.perf_counter() - t0
        out[name] = round(reps * (K + 1) * L * 8 / dt / 1e9, 2)
    # per arrival, asynchronous: each fold is queued (ipls_agg_accumulate_async)
    # and the round waits once, at AggregatePartition
    for pb in pinned:                                    # warm
        agg.UpdateAsync(pb, 0)
    agg.AggregatePartition(0, sum_out=sum_pinned)
    t0 = time.perf_counter()
    for _ in range(reps):
        for pb in pinned:
            agg.UpdateAsync(pb, 0)
        agg.AggregatePartition(0, sum_out=sum_pinned)
    out["pinned_async"] = round(reps * (K + 1) * L * 8 / (time.perf_counter() - t0) / 1e9, 2)
    agg.close()
    for pb in pinned:
        pb.close()
    sum_pinned.close()
    return {"unit": "GB/s", **out,
            "sample": f"{reps} rounds x 1 partition x {K} peers x {L} doubles: each BE bucket from host memory "
                      f"(pinned: per-arrival zero-copy fold; pinned_async: the same, queued without waiting; "
                      f"pinned_batched: one launch over all K; pageable: "
                      f"staged H2D) + finalize + D2H of the BE sum (into pinned memory, pageable for the pageable "
                      f"leg), algorithmic bytes (K+1)*L*8 per round, Python/ctypes caller",
            "pcie_ceiling": "~56 GB/s per direction measured (tools/h2d_bench.hip, profiles/r01/h2d_bench.txt)"}


def f_stream_leg(ipls, torch, device: int, P: int = 16, L: int = 8388608, K: int = 64, ring: int = 16,
                 lag: int = 4, producers: int = 8, verify: bool = True) -> dict:
    """Config F end to end at F's own shape (BASELINE configs[4], one GPU's
    slice): 16 partitions x 64 peers x 8,388,608 big-endian doubles start as
    host IPFS bytes and every partition's BE sum ends in host memory.

    The `ipfs cat` bytes of all 1,024 buckets (68.7 GB) sit in pageable host
    memory -- the stand-in for the network.  They land, one arrival at a time,
    in a bounded ring of `ring` pinned 64 MiB slots (direct ByteBuffers in
    the Java drop-in), copied by `producers` host threads
    the way a socket read fills the buffer.  Each landed slot is one
    Updater._Update (ipls_agg_accumulate_async on pinned memory: the fold
    reads the slot over PCIe, zero copy, Updater.java:115-117 after
    GetParameters' BE decode, MyIPFSClass.java:444-455); a slot is refilled
    once its fold's ticket completed (`lag` folds in flight).  After a
    partition's 64 arrivals, AggregatePartition writes its update_file bytes
    (BE sum, MyIPFSClass.java:105-116) to a pinned sum buffer.  Timed from the
    first landing to the last sum in host memory; bytes = P*(K+1)*L*8."""
    from concurrent.futures import ThreadPoolExecutor
    nb = 8 * L
    N = P * K
    try:   # the pool is faulted in page by page: never let it run the host out of memory
        import psutil
        avail = psutil.virtual_memory().available
        if avail < 1.25 * (N + ring + P) * nb:
            return {"error": f"skipped: {avail / 2**30:.0f} GiB of host memory available, "
                             f"{1.25 * (N + ring + P) * nb / 2**30:.0f} GiB needed"}
    except ImportError:
        pass
    t_prep = time.perf_counter()
    pool = torch.empty(N * nb, dtype=torch.uint8)           # pageable host bytes: every bucket's `ipfs cat`
    tmp = torch.empty(nb, dtype=torch.uint8, device=torch.device("cuda", device))
    for i in range(N):
        ipls.synth_fill(ipls.DeviceBuffer(int(tmp.data_ptr()), L, big_endian=True), i // K, i % K, ipls.SEED)
        pool[i * nb:(i + 1) * nb].copy_(tmp)
    del tmp
    pool_np = pool.numpy()
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, device=device)
    slots = [ipls.PinnedBuffer(nb) for _ in range(ring)]
    sums = [ipls.PinnedBuffer(nb) for _ in range(P)]
    for b in slots + sums:                                  # fault the pinned pages in before timing
        b.view()[::4096] = 0
    prep_s = time.perf_counter() - t_prep
    exe = ThreadPoolExecutor(producers)

    def land(i):
        np.copyto(slots[i % ring].view(), pool_np[i * nb:(i + 1) * nb])

    fills = {i: exe.submit(land, i) for i in range(min(ring, N))}
    tickets = {}
    t0 = time.perf_counter()
    for i in range(N):
        p, k = divmod(i, K)
        fills.pop(i).result()
        tickets[i] = agg.UpdateAsync(slots[i % ring], p)
        j = i - lag                                          # the oldest fold allowed to be still running
        if j in tickets:
            agg.Wait(tickets.pop(j))
            if j + ring < N:
                fills[j + ring] = exe.submit(land, j + ring)   # its slot is free again
        if k == K - 1:
            agg.AggregatePartition(p, sum_out=sums[p])        # waits for p's folds; BE sum -> pinned
            for jj in sorted(tickets):                        # every earlier fold is done now
                del tickets[jj]
                if jj + ring < N:
                    fills[jj + ring] = exe.submit(land, jj + ring)
    dt = time.perf_counter() - t0
    exe.shutdown()
    nbytes = P * (K + 1) * L * 8
    ok = None
    if verify:
        from oracle import oracle as O   # checker only
        good = sum(int(ipls.checksum_dev(ipls.DeviceBuffer(sums[p].ptr, L, big_endian=True))
                       == O.c_synth_sum_checksum(L, p, K)) for p in range(P))
        ok = f"{good}/{P}"
    agg.close()
    for b in slots + sums:
        b.close()
    del pool, pool_np
    return {"workload": f"{P} x {K} x {L // 1048576}M streamed: {P} partitions x {K} peers x {L} BE doubles from "
                        f"host bytes through a ring of {ring} pinned slots, BE sums to pinned host memory",
            "GBps": round(nbytes / dt / 1e9, 2), "seconds": round(dt, 3), "algorithmic_bytes": nbytes,
            "frac_of_pcie": round(nbytes / dt / 1e9 / PCIE_GBS, 4), "pcie_ceiling_GBps": PCIE_GBS,
            "peak_pinned_host_bytes": (ring + P) * nb, "host_source_bytes": N * nb,
            "verified_partitions": ok, "prep_s": round(prep_s, 1),
            "note": f"{producers} host threads land the bytes (a memcpy from pageable memory, as a socket read fills "
                    f"a direct ByteBuffer); per arrival one ipls_agg_accumulate_async zero-copy fold over PCIe, "
                    f"<= {lag + 1} folds in flight; per partition ipls_agg_finalize with the BE sum into pinned "
                    f"memory; Python caller"}


def jni_heap_leg(L: int = 4194304, reps: int = 20) -> dict:
    """The JNI shim's heap-array natives against its direct-buffer ones
    (DESIGN.md §5.2): tools/jni_heap_probe.py in a child
    process -- the shim and the fake JVM (tests/jni/fake_jvm.c) built with
    gcc, driving the real library on this GPU, one partition of L doubles per
    call.  GB/s = bytes of the Java-side array / wall time per call.  No JDK
    exists here: the fake JVM's Get/Set<T>ArrayRegion and critical regions
    are plain memcpy / pointer hand-outs, as HotSpot's are for primitive
    arrays.  Never the value."""
    import subprocess
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "jni_heap_probe.py"), str(L), str(reps)],
                       capture_output=True, text=True, timeout=240,
                       env={k: v for k, v in os.environ.items() if not k.startswith("IPLS_JNI_")})
    if r.returncode != 0:
        return {"error": r.stderr[-400:]}
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    keep = ("accumulate_heap_double[]", "accumulateDirect_pinned_BE", "finalize_heap_byte[]", "finalizeDirect_pinned",
            "getPartitions_heap_double[]", "getPartitionsWire_pinned")
    out = {k: d[k]["GBps"] for k in keep if k in d}
    out.update(unit="GB/s", bucket_doubles=L, copy_threads=d.get("copy_threads"), ring_chunk=d.get("ring_chunk"),
               source="tools/jni_heap_probe.py (shim + fake JVM, gcc-built in a child process)")
    return out


def middleware_socket_leg(ipls, torch, device: int, P: int = 16, Lv: int = 4194303, K: int = 32, D: int = 4,
                          verify: bool = True, warm_rounds: int = 3) -> dict:
    """The north_star's host boundary at model scale: the Middleware loopback
    socket (Middleware.java:212-268) carrying K task-2 updates of M = P x Lv
    doubles (Deserialize, :156-160, 537 MB each) and one task-3 reply
    (Serialize, :164-170), through ipls.middleware.serve on TCP 127.0.0.1.

    Server (ipls.middleware.LoopbackAggregator, -pa P -n K): each task-2
    update is UpdateGradient over every partition (IPLS.java:1737-1743),
    streamed: partition p's slice is one ipls_agg_accumulate_chunked call
    whose source receives each 4 MiB chunk straight into the library's
    pinned ring, so the H2D copy of a chunk overlaps the receive of the next
    and the BE decode is fused into the fold; after K updates the round
    closes (AggregatePartition for every p, IPLS.java:1248-1274).  Task 3 is
    GetPartitions (IPLS.java:1159-1174): the divide kernel writes the
    writeDouble stream (big-endian, NaN canonical) and
    ipls_agg_get_partitions_wire_chunked hands it to sendall() chunk by chunk
    from the pinned ring.  Client: the Python IPLS API's side, one
    connection per task (D distinct update vectors cycled).

    Ceiling: the same client against a server that receives each payload into
    one pinned buffer and answers task 3 from it, with no aggregator --
    the loopback socket alone, measured in the same process and listening at
    the same time.  One cold round of each (first-use allocations), then
    `warm_rounds` rounds alternating ceiling / aggregator: the box's CPU share
    moves between rounds, and a pair sees the same conditions.
    The reply is checked byte for byte against the oracle's writeDouble
    stream of the fixed-order average ((((+0.0 + u_0) + u_1) ...) + 0.0) / K."""
    import socket
    import struct
    import threading
    from ipls import middleware as MW
    M = P * Lv
    nbytes = 8 * M
    t_prep = time.perf_counter()
    ups = []
    tmp = torch.empty(nbytes, dtype=torch.uint8, device=torch.device("cuda", device))
    for d in range(D):
        ipls.synth_fill(ipls.DeviceBuffer(int(tmp.data_ptr()), M, big_endian=True), 200 + d, 0, ipls.SEED)
        torch.cuda.synchronize()
        ups.append(tmp.cpu().numpy())
    del tmp
    reply = np.empty(nbytes, dtype=np.uint8)
    reply[::4096] = 0
    prep_s = time.perf_counter() - t_prep
    hdr2, hdr3 = struct.pack(">h", 2), struct.pack(">h", 3)

    def task(port, hdr, payload, n_reply, into=None):
        with socket.create_connection(("127.0.0.1", port)) as s:
            s.sendall(hdr)
            if payload is not None:
                s.sendall(memoryview(payload))
            return MW._recv_exact(s, n_reply, into)

    def one_round(port):
        """K task 2 + one task 3; per-task client wall times."""
        t2 = []
        t0 = time.perf_counter()
        for k in range(K):
            a = time.perf_counter()
            assert bytes(task(port, hdr2, ups[k % D], 2)) == MW.ACK
            t2.append(time.perf_counter() - a)
        a = time.perf_counter()
        task(port, hdr3, None, nbytes, reply)
        t3 = time.perf_counter() - a
        return time.perf_counter() - t0, t2, t3

    def summary(dt, t2, t3):
        moved = (K + 1) * nbytes
        return {"seconds": round(dt, 3), "GBps": round(moved / dt / 1e9, 3),
                "task2_ms_mean": round(1e3 * float(np.mean(t2)), 2), "task2_GBps": round(nbytes / float(np.mean(t2)) / 1e9, 3),
                "task3_ms": round(1e3 * t3, 2), "task3_GBps": round(nbytes / t3 / 1e9, 3)}

    def listener():
        srv = socket.socket()
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind(("127.0.0.1", 0))
        srv.listen(16)
        return srv

    # --- the ceiling: the loopback socket alone, same staging, same client
    staging = ipls.PinnedBuffer(nbytes)
    staging.view()[::4096] = 0
    srv = listener()
    ceil_port = srv.getsockname()[1]
    n_rounds = 1 + warm_rounds

    def null_server(n_conn):
        for _ in range(n_conn):
            conn, _ = srv.accept()
            with conn:
                (t,) = struct.unpack(">h", MW._recv_exact(conn, 2))
                if t == 2:
                    MW._recv_exact(conn, nbytes, staging.view())
                    conn.sendall(MW.ACK)
                elif t == 3:
                    conn.sendall(memoryview(staging.view())[:nbytes])
    th_ceil = threading.Thread(target=null_server, args=(n_rounds * (K + 1),), daemon=True)
    th_ceil.start()

    # --- the aggregator behind the same socket, listening at the same time
    opts = MW.parse_arguments(f"-p 0 -pa {P} -mp 1 -n {K} -i 0 -training 0 -aggr 0".split())
    got_port, daemons = [], []
    ready = threading.Event()
    th = threading.Thread(target=MW.serve, kwargs=dict(opts=opts, max_connections=1 + n_rounds * (K + 1),
                                                       device=device, ready=ready, on_listen=got_port.append,
                                                       on_daemon=daemons.append), daemon=True)
    th.start()
    if not ready.wait(60):
        return {"error": "the middleware server did not start"}
    port = got_port[0]
    assert bytes(task(port, MW.encode_init(False, [], "/ip4/127.0.0.1/tcp/5001", "bench", M), None, 2)) == MW.ACK
    # rounds alternate ceiling / aggregator, so that each pair sees the same
    # host conditions (the box's CPU share is shared); the last round is the
    # aggregator's, whose reply is verified
    ceil, runs = [], []
    for r in range(n_rounds):
        ceil.append(one_round(ceil_port))
        st0 = dict(daemons[0].stats)
        dt, t2, t3 = one_round(port)
        st1 = daemons[0].stats
        runs.append((dt, t2, t3, {"update_s": st1["update_s"] - st0["update_s"],
                                  "reply_s": st1["reply_s"] - st0["reply_s"]}))
    th.join(120)
    th_ceil.join(60)
    srv.close()
    staging.close()
    progress("middleware leg: socket ceiling and aggregator done")
    ok = None
    want_sum = None
    if verify:
        from oracle import oracle as O   # checker only
        acc = np.zeros(M)
        vals = [np.frombuffer(u, dtype=">f8").astype(np.float64) for u in ups]
        for k in range(K):
            O.fold(acc, vals[k % D])
        avg = (acc + 0.0) / float(K)
        want = O.be_encode_canonical(avg)
        ok = bool(reply.tobytes() == want)
        want_sum = O.checksum(avg)
        del vals, acc, want, avg
    ceil_s = [summary(*c) for c in ceil]
    agg_s = [summary(*rr[:3]) for rr in runs]
    for g, rr in zip(agg_s, runs):
        g["server_ms_per_task2"] = round(1e3 * rr[3]["update_s"] / K, 2)
        g["server_ms_task3"] = round(1e3 * rr[3]["reply_s"], 2)
    cold, g_cold = ceil_s[0], agg_s[0]
    # the warm rounds' median pair (by the aggregator's rate), and each pair's ratio
    ratios = [a["GBps"] / c["GBps"] for a, c in zip(agg_s[1:], ceil_s[1:])]
    mid = sorted(range(warm_rounds), key=lambda i: agg_s[1 + i]["GBps"])[warm_rounds // 2]
    g_warm, warm = agg_s[1 + mid], ceil_s[1 + mid]
    del ups, reply
    # the same traffic through the native server (host/ipls_middleware.hpp, Middleware.main in C++ over the
    # C-ABI) and a native client: tools/middleware_e2e.cpp, a child process, the same update vectors
    native = None
    exe = ROOT / "ipls-java-api_amd" / "lib" / "middleware_e2e"
    if exe.exists():
        import subprocess
        r = subprocess.run([str(exe), str(M), str(P), str(K), str(D)], capture_output=True, text=True, timeout=300)
        if r.returncode == 0:
            native = json.loads(r.stdout.strip().splitlines()[-1])
            native["frac_of_ceiling"] = round(native["aggregator"]["GBps"] / native["socket_ceiling"]["GBps"], 4)
            native["verified_task3_checksum"] = (int(native["reply_checksum"]) == want_sum) if want_sum is not None else None
            native["source"] = "tools/middleware_e2e.cpp: ipls_host::MiddlewareServer + MiddlewareClient, C++"
        else:
            native = {"error": f"rc {r.returncode}: {r.stderr[-400:]}"}
    else:
        native = {"error": "ipls-java-api_amd/lib/middleware_e2e not built (make -C ipls-java-api_amd host_e2e)"}
    progress("middleware leg: native server done")
    return {"workload": f"Middleware over TCP loopback: -pa {P} -n {K}, model {M} doubles ({nbytes / 1e6:.0f} MB per "
                        f"task): {K} task-2 updates + 1 task-3 reply per round, one connection per task",
            "GBps": g_warm["GBps"], "ceiling_GBps": warm["GBps"], "frac_of_ceiling": round(g_warm["GBps"] / warm["GBps"], 4),
            "frac_of_ceiling_per_round": [round(x, 4) for x in ratios],
            "GBps_per_round": [a["GBps"] for a in agg_s[1:]], "ceiling_GBps_per_round": [c["GBps"] for c in ceil_s[1:]],
            "aggregator": g_warm, "aggregator_cold_round": g_cold, "socket_ceiling": warm,
            "socket_ceiling_cold_round": cold, "verified_task3_bytes": ok, "prep_s": round(prep_s, 1),
            "native": native,
            "note": "bytes = (K + 1) x 8M moved over the socket per round / client wall time.  Task 2: each "
                    "partition's slice is received chunk by chunk (4 MiB) straight into the library's pinned ring "
                    "by ipls_agg_accumulate_chunked's source, sent to the GPU while the next chunk is received, "
                    "folded once landed; sync before the ACK.  Task 3: the divide kernel's writeDouble stream "
                    "sent chunk by chunk from the pinned ring (ipls_agg_get_partitions_wire_chunked).  "
                    "server_ms_*: time inside the aggregator's socket handlers (socket reads/writes included).  "
                    "Ceiling = the same socket traffic into / out of one pinned buffer with no aggregator.  "
                    f"One cold round of each, then {warm_rounds} warm rounds alternating ceiling / aggregator; "
                    "the headline pair is the warm round with the median aggregator rate.  "
                    "Python server and client threads in one process"}


def e2e_multi(ipls, torch, dist, group, rank, world, local, L, K, reps, verify) -> dict:
    """Config F's end-to-end leg at N > 1: every rank at once folds K peers'
    big-endian byte buckets that start in pinned host memory (as pulled from
    IPFS; zero-copy reads over its own PCIe link, one launch) and writes the
    BE sum bytes back to pinned host memory (commit_update's update_file),
    between host-side barriers.  Aggregate rate = all ranks' algorithmic
    bytes / the slowest rank's time (the host's memory system and every
    GPU's PCIe link are loaded together)."""
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L, device=local)
    pinned = []
    tmp = torch.empty(8 * L, dtype=torch.uint8, device="cuda")
    for k in range(K):
        ipls.synth_fill(ipls.DeviceBuffer(int(tmp.data_ptr()), L, big_endian=True), rank, k, ipls.SEED)
        pb = ipls.PinnedBuffer(8 * L)
        pb.view()[:] = tmp.cpu().numpy()
        pinned.append(pb)
    del tmp
    sum_pinned = ipls.PinnedBuffer(8 * L)
    row = [[ipls.DeviceBuffer(pb.ptr, L, big_endian=True) for pb in pinned]]

    def one_round():
        agg.reduce_batch(0, row, start_mode=ipls.START_ZERO, big_endian=True)
        agg.AggregatePartition(0, sum_out=sum_pinned)

    one_round()
    dist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(reps):
        one_round()
    dt = time.perf_counter() - t0
    times = [None] * world
    dist.all_gather_object(times, dt, group=group)
    ok = None
    if verify and rank == 0:
        from oracle import oracle as O   # checker only
        ok = ipls.checksum_dev(ipls.DeviceBuffer(sum_pinned.ptr, L, big_endian=True)) == O.c_synth_sum_checksum(L, 0, K)
    agg.close()
    for pb in pinned:
        pb.close()
    sum_pinned.close()
    per_rank = reps * (K + 1) * L * 8
    return {"workload": f"F slice per GPU: 1 partition x {K} peers x {L} doubles of BE host bytes per rank, "
                        f"all {world} ranks at once",
            "GBps_total": round(world * per_rank / max(times) / 1e9, 2),
            "GBps_per_gpu_min": round(per_rank / max(times) / 1e9, 2),
            "GBps_per_gpu_max": round(per_rank / min(times) / 1e9, 2),
            "verified_checksum_rank0": ok,
            "note": "pinned host BE buckets read zero-copy by one launch per round + AggregatePartition with the BE "
                    "sum written to pinned host memory; algorithmic bytes (K+1)*L*8 per rank per round; "
                    "PCIe Gen5 x16 per GPU ~56 GB/s per direction"}


def rccl_reduce_leg(ipls, torch, dist, rank: int, world: int, local: int, L: int, reps: int,
                    backend: str = "nccl") -> dict:
    """RCCL's own reduction (ncclReduce(sum) = dist.reduce
    over the world) of one partial per rank, against the fixed-order fold
    ((+0.0 + R_0) + R_1 ...) that the replica exchange computes bit-exactly:
    its max-ULP distance (ipls.distributed.rccl_reduce_ulp, rank 0 folds the
    gathered partials) and its time.  Every rank's partial is a synthetic
    bucket (partition 0, peer = rank).  Comparison only: the product exchange
    stays fixed-order."""
    from ipls.distributed import rccl_reduce_ulp
    x = torch.empty(L, dtype=torch.float64, device=torch.device("cuda", local))
    ipls.synth_fill(ipls.DeviceBuffer.from_tensor(x), 0, rank, ipls.SEED)
    torch.cuda.synchronize()
    if backend != "nccl":
        x = x.cpu()
    try:
        rep = rccl_reduce_ulp(x, rank, world)
    except Exception as e:     # rank 0's local fold/compare failed: keep the ranks' collectives in step
        rep = {"error": f"{type(e).__name__}: {e}"}
    red = x.clone()
    dist.reduce(red, dst=0, op=dist.ReduceOp.SUM)     # warm
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.reduce(red, dst=0, op=dist.ReduceOp.SUM)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=x.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = float(t[0].item()) / reps * 1e3
    if rank != 0:
        return {}
    rep.update(reduce_ms=round(ms, 4), L=L, backend=backend,
               reduce_GBps_in=round(world * L * 8 / ms / 1e6, 1),
               note="dist.reduce of one L-double partial per rank to rank 0 (RCCL picks the association) vs the "
                    "fixed rank-order fold from +0.0; max_ulp over all elements; reduce_GBps_in = partial bytes "
                    "of all ranks / reduce time, max over ranks")
    return rep


def replica_exchange(ipls, agg, rows, P, L, K, rank, world, local, reps, verify, backend="nccl") -> dict:
    """Config E (N > 1): a partition's contributors span GPUs.  Every rank owns
    its P partitions and folds their first K/2 peers; it is also the replica
    aggregator of P partitions owned by the other ranks (ReplicaPlan.spread:
    each rank sends partials to, and receives them from, every other rank),
    folding their last K/2 peers into a second handle.  One round = both
    folds, the exchange of the P partials each way over RCCL point-to-point
    (one batched group, every xGMI link at once), the fixed-order fold of
    the landed partials into REP and AggregatePartition (W = AGG + REP,
    IPLS.java:1256).  Reuses the main bench's bucket pool: the last K/2
    slots of each row are refilled with the replicated partitions' buckets."""
    import torch
    import torch.distributed as dist
    from ipls.distributed import RankShard, ReplicaPlan, combine_replicas, finish_exchange, start_exchange
    plan = ReplicaPlan.spread(P * world, world)
    rep_ids = plan.replicated_on(rank)
    assert len(rep_ids) == P
    kh = K // 2
    for i, p in enumerate(rep_ids):
        for k in range(kh, K):
            ipls.synth_fill(rows[i][k], p, k, ipls.SEED)
    torch.cuda.synchronize()
    own_rows = [r[:kh] for r in rows]
    rep_rows = [r[kh:] for r in rows]
    rep = ipls.Aggregator(n_partitions=P, bucket_len=L, device=local)
    xdev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")
    shard = RankShard(agg, rank * P, rep, rep_ids, device=xdev)

    def one_round():
        agg.reduce_batch(0, own_rows, start_mode=ipls.START_ZERO)
        rep.reduce_batch(0, rep_rows, start_mode=ipls.START_ZERO)
        rep.sync()
        agg.sync()
        t0 = time.perf_counter()
        combine_replicas(shard, plan, rank, device=xdev)
        agg.sync()
        t1 = time.perf_counter()
        agg.AggregatePartition(ipls.ALL_PARTITIONS)
        agg.sync()
        return t1 - t0

    def one_round_overlapped():
        # the replica partials first, then the exchange in flight on RCCL's
        # stream while this GPU folds its own partitions on the handle's stream
        rep.reduce_batch(0, rep_rows, start_mode=ipls.START_ZERO)
        ex = start_exchange(shard, plan, rank, device=xdev)
        agg.reduce_batch(0, own_rows, start_mode=ipls.START_ZERO)
        finish_exchange(ex)
        agg.AggregatePartition(ipls.ALL_PARTITIONS)
        agg.sync()

    def timed(fn):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ex = 0.0
        for _ in range(reps):
            ex += fn() or 0.0
        dist.barrier()
        dt = time.perf_counter() - t0
        t = torch.tensor([dt, ex], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0].item()) / reps, float(t[1].item()) / reps

    def check():
        if not (verify and rank == 0):
            return None
        from oracle import oracle as O              # checker only
        return agg.checksum(0, ipls.TGT_WEIGHTS) == O.c_synth_replica_checksum(L, 0, K, kh)

    one_round()                                     # warm: RCCL P2P channels, transport buffers
    verified = check()
    dt, ex = timed(one_round)
    one_round_overlapped()
    verified_ov = check()
    dt_ov, _ = timed(one_round_overlapped)
    rep.close()
    sent = P * L * 8                                # each rank sends P partials, receives P
    return {
        "workload": f"E-style: {P} partitions per GPU owned, K={K} peers split {kh}/{K - kh} between the owner "
                    f"and one replica GPU (ReplicaPlan.spread: every rank exchanges with all {world - 1} others)",
        "round_ms": round(dt * 1e3, 3),
        "exchange_ms": round(ex * 1e3, 3),
        "xgmi_bytes_per_rank_each_way": sent,
        "exchange_GBps_per_rank_each_way": round(sent / ex / 1e9, 2),
        "exchange_GBps_aggregate": round(world * sent / ex / 1e9, 2),
        "round_GBps_algorithmic": round(world * P * (K + 1) * L * 8 / dt / 1e9, 1),
        "verified_checksum_p0": verified,
        "round_ms_overlapped": round(dt_ov * 1e3, 3),
        "round_GBps_algorithmic_overlapped": round(world * P * (K + 1) * L * 8 / dt_ov / 1e9, 1),
        "verified_checksum_p0_overlapped": verified_ov,
        "note": "exchange_ms = export of the partials, one batched RCCL send/recv group, fold into REP "
                "(max over ranks); round adds both folds and AggregatePartition.  overlapped: the replica "
                "folds, then the exchange started (ipls.distributed.start_exchange) and the owner's own "
                "folds queued while it is in flight, then finish_exchange and AggregatePartition",
    }


def c_abi_multi_gpu(ipls, torch, devices, P: int, L: int, K: int, reps: int = 5, verify: bool = True) -> dict:
    """ONE C-ABI handle over several GPUs (cfg.devices), as a single JVM drives
    a node through the JNI shim: the -pa partitions sharded P per device in
    contiguous blocks (ipls_shard_plan), K peers each.
    (a) one ipls_agg_reduce_batch over all partitions: the front queues every
        shard's launch on its own stream, so the GPUs fold concurrently;
    (b) contributors spanning GPUs (the reference's replica
        aggregators, IPLS.java:1402-1468): each partition's first K/2 peers fold
        on its owner, the other K/2 on a replica slot (spread: partition q of
        owner o on GPU (o + 1 + q mod (G-1)) mod G, so every owner pulls from
        all G-1 others), ipls_agg_reduce_partial; ipls_agg_combine_partials
        then pulls each partial over xGMI with peer loads in the owner's fold
        kernel into REP, and AggregatePartition forms W = AGG + REP.
    Buckets are resident on the GPU that folds them.  Checked against the
    oracle's checksums (first and last partition; W of partition 0)."""
    G = len(devices)
    PT = P * G
    kh = K // 2
    elem = L + 32
    pools, rows = [], []
    for s, d in enumerate(devices):
        with torch.cuda.device(d):
            t = torch.empty(P * K * elem + 32, dtype=torch.float64, device=f"cuda:{d}")
            base = (int(t.data_ptr()) + 255) // 256 * 256
            pools.append(t)
            for q in range(P):
                row = [ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L) for k in range(K)]
                for k in range(K):
                    ipls.synth_fill(row[k], s * P + q, k, ipls.SEED)
                rows.append(row)
    for d in sorted(set(devices)):
        torch.cuda.synchronize(d)
    agg = ipls.Aggregator(n_partitions=PT, bucket_len=L, devices=list(devices))
    out = {"devices": list(devices), "workload": f"{PT} partitions ({P} per GPU) x {L} doubles x {K} peers, "
                                                 f"one handle over {G} GPUs"}
    agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
    agg.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
    agg.sync()
    dt = (time.perf_counter() - t0) / reps
    nbytes = PT * (K + 1) * L * 8
    out["reduce_ms"] = round(dt * 1e3, 4)
    out["reduce_GBps"] = round(nbytes / dt / 1e9, 1)
    out["reduce_GBps_per_gpu"] = round(nbytes / dt / 1e9 / G, 1)
    if verify:
        from oracle import oracle as O   # checker only
        out["verified_checksums"] = (agg.checksum(0) == O.c_synth_sum_checksum(L, 0, K) and
                                     agg.checksum(PT - 1) == O.c_synth_sum_checksum(L, PT - 1, K))
    if G > 1:
        slot = {}
        for o in range(G):
            for q in range(P):
                slot[o * P + q] = (o + 1 + q % (G - 1)) % G
        spare = {s: [rows[s * P + q][kh:] for q in range(P)] for s in range(G)}
        far = {}
        for p in range(PT):
            s = slot[p]
            far[p] = spare[s].pop(0)
            with torch.cuda.device(devices[s]):
                for k in range(kh, K):
                    ipls.synth_fill(far[p][k - kh], p, k, ipls.SEED)
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)
        own = [r[:kh] for r in rows]

        links = [len({devices[slot[o * P + q]] for q in range(P)} - {devices[o]}) for o in range(G)]

        def measure(h, staged: bool) -> dict:
            # per owner shard: its stream (HIP events around the combine's launch there)
            owner_streams = []
            for o in range(G):
                d, st = h.partition_device(o * P)
                owner_streams.append(torch.cuda.ExternalStream(st, device=torch.device("cuda", d)))

            def one_round():
                h.reduce_batch(0, own, start_mode=ipls.START_ZERO)
                for p in range(PT):
                    h.reduce_partial(slot[p], p, [far[p]], start_mode=ipls.START_ZERO)
                h.sync()
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(G)]
                for o in range(G):
                    evs[o][0].record(owner_streams[o])
                t0 = time.perf_counter()
                n = h.combine_partials()
                for o in range(G):
                    evs[o][1].record(owner_streams[o])
                h.sync()
                t1 = time.perf_counter()
                h.AggregatePartition(ipls.ALL_PARTITIONS)
                h.sync()
                return t1 - t0, n, [a.elapsed_time(b) for a, b in evs]
            one_round()
            ex, per_owner = [], []
            for _ in range(reps):
                t, _, ev_ms = one_round()
                ex.append(t)
                per_owner.append(ev_ms)
            tex = float(np.median(ex))
            # the combine's roofline: per owner, its P partials arrive
            # over the xGMI links of the distinct GPUs holding them; algorithmic
            # bytes = partials * L * 8 over xGMI + L * 8 REP write per partition
            # (+ L * 8 REP read when REP already held a value -- not in this leg)
            own_ms = np.median(np.asarray(per_owner), axis=0)
            xg = P * L * 8
            fr = [xg / (own_ms[o] / 1e3) / (links[o] * XGMI_LINK_GBS * 1e9) if links[o] else None for o in range(G)]
            res = {
                "transfer": ("hipMemcpyPeerAsync of each partial into an owner-side buffer, then the fold "
                             "(IPLS_PEER_STAGED=1)" if staged else "peer loads in the owner's fold kernel"),
                "combine_ms": round(tex * 1e3, 4), "combine_xgmi_GBps": round(PT * L * 8 / tex / 1e9, 1),
                "bytes_formula": "per partition: S*L*8 (S remote partials over xGMI) + L*8 (REP write) [+ L*8 REP read]",
                "xgmi_bytes_per_owner": xg, "algorithmic_bytes_per_owner": xg + P * L * 8,
                "owner_kernel_ms": [round(float(x), 4) for x in own_ms], "links_per_owner": links,
                "xgmi_link_GBps": XGMI_LINK_GBS,
                "frac_of_xgmi": [None if f is None else round(f, 4) for f in fr],
                "frac_of_xgmi_min": None if None in fr else round(min(fr), 4),
                "staged_partials": h.last_launch()["staged"],
                "status": ("rehearsal: every shard on one GPU, local reads (no xGMI link); unmeasured on hardware"
                           if len(set(devices)) == 1 else "measured: distinct GPUs over xGMI"),
                "timing": "HIP events on each owner's stream around the combine (median of the rounds); "
                          "combine_ms = host wall time of the combine call + sync"}
            if verify:
                from oracle import oracle as O   # checker only
                res["verified_replica_checksum_p0"] = (h.checksum(0, ipls.TGT_WEIGHTS) ==
                                                       O.c_synth_replica_checksum(L, 0, K, kh))
            return res

        out["combine"] = measure(agg, False)
        out["combine_ms"] = out["combine"]["combine_ms"]
        out["combine_xgmi_GBps"] = out["combine"]["combine_xgmi_GBps"]
        out["verified_replica_checksum_p0"] = out["combine"].get("verified_replica_checksum_p0")
        out["combine_note"] = (f"{PT} partials of {L * 8 / 2**20:.0f} MiB pulled by their owners "
                               "(peer loads over xGMI; shards on one GPU read local memory), folded into REP in "
                               "slot order; median of the combine step alone")
        # the other transfer: each partial copied to its owner first (the
        # no-peer-access fallback, forced), then the same fold -- copy engines
        # instead of the owner's CUs pulling over xGMI
        agg.close()
        os.environ["IPLS_PEER_STAGED"] = "1"
        try:
            agg = ipls.Aggregator(n_partitions=PT, bucket_len=L, devices=list(devices))
        finally:
            del os.environ["IPLS_PEER_STAGED"]
        out["combine_staged"] = measure(agg, True)
    agg.close()
    del pools, rows
    torch.cuda.empty_cache()
    return out


def config_leg(ipls, torch, name: str, be: bool, device: int, steps: int = 5, verify: bool = True,
               rounds: int = 4, build: dict | None = None) -> dict:
    """One more BASELINE config on the same box, N=1: B
    (16 x 1M x 8, native doubles) or D (64 x 4M x 32) with big-endian IPFS
    bytes in and the sum packed to big-endian bytes out, i.e. config D's
    'double<->byte pack/unpack in the timed region', or F (one GPU's slice of
    config F: 16 x 8M x 64, 69.8 GB of buckets resident).  Same algorithmic-bytes
    accounting as the headline; kernel time by HIP events on the handle's
    stream at the two ends of each of `rounds` rounds of `steps` back-to-back
    launches (so it includes the ~1.6 us boundary between launches), the
    median round reported
    (the first launches after a fresh allocation can run a few % slow);
    partition 0 checked against the oracle's checksum."""
    P, L, K = CONFIGS[name]
    elem = L + 32
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L, big_endian=be) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], q, k, ipls.SEED)
    out_arena = torch.empty(P * elem + 32, dtype=torch.float64, device="cuda")
    obase = (int(out_arena.data_ptr()) + 255) // 256 * 256
    dsts = [obase + 8 * q * elem for q in range(P)]
    torch.cuda.synchronize()
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, device=device)
    stream = torch.cuda.ExternalStream(agg.stream, device=torch.device("cuda", device))

    def step():
        agg.reduce_batch_out(0, rows, dsts, start_mode=ipls.START_ZERO, big_endian_in=be, big_endian_out=be)
    step()
    step()
    agg.sync()
    # one HIP event at each end of a round of back-to-back launches: an event
    # packet after every launch added 4.6 us to each 0.18 ms B launch (2.5 % of
    # the line, tools/b_gap_probe.py, profiles/r05/b_gap/); what remains
    # between launches is the in-order dependent-launch boundary (~1.6 us)
    # and one untimed launch before the first event keeps the GPU busy while the
    # timed ones are issued, so the first launch's host latency (~55 us per
    # call here) is not in the span
    per_round = []
    for _ in range(rounds):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        step()
        ev0.record(stream)
        for i in range(steps):
            step()
        ev1.record(stream)
        agg.sync()
        per_round.append(ev0.elapsed_time(ev1) / steps)
    ms = float(np.median(per_round))
    launch = agg.last_launch()
    nbytes = P * (K + 1) * L * 8
    verified = None
    checked = []
    if verify:
        from oracle import oracle as O   # checker only
        # every partition of B and F; every 4th and the last of D's 64 (its
        # oracle checksums cost ~0.25 s each on the host)
        checked = list(range(P)) if P <= 16 else sorted(set(range(0, P, 4)) | {P - 1})
        good = sum(int(ipls.checksum_dev(ipls.DeviceBuffer(dsts[q], L, big_endian=be))
                       == O.c_synth_sum_checksum(L, q, K)) for q in checked)
        verified = f"{good}/{len(checked)}"
    agg.close()
    del arena, out_arena, rows
    torch.cuda.empty_cache()
    # HBM bytes per launch from the committed PMC passes of this config, for this build only
    traffic, traffic_prov = pmc_traffic(f"{name}{'-be' if be else ''}", build or {})
    return {"workload": f"{name}: {P} partitions x {L} doubles x {K} peers"
                        + (" (BE IPFS bytes in, BE sum bytes out: fused unpack/pack)" if be else ""),
            "kernel_ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1),
            "frac": round(nbytes / ms / 1e6 / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": nbytes,
            "round_ms": [round(x, 4) for x in per_round],
            "launch": {k: launch[k] for k in ("shape", "block", "vectors", "seqf", "map", "grid")},
            "traffic": traffic, "traffic_provenance": traffic_prov,
            "verified_partitions": verified,
            "verified_which": "all" if len(checked) == P else f"p = 0, 4, 8, ..., {P - 1}"}


def be_schedule_ab(ipls, torch, device: int, rounds: int = 4, steps: int = 5, verify: bool = True) -> dict:
    """Config D's big-endian schedules A/B'd in ONE process on the SAME
    buckets: the shipped library (R = 16, a fence after
    every 3 vectors) against round 1's R = 16 fence-every-2-last-4-free
    (IPLS_BE_SEQF=42) and hipcc's own schedule at R = 8, each a build of the
    same sources (make -C ipls-java-api_amd variants) loaded beside the
    shipped one.  64 x 4M x 32 BE buckets in, BE sums out; the variants'
    launches are interleaved round by round so the layout is
    common to all three; HIP events on each handle's stream."""
    from ipls import _native as N
    P, L, K = CONFIGS["D"]
    ab = N.PKG_ROOT / "lib" / "ab"
    libs = {"shipped_seqf3": None, "seqf42": N.load(ab / "libipls_agg_seqf42.so"),
            "r8_compiler": N.load(ab / "libipls_agg_r8.so")}
    elem = L + 32
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L, big_endian=True) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], q, k, ipls.SEED)
    out_arena = torch.empty(P * elem + 32, dtype=torch.float64, device="cuda")
    obase = (int(out_arena.data_ptr()) + 255) // 256 * 256
    dsts = [obase + 8 * q * elem for q in range(P)]
    torch.cuda.synchronize()
    nbytes = P * (K + 1) * L * 8
    aggs = {nm: ipls.Aggregator(n_partitions=P, bucket_len=L, device=device, library=lb) for nm, lb in libs.items()}
    res = {nm: {"ms": [], "launch": None, "verified_checksum_p0": None} for nm in libs}
    for r in range(rounds):
        for nm, agg in aggs.items():
            stream = torch.cuda.ExternalStream(agg.stream, device=torch.device("cuda", device))
            agg.reduce_batch_out(0, rows, dsts, start_mode=ipls.START_ZERO, big_endian_in=True, big_endian_out=True)
            agg.sync()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
            ev[0].record(stream)
            for i in range(steps):
                agg.reduce_batch_out(0, rows, dsts, start_mode=ipls.START_ZERO, big_endian_in=True,
                                     big_endian_out=True)
                ev[i + 1].record(stream)
            agg.sync()
            res[nm]["ms"].append(round(float(np.mean([ev[i].elapsed_time(ev[i + 1]) for i in range(steps)])), 4))
            if r == 0:
                res[nm]["launch"] = agg.last_launch()
                if verify:
                    from oracle import oracle as O   # checker only
                    res[nm]["verified_checksum_p0"] = (
                        ipls.checksum_dev(ipls.DeviceBuffer(dsts[0], L, big_endian=True)) ==
                        O.c_synth_sum_checksum(L, 0, K))
    for nm, agg in aggs.items():
        agg.close()
        ms = float(np.median(res[nm]["ms"]))
        res[nm].update(median_ms=round(ms, 4), frac=round(nbytes / ms / 1e6 / HBM_PEAK_GBS, 4))
    del arena, out_arena, rows
    torch.cuda.empty_cache()
    return {"workload": f"D: {P} x {L} x {K}, BE in + BE out", "rounds": rounds, "steps_per_round": steps,
            "algorithmic_bytes_per_launch": nbytes, "variants": res}


def few_partitions_leg(ipls, torch, device: int, P: int = 3, L: int = 4194304, K: int = 32, steps: int = 10,
                       verify: bool = True) -> dict:
    """A shard's share when -pa is small (-pa 24 over 8 GPUs: 3 partitions of
    4M per GPU), N=1, never the value: the fold and the fused round on 3 x 4M
    x 32, which run the 512-lane half shape; HIP events over
    back-to-back launches, partition 0 checked against the oracle."""
    elem = L + 32
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], q, k, ipls.SEED)
    avg = torch.empty(P * (L - 1) + 2, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, device=device)
    stream = torch.cuda.ExternalStream(agg.stream, device=torch.device("cuda", device))
    out = {"workload": f"{P} partitions x {L} doubles x {K} peers (a GPU's share of -pa {8 * P} over 8 GPUs)"}
    for name, fn, nbytes in (
            ("fold", lambda: agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO), P * (K + 1) * L * 8),
            ("fused_round", lambda: agg.aggregate_round(0, rows, out=ipls.DeviceBuffer.from_tensor(avg)),
             P * (K + 2) * L * 8)):
        fn()
        agg.sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()   # untimed, in flight while the timed launches are issued
        e0.record(stream)
        for _ in range(steps):
            fn()
        e1.record(stream)
        agg.sync()
        ms = e0.elapsed_time(e1) / steps
        li = agg.last_launch()
        out[name] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1),
                     "frac": round(nbytes / ms / 1e6 / HBM_PEAK_GBS, 4),
                     "launch": {k: li[k] for k in ("shape", "block", "vectors", "map", "grid")}}
    if verify:
        from oracle import oracle as O   # checker only
        out["verified_checksum_p0"] = agg.checksum(0, ipls.TGT_WEIGHTS) == O.c_synth_sum_checksum(L, 0, K)
    agg.close()
    del arena, avg, rows
    torch.cuda.empty_cache()
    return out


def config_a_leg(ipls, reps: int = 20) -> dict:
    """BASELINE configs[0], the reference's own CPU-runnable case: ETHModel
    (M = 443,610, tests/golden/ethmodel.f64be.gz), -pa 3 -n 3, three peers.
    One round as the Java API runs it: UpdateGradient of this peer's
    gradients (IPLS.java:1737), the two other peers' partitions arriving as
    `ipfs cat` BE bytes (Updater._Update), AggregatePartition for the three
    partitions and GetPartitions -- host memory in, host memory out.  Beside
    it the CPU port of the reference's loop on the same bytes (BE decode +
    fold per bucket, then the divide; 1 thread).  The averaged models must be
    bit-identical.  A latency line (14 MB of buckets), never the value."""
    import gzip
    from oracle import oracle as O   # checker + the CPU port timed beside the GPU round
    raw = gzip.decompress((Path(__file__).resolve().parent / "tests" / "golden" / "ethmodel.f64be.gz").read_bytes())
    model = np.frombuffer(raw, dtype=">f8").astype(np.float64)
    M, P = model.size, 3
    peers = [model + O.synth_bucket(M + 1, 0, k)[:M] for k in range(3)]
    parts = [O.organize_gradients(g, M, P) for g in peers]
    be = [[np.frombuffer(O.be_encode(parts[k][p]), dtype=np.uint8) for p in range(P)] for k in range(3)]
    agg = ipls.Aggregator(M, P, max_peers=3)

    def gpu_round():
        agg.UpdateGradient(peers[0], auth_list=[0, 1, 2])
        for k in (1, 2):
            for p in range(P):
                agg.Update(be[k][p].tobytes(), p)
        for p in range(P):
            agg.AggregatePartition(p)
        return agg.GetPartitions()

    def cpu_round():
        out = []
        for p in range(P):
            s = O.c_updater_loop([be[k][p] for k in range(3)], len(parts[0][p]))
            out.append(O.c_divide(s))
        return np.concatenate(out)

    # the same round the way INTEGRATION.md §4 wires it: the `ipfs cat` bytes
    # and this peer's gradients land in pinned memory (direct ByteBuffers from
    # hostAlloc), the kernels read them over PCIe (zero copy), and one fused
    # launch does the folds + AggregatePartition(all) + GetPartitions into a
    # pinned output (ipls_agg_aggregate_round): two C-ABI calls per round
    pin_own = ipls.PinnedBuffer(8 * M)
    pin_own.view()[:] = np.frombuffer(peers[0].tobytes(), dtype=np.uint8)
    pin_be = [[None] * P for _ in range(3)]
    for k in (1, 2):
        for p in range(P):
            pin_be[k][p] = ipls.PinnedBuffer(be[k][p].size)
            pin_be[k][p].view()[:] = be[k][p]
    pin_out = ipls.PinnedBuffer(8 * M)
    own_dev = ipls.DeviceBuffer(pin_own.ptr, M)
    rows = [[ipls.DeviceBuffer(pin_be[k][p].ptr, len(parts[0][p]), big_endian=True) for k in (1, 2)]
            for p in range(P)]
    out_dev = ipls.DeviceBuffer(pin_out.ptr, M)

    def gpu_round_pinned():
        agg.UpdateGradient(own_dev, auth_list=[0, 1, 2])
        agg.aggregate_round(0, rows, big_endian=True, out=out_dev)
        agg.sync()
        return np.frombuffer(bytes(pin_out.view()[:8 * M]), dtype=np.float64)

    got, want = gpu_round(), cpu_round()
    same = bool(np.array_equal(got.view(np.int64), want.view(np.int64)))
    got_p = gpu_round_pinned()
    same_p = bool(np.array_equal(got_p.view(np.int64), want.view(np.int64)))
    t0 = time.perf_counter()
    for _ in range(reps):
        gpu_round()
    g_ms = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    for _ in range(reps):
        agg.UpdateGradient(own_dev, auth_list=[0, 1, 2])
        agg.aggregate_round(0, rows, big_endian=True, out=out_dev)
        agg.sync()
    gp_ms = (time.perf_counter() - t0) / reps * 1e3
    for b in [pin_own, pin_out] + [x for k in (1, 2) for x in pin_be[k]]:
        b.close()
    t0 = time.perf_counter()
    for _ in range(reps):
        cpu_round()
    c_ms = (time.perf_counter() - t0) / reps * 1e3
    agg.close()
    return {"workload": "A: ETHModel M=443,610, -pa 3 -n 3, 3 peers (host buffers in, averaged model out)",
            "gpu_round_ms": round(g_ms, 3), "cpu_port_round_ms": round(c_ms, 3), "cpu_port_cores": 1,
            "bit_identical": same,
            "gpu_round_pinned_fused_ms": round(gp_ms, 3), "pinned_fused_bit_identical": same_p,
            "pinned_fused_note": "buckets and own gradients in pinned host memory (direct ByteBuffers), read over "
                                 "PCIe by the kernels; UpdateGradient + one ipls_agg_aggregate_round (folds + "
                                 "AggregatePartition(all) + GetPartitions) writing the model to pinned memory",
            "note": f"wall time per round, mean of {reps}; GPU = Python caller through the C-ABI (H2D of 9 BE "
                    "buckets + own gradients, folds, AggregatePartition, divide, D2H of the model); CPU = the C "
                    "port of the Updater BE decode + fold and the GetPartitions divide"}


def per_arrival_leg(ipls, torch, agg, rows, P: int, L: int, K: int, stream, verify: bool, reps: int = 7) -> dict:
    """The headline workload folded the way Updater._Update folds its queue
    (Updater.java:115-117): one call per arriving bucket, peers arriving in
    turn (peer 0's P buckets, then peer 1's ...).  'each' is one fold launch
    per arrival (ipls_agg_accumulate: 24 B of HBM traffic per element);
    'coalesced' queues the device buckets (ipls_agg_accumulate_async) and folds
    them together when the queues fill.  Time = HIP events on the handle's
    stream around the K*P calls, so it includes the host-side queueing; bytes
    are the batch's algorithmic P*(K+1)*L*8.  Never the value."""
    nbytes = P * (K + 1) * L * 8
    out = {}
    want = None
    if verify:
        from oracle import oracle as O   # checker only
        want = O.c_synth_sum_checksum(L, 0, K)
    for mode in ("each", "coalesced", "coalesced_per_peer"):
        times = []
        for _ in range(reps):
            agg.reset()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            t = 0
            for k in range(K):
                if mode == "coalesced_per_peer":     # one call for peer k's P buckets (UpdateAsyncMany)
                    t = agg.UpdateAsyncMany([(rows[q][k], q) for q in range(P)])
                    continue
                for q in range(P):
                    if mode == "each":
                        agg.Update(rows[q][k], q)
                    else:
                        t = agg.UpdateAsync(rows[q][k], q)
            if mode != "each":
                agg.Wait(t)
            e1.record(stream)
            agg.sync()
            times.append(e0.elapsed_time(e1))
        best, med = min(times), float(np.median(times))
        out[mode] = {"ms": round(best, 4), "GBps": round(nbytes / best / 1e6, 1),
                     "frac": round(nbytes / best / 1e6 / HBM_PEAK_GBS, 4),
                     "ms_median": round(med, 4), "frac_median": round(nbytes / med / 1e6 / HBM_PEAK_GBS, 4),
                     "verified_checksum_p0": (agg.checksum(0) == want) if verify else None}
    out["note"] = ("one call per arriving bucket (peer-major); each = a fold launch per arrival, "
                   "coalesced = queued device buckets folded together (ipls_agg_accumulate_async), "
                   "coalesced_per_peer = the same queue fed one call per peer (Aggregator.UpdateAsyncMany: "
                   "one Python -> C transition for a peer's P buckets), best (and median) of "
                   f"{reps}; algorithmic bytes P*(K+1)*L*8; Python caller through "
                   + ("ipls._fast (CPython extension, csrc/pyfast.c)" if agg._fast is not None else "ctypes"))
    # the same calls from a native caller (what a JNI shim sees): tools/host_e2e.cpp, a child process
    exe = Path(__file__).resolve().parent / "ipls-java-api_amd" / "lib" / "host_e2e"
    if exe.exists():
        import subprocess
        r = subprocess.run([str(exe), str(L), str(K), "3", str(P), "--device-only"], capture_output=True,
                           text=True, timeout=180)
        native = {}
        for line in r.stdout.splitlines():
            for key, tag in (("each", "one launch per arrival"), ("coalesced", "queued"), ("batch", "reduce_batch")):
                if line.startswith("device,") and tag in line:
                    f = line.split()
                    ms = float(f[f.index("best") + 1])
                    native[key] = {"ms": ms, "GBps": round(nbytes / ms / 1e6, 1),
                                   "frac": round(nbytes / ms / 1e6 / HBM_PEAK_GBS, 4)}
        native["source"] = "tools/host_e2e.cpp --device-only (C-ABI calls, no Python), wall clock, best of 3"
        out["native_c_abi"] = native if r.returncode == 0 else {"error": r.stderr[-300:]}
    return out


def round_leg(ipls, torch, agg, rows, P: int, L: int, K: int, stream, kern_ms: float, build: dict | None = None,
              config: str = "C") -> dict:
    """The rest of an aggregation round on the same handle, one launch each:
    AggregatePartition for all partitions (k_finalize: read AGG, write W ->
    16 B/element) and GetPartitions into a device buffer (k_divide: read W,
    write the flat model -> 16 B/element); then the same round fused into one
    launch (ipls_agg_aggregate_round), checked bit-identical."""
    flat = torch.empty(P * (L - 1), dtype=torch.float64, device="cuda")
    fb = ipls.DeviceBuffer.from_tensor(flat)
    # finalize / divide: each reads a freshly folded AGG, so one launch per
    # round; 5 rounds, median of each launch
    fin, div = [], []
    for _ in range(5):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)
        e[0].record(stream)
        agg.AggregatePartition(ipls.ALL_PARTITIONS)
        e[1].record(stream)
        agg.GetPartitions(out=fb)
        e[2].record(stream)
        agg.sync()
        fin.append(e[0].elapsed_time(e[1]))
        div.append(e[1].elapsed_time(e[2]))
    fin_ms, div_single_ms = float(np.median(fin)), float(np.median(div))
    # GetPartitions only reads W, so the divide can also run back to back: 20
    # launches between two events (no event packet between launches, like the
    # config legs), the steady-state per-launch time
    agg.sync()
    d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    agg.GetPartitions(out=fb)   # untimed, in flight while the timed launches are issued (no launch latency in d0..d1)
    d0.record(stream)
    for _ in range(20):
        agg.GetPartitions(out=fb)
    d1.record(stream)
    agg.sync()
    div_ms = d0.elapsed_time(d1) / 20
    n_el = P * L
    ref_flat = flat.clone()
    # the same round as ONE launch (ipls_agg_aggregate_round): folds + W + averages;
    # one untimed call first (its descriptor table upload), then 20 back to back
    agg.aggregate_round(0, rows, out=fb)
    reps = 20
    fe = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    for i in range(reps):
        fe[i].record(stream)
        agg.aggregate_round(0, rows, out=fb)
    fe[reps].record(stream)
    agg.sync()
    fused_ms = fe[0].elapsed_time(fe[reps]) / reps
    fused_same = bool(torch.equal(flat.view(torch.int64), ref_flat.view(torch.int64)))
    fused_bytes = P * (K + 1) * L * 8 + 8 * (n_el - P)   # K buckets in, W out, averages out
    # HBM bytes per launch from the committed PMC passes of this build (as roofline.traffic)
    fin_t, fin_prov = pmc_traffic(f"{config}-finalize", build or {})
    div_t, div_prov = pmc_traffic(f"{config}-divide", build or {})
    info = {
        "finalize_ms": round(fin_ms, 4), "finalize_GBps": round(16 * n_el / fin_ms / 1e6, 1),
        "finalize_frac": round(16 * n_el / fin_ms / 1e6 / HBM_PEAK_GBS, 4),
        "finalize_algorithmic_bytes": 16 * n_el, "finalize_traffic": fin_t, "finalize_traffic_provenance": fin_prov,
        "divide_ms": round(div_ms, 4), "divide_ms_single_launch": round(div_single_ms, 4),
        "divide_GBps": round(16 * (n_el - P) / div_ms / 1e6, 1),
        "divide_frac": round(16 * (n_el - P) / div_ms / 1e6 / HBM_PEAK_GBS, 4),
        "divide_algorithmic_bytes": 16 * (n_el - P), "divide_traffic": div_t, "divide_traffic_provenance": div_prov,
        "round_ms": round(kern_ms + fin_ms + div_single_ms, 4),
        "fused_round_ms": round(fused_ms, 4),
        "fused_round_GBps": round(fused_bytes / fused_ms / 1e6, 1),
        "fused_round_bit_identical": fused_same,
        "note": "one aggregation round on device: reduce (K buckets) + AggregatePartition(all) + GetPartitions "
                "as three launches (round_ms), and fused into one (fused_round_ms); finalize_ms: one launch "
                "between two events (it consumes AGG, so it cannot repeat); divide_ms: 20 back-to-back launches",
    }
    del flat, ref_flat
    return info


def publish_leg(ipls, torch, agg, stream, L: int, reps: int = 10, verify: bool = True) -> dict:
    """a9: the aggregator's partial sum published every round (IPLS.java:
    1429-1430: Marshall_Packet + Base64.getUrlEncoder, MyIPFSClass.java:
    990-1016), encoded on the GPU straight from an accumulator
    (k_b64url_encode_frame): here Weights[0], which the fused round left
    holding partition 0's sum (AGG is logically zero after it; same kernel).
    Device text: HIP events around the call on the handle's stream;
    algorithmic bytes = 8 L read + the text written.  Host text: wall clock,
    the D2H of the text included (PCIe-bound).  Checked against the oracle's
    Java encoder on the partition's values."""
    origin = b"QmPublishingPeerIdentity0123456789abcdefghijk"   # a 46-char IPFS peer id
    text_len = 4 * -(-(14 + 8 * L + len(origin)) // 3)
    buf = torch.empty(text_len + 64, dtype=torch.uint8, device="cuda")
    ptr = int(buf.data_ptr())
    agg.publish_partial(0, 7, 33, origin=origin, target=ipls.TGT_WEIGHTS, out=ptr, out_cap=text_len + 64)
    agg.sync()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(stream)
    for i in range(reps):
        agg.publish_partial(0, 7, 33, origin=origin, target=ipls.TGT_WEIGHTS, out=ptr, out_cap=text_len + 64)
        ev[i + 1].record(stream)
    agg.sync()
    ms = float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]))
    nbytes = 8 * L + text_len
    pinned = ipls.PinnedBuffer(text_len)
    agg.publish_partial(0, 7, 33, origin=origin, target=ipls.TGT_WEIGHTS, out=pinned)
    t0 = time.perf_counter()
    for _ in range(5):
        agg.publish_partial(0, 7, 33, origin=origin, target=ipls.TGT_WEIGHTS, out=pinned)
    dt = (time.perf_counter() - t0) / 5
    host = bytes(pinned.view()[:text_len])
    pinned.close()
    ok = None
    if verify:
        from oracle import oracle as O   # checker only
        ok = (host == O.java_b64url_encode(O.frame_encode(agg.read(0, ipls.TGT_WEIGHTS), 7, 33, 3, origin)) and
              bytes(buf[:text_len].cpu().numpy()) == host)
    del buf
    # a round's publish loop over all P partitions (IPLS.java:1423-1431): P
    # single calls vs one ipls_agg_publish_partials launch, device text
    P = agg.n_partitions
    parts, bs = list(range(P)), [33] * P
    total = 0
    for _ in range(P):
        total = (total + 63) // 64 * 64 + text_len
    big = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    bptr = int(big.data_ptr())
    lens, offs = agg.publish_partials(parts, 7, bs, origin=origin, target=ipls.TGT_WEIGHTS, out=bptr, out_cap=total + 64)
    agg.sync()
    ev2 = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    t_loop, t_batch = [], []
    for _ in range(reps):
        ev2[0].record(stream)
        for p in parts:
            agg.publish_partial(p, 7, 33, origin=origin, target=ipls.TGT_WEIGHTS, out=bptr + offs[p],
                                  out_cap=total + 64 - offs[p])
        ev2[1].record(stream)
        agg.publish_partials(parts, 7, bs, origin=origin, target=ipls.TGT_WEIGHTS, out=bptr, out_cap=total + 64)
        ev2[2].record(stream)
        agg.sync()
        t_loop.append(ev2[0].elapsed_time(ev2[1]))
        t_batch.append(ev2[1].elapsed_time(ev2[2]))
    ok_all = None
    if verify:
        from oracle import oracle as O   # checker only
        host_all = big.cpu().numpy().tobytes()
        ok_all = all(host_all[offs[p]:offs[p] + lens[p]] ==
                     O.java_b64url_encode(O.frame_encode(agg.read(p, ipls.TGT_WEIGHTS), 7, 33, 3, origin))
                     for p in (0, P - 1))
    del big
    ms_loop, ms_batch = float(np.median(t_loop)), float(np.median(t_batch))
    all_bytes = P * nbytes
    all_parts = {"partitions": P, "loop_ms": round(ms_loop, 4), "batch_ms": round(ms_batch, 4),
                 "batch_GBps": round(all_bytes / ms_batch / 1e6, 1),
                 "batch_frac": round(all_bytes / ms_batch / 1e6 / HBM_PEAK_GBS, 4),
                 "verified_first_last_vs_java_encoder": ok_all,
                 "note": "the round's publish of every partition: P ipls_agg_publish_partial calls vs one "
                         "ipls_agg_publish_partials launch (texts at 64-B aligned offsets), HIP events"}
    return {"partition_doubles": L, "text_bytes": text_len, "device_ms": round(ms, 4),
            "device_GBps": round(nbytes / ms / 1e6, 1), "device_frac": round(nbytes / ms / 1e6 / HBM_PEAK_GBS, 4),
            "host_text_ms": round(dt * 1e3, 3), "host_text_GBps": round(text_len / dt / 1e9, 2),
            "verified_vs_java_encoder": ok, "all_partitions": all_parts,
            "note": "Marshall_Packet(W[0], origin, 7, 33, pid 3) -> base64url with padding; device_GBps counts "
                    "8L read + the text written; host_text: the same call with the text landing in pinned host "
                    "memory (C-ABI call wall time, D2H included)"}


def strong_leg(ipls, torch, dist, rank: int, world: int, local: int, steps: int = 5, verify: bool = True) -> dict:
    """Fixed total work ('at fixed total work (config D)'):
    config D's 64 partitions x 4M doubles x 32 peers split over the ranks in
    contiguous blocks, native doubles, no data-path collective.  Timed like the
    headline: barrier + sync on both sides, max over ranks; bytes = the whole
    config's algorithmic bytes.  Never the value."""
    P_all, L, K = CONFIGS["D"]
    if P_all % world:
        return {"error": f"{P_all} partitions do not split over {world} ranks"}
    P = P_all // world
    p0 = rank * P
    elem = L + 32
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = [[ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L) for k in range(K)] for q in range(P)]
    for q in range(P):
        for k in range(K):
            ipls.synth_fill(rows[q][k], p0 + q, k, ipls.SEED)
    torch.cuda.synchronize()
    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, device=local)
    agg.reduce_batch(0, rows)
    agg.sync()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        agg.reduce_batch(0, rows)
    agg.sync()
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ok = None
    if verify and rank == 0:
        from oracle import oracle as O   # checker only
        ok = agg.checksum(0) == O.c_synth_sum_checksum(L, 0, K)
    agg.close()
    del arena, rows
    torch.cuda.empty_cache()
    total = P_all * (K + 1) * L * 8 * steps
    return {"workload": f"D: {P_all} partitions x {L} doubles x {K} peers in total, {P} per rank",
            "ms_per_step": round(dt / steps * 1e3, 4), "GBps_total": round(total / dt / 1e9, 1),
            "GBps_per_gpu": round(total / dt / 1e9 / world, 1), "verified_checksum_p0": ok}


def pmc_traffic(workload_key: str, build: dict):
    """HBM bytes per launch from the committed rocprofv3 PMC passes for this
    workload (profiles/pmc_traffic.json), tied to the code that was profiled:
    every entry carries the build record (ipls.build_info()) of the process the
    counters came from.  Returns (traffic or None, provenance).  The traffic is
    reported only when the entry was taken on this very library (same .so
    sha256), on a library with the same device code (sha256 of the .so's
    .hip_fatbin section: the same kernel ISA, host code changed), or on one
    built from the same kernel sources (ipls_kernels.hpp + engine.hip);
    otherwise None with traffic_stale = True."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    prov = {"source": "profiles/pmc_traffic.json", "entry": workload_key, "traffic_stale": True, "match": None}
    try:
        e = json.loads(f.read_text()).get(workload_key)
    except (OSError, ValueError):
        e = None
    if e is None:
        prov["why"] = "no PMC entry for this workload"
        return None, prov
    eb = e.get("build") or {}
    prov.update(entry_git_rev=eb.get("git_rev"), entry_so_sha256=eb.get("so_sha256"), profile=e.get("source"))
    if eb.get("so_sha256") and eb.get("so_sha256") == build.get("so_sha256"):
        prov.update(traffic_stale=False, match="so_sha256")
    elif eb.get("device_code_sha256") and eb.get("device_code_sha256") == build.get("device_code_sha256"):
        prov.update(traffic_stale=False, match="device_code_sha256")    # same kernel ISA, host code changed
    elif eb.get("kernel_src_sha256") and eb.get("kernel_src_sha256") == build.get("kernel_src_sha256"):
        prov.update(traffic_stale=False, match="kernel_src_sha256")
    else:
        prov["why"] = "the PMC entry was taken on another build of the kernels"
        return None, prov
    return e.get("hbm_bytes_per_launch"), prov


class Watchdog:
    """Bounds the N>1 side legs (replica exchange, strong-scaling D, the
    all-ranks host-inclusive leg, the single-handle C-ABI leg).  On expiry it
    records the leg that was running as {"error": "timed out ..."} in the JSON
    line, prints the line (rank 0, once) and ends the process with EXIT_CODE:
    a stuck RCCL/xGMI exchange must show up as a failed run, never as rc 0."""
    EXIT_CODE = 3

    def __init__(self, timeout: float, out):
        import threading
        self.timeout = timeout
        self.out = out                 # rank 0's line (None on other ranks)
        self.stage = ["replica_exchange"]
        self._lock = threading.Lock()
        self._state = "running"        # -> "finished" (main prints) or "expired" (the dog prints and exits)
        self._t = threading.Timer(timeout, self.expire)
        self._t.daemon = True

    def start(self):
        self._t.start()

    def cancel(self):
        """The legs are done: True if the main thread may print the line.  If
        the dog already fired, this thread parks until its os._exit ends it."""
        with self._lock:
            if self._state == "running":
                self._state = "finished"
                self._t.cancel()
                return True
        time.sleep(3600)
        return False

    def expire(self):
        with self._lock:
            if self._state != "running":
                return
            self._state = "expired"
        msg = f"timed out after {self.timeout} s (watchdog; exit code {self.EXIT_CODE})"
        if self.out is not None:
            self.out[self.stage[0]] = {"error": msg}
            self.out["watchdog"] = {"expired": True, "stage": self.stage[0], "exit_code": self.EXIT_CODE}
            emit(self.out)
        print(f"bench.py: side leg {self.stage[0]} {msg}", file=sys.stderr, flush=True)
        os._exit(self.EXIT_CODE)


def rccl_record(torch, dist, group, rank: int, local: int, build: dict) -> dict:
    """What the process group saw after init_process_group: the backend, its
    world size, and per rank the HIP device it drives (ordinal, name, PCI bus
    and the library build it loaded), gathered over the host-side group."""
    me = {"rank": rank, "local_rank": local, "device": None, "name": None, "pci_bus_id": None,
          "so_sha256": build.get("so_sha256")}
    try:
        d = torch.cuda.current_device()
        pr = torch.cuda.get_device_properties(d)
        me.update(device=d, name=pr.name)
        bus = getattr(pr, "pci_bus_id", None)
        if bus is not None:
            me["pci_bus_id"] = f"{getattr(pr, 'pci_domain_id', 0):04x}:{bus:02x}:{getattr(pr, 'pci_device_id', 0):02x}"
    except Exception as e:   # noqa: BLE001 -- the record never costs the run
        me["error"] = f"{type(e).__name__}: {e}"
    ranks = [None] * dist.get_world_size()
    dist.all_gather_object(ranks, me, group=group)
    buses = [r.get("pci_bus_id") for r in ranks]
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "ranks": ranks,
            "distinct_devices": len(set(buses)) if all(buses) else None}


def watchdog_selftest(args) -> None:
    """CPU rehearsal of the N>1 watchdog (no GPU): every rank joins a gloo
    group, then gets stuck in a point-to-point exchange that never completes
    (each rank waits to receive from the next one; nobody sends) -- the shape of
    a hung replica exchange.  The watchdog must print rank 0's line with the
    stuck leg's error and end every rank with Watchdog.EXIT_CODE."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "selftest": "watchdog"} \
        if rank == 0 else None
    dog = Watchdog(args.replica_timeout, out)
    dog.start()
    dog.stage[0] = "replica_exchange"
    buf = torch.zeros(1)
    dist.recv(buf, src=(rank + 1) % world)     # never sent: stuck until the watchdog fires
    if dog.cancel() and out is not None:       # not reached
        emit(out)


_T0 = time.perf_counter()
_JSON_OUT = None


def claim_stdout() -> None:
    """Keep fd 1 for the one JSON line: a dup of it is kept for emit(), and
    fd 1 itself is pointed at stderr, so anything else a rank's libraries
    print there (gloo's "[Gloo] Rank k is connected to ..." when the side
    group forms, runtime notices) cannot interleave with the line a driver
    parses.  Called in every rank (and the single process), never in the
    spawning parent, whose fd 1 the ranks inherit."""
    global _JSON_OUT
    if _JSON_OUT is None:
        sys.stdout.flush()
        _JSON_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)


TAIL_KEYS = ("scaling_check", "verified", "verified_partitions", "build")
BUILD_TAIL = ("so_sha256", "device_code_sha256", "built_utc", "stamp_matches_so", "sources_match")


def proof_last(obj: dict) -> dict:
    """The line with the headline's proof as its LAST keys: whether every
    timed partition matched the oracle, and which library ran (ending with
    sources_match).  The driver's record keeps only the tail of stdout, so
    these are what it must still hold when the side legs have made the line
    long."""
    out = {k: v for k, v in obj.items() if k not in TAIL_KEYS}
    for k in TAIL_KEYS:
        if k in obj:
            v = obj[k]
            if k == "build" and isinstance(v, dict):
                v = {**{b: x for b, x in v.items() if b not in BUILD_TAIL}, **{b: v[b] for b in BUILD_TAIL if b in v}}
            out[k] = v
    return out


def emit(obj) -> None:
    """Write the JSON line to the real stdout (the proof of the headline last)."""
    if isinstance(obj, dict):
        obj = proof_last(obj)
    out = _JSON_OUT if _JSON_OUT is not None else sys.stdout
    out.write(json.dumps(obj) + "\n")
    out.flush()


def progress(msg: str) -> None:
    """One stderr line per finished leg (rank-tagged, seconds since start): a
    long run keeps showing that it is alive, and a stuck leg is named."""
    print(f"[bench rank {os.environ.get('RANK', '0')} +{time.perf_counter() - _T0:.1f}s] {msg}", file=sys.stderr,
          flush=True)


def spawn_ranks(n: int) -> int:
    """`python3 bench.py --gpus N` with N > 1 and no launcher (WORLD_SIZE
    unset): start the N rank processes here, one per GPU, the way torchrun
    would -- each child is this same command with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT in its environment.  The parent
    never touches the GPU (no torch import, no HIP call) and never execs: the
    children are subprocesses, their stdout is this process's stdout (rank 0
    prints the JSON line), and the parent exits with the worst child code.
    A child that fails ends the others (by their own PIDs), so a run that lost
    a rank is a failed run -- never a one-GPU line."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    def die_with_parent():
        # a rank must not outlive a parent that was killed outright (SIGKILL
        # at a driver's time limit): Linux sends it SIGTERM then
        try:
            import ctypes
            ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM)   # PR_SET_PDEATHSIG
        except Exception:   # noqa: BLE001 -- best effort
            pass
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), IPLS_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]], env=env,
                                      preexec_fn=die_with_parent))

    def stop_all(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    signal.signal(signal.SIGTERM, lambda *a: (stop_all(), sys.exit(143)))
    first_bad = None
    while any(p.poll() is None for p in procs):
        for r, p in enumerate(procs):
            if first_bad is None and p.poll() not in (None, 0):
                first_bad = r
                print(f"bench.py: rank {r} exited with code {p.returncode}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                stop_all()
        time.sleep(0.1)
    for p in procs:
        p.wait()
    rcs = [p.returncode for p in procs]
    if first_bad is not None:
        rc = rcs[first_bad]
        return rc if rc > 0 else 1           # killed by a signal: still a failure
    return max((c if c >= 0 else 1) for c in rcs)


def plumbing_selftest(args) -> None:
    """CPU rehearsal of the N>1 launch plumbing (no GPU, tests/test_bench_spawn.py):
    every rank joins a gloo group, records what the group saw, and rank 0 prints
    the line with that record (`rccl`, the same keys as a GPU run's).
    --selftest-fail-rank R makes rank R exit with code 7 right after joining,
    the shape of a rank that found no GPU."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if rank == args.selftest_fail_rank:
        os._exit(7)
    me = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "pid": os.getpid(),
          "spawned_by_bench": os.environ.get("IPLS_BENCH_SPAWNED") == "1"}
    ranks = [None] * dist.get_world_size()
    dist.all_gather_object(ranks, me)
    if rank == 0:
        line = {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "selftest": "plumbing",
                "rccl": {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "ranks": ranks}}
        if world > 1:
            line["scaling_check"] = scaling_check(world, line)
        emit(line)
    dist.barrier()
    dist.destroy_process_group()


def main():
    args = parse()
    launched = "WORLD_SIZE" in os.environ
    if args.gpus > 1 and not launched:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    claim_stdout()
    if args.watchdog_selftest:
        return watchdog_selftest(args)
    if args.plumbing_selftest:
        return plumbing_selftest(args)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend == "nccl" and torch.cuda.device_count() < world:
        # counted before any HIP call (device_count does not initialise the runtime on this image)
        sys.exit(f"bench.py: {world} ranks need {world} GPUs, {torch.cuda.device_count()} visible")
    if not torch.cuda.is_available():
        sys.exit("bench.py needs an MI355X (no HIP device visible)")
    if args.dist_backend == "gloo":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        side_group = dist.new_group(backend="gloo")   # host-side barriers of the side legs

    import ipls
    build = ipls.build_info()   # the code every number below was measured on
    rccl = rccl_record(torch, dist, side_group, rank, local, build) if world > 1 else None
    P, L, K = CONFIGS[args.config]
    if args.strong:
        if P % world:
            sys.exit(f"--strong: {P} partitions do not split over {world} ranks")
        P //= world
    p0 = rank * P                                  # this GPU's -pa segment (contiguous block)
    elem = L + 32                                  # 256-B pad between buckets
    arena = torch.empty(P * K * elem + 32, dtype=torch.float64, device="cuda")
    base = (int(arena.data_ptr()) + 255) // 256 * 256
    rows = []
    for q in range(P):
        row = []
        for k in range(K):
            b = ipls.DeviceBuffer(base + 8 * (q * K + k) * elem, L, big_endian=args.be)
            ipls.synth_fill(b, p0 + q, k, ipls.SEED)
            row.append(b)
        rows.append(row)
    torch.cuda.synchronize()

    agg = ipls.Aggregator(n_partitions=P, bucket_len=L, device=local)
    stream = torch.cuda.ExternalStream(agg.stream, device=torch.device("cuda", local))

    if args.be:
        # BE bytes in -> fold -> BE bytes out (the update_file image of each sum)
        out_arena = torch.empty(P * elem + 32, dtype=torch.float64, device="cuda")
        obase = (int(out_arena.data_ptr()) + 255) // 256 * 256
        dsts = [obase + 8 * q * elem for q in range(P)]

        def step():
            agg.reduce_batch_out(0, rows, dsts, start_mode=ipls.START_ZERO, big_endian_in=True,
                                 big_endian_out=True)
    else:
        def step():
            agg.reduce_batch(0, rows, start_mode=ipls.START_ZERO)

    for _ in range(args.warmup):
        step()
    agg.sync()

    # HIP events at the two ends of the K back-to-back launches on the handle's
    # stream: kern_ms = their span / K, the launch's average duration (plus the
    # ~1.6 us in-order boundary to the next launch).  An event packet around
    # every launch added ~4.6 us each to the timed region (tools/b_gap_probe.py,
    # profiles/r05/b_gap/), so none sits between the launches.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step()
    ev1.record(stream)
    agg.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps

    t = torch.tensor([dt], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt_max = float(t.item())

    progress(f"headline: {args.steps} steps in {dt:.3f} s")
    bytes_step = P * (K + 1) * L * 8
    total_bytes = bytes_step * args.steps * world
    value = total_bytes / dt_max / 1e9

    # every partition of the last timed launch against the oracle's checksum
    # of its fixed-order sum; at N > 1 each rank checks its own block and rank
    # 0 gathers the counts
    verified = None
    ver_parts = None
    if not args.no_verify:
        from oracle import oracle as O   # checker only: the oracle's checksum of the fixed-order sum
        ok = 0
        for q in range(P):
            if args.be:
                got = ipls.checksum_dev(ipls.DeviceBuffer(dsts[q], L, big_endian=True))
            else:
                got = agg.checksum(q)
            ok += int(got == O.c_synth_sum_checksum(L, p0 + q, K))
        counts = [(ok, P)]
        if world > 1:
            counts = [None] * world
            dist.all_gather_object(counts, (ok, P), group=side_group)
        good, total = sum(c[0] for c in counts), sum(c[1] for c in counts)
        verified = good == total
        ver_parts = f"{good}/{total}"

    # the rest of an aggregation round on the same handle (round_leg)
    round_info = None
    if not args.be:
        try:
            round_info = round_leg(ipls, torch, agg, rows, P, L, K, stream, kern_ms, build, args.config)
        except Exception as e:   # a side measurement never costs the headline line
            round_info = {"error": f"{type(e).__name__}: {e}"}

    out = None
    if rank == 0:
        achieved = bytes_step / (kern_ms / 1e3) / 1e9
        wkey = f"{args.config}{'-be' if args.be else ''}"
        traffic, traffic_prov = pmc_traffic(wkey, build)
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (splitmix64 counter buckets generated on device, SURVEY.md 8(d))",
            "config": {
                "workload": f"{args.config}: {P} partitions x {L} doubles x {K} peers per GPU"
                            + (f" ({P * world} in total, split over {world} GPUs)" if args.strong else "")
                            + (" (BE IPFS bytes in, BE sum bytes out: fused unpack/pack)" if args.be else ""),
                "partitions": P * world, "bucket_len": L, "peers": K,
                "parallelism": f"partition-sharded x{world} (no data-path collective)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "ipls::k_reduce",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_provenance": traffic_prov,
                "algorithmic_bytes_per_launch": bytes_step,
                "kernel_ms": round(kern_ms, 4),
            },
            "verified": verified,
            "verified_partitions": ver_parts,
            "build": build,
        }
        if rccl is not None:
            out["rccl"] = rccl
        if round_info:
            out["round"] = round_info
        def side(fn, *a, **kw):
            # a side measurement never costs the headline line: its failure is reported in place
            try:
                return fn(*a, **kw)
            except Exception as e:   # noqa: BLE001
                return {"error": f"{type(e).__name__}: {e}"}
            finally:
                progress(f"{fn.__name__} done")
        if world == 1 and not args.be:
            out["publish"] = side(publish_leg, ipls, torch, agg, stream, L, verify=not args.no_verify)
        if world == 1 and not args.be and not args.no_per_arrival:
            out["per_arrival"] = side(per_arrival_leg, ipls, torch, agg, rows, P, L, K, stream, not args.no_verify)
        if world == 1 and not args.no_e2e:
            out["host_inclusive"] = side(host_inclusive, ipls, ipls.Aggregator, L, K, args.e2e_reps, local)
        if world == 1 and not args.no_e2e and not args.no_middleware:
            out["middleware_socket"] = side(middleware_socket_leg, ipls, torch, local, verify=not args.no_verify)
        if world == 1 and not args.no_e2e:
            out["jni_heap"] = side(jni_heap_leg)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = side(cpu_baseline, L, K, args.cpu_passes)
        if world == 1 and not args.no_other_configs and args.config == "C" and not args.be:
            # the other single-GPU BASELINE configs, measured in the same run (never the value)
            del arena, rows
            torch.cuda.empty_cache()
            # B's launch is 0.19 ms: 50 launches (10 ms) per round average out the ramp of the first ones
            out["other_configs"] = {nm: side(config_leg, ipls, torch, nm, be, local, steps=st,
                                             verify=not args.no_verify, build=build)
                                    for nm, be, st in (("B", False, 50), ("D", True, 5), ("F", False, 5))}
            out["other_configs"]["A"] = side(config_a_leg, ipls)
            out["few_partitions"] = side(few_partitions_leg, ipls, torch, local, verify=not args.no_verify)
            if isinstance(out["other_configs"]["F"], dict) and not args.no_e2e:
                # config F is the end-to-end case: its buckets start as host IPFS bytes
                _, LF, KF = CONFIGS["F"]
                # the whole slice streamed from host bytes through a bounded pinned ring
                out["other_configs"]["F"]["host_inclusive"] = side(f_stream_leg, ipls, torch, local,
                                                                   verify=not args.no_verify)
    if world == 1 and args.be_schedule_ab and out is not None:
        if "arena" in locals():
            del arena, rows
        torch.cuda.empty_cache()
        out["be_schedule_ab"] = side(be_schedule_ab, ipls, torch, local, verify=not args.no_verify)
    dog = None
    if world > 1 and not args.be and not (args.no_replica_leg and args.no_ulp_leg and args.no_strong_leg
                                          and args.no_multi_leg
                                          and args.no_e2e):
        # the multi-rank side legs are extra measurements: a watchdog ends a
        # stuck exchange (or a teardown stuck behind a peer that failed in it)
        # -- the line is printed with the stuck leg's error and every rank exits
        # NON-zero, so a hang is never recorded as a clean run
        dog = Watchdog(args.replica_timeout, out)
        dog.start()
        stage = dog.stage
        if not args.no_replica_leg:
            progress(f"{stage[0]} done; starting replica_exchange" if stage[0] != "replica_exchange" else "starting replica_exchange")
            stage[0] = "replica_exchange"
            try:
                leg = replica_exchange(ipls, agg, rows, P, L, K, rank, world, local, args.replica_reps,
                                       not args.no_verify, args.dist_backend)
            except Exception as e:                   # reported, never fatal to the main line
                leg = {"error": f"{type(e).__name__}: {e}"}
            if out is not None:
                out["replica_exchange"] = leg
        if not args.no_ulp_leg:
            progress(f"{stage[0]} done; starting rccl_reduce_ulp" if stage[0] != "rccl_reduce_ulp" else "starting rccl_reduce_ulp")
            stage[0] = "rccl_reduce_ulp"
            try:
                ul = rccl_reduce_leg(ipls, torch, dist, rank, world, local, L, args.replica_reps,
                                     args.dist_backend)
            except Exception as e:                   # reported, never fatal to the main line
                ul = {"error": f"{type(e).__name__}: {e}"}
            if out is not None:
                out["rccl_reduce_ulp"] = ul
        if not args.no_strong_leg and not args.strong:
            progress(f"{stage[0]} done; starting strong_scaling_D" if stage[0] != "strong_scaling_D" else "starting strong_scaling_D")
            stage[0] = "strong_scaling_D"
            del arena, rows
            torch.cuda.empty_cache()
            try:
                sl = strong_leg(ipls, torch, dist, rank, world, local, verify=not args.no_verify)
            except Exception as e:                   # reported, never fatal to the main line
                sl = {"error": f"{type(e).__name__}: {e}"}
            if out is not None:
                out["strong_scaling_D"] = sl
        if not args.no_e2e:
            progress(f"{stage[0]} done; starting host_inclusive_multi" if stage[0] != "host_inclusive_multi" else "starting host_inclusive_multi")
            stage[0] = "host_inclusive_multi"
            if "arena" in locals():
                del arena, rows
            torch.cuda.empty_cache()
            _, LF, KF = CONFIGS["F"]
            try:
                el = e2e_multi(ipls, torch, dist, side_group, rank, world, local, LF, KF, args.e2e_reps,
                               not args.no_verify)
            except Exception as e:                   # reported, never fatal to the main line
                el = {"error": f"{type(e).__name__}: {e}"}
            if out is not None:
                out["host_inclusive_multi"] = el
        if not args.no_multi_leg:
            # rank 0 drives every GPU through ONE C-ABI handle (what a JVM would
            # do); the other ranks wait on a host-side (gloo) barrier, so no
            # spinning collective kernel shares their GPUs with the leg
            progress(f"{stage[0]} done; starting c_abi_multi_gpu" if stage[0] != "c_abi_multi_gpu" else "starting c_abi_multi_gpu")
            stage[0] = "c_abi_multi_gpu"
            if "arena" in locals():
                del arena, rows
            torch.cuda.empty_cache()
            devs = [0] * world if args.dist_backend == "gloo" else list(range(world))
            if rank == 0:
                P_m, L_m, K_m = CONFIGS["C"]
                try:
                    ml = c_abi_multi_gpu(ipls, torch, devs, P_m, L_m, K_m, verify=not args.no_verify)
                except Exception as e:               # reported, never fatal to the main line
                    ml = {"error": f"{type(e).__name__}: {e}"}
                out["c_abi_multi_gpu"] = ml
            dist.barrier(group=side_group)
    if world == 1 and args.multi_rehearsal and out is not None:
        if "arena" in locals():
            del arena, rows
        torch.cuda.empty_cache()
        P_m, L_m, K_m = CONFIGS["C"]
        out["c_abi_multi_gpu"] = side(c_abi_multi_gpu, ipls, torch, [local, local], P_m // 2, L_m, K_m,
                                      verify=not args.no_verify)
        out["c_abi_multi_gpu"]["note"] = "rehearsal: two shards of one GPU (same code path, no xGMI)"
    if dog is not None:
        dog.cancel()          # every leg finished: the line is printed once, here
                              # (if the dog fired first, it printed and exits)
    if out is not None and world > 1:
        out["scaling_check"] = scaling_check(world, out)
    if out is not None:
        emit(out)
    agg.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
