// ipls_agg.cpp -- the exported C-ABI (include/ipls_agg.h).
//
// A handle is the aggregator state of one IPLS peer (PeerData's accumulators,
// PeerData.java:137-189) over one or more GPUs.  The -pa partitions are cut
// into contiguous blocks, one per entry of cfg.devices (SURVEY.md §8(e):
// partition p on shard p / ceil(P/G)); each block lives in one engine
// (engine.hip: its device, HIP stream, accumulator arena and mutex).  Every
// entry point routes a partition to its owner shard, and a range of
// partitions to the shards it covers -- launches on several GPUs are queued
// back to back, so the shards run concurrently; calls that wait on host
// memory run one host thread per shard.
//
// The only data-path exchange is the one the reference has: several
// aggregators of one partition (IPLS.java:1402-1468).  A shard that is not
// the owner of p may fold buckets resident on its GPU into its partial sum of
// p (ipls_agg_reduce_partial); ipls_agg_combine_partials makes the owner's
// stream wait for those folds and then runs ONE fold kernel on the owner that
// reads every partial over xGMI (peer loads, peer access enabled at open) and
// adds them to REP[p] in ascending slot order -- the reference's
// Replicas_Gradients expression, bit for bit.
//
// With one device the front forwards every call unchanged to its engine.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ipls_agg.h"
#include "engine.hpp"
#include "java_hashmap.hpp"
#include "pubsub_host.hpp"

namespace {

// A replica slot's partial sum of one partition (on the slot's device).
struct Partial {
  double* d = nullptr;
  bool live = false;               // holds folds not yet combined (else logically +0.0)
  hipEvent_t ready = nullptr;      // recorded on the slot's stream after its last fold
  hipEvent_t consumed = nullptr;   // recorded on the owner's stream after the combine read it
  bool consumed_pending = false;
  double* stage = nullptr;         // owner-side copy, when the owner cannot load d over xGMI
};

// Persistent host workers, one per shard after the first: a call that waits
// on host memory (sync, get_partitions into host memory, collect_replicas,
// ingest ...) hands each shard's part to that shard's worker instead of
// spawning a thread per shard per call.  A worker only ever drives its own
// shard's GPU, so after its first call its device is current and every
// dev_use on it is free.
class ShardPool {
 public:
  explicit ShardPool(int n) : w_(n) {
    try {
      for (int s = 1; s < n; ++s) {
        w_[s] = std::make_unique<W>();
        w_[s]->th = std::thread([w = w_[s].get()] { run(w); });
      }
    } catch (...) {   // a later thread could not start: end the ones already running, then report
      stop_all();
      throw;
    }
  }
  ~ShardPool() { stop_all(); }
  void post(int s, std::function<void()> fn) {
    W* w = w_[s].get();
    {
      std::lock_guard<std::mutex> lk(w->m);
      w->q.push_back(std::move(fn));
    }
    w->cv.notify_one();
  }

 private:
  struct W {
    std::thread th;
    std::mutex m;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    bool stop = false;
  };
  void stop_all() noexcept {
    for (auto& w : w_)
      if (w && w->th.joinable()) {
        {
          std::lock_guard<std::mutex> lk(w->m);
          w->stop = true;
        }
        w->cv.notify_one();
        w->th.join();
      }
  }
  static void run(W* w) {
    for (;;) {
      std::function<void()> fn;
      {
        std::unique_lock<std::mutex> lk(w->m);
        w->cv.wait(lk, [w] { return w->stop || !w->q.empty(); });
        if (w->q.empty()) return;   // stop requested and drained
        fn = std::move(w->q.front());
        w->q.pop_front();
      }
      fn();
    }
  }
  std::vector<std::unique_ptr<W>> w_;
};

}  // namespace

struct ipls_agg {
  std::mutex mu;       // front bookkeeping only (tickets, partials); never held across a host wait
  mutable std::mutex err_mu;
  std::string err;
  int P = 0;
  int64_t chunk = 0, flat_total = 0;
  std::vector<int64_t> len, off;     // handle geometry (IPLS.java:1019-1028)
  std::vector<int32_t> devices;      // device of each shard
  std::vector<ipls_dev*> sh;         // one engine per shard (possibly owning no partition)
  std::vector<int> lo;               // shard s owns partitions [lo[s], lo[s+1])
  std::vector<int> owner;            // partition -> shard
  std::vector<std::vector<char>> peer;   // peer[a][b]: shard a's device reads shard b's memory
  bool force_staged = false;         // IPLS_PEER_STAGED=1: stage every cross-device read (test switch)
  std::vector<hipEvent_t> xev;       // per shard: cross-shard ordering point (used under gbuf_mu)
  // the handle's ONE Gradient_Buff lives on shard 0 (one Updater thread,
  // Updater.java:162): a request's load, its fold on the partition's shard and
  // the hand-back run as one sequence under gbuf_mu (the sequence may wait on
  // the host for a pinned zero-copy load; mu is never held across that)
  std::mutex gbuf_mu;
  std::vector<double*> gstage;       // per shard: Gradient_Buff copy when shard 0 is not peer-readable
  std::atomic<int> last_shard{0};
  std::atomic<int> last_staged{0};   // partials the last combine staged (ipls_launch_info.staged)
  std::unique_ptr<ShardPool> pool;   // S > 1 only
  // asynchronous folds across shards: per shard, (handle ticket, engine ticket) in issue order
  uint64_t ticket_next = 1;
  std::vector<std::deque<std::pair<uint64_t, uint64_t>>> tickets;
  std::vector<std::vector<Partial>> part;   // [slot][p]
  // PeerData.Other_Replica_Gradients' key set as the JDK HashMap holds it (one
  // map for the whole peer, PeerData.java:140): which (p, aggregator) keys are
  // stored, their Pair hashCodes, insertion order and the table capacity --
  // the order Collect_Replicas folds them in (java_hashmap.hpp).  The arrays
  // themselves live on the partitions' shards.
  std::mutex rep_mu;
  ipls::JavaHashOrder rep_order;

  int S() const { return (int)sh.size(); }
};

namespace {

thread_local std::string g_front_err;

int ferr(ipls_agg* H, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (H) {
    std::lock_guard<std::mutex> lk(H->err_mu);
    H->err = buf;
  }
  dev_set_thread_error(buf);
  return code;
}

// An engine call's failure becomes the handle's last error.  The engine left
// its message in this thread's slot (the engine's own copy may already hold
// another caller's failure on the same shard).
void set_err(ipls_agg* H, const std::string& m) {
  {
    std::lock_guard<std::mutex> lk(H->err_mu);
    H->err = m;
  }
  dev_set_thread_error(m.c_str());
}
template <class T>
T fwd(ipls_agg* H, int s, T rc) {
  (void)s;
  if (rc < 0) set_err(H, dev_last_error(nullptr));
  return rc;
}

// Every entry point leaves the calling thread's current HIP device as it
// found it: the engines switch devices internally (one per shard), and a
// caller that also drives the GPU (torch, another library) must not find its
// device changed behind its back.
struct KeepDevice {
  int d = -1;
  KeepDevice() {
    if (hipGetDevice(&d) != hipSuccess) {
      (void)hipGetLastError();
      d = -1;
    }
    dev_track(d);
  }
  ~KeepDevice() {
    if (d >= 0 && dev_tracked() != d && hipSetDevice(d) != hipSuccess) (void)hipGetLastError();
    dev_track(-1);   // outside a call the caller may switch devices on its own
  }
  KeepDevice(const KeepDevice&) = delete;
  KeepDevice& operator=(const KeepDevice&) = delete;
};

bool part_ok(const ipls_agg* H, int p) { return p >= 0 && p < H->P; }

int range_err(ipls_agg* H, int p) { return ferr(H, IPLS_E_RANGE, "partition %d out of range [0,%d)", p, H->P); }

// partition p -> (shard, engine-local index)
inline int route(ipls_agg* H, int p, int* local) {
  const int s = H->owner[p];
  *local = p - H->lo[s];
  H->last_shard.store(s, std::memory_order_relaxed);
  return s;
}

// Shards overlapping partitions [p0, p1).
std::vector<int> shards_of(const ipls_agg* H, int p0, int p1) {
  std::vector<int> out;
  if (p1 <= p0) return out;
  for (int s = H->owner[p0]; s <= H->owner[p1 - 1]; ++s)
    if (H->lo[s + 1] > H->lo[s]) out.push_back(s);
  return out;
}

std::vector<int> nonempty_shards(const ipls_agg* H) { return shards_of(H, 0, H->P); }

// Run fn(s) for each shard: the first in this thread, every other on its
// shard's persistent worker (calls that wait on host copies overlap across
// GPUs).  Returns the first negative code, with that shard's message.
template <class F>
int par_shards(ipls_agg* H, const std::vector<int>& ss, F fn) {
  if (ss.size() <= 1) {
    for (int s : ss)
      if (int rc = fn(s); rc < 0) return fwd(H, s, rc);
    return IPLS_OK;
  }
  std::vector<int> rc(ss.size(), 0);
  std::vector<std::string> msg(ss.size());   // a worker's message lives in the worker's thread slot
  std::mutex m;
  std::condition_variable cv;
  size_t left = ss.size() - 1;
  // one shard's part; never throws (the caller waits for every part, and the
  // parts reference this frame)
  auto part = [&](size_t i) noexcept {
    try {
      rc[i] = fn(ss[i]);
      if (rc[i] < 0) msg[i] = dev_last_error(nullptr);
    } catch (...) {
      rc[i] = IPLS_E_NOMEM;
    }
  };
  for (size_t i = 1; i < ss.size(); ++i) {
    auto task = [&, i]() noexcept {
      part(i);
      std::lock_guard<std::mutex> lk(m);
      if (--left == 0) cv.notify_one();
    };
    try {
      H->pool->post(ss[i], task);
    } catch (...) {   // could not queue it (allocation): run that shard's part here
      task();
    }
  }
  part(0);
  {
    std::unique_lock<std::mutex> lk(m);
    cv.wait(lk, [&] { return left == 0; });
  }
  for (size_t i = 0; i < ss.size(); ++i)
    if (rc[i] < 0) {
      set_err(H, msg[i]);
      return rc[i];
    }
  return IPLS_OK;
}

// A device operand that shard s's GPU reads or writes (an output of a call
// over several shards, a text buffer): it must be s's own memory or that of a
// device s has peer access to -- anything else would fault the GPU instead of
// failing the call.  Host memory and unknown pointers are left to the engine.
int check_reach(ipls_agg* H, int s, const void* ptr, const char* what) {
  if (!ptr) return IPLS_OK;
  hipPointerAttribute_t at{};
  const hipError_t e = hipPointerGetAttributes(&at, ptr);
  (void)hipGetLastError();
  if (e != hipSuccess || at.type != hipMemoryTypeDevice || at.device == H->devices[s]) return IPLS_OK;
  for (int t = 0; t < H->S(); ++t)
    if (H->devices[t] == at.device && H->peer[s][t]) return IPLS_OK;
  return ferr(H, IPLS_E_DEVICE, "device %d cannot reach the %s on device %d (no peer access)", H->devices[s], what,
              at.device);
}

// Order shard b's stream after the work queued so far on shard a's stream.
int order_after(ipls_agg* H, int a, int b) {
  if (a == b) return IPLS_OK;
  if (dev_use(H->devices[a]) != hipSuccess || hipEventRecord(H->xev[a], (hipStream_t)dev_stream(H->sh[a])) != hipSuccess ||
      dev_use(H->devices[b]) != hipSuccess ||
      hipStreamWaitEvent((hipStream_t)dev_stream(H->sh[b]), H->xev[a], 0) != hipSuccess) {
    (void)hipGetLastError();
    return ferr(H, IPLS_E_DEVICE, "cross-shard stream ordering failed");
  }
  return IPLS_OK;
}

void destroy(ipls_agg* H) {
  H->pool.reset();   // join the workers first: none may be inside an engine call below
  for (auto& row : H->part)
    for (Partial& q : row) {
      if (q.d) hipFree(q.d);
      if (q.stage) hipFree(q.stage);
      if (q.ready) hipEventDestroy(q.ready);
      if (q.consumed) hipEventDestroy(q.consumed);
    }
  for (double* g : H->gstage)
    if (g) hipFree(g);
  for (size_t s = 0; s < H->sh.size(); ++s) {
    if (H->sh[s]) dev_close(H->sh[s]);
    if (s < H->xev.size() && H->xev[s]) hipEventDestroy(H->xev[s]);
  }
  delete H;
}

}  // namespace

extern "C" {

int ipls_agg_abi_version(void) { return IPLS_AGG_ABI_VERSION; }

const char* ipls_agg_last_error(const ipls_agg* h) {
  if (!h) return dev_last_error(nullptr);
  // a snapshot per calling thread: another thread's failure on the same handle
  // may replace h->err while this caller still reads the returned string
  thread_local std::string snap;
  {
    std::lock_guard<std::mutex> lk(h->err_mu);
    snap = h->err;
  }
  return snap.c_str();
}

int ipls_shard_plan(int32_t n_partitions, int32_t n_shards, int32_t* owner) {
  if (n_partitions <= 0 || n_shards <= 0 || !owner) return ferr(nullptr, IPLS_E_INVAL, "bad shard plan arguments");
  const int per = (n_partitions + n_shards - 1) / n_shards;   // ceil(P / G)
  for (int p = 0; p < n_partitions; ++p) owner[p] = p / per;
  return IPLS_OK;
}

int ipls_agg_open(const ipls_agg_cfg* cfg, ipls_agg** out) {
  KeepDevice keep_device;
  if (!cfg || !out) return ferr(nullptr, IPLS_E_INVAL, "null cfg/out");
  *out = nullptr;
  if (cfg->n_partitions <= 0) return ferr(nullptr, IPLS_E_INVAL, "n_partitions must be > 0 (-pa)");
  if (cfg->model_size < 0) return ferr(nullptr, IPLS_E_INVAL, "model_size < 0");
  if (cfg->flags != 0 || cfg->reserved != 0) return ferr(nullptr, IPLS_E_INVAL, "cfg.flags / cfg.reserved must be 0");
  if (cfg->n_devices < 0 || (cfg->n_devices > 0 && !cfg->devices))
    return ferr(nullptr, IPLS_E_INVAL, "bad device list");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    (void)hipGetLastError();
    return ferr(nullptr, IPLS_E_NODEV, "no HIP device available");
  }
  std::vector<int32_t> devs;
  if (cfg->n_devices > 0 && cfg->devices) devs.assign(cfg->devices, cfg->devices + cfg->n_devices);
  else devs.push_back(cfg->device);
  for (int32_t d : devs)
    if (d < 0 || d >= ndev) return ferr(nullptr, IPLS_E_NODEV, "device %d not in [0,%d)", d, ndev);

  ipls_agg* H = new (std::nothrow) ipls_agg();
  if (!H) return ferr(nullptr, IPLS_E_NOMEM, "host allocation failed");
  std::string why;
  if (int rc = dev_geometry(cfg, H->len, H->off, H->chunk, why)) {
    delete H;
    return ferr(nullptr, rc, "%s", why.c_str());
  }
  H->P = cfg->n_partitions;
  for (int p = 0; p < H->P; ++p) H->flat_total = std::max(H->flat_total, H->off[p] + H->len[p] - 1);
  const int S = (int)devs.size();
  H->devices = devs;
  H->owner.resize(H->P);
  ipls_shard_plan(H->P, S, H->owner.data());
  H->lo.assign(S + 1, H->P);
  for (int s = S - 1; s >= 0; --s)
    for (int p = 0; p < H->P; ++p)
      if (H->owner[p] == s) { H->lo[s] = p; break; }
  for (int s = S - 1; s >= 0; --s) H->lo[s] = std::min(H->lo[s], H->lo[s + 1]);   // empty shards
  H->sh.assign(S, nullptr);
  H->xev.assign(S, nullptr);
  H->tickets.resize(S);
  H->part.resize(S);
  for (int s = 0; s < S; ++s) {
    if (int rc = dev_open(cfg, devs[s], H->lo[s], H->lo[s + 1], &H->sh[s])) {
      const std::string m = dev_last_error(nullptr);
      H->sh[s] = nullptr;
      destroy(H);
      return ferr(nullptr, rc, "shard %d (device %d): %s", s, devs[s], m.c_str());
    }
    if (dev_use(devs[s]) != hipSuccess || hipEventCreateWithFlags(&H->xev[s], hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      destroy(H);
      return ferr(nullptr, IPLS_E_DEVICE, "event creation on device %d failed", devs[s]);
    }
  }
  // xGMI peer access between every pair of distinct devices (the combine's
  // fold kernel reads the other GPUs' partials directly)
  H->peer.assign(S, std::vector<char>(S, 0));
  for (int a = 0; a < S; ++a)
    for (int b = 0; b < S; ++b) {
      if (devs[a] == devs[b]) { H->peer[a][b] = 1; continue; }
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, devs[a], devs[b]) != hipSuccess) can = 0;
      if (can) {
        dev_use(devs[a]);
        const hipError_t e = hipDeviceEnablePeerAccess(devs[b], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) can = 0;
      }
      (void)hipGetLastError();
      H->peer[a][b] = (char)can;
    }
  const char* st = std::getenv("IPLS_PEER_STAGED");
  H->force_staged = st && st[0] == '1';
  H->gstage.assign(S, nullptr);
  if (S > 1) {
    try {
      H->pool = std::make_unique<ShardPool>(S);
    } catch (const std::exception& e) {   // thread creation failed: no exception crosses the C-ABI
      destroy(H);
      return ferr(nullptr, IPLS_E_NOMEM, "shard worker threads: %s", e.what());
    }
  }
  *out = H;
  return IPLS_OK;
}

int ipls_agg_close(ipls_agg* h) {
  KeepDevice keep_device;
  if (!h) return IPLS_OK;
  destroy(h);
  return IPLS_OK;
}

int ipls_agg_partition_len(const ipls_agg* h, int p, int64_t* L) {
  ipls_agg* H = const_cast<ipls_agg*>(h);
  if (!H || !L) return ferr(H, IPLS_E_INVAL, "null argument");
  if (!part_ok(H, p)) return range_err(H, p);
  *L = H->len[p];
  return IPLS_OK;
}

int ipls_agg_partition_offset(const ipls_agg* h, int p, int64_t* off) {
  ipls_agg* H = const_cast<ipls_agg*>(h);
  if (!H || !off) return ferr(H, IPLS_E_INVAL, "null argument");
  if (!part_ok(H, p)) return range_err(H, p);
  *off = H->off[p];
  return IPLS_OK;
}

int ipls_agg_flat_size(const ipls_agg* h, int64_t* n) {
  ipls_agg* H = const_cast<ipls_agg*>(h);
  if (!H || !n) return ferr(H, IPLS_E_INVAL, "null argument");
  *n = H->flat_total;
  return IPLS_OK;
}

int ipls_agg_partition_device(ipls_agg* H, int p, int32_t* device, void** stream) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  const int s = H->owner[p];
  if (device) *device = H->devices[s];
  if (stream) *stream = dev_stream(H->sh[s]);
  return IPLS_OK;
}

void* ipls_agg_stream(ipls_agg* H) { return H ? dev_stream(H->sh[0]) : nullptr; }

int ipls_agg_sync(ipls_agg* H) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  // start every shard's queued folds first, then wait on the streams one by
  // one: the waits overlap the GPUs' work anyway (the total is the slowest
  // shard), and no host thread needs to wake per shard
  for (int s = 0; s < H->S(); ++s)
    if (int rc = fwd(H, s, dev_flush(H->sh[s]))) return rc;
  for (int s = 0; s < H->S(); ++s)
    if (int rc = fwd(H, s, dev_sync(H->sh[s]))) return rc;
  return IPLS_OK;
}

int ipls_agg_flush(ipls_agg* H) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  for (int s = 0; s < H->S(); ++s)
    if (int rc = fwd(H, s, dev_flush(H->sh[s]))) return rc;
  return IPLS_OK;
}

int ipls_agg_set_coalesce(ipls_agg* H, int max_group) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  for (int s = 0; s < H->S(); ++s)
    if (int rc = fwd(H, s, dev_set_coalesce(H->sh[s], max_group))) return rc;
  return IPLS_OK;
}

int ipls_agg_last_launch(ipls_agg* H, ipls_launch_info* out) {
  KeepDevice keep_device;
  if (!H || !out) return ferr(H, IPLS_E_INVAL, "null argument");
  const int rc = dev_last_launch(H->sh[H->last_shard.load(std::memory_order_relaxed)], out);
  out->staged = H->last_staged.load(std::memory_order_relaxed);
  return rc;
}

int ipls_agg_load_model(ipls_agg* H, const void* src, int64_t n, int src_kind) {
  KeepDevice keep_device;
  if (!H || !src) return ferr(H, IPLS_E_INVAL, "null argument");
  if (H->S() == 1) return fwd(H, 0, dev_load_model(H->sh[0], src, n, src_kind));
  if (n < H->flat_total)
    return ferr(H, IPLS_E_RANGE, "model of %lld values < model size %lld", (long long)n, (long long)H->flat_total);
  return par_shards(H, nonempty_shards(H), [&](int s) { return dev_load_model(H->sh[s], src, n, src_kind); });
}

int ipls_agg_split(ipls_agg* H, const void* flat, int64_t n, int src_kind, int p, void* dst, int dst_kind) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_split(H->sh[s], flat, n, src_kind, q, dst, dst_kind));
}

int ipls_agg_update_gradient(ipls_agg* H, const void* flat, int64_t n, int src_kind, const int32_t* owned,
                             int n_owned) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (H->S() == 1) return fwd(H, 0, dev_update_gradient(H->sh[0], flat, n, src_kind, owned, n_owned));
  if (!flat) return IPLS_OK;   // Gradients == null (IPLS.java:1708-1713)
  if (n_owned < 0 || (n_owned > 0 && !owned)) return ferr(H, IPLS_E_INVAL, "bad owned list");
  // OrganizeGradients splits EVERY partition before anything is accumulated
  // (IPLS.java:1709): a length error leaves all shards untouched
  for (int p = 0; p < H->P; ++p) {
    const int64_t nc = std::max<int64_t>(0, std::min(H->off[p] + H->chunk, n) - H->off[p]);
    if (nc > H->len[p] - 1)
      return ferr(H, IPLS_E_RANGE, "gradient vector of %lld values overruns partition %d "
                  "(ArrayIndexOutOfBounds, IPLS.java:1030)", (long long)n, p);
  }
  for (int i = 0; i < n_owned; ++i)
    if (!part_ok(H, owned[i])) return range_err(H, owned[i]);
  std::vector<std::vector<int32_t>> per(H->S());
  for (int i = 0; i < n_owned; ++i) per[H->owner[owned[i]]].push_back(owned[i] - H->lo[H->owner[owned[i]]]);
  std::vector<int> ss;
  for (int s = 0; s < H->S(); ++s)
    if (!per[s].empty()) ss.push_back(s);
  return par_shards(H, ss, [&](int s) {
    return dev_update_gradient(H->sh[s], flat, n, src_kind, per[s].data(), (int)per[s].size());
  });
}

int ipls_agg_accumulate(ipls_agg* H, int p, int target, const void* src, int64_t n, int src_kind) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_accumulate(H->sh[s], q, target, src, n, src_kind));
}

int ipls_agg_accumulate_async(ipls_agg* H, int p, int target, const void* src, int64_t n, int src_kind,
                              uint64_t* ticket) {
  KeepDevice keep_device;
  if (!H || !ticket) return ferr(H, IPLS_E_INVAL, "null argument");
  if (H->S() == 1) return fwd(H, 0, dev_accumulate_async(H->sh[0], p, target, src, n, src_kind, ticket));
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  uint64_t lt = 0;
  if (int rc = fwd(H, s, dev_accumulate_async(H->sh[s], q, target, src, n, src_kind, &lt))) return rc;
  std::vector<std::pair<int, uint64_t>> drain;
  {
    std::lock_guard<std::mutex> lk(H->mu);
    *ticket = H->ticket_next++;
    auto& dq = H->tickets[s];
    dq.emplace_back(*ticket, lt);
    if (dq.size() > 65536) {   // bound the bookkeeping: retire the oldest half
      drain.emplace_back(s, dq[dq.size() / 2].second);
      dq.erase(dq.begin(), dq.begin() + dq.size() / 2 + 1);
    }
  }
  for (auto& d : drain)
    if (int rc = fwd(H, d.first, dev_wait(H->sh[d.first], d.second))) return rc;
  return IPLS_OK;
}

int ipls_agg_accumulate_range(ipls_agg* H, int p, int target, const void* src, int64_t offset, int64_t n,
                              int src_kind, uint64_t* ticket) {
  KeepDevice keep_device;
  if (!H || !ticket) return ferr(H, IPLS_E_INVAL, "null argument");
  if (H->S() == 1) return fwd(H, 0, dev_accumulate_range(H->sh[0], p, target, src, offset, n, src_kind, ticket));
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  uint64_t lt = 0;
  if (int rc = fwd(H, s, dev_accumulate_range(H->sh[s], q, target, src, offset, n, src_kind, &lt))) return rc;
  std::vector<std::pair<int, uint64_t>> drain;
  {
    std::lock_guard<std::mutex> lk(H->mu);
    *ticket = H->ticket_next++;
    auto& dq = H->tickets[s];
    dq.emplace_back(*ticket, lt);
    if (dq.size() > 65536) {   // bound the bookkeeping: retire the oldest half
      drain.emplace_back(s, dq[dq.size() / 2].second);
      dq.erase(dq.begin(), dq.begin() + dq.size() / 2 + 1);
    }
  }
  for (auto& d : drain)
    if (int rc = fwd(H, d.first, dev_wait(H->sh[d.first], d.second))) return rc;
  return IPLS_OK;
}

// The chunked calls run entirely on p's shard, on the calling thread (the
// source / sink are the caller's code and must run there).
int ipls_agg_accumulate_chunked(ipls_agg* H, int p, int target, int64_t n, int src_kind, int64_t chunk,
                                ipls_chunk_source source, void* ctx) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_accumulate_chunked(H->sh[s], q, target, n, src_kind, chunk, source, ctx));
}

int ipls_agg_finalize_chunked(ipls_agg* H, int p, int sum_kind, int64_t chunk, ipls_chunk_sink sink, void* ctx) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_finalize_chunked(H->sh[s], q, sum_kind, chunk, sink, ctx));
}

int ipls_agg_read_range(ipls_agg* H, int p, int target, void* dst, int64_t offset, int64_t n, int dst_kind,
                        uint64_t* ticket) {
  KeepDevice keep_device;
  if (!H || !ticket) return ferr(H, IPLS_E_INVAL, "null argument");
  if (H->S() == 1) return fwd(H, 0, dev_read_range(H->sh[0], p, target, dst, offset, n, dst_kind, ticket));
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  uint64_t lt = 0;
  if (int rc = fwd(H, s, dev_read_range(H->sh[s], q, target, dst, offset, n, dst_kind, &lt))) return rc;
  std::vector<std::pair<int, uint64_t>> drain;
  {
    std::lock_guard<std::mutex> lk(H->mu);
    *ticket = H->ticket_next++;
    auto& dq = H->tickets[s];
    dq.emplace_back(*ticket, lt);
    if (dq.size() > 65536) {   // bound the bookkeeping: retire the oldest half
      drain.emplace_back(s, dq[dq.size() / 2].second);
      dq.erase(dq.begin(), dq.begin() + dq.size() / 2 + 1);
    }
  }
  for (auto& d : drain)
    if (int rc = fwd(H, d.first, dev_wait(H->sh[d.first], d.second))) return rc;
  return IPLS_OK;
}

int ipls_agg_wait(ipls_agg* H, uint64_t ticket) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (H->S() == 1) return fwd(H, 0, dev_wait(H->sh[0], ticket));
  std::vector<std::pair<int, uint64_t>> w;   // (shard, newest engine ticket issued at or before `ticket`)
  {
    std::lock_guard<std::mutex> lk(H->mu);
    if (ticket >= H->ticket_next) return ferr(H, IPLS_E_INVAL, "ticket %llu was never issued", (unsigned long long)ticket);
    for (int s = 0; s < H->S(); ++s) {
      const auto& dq = H->tickets[s];
      auto it = std::upper_bound(dq.begin(), dq.end(), std::make_pair(ticket, UINT64_MAX));
      if (it != dq.begin()) w.emplace_back(s, std::prev(it)->second);
    }
  }
  for (auto& x : w)
    if (int rc = fwd(H, x.first, dev_wait(H->sh[x.first], x.second))) return rc;
  std::lock_guard<std::mutex> lk(H->mu);
  for (auto& dq : H->tickets)
    while (!dq.empty() && dq.front().first <= ticket) dq.pop_front();
  return IPLS_OK;
}

int ipls_agg_update_indirect(ipls_agg* H, int p, int target, const void* bytes, int64_t n_bytes) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  if (H->S() == 1) return fwd(H, 0, dev_update_indirect(H->sh[0], q, target, bytes, n_bytes));
  // The handle has ONE Gradient_Buff (one Updater thread, Updater.java:162),
  // on shard 0: load it there, then fold it into p's owner (over xGMI, or
  // from a staged copy when the owner cannot read shard 0's memory).  The
  // whole sequence is one critical section for every shard, shard 0
  // included: another request's load must not overwrite the buffer between
  // this load and this fold's reads.
  std::lock_guard<std::mutex> gk(H->gbuf_mu);
  if (s == 0) return fwd(H, 0, dev_update_indirect(H->sh[0], q, target, bytes, n_bytes));
  const void* g = nullptr;
  int64_t glen = 0;
  if (int rc = fwd(H, 0, dev_gbuf_load(H->sh[0], bytes, n_bytes, &g, &glen))) return rc;
  if (int rc = order_after(H, 0, s)) return rc;
  if (!H->peer[s][0] || H->force_staged) {
    hipStream_t st = (hipStream_t)dev_stream(H->sh[s]);
    if (dev_use(H->devices[s]) != hipSuccess ||
        (!H->gstage[s] && hipMalloc(&H->gstage[s], (size_t)std::max<int64_t>(glen, 1) * 8) != hipSuccess)) {
      (void)hipGetLastError();
      return ferr(H, IPLS_E_NOMEM, "Gradient_Buff copy on device %d", H->devices[s]);
    }
    if (hipMemcpyPeerAsync(H->gstage[s], H->devices[s], g, H->devices[0], (size_t)glen * 8, st) != hipSuccess) {
      (void)hipGetLastError();
      return ferr(H, IPLS_E_DEVICE, "Gradient_Buff copy from device %d to %d failed", H->devices[0], H->devices[s]);
    }
    g = H->gstage[s];
  }
  const int rc = fwd(H, s, dev_accumulate(H->sh[s], q, target, g, glen, IPLS_DEV_F64));
  if (int r2 = order_after(H, s, 0)) return r2;   // the next load waits for this fold's reads
  return rc;
}

int ipls_java_pair_hash(int32_t p, const uint8_t* id, int64_t len, int32_t* hash) {
  if (!hash || len < 0 || (len > 0 && !id)) return ferr(nullptr, IPLS_E_INVAL, "bad peer-ID bytes");
  int32_t sh;
  if (!ipls::java_string_hash(id, len, &sh)) return ferr(nullptr, IPLS_E_FORMAT, "peer ID is not valid UTF-8");
  *hash = ipls::java_pair_hash_of(p, sh);
  return IPLS_OK;
}

int ipls_agg_other_replica_keyed(ipls_agg* H, int p, int32_t aggregator, int32_t key_hash, const void* src,
                                 int64_t n, int src_kind) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  std::lock_guard<std::mutex> lk(H->rep_mu);
  const ipls::JavaHashOrder::Key key{p, aggregator};
  int32_t h0 = 0;
  const bool had = H->rep_order.hash_of(key, &h0);
  if (had && h0 != key_hash)
    return ferr(H, IPLS_E_INVAL, "key hash %d of (%d, %d) differs from the one it was stored with (%d)", key_hash, p,
                aggregator, h0);
  if (int rc = fwd(H, s, dev_other_replica(H->sh[s], q, aggregator, src, n, src_kind))) return rc;
  if (!had) H->rep_order.put_new(key, key_hash);   // Other_Replica_Gradients.put (Download_Scheduler.java:266)
  return IPLS_OK;
}

int ipls_agg_other_replica(ipls_agg* H, int p, int32_t aggregator, const void* src, int64_t n, int src_kind) {
  // the aggregator's ID is taken to be Integer.toString(aggregator)
  return ipls_agg_other_replica_keyed(H, p, aggregator, ipls::java_pair_hash_of(p, ipls::java_index_id_hash(aggregator)),
                                      src, n, src_kind);
}

int ipls_agg_other_replica_drop(ipls_agg* H, int p, int32_t aggregator) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  std::lock_guard<std::mutex> lk(H->rep_mu);
  const int rc = fwd(H, s, dev_other_replica_drop(H->sh[s], q, aggregator));
  if (rc > 0) H->rep_order.remove({p, aggregator});
  return rc;
}

int ipls_agg_collect_replicas(ipls_agg* H, int32_t* participants) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  std::lock_guard<std::mutex> lk(H->rep_mu);
  // new ArrayList<>(Other_Replica_Gradients.keySet()) (IPLS.java:1218), cut
  // per shard as engine-local (p, aggregator) pairs in that order (only the
  // order within a partition changes a result; partitions live on one shard)
  std::vector<std::vector<int32_t>> per(H->S());
  for (const auto& k : H->rep_order.order()) {
    const int s = H->owner[k.first];
    per[s].push_back(k.first - H->lo[s]);
    per[s].push_back(k.second);
  }
  if (H->S() == 1) {
    const int rc = fwd(H, 0, dev_collect_replicas(H->sh[0], participants, per[0].data(), (int)per[0].size() / 2));
    if (rc >= 0) H->rep_order.clear();   // Other_Replica_Gradients = new HashMap<>() (:1238)
    return rc;
  }
  const std::vector<int> ss = nonempty_shards(H);
  for (int s : ss)   // the length rule over every shard before anything is folded
    if (int rc = fwd(H, s, dev_other_check(H->sh[s]))) return rc;
  std::vector<std::vector<int32_t>> cnt(H->S());
  std::vector<int> folded(H->S(), -1);
  const int rc = par_shards(H, ss, [&](int s) {
    cnt[s].assign(H->lo[s + 1] - H->lo[s], 0);
    const int r = dev_collect_replicas(H->sh[s], participants ? cnt[s].data() : nullptr, per[s].data(),
                                       (int)per[s].size() / 2);
    if (r >= 0) folded[s] = r;
    return r;
  });
  if (rc < 0) {   // the shards that did collect cleared their stores: so does the model, for their keys
    for (const auto& k : H->rep_order.order())
      if (folded[H->owner[k.first]] >= 0) H->rep_order.remove(k);
    return rc;
  }
  H->rep_order.clear();
  int total = 0;
  for (int s : ss) {
    total += folded[s];
    if (participants) std::copy(cnt[s].begin(), cnt[s].end(), participants + H->lo[s]);
  }
  return total;
}

int ipls_agg_replica_order(ipls_agg* H, int32_t* pairs, int max_pairs, int32_t* capacity) {
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (max_pairs < 0 || (max_pairs > 0 && !pairs)) return ferr(H, IPLS_E_INVAL, "bad pairs buffer");
  std::lock_guard<std::mutex> lk(H->rep_mu);
  const auto ord = H->rep_order.order();
  for (size_t i = 0; i < ord.size() && (int)i < max_pairs; ++i) {
    pairs[2 * i] = ord[i].first;
    pairs[2 * i + 1] = ord[i].second;
  }
  if (capacity) *capacity = (int32_t)H->rep_order.capacity();
  return (int)ord.size();
}

int ipls_agg_reduce_batch(ipls_agg* H, int p_first, int n_parts, const void* const* bufs, int k, int src_kind,
                          int start_mode, int target) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (H->S() == 1) return fwd(H, 0, dev_reduce_batch(H->sh[0], p_first, n_parts, bufs, k, src_kind, start_mode, target));
  if (n_parts <= 0 || p_first < 0 || p_first + n_parts > H->P)
    return ferr(H, IPLS_E_RANGE, "partitions [%d,%d) out of range [0,%d)", p_first, p_first + n_parts, H->P);
  if (k < 0 || (k > 0 && !bufs)) return ferr(H, IPLS_E_INVAL, "bad bucket list");
  for (int s : shards_of(H, p_first, p_first + n_parts)) {   // launches only: GPUs run concurrently
    const int q0 = std::max(p_first, H->lo[s]), q1 = std::min(p_first + n_parts, H->lo[s + 1]);
    H->last_shard = s;
    if (int rc = fwd(H, s, dev_reduce_batch(H->sh[s], q0 - H->lo[s], q1 - q0, bufs + (size_t)(q0 - p_first) * k, k,
                                            src_kind, start_mode, target)))
      return rc;
  }
  return IPLS_OK;
}

int ipls_agg_reduce_batch_out(ipls_agg* H, int p_first, int n_parts, const void* const* bufs, int k, int src_kind,
                              int start_mode, void* const* dst, int dst_kind) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (H->S() == 1)
    return fwd(H, 0, dev_reduce_batch_out(H->sh[0], p_first, n_parts, bufs, k, src_kind, start_mode, dst, dst_kind));
  if (n_parts <= 0 || p_first < 0 || p_first + n_parts > H->P)
    return ferr(H, IPLS_E_RANGE, "partitions [%d,%d) out of range [0,%d)", p_first, p_first + n_parts, H->P);
  if (!dst || k < 0 || (k > 0 && !bufs)) return ferr(H, IPLS_E_INVAL, "bad bucket/destination list");
  const std::vector<int> ss = shards_of(H, p_first, p_first + n_parts);
  if (dst_kind == IPLS_DEV_F64 || dst_kind == IPLS_DEV_BE)
    for (int s : ss)   // every destination is written by its partition's GPU: checked before any launch
      for (int p = std::max(p_first, H->lo[s]); p < std::min(p_first + n_parts, H->lo[s + 1]); ++p)
        if (int rc = check_reach(H, s, dst[p - p_first], "destination")) return rc;
  for (int s : ss) {
    const int q0 = std::max(p_first, H->lo[s]), q1 = std::min(p_first + n_parts, H->lo[s + 1]);
    H->last_shard = s;
    if (int rc = fwd(H, s, dev_reduce_batch_out(H->sh[s], q0 - H->lo[s], q1 - q0, bufs + (size_t)(q0 - p_first) * k,
                                                k, src_kind, start_mode, dst + (q0 - p_first), dst_kind)))
      return rc;
  }
  return IPLS_OK;
}

int ipls_agg_aggregate_round(ipls_agg* H, int p_first, int n_parts, const void* const* bufs, int k, int src_kind,
                             void* avg_out, int avg_kind) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (H->S() == 1)
    return fwd(H, 0, dev_aggregate_round(H->sh[0], p_first, n_parts, bufs, k, src_kind, avg_out, avg_kind));
  if (n_parts <= 0 || p_first < 0 || p_first + n_parts > H->P)
    return ferr(H, IPLS_E_RANGE, "partitions [%d,%d) out of range [0,%d)", p_first, p_first + n_parts, H->P);
  if (k < 0 || (k > 0 && !bufs)) return ferr(H, IPLS_E_INVAL, "bad bucket list");
  const std::vector<int> ss = shards_of(H, p_first, p_first + n_parts);
  auto one = [&](int s) {
    const int q0 = std::max(p_first, H->lo[s]), q1 = std::min(p_first + n_parts, H->lo[s + 1]);
    // the averages of partition q land at flat offset off[q] - off[p_first]
    void* a = avg_out ? (void*)((char*)avg_out + 8 * (H->off[q0] - H->off[p_first])) : nullptr;
    return dev_aggregate_round(H->sh[s], q0 - H->lo[s], q1 - q0, bufs + (size_t)(q0 - p_first) * k, k, src_kind, a,
                               avg_kind);
  };
  if (avg_out && avg_kind == IPLS_DEV_F64)
    for (int s : ss)   // each shard writes its partitions' averages into avg_out
      if (int rc = check_reach(H, s, avg_out, "averages buffer")) return rc;
  H->last_shard = ss.back();
  if (avg_out && avg_kind == IPLS_HOST_F64) return par_shards(H, ss, one);   // each shard copies its averages back
  for (int s : ss)
    if (int rc = fwd(H, s, one(s))) return rc;
  return IPLS_OK;
}

int ipls_agg_ingest_pubsub(ipls_agg* H, int target, const uint8_t* const* msgs, const int64_t* lens, int n_msgs,
                           int layers, const int32_t* parts, int32_t* status) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (H->S() == 1) return fwd(H, 0, dev_ingest_pubsub(H->sh[0], target, msgs, lens, n_msgs, layers, parts, status));
  if (n_msgs < 0 || (n_msgs > 0 && (!msgs || !lens))) return ferr(H, IPLS_E_INVAL, "bad message list");
  if (layers < 1 || layers > 2) return ferr(H, IPLS_E_INVAL, "layers must be 1 or 2");
  if (n_msgs == 0) return 0;
  // route each text to its partition's shard: the frame's partition field (or
  // the caller's), read from the text's ends on the host (pubsub_host.cpp);
  // a text with no valid partition still goes through a shard's decode, so
  // it reports FORMAT before RANGE, as Java throws while decoding first
  std::vector<std::vector<int>> idx(H->S());
  std::vector<int32_t> st(n_msgs, 0), local(n_msgs, -1);
  for (int i = 0; i < n_msgs; ++i) {
    int p = parts ? parts[i] : -1;
    if (!parts) {
      const ipls::pubsub::Pre pre = ipls::pubsub::precheck(msgs[i], lens[i], layers);
      if (pre.status) { st[i] = pre.status; continue; }
      p = pre.a;
    }
    const int s = part_ok(H, p) ? H->owner[p] : 0;
    local[i] = part_ok(H, p) ? p - H->lo[s] : -1;
    idx[s].push_back(i);
  }
  std::vector<int> ss, folded(H->S(), 0);
  for (int s = 0; s < H->S(); ++s)
    if (!idx[s].empty()) ss.push_back(s);
  std::vector<std::vector<int32_t>> sst(H->S());
  const int rc = par_shards(H, ss, [&](int s) {
    const size_t m = idx[s].size();
    std::vector<const uint8_t*> mp(m);
    std::vector<int64_t> ml(m);
    std::vector<int32_t> lp(m);
    sst[s].assign(m, 0);
    for (size_t j = 0; j < m; ++j) {
      mp[j] = msgs[idx[s][j]];
      ml[j] = lens[idx[s][j]];
      lp[j] = local[idx[s][j]];
    }
    const int r = dev_ingest_pubsub(H->sh[s], target, mp.data(), ml.data(), (int)m, layers, lp.data(), sst[s].data());
    if (r >= 0) folded[s] = r;
    return r;
  });
  if (rc < 0) return rc;
  int total = 0;
  for (int s : ss) {
    total += folded[s];
    for (size_t j = 0; j < idx[s].size(); ++j) st[idx[s][j]] = sst[s][j];
  }
  if (status) std::memcpy(status, st.data(), sizeof(int32_t) * n_msgs);
  return total;
}

int ipls_agg_blend(ipls_agg* H, int p, int target, const void* src, int64_t n, int src_kind, double a, double b) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_blend(H->sh[s], q, target, src, n, src_kind, a, b));
}

int ipls_agg_scale(ipls_agg* H, int p, int dst_target, int src_target, double c) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_scale(H->sh[s], q, dst_target, src_target, c));
}

int ipls_agg_finalize(ipls_agg* H, int p, void* sum_out, int sum_kind, double* avg_out) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (H->S() == 1) return fwd(H, 0, dev_finalize(H->sh[0], p, sum_out, sum_kind, avg_out));
  if (p == IPLS_ALL_PARTITIONS) {
    if (sum_out || avg_out) return ferr(H, IPLS_E_INVAL, "host outputs need a single partition");
    for (int s : nonempty_shards(H))
      if (int rc = fwd(H, s, dev_finalize(H->sh[s], IPLS_ALL_PARTITIONS, nullptr, sum_kind, nullptr))) return rc;
    return IPLS_OK;
  }
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_finalize(H->sh[s], q, sum_out, sum_kind, avg_out));
}

int ipls_agg_set_weights(ipls_agg* H, int p, const void* src, int64_t n, int src_kind) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_set_weights(H->sh[s], q, src, n, src_kind));
}

int ipls_agg_get_partitions(ipls_agg* H, void* out, int64_t n, int out_kind) {
  KeepDevice keep_device;
  if (!H || !out) return ferr(H, IPLS_E_INVAL, "null argument");
  if (H->S() == 1) return fwd(H, 0, dev_get_partitions(H->sh[0], out, n, out_kind));
  if (n < H->flat_total)
    return ferr(H, IPLS_E_RANGE, "output of %lld < model size %lld", (long long)n, (long long)H->flat_total);
  if (out_kind != IPLS_HOST_F64 && out_kind != IPLS_HOST_BE_CANON && out_kind != IPLS_DEV_F64)
    return ferr(H, IPLS_E_INVAL, "bad out_kind %d", out_kind);
  if (out_kind == IPLS_DEV_F64)
    for (int s : nonempty_shards(H))
      if (int rc = check_reach(H, s, out, "model buffer")) return rc;
  // every shard writes its flat segment [off[lo_s], ...) of the model
  return par_shards(H, nonempty_shards(H), [&](int s) {
    const int64_t base = H->off[H->lo[s]];
    return dev_get_partitions(H->sh[s], (char*)out + 8 * base, n - base, out_kind);
  });
}

namespace {
int get_partitions_chunked(ipls_agg* H, int64_t chunk, ipls_chunk_sink sink, void* ctx, bool wire) {
  KeepDevice keep_device;
  if (!H || !sink) return ferr(H, IPLS_E_INVAL, "null argument");
  // Every shard's divide into a staging of this call first, each under its
  // own shard lock for that launch only; then the snapshots go to the sink
  // shard by shard in model order with no lock held, on the calling thread
  // (a JNIEnv belongs to its thread).  So the whole model is one snapshot,
  // and a slow sink holds no shard.
  const std::vector<int> ss = nonempty_shards(H);
  std::vector<ipls_stage*> st(ss.size(), nullptr);
  int rc = IPLS_OK;
  size_t i = 0;
  for (; i < ss.size() && !rc; ++i) rc = fwd(H, ss[i], dev_get_partitions_snapshot(H->sh[ss[i]], chunk, wire, &st[i]));
  for (size_t j = 0; j < ss.size(); ++j) {
    if (!rc && j < i) {
      rc = fwd(H, ss[j], dev_get_partitions_deliver(H->sh[ss[j]], st[j], chunk, sink, ctx));
    } else if (st[j]) {
      dev_stage_release(H->sh[ss[j]], st[j]);   // after a failure: nothing more is delivered
    }
  }
  return rc;
}
}  // namespace

int ipls_agg_get_partitions_chunked(ipls_agg* H, int64_t chunk, ipls_chunk_sink sink, void* ctx) {
  return get_partitions_chunked(H, chunk, sink, ctx, false);
}

int ipls_agg_get_partitions_wire_chunked(ipls_agg* H, int64_t chunk, ipls_chunk_sink sink, void* ctx) {
  return get_partitions_chunked(H, chunk, sink, ctx, true);
}

int ipls_agg_read(ipls_agg* H, int p, int target, void* dst, int64_t n, int dst_kind) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_read(H->sh[s], q, target, dst, n, dst_kind));
}

int ipls_agg_promote_future(ipls_agg* H, const int32_t* parts, int n_parts) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (H->S() == 1) return fwd(H, 0, dev_promote_future(H->sh[0], parts, n_parts));
  if (n_parts < 0 || (n_parts > 0 && !parts)) return ferr(H, IPLS_E_INVAL, "bad partition list");
  for (int i = 0; i < n_parts; ++i)
    if (!part_ok(H, parts[i])) return range_err(H, parts[i]);
  std::vector<std::vector<int32_t>> per(H->S());
  for (int i = 0; i < n_parts; ++i) per[H->owner[parts[i]]].push_back(parts[i] - H->lo[H->owner[parts[i]]]);
  for (int s = 0; s < H->S(); ++s)
    if (!per[s].empty())
      if (int rc = fwd(H, s, dev_promote_future(H->sh[s], per[s].data(), (int)per[s].size()))) return rc;
  return IPLS_OK;
}

int ipls_agg_reset(ipls_agg* H, int p) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (H->S() == 1) return fwd(H, 0, dev_reset(H->sh[0], p));
  if (p == IPLS_ALL_PARTITIONS) {
    for (int s : nonempty_shards(H))
      if (int rc = fwd(H, s, dev_reset(H->sh[s], IPLS_ALL_PARTITIONS))) return rc;
    return IPLS_OK;
  }
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_reset(H->sh[s], q));
}

int ipls_agg_device_ptr(ipls_agg* H, int p, int target, void** ptr) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_device_ptr(H->sh[s], q, target, ptr));
}

int ipls_agg_checksum(ipls_agg* H, int p, int target, uint64_t* out) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_checksum(H->sh[s], q, target, out));
}

int64_t ipls_agg_commit_partial(ipls_agg* H, int p, int32_t workers, uint8_t* out, int64_t out_cap) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_commit_partial(H->sh[s], q, workers, out, out_cap));
}

int64_t ipls_agg_merge_files(ipls_agg* H, const uint8_t* const* files, const int64_t* lens, int k, int file_kind,
                             uint8_t* out, int64_t out_cap) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  return fwd(H, 0, dev_merge_files(H->sh[0], files, lens, k, file_kind, out, out_cap));
}

int64_t ipls_agg_publish_partial(ipls_agg* H, int p, int target, int32_t a, int32_t b, int16_t pid,
                                 const uint8_t* origin, int32_t origin_len, void* out, int64_t out_cap,
                                 int out_kind) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (!part_ok(H, p)) return range_err(H, p);
  int q;
  const int s = route(H, p, &q);
  return fwd(H, s, dev_publish(H->sh[s], q, target, a, b, pid, origin, origin_len, out, out_cap, out_kind));
}

int64_t ipls_agg_publish_partials(ipls_agg* H, const int32_t* parts, int n_parts, int target, int32_t a,
                                  const int32_t* b, int16_t pid, const uint8_t* origin, int32_t origin_len, void* out,
                                  int64_t out_cap, int out_kind, int64_t* lens, int64_t* offs) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (n_parts < 0 || (n_parts > 0 && (!parts || (out && !b)))) return ferr(H, IPLS_E_INVAL, "bad partition list");
  if (origin_len < 0 || (out && origin_len > 0 && !origin)) return ferr(H, IPLS_E_INVAL, "bad origin");
  if (out_kind != IPLS_HOST_TEXT && out_kind != IPLS_DEV_TEXT) return ferr(H, IPLS_E_INVAL, "out_kind HOST_TEXT/DEV_TEXT");
  std::vector<int64_t> L(n_parts), O(n_parts);
  int64_t total = 0;
  for (int i = 0; i < n_parts; ++i) {
    if (!part_ok(H, parts[i])) return range_err(H, parts[i]);
    O[i] = (total + 63) / 64 * 64;                        // every text 64-B aligned
    L[i] = ipls::pubsub::b64_enc_len(14 + 8 * H->len[parts[i]] + origin_len);
    total = O[i] + L[i];
  }
  if (lens) std::copy(L.begin(), L.end(), lens);
  if (offs) std::copy(O.begin(), O.end(), offs);
  if (!out || n_parts == 0) return total;
  if (out_cap < total) return ferr(H, IPLS_E_RANGE, "publish texts need %lld bytes", (long long)total);
  // group by owner shard; each shard encodes its texts in one launch
  std::vector<std::vector<int>> idx(H->S());
  for (int i = 0; i < n_parts; ++i) idx[H->owner[parts[i]]].push_back(i);
  for (int s = 0; s < H->S(); ++s) {
    if (idx[s].empty()) continue;
    if (out_kind == IPLS_DEV_TEXT)   // the texts are written by shard s's device
      if (int rc = check_reach(H, s, out, "text buffer")) return rc;
    std::vector<int> lp;
    std::vector<int32_t> bb;
    std::vector<int64_t> oo, ll;
    for (int i : idx[s]) {
      lp.push_back(parts[i] - H->lo[s]);
      bb.push_back(b[i]);
      oo.push_back(O[i]);
      ll.push_back(L[i]);
    }
    H->last_shard = s;
    if (int64_t rc = dev_publish_many(H->sh[s], (int)lp.size(), lp.data(), target, a, bb.data(), pid, origin,
                                      origin_len, out, oo.data(), ll.data(), out_kind);
        rc < 0)
      return fwd(H, s, (int)rc);
  }
  return total;
}

// ---- replica slots across GPUs ----

int ipls_agg_reduce_partial(ipls_agg* H, int slot, int p_first, int n_parts, const void* const* bufs, int k,
                            int src_kind, int start_mode) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (slot < 0 || slot >= H->S()) return ferr(H, IPLS_E_INVAL, "slot %d not in [0,%d)", slot, H->S());
  if (n_parts <= 0 || p_first < 0 || p_first + n_parts > H->P)
    return ferr(H, IPLS_E_RANGE, "partitions [%d,%d) out of range [0,%d)", p_first, p_first + n_parts, H->P);
  if (src_kind != IPLS_DEV_F64 && src_kind != IPLS_DEV_BE)
    return ferr(H, IPLS_E_INVAL, "reduce_partial takes device buckets (DEV_F64/DEV_BE)");
  if (start_mode < IPLS_START_ACCUM || start_mode > IPLS_START_FIRST) return ferr(H, IPLS_E_INVAL, "bad start mode");
  if (k < 0 || (k > 0 && !bufs)) return ferr(H, IPLS_E_INVAL, "bad bucket list");
  for (int p = p_first; p < p_first + n_parts; ++p)
    if (H->owner[p] == slot)
      return ferr(H, IPLS_E_INVAL, "slot %d owns partition %d: fold its buckets with reduce_batch", slot, p);
  std::lock_guard<std::mutex> lk(H->mu);
  auto& row = H->part[slot];
  if (row.empty()) row.resize(H->P);
  hipStream_t st = (hipStream_t)dev_stream(H->sh[slot]);
  if (dev_use(H->devices[slot]) != hipSuccess) return ferr(H, IPLS_E_DEVICE, "hipSetDevice failed");
  std::vector<void*> dst(n_parts);
  std::vector<int64_t> lens(n_parts);
  int n_live = 0;
  for (int q = 0; q < n_parts; ++q) {
    Partial& x = row[p_first + q];
    if (!x.d) {
      // an event is recorded only on a stream of the device it was created
      // on: `ready` on the slot's stream, `consumed` on the owner's
      const int od = H->devices[H->owner[p_first + q]];
      const bool ok = hipMalloc(&x.d, (size_t)H->len[p_first + q] * 8) == hipSuccess &&
                      hipEventCreateWithFlags(&x.ready, hipEventDisableTiming) == hipSuccess &&
                      dev_use(od) == hipSuccess &&
                      hipEventCreateWithFlags(&x.consumed, hipEventDisableTiming) == hipSuccess;
      if (dev_use(H->devices[slot]) != hipSuccess || !ok) {
        (void)hipGetLastError();
        return ferr(H, IPLS_E_NOMEM, "partial buffer of partition %d on device %d", p_first + q, H->devices[slot]);
      }
    }
    if (x.consumed_pending) {   // the last combine's reads of this buffer come first
      if (hipStreamWaitEvent(st, x.consumed, 0) != hipSuccess) return ferr(H, IPLS_E_DEVICE, "hipStreamWaitEvent failed");
      x.consumed_pending = false;
    }
    dst[q] = x.d;
    lens[q] = H->len[p_first + q];
    n_live += x.live;
  }
  // ACCUM onto partials that are logically +0.0 is a ZERO-start fold; a mix
  // makes the zero ones physical first
  int start = start_mode;
  if (start_mode == IPLS_START_ACCUM) {
    if (n_live == 0) start = IPLS_START_ZERO;
    else if (n_live < n_parts)
      for (int q = 0; q < n_parts; ++q)
        if (!row[p_first + q].live && hipMemsetAsync(dst[q], 0, (size_t)lens[q] * 8, st) != hipSuccess)
          return ferr(H, IPLS_E_DEVICE, "hipMemsetAsync failed");
  }
  H->last_shard = slot;
  if (int rc = fwd(H, slot, dev_reduce_ext(H->sh[slot], n_parts, lens.data(), bufs, k, src_kind == IPLS_DEV_BE, start,
                                           dst.data())))
    return rc;
  if (dev_use(H->devices[slot]) != hipSuccess) return ferr(H, IPLS_E_DEVICE, "hipSetDevice failed");
  for (int q = 0; q < n_parts; ++q) {
    Partial& x = row[p_first + q];
    if (hipEventRecord(x.ready, st) != hipSuccess) return ferr(H, IPLS_E_DEVICE, "hipEventRecord failed");
    x.live = x.live || k > 0 || start != IPLS_START_ACCUM;
  }
  return IPLS_OK;
}

int ipls_agg_combine_partials(ipls_agg* H, int p_first, int n_parts) {
  KeepDevice keep_device;
  if (!H) return ferr(nullptr, IPLS_E_INVAL, "null handle");
  if (n_parts <= 0 || p_first < 0 || p_first + n_parts > H->P)
    return ferr(H, IPLS_E_RANGE, "partitions [%d,%d) out of range [0,%d)", p_first, p_first + n_parts, H->P);
  std::lock_guard<std::mutex> lk(H->mu);
  const int S = H->S(), end = p_first + n_parts;
  auto live_slots = [&](int q) {
    std::vector<int> v;
    for (int s = 0; s < S; ++s)
      if (!H->part[s].empty() && H->part[s][q].live) v.push_back(s);
    return v;
  };
  int total = 0, n_staged = 0;
  int p = p_first;
  while (p < end) {
    // A run of partitions of one owner with the same NUMBER of live slots is
    // one launch, whichever GPUs hold them: the pointer table is per
    // partition, so an owner whose partitions' replicas sit on different GPUs
    // (ReplicaPlan.spread: every owner pulls from all G-1 others) reads them
    // all at once, over every link, instead of one link per launch.
    const int o = H->owner[p];
    std::vector<std::vector<int>> sl{live_slots(p)};
    const size_t k = sl[0].size();
    int e = p + 1;
    while (e < end && H->owner[e] == o) {
      std::vector<int> v = live_slots(e);
      if (v.size() != k) break;
      sl.push_back(std::move(v));
      ++e;
    }
    if (k > 0) {
      const int od = H->devices[o];
      hipStream_t ost = (hipStream_t)dev_stream(H->sh[o]);
      // no xGMI peer access (or IPLS_PEER_STAGED=1): copy each such partial
      // into an owner-side buffer on its SLOT's stream -- the copies of
      // different slots run on their own engines at once -- and re-record its
      // `ready` there; the same fold then reads the copies in the same order
      std::vector<std::vector<char>> staged(e - p, std::vector<char>(k, 0));
      for (int q = p; q < e; ++q)
        for (size_t j = 0; j < k; ++j) {
          const int s = sl[q - p][j];
          if (H->peer[o][s] && !(H->force_staged && s != o)) continue;
          Partial& x = H->part[s][q];
          const size_t nb = (size_t)H->len[q] * 8;
          if (!x.stage && (dev_use(od) != hipSuccess || hipMalloc(&x.stage, nb) != hipSuccess)) {
            (void)hipGetLastError();
            return ferr(H, IPLS_E_NOMEM, "staging buffer of partition %d on device %d", q, od);
          }
          hipStream_t sst = (hipStream_t)dev_stream(H->sh[s]);
          if (dev_use(H->devices[s]) != hipSuccess ||
              hipMemcpyPeerAsync(x.stage, od, x.d, H->devices[s], nb, sst) != hipSuccess ||
              hipEventRecord(x.ready, sst) != hipSuccess) {
            (void)hipGetLastError();
            return ferr(H, IPLS_E_DEVICE, "partial copy from device %d to %d failed", H->devices[s], od);
          }
          staged[q - p][j] = 1;
          ++n_staged;
        }
      if (dev_use(od) != hipSuccess) return ferr(H, IPLS_E_DEVICE, "hipSetDevice failed");
      std::vector<const void*> ptrs((size_t)(e - p) * k);
      for (int q = p; q < e; ++q)
        for (size_t j = 0; j < k; ++j) {
          Partial& x = H->part[sl[q - p][j]][q];
          if (hipStreamWaitEvent(ost, x.ready, 0) != hipSuccess) return ferr(H, IPLS_E_DEVICE, "hipStreamWaitEvent failed");
          ptrs[(size_t)(q - p) * k + j] = staged[q - p][j] ? (const void*)x.stage : (const void*)x.d;
        }
      // REP[q] = ((REP[q] + R_s1) + R_s2) ..., slots ascending per partition:
      // the Updater replica branch / Collect_Replicas fold (Updater.java:40-44,
      // IPLS.java:1222-1234)
      H->last_shard = o;
      if (int rc = fwd(H, o, dev_reduce_batch(H->sh[o], p - H->lo[o], e - p, ptrs.data(), (int)k, IPLS_DEV_F64,
                                              IPLS_START_ACCUM, IPLS_TGT_REP)))
        return rc;
      if (dev_use(od) != hipSuccess) return ferr(H, IPLS_E_DEVICE, "hipSetDevice failed");
      for (int q = p; q < e; ++q)
        for (int s : sl[q - p]) {
          Partial& x = H->part[s][q];
          if (hipEventRecord(x.consumed, ost) != hipSuccess) return ferr(H, IPLS_E_DEVICE, "hipEventRecord failed");
          x.consumed_pending = true;
          x.live = false;
        }
      total += (e - p) * (int)k;
    }
    p = e;
  }
  H->last_staged.store(n_staged, std::memory_order_relaxed);
  return total;
}

}  // extern "C"
