// engine.hip -- the single-device aggregation engine behind the C-ABI
// (include/ipls_agg.h; the exported entry points are in ipls_agg.cpp, which
// shards a handle's partitions over one engine per device).  One engine =
// the PeerData accumulator state of a contiguous block of partitions on one
// GPU, one HIP stream, one mutex.
//
// Device layout: one arena of doubles per handle holding, for
// every partition p, four arrays of L_p doubles -- AGG (Aggregated_Gradients,
// PeerData.java:144), REP (Replicas_Gradients, :137), FUT (Aggregated_
// Gradients_from_future) and W (Weights, :149, which IPLS.java:1141 aliases
// with Weight_Address, :189) -- each starting on a 256-byte boundary.
// Device-side tables (partition descriptors + bucket pointers) are uploaded
// through a small pinned ring and cached, so a repeated reduce over resident
// buckets is one kernel launch and nothing else.  The chunked calls stage
// through a stage each (struct ipls_stage, pooled per engine) and take the
// engine lock only for their fold or snapshot.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ipls_agg.h"
#include "ipls_kernels.hpp"
#include "javaser.hpp"
#include "engine.hpp"
#include "pubsub_host.hpp"

using namespace ipls;

namespace {

thread_local std::string g_tls_err;

constexpr int64_t kAlignElems = 32;  // 256 B
constexpr int kRingSlots = 4;
constexpr int kStageSlots = 3;   // pinned slots of a chunked call's ring (IPLS_STAGE_SLOTS overrides)

int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

struct PinnedSlot {
  void* host = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  bool pending = false;
};

}  // namespace

// The staging of one chunked call (accumulate / finalize / get_partitions
// _chunked), owned by that call alone from acquire to release, so the
// caller's source or sink -- a socket recv/send, a JNI array copy -- runs
// with no engine lock held.  A pinned host ring,
// a device buffer for the whole bucket (or snapshot) and two copy streams of its
// own.  Stages are pooled per shard and freed only at close.
// Invariants at release: every pinned slot whose copy may still be in flight
// is `pending` (its event recorded after that copy); `free_pending` says a
// kernel on the shard stream may still read `d` (recorded after it).
struct ipls_stage {
  // chunk k crosses PCIe on copy[k % n_copy]: with two streams the DMA setup
  // of chunk k + 1 overlaps the transfer of chunk k (IPLS_STAGE_STREAMS=1
  // gives one stream, the A/B of profiles/r06)
  hipStream_t copy[2] = {};
  int n_copy = 0;
  // the pinned host ring: chunk k in slot k % n_slot, so the copy engine can
  // run up to n_slot - 1 chunks ahead of a caller's slow source or sink
  // (IPLS_STAGE_SLOTS, 2..4)
  static constexpr int kMaxSlots = 4;
  PinnedSlot slot[kMaxSlots];
  int n_slot = 0;
  void* d = nullptr;
  size_t d_cap = 0;
  hipEvent_t landed[2] = {};      // copy streams -> shard stream: every chunk is in `d`
  hipEvent_t ready = nullptr;     // shard stream -> copy streams: the snapshot is in `d`
  hipEvent_t free_ev = nullptr;   // shard stream: the fold that read `d` has run
  bool free_pending = false;
};

struct ipls_dev {
  std::mutex mu;
  std::string err;
  int device = 0;
  hipStream_t stream = nullptr;

  // geometry
  int64_t model_size = 0;  // 0 => synthetic geometry
  int P = 0;
  int64_t chunk = 0;  // flat stride between partitions
  int secure = 0;
  std::vector<int64_t> len, flat_off;
  int64_t max_len = 0, flat_total = 0;   // flat_total: end of this engine's flat segment
  int p_lo = 0;                           // first partition of the handle held here
  int64_t flat_base = 0;                  // flat offset of partition p_lo

  // arena
  double* arena = nullptr;
  int64_t arena_elems = 0;
  std::vector<int64_t> agg_off, rep_off, w_off, fut_off;
  std::vector<uint8_t> agg_zero, rep_zero, fut_zero;  // "logically +0.0" flags

  // table upload ring (pinned host slots -> device slots)
  PinnedSlot ring[kRingSlots];
  void* d_table[kRingSlots] = {};
  size_t d_table_cap[kRingSlots] = {};
  int ring_next = 0;
  std::vector<unsigned char> last_table;  // cache of the last uploaded table
  int last_slot = -1;

  // staging of the chunked calls: one per concurrent call, pooled (lazily,
  // freed at close); stage_mu guards the pool only, never taken with mu held
  // for longer than a push
  std::mutex stage_mu;
  std::vector<ipls_stage*> stage_all, stage_idle;
  // staging
  void* d_scratch = nullptr;
  size_t scratch_bytes = 0;
  hipEvent_t copy_ev = nullptr;
  // pubsub ingest pipeline: text copies on their own stream, the decodes on
  // `stream` behind an event per message (created on first use)
  static constexpr int kCopyThreads = 4;
  hipStream_t copy_stream[kCopyThreads] = {};
  hipEvent_t ingest_ev = nullptr;
  std::vector<hipEvent_t> msg_ev;
  // Per-arrival staging of pageable buckets, double-buffered: bucket k+1 is
  // copied into one slot while the fold of bucket k still reads the other.
  struct StageSlot {
    void* d = nullptr;
    size_t cap = 0;
    hipEvent_t free_ev = nullptr;   // recorded after the fold that reads the slot
    bool pending = false;
  };
  StageSlot stage[2];
  int stage_next = 0;
  // Asynchronous folds (ipls_agg_accumulate_async).  Device buckets are not
  // folded on arrival: per (target, partition) their pointers queue up and the
  // next flush folds each queue in one launch, in call order -- the same
  // expression (((acc + b0) + b1) + ...) the per-arrival folds evaluate, at
  // (k+2)/k x 8 B per element instead of 24.  Every other entry point flushes
  // first (IPLS_LOCK).  Pinned host buckets fold at once (zero copy).
  struct Pending {
    std::vector<const void*> bufs;
    bool be = false;
  };
  // queue of (target, p) at pend[target * P + p]; pend_keys lists the
  // non-empty ones (a flat table: the per-arrival call is a few loads and a
  // push, no map walk)
  std::vector<Pending> pend;
  std::vector<int> pend_keys;
  int pending_n = 0;
  int coalesce = 32;                                // queue length that triggers a flush (ipls_agg_set_coalesce)
  // Tickets complete in issue order: a launch happens only after every earlier
  // ticket was launched, and batch b completes tickets (prev.max, b.max_ticket].
  struct Batch {
    uint64_t max_ticket;
    hipEvent_t ev;
  };
  static constexpr int kMaxBatches = 64;
  std::deque<Batch> batches;
  std::vector<hipEvent_t> ev_free;
  uint64_t ticket_next = 1, ticket_done = 0, launched_upto = 0;

  // checksum result
  unsigned long long* d_sum = nullptr;
  double* d_cnt = nullptr;   // per-partition count slots of a fused round (P doubles)
  unsigned long long* d_gbuf = nullptr;   // Updater.run's Gradient_Buff (Updater.java:162), lazily
  unsigned long long* d_merge = nullptr;  // storage-merge accumulator, grown on demand
  int64_t merge_cap = 0;
  // PeerData.Other_Replica_Gradients / _Received, keyed (partition, aggregator);
  // Collect_Replicas folds them in the order the front's HashMap model gives
  struct OtherRep {
    unsigned long long* d = nullptr;
    int64_t n = 0;
    int32_t received = 0;
  };
  std::map<std::pair<int, int32_t>, OtherRep> other;
  int64_t gbuf_len = 0;
  ipls_launch_info last_launch{};   // the last fold launch (ipls_agg_last_launch)
};

namespace {

int fail(ipls_dev* h, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (h) h->err = buf;
  g_tls_err = buf;
  return code;
}

int flush_pending(ipls_dev* h);

// Take the handle's lock and fold any queued asynchronous device arrivals
// first, so every entry point sees the accumulators in call order.
#define IPLS_LOCK(h)                            \
  std::lock_guard<std::mutex> lk_(h->mu);       \
  if (int rc_ = flush_pending(h)) return rc_

// A failed call also leaves HIP's per-thread last error set; it is cleared
// here so that the next launch check (hipGetLastError) does not report it.
#define HIP_TRY(h, expr)                                                                \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      (void)hipGetLastError();                                                          \
      return fail((h), e_ == hipErrorOutOfMemory ? IPLS_E_NOMEM : IPLS_E_DEVICE,        \
                  "%s failed: %s", #expr, hipGetErrorString(e_));                       \
    }                                                                                   \
  } while (0)

int64_t ref_chunk(int64_t m, int p) { return (int64_t)(int32_t)(m / p) + 1; }  // IPLS.java:1019


int check_part(ipls_dev* h, int p) {
  if (p < 0 || p >= h->P) return fail(h, IPLS_E_RANGE, "partition %d out of range [0,%d)", p, h->P);
  return IPLS_OK;
}

int64_t target_off(ipls_dev* h, int p, int target) {
  switch (target) {
    case IPLS_TGT_AGG: return h->agg_off[p];
    case IPLS_TGT_REP: return h->rep_off[p];
    case IPLS_TGT_WEIGHTS:
    case IPLS_TGT_WADDR: return h->w_off[p];
    case IPLS_TGT_FUTURE: return h->fut_off[p];
    default: return -1;
  }
}

uint8_t* zero_flag(ipls_dev* h, int p, int target) {
  if (target == IPLS_TGT_AGG) return &h->agg_zero[p];
  if (target == IPLS_TGT_REP) return &h->rep_zero[p];
  if (target == IPLS_TGT_FUTURE) return &h->fut_zero[p];
  return nullptr;
}

// Make a logically-zero accumulator physically zero (before anything reads it
// with ACCUM semantics or hands its address out).
int materialize(ipls_dev* h, int p, int target) {
  uint8_t* f = zero_flag(h, p, target);
  if (f && *f) {
    HIP_TRY(h, hipMemsetAsync(h->arena + target_off(h, p, target), 0, (size_t)h->len[p] * 8, h->stream));
    *f = 0;
  }
  return IPLS_OK;
}

int ensure_pinned(ipls_dev* h, PinnedSlot& s, size_t bytes) {
  if (s.pending) {
    HIP_TRY(h, hipEventSynchronize(s.ev));
    s.pending = false;
  }
  if (s.cap < bytes) {
    if (s.host) HIP_TRY(h, hipHostFree(s.host));
    s.host = nullptr;
    s.cap = 0;
    size_t cap = std::max<size_t>(bytes, 64 << 10);
    HIP_TRY(h, hipHostMalloc(&s.host, cap, hipHostMallocDefault));
    s.cap = cap;
  }
  if (!s.ev) HIP_TRY(h, hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
  return IPLS_OK;
}

// ---- chunked-call staging (ipls_stage) ----
// A failure outside the engine lock: the calling thread's message, and the
// handle's under its lock (h->err is shared with the locked paths).
int fail_nl(ipls_dev* h, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_tls_err = buf;
  if (h) {
    std::lock_guard<std::mutex> lk(h->mu);
    h->err = buf;
  }
  return code;
}

#define HIP_TRY_NL(h, expr)                                                             \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      (void)hipGetLastError();                                                          \
      return fail_nl((h), e_ == hipErrorOutOfMemory ? IPLS_E_NOMEM : IPLS_E_DEVICE,     \
                     "%s failed: %s", #expr, hipGetErrorString(e_));                    \
    }                                                                                   \
  } while (0)

// Take an idle stage of the pool (or make one) and size it: `dev_bytes` of
// device buffer, two pinned slots of `slot_bytes`.  Called with the engine
// lock NOT held, on the shard's device.  Regrowing frees only memory this
// call owns, after the copies and the kernel that last used it are done.
int stage_acquire(ipls_dev* h, size_t dev_bytes, size_t slot_bytes, ipls_stage** out) {
  *out = nullptr;
  ipls_stage* st = nullptr;
  {
    std::lock_guard<std::mutex> lk(h->stage_mu);
    if (!h->stage_idle.empty()) {
      st = h->stage_idle.back();
      h->stage_idle.pop_back();
    } else {
      st = new ipls_stage();
      h->stage_all.push_back(st);
    }
  }
  auto give_back = [&](int rc) {
    std::lock_guard<std::mutex> lk(h->stage_mu);
    h->stage_idle.push_back(st);
    return rc;
  };
  auto try_hip = [&](hipError_t e, const char* what) -> int {
    if (e == hipSuccess) return IPLS_OK;
    (void)hipGetLastError();
    return fail_nl(h, e == hipErrorOutOfMemory ? IPLS_E_NOMEM : IPLS_E_DEVICE, "%s failed: %s", what,
                   hipGetErrorString(e));
  };
  int rc = IPLS_OK;
  if (!st->n_copy) {
    const char* e = std::getenv("IPLS_STAGE_STREAMS");
    st->n_copy = (e && std::atoi(e) == 1) ? 1 : 2;
    const char* sl = std::getenv("IPLS_STAGE_SLOTS");
    st->n_slot = sl ? std::max(2, std::min(ipls_stage::kMaxSlots, std::atoi(sl))) : kStageSlots;
  }
  for (int i = 0; i < st->n_copy && !rc; ++i)
    if (!st->copy[i]) rc = try_hip(hipStreamCreateWithFlags(&st->copy[i], hipStreamNonBlocking), "hipStreamCreate");
  for (hipEvent_t* e : {&st->landed[0], &st->landed[1], &st->ready, &st->free_ev})
    if (!rc && !*e) rc = try_hip(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate");
  if (!rc && st->d_cap < dev_bytes) {
    if (st->d) {
      // the fold that last read `d` and every copy of the stage are done before it is freed
      if (st->free_pending) rc = try_hip(hipEventSynchronize(st->free_ev), "hipEventSynchronize");
      for (int i = 0; i < st->n_copy && !rc; ++i) rc = try_hip(hipStreamSynchronize(st->copy[i]), "hipStreamSynchronize");
      if (!rc) rc = try_hip(hipFree(st->d), "hipFree");
      if (!rc) {
        st->d = nullptr;
        st->d_cap = 0;
        st->free_pending = false;
      }
    }
    const size_t cap = (size_t)align_up((int64_t)dev_bytes, 1 << 20);
    if (!rc) rc = try_hip(hipMalloc(&st->d, cap), "hipMalloc");
    if (!rc) st->d_cap = cap;
  }
  for (int i = 0; i < st->n_slot; ++i) {
    PinnedSlot& s = st->slot[i];
    if (rc) break;
    if (s.cap < slot_bytes) {
      if (s.pending) rc = try_hip(hipEventSynchronize(s.ev), "hipEventSynchronize");
      if (!rc) s.pending = false;
      // never free a slot a copy may still read or write (the r05/h fault
      // analysis): its last copy's event must have completed
      if (!rc && s.host && s.ev && hipEventQuery(s.ev) != hipSuccess) {
        (void)hipGetLastError();
        rc = fail_nl(h, IPLS_E_DEVICE, "internal: pinned slot regrown with a copy in flight");
      }
      if (!rc && s.host) rc = try_hip(hipHostFree(s.host), "hipHostFree");
      if (!rc) {
        s.host = nullptr;
        s.cap = 0;
        const size_t cap = std::max<size_t>(slot_bytes, 64 << 10);
        rc = try_hip(hipHostMalloc(&s.host, cap, hipHostMallocDefault), "hipHostMalloc");
        if (!rc) s.cap = cap;
      }
    }
    if (!rc && !s.ev) rc = try_hip(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming), "hipEventCreate");
  }
  if (rc) return give_back(rc);
  *out = st;
  return IPLS_OK;
}

void stage_release(ipls_dev* h, ipls_stage* st) {
  if (!st) return;
  std::lock_guard<std::mutex> lk(h->stage_mu);
  h->stage_idle.push_back(st);
}

// The host may write this pinned slot again: the copy that last read it is done.
int stage_slot_free(ipls_dev* h, PinnedSlot& sl) {
  if (sl.pending) {
    HIP_TRY_NL(h, hipEventSynchronize(sl.ev));
    sl.pending = false;
  }
  return IPLS_OK;
}

int ensure_scratch(ipls_dev* h, size_t bytes) {
  if (h->scratch_bytes >= bytes) return IPLS_OK;
  if (h->d_scratch) {
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    HIP_TRY(h, hipFree(h->d_scratch));
    h->d_scratch = nullptr;
    h->scratch_bytes = 0;
  }
  size_t cap = (size_t)align_up((int64_t)bytes, 1 << 20);
  HIP_TRY(h, hipMalloc(&h->d_scratch, cap));
  h->scratch_bytes = cap;
  return IPLS_OK;
}

// Upload a table through the pinned ring; returns its device address.  An
// identical table to the previous upload is not re-sent.
int upload_table(ipls_dev* h, const void* data, size_t bytes, void** dev) {
  if (h->last_slot >= 0 && h->last_table.size() == bytes &&
      std::memcmp(h->last_table.data(), data, bytes) == 0) {
    *dev = h->d_table[h->last_slot];
    return IPLS_OK;
  }
  const int s = h->ring_next;
  h->ring_next = (s + 1) % kRingSlots;
  int rc = ensure_pinned(h, h->ring[s], bytes);
  if (rc) return rc;
  if (h->d_table_cap[s] < bytes) {
    if (h->d_table[s]) {
      HIP_TRY(h, hipStreamSynchronize(h->stream));
      HIP_TRY(h, hipFree(h->d_table[s]));
    }
    h->d_table[s] = nullptr;
    h->d_table_cap[s] = 0;
    size_t cap = std::max<size_t>(bytes, 64 << 10);
    HIP_TRY(h, hipMalloc(&h->d_table[s], cap));
    h->d_table_cap[s] = cap;
  }
  std::memcpy(h->ring[s].host, data, bytes);
  HIP_TRY(h, hipMemcpyAsync(h->d_table[s], h->ring[s].host, bytes, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(h, hipEventRecord(h->ring[s].ev, h->stream));
  h->ring[s].pending = true;
  h->last_table.assign((const unsigned char*)data, (const unsigned char*)data + bytes);
  h->last_slot = s;
  *dev = h->d_table[s];
  return IPLS_OK;
}

// Copy `bytes` of host memory to device `dst` through the pinned double buffer.
// The caller's buffer is no longer referenced when this returns.
bool is_pinned_host(const void* p, void** dev_alias = nullptr) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: clear the sticky error
    return false;
  }
  if (a.type != hipMemoryTypeHost) return false;
  if (dev_alias) {
    // device address of the same bytes (== p for hipHostMalloc; may differ
    // for hipHostRegister'ed memory)
    const char* base_h = (const char*)a.hostPointer;
    const char* base_d = (const char*)a.devicePointer;
    *dev_alias = (base_h && base_d) ? (void*)(base_d + ((const char*)p - base_h)) : nullptr;
  }
  return true;
}

// Memory a kernel of this process may write at the address p itself: device
// memory, or pinned host memory mapped at the same address (hipHostMalloc).
// Pageable memory is rejected before any launch (a kernel store there faults).
bool kernel_writable(const void* p) {
  hipPointerAttribute_t a;
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) return true;
  void* alias = nullptr;
  return a.type == hipMemoryTypeHost && is_pinned_host(p, &alias) && alias == p;
}

// Copy `bytes` of host memory (pinned or pageable) to device `dst` on the
// handle's stream and wait for that copy only: the caller may reuse its buffer
// on return, kernels queued behind the copy keep running.  HIP's own path for
// pageable sources runs at the PCIe rate (56 GB/s measured, tools/h2d_bench.hip),
// where a memcpy into pinned staging was capped at ~31 GB/s by one CPU thread.
int stage_h2d(ipls_dev* h, void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return IPLS_OK;
  if (!h->copy_ev) HIP_TRY(h, hipEventCreateWithFlags(&h->copy_ev, hipEventDisableTiming));
  HIP_TRY(h, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(h, hipEventRecord(h->copy_ev, h->stream));
  HIP_TRY(h, hipEventSynchronize(h->copy_ev));
  return IPLS_OK;
}

// Host-synchronous H2D copy of a pageable buffer on a copy stream: no
// ordering against `stream` (the caller owns `dst`), so it overlaps the fold
// of the previous arrival.  (Splitting it over two threads measured within
// noise at 32 MiB and +1.6 % at 64 MiB, profiles/r01/host_e2e_pageable_split.txt.)
int copy_pageable(ipls_dev* h, void* dst, const void* src, size_t bytes) {
  if (!h->copy_stream[0]) HIP_TRY(h, hipStreamCreateWithFlags(&h->copy_stream[0], hipStreamNonBlocking));
  HIP_TRY(h, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, h->copy_stream[0]));
  HIP_TRY(h, hipStreamSynchronize(h->copy_stream[0]));
  return IPLS_OK;
}

// Stage one pageable per-arrival bucket into the next of the two staging
// slots; release_stage() marks the slot busy until the fold queued after it.
int stage_bucket(ipls_dev* h, const void* src, size_t bytes, const void** dptr) {
  ipls_dev::StageSlot& sl = h->stage[h->stage_next];
  if (sl.pending) {   // the fold that read this slot two arrivals ago
    HIP_TRY(h, hipEventSynchronize(sl.free_ev));
    sl.pending = false;
  }
  if (sl.cap < bytes) {
    if (sl.d) HIP_TRY(h, hipFree(sl.d));
    sl.d = nullptr;
    sl.cap = 0;
    const size_t cap = (size_t)align_up((int64_t)bytes, 1 << 20);
    HIP_TRY(h, hipMalloc(&sl.d, cap));
    sl.cap = cap;
  }
  if (!sl.free_ev) HIP_TRY(h, hipEventCreateWithFlags(&sl.free_ev, hipEventDisableTiming));
  if (int rc = copy_pageable(h, sl.d, src, bytes)) return rc;
  *dptr = sl.d;
  return IPLS_OK;
}

int release_stage(ipls_dev* h) {
  ipls_dev::StageSlot& sl = h->stage[h->stage_next];
  HIP_TRY(h, hipEventRecord(sl.free_ev, h->stream));
  sl.pending = true;
  h->stage_next ^= 1;
  return IPLS_OK;
}

int d2h(ipls_dev* h, void* dst, const void* src, size_t bytes) {
  HIP_TRY(h, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return IPLS_OK;
}

unsigned blocks_for(int64_t n, int64_t per_block) { return (unsigned)((n + per_block - 1) / per_block); }

// The elementwise kernels (k_fold_n, k_blend, k_scale, k_encode_secure) take
// their 16-B tile shape when every operand is 16-B aligned: one block per
// kEwTile elements; otherwise the 8-B grid-stride loop on a capped grid.
static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
static dim3 ew_grid(int64_t n, bool vec, unsigned cap) {
  return dim3(std::max(1u, vec ? blocks_for(n, kEwTile) : std::min<unsigned>(blocks_for(n, kBlock), cap)));
}
static void launch_bswap(hipStream_t st, const unsigned long long* in, unsigned long long* out, int64_t n) {
  if (al16(in) && al16(out)) hipLaunchKernelGGL(k_bswap64<true>, ew_grid(n, true, 4096), dim3(kBlock), 0, st, in, out, n);
  else hipLaunchKernelGGL(k_bswap64<false>, ew_grid(n, false, 4096), dim3(kBlock), 0, st, in, out, n);
}

// ---- kernel dispatch: k_reduce ----
// Three shapes (tools/reduce_sweep.hip, profiles/r01/sweep*.txt), the first
// whose tiles fill the 256 CUs (fill()):
//  * big: 1024-lane workgroups, 1 peer in flight x 16 x 16 B per lane, i.e.
//    each CU streams one 256 KiB contiguous chunk of one bucket at a time
//    (fewer, longer DRAM streams): 85-89 % of 8 TB/s on config C over every
//    bucket layout tried, vs 80-86 % for 256-lane / 64 KiB blocks;
//  * mid: the same per-lane work on 256-lane workgroups (64 KiB chunks), for
//    batches of one or a few partitions: 1 x 4M x 32 at 86.2 % vs 72.7 % for
//    the small shape and 55.8 % for the big one on 128 CUs
//    (profiles/r01/sweep_few_partitions.txt);
//  * small: 256 lanes, 8 peers in flight x 16 B per lane, partition-major --
//    enough blocks for short partitions (ETHModel's 3 x 147,872).
constexpr int kBigG = 1, kBigMap = 0, kBigBS = 1024, kMidBS = 256;
constexpr int kSmallG = 8, kSmallR = 1, kSmallMap = 0;
// A tile count fills the chip when it is at least two waves of 256 CUs, or
// one or more waves with at most a fifth of the last one idle.
inline bool fill(int64_t tiles) {
  if (tiles >= 512) return true;
  if (tiles < 256) return false;
  const int64_t waves = (tiles + 255) / 256;
  return tiles * 5 >= waves * 256 * 4;
}
// 16 x 16 B per lane in the 128-VGPR budget of a 1024-lane workgroup:
// native doubles 126 VGPRs; big-endian input 110 with the SEQ schedule of
// reduce_tiles (hipcc's own schedule hoisted the loads around the bswap and
// spilled 184 B).  The ACCUM start keeps 8 (at 16 it still spills around
// the loop -- checked with -Rpass-analysis=kernel-resource-usage).
// IPLS_BE_BIG_R / IPLS_BE_SEQF rebuild the big-endian big shape with another
// schedule for same-process A/B runs (make -C ipls-java-api_amd variants,
// bench.py --be-schedule-ab); the shipped library uses the defaults.
#ifndef IPLS_BE_BIG_R
#define IPLS_BE_BIG_R 16
#endif
#ifndef IPLS_BE_SEQF
#define IPLS_BE_SEQF 3
#endif
template <bool BE_IN, int START, bool FIN = false>
constexpr int big_r() { return START != kAccum ? (BE_IN ? IPLS_BE_BIG_R : 16) : 8; }
// SEQ schedule of the big shape (0 = hipcc's own): big-endian input at R = 16
// loads, decodes and adds a peer's vectors three at a time with a fence after
// each group (SEQF = 3; 118 VGPRs, no spills).  Round 2 swept fence periods
// 1-8 with and without a free tail in one process (profiles/r02/s3/
// sweep_be_tail{1,2}*.txt): 3 beats round 1's every-2-with-the-last-4-free
// (SEQF = 42) by 0.7-1.6 points on C's and D's shapes, BE in and in + out;
// periods >= 5, a free tail on period 3, and period 1 are all slower.
template <bool BE_IN, int START>
constexpr int big_seqf() { return (BE_IN && big_r<BE_IN, START>() > 8) ? IPLS_BE_SEQF : 0; }
// Block order of the big shape over whole tiles: partition-major (map 0),
// except big-endian input on grids of at most 4096 tiles, which runs
// XCD-chunked (map 2: each XCD walks one contiguous eighth of the work).  With
// SEQF = 3, map 2 measured +2 to +3.6 points at 2-4 partitions of 4M x 32,
// +0.2 to +0.6 at 16, and -3.6 at 64 (config D, 8192 tiles); native doubles
// gain nothing from it at 16 (profiles/r02/s3/sweep_be_map.txt,
// sweep_map_fewp.txt) and run the half shape below on short grids.
template <bool BE_IN>
inline int big_map(int64_t tiles) { return (BE_IN && tiles <= 4096) ? 2 : kBigMap; }
// The half shape (round 3): ZERO/FIRST start, batches of fewer than 4
// rounds of big tiles on 256 CUs (fewer than 1024 whole big tiles: one to
// seven partitions of 4M, config B), and larger grids that the big tiles
// would leave partly idle in their last round (below).  512-lane workgroups at R = 16 -- 128
// KiB of a bucket per block, one workgroup per CU, no spills, every load of a
// peer's chunk in flight: native doubles at 164 VGPRs, big-endian input on
// hipcc's own schedule at 172 (the 256-VGPR budget of 512 lanes needs no SEQ
// fences).  Same process, same buckets (profiles/r03/e/sweep_fewp.txt,
// r03/f/sweep_512_*.txt, r03/h/sweep_fewp_be.txt): native 1/2/3/5/7
// partitions of 4M x 32 at 87.1/83.2/89.8/89.5/89.1 % against 56.2/80.5/
// 74.9/80.7/82.7 % for the big shape (whose 128 tiles per partition leave
// half a round idle at odd counts) and 87.4/70.1/85.2/78.5/81.0 % for mid;
// big-endian in + out 88.2/87.8/87.0/86.0/85.0 % against 84.3 (mid)/82.7/
// 84.5 (mid)/79.6/82.9 % for what shipped; config B 80.2-82.3 % against
// 78.7-81.8 %.  At config C (2048 big tiles) the big shape stays ahead
// (87.1-87.8 vs 85.0-87.1 %), at F they tie, at D (BE) big SEQF = 3 wins.
// Both counts are of WHOLE tiles: a partial last tile (map 3) is scheduled
// first and runs beside the first round, so 4M + 3 doubles is one round of
// 256 half tiles, not 257.
constexpr int kHalfBS = 512, kHalfR = 16;
// The fused round (k_round, 166 VGPRs native / 174 big-endian at 512 lanes,
// no spills) takes the half shape on the same rule: same process, same
// buckets against its big/mid shapes (tools/half_round_probe.py,
// profiles/r03/i/half_round_probe.jsonl): 1/2/3/5 partitions of 4M x 32 at
// 85.4/81.2/80.8/81.0 % vs 84.5/79.0/78.1/74.2 %, 3 x 4M big-endian 80.2 vs
// 74.3 %, config B's shape 71.9 vs 72.8 %.  IPLS_HALF_ROUND=0 builds the
// fused round without it (the A/B variant, make variants).
#ifndef IPLS_HALF_ROUND
#define IPLS_HALF_ROUND 1
#endif
// ACCUM (the fold reads its target too) on fewer than 1024 big R = 16
// tiles: the half shape at R = 16 (202 VGPRs native, 204 big-endian, no
// spills) instead of the big R = 8 tiles of the same size.  Same process
// (profiles/r03/k/sweep_accum.txt, r03/l/sweep_accum2*.txt): 1/2/3/5
// partitions of 4M x 32 at 83.9/82.7/85.3/84.9 % vs 81.0/80.9/82.3/82.5 %,
// big-endian 1/3 at 81.8/82.9 vs 79.2/81.4 %; at 16/32/64 partitions the two
// tie (82.3/79.9/81.6 vs 81.8/80.2/81.2 %), which the big R = 8 tiles keep.
// The fused round's ACCUM start (AGG already holds arrivals) keeps big/mid.
#ifndef IPLS_HALF_ACCUM
#define IPLS_HALF_ACCUM 1
#endif
// Past 4 rounds the half shape also takes grids whose big tiles leave part
// of the last round idle while its own tiles do not (with L = 4M: 9, 11, 13,
// 15 partitions; profiles/r03/k/sweep_midp.txt: 9 x 4M 87.3-87.5 vs 82.8-83.0 %,
// 13 x 4M 84.3-84.4 vs 83.4-83.5 %), and leaves whole rounds to the big shape
// (8, 10, 12 x 4M: big ahead by 0-0.8 points).
inline double round_eff(int64_t tiles) {   // busy fraction of the rounds of 256 one-workgroup CUs
  const int64_t r = (tiles + 255) / 256;
  return r > 0 ? (double)tiles / (double)(r * 256) : 0.0;
}
// The big tiles counted are the R = 16 ones (32768 doubles) for every start
// mode: ACCUM's big shape runs R = 8 tiles the size of a half tile.
// IPLS_HALF_ALWAYS=1 (A/B builds only) sends every grid that fills to it.
#ifndef IPLS_HALF_ALWAYS
#define IPLS_HALF_ALWAYS 0
#endif
inline bool use_half(int64_t maxL, int n_parts, int64_t half_tile) {
  const int64_t tb = (maxL / ((int64_t)kBigBS * 2 * 16)) * n_parts, th = (maxL / half_tile) * n_parts;
  return fill(th) && (IPLS_HALF_ALWAYS || tb < 1024 || round_eff(th) > round_eff(tb) + 0.06);
}
// The mid shape (256 lanes, one or two partitions: per-partition flushes, the
// storage merge of one partition's files) with big-endian input runs 8
// vectors per lane on hipcc's own schedule (100 VGPRs, no spills): one
// partition of 4M x 32 peers at 83-86 % against 55-64 % for the big shape's
// R = 16 SEQ schedules at 256 lanes (profiles/r02/s3/sweep_be_p1.txt, BE in
// and BE in + out, two processes each).  Native doubles keep R = 16 (86-88 %).
template <bool BE_IN, int START>
constexpr int mid_r() { return BE_IN ? 8 : big_r<BE_IN, START>(); }
template <bool BE_IN, int START>
constexpr int mid_seqf() { return mid_r<BE_IN, START>() > 8 ? big_seqf<BE_IN, START>() : 0; }

// C-ABI start mode -> kernel template start
int kstart(int start_mode) {
  return start_mode == IPLS_START_ZERO ? kZero : start_mode == IPLS_START_FIRST ? kFirst : kAccum;
}

// What a fold launch ran (ipls_agg_last_launch): tests assert that a case
// reaches the kernel shape it was written for.
ipls_launch_info launch_info(int kernel, int shape, int block, int r, int seqf, int map, int64_t grid, bool be_in,
                             bool be_out, int start) {
  ipls_launch_info li{};
  li.kernel = kernel;
  li.shape = shape;
  li.block = block;
  li.vectors = r;
  li.seqf = seqf;
  li.map = map;
  li.grid = grid;
  li.be_in = be_in;
  li.be_out = be_out;
  li.start = start == kZero ? IPLS_START_ZERO : start == kFirst ? IPLS_START_FIRST : IPLS_START_ACCUM;
  return li;
}

template <bool BE_IN, bool BE_OUT, int START, bool FIN = false>
ipls_launch_info launch_reduce_v(int64_t maxL, int n_parts, hipStream_t st, const unsigned long long* const* bufs,
                                 const PartDesc* parts, int k, int secure = 0, const double* cnts = nullptr) {
  constexpr int R = big_r<BE_IN, START, FIN>();
  constexpr int RM = mid_r<BE_IN, START>();
  constexpr int KER = FIN ? IPLS_KERNEL_ROUND : IPLS_KERNEL_REDUCE;
  const int64_t big_tile = (int64_t)kBigBS * 2 * R;
  const int64_t big_tpp = (maxL + big_tile - 1) / big_tile;
  const int64_t mid_tile = (int64_t)kMidBS * 2 * RM;
  const int64_t mid_tpp = (maxL + mid_tile - 1) / mid_tile;
  if constexpr ((!FIN || IPLS_HALF_ROUND) && (START != kAccum || (IPLS_HALF_ACCUM && !FIN))) {
    const int64_t half_tile = (int64_t)kHalfBS * 2 * kHalfR;
    const int64_t half_tpp = (maxL + half_tile - 1) / half_tile;
    if (use_half(maxL, n_parts, half_tile)) {
      const bool partial = half_tpp > 1 && maxL % half_tile != 0;
      const dim3 grid((unsigned)(half_tpp * n_parts));
#define HALF(MAP)                                                                                         \
      do {                                                                                                \
        if constexpr (FIN)                                                                                \
          hipLaunchKernelGGL((k_round<BE_IN, START, kBigG, kHalfR, MAP, kHalfBS, 0>), grid, dim3(kHalfBS), \
                             0, st, bufs, parts, k, (int)half_tpp, n_parts, secure, cnts);                \
        else                                                                                              \
          hipLaunchKernelGGL((k_reduce<BE_IN, BE_OUT, START, kBigG, kHalfR, true, MAP, kHalfBS>), grid,   \
                             dim3(kHalfBS), 0, st, bufs, parts, k, (int)half_tpp, n_parts);               \
      } while (0)
      if (partial) HALF(3);
      else HALF(kBigMap);
#undef HALF
      return launch_info(KER, IPLS_SHAPE_HALF, kHalfBS, kHalfR, 0, partial ? 3 : kBigMap, grid.x, BE_IN, BE_OUT,
                         START);
    }
  }
  if (fill(big_tpp * n_parts)) {
    // partial last tiles are scheduled first (map 3, ipls_kernels.hpp map_block)
    const bool partial = big_tpp > 1 && maxL % big_tile != 0;
    const int map = partial ? 3 : big_map<BE_IN>(big_tpp * n_parts);
    const dim3 grid((unsigned)grid_blocks(map, big_tpp * n_parts));
#define BIG(MAP)                                                                                          \
    do {                                                                                                  \
      if constexpr (FIN)                                                                                  \
        hipLaunchKernelGGL((k_round<BE_IN, START, kBigG, R, MAP, kBigBS, big_seqf<BE_IN, START>()>), grid, \
                           dim3(kBigBS), 0, st, bufs, parts, k, (int)big_tpp, n_parts, secure, cnts);     \
      else                                                                                                \
        hipLaunchKernelGGL((k_reduce<BE_IN, BE_OUT, START, kBigG, R, true, MAP, kBigBS,                   \
                                     big_seqf<BE_IN, START>()>),                                          \
                           grid, dim3(kBigBS), 0, st, bufs, parts, k, (int)big_tpp, n_parts);             \
    } while (0)
    if (map == 3) BIG(3);
    else if (map == 2) BIG(2);
    else BIG(kBigMap);
#undef BIG
    return launch_info(KER, IPLS_SHAPE_BIG, kBigBS, R, big_seqf<BE_IN, START>(), map, grid.x, BE_IN, BE_OUT, START);
  } else if (fill(mid_tpp * n_parts)) {
    const dim3 grid((unsigned)grid_blocks(kBigMap, mid_tpp * n_parts));
    const bool partial = mid_tpp > 1 && maxL % mid_tile != 0;
#define MID(MAP)                                                                                          \
    do {                                                                                                  \
      if constexpr (FIN)                                                                                  \
        hipLaunchKernelGGL((k_round<BE_IN, START, kBigG, RM, MAP, kMidBS, mid_seqf<BE_IN, START>()>), grid, \
                           dim3(kMidBS), 0, st, bufs, parts, k, (int)mid_tpp, n_parts, secure, cnts);     \
      else                                                                                                \
        hipLaunchKernelGGL((k_reduce<BE_IN, BE_OUT, START, kBigG, RM, true, MAP, kMidBS,                  \
                                     mid_seqf<BE_IN, START>()>),                                          \
                           grid, dim3(kMidBS), 0, st, bufs, parts, k, (int)mid_tpp, n_parts);             \
    } while (0)
    if (partial) MID(3);
    else MID(kBigMap);
#undef MID
    return launch_info(KER, IPLS_SHAPE_MID, kMidBS, RM, mid_seqf<BE_IN, START>(), partial ? 3 : kBigMap, grid.x,
                       BE_IN, BE_OUT, START);
  } else {
    const int64_t tile = (int64_t)kBlock * 2 * kSmallR;
    const int64_t tpp = (maxL + tile - 1) / tile;
    const dim3 grid((unsigned)grid_blocks(kSmallMap, tpp * n_parts));
    if constexpr (FIN)
      hipLaunchKernelGGL((k_round<BE_IN, START, kSmallG, kSmallR, kSmallMap, kBlock>), grid, dim3(kBlock), 0, st,
                         bufs, parts, k, (int)tpp, n_parts, secure, cnts);
    else
      hipLaunchKernelGGL((k_reduce<BE_IN, BE_OUT, START, kSmallG, kSmallR, true, kSmallMap>), grid, dim3(kBlock), 0,
                         st, bufs, parts, k, (int)tpp, n_parts);
    return launch_info(KER, IPLS_SHAPE_SMALL, kBlock, kSmallR, 0, kSmallMap, grid.x, BE_IN, BE_OUT, START);
  }
}

ipls_launch_info launch_reduce(bool be_in, bool be_out, int start, int64_t maxL, int n_parts, hipStream_t st,
                               const unsigned long long* const* bufs, const PartDesc* parts, int k) {
#define LV(BI, BO)                                                                                         \
  do {                                                                                                     \
    if (start == kZero) return launch_reduce_v<BI, BO, kZero>(maxL, n_parts, st, bufs, parts, k);          \
    else if (start == kFirst) return launch_reduce_v<BI, BO, kFirst>(maxL, n_parts, st, bufs, parts, k);   \
    else return launch_reduce_v<BI, BO, kAccum>(maxL, n_parts, st, bufs, parts, k);                        \
  } while (0)
  if (be_in) { if (be_out) LV(true, true); else LV(true, false); }
  else { if (be_out) LV(false, true); else LV(false, false); }
#undef LV
}

// fused round: native-double Weights out, ZERO or ACCUM start (AGG is never
// FIRST-started).  A one-block pre-pass folds each partition's count slot
// (k + 2 scalar loads per partition) so that the wide kernel reads one value
// per block instead of a k-long chain of dependent loads.
ipls_launch_info launch_reduce_fin(bool be_in, int start, int secure, int64_t maxL, int n_parts, hipStream_t st,
                                   const unsigned long long* const* bufs, const PartDesc* parts, int k,
                                   double* cnts) {
#define FIN(BI, ST)                                                                                   \
  do {                                                                                                \
    hipLaunchKernelGGL((k_round_counts<BI, ST>), dim3(n_parts), dim3(64), 0, st,                     \
                       bufs, parts, k, n_parts, cnts);                                                 \
    return launch_reduce_v<BI, false, ST, true>(maxL, n_parts, st, bufs, parts, k, secure, cnts);    \
  } while (0)
  if (be_in) { if (start == kZero) FIN(true, kZero); else FIN(true, kAccum); }
  else { if (start == kZero) FIN(false, kZero); else FIN(false, kAccum); }
#undef FIN
}

void launch_reduce_scalar(bool be_in, bool be_out, int start, dim3 grid, hipStream_t st,
                          const unsigned long long* const* bufs, const PartDesc* parts, int k, int tpp,
                          int64_t tile) {
#define RS(BI, BO, ST) hipLaunchKernelGGL((k_reduce_scalar<BI, BO, ST>), grid, dim3(kBlock), 0, st, bufs, parts, k, tpp, tile)
#define RS2(BI, BO) do { if (start == kZero) RS(BI, BO, kZero); else if (start == kFirst) RS(BI, BO, kFirst); else RS(BI, BO, kAccum); } while (0)
  if (be_in) { if (be_out) RS2(true, true); else RS2(true, false); }
  else { if (be_out) RS2(false, true); else RS2(false, false); }
#undef RS2
#undef RS
}

// Core of accumulate / reduce_batch: all pointers device-resident.  The
// destination is the handle's `target` accumulators, or -- when ext_dst is
// given -- one caller buffer per partition (doubles or, be_out, BE bytes).
// fused round (fin != nullptr): fold into AGG's values and write
// W = fold + REP to Weights, plus the averages at fin->avg (if set); AGG and
// REP end logically zero.  Callers guarantee 16-B aligned buckets.
struct FinOut {
  unsigned long long* avg;   // averages of p_first.. at flat_off[p] - flat_off[p_first], or null
};

// host_src: the bucket is pinned host memory read over PCIe (zero copy); the
// single-bucket fold then runs on 128 workgroups, which measured 1-2.5 GB/s
// above 256..4096 (tools/h2d_bench.hip, profiles/r01/h2d_bench_fold1.txt).
int reduce_dev(ipls_dev* h, int p_first, int n_parts, const void* const* bufs, int k, bool be_in,
               int start_mode, int target, void* const* ext_dst = nullptr, bool be_out = false,
               const FinOut* fin = nullptr, bool host_src = false, const int64_t* lens = nullptr) {
  // lens: lengths of caller destinations that are not this engine's
  // partitions (ext_dst only, e.g. a replica slot's partial sums)
  auto len_of = [&](int q) -> int64_t { return lens ? lens[q] : h->len[p_first + q]; };
  auto dst_of = [&](int q) -> unsigned long long* {
    if (fin) return (unsigned long long*)(h->arena + h->w_off[p_first + q]);
    return ext_dst ? (unsigned long long*)ext_dst[q]
                   : (unsigned long long*)(h->arena + target_off(h, p_first + q, target));
  };
  if (k <= 0 && !fin) {
    if (start_mode == IPLS_START_ZERO) {
      for (int q = 0; q < n_parts; ++q) {
        uint8_t* f = ext_dst ? nullptr : zero_flag(h, p_first + q, target);
        if (f) *f = 1;
        else HIP_TRY(h, hipMemsetAsync(dst_of(q), 0, (size_t)len_of(q) * 8, h->stream));
      }
    }
    return IPLS_OK;  // ACCUM / FIRST with no bucket: nothing to fold
  }
  // Resolve start mode per the logically-zero flags: an ACCUM into a +0.0
  // accumulator is exactly a ZERO-start fold.
  int start = start_mode;
  if (start_mode == IPLS_START_ACCUM && !ext_dst) {
    int nz = 0;
    for (int q = 0; q < n_parts; ++q) {
      uint8_t* f = zero_flag(h, p_first + q, target);
      nz += (f && *f) ? 1 : 0;
    }
    if (nz == n_parts) start = IPLS_START_ZERO;
    else if (nz) {
      for (int q = 0; q < n_parts; ++q) {
        int rc = materialize(h, p_first + q, target);
        if (rc) return rc;
      }
    }
  }
  // one bucket into one partition (every per-arrival fold): pointers go as
  // kernel arguments, no table upload
  if (!fin && n_parts == 1 && k == 1 && bufs[0]) {
    unsigned long long* d0 = dst_of(0);
    const int64_t L = len_of(0);
    if (d0 && !((uintptr_t)bufs[0] & 15) && !((uintptr_t)d0 & 15) && L > 0) {
      const auto* s0 = (const unsigned long long*)bufs[0];
      const unsigned blocks =
          std::max(1u, std::min<unsigned>(blocks_for((L >> 1), kBlock * 4), host_src ? 128u : 4096u));
#define F1(BI, BO, ST) hipLaunchKernelGGL((k_fold1<BI, BO, ST>), dim3(blocks), dim3(kBlock), 0, h->stream, d0, s0, L)
#define F1S(BI, BO) do { if (start == kZero) F1(BI, BO, kZero); else if (start == kFirst) F1(BI, BO, kFirst); else F1(BI, BO, kAccum); } while (0)
      if (be_in) { if (be_out) F1S(true, true); else F1S(true, false); }
      else { if (be_out) F1S(false, true); else F1S(false, false); }
#undef F1S
#undef F1
      HIP_TRY(h, hipGetLastError());
      h->last_launch = launch_info(IPLS_KERNEL_FOLD1, 0, kBlock, 4, 0, 0, blocks, be_in, be_out, kstart(start));
      if (!ext_dst)
        if (uint8_t* f = zero_flag(h, p_first, target)) *f = 0;
      return IPLS_OK;
    }
  }
  bool aligned16 = true;
  int64_t maxL = 0;
  for (int q = 0; q < n_parts; ++q) maxL = std::max(maxL, len_of(q));
  for (int64_t i = 0; i < (int64_t)n_parts * k; ++i) {
    if (!bufs[i]) return fail(h, IPLS_E_INVAL, "bucket pointer %lld is NULL", (long long)i);
    uintptr_t a = (uintptr_t)bufs[i];
    if (a & 7) return fail(h, IPLS_E_INVAL, "bucket %lld not 8-byte aligned", (long long)i);
    if (a & 15) aligned16 = false;
  }
  // table = [PartDesc x n_parts][ptr x n_parts*k]
  const size_t desc_bytes = sizeof(PartDesc) * n_parts;
  const size_t bytes = desc_bytes + sizeof(void*) * (size_t)n_parts * k;
  std::vector<unsigned char> tbl(bytes);
  PartDesc* pd = (PartDesc*)tbl.data();
  for (int q = 0; q < n_parts; ++q) {
    const int p = p_first + q;
    pd[q].len = len_of(q);
    pd[q].dst = dst_of(q);
    pd[q].init = pd[q].dst;
    pd[q].rep = nullptr;
    pd[q].avg = nullptr;
    if (fin) {
      pd[q].init = (const unsigned long long*)(h->arena + h->agg_off[p]);
      if (!h->rep_zero[p]) pd[q].rep = (const unsigned long long*)(h->arena + h->rep_off[p]);
      if (fin->avg) pd[q].avg = fin->avg + (h->flat_off[p] - h->flat_off[p_first]);
    }
    if (!pd[q].dst) return fail(h, IPLS_E_INVAL, "destination %d is NULL", q);
    if ((uintptr_t)pd[q].dst & 7) return fail(h, IPLS_E_INVAL, "destination %d not 8-byte aligned", q);
    if ((uintptr_t)pd[q].dst & 15) aligned16 = false;
  }
  if (k > 0) std::memcpy(tbl.data() + desc_bytes, bufs, sizeof(void*) * (size_t)n_parts * k);
  void* dtab = nullptr;
  int rc = upload_table(h, tbl.data(), bytes, &dtab);
  if (rc) return rc;
  const PartDesc* dparts = (const PartDesc*)dtab;
  auto dbufs = (const unsigned long long* const*)((char*)dtab + desc_bytes);
  if (fin) {
    if (!aligned16) return fail(h, IPLS_E_INVAL, "fused round needs 16-B aligned buckets");
    h->last_launch = launch_reduce_fin(be_in, start, h->secure, maxL, n_parts, h->stream, dbufs, dparts, k, h->d_cnt);
    HIP_TRY(h, hipGetLastError());
    for (int q = p_first; q < p_first + n_parts; ++q) h->agg_zero[q] = h->rep_zero[q] = 1;
    return IPLS_OK;
  }
  if (aligned16) {
    h->last_launch = launch_reduce(be_in, be_out, start, maxL, n_parts, h->stream, dbufs, dparts, k);
  } else {
    const int64_t tile = (int64_t)kBlock * 8;
    const int tpp = (int)((maxL + tile - 1) / tile);
    launch_reduce_scalar(be_in, be_out, start, dim3((unsigned)tpp * n_parts), h->stream, dbufs, dparts, k, tpp,
                         tile);
    h->last_launch = launch_info(IPLS_KERNEL_REDUCE_SCALAR, 0, kBlock, 1, 0, 0, (int64_t)tpp * n_parts, be_in, be_out,
                                 kstart(start));
  }
  HIP_TRY(h, hipGetLastError());
  if (!ext_dst)
    for (int q = 0; q < n_parts; ++q) {
      uint8_t* f = zero_flag(h, p_first + q, target);
      if (f) *f = 0;
    }
  return IPLS_OK;
}

int partition_geometry(const ipls_agg_cfg* c, std::vector<int64_t>& len, std::vector<int64_t>& off,
                       int64_t& chunk, std::string& why) {
  const int P = c->n_partitions;
  len.resize(P);
  off.resize(P);
  if (c->model_size > 0) {
    chunk = ref_chunk(c->model_size, P);
    for (int i = 0; i < P; ++i) {
      // IPLS.java:1023-1028 / 1862-1872
      int64_t L = ((int64_t)(i + 1) * chunk > c->model_size) ? c->model_size - (int64_t)i * chunk + 1
                                                             : chunk + 1;
      if (L < 1) {
        // L < 0: new double[L] throws NegativeArraySizeException (IPLS.java:1863);
        // L == 0: the count-slot store overruns the array (IPLS.java:1894, 1033).
        char b[160];
        snprintf(b, sizeof b, "partition %d length %lld < 1 (%s)", i, (long long)L,
                 L < 0 ? "NegativeArraySizeException, IPLS.java:1863"
                       : "ArrayIndexOutOfBoundsException, IPLS.java:1894");
        why = b;
        return L < 0 ? IPLS_E_NEGSIZE : IPLS_E_RANGE;
      }
      len[i] = L;
      off[i] = (int64_t)i * chunk;
    }
  } else {
    if (c->bucket_len < 1) {
      why = "bucket_len must be >= 1 when model_size == 0";
      return IPLS_E_INVAL;
    }
    chunk = c->bucket_len - 1;
    for (int i = 0; i < P; ++i) {
      len[i] = c->bucket_len;
      off[i] = (int64_t)i * chunk;
    }
  }
  return IPLS_OK;
}

int host_decode_count(int kind, int64_t n, int64_t L, ipls_dev* h) {
  if (n < L) return fail(h, IPLS_E_RANGE, "bucket of %lld doubles shorter than partition length %lld", (long long)n, (long long)L);
  (void)kind;
  return IPLS_OK;
}

}  // namespace

// ===========================================================================
// Engine entry points (engine.hpp).  The handle-free ipls_* utilities further
// down keep the C linkage of their declarations in include/ipls_agg.h.
// ===========================================================================
const char* dev_last_error(const ipls_dev* h) {
  if (h) return h->err.c_str();
  return g_tls_err.c_str();
}

// The front's own failures land in the same per-thread message that
// ipls_agg_last_error(NULL) reads.
void dev_set_thread_error(const char* msg) { g_tls_err = msg ? msg : ""; }

namespace {
thread_local int t_dev = -1;   // this thread's current device inside a C-ABI call, -1 = unknown
}
hipError_t dev_use(int device) {
  if (t_dev == device) return hipSuccess;
  const hipError_t e = hipSetDevice(device);
  t_dev = e == hipSuccess ? device : -1;
  return e;
}
void dev_track(int device) { t_dev = device; }
int dev_tracked() { return t_dev; }

int dev_geometry(const ipls_agg_cfg* cfg, std::vector<int64_t>& len, std::vector<int64_t>& off, int64_t& chunk,
                 std::string& why) {
  return partition_geometry(cfg, len, off, chunk, why);
}

// One engine for the partitions [p_lo, p_hi) of the handle's geometry on
// `device` (the front has validated cfg and the device ordinal).  Partition
// q of the engine is partition p_lo + q of the handle; flat offsets stay the
// handle's (flat model coordinates), flat_base is the first one.
int dev_open(const ipls_agg_cfg* cfg, int device, int p_lo, int p_hi, ipls_dev** out) {
  if (!cfg || !out || p_lo < 0 || p_hi < p_lo || p_hi > cfg->n_partitions)
    return fail(nullptr, IPLS_E_INVAL, "bad engine range");
  *out = nullptr;
  ipls_dev* h = new (std::nothrow) ipls_dev();
  if (!h) return fail(nullptr, IPLS_E_NOMEM, "host allocation failed");
  std::string why;
  std::vector<int64_t> glen, goff;
  int rc = partition_geometry(cfg, glen, goff, h->chunk, why);
  if (rc) {
    delete h;
    return fail(nullptr, rc, "%s", why.c_str());
  }
  h->len.assign(glen.begin() + p_lo, glen.begin() + p_hi);
  h->flat_off.assign(goff.begin() + p_lo, goff.begin() + p_hi);
  h->p_lo = p_lo;
  // an empty engine (p_hi == p_lo) owns no partition: a replica slot only
  h->flat_base = p_hi > p_lo ? h->flat_off[0] : 0;
  h->P = p_hi - p_lo;
  h->device = device;
  h->model_size = cfg->model_size;
  h->secure = cfg->secure;
  h->agg_off.resize(h->P);
  h->rep_off.resize(h->P);
  h->w_off.resize(h->P);
  h->fut_off.resize(h->P);
  h->agg_zero.assign(h->P, 1);
  h->rep_zero.assign(h->P, 1);
  h->fut_zero.assign(h->P, 1);
  int64_t cur = 0;
  for (int p = 0; p < h->P; ++p) {
    h->max_len = std::max(h->max_len, h->len[p]);
    h->flat_total = std::max(h->flat_total, h->flat_off[p] + h->len[p] - 1);
    h->agg_off[p] = cur; cur = align_up(cur + h->len[p], kAlignElems);
    h->rep_off[p] = cur; cur = align_up(cur + h->len[p], kAlignElems);
    h->w_off[p] = cur;   cur = align_up(cur + h->len[p], kAlignElems);
    h->fut_off[p] = cur; cur = align_up(cur + h->len[p], kAlignElems);
  }
  h->arena_elems = cur;
  // new double[(int)_MODEL_SIZE/_PARTITIONS + 2] (Updater.java:162)
  h->gbuf_len = h->model_size > 0 ? (int64_t)((int32_t)h->model_size / cfg->n_partitions) + 2 : cfg->bucket_len;
  auto cleanup = [&](int code) {
    (void)hipGetLastError();   // the failed call's error must not reach a later launch check
    dev_close(h);
    return code;
  };
  if (dev_use(h->device) != hipSuccess) return cleanup(fail(nullptr, IPLS_E_DEVICE, "dev_use(%d) failed", h->device));
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail(nullptr, IPLS_E_DEVICE, "hipStreamCreate failed"));
  if (h->arena_elems > 0 && hipMalloc(&h->arena, (size_t)h->arena_elems * 8) != hipSuccess) {
    (void)hipGetLastError();   // not sticky: the next launch check must not see it
    h->arena = nullptr;
    return cleanup(fail(nullptr, IPLS_E_NOMEM, "hipMalloc of %lld-byte arena failed", (long long)h->arena_elems * 8));
  }
  if (hipMalloc(&h->d_sum, 64) != hipSuccess) return cleanup(fail(nullptr, IPLS_E_NOMEM, "hipMalloc failed"));
  if (hipMalloc(&h->d_cnt, sizeof(double) * std::max(1, h->P)) != hipSuccess)
    return cleanup(fail(nullptr, IPLS_E_NOMEM, "hipMalloc failed"));
  // InitializeWeights(): new double[] -> all zero (IPLS.java:1860-1878).
  if ((h->arena && hipMemsetAsync(h->arena, 0, (size_t)h->arena_elems * 8, h->stream) != hipSuccess) ||
      hipStreamSynchronize(h->stream) != hipSuccess)
    return cleanup(fail(nullptr, IPLS_E_DEVICE, "arena clear failed"));
  *out = h;
  return IPLS_OK;
}

int dev_close(ipls_dev* h) {
  if (!h) return IPLS_OK;
  dev_use(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  for (auto& s : h->ring) {
    if (s.host) hipHostFree(s.host);
    if (s.ev) hipEventDestroy(s.ev);
  }
  for (ipls_stage* st : h->stage_all) {
    for (hipStream_t cs : st->copy)
      if (cs) {
        hipStreamSynchronize(cs);
        hipStreamDestroy(cs);
      }
    for (auto& s : st->slot) {
      if (s.host) hipHostFree(s.host);
      if (s.ev) hipEventDestroy(s.ev);
    }
    if (st->d) hipFree(st->d);
    for (hipEvent_t e : {st->landed[0], st->landed[1], st->ready, st->free_ev})
      if (e) hipEventDestroy(e);
    delete st;
  }
  if (h->copy_ev) hipEventDestroy(h->copy_ev);
  for (hipStream_t cs : h->copy_stream)
    if (cs) {
      hipStreamSynchronize(cs);
      hipStreamDestroy(cs);
    }
  for (auto& sl : h->stage) {
    if (sl.d) hipFree(sl.d);
    if (sl.free_ev) hipEventDestroy(sl.free_ev);
  }
  if (h->ingest_ev) hipEventDestroy(h->ingest_ev);
  for (hipEvent_t e : h->msg_ev) hipEventDestroy(e);
  for (auto& b : h->batches) hipEventDestroy(b.ev);
  for (hipEvent_t e : h->ev_free) hipEventDestroy(e);
  for (void* d : h->d_table)
    if (d) hipFree(d);
  if (h->d_scratch) hipFree(h->d_scratch);
  if (h->d_sum) hipFree(h->d_sum);
  if (h->d_cnt) hipFree(h->d_cnt);
  if (h->d_gbuf) hipFree(h->d_gbuf);
  if (h->d_merge) hipFree(h->d_merge);
  for (auto& kv : h->other)
    if (kv.second.d) hipFree(kv.second.d);
  if (h->arena) hipFree(h->arena);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return IPLS_OK;
}

void* dev_stream(ipls_dev* h) { return h ? (void*)h->stream : nullptr; }

// sync and wait hold the handle's lock only to flush and to book-keep: the
// host waits with it released, so the Updater and daemon threads (or any
// other caller) keep queueing folds meanwhile.
int dev_sync(ipls_dev* h) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  std::unique_lock<std::mutex> lk(h->mu);
  if (int rc = flush_pending(h)) return rc;
  lk.unlock();
  const hipError_t e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    lk.lock();
    return fail(h, IPLS_E_DEVICE, "hipStreamSynchronize failed: %s", hipGetErrorString(e));
  }
  return IPLS_OK;
}

int dev_wait(ipls_dev* h, uint64_t ticket) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  std::unique_lock<std::mutex> lk(h->mu);
  if (ticket >= h->ticket_next) return fail(h, IPLS_E_INVAL, "ticket %llu was never issued", (unsigned long long)ticket);
  if (ticket <= h->ticket_done) return IPLS_OK;
  if (ticket > h->launched_upto)
    if (int rc = flush_pending(h)) return rc;
  // the first launch group that covers `ticket` (groups complete in order)
  hipEvent_t ev = nullptr;
  uint64_t covered = 0;
  for (const auto& b : h->batches)
    if (b.max_ticket >= ticket) {
      ev = b.ev;
      covered = b.max_ticket;
      break;
    }
  if (!ev) return IPLS_OK;   // already retired by another waiter
  lk.unlock();
  // If another thread retires and re-records this event meanwhile, the wait
  // only gets longer: the re-recorded work was queued after ours.
  const hipError_t e = hipEventSynchronize(ev);
  lk.lock();
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(h, IPLS_E_DEVICE, "hipEventSynchronize failed: %s", hipGetErrorString(e));
  }
  while (!h->batches.empty() && h->batches.front().max_ticket <= covered) {
    h->ev_free.push_back(h->batches.front().ev);
    h->batches.pop_front();
  }
  h->ticket_done = std::max(h->ticket_done, covered);
  return IPLS_OK;
}

int dev_flush(ipls_dev* h) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);   // launches the queued folds; does not wait for them
  return IPLS_OK;
}

int dev_set_coalesce(ipls_dev* h, int max_group) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  h->coalesce = std::max(1, max_group);
  return IPLS_OK;
}

namespace {

// Close the launches queued since the last batch: tickets up to ticket_next-1
// complete at the event recorded now.
int end_batch(ipls_dev* h) {
  hipEvent_t ev;
  if (!h->ev_free.empty()) {
    ev = h->ev_free.back();
    h->ev_free.pop_back();
  } else {
    HIP_TRY(h, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  }
  HIP_TRY(h, hipEventRecord(ev, h->stream));
  h->batches.push_back({h->ticket_next - 1, ev});
  h->launched_upto = h->ticket_next - 1;
  while ((int)h->batches.size() > ipls_dev::kMaxBatches) {   // bound the events in flight
    const ipls_dev::Batch b = h->batches.front();
    HIP_TRY(h, hipEventSynchronize(b.ev));
    h->batches.pop_front();
    h->ev_free.push_back(b.ev);
    h->ticket_done = std::max(h->ticket_done, b.max_ticket);
  }
  return IPLS_OK;
}

// Fold every queued device arrival: runs of consecutive partitions of one
// target with the same queue length and byte order go as one launch (the
// batch kernel's table is [partition][peer]).
int flush_pending(ipls_dev* h) {
  if (h->pend_keys.empty()) return IPLS_OK;
  HIP_TRY(h, dev_use(h->device));
  int rc = IPLS_OK;
  std::vector<int>& keys = h->pend_keys;
  std::sort(keys.begin(), keys.end());   // (target, p) ascending
  std::vector<const void*> tab;
  for (size_t i = 0; i < keys.size() && !rc;) {
    const int key = keys[i], target = key / h->P, p0 = key % h->P;
    const ipls_dev::Pending& q0 = h->pend[key];
    const size_t k = q0.bufs.size();
    size_t j = i + 1;
    int n = 1;
    while (j < keys.size() && keys[j] == key + n && keys[j] / h->P == target && h->pend[keys[j]].bufs.size() == k &&
           h->pend[keys[j]].be == q0.be) {
      ++n;
      ++j;
    }
    tab.clear();
    for (size_t t = i; t < j; ++t) tab.insert(tab.end(), h->pend[keys[t]].bufs.begin(), h->pend[keys[t]].bufs.end());
    rc = reduce_dev(h, p0, n, tab.data(), (int)k, q0.be, IPLS_START_ACCUM, target);
    i = j;
  }
  for (int key : keys) h->pend[key].bufs.clear();   // keeps the capacity
  keys.clear();
  h->pending_n = 0;
  if (rc) return rc;
  return end_batch(h);
}

}  // namespace

int dev_reduce_batch(ipls_dev* h, int p_first, int n_parts, const void* const* bufs, int k,
                          int src_kind, int start_mode, int target) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (n_parts <= 0 || p_first < 0 || p_first + n_parts > h->P)
    return fail(h, IPLS_E_RANGE, "partitions [%d,%d) out of range [0,%d)", p_first, p_first + n_parts, h->P);
  if (src_kind != IPLS_DEV_F64 && src_kind != IPLS_DEV_BE)
    return fail(h, IPLS_E_INVAL, "reduce_batch takes device buckets (DEV_F64/DEV_BE)");
  if (start_mode < IPLS_START_ACCUM || start_mode > IPLS_START_FIRST) return fail(h, IPLS_E_INVAL, "bad start mode");
  if (target_off(h, 0, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  if (k < 0 || (k > 0 && !bufs)) return fail(h, IPLS_E_INVAL, "bad bucket list");
  HIP_TRY(h, dev_use(h->device));
  return reduce_dev(h, p_first, n_parts, bufs, k, src_kind == IPLS_DEV_BE, start_mode, target);
}

int dev_accumulate(ipls_dev* h, int p, int target, const void* src, int64_t n, int src_kind) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  if (target_off(h, p, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  if (!src) return IPLS_OK;  // Gradient == null: the Updater loops do nothing (Updater.java:115)
  HIP_TRY(h, dev_use(h->device));
  const int64_t L = h->len[p];
  const void* dptr = nullptr;
  bool be = false, staged = false;
  switch (src_kind) {
    case IPLS_DEV_F64:
    case IPLS_DEV_BE:
      if (int rc = host_decode_count(src_kind, n, L, h)) return rc;
      dptr = src;
      be = src_kind == IPLS_DEV_BE;
      break;
    case IPLS_HOST_F64:
    case IPLS_HOST_BE: {
      if (int rc = host_decode_count(src_kind, n, L, h)) return rc;
      be = src_kind == IPLS_HOST_BE;
      void* alias = nullptr;
      if (((uintptr_t)src & 7) == 0 && (size_t)L * 8 >= (1u << 16) && is_pinned_host(src, &alias) && alias) {
        // Zero copy: the fold kernel reads the pinned bucket over PCIe (no
        // staging copy, no second pass).  The call returns once the kernel
        // is done with the caller's bytes.
        const void* bl[1] = {alias};
        if (int rc = reduce_dev(h, p, 1, bl, 1, be, IPLS_START_ACCUM, target, nullptr, false, nullptr, true))
          return rc;
        HIP_TRY(h, hipStreamSynchronize(h->stream));
        return IPLS_OK;
      }
      if (int rc = stage_bucket(h, src, (size_t)L * 8, &dptr)) return rc;
      staged = true;
      break;
    }
    case IPLS_HOST_FRAME: {
      int16_t pid;
      int32_t a, b;
      int64_t poff, ooff;
      int64_t nd = ipls_frame_parse((const uint8_t*)src, n, &pid, &a, &b, &poff, &ooff);
      if (nd < 0) return fail(h, IPLS_E_FORMAT, "malformed frame (BufferUnderflowException)");
      if (nd == 0) return IPLS_OK;  // arr_len == 0 -> Gradients = null (MyIPFSClass.java:1449-1451)
      if (int rc = host_decode_count(src_kind, nd, L, h)) return rc;
      // The payload starts at byte 14 (unaligned); staging realigns it.
      if (int rc = stage_bucket(h, (const char*)src + poff, (size_t)L * 8, &dptr)) return rc;
      staged = true;
      be = true;
      break;
    }
    case IPLS_HOST_PAIR: {
      // Download_Partial_Updates(hash).getValue1() -> queue -> _Update (Download_Scheduler.java:324)
      int32_t workers;
      int64_t poff;
      const char* why = nullptr;
      const int64_t nd = javaser::parse_pair((const uint8_t*)src, n, &workers, &poff, &why);
      if (nd < 0) return fail(h, IPLS_E_FORMAT, "partial update: %s (ObjectInputStream)", why ? why : "malformed");
      if (int rc = host_decode_count(src_kind, nd, L, h)) return rc;
      if (int rc = stage_bucket(h, (const char*)src + poff, (size_t)L * 8, &dptr)) return rc;
      staged = true;
      be = true;
      break;
    }
    default:
      return fail(h, IPLS_E_INVAL, "bad src_kind %d", src_kind);
  }
  const void* bl[1] = {dptr};
  if (int rc = reduce_dev(h, p, 1, bl, 1, be, IPLS_START_ACCUM, target)) return rc;
  return staged ? release_stage(h) : IPLS_OK;
}

int dev_accumulate_async(ipls_dev* h, int p, int target, const void* src, int64_t n, int src_kind,
                              uint64_t* ticket) {
  if (!h || !ticket) return fail(h, IPLS_E_INVAL, "null argument");
  if (src && (src_kind == IPLS_DEV_F64 || src_kind == IPLS_DEV_BE)) {
    // device bucket: queued, folded with the partition's other queued buckets
    std::lock_guard<std::mutex> lk(h->mu);
    if (int rc = check_part(h, p)) return rc;
    if (target_off(h, p, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
    if (n < h->len[p])
      return fail(h, IPLS_E_RANGE, "bucket of %lld doubles shorter than partition length %lld", (long long)n,
                  (long long)h->len[p]);
    if ((uintptr_t)src & 7) return fail(h, IPLS_E_INVAL, "device bucket not 8-byte aligned");
    const bool be = src_kind == IPLS_DEV_BE;
    // Weights and Weight_Address are one array (IPLS.java:1141): one queue
    const int qt = target == IPLS_TGT_WADDR ? IPLS_TGT_WEIGHTS : target;
    if (h->pend.empty()) h->pend.resize((size_t)5 * h->P);   // 5 targets (include/ipls_agg.h)
    ipls_dev::Pending& q = h->pend[(size_t)qt * h->P + p];
    if (!q.bufs.empty() && q.be != be)
      if (int rc = flush_pending(h)) return rc;
    if (q.bufs.empty()) h->pend_keys.push_back(qt * h->P + p);
    q.be = be;
    q.bufs.push_back(src);
    ++h->pending_n;
    *ticket = h->ticket_next++;
    // flush when the queues average `coalesce` buckets (arrivals spread over
    // partitions flush as one rectangular launch), or one queue holds twice that
    if ((int)q.bufs.size() >= 2 * h->coalesce || h->pending_n >= h->coalesce * (int)h->pend_keys.size())
      return flush_pending(h);
    return IPLS_OK;
  }
  void* alias = nullptr;
  const bool host = src_kind == IPLS_HOST_F64 || src_kind == IPLS_HOST_BE;
  if (!src || !host || ((uintptr_t)src & 15) || !is_pinned_host(src, &alias) || !alias) {
    // not a pinned host bucket: the synchronous path, already complete on return
    int rc = dev_accumulate(h, p, target, src, n, src_kind);
    std::lock_guard<std::mutex> lk(h->mu);
    *ticket = h->ticket_done;
    return rc;
  }
  IPLS_LOCK(h);   // earlier queued device buckets fold first
  if (int rc = check_part(h, p)) return rc;
  if (target_off(h, p, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  if (int rc = host_decode_count(src_kind, n, h->len[p], h)) return rc;
  HIP_TRY(h, dev_use(h->device));
  const void* bl[1] = {alias};   // zero copy: the kernel reads the pinned bucket over PCIe
  if (int rc = reduce_dev(h, p, 1, bl, 1, src_kind == IPLS_HOST_BE, IPLS_START_ACCUM, target, nullptr, false, nullptr,
                          true))
    return rc;
  *ticket = h->ticket_next++;
  return end_batch(h);
}

// One range of one arrival: src[0..n) folded into target[off..off+n) of
// partition p, zero copy from pinned host memory, asynchronous.  The JNI
// shim's heap-array natives copy a Java double[] into pinned staging chunk by
// chunk and fold each chunk as soon as it has landed, so the copy of the next
// chunk overlaps the fold of this one.  Whatever the split, every element of
// the bucket is added exactly once, in call order: the bits of the
// whole-bucket fold (Updater.java:115-117).
int dev_accumulate_range(ipls_dev* h, int p, int target, const void* src, int64_t off, int64_t n, int src_kind,
                         uint64_t* ticket) {
  if (!h || !ticket || !src) return fail(h, IPLS_E_INVAL, "null argument");
  IPLS_LOCK(h);   // earlier queued device buckets fold first
  if (int rc = check_part(h, p)) return rc;
  if (target_off(h, p, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  if (src_kind != IPLS_HOST_F64 && src_kind != IPLS_HOST_BE)
    return fail(h, IPLS_E_INVAL, "a ranged fold reads a pinned host bucket (HOST_F64 / HOST_BE), not kind %d", src_kind);
  const int64_t L = h->len[p];
  if (off < 0 || n < 0 || off > L || n > L - off)
    return fail(h, IPLS_E_RANGE, "range [%lld, %lld) outside partition %d of length %lld", (long long)off,
                (long long)(off + n), p, (long long)L);
  if ((off & 1) || ((uintptr_t)src & 15))
    return fail(h, IPLS_E_INVAL, "a ranged fold needs an even start and 16-B aligned bytes");
  void* alias = nullptr;
  if (!is_pinned_host(src, &alias) || !alias)
    return fail(h, IPLS_E_INVAL, "a ranged fold reads pinned host memory (ipls_host_alloc)");
  if (n == 0) {
    *ticket = h->ticket_done;
    return IPLS_OK;
  }
  HIP_TRY(h, dev_use(h->device));
  if (int rc = materialize(h, p, target)) return rc;   // a logically-zero target becomes real zeros first
  unsigned long long* d0 = (unsigned long long*)(h->arena + target_off(h, p, target)) + off;
  const auto* s0 = (const unsigned long long*)alias;
  const unsigned blocks = std::max(1u, std::min<unsigned>(blocks_for(n >> 1, kBlock * 4), 128u));
  const bool be = src_kind == IPLS_HOST_BE;
  if (be) hipLaunchKernelGGL((k_fold1<true, false, kAccum>), dim3(blocks), dim3(kBlock), 0, h->stream, d0, s0, n);
  else hipLaunchKernelGGL((k_fold1<false, false, kAccum>), dim3(blocks), dim3(kBlock), 0, h->stream, d0, s0, n);
  HIP_TRY(h, hipGetLastError());
  h->last_launch = launch_info(IPLS_KERNEL_FOLD1, 0, kBlock, 4, 0, 0, blocks, be, false, kstart(IPLS_START_ACCUM));
  *ticket = h->ticket_next++;
  return end_batch(h);
}

// One arrival produced by the caller chunk by chunk, as one call (Updater's
// whole-bucket fold under PeerData.mtx, Updater.java:72-149, 115-117).
// Chunk k is filled by source() into pinned slot k % 2 of a staging of this
// call's own and sent to its device buffer on the stage's copy stream while
// the source fills chunk k + 1 -- all with NO engine lock held, so a source
// that blocks (a socket recv) stalls only this call.  Once every chunk has
// landed, the lock is taken for the fold alone: the shard stream waits for
// the copies (an event, no host wait) and folds the whole bucket in one launch
// (24 B per element).  So the arrival takes effect, as one unit, when its last
// chunk has landed -- the reference's order: Middleware's Deserialize reads
// the whole stream before UpdateModel takes PeerData.mtx (Middleware.java:224,
// 246).  A source that stops leaves the target untouched.
int dev_accumulate_chunked(ipls_dev* h, int p, int target, int64_t n, int src_kind, int64_t chunk,
                           ipls_chunk_source source, void* ctx) {
  if (!h || !source) return fail_nl(h, IPLS_E_INVAL, "null argument");
  if (chunk < 2 || (chunk & 1))
    return fail_nl(h, IPLS_E_INVAL, "chunk of %lld values: even and >= 2", (long long)chunk);
  // geometry is fixed at open: validated without the lock (the target's
  // offset is not read here: promote_future swaps AGG/FUT storage under it)
  if (p < 0 || p >= h->P) return fail_nl(h, IPLS_E_RANGE, "partition %d out of range [0,%d)", p, h->P);
  if (target < IPLS_TGT_AGG || target > IPLS_TGT_FUTURE) return fail_nl(h, IPLS_E_INVAL, "bad target %d", target);
  if (src_kind != IPLS_HOST_F64 && src_kind != IPLS_HOST_BE)
    return fail_nl(h, IPLS_E_INVAL, "a chunked fold takes HOST_F64 or HOST_BE values, not kind %d", src_kind);
  const int64_t L = h->len[p];
  if (n < L)   // before any source call (Updater.java:115)
    return fail_nl(h, IPLS_E_RANGE, "bucket of %lld doubles shorter than partition length %lld", (long long)n,
                   (long long)L);
  HIP_TRY_NL(h, dev_use(h->device));
  const int64_t c = std::min(chunk, L);
  ipls_stage* st = nullptr;
  if (int rc = stage_acquire(h, (size_t)L * 8, (size_t)c * 8, &st)) return rc;
  unsigned long long* d_in = (unsigned long long*)st->d;
  int rc = IPLS_OK;
  auto try_hip = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && !rc) {
      (void)hipGetLastError();
      rc = fail_nl(h, IPLS_E_DEVICE, "%s failed: %s", what, hipGetErrorString(e));
    }
  };
  // the fold that last read the device buffer runs before these copies overwrite it
  for (int i = 0; i < st->n_copy && st->free_pending; ++i)
    try_hip(hipStreamWaitEvent(st->copy[i], st->free_ev, 0), "hipStreamWaitEvent");
  for (int64_t k = 0, off = 0; off < L && !rc; ++k, off += c) {
    PinnedSlot& sl = st->slot[k % st->n_slot];
    if ((rc = stage_slot_free(h, sl))) break;   // the copy of chunk k - n_slot still reads this slot
    const int64_t len = std::min(c, L - off);
    if (source(ctx, sl.host, off, len) != 0) {
      rc = fail_nl(h, IPLS_E_INVAL, "the chunk source stopped at offset %lld: nothing folded", (long long)off);
      break;
    }
    hipStream_t cs = st->copy[k % st->n_copy];
    try_hip(hipMemcpyAsync(d_in + off, sl.host, (size_t)len * 8, hipMemcpyHostToDevice, cs), "hipMemcpyAsync");
    try_hip(hipEventRecord(sl.ev, cs), "hipEventRecord");
    if (!rc) sl.pending = true;
  }
  for (int i = 0; i < st->n_copy && !rc; ++i) try_hip(hipEventRecord(st->landed[i], st->copy[i]), "hipEventRecord");
  if (rc) {
    // nothing folded; the copies already queued finish before the stage is reused
    for (int i = 0; i < st->n_copy; ++i) (void)hipStreamSynchronize(st->copy[i]);
    (void)hipGetLastError();
    for (auto& sl : st->slot) sl.pending = false;
    stage_release(h, st);
    return rc;
  }
  {
    std::lock_guard<std::mutex> lk(h->mu);
    rc = flush_pending(h);   // earlier queued device buckets fold first
    for (int i = 0; i < st->n_copy && !rc; ++i) {
      const hipError_t e = hipStreamWaitEvent(h->stream, st->landed[i], 0);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        rc = fail(h, IPLS_E_DEVICE, "hipStreamWaitEvent failed: %s", hipGetErrorString(e));
      }
    }
    const void* bl[1] = {d_in};
    if (!rc) rc = reduce_dev(h, p, 1, bl, 1, src_kind == IPLS_HOST_BE, IPLS_START_ACCUM, target);
    // whatever ran, nothing queued on the shard stream after this point reads `d`
    if (hipEventRecord(st->free_ev, h->stream) == hipSuccess) {
      st->free_pending = true;
    } else {
      (void)hipGetLastError();
      (void)hipStreamSynchronize(h->stream);
      st->free_pending = false;
    }
  }
  if (rc) {   // the shard stream may not have waited for the copies: drain them
    for (int i = 0; i < st->n_copy; ++i) (void)hipStreamSynchronize(st->copy[i]);
    (void)hipGetLastError();
  }
  stage_release(h, st);
  return rc;
}

// Hand n values of a stage's device snapshot (complete once st->ready fires)
// to the sink in chunks of c, with no engine lock held: chunk k + 1 crosses
// PCIe into one pinned slot on the stage's copy stream while sink() consumes
// chunk k from the other.  `base` is added to the offsets the sink sees.
// Releases the stage.
static int stage_deliver(ipls_dev* h, ipls_stage* st, int64_t n, int64_t c, int64_t base, ipls_chunk_sink sink, void* ctx,
                  const char* stopped_note) {
  const double* d = (const double*)st->d;
  int rc = IPLS_OK;
  auto try_hip = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && !rc) {
      (void)hipGetLastError();
      rc = fail_nl(h, IPLS_E_DEVICE, "%s failed: %s", what, hipGetErrorString(e));
    }
  };
  // a previous call's H2D may still read a slot (accumulate_chunked does not
  // wait for its copies on the host): the D2H into it waits for that copy
  for (auto& sl : st->slot)
    if (!rc) rc = stage_slot_free(h, sl);
  for (int i = 0; i < st->n_copy; ++i) try_hip(hipStreamWaitEvent(st->copy[i], st->ready, 0), "hipStreamWaitEvent");
  const int64_t K = n > 0 ? (n + c - 1) / c : 0;
  const int S = st->n_slot;
  int64_t issued = 0;
  auto issue = [&]() {   // the next chunk, into slot issued % S (its previous chunk's sink has returned)
    const int64_t k = issued++;
    PinnedSlot& sl = st->slot[k % S];
    const int64_t off = k * c, len = std::min(c, n - off);
    hipStream_t cs = st->copy[k % st->n_copy];
    try_hip(hipMemcpyAsync(sl.host, d + off, (size_t)len * 8, hipMemcpyDeviceToHost, cs), "hipMemcpyAsync");
    try_hip(hipEventRecord(sl.ev, cs), "hipEventRecord");
  };
  while (issued < K && issued < S && !rc) issue();   // the ring's first fill
  for (int64_t k = 0; k < K && !rc; ++k) {
    PinnedSlot& sl = st->slot[k % S];
    try_hip(hipEventSynchronize(sl.ev), "hipEventSynchronize");
    if (rc) break;
    const int64_t off = k * c, len = std::min(c, n - off);
    if (sink(ctx, (const double*)sl.host, base + off, len) != 0)
      rc = fail_nl(h, IPLS_E_INVAL, "the chunk sink stopped the transfer at offset %lld%s", (long long)(base + off),
                   stopped_note);
    else if (issued < K)
      issue();   // into the slot just consumed
  }
  // every copy of this call is done before the stage can be reused (on the
  // success path they already are: each chunk's event was waited for)
  if (rc) {
    for (int i = 0; i < st->n_copy; ++i) (void)hipStreamSynchronize(st->copy[i]);
    (void)hipGetLastError();
  }
  for (auto& sl : st->slot) sl.pending = false;
  stage_release(h, st);
  return rc;
}

// The reverse: target[off..off+n) of partition p into pinned host memory,
// native or big-endian (putDouble order, as update_file writes it,
// MyIPFSClass.java:105-116), asynchronous.  The JNI shim's byte[] outputs
// copy chunk k into the Java array while chunk k+1 is still in flight.
int dev_read_range(ipls_dev* h, int p, int target, void* dst, int64_t off, int64_t n, int dst_kind, uint64_t* ticket) {
  if (!h || !ticket || !dst) return fail(h, IPLS_E_INVAL, "null argument");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  if (target_off(h, p, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  if (dst_kind != IPLS_HOST_F64 && dst_kind != IPLS_HOST_BE)
    return fail(h, IPLS_E_INVAL, "a ranged read writes pinned host memory (HOST_F64 / HOST_BE), not kind %d", dst_kind);
  const int64_t L = h->len[p];
  if (off < 0 || n < 0 || off > L || n > L - off)
    return fail(h, IPLS_E_RANGE, "range [%lld, %lld) outside partition %d of length %lld", (long long)off,
                (long long)(off + n), p, (long long)L);
  void* alias = nullptr;
  if (!is_pinned_host(dst, &alias) || !alias)
    return fail(h, IPLS_E_INVAL, "a ranged read writes pinned host memory (ipls_host_alloc)");
  if (n == 0) {
    *ticket = h->ticket_done;
    return IPLS_OK;
  }
  HIP_TRY(h, dev_use(h->device));
  if (int rc = materialize(h, p, target)) return rc;
  const unsigned long long* src = (const unsigned long long*)(h->arena + target_off(h, p, target)) + off;
  if (dst_kind == IPLS_HOST_BE) {
    // byte-swapped into the same offsets of the device scratch, then copied
    if (int rc = ensure_scratch(h, (size_t)L * 8)) return rc;
    unsigned long long* sc = (unsigned long long*)h->d_scratch + off;
    launch_bswap(h->stream, src, sc, n);
    HIP_TRY(h, hipGetLastError());
    src = sc;
  }
  HIP_TRY(h, hipMemcpyAsync(dst, src, (size_t)n * 8, hipMemcpyDeviceToHost, h->stream));
  *ticket = h->ticket_next++;
  return end_batch(h);
}

// GetParameters(hash, Gradient_Buff) (MyIPFSClass.java:444-455) into the
// engine's Gradient_Buff (Updater.java:162, zeroed once, Updater.java:165-167):
// arr[i] = getDouble() for i < data.length/8; past arr.length it throws after
// the in-range stores (IPLS_E_RANGE, buffer already overwritten).  Entries
// beyond the file keep the previous request's values.  *zero_copy: the kernel
// reads the caller's pinned bytes (wait before returning to the caller).
static int gbuf_load(ipls_dev* h, const void* bytes, int64_t n_bytes, bool* zero_copy) {
  const int64_t G = h->gbuf_len;
  *zero_copy = false;
  if (!h->d_gbuf) {
    HIP_TRY(h, hipMalloc(&h->d_gbuf, (size_t)std::max<int64_t>(G, 1) * 8));
    HIP_TRY(h, hipMemsetAsync(h->d_gbuf, 0, (size_t)std::max<int64_t>(G, 1) * 8, h->stream));
  }
  const int64_t nd = n_bytes / 8;
  const int64_t nw = std::min(nd, G);
  if (nw > 0) {
    const void* dsrc = nullptr;
    void* alias = nullptr;
    if (((uintptr_t)bytes & 7) == 0 && (size_t)nw * 8 >= (1u << 16) && is_pinned_host(bytes, &alias) && alias) {
      dsrc = alias;
      *zero_copy = true;
    } else {
      // double-buffered like the per-arrival buckets (stage_bucket)
      if (int rc = stage_bucket(h, bytes, (size_t)nw * 8, &dsrc)) return rc;
    }
    launch_bswap(h->stream, (const unsigned long long*)dsrc, h->d_gbuf, nw);
    HIP_TRY(h, hipGetLastError());
    if (!*zero_copy)
      if (int rc = release_stage(h)) return rc;
  }
  if (nd > G) {
    if (*zero_copy) HIP_TRY(h, hipStreamSynchronize(h->stream));
    return fail(h, IPLS_E_RANGE, "GetParameters: %lld doubles > Gradient_Buff length %lld "
                "(ArrayIndexOutOfBoundsException, MyIPFSClass.java:451)", (long long)nd, (long long)G);
  }
  return IPLS_OK;
}

int dev_update_indirect(ipls_dev* h, int p, int target, const void* bytes, int64_t n_bytes) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  if (target_off(h, p, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  if (n_bytes < 0 || (n_bytes > 0 && !bytes)) return fail(h, IPLS_E_INVAL, "bad byte buffer");
  HIP_TRY(h, dev_use(h->device));
  const int64_t G = h->gbuf_len;
  bool zero_copy = false;
  if (int rc = gbuf_load(h, bytes, n_bytes, &zero_copy)) return rc;
  // _Update(Gradient_Buff, ...): target[p][i] += Gradient_Buff[i], i < L_p
  if (h->len[p] > G)
    return fail(h, IPLS_E_RANGE, "partition length %lld > Gradient_Buff length %lld", (long long)h->len[p],
                (long long)G);
  const void* bl[1] = {h->d_gbuf};
  if (int rc = reduce_dev(h, p, 1, bl, 1, false, IPLS_START_ACCUM, target)) return rc;
  if (zero_copy) HIP_TRY(h, hipStreamSynchronize(h->stream));
  return IPLS_OK;
}

// The Gradient_Buff load alone, for a request whose partition lives in
// another engine (the handle keeps ONE Gradient_Buff, as the reference has
// one Updater thread): *gbuf / *glen describe the device buffer afterwards;
// the caller orders the fold after this engine's stream.
int dev_gbuf_load(ipls_dev* h, const void* bytes, int64_t n_bytes, const void** gbuf, int64_t* glen) {
  if (!h || !gbuf || !glen) return fail(h, IPLS_E_INVAL, "null argument");
  IPLS_LOCK(h);
  if (n_bytes < 0 || (n_bytes > 0 && !bytes)) return fail(h, IPLS_E_INVAL, "bad byte buffer");
  HIP_TRY(h, dev_use(h->device));
  bool zero_copy = false;
  if (int rc = gbuf_load(h, bytes, n_bytes, &zero_copy)) return rc;
  if (zero_copy) HIP_TRY(h, hipStreamSynchronize(h->stream));
  *gbuf = h->d_gbuf;
  *glen = h->gbuf_len;
  return IPLS_OK;
}

int dev_reset(ipls_dev* h, int p) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (p == IPLS_ALL_PARTITIONS) {
    for (int q = 0; q < h->P; ++q) h->agg_zero[q] = h->rep_zero[q] = 1;
    return IPLS_OK;
  }
  if (int rc = check_part(h, p)) return rc;
  h->agg_zero[p] = h->rep_zero[p] = 1;
  return IPLS_OK;
}

int dev_promote_future(ipls_dev* h, const int32_t* parts, int n_parts) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (n_parts < 0 || (n_parts > 0 && !parts)) return fail(h, IPLS_E_INVAL, "bad partition list");
  for (int i = 0; i < n_parts; ++i)
    if (int rc = check_part(h, parts[i])) return rc;
  for (int i = 0; i < n_parts; ++i) {
    const int p = parts[i];
    // AGG[p][j] = FUTURE[p].get(j); FUTURE[p].set(j, 0.0)   (IPLS.java:1558-1561)
    std::swap(h->agg_off[p], h->fut_off[p]);
    h->agg_zero[p] = h->fut_zero[p];
    h->fut_zero[p] = 1;
  }
  return IPLS_OK;
}

int dev_device_ptr(ipls_dev* h, int p, int target, void** ptr) {
  if (!h || !ptr) return fail(h, IPLS_E_INVAL, "null argument");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  if (target_off(h, p, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  HIP_TRY(h, dev_use(h->device));
  if (int rc = materialize(h, p, target)) return rc;
  *ptr = h->arena + target_off(h, p, target);
  return IPLS_OK;
}

int dev_read(ipls_dev* h, int p, int target, void* dst, int64_t n, int dst_kind) {
  if (!h || !dst) return fail(h, IPLS_E_INVAL, "null argument");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  if (target_off(h, p, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  const int64_t L = h->len[p];
  if (n < L) return fail(h, IPLS_E_RANGE, "output of %lld < partition length %lld", (long long)n, (long long)L);
  HIP_TRY(h, dev_use(h->device));
  if (int rc = materialize(h, p, target)) return rc;
  const double* srcd = h->arena + target_off(h, p, target);
  switch (dst_kind) {
    case IPLS_HOST_F64:
      return d2h(h, dst, srcd, (size_t)L * 8);
    case IPLS_DEV_F64:
      HIP_TRY(h, hipMemcpyAsync(dst, srcd, (size_t)L * 8, hipMemcpyDeviceToDevice, h->stream));
      return IPLS_OK;
    case IPLS_DEV_BE:
      launch_bswap(h->stream, (const unsigned long long*)srcd, (unsigned long long*)dst, L);
      HIP_TRY(h, hipGetLastError());
      return IPLS_OK;
    case IPLS_HOST_BE: {
      if (int rc = ensure_scratch(h, (size_t)L * 8)) return rc;
      launch_bswap(h->stream, (const unsigned long long*)srcd, (unsigned long long*)h->d_scratch, L);
      HIP_TRY(h, hipGetLastError());
      return d2h(h, dst, h->d_scratch, (size_t)L * 8);
    }
    default:
      return fail(h, IPLS_E_INVAL, "bad dst_kind %d", dst_kind);
  }
}

int dev_checksum(ipls_dev* h, int p, int target, uint64_t* out) {
  if (!h || !out) return fail(h, IPLS_E_INVAL, "null argument");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  if (target_off(h, p, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  HIP_TRY(h, dev_use(h->device));
  if (int rc = materialize(h, p, target)) return rc;
  HIP_TRY(h, hipMemsetAsync(h->d_sum, 0, 8, h->stream));
  const int64_t L = h->len[p];
  hipLaunchKernelGGL(k_checksum<false>, dim3(std::max(1u, std::min<unsigned>(blocks_for(L, kBlock * 8), 2048))),
                     dim3(kBlock), 0, h->stream,
                     (const unsigned long long*)(h->arena + target_off(h, p, target)), L, h->d_sum);
  HIP_TRY(h, hipGetLastError());
  unsigned long long v = 0;
  if (int rc = d2h(h, &v, h->d_sum, 8)) return rc;
  *out = v;
  return IPLS_OK;
}

// AggregatePartition's W = AGG + REP for partitions [p0, p0+np) (IPLS.java:1256-1269).
static int finalize_range(ipls_dev* h, int p0, int np) {
  // AGG logically zero but present as an operand -> make it physical.
  bool rep_zero_all = true;
  for (int q = p0; q < p0 + np; ++q) {
    if (int rc = materialize(h, q, IPLS_TGT_AGG)) return rc;
    rep_zero_all = rep_zero_all && h->rep_zero[q];
  }
  if (!rep_zero_all)
    for (int q = p0; q < p0 + np; ++q)
      if (int rc = materialize(h, q, IPLS_TGT_REP)) return rc;
  std::vector<FinDesc> fd(np);
  int64_t maxL = 0;
  for (int q = 0; q < np; ++q) {
    fd[q] = FinDesc{h->len[p0 + q], h->agg_off[p0 + q], h->rep_off[p0 + q], h->w_off[p0 + q]};
    maxL = std::max(maxL, fd[q].len);
  }
  void* dtab = nullptr;
  if (int rc = upload_table(h, fd.data(), fd.size() * sizeof(FinDesc), &dtab)) return rc;
  const int64_t tile = kFinTile;
  const int tpp = (int)((maxL + tile - 1) / tile);
  // AGG/REP are left in place and flagged logically zero (IPLS.java:1268-1269
  // zeroes them; the next fold starts from +0.0 without reading them).
  if (rep_zero_all)
    hipLaunchKernelGGL((k_finalize<true, false>), dim3((unsigned)tpp * np), dim3(kBlock), 0, h->stream,
                       (const FinDesc*)dtab, h->arena, tpp);
  else
    hipLaunchKernelGGL((k_finalize<false, false>), dim3((unsigned)tpp * np), dim3(kBlock), 0, h->stream,
                       (const FinDesc*)dtab, h->arena, tpp);
  HIP_TRY(h, hipGetLastError());
  for (int q = p0; q < p0 + np; ++q) h->agg_zero[q] = h->rep_zero[q] = 1;
  return IPLS_OK;
}

// GetPartitions' divide (IPLS.java:1159-1174) of Weights[p0..p0+np) into d_out,
// partition p at flat_off[p] - flat_off[p0].
static int divide_range(ipls_dev* h, int p0, int np, unsigned long long* d_out, bool be) {
  std::vector<DivDesc> dd(np);
  int64_t maxn = 0;
  for (int q = 0; q < np; ++q) {
    const int p = p0 + q;
    dd[q] = DivDesc{h->len[p], h->w_off[p], h->flat_off[p] - h->flat_off[p0]};
    maxn = std::max(maxn, h->len[p] - 1);
  }
  if (maxn <= 0) return IPLS_OK;
  void* dtab = nullptr;
  if (int rc = upload_table(h, dd.data(), dd.size() * sizeof(DivDesc), &dtab)) return rc;
  const int64_t tile = kDivTile;
  const int tpp = (int)((maxn + tile - 1) / tile);
  const dim3 g((unsigned)tpp * np);
#define DIV(B, S) hipLaunchKernelGGL((k_divide<B, S>), g, dim3(kBlock), 0, h->stream, (const DivDesc*)dtab, (const double*)h->arena, d_out, tpp)
  if (be) { if (h->secure) DIV(true, true); else DIV(true, false); }
  else { if (h->secure) DIV(false, true); else DIV(false, false); }
#undef DIV
  HIP_TRY(h, hipGetLastError());
  return IPLS_OK;
}

int dev_finalize(ipls_dev* h, int p, void* sum_out, int sum_kind, double* avg_out) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  int p0 = p, np = 1;
  if (p == IPLS_ALL_PARTITIONS) {
    p0 = 0;
    np = h->P;
    if (sum_out || avg_out) return fail(h, IPLS_E_INVAL, "host outputs need a single partition");
  } else if (int rc = check_part(h, p)) {
    return rc;
  }
  // validate the outputs before anything is consumed: finalize_range flags
  // AGG/REP logically zero, so a rejected call must not get that far
  if (sum_out && sum_kind != IPLS_HOST_F64 && sum_kind != IPLS_HOST_BE)
    return fail(h, IPLS_E_INVAL, "sum_kind must be HOST_F64 or HOST_BE");
  HIP_TRY(h, dev_use(h->device));
  if (int rc = finalize_range(h, p0, np)) return rc;

  if (np == 1 && (sum_out || avg_out)) {
    const int64_t L = h->len[p0];
    const double* w = h->arena + h->w_off[p0];
    if (sum_out) {
      if (sum_kind == IPLS_HOST_F64) {
        if (int rc = d2h(h, sum_out, w, (size_t)L * 8)) return rc;
      } else if (sum_kind == IPLS_HOST_BE) {
        if (int rc = ensure_scratch(h, (size_t)L * 8)) return rc;
        launch_bswap(h->stream, (const unsigned long long*)w, (unsigned long long*)h->d_scratch, L);
        HIP_TRY(h, hipGetLastError());
        if (int rc = d2h(h, sum_out, h->d_scratch, (size_t)L * 8)) return rc;
      } else {
        return fail(h, IPLS_E_INVAL, "sum_kind must be HOST_F64 or HOST_BE");
      }
    }
    if (avg_out && L > 1) {
      if (int rc = ensure_scratch(h, (size_t)L * 8)) return rc;
      if (int rc = divide_range(h, p0, 1, (unsigned long long*)h->d_scratch, false)) return rc;
      if (int rc = d2h(h, avg_out, h->d_scratch, (size_t)(L - 1) * 8)) return rc;
    }
  }
  return IPLS_OK;
}

// AggregatePartition of one partition with the commit_update bytes (or the
// sum as doubles) handed to a sink chunk by chunk, as one call.  Under the
// engine lock: W = AGG + REP and a snapshot of W (or of its big-endian bytes)
// into this call's own staging -- one kernel or copy on the shard stream.
// The lock is then released and the snapshot goes to the sink through the
// pinned ring, chunks k + 1 .. k + 2 in flight while sink() copies chunk k.
// The bytes are the W of this call's AggregatePartition whatever another
// caller's set_weights / fold / finalize does meanwhile (the per-range reads
// of dev_read_range cannot promise that), and a slow sink (a socket send)
// holds nothing: the reference writes after Get_Partitions has returned
// (Middleware.java:254).
int dev_finalize_chunked(ipls_dev* h, int p, int sum_kind, int64_t chunk, ipls_chunk_sink sink, void* ctx) {
  if (!h || !sink) return fail_nl(h, IPLS_E_INVAL, "null argument");
  if (chunk < 2 || (chunk & 1))
    return fail_nl(h, IPLS_E_INVAL, "chunk of %lld values: even and >= 2", (long long)chunk);
  if (p < 0 || p >= h->P) return fail_nl(h, IPLS_E_RANGE, "partition %d out of range [0,%d)", p, h->P);
  if (sum_kind != IPLS_HOST_F64 && sum_kind != IPLS_HOST_BE)
    return fail_nl(h, IPLS_E_INVAL, "sum_kind must be HOST_F64 or HOST_BE");
  const int64_t L = h->len[p];
  HIP_TRY_NL(h, dev_use(h->device));
  const int64_t c = std::min(chunk, L);
  // every buffer first: a failure here leaves the round in place
  ipls_stage* st = nullptr;
  if (int rc = stage_acquire(h, (size_t)L * 8, (size_t)c * 8, &st)) return rc;
  int rc = IPLS_OK;
  {
    std::lock_guard<std::mutex> lk(h->mu);
    rc = flush_pending(h);
    if (!rc) rc = finalize_range(h, p, 1);
    if (!rc) {
      const unsigned long long* w = (const unsigned long long*)(h->arena + h->w_off[p]);
      hipError_t e;
      if (sum_kind == IPLS_HOST_BE) {
        launch_bswap(h->stream, w, (unsigned long long*)st->d, L);
        e = hipGetLastError();
      } else {
        e = hipMemcpyAsync(st->d, w, (size_t)L * 8, hipMemcpyDeviceToDevice, h->stream);
      }
      if (e == hipSuccess) e = hipEventRecord(st->ready, h->stream);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        rc = fail(h, IPLS_E_DEVICE, "W snapshot: %s", hipGetErrorString(e));
      }
    }
  }
  if (rc) {   // a kernel of this call may have been queued before the failure
    (void)hipStreamSynchronize(h->stream);
    (void)hipGetLastError();
    stage_release(h, st);
    return rc;
  }
  return stage_deliver(h, st, L, c, 0, sink, ctx, " (the round is consumed)");
}

int dev_set_weights(ipls_dev* h, int p, const void* src, int64_t n, int src_kind) {
  if (!h || !src) return fail(h, IPLS_E_INVAL, "null argument");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  const int64_t L = h->len[p];
  if (src_kind == IPLS_HOST_FRAME) {
    // ThreadReceiver pid 4 (IPLS.java:491-498): Weight_Address[p][i] =
    // GET_GRADIENTS(frame) payload[i] for i < L_p.
    int16_t pid;
    int32_t a, b;
    int64_t poff, ooff;
    const int64_t nd = ipls_frame_parse((const uint8_t*)src, n, &pid, &a, &b, &poff, &ooff);
    if (nd < 0) return fail(h, IPLS_E_FORMAT, "malformed frame (BufferUnderflowException)");
    if (nd == 0) return fail(h, IPLS_E_INVAL, "frame without gradients (NullPointerException, IPLS.java:498)");
    if (nd < L)
      return fail(h, IPLS_E_RANGE, "frame payload of %lld doubles < length %lld (IPLS.java:498)", (long long)nd,
                  (long long)L);
    HIP_TRY(h, dev_use(h->device));
    if (int rc = ensure_scratch(h, (size_t)L * 8)) return rc;
    if (int rc = stage_h2d(h, h->d_scratch, (const char*)src + poff, (size_t)L * 8)) return rc;
    launch_bswap(h->stream, (const unsigned long long*)h->d_scratch, (unsigned long long*)(h->arena + h->w_off[p]), L);
    HIP_TRY(h, hipGetLastError());
    return IPLS_OK;
  }
  // GetParameters(hash, arr) writes data.length/8 values (MyIPFSClass.java:449-452);
  // more than arr.length -> ArrayIndexOutOfBoundsException.
  if (n > L) return fail(h, IPLS_E_RANGE, "downloaded partition of %lld doubles > length %lld", (long long)n, (long long)L);
  if (n <= 0) return IPLS_OK;
  HIP_TRY(h, dev_use(h->device));
  double* w = h->arena + h->w_off[p];
  switch (src_kind) {
    case IPLS_HOST_F64:
      return stage_h2d(h, w, src, (size_t)n * 8);
    case IPLS_HOST_BE: {
      if (int rc = ensure_scratch(h, (size_t)n * 8)) return rc;
      if (int rc = stage_h2d(h, h->d_scratch, src, (size_t)n * 8)) return rc;
      launch_bswap(h->stream, (const unsigned long long*)h->d_scratch, (unsigned long long*)w, n);
      HIP_TRY(h, hipGetLastError());
      return IPLS_OK;
    }
    case IPLS_DEV_F64:
      HIP_TRY(h, hipMemcpyAsync(w, src, (size_t)n * 8, hipMemcpyDeviceToDevice, h->stream));
      return IPLS_OK;
    case IPLS_DEV_BE:
      launch_bswap(h->stream, (const unsigned long long*)src, (unsigned long long*)w, n);
      HIP_TRY(h, hipGetLastError());
      return IPLS_OK;
    default:
      return fail(h, IPLS_E_INVAL, "bad src_kind %d", src_kind);
  }
}

// Bring a flat vector of n doubles (host or device, native or BE) onto the
// device; returns a device pointer and whether it is big-endian.
static int flat_to_device(ipls_dev* h, const void* flat, int64_t n, int kind, const unsigned long long** d,
                          bool* be) {
  switch (kind) {
    case IPLS_DEV_F64:
    case IPLS_DEV_BE:
      *d = (const unsigned long long*)flat;
      *be = kind == IPLS_DEV_BE;
      return IPLS_OK;
    case IPLS_HOST_F64:
    case IPLS_HOST_BE:
      if (int rc = ensure_scratch(h, (size_t)std::max<int64_t>(n, 1) * 8)) return rc;
      if (n > 0)
        if (int rc = stage_h2d(h, h->d_scratch, flat, (size_t)n * 8)) return rc;
      *d = (const unsigned long long*)h->d_scratch;
      *be = kind == IPLS_HOST_BE;
      return IPLS_OK;
    default:
      return fail(h, IPLS_E_INVAL, "bad flat kind %d", kind);
  }
}

int dev_other_replica(ipls_dev* h, int p, int32_t aggregator, const void* src, int64_t n, int src_kind) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  if (n < 0 || (n > 0 && !src)) return fail(h, IPLS_E_INVAL, "bad bucket");
  if ((src_kind == IPLS_DEV_F64 || src_kind == IPLS_DEV_BE) && ((uintptr_t)src & 7))
    return fail(h, IPLS_E_INVAL, "device bucket not 8-byte aligned");
  HIP_TRY(h, dev_use(h->device));
  auto key = std::make_pair(p, aggregator);
  auto it = h->other.find(key);
  const bool first = it == h->other.end();
  // Download_Scheduler.java:254-260: `for j < gradients.length: Other[j] += g[j]`
  // -- a longer download overruns the stored array (rejected before folding).
  if (!first && n > it->second.n)
    return fail(h, IPLS_E_RANGE, "replica download of %lld doubles > stored %lld "
                "(ArrayIndexOutOfBoundsException, Download_Scheduler.java:257)", (long long)n,
                (long long)it->second.n);
  const unsigned long long* d;
  bool be;
  if (int rc = flat_to_device(h, src, n, src_kind, &d, &be)) return rc;
  unsigned long long* dst = first ? nullptr : it->second.d;
  // Other.put(key, GetParameters(Hash)): a new array of the file's length (:263)
  if (first) HIP_TRY(h, hipMalloc(&dst, (size_t)std::max<int64_t>(n, 1) * 8));
  hipError_t e = hipSuccess;
  if (n > 0) {
    const bool vec = al16(dst) && al16(d);
    const dim3 g = ew_grid(n, vec, 4096);
#define FN(B, F)                                                                                         \
  do {                                                                                                   \
    if (vec) hipLaunchKernelGGL((k_fold_n<B, F, true>), g, dim3(kBlock), 0, h->stream, dst, d, n);      \
    else hipLaunchKernelGGL((k_fold_n<B, F, false>), g, dim3(kBlock), 0, h->stream, dst, d, n);         \
  } while (0)
    if (be) { if (first) FN(true, true); else FN(true, false); }
    else { if (first) FN(false, true); else FN(false, false); }
#undef FN
    e = hipGetLastError();
  }
  if (e == hipSuccess && (src_kind == IPLS_HOST_F64 || src_kind == IPLS_HOST_BE)) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) {   // the store is left as it was (the front's key model relies on it)
    (void)hipGetLastError();
    if (first) hipFree(dst);
    return fail(h, IPLS_E_DEVICE, "replica fold failed: %s", hipGetErrorString(e));
  }
  if (first) h->other[key] = ipls_dev::OtherRep{dst, n, 1};
  else it->second.received += 1;   // Other_Replica_Gradients_Received + 1 (:260)
  return IPLS_OK;
}

int dev_other_replica_drop(ipls_dev* h, int p, int32_t aggregator) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  auto it = h->other.find(std::make_pair(p, aggregator));
  if (it == h->other.end()) return 0;   // containsKey false: nothing to remove
  // Other_Replica_Gradients.remove(key) + Other_Replica_Gradients_Received.remove(key)
  // (Download_Scheduler.java:215-217, 329-332, 438-440).  Folds into the array
  // may still be queued on the stream: free it only after them.
  HIP_TRY(h, dev_use(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  hipFree(it->second.d);
  h->other.erase(it);
  return 1;
}

int dev_collect_replicas(ipls_dev* h, int32_t* participants, const int32_t* order, int n_order) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  HIP_TRY(h, dev_use(h->device));
  // the fold order: `new ArrayList<>(Other_Replica_Gradients.keySet())`
  // (IPLS.java:1218), given by the front's model of the JDK HashMap
  // (java_hashmap.hpp) as engine-local (p, aggregator) pairs -- every stored
  // key exactly once
  if (n_order != (int)h->other.size() || (n_order > 0 && !order))
    return fail(h, IPLS_E_INVAL, "collect order lists %d keys, the store holds %zu", n_order, h->other.size());
  std::vector<std::map<std::pair<int, int32_t>, ipls_dev::OtherRep>::iterator> seq;
  seq.reserve(n_order);
  std::set<std::pair<int, int32_t>> seen;   // each key once (O(n log n) for large stores)
  for (int i = 0; i < n_order; ++i) {
    const std::pair<int, int32_t> key((int)order[2 * i], order[2 * i + 1]);
    auto it = h->other.find(key);
    if (it == h->other.end() || !seen.insert(key).second)
      return fail(h, IPLS_E_INVAL, "collect order key (%d, %d) is not a stored key", order[2 * i] + h->p_lo,
                  order[2 * i + 1]);
    seq.push_back(it);
  }
  // REP[p] is a double[L_p]: a longer stored array overruns it (IPLS.java:1225).
  for (auto& kv : h->other)
    if (kv.second.n > h->len[kv.first.first])
      return fail(h, IPLS_E_RANGE, "stored replica of %lld doubles > partition %d length %lld "
                  "(ArrayIndexOutOfBoundsException, IPLS.java:1225)", (long long)kv.second.n, kv.first.first,
                  (long long)h->len[kv.first.first]);
  if (participants)
    for (int q = 0; q < h->P; ++q) participants[q] = 0;
  int folded = 0;
  for (auto& it : seq) {   // IPLS.java:1222-1234: REP[p][j] = REP[p][j] + Other[j], j < Other.length
    const int p = it->first.first;
    const int64_t n = it->second.n;
    // PeerData.Participants (IPLS.java:1229-1234): the put / replace sits INSIDE
    // the j loop, so the reference adds the key's download count once per
    // element -- received * n in all, in wrapping int arithmetic
    if (participants)
      participants[p] = (int32_t)((uint32_t)participants[p] + (uint32_t)it->second.received * (uint32_t)n);
    if (n > 0) {
      if (int rc = materialize(h, p, IPLS_TGT_REP)) return rc;
      auto rdst = (unsigned long long*)(h->arena + h->rep_off[p]);
      const bool vec = al16(rdst) && al16(it->second.d);
      if (vec)
        hipLaunchKernelGGL((k_fold_n<false, false, true>), ew_grid(n, true, 4096), dim3(kBlock), 0, h->stream, rdst,
                           it->second.d, n);
      else
        hipLaunchKernelGGL((k_fold_n<false, false, false>), ew_grid(n, false, 4096), dim3(kBlock), 0, h->stream,
                           rdst, it->second.d, n);
      HIP_TRY(h, hipGetLastError());
    }
    ++folded;
  }
  // Other_Replica_Gradients = new HashMap<>() (:1237-1238)
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  for (auto& kv : h->other) hipFree(kv.second.d);
  h->other.clear();
  return folded;
}

int dev_load_model(ipls_dev* h, const void* src, int64_t n, int src_kind) {
  if (!h || !src) return fail(h, IPLS_E_INVAL, "null argument");
  IPLS_LOCK(h);
  if (n < h->flat_total)
    return fail(h, IPLS_E_RANGE, "model of %lld values < model size %lld", (long long)n, (long long)h->flat_total);
  HIP_TRY(h, dev_use(h->device));
  const unsigned long long* d;
  bool be;
  // only this engine's segment [flat_base, flat_total) of the model
  if (int rc = flat_to_device(h, (const char*)src + 8 * h->flat_base, h->flat_total - h->flat_base, src_kind, &d,
                              &be))
    return rc;
  for (int p = 0; p < h->P; ++p) {
    const int64_t L = h->len[p];
    // IPLS.java:1883-1895: values for j < min((i+1)c, M), count slot 0.0
    if (be)
      hipLaunchKernelGGL(k_load_model<true>, dim3(blocks_for(L, kBlock)), dim3(kBlock), 0, h->stream, d,
                         h->flat_off[p] - h->flat_base, L - 1, L, h->arena + h->w_off[p]);
    else
      hipLaunchKernelGGL(k_load_model<false>, dim3(blocks_for(L, kBlock)), dim3(kBlock), 0, h->stream, d,
                         h->flat_off[p] - h->flat_base, L - 1, L, h->arena + h->w_off[p]);
    HIP_TRY(h, hipGetLastError());
    h->agg_zero[p] = h->rep_zero[p] = h->fut_zero[p] = 1;   // IPLS.java:1886-1898
  }
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return IPLS_OK;
}

// OrganizeGradients bounds for partition p of a flat vector of n values.
static int split_bounds(ipls_dev* h, int p, int64_t n, int64_t* ncopy) {
  const int64_t lo = h->flat_off[p];
  const int64_t hi = std::min(lo + h->chunk, n);
  const int64_t nc = std::max<int64_t>(0, hi - lo);
  if (nc > h->len[p] - 1)
    return fail(h, IPLS_E_RANGE, "gradient vector of %lld values overruns partition %d (ArrayIndexOutOfBounds, IPLS.java:1030)",
                (long long)n, p);
  *ncopy = nc;
  return IPLS_OK;
}

int dev_split(ipls_dev* h, const void* flat, int64_t n, int src_kind, int p, void* dst, int dst_kind) {
  if (!h || !flat || !dst) return fail(h, IPLS_E_INVAL, "null argument");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  int64_t ncopy;
  if (int rc = split_bounds(h, p, n, &ncopy)) return rc;
  HIP_TRY(h, dev_use(h->device));
  const int64_t L = h->len[p];
  const unsigned long long* d;
  bool be_in;
  // only the partition's own slice is needed on the device
  const int64_t lo = h->flat_off[p];
  if (src_kind == IPLS_HOST_F64 || src_kind == IPLS_HOST_BE) {
    if (int rc = ensure_scratch(h, (size_t)(2 * L + 2) * 8)) return rc;
    if (ncopy > 0)
      if (int rc = stage_h2d(h, h->d_scratch, (const char*)flat + lo * 8, (size_t)ncopy * 8)) return rc;
    d = (const unsigned long long*)h->d_scratch;
    be_in = src_kind == IPLS_HOST_BE;
  } else if (src_kind == IPLS_DEV_F64 || src_kind == IPLS_DEV_BE) {
    d = (const unsigned long long*)flat + lo;
    be_in = src_kind == IPLS_DEV_BE;
    if (int rc = ensure_scratch(h, (size_t)(L + 1) * 8)) return rc;
  } else {
    return fail(h, IPLS_E_INVAL, "bad src_kind %d", src_kind);
  }
  const bool host_out = dst_kind == IPLS_HOST_F64 || dst_kind == IPLS_HOST_BE;
  const bool be_out = dst_kind == IPLS_HOST_BE || dst_kind == IPLS_DEV_BE;
  if (!host_out && dst_kind != IPLS_DEV_F64 && dst_kind != IPLS_DEV_BE)
    return fail(h, IPLS_E_INVAL, "bad dst_kind %d", dst_kind);
  unsigned long long* out = host_out ? (unsigned long long*)((char*)h->d_scratch + (size_t)(L + 1) * 8)
                                     : (unsigned long long*)dst;
  if (host_out && src_kind != IPLS_HOST_F64 && src_kind != IPLS_HOST_BE)
    out = (unsigned long long*)h->d_scratch;
  const bool vec = al16(d) && al16(out);
  const dim3 g = vec ? dim3(std::max(1u, blocks_for(L, kEwTile))) : dim3(blocks_for(L, kBlock));
#define SPL(BI, BO)                                                                                              \
  do {                                                                                                           \
    if (vec) hipLaunchKernelGGL((k_split<BI, BO, 0, true>), g, dim3(kBlock), 0, h->stream, d, (int64_t)0, ncopy, L, out); \
    else hipLaunchKernelGGL((k_split<BI, BO, 0, false>), g, dim3(kBlock), 0, h->stream, d, (int64_t)0, ncopy, L, out); \
  } while (0)
  if (be_in) { if (be_out) SPL(true, true); else SPL(true, false); }
  else { if (be_out) SPL(false, true); else SPL(false, false); }
#undef SPL
  HIP_TRY(h, hipGetLastError());
  if (host_out) return d2h(h, dst, out, (size_t)L * 8);
  return IPLS_OK;
}

int dev_update_gradient(ipls_dev* h, const void* flat, int64_t n, int src_kind, const int32_t* owned,
                             int n_owned) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  if (!flat) return IPLS_OK;  // Gradients == null (IPLS.java:1708-1713, 1738 `&& Gradients != null`)
  IPLS_LOCK(h);
  if (n_owned < 0 || (n_owned > 0 && !owned)) return fail(h, IPLS_E_INVAL, "bad owned list");
  // OrganizeGradients splits every partition before anything is accumulated
  // (IPLS.java:1709), so a length error leaves the accumulators untouched.
  std::vector<int64_t> nc(h->P);
  for (int p = 0; p < h->P; ++p)
    if (int rc = split_bounds(h, p, n, &nc[p])) return rc;
  for (int i = 0; i < n_owned; ++i)
    if (int rc = check_part(h, owned[i])) return rc;
  if (n_owned == 0) return IPLS_OK;
  HIP_TRY(h, dev_use(h->device));
  const unsigned long long* d;
  bool be;
  // only this engine's segment of the gradient vector (flat_base on)
  const int64_t seg = std::max<int64_t>(0, std::min(n, h->flat_total) - h->flat_base);
  if (src_kind == IPLS_HOST_F64 || src_kind == IPLS_HOST_BE) {
    // from host memory only the owned partitions' values cross PCIe: the
    // others are split by OrganizeGradients too, but never accumulated
    // (IPLS.java:1737-1743), so their bytes are never read here
    if (int rc = ensure_scratch(h, (size_t)std::max<int64_t>(seg, 1) * 8)) return rc;
    const char* base = (const char*)flat + 8 * h->flat_base;
    for (int i = 0; i < n_owned; ++i) {
      const int64_t lo = h->flat_off[owned[i]] - h->flat_base;
      if (nc[owned[i]] > 0)
        if (int rc = stage_h2d(h, (char*)h->d_scratch + 8 * lo, base + 8 * lo, (size_t)nc[owned[i]] * 8)) return rc;
    }
    d = (const unsigned long long*)h->d_scratch;
    be = src_kind == IPLS_HOST_BE;
  } else if (int rc = flat_to_device(h, (const char*)flat + 8 * h->flat_base, seg, src_kind, &d, &be)) {
    return rc;
  }
  for (int i = 0; i < n_owned; ++i) {
    const int p = owned[i];
    const int64_t L = h->len[p];
    unsigned long long* acc = (unsigned long long*)(h->arena + h->agg_off[p]);
    const bool zero = h->agg_zero[p];
    const int64_t lo = h->flat_off[p] - h->flat_base;
    // the segment's start decides: partitions whose flat offset is odd read
    // their values at 8 mod 16 and keep the element-per-lane shape
    const bool vec = al16(d + lo) && al16(acc);
    const dim3 g = vec ? dim3(std::max(1u, blocks_for(L, kEwTile))) : dim3(blocks_for(L, kBlock));
    // Logically-zero accumulator: MODE 2 writes +0.0 + v without reading it
    // (the bits of a fold into zeros)
#define UPD(BI, M)                                                                                              \
  do {                                                                                                          \
    if (vec) hipLaunchKernelGGL((k_split<BI, false, M, true>), g, dim3(kBlock), 0, h->stream, d, lo, nc[p], L, acc); \
    else hipLaunchKernelGGL((k_split<BI, false, M, false>), g, dim3(kBlock), 0, h->stream, d, lo, nc[p], L, acc); \
  } while (0)
    if (be) { if (zero) UPD(true, 2); else UPD(true, 1); }
    else { if (zero) UPD(false, 2); else UPD(false, 1); }
#undef UPD
    HIP_TRY(h, hipGetLastError());
    h->agg_zero[p] = 0;
  }
  return IPLS_OK;
}

int dev_get_partitions(ipls_dev* h, void* out, int64_t n, int out_kind) {
  if (!h || !out) return fail(h, IPLS_E_INVAL, "null argument");
  IPLS_LOCK(h);
  // out holds this engine's segment: flat offsets [flat_base, flat_total)
  const int64_t M = h->flat_total - h->flat_base;
  if (n < M) return fail(h, IPLS_E_RANGE, "output of %lld < model size %lld", (long long)n, (long long)M);
  if (out_kind != IPLS_HOST_F64 && out_kind != IPLS_HOST_BE_CANON && out_kind != IPLS_DEV_F64)
    return fail(h, IPLS_E_INVAL, "bad out_kind %d", out_kind);
  HIP_TRY(h, dev_use(h->device));
  unsigned long long* d_out;
  if (out_kind == IPLS_DEV_F64) {
    if ((uintptr_t)out & 7) return fail(h, IPLS_E_INVAL, "device output not 8-byte aligned");
    d_out = (unsigned long long*)out;
  } else {
    if (int rc = ensure_scratch(h, (size_t)std::max<int64_t>(M, 1) * 8)) return rc;
    d_out = (unsigned long long*)h->d_scratch;
  }
  if (int rc = divide_range(h, 0, h->P, d_out, out_kind == IPLS_HOST_BE_CANON)) return rc;
  if (out_kind == IPLS_DEV_F64) return IPLS_OK;
  return d2h(h, out, d_out, (size_t)M * 8);
}

// GetPartitions (IPLS.java:1159-1174) handed to the caller chunk by chunk,
// in two phases so that a multi-shard handle snapshots every shard before it
// delivers any byte (ipls_agg.cpp):
//  * snapshot, under the engine lock: the divide runs once into this call's
//    own staging (wire: the same values as Middleware's task-3 writeDouble
//    stream -- big-endian, NaN canonical: k_divide's OUT_BE form);
//  * deliver, with no lock held: chunk k + 1 is copied into one slot of the
//    stage's pinned ring while sink() consumes chunk k from another slot,
//    on the calling thread (the JNI shim's sink is SetDoubleArrayRegion, the
//    Middleware's a socket send).  sink gets flat model offsets (this engine's
//    segment starts at flat_base); a non-zero return stops the transfer
//    (IPLS_E_INVAL, nothing further is delivered).
// *st is null when the engine's segment is empty.
int dev_get_partitions_snapshot(ipls_dev* h, int64_t chunk, bool wire, ipls_stage** st_out) {
  *st_out = nullptr;
  if (!h) return fail_nl(h, IPLS_E_INVAL, "null argument");
  if (chunk < 2 || (chunk & 1))
    return fail_nl(h, IPLS_E_INVAL, "chunk of %lld doubles: even and >= 2", (long long)chunk);
  const int64_t M = h->flat_total - h->flat_base;
  if (M <= 0) return IPLS_OK;
  HIP_TRY_NL(h, dev_use(h->device));
  ipls_stage* st = nullptr;
  if (int rc = stage_acquire(h, (size_t)M * 8, (size_t)std::min(chunk, M) * 8, &st)) return rc;
  int rc = IPLS_OK;
  {
    std::lock_guard<std::mutex> lk(h->mu);
    rc = flush_pending(h);
    if (!rc) rc = divide_range(h, 0, h->P, (unsigned long long*)st->d, wire);
    if (!rc) {
      const hipError_t e = hipEventRecord(st->ready, h->stream);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        rc = fail(h, IPLS_E_DEVICE, "hipEventRecord failed: %s", hipGetErrorString(e));
      }
    }
  }
  if (rc) {   // a kernel of this call may have been queued before the failure
    (void)hipStreamSynchronize(h->stream);
    (void)hipGetLastError();
    stage_release(h, st);
    return rc;
  }
  *st_out = st;
  return IPLS_OK;
}

int dev_get_partitions_deliver(ipls_dev* h, ipls_stage* st, int64_t chunk, ipls_chunk_sink sink, void* ctx) {
  if (!st) return IPLS_OK;
  const int64_t M = h->flat_total - h->flat_base;
  HIP_TRY_NL(h, dev_use(h->device));
  return stage_deliver(h, st, M, std::min(chunk, M), h->flat_base, sink, ctx, "");
}

// A snapshot that is not delivered (another shard failed first): the divide
// that writes it finishes before the stage can be reused.
void dev_stage_release(ipls_dev* h, ipls_stage* st) {
  if (!st) return;
  (void)dev_use(h->device);
  if (hipEventSynchronize(st->ready) != hipSuccess) (void)hipGetLastError();
  stage_release(h, st);
}

int dev_get_partitions_chunked(ipls_dev* h, int64_t chunk, ipls_chunk_sink sink, void* ctx, bool wire) {
  if (!h || !sink) return fail_nl(h, IPLS_E_INVAL, "null argument");
  ipls_stage* st = nullptr;
  if (int rc = dev_get_partitions_snapshot(h, chunk, wire, &st)) return rc;
  return dev_get_partitions_deliver(h, st, chunk, sink, ctx);
}

// ---- device utilities ----
int ipls_synth_fill(void* dst, int64_t len, uint64_t seed, int p, int k, int dst_kind, void* stream) {
  if (!dst || len < 0) return fail(nullptr, IPLS_E_INVAL, "bad argument");
  if (len == 0) return IPLS_OK;
  const unsigned long long key = seed ^ ((unsigned long long)(uint32_t)p << 40) ^ ((unsigned long long)(uint32_t)k << 32);
  const dim3 g(std::min<unsigned>(blocks_for(len, kBlock * 4), 8192));
  if (dst_kind == IPLS_DEV_BE)
    hipLaunchKernelGGL(k_synth<true>, g, dim3(kBlock), 0, (hipStream_t)stream, (unsigned long long*)dst, len, key);
  else if (dst_kind == IPLS_DEV_F64)
    hipLaunchKernelGGL(k_synth<false>, g, dim3(kBlock), 0, (hipStream_t)stream, (unsigned long long*)dst, len, key);
  else
    return fail(nullptr, IPLS_E_INVAL, "dst_kind must be DEV_F64 or DEV_BE");
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(nullptr, IPLS_E_DEVICE, "k_synth launch: %s", hipGetErrorString(e));
  return IPLS_OK;
}

int ipls_checksum_dev(const void* src, int64_t n, int src_kind, uint64_t* out, void* stream) {
  if (!out || n < 0 || (n > 0 && !src)) return fail(nullptr, IPLS_E_INVAL, "bad argument");
  if (n == 0) {
    *out = 0;
    return IPLS_OK;
  }
  hipStream_t st = (hipStream_t)stream;
  unsigned long long* d = nullptr;
  if (hipMallocAsync((void**)&d, 8, st) != hipSuccess) {
    (void)hipGetLastError();
    return fail(nullptr, IPLS_E_NOMEM, "hipMallocAsync failed");
  }
  hipMemsetAsync(d, 0, 8, st);
  const dim3 g(std::max(1u, std::min<unsigned>(blocks_for(n, kBlock * 8), 2048)));
  if (src_kind == IPLS_DEV_BE)
    hipLaunchKernelGGL(k_checksum<true>, g, dim3(kBlock), 0, st, (const unsigned long long*)src, n, d);
  else
    hipLaunchKernelGGL(k_checksum<false>, g, dim3(kBlock), 0, st, (const unsigned long long*)src, n, d);
  unsigned long long v = 0;
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(&v, d, 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  hipFreeAsync(d, st);
  if (e != hipSuccess) return fail(nullptr, IPLS_E_DEVICE, "checksum: %s", hipGetErrorString(e));
  *out = v;
  return IPLS_OK;
}

int dev_reduce_batch_out(ipls_dev* h, int p_first, int n_parts, const void* const* bufs, int k, int src_kind,
                              int start_mode, void* const* dst, int dst_kind) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (n_parts <= 0 || p_first < 0 || p_first + n_parts > h->P)
    return fail(h, IPLS_E_RANGE, "partitions [%d,%d) out of range [0,%d)", p_first, p_first + n_parts, h->P);
  if (src_kind != IPLS_DEV_F64 && src_kind != IPLS_DEV_BE)
    return fail(h, IPLS_E_INVAL, "reduce_batch_out takes device buckets (DEV_F64/DEV_BE)");
  if (dst_kind != IPLS_DEV_F64 && dst_kind != IPLS_DEV_BE)
    return fail(h, IPLS_E_INVAL, "reduce_batch_out writes device buffers (DEV_F64/DEV_BE)");
  if (start_mode < IPLS_START_ACCUM || start_mode > IPLS_START_FIRST) return fail(h, IPLS_E_INVAL, "bad start mode");
  if (!dst || k < 0 || (k > 0 && !bufs)) return fail(h, IPLS_E_INVAL, "bad bucket/destination list");
  HIP_TRY(h, dev_use(h->device));
  return reduce_dev(h, p_first, n_parts, bufs, k, src_kind == IPLS_DEV_BE, start_mode, IPLS_TGT_AGG, dst,
                    dst_kind == IPLS_DEV_BE);
}

int dev_aggregate_round(ipls_dev* h, int p_first, int n_parts, const void* const* bufs, int k, int src_kind,
                             void* avg_out, int avg_kind) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (n_parts <= 0 || p_first < 0 || p_first + n_parts > h->P)
    return fail(h, IPLS_E_RANGE, "partitions [%d,%d) out of range [0,%d)", p_first, p_first + n_parts, h->P);
  if (src_kind != IPLS_DEV_F64 && src_kind != IPLS_DEV_BE)
    return fail(h, IPLS_E_INVAL, "aggregate_round takes device buckets (DEV_F64/DEV_BE)");
  if (avg_out && avg_kind != IPLS_DEV_F64 && avg_kind != IPLS_HOST_F64)
    return fail(h, IPLS_E_INVAL, "avg_kind must be DEV_F64 or HOST_F64");
  if (k < 0 || (k > 0 && !bufs)) return fail(h, IPLS_E_INVAL, "bad bucket list");
  HIP_TRY(h, dev_use(h->device));
  const int p_last = p_first + n_parts - 1;
  const int64_t n_avg = h->flat_off[p_last] + h->len[p_last] - 1 - h->flat_off[p_first];
  unsigned long long* d_avg = nullptr;
  if (avg_out && n_avg > 0) {
    if (avg_kind == IPLS_DEV_F64) {
      if ((uintptr_t)avg_out & 7) return fail(h, IPLS_E_INVAL, "device output not 8-byte aligned");
      d_avg = (unsigned long long*)avg_out;
    } else {
      if (int rc = ensure_scratch(h, (size_t)n_avg * 8)) return rc;
      d_avg = (unsigned long long*)h->d_scratch;
    }
  }
  bool aligned16 = true;
  for (int64_t i = 0; i < (int64_t)n_parts * k; ++i) aligned16 = aligned16 && !((uintptr_t)bufs[i] & 15);
  if (aligned16) {
    FinOut fo{d_avg};
    if (int rc = reduce_dev(h, p_first, n_parts, bufs, k, src_kind == IPLS_DEV_BE, IPLS_START_ACCUM, IPLS_TGT_AGG,
                            nullptr, false, &fo))
      return rc;
  } else {
    // 8-B aligned buckets (frames at odd offsets): the same three steps unfused
    if (int rc = reduce_dev(h, p_first, n_parts, bufs, k, src_kind == IPLS_DEV_BE, IPLS_START_ACCUM, IPLS_TGT_AGG))
      return rc;
    if (int rc = finalize_range(h, p_first, n_parts)) return rc;
    if (d_avg)
      if (int rc = divide_range(h, p_first, n_parts, d_avg, false)) return rc;
  }
  if (d_avg && avg_kind == IPLS_HOST_F64) return d2h(h, avg_out, d_avg, (size_t)n_avg * 8);
  return IPLS_OK;
}

// ---- pubsub ingest: base64url (x layers) -> frame -> fold, on the device ----
namespace {

// Copy-issuing threads of the pubsub ingest (IPLS_INGEST_COPY_THREADS, 1..4).
int ingest_copy_threads() {
  static const int n = [] {
    const char* e = std::getenv("IPLS_INGEST_COPY_THREADS");
    const int v = e ? std::atoi(e) : 2;
    return std::max(1, std::min(v, (int)ipls_dev::kCopyThreads));
  }();
  return n;
}

}  // namespace

// Pipeline: the host reads each text's ends (the '=' rules of both layers and
// the 14-byte frame header need only the first 28 and last 8 chars), so no
// device round trip sits between the copies and the decodes.  Texts go up on
// copy_stream while `stream` decodes the previous ones behind a per-message
// event; one sync reads the invalid-char flags, then each partition's frames
// are folded in message order.
int dev_ingest_pubsub(ipls_dev* h, int target, const uint8_t* const* msgs, const int64_t* lens, int n_msgs,
                           int layers, const int32_t* parts, int32_t* status) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (n_msgs < 0 || (n_msgs > 0 && (!msgs || !lens))) return fail(h, IPLS_E_INVAL, "bad message list");
  if (layers < 1 || layers > 2) return fail(h, IPLS_E_INVAL, "layers must be 1 or 2");
  if (target_off(h, 0, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  if (n_msgs == 0) return 0;
  HIP_TRY(h, dev_use(h->device));

  // 1. host: tail rules, frame header, routing (GET_GRADIENTS, MyIPFSClass.java:1437-1459).
  //    post[i] = the status if the device finds no invalid char; decode[i] = needs the device.
  std::vector<int32_t> st(n_msgs, 0), post(n_msgs, 0), route(n_msgs, -1);
  std::vector<int64_t> dc(n_msgs, 0), dc2(n_msgs, 0);
  std::vector<uint8_t> decode(n_msgs, 0);
  for (int i = 0; i < n_msgs; ++i) {
    const pubsub::Pre pre = pubsub::precheck(msgs[i], lens[i], layers);   // pubsub_host.cpp
    if (pre.status) { st[i] = pre.status; continue; }
    dc[i] = pre.dc;
    dc2[i] = pre.dc2;
    decode[i] = 1;
    if (pre.n == 0) { post[i] = 1; continue; }      // arr_len == 0 -> null gradient: no fold
    const int p = parts ? parts[i] : pre.a;
    if (p < 0 || p >= h->P || pre.n < h->len[p]) { post[i] = IPLS_E_RANGE; continue; }
    route[i] = p;
  }

  // 2. device: scratch [texts][layer-1 output][frames], 256-B aligned per message;
  //    frames start 2 bytes in so the payload (frame byte 14) is 16-B aligned.
  std::vector<int64_t> text_off(n_msgs, 0), mid_off(n_msgs, 0), frame_off(n_msgs, 0);
  int64_t off = 0;
  for (int i = 0; i < n_msgs; ++i)
    if (decode[i]) { text_off[i] = off; off = align_up(off + lens[i] + 16, 256); }
  if (layers == 2)
    for (int i = 0; i < n_msgs; ++i)
      if (decode[i]) { mid_off[i] = off; off = align_up(off + lens[i] + 16, 256); }
  for (int i = 0; i < n_msgs; ++i)
    if (decode[i]) { frame_off[i] = off + 2; off = align_up(off + 2 + lens[i] + 16, 256); }
  int n_dec = 0;
  for (int i = 0; i < n_msgs; ++i) n_dec += decode[i];
  if (n_dec) {
    if (int rc = ensure_scratch(h, (size_t)off + 64 * (size_t)n_msgs + 4096)) return rc;
    unsigned char* base = (unsigned char*)h->d_scratch;
    int* d_err = (int*)(base + off);
    std::vector<B64Desc> desc(2 * (size_t)n_msgs);
    for (int i = 0; i < n_msgs; ++i) {
      if (!decode[i]) continue;
      desc[i] = B64Desc{text_off[i], dc[i] / 4, layers == 2 ? mid_off[i] : frame_off[i], (int32_t)(dc[i] % 4), 0};
      desc[n_msgs + i] = B64Desc{mid_off[i], dc2[i] / 4, frame_off[i], (int32_t)(dc2[i] % 4), 0};
    }
    void* dtab = nullptr;
    if (int rc = upload_table(h, desc.data(), sizeof(B64Desc) * desc.size(), &dtab)) return rc;
    const B64Desc* d1 = (const B64Desc*)dtab;
    HIP_TRY(h, hipMemsetAsync(d_err, 0, sizeof(int) * n_msgs, h->stream));
    // Texts are pageable: each hipMemcpyAsync blocks its calling thread and
    // pays ~45 us of setup between transfers, so T threads issue the copies
    // (message j of the batch on thread j % T, its own stream) and this thread
    // queues each message's decodes behind that copy's event as it lands.
    const int T = std::max(1, std::min(ingest_copy_threads(), n_dec));
    for (int t = 0; t < T; ++t)
      if (!h->copy_stream[t]) HIP_TRY(h, hipStreamCreateWithFlags(&h->copy_stream[t], hipStreamNonBlocking));
    if (!h->ingest_ev) HIP_TRY(h, hipEventCreateWithFlags(&h->ingest_ev, hipEventDisableTiming));
    while ((int)h->msg_ev.size() < n_msgs) {
      hipEvent_t e;
      HIP_TRY(h, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      h->msg_ev.push_back(e);
    }
    // the scratch may still be read by earlier work on `stream`
    HIP_TRY(h, hipEventRecord(h->ingest_ev, h->stream));
    for (int t = 0; t < T; ++t) HIP_TRY(h, hipStreamWaitEvent(h->copy_stream[t], h->ingest_ev, 0));
    std::vector<int> order;
    for (int i = 0; i < n_msgs; ++i)
      if (decode[i]) order.push_back(i);
    std::unique_ptr<std::atomic<int>[]> ready(new std::atomic<int>[n_dec]);   // 0 pending, 1 recorded, <0 error
    for (int j = 0; j < n_dec; ++j) ready[j].store(0);
    auto copier = [&](int t) {
      dev_use(h->device);
      for (int j = t; j < n_dec; j += T) {
        const int i = order[j];
        hipError_t e = hipMemcpyAsync(base + text_off[i], msgs[i], lens[i], hipMemcpyHostToDevice, h->copy_stream[t]);
        if (e == hipSuccess) e = hipEventRecord(h->msg_ev[i], h->copy_stream[t]);
        ready[j].store(e == hipSuccess ? 1 : -(int)e, std::memory_order_release);
        if (e != hipSuccess) {
          for (int r = j + T; r < n_dec; r += T) ready[r].store(-(int)e, std::memory_order_release);
          return;
        }
      }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t) pool.emplace_back(copier, t);
    if (T == 1) copier(0);
    else pool.emplace_back(copier, 0);
    int copy_err = 0;
    for (int j = 0; j < n_dec && !copy_err; ++j) {
      int r;
      while ((r = ready[j].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
      if (r < 0) { copy_err = -r; break; }
      const int i = order[j];
      hipStreamWaitEvent(h->stream, h->msg_ev[i], 0);
      hipLaunchKernelGGL(k_b64url_decode, dim3(blocks_for(dc[i] / 16 + 1, kBlock)), dim3(kBlock), 0, h->stream,
                         (const unsigned char*)base, d1 + i, base, d_err + i);
      if (layers == 2)
        hipLaunchKernelGGL(k_b64url_decode, dim3(blocks_for(dc2[i] / 16 + 1, kBlock)), dim3(kBlock), 0, h->stream,
                           (const unsigned char*)base, d1 + n_msgs + i, base, d_err + i);
    }
    for (auto& th : pool) th.join();
    if (copy_err) return fail(h, IPLS_E_DEVICE, "pubsub text copy failed: %s", hipGetErrorString((hipError_t)copy_err));
    HIP_TRY(h, hipGetLastError());
    std::vector<int> herr(n_msgs, 0);
    HIP_TRY(h, hipMemcpyAsync(herr.data(), d_err, sizeof(int) * n_msgs, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    for (int i = 0; i < n_msgs; ++i)
      if (decode[i]) st[i] = herr[i] ? IPLS_E_FORMAT : post[i];
    // 3. fold each partition's frames in message order
    std::vector<std::vector<const void*>> per_part(h->P);
    for (int i = 0; i < n_msgs; ++i)
      if (decode[i] && st[i] == 0) per_part[route[i]].push_back(base + frame_off[i] + 14);
    int folded = 0;
    for (int p = 0; p < h->P; ++p) {
      if (per_part[p].empty()) continue;
      if (int rc = reduce_dev(h, p, 1, per_part[p].data(), (int)per_part[p].size(), true, IPLS_START_ACCUM, target))
        return rc;
      folded += (int)per_part[p].size();
    }
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    if (status) std::memcpy(status, st.data(), sizeof(int32_t) * n_msgs);
    return folded;
  }
  if (status) std::memcpy(status, st.data(), sizeof(int32_t) * n_msgs);
  return 0;
}

int dev_blend(ipls_dev* h, int p, int target, const void* src, int64_t n, int src_kind, double a, double b) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  if (target_off(h, p, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  if (!src) return IPLS_OK;
  const int64_t L = h->len[p];
  if (n < L) return fail(h, IPLS_E_RANGE, "bucket of %lld doubles shorter than partition length %lld", (long long)n, (long long)L);
  HIP_TRY(h, dev_use(h->device));
  const void* d = src;
  bool be = src_kind == IPLS_HOST_BE || src_kind == IPLS_DEV_BE;
  if (src_kind == IPLS_HOST_F64 || src_kind == IPLS_HOST_BE) {
    if (int rc = ensure_scratch(h, (size_t)L * 8)) return rc;
    if (int rc = stage_h2d(h, h->d_scratch, src, (size_t)L * 8)) return rc;
    d = h->d_scratch;
  } else if (src_kind != IPLS_DEV_F64 && src_kind != IPLS_DEV_BE) {
    return fail(h, IPLS_E_INVAL, "bad src_kind %d", src_kind);
  }
  if (int rc = materialize(h, p, target)) return rc;
  double* t = h->arena + target_off(h, p, target);
  const bool vec = al16(t) && al16(d);
  const dim3 g = ew_grid(L, vec, 8192);
  auto gs = (const unsigned long long*)d;
  if (be) {
    if (vec) hipLaunchKernelGGL((k_blend<true, true>), g, dim3(kBlock), 0, h->stream, t, gs, L, a, b);
    else hipLaunchKernelGGL((k_blend<true, false>), g, dim3(kBlock), 0, h->stream, t, gs, L, a, b);
  } else {
    if (vec) hipLaunchKernelGGL((k_blend<false, true>), g, dim3(kBlock), 0, h->stream, t, gs, L, a, b);
    else hipLaunchKernelGGL((k_blend<false, false>), g, dim3(kBlock), 0, h->stream, t, gs, L, a, b);
  }
  HIP_TRY(h, hipGetLastError());
  return IPLS_OK;
}

int dev_scale(ipls_dev* h, int p, int dst_target, int src_target, double c) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  if (target_off(h, p, dst_target) < 0 || target_off(h, p, src_target) < 0) return fail(h, IPLS_E_INVAL, "bad target");
  HIP_TRY(h, dev_use(h->device));
  if (int rc = materialize(h, p, src_target)) return rc;
  if (uint8_t* f = zero_flag(h, p, dst_target)) *f = 0;
  const int64_t L = h->len[p];
  double* sd = h->arena + target_off(h, p, dst_target);
  auto ss = (const double*)(h->arena + target_off(h, p, src_target));
  if (al16(sd) && al16(ss))
    hipLaunchKernelGGL(k_scale<true>, ew_grid(L, true, 8192), dim3(kBlock), 0, h->stream, sd, ss, L, c);
  else
    hipLaunchKernelGGL(k_scale<false>, ew_grid(L, false, 8192), dim3(kBlock), 0, h->stream, sd, ss, L, c);
  HIP_TRY(h, hipGetLastError());
  return IPLS_OK;
}

int ipls_encode_secure(const void* src, void* dst, int64_t n, int src_kind, int dst_kind, void* stream) {
  if (!src || !dst || n < 0) return fail(nullptr, IPLS_E_INVAL, "bad argument");
  if ((src_kind != IPLS_DEV_F64 && src_kind != IPLS_DEV_BE) || (dst_kind != IPLS_DEV_F64 && dst_kind != IPLS_DEV_BE))
    return fail(nullptr, IPLS_E_INVAL, "device operands only (DEV_F64 / DEV_BE)");
  if (n == 0) return IPLS_OK;
  hipStream_t st = (hipStream_t)stream;
  auto s = (const unsigned long long*)src;
  auto d = (unsigned long long*)dst;
  const bool bi = src_kind == IPLS_DEV_BE, bo = dst_kind == IPLS_DEV_BE;
  const bool vec = al16(s) && al16(d);
  const dim3 g = ew_grid(n, vec, 8192);
#define ENC(BI, BO)                                                                                     \
  do {                                                                                                  \
    if (vec) hipLaunchKernelGGL((k_encode_secure<BI, BO, true>), g, dim3(kBlock), 0, st, s, d, n);      \
    else hipLaunchKernelGGL((k_encode_secure<BI, BO, false>), g, dim3(kBlock), 0, st, s, d, n);         \
  } while (0)
  if (bi && bo) ENC(true, true);
  else if (bi) ENC(true, false);
  else if (bo) ENC(false, true);
  else ENC(false, false);
#undef ENC
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(nullptr, IPLS_E_DEVICE, "k_encode_secure: %s", hipGetErrorString(e));
  return IPLS_OK;
}

int ipls_host_alloc(size_t bytes, void** ptr) {
  if (!ptr) return fail(nullptr, IPLS_E_INVAL, "null ptr");
  *ptr = nullptr;
  if (bytes == 0) return IPLS_OK;
  hipError_t e = hipHostMalloc(ptr, bytes, hipHostMallocDefault);
  if (e != hipSuccess) {
    *ptr = nullptr;
    (void)hipGetLastError();
    return fail(nullptr, e == hipErrorNoDevice ? IPLS_E_NODEV : IPLS_E_NOMEM, "hipHostMalloc(%zu): %s", bytes,
                hipGetErrorString(e));
  }
  return IPLS_OK;
}

int ipls_host_free(void* ptr) {
  if (!ptr) return IPLS_OK;
  hipError_t e = hipHostFree(ptr);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(nullptr, IPLS_E_INVAL, "hipHostFree: %s", hipGetErrorString(e));
  }
  return IPLS_OK;
}

static uint32_t rd_be32(const uint8_t* b) {
  return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}

int64_t ipls_frame_parse(const uint8_t* frame, int64_t len, int16_t* pid, int32_t* a, int32_t* b,
                         int64_t* payload_off, int64_t* origin_off) {
  if (!frame || len < 14) return fail(nullptr, IPLS_E_FORMAT, "frame shorter than its 14-byte header");
  const int16_t pd = (int16_t)(((uint16_t)frame[0] << 8) | frame[1]);
  const int32_t n = (int32_t)rd_be32(frame + 2);
  if (n < 0 || 14 + 8 * (int64_t)n > len)
    return fail(nullptr, IPLS_E_FORMAT, "frame declares %d doubles but holds %lld bytes", n, (long long)len);
  if (pid) *pid = pd;
  if (a) *a = (int32_t)rd_be32(frame + 6);
  if (b) *b = (int32_t)rd_be32(frame + 10);
  if (payload_off) *payload_off = 14;
  if (origin_off) *origin_off = 14 + 8 * (int64_t)n;
  return n;
}

int64_t ipls_pair_parse(const uint8_t* buf, int64_t len, int32_t* workers, int64_t* payload_off) {
  if (!buf || len < 0) return fail(nullptr, IPLS_E_INVAL, "bad argument");
  const char* why = nullptr;
  const int64_t nd = javaser::parse_pair(buf, len, workers, payload_off, &why);
  if (nd < 0) return fail(nullptr, IPLS_E_FORMAT, "partial update: %s", why ? why : "malformed");
  return nd;
}

int64_t ipls_pair_encode(int32_t workers, const void* g, int64_t n, int g_kind, uint8_t* out, int64_t out_cap) {
  if (n < 0 || n > INT32_MAX || (n > 0 && out && !g)) return fail(nullptr, IPLS_E_INVAL, "bad argument");
  if (g_kind != IPLS_HOST_F64 && g_kind != IPLS_HOST_BE) return fail(nullptr, IPLS_E_INVAL, "g_kind must be HOST_F64/BE");
  const int64_t hl = javaser::pair_header_len(), total = hl + 8 * n + javaser::pair_trailer_len();
  if (!out) return total;
  if (out_cap < total) return fail(nullptr, IPLS_E_RANGE, "partial update needs %lld bytes", (long long)total);
  javaser::write_pair_header(out, workers, (int32_t)n);
  if (g_kind == IPLS_HOST_BE) {
    std::memcpy(out + hl, g, (size_t)n * 8);
  } else {
    for (int64_t i = 0; i < n; ++i) {   // ObjectOutputStream: writeDouble = BE doubleToLongBits
      uint64_t v;
      std::memcpy(&v, (const char*)g + 8 * i, 8);
      v = __builtin_bswap64(v);
      std::memcpy(out + hl + 8 * i, &v, 8);
    }
  }
  javaser::write_pair_trailer(out + hl + 8 * n);
  return total;
}

int64_t dev_commit_partial(ipls_dev* h, int p, int32_t workers, uint8_t* out, int64_t out_cap) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  const int64_t L = h->len[p];
  const int64_t hl = javaser::pair_header_len(), total = hl + 8 * L + javaser::pair_trailer_len();
  if (!out) return total;
  if (out_cap < total) return fail(h, IPLS_E_RANGE, "partial update needs %lld bytes", (long long)total);
  HIP_TRY(h, dev_use(h->device));
  javaser::write_pair_header(out, workers, (int32_t)L);
  if (h->agg_zero[p]) {
    std::memset(out + hl, 0, (size_t)L * 8);   // +0.0 in any byte order
  } else {
    if (int rc = ensure_scratch(h, (size_t)L * 8)) return rc;
    launch_bswap(h->stream, (const unsigned long long*)(h->arena + h->agg_off[p]), (unsigned long long*)h->d_scratch, L);
    HIP_TRY(h, hipGetLastError());
    if (int rc = d2h(h, out + hl, h->d_scratch, (size_t)L * 8)) return rc;
  }
  javaser::write_pair_trailer(out + hl + 8 * L);
  return total;
}

int64_t dev_merge_files(ipls_dev* h, const uint8_t* const* files, const int64_t* lens, int k, int file_kind,
                             uint8_t* out, int64_t out_cap) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (k < 1 || !files || !lens) return fail(h, IPLS_E_INVAL, "need at least one file");
  if (file_kind != IPLS_HOST_BE && file_kind != IPLS_HOST_PAIR) return fail(h, IPLS_E_INVAL, "file_kind BE or PAIR");
  // decode every file's payload position first (GetParameters / Download_Partial_Updates)
  std::vector<int64_t> nd(k), off(k);
  for (int i = 0; i < k; ++i) {
    if (!files[i] && lens[i] > 0) return fail(h, IPLS_E_INVAL, "file %d is NULL", i);
    if (file_kind == IPLS_HOST_BE) {
      nd[i] = lens[i] / 8;
      off[i] = 0;
    } else {
      int32_t w;
      const char* why = nullptr;
      nd[i] = javaser::parse_pair(files[i], lens[i], &w, &off[i], &why);
      if (nd[i] < 0) return fail(h, IPLS_E_FORMAT, "file %d: %s (ObjectInputStream)", i, why ? why : "malformed");
    }
    if (i > 0 && nd[i] > nd[0])   // Aggregation[j] += Gradient[j] for j < Gradient.length (:244-246)
      return fail(h, IPLS_E_RANGE, "file %d has %lld doubles > %lld of the first "
                  "(ArrayIndexOutOfBoundsException, Decentralized_Storage_Receiver.java:245)", i,
                  (long long)nd[i], (long long)nd[0]);
  }
  const int64_t n0 = nd[0];
  if (out_cap < 8 * n0 || (!out && n0 > 0)) return fail(h, IPLS_E_RANGE, "merge output needs %lld bytes", (long long)(8 * n0));
  if (n0 == 0) return 0;
  HIP_TRY(h, dev_use(h->device));
  if (h->merge_cap < n0) {
    if (h->d_merge) {
      HIP_TRY(h, hipStreamSynchronize(h->stream));
      HIP_TRY(h, hipFree(h->d_merge));
      h->d_merge = nullptr;
      h->merge_cap = 0;
    }
    HIP_TRY(h, hipMalloc(&h->d_merge, (size_t)n0 * 8));
    h->merge_cap = n0;
  }
  for (int i = 0; i < k; ++i) {
    if (nd[i] == 0) continue;
    if (int rc = ensure_scratch(h, (size_t)nd[i] * 8)) return rc;
    if (int rc = stage_h2d(h, h->d_scratch, files[i] + off[i], (size_t)nd[i] * 8)) return rc;
    // (both device buffers come from hipMalloc: the tile shape)
    const bool vec = al16(h->d_merge) && al16(h->d_scratch);
    const dim3 g = ew_grid(nd[i], vec, 4096);
    auto msrc = (const unsigned long long*)h->d_scratch;
    if (i == 0) {   // Aggregation = GetParameters(Hashes.get(0)): the first file as is
      if (vec) hipLaunchKernelGGL((k_fold_n<true, true, true>), g, dim3(kBlock), 0, h->stream, h->d_merge, msrc, nd[i]);
      else hipLaunchKernelGGL((k_fold_n<true, true, false>), g, dim3(kBlock), 0, h->stream, h->d_merge, msrc, nd[i]);
    } else {
      if (vec) hipLaunchKernelGGL((k_fold_n<true, false, true>), g, dim3(kBlock), 0, h->stream, h->d_merge, msrc, nd[i]);
      else hipLaunchKernelGGL((k_fold_n<true, false, false>), g, dim3(kBlock), 0, h->stream, h->d_merge, msrc, nd[i]);
    }
    HIP_TRY(h, hipGetLastError());
  }
  // update_file(..., Aggregation): putDouble per element (MyIPFSClass.java:105-116)
  if (int rc = ensure_scratch(h, (size_t)n0 * 8)) return rc;
  launch_bswap(h->stream, (const unsigned long long*)h->d_merge, (unsigned long long*)h->d_scratch, n0);
  HIP_TRY(h, hipGetLastError());
  if (int rc = d2h(h, out, h->d_scratch, (size_t)n0 * 8)) return rc;
  return 8 * n0;
}

int64_t ipls_frame_encode(const double* g, int64_t n, int g_kind, int32_t a, int32_t b, int16_t pid,
                          const uint8_t* origin, int32_t origin_len, uint8_t* out, int64_t out_cap) {
  if (n < 0 || n > INT32_MAX || origin_len < 0 || !out || (n > 0 && !g) || (origin_len > 0 && !origin))
    return fail(nullptr, IPLS_E_INVAL, "bad argument");
  const int64_t total = 14 + 8 * n + origin_len;
  if (out_cap < total) return fail(nullptr, IPLS_E_RANGE, "frame needs %lld bytes", (long long)total);
  out[0] = (uint8_t)((uint16_t)pid >> 8);
  out[1] = (uint8_t)pid;
  const uint32_t hv[3] = {(uint32_t)n, (uint32_t)a, (uint32_t)b};
  for (int f = 0; f < 3; ++f)
    for (int i = 0; i < 4; ++i) out[2 + 4 * f + i] = (uint8_t)(hv[f] >> (24 - 8 * i));
  if (n > 0) {
    std::vector<double> tmp;
    const double* src = g;
    if (g_kind == IPLS_DEV_F64) {
      tmp.resize(n);
      if (hipMemcpy(tmp.data(), g, (size_t)n * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(nullptr, IPLS_E_DEVICE, "frame encode D2H failed");
      src = tmp.data();
    } else if (g_kind != IPLS_HOST_F64) {
      return fail(nullptr, IPLS_E_INVAL, "g_kind must be HOST_F64 or DEV_F64");
    }
    for (int64_t i = 0; i < n; ++i) {  // putDouble(14 + 8i, g[i]) -- raw bits, BE
      uint64_t v;
      std::memcpy(&v, &src[i], 8);
      v = __builtin_bswap64(v);
      std::memcpy(out + 14 + 8 * i, &v, 8);
    }
  }
  if (origin_len) std::memcpy(out + 14 + 8 * n, origin, (size_t)origin_len);
  return total;
}

// ---- Marshall_Packet of an accumulator, encoded on the device (a9) ----
// IPLS.java:1429-1430 publishes the aggregator's partial sum as
// Marshall_Packet(Aggregated_Gradients[p], id, iteration, workers + 1, 3):
// the frame (MyIPFSClass.java:990-1013) base64url-encoded with padding
// (:1016).  The text is produced by k_b64url_encode_frame straight from the
// accumulator: no host pass over the doubles, no blocking copy of them.
int64_t dev_publish(ipls_dev* h, int p, int target, int32_t a, int32_t b, int16_t pid, const uint8_t* origin,
                    int32_t origin_len, void* out, int64_t out_cap, int out_kind) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (int rc = check_part(h, p)) return rc;
  if (target_off(h, p, target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  if (origin_len < 0 || (origin_len > 0 && !origin)) return fail(h, IPLS_E_INVAL, "bad origin");
  if (out_kind != IPLS_HOST_TEXT && out_kind != IPLS_DEV_TEXT) return fail(h, IPLS_E_INVAL, "out_kind HOST_TEXT/DEV_TEXT");
  const int64_t n = h->len[p];
  const int64_t F = 14 + 8 * n + origin_len;
  const int64_t T = pubsub::b64_enc_len(F);
  if (!out) return T;
  if (out_cap < T) return fail(h, IPLS_E_RANGE, "publish text needs %lld bytes", (long long)T);
  HIP_TRY(h, dev_use(h->device));
  FrameEnc fe{};
  const uint32_t hv[3] = {(uint32_t)n, (uint32_t)a, (uint32_t)b};
  fe.hdr[0] = (unsigned char)((uint16_t)pid >> 8);   // putShort(0, pid)
  fe.hdr[1] = (unsigned char)pid;
  for (int f = 0; f < 3; ++f)                        // putInt(2 | 6 | 10, ...)
    for (int i = 0; i < 4; ++i) fe.hdr[2 + 4 * f + i] = (unsigned char)(hv[f] >> (24 - 8 * i));
  fe.n = n;
  fe.origin_len = origin_len;
  fe.origin = nullptr;
  if (origin_len > 0) {
    void* d = nullptr;
    if (int rc = upload_table(h, origin, (size_t)origin_len, &d)) return rc;
    fe.origin = (const unsigned char*)d;
  }
  uint8_t* zf = zero_flag(h, p, target);
  const unsigned long long* src =
      (zf && *zf) ? nullptr : (const unsigned long long*)(h->arena + target_off(h, p, target));
  unsigned char* dst = (unsigned char*)out;
  if (out_kind == IPLS_DEV_TEXT && !kernel_writable(out))
    return fail(h, IPLS_E_INVAL, "DEV_TEXT output is neither device memory nor pinned host memory");
  const bool dev_direct = out_kind == IPLS_DEV_TEXT && !((uintptr_t)out & 15);
  if (!dev_direct) {
    if (int rc = ensure_scratch(h, (size_t)T + 64)) return rc;
    dst = (unsigned char*)h->d_scratch;
  }
  const int64_t groups = (F + 23) / 24;
  hipLaunchKernelGGL(k_b64url_encode_frame, dim3(std::max(1u, std::min<unsigned>(blocks_for(groups, kBlock), 16384))),
                     dim3(kBlock), 0, h->stream, fe, src, dst, groups, T);
  HIP_TRY(h, hipGetLastError());
  if (out_kind == IPLS_DEV_TEXT) {
    // stream-ordered like every device-only call (the origin bytes were
    // already copied into the pinned upload ring)
    if (!dev_direct) HIP_TRY(h, hipMemcpyAsync(out, dst, (size_t)T, hipMemcpyDeviceToDevice, h->stream));
    return T;
  }
  if (int rc = d2h(h, out, dst, (size_t)T)) return rc;
  return T;
}

// Several partitions' publish texts in one launch (the loop over Auth_List,
// IPLS.java:1423-1431): text i of local partition parts[i] (field b = b[i])
// lands at out + offs[i], lens[i] bytes; offs are 64-byte multiples (the
// front lays them out).  HOST_TEXT: one D2H per text after the launch.
int64_t dev_publish_many(ipls_dev* h, int n, const int* parts, int target, int32_t a, const int32_t* b, int16_t pid,
                         const uint8_t* origin, int32_t origin_len, void* out, const int64_t* offs,
                         const int64_t* lens, int out_kind) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  if (n <= 0) return IPLS_OK;
  if (origin_len < 0 || (origin_len > 0 && !origin)) return fail(h, IPLS_E_INVAL, "bad origin");
  if (out_kind != IPLS_HOST_TEXT && out_kind != IPLS_DEV_TEXT) return fail(h, IPLS_E_INVAL, "out_kind HOST_TEXT/DEV_TEXT");
  for (int i = 0; i < n; ++i) {
    if (int rc = check_part(h, parts[i])) return rc;
    if (target_off(h, parts[i], target) < 0) return fail(h, IPLS_E_INVAL, "bad target %d", target);
  }
  HIP_TRY(h, dev_use(h->device));
  if (out_kind == IPLS_DEV_TEXT && !kernel_writable(out))
    return fail(h, IPLS_E_INVAL, "DEV_TEXT output is neither device memory nor pinned host memory");
  const unsigned char* dorig = nullptr;
  if (origin_len > 0) {
    void* d = nullptr;
    if (int rc = upload_table(h, origin, (size_t)origin_len, &d)) return rc;
    dorig = (const unsigned char*)d;
  }
  // texts land straight in a 16-B aligned device buffer; else in the scratch
  // buffer at the same offsets, then copied out
  const bool direct = out_kind == IPLS_DEV_TEXT && !((uintptr_t)out & 15);
  int64_t span = 0;
  for (int i = 0; i < n; ++i) span = std::max(span, offs[i] + lens[i]);
  int64_t lo = span;
  for (int i = 0; i < n; ++i) lo = std::min(lo, offs[i]);
  unsigned char* base = (unsigned char*)out;
  if (!direct) {
    if (int rc = ensure_scratch(h, (size_t)(span - lo) + 64)) return rc;
    base = (unsigned char*)h->d_scratch - lo;
  }
  std::vector<FrameJob> jobs(n);
  int64_t max_groups = 1;
  for (int i = 0; i < n; ++i) {
    const int p = parts[i];
    FrameJob& j = jobs[i];
    j = FrameJob{};
    const int64_t L = h->len[p];
    const uint32_t hv[3] = {(uint32_t)L, (uint32_t)a, (uint32_t)b[i]};
    j.f.hdr[0] = (unsigned char)((uint16_t)pid >> 8);   // putShort(0, pid)
    j.f.hdr[1] = (unsigned char)pid;
    for (int f = 0; f < 3; ++f)                         // putInt(2 | 6 | 10, ...)
      for (int k = 0; k < 4; ++k) j.f.hdr[2 + 4 * f + k] = (unsigned char)(hv[f] >> (24 - 8 * k));
    j.f.n = L;
    j.f.origin_len = origin_len;
    j.f.origin = dorig;
    uint8_t* zf = zero_flag(h, p, target);
    j.src = (zf && *zf) ? nullptr : (const unsigned long long*)(h->arena + target_off(h, p, target));
    j.out = base + offs[i];
    j.groups = (14 + 8 * L + origin_len + 23) / 24;
    j.text_len = lens[i];
    max_groups = std::max(max_groups, j.groups);
  }
  void* djobs = nullptr;
  if (int rc = upload_table(h, jobs.data(), jobs.size() * sizeof(FrameJob), &djobs)) return rc;
  const unsigned gx = std::max(1u, std::min<unsigned>(blocks_for(max_groups, kBlock), 16384));
  hipLaunchKernelGGL(k_b64url_encode_frames, dim3(gx, (unsigned)n), dim3(kBlock), 0, h->stream,
                     (const FrameJob*)djobs);
  HIP_TRY(h, hipGetLastError());
  if (direct) return IPLS_OK;                           // stream-ordered
  const hipMemcpyKind kind = out_kind == IPLS_DEV_TEXT ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  for (int i = 0; i < n; ++i)
    HIP_TRY(h, hipMemcpyAsync((unsigned char*)out + offs[i], base + offs[i], (size_t)lens[i], kind, h->stream));
  if (out_kind == IPLS_HOST_TEXT) HIP_TRY(h, hipStreamSynchronize(h->stream));
  return IPLS_OK;
}

// ---- engine plumbing used by the multi-device front (ipls_agg.cpp) ----
int dev_device(const ipls_dev* h) { return h ? h->device : -1; }

int dev_last_launch(const ipls_dev* h, ipls_launch_info* out) {
  if (!h || !out) return IPLS_E_INVAL;
  *out = h->last_launch;
  return IPLS_OK;
}

// Fixed-order fold of k device buckets per destination into caller device
// buffers that are NOT this engine's partitions (a replica slot's partial
// sums): lens[q] doubles each, dst[q] native doubles.  Same kernels, same
// order as reduce_batch_out.
int dev_reduce_ext(ipls_dev* h, int n, const int64_t* lens, const void* const* bufs, int k, bool be_in,
                   int start_mode, void* const* dst) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  IPLS_LOCK(h);
  HIP_TRY(h, dev_use(h->device));
  return reduce_dev(h, 0, n, bufs, k, be_in, start_mode, IPLS_TGT_AGG, dst, false, nullptr, false, lens);
}

// Collect_Replicas' length rule (IPLS.java:1225) over this engine's stored
// Other_Replica_Gradients, without folding anything.
int dev_other_check(ipls_dev* h) {
  if (!h) return fail(nullptr, IPLS_E_INVAL, "null handle");
  std::lock_guard<std::mutex> lk(h->mu);
  for (auto& kv : h->other)
    if (kv.second.n > h->len[kv.first.first])
      return fail(h, IPLS_E_RANGE, "stored replica of %lld doubles > partition %d length %lld "
                  "(ArrayIndexOutOfBoundsException, IPLS.java:1225)", (long long)kv.second.n,
                  kv.first.first + h->p_lo, (long long)h->len[kv.first.first]);
  return IPLS_OK;
}
