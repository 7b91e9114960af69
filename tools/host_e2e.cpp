// host_e2e.cpp -- dev tool: host-inclusive aggregation rate through the C-ABI
// alone (what a JNI caller sees), without the Python/ctypes layer of bench.py.
//
// Usage: host_e2e L K REPS [P [--device-only]]   (P: also the device-resident per-arrival legs)
// K big-endian buckets of L doubles (update_file bytes) start in host memory;
// one round = K arrivals folded into AGG[0] + AggregatePartition with the BE
// sum written back to host memory (commit_update's update_file image).
// Algorithmic bytes per round: (K+1) * L * 8, as bench.py's host_inclusive.
// Modes: pinned per-arrival (ipls_agg_accumulate), pinned queued
// (ipls_agg_accumulate_async + one wait at finalize), pinned batched
// (ipls_agg_reduce_batch over the host pointers), pageable per-arrival.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "ipls_agg.h"

#define CK(x)                                                                             \
  do {                                                                                    \
    int rc_ = (x);                                                                        \
    if (rc_) {                                                                            \
      fprintf(stderr, "%s:%d %s = %d (%s)\n", __FILE__, __LINE__, #x, rc_,               \
              h ? ipls_agg_last_error(h) : "");                                           \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void fill_be(uint8_t* b, int64_t L, int k) {
  for (int64_t i = 0; i < L; ++i) {
    double v = (i == L - 1) ? 1.0 : ((double)((i * 7 + k * 13) % 2001) - 1000.0) * 1e-5;
    uint64_t u;
    std::memcpy(&u, &v, 8);
    u = __builtin_bswap64(u);
    std::memcpy(b + 8 * i, &u, 8);
  }
}

int main(int argc, char** argv) {
  const int64_t L = argc > 1 ? atoll(argv[1]) : 4194304;
  const int K = argc > 2 ? atoi(argv[2]) : 32;
  const int REPS = argc > 3 ? atoi(argv[3]) : 4;
  const size_t bytes = (size_t)L * 8;
  ipls_agg* h = nullptr;
  ipls_agg_cfg cfg{};
  cfg.n_partitions = 1;
  cfg.bucket_len = L;
  CK(ipls_agg_open(&cfg, &h));
  const bool device_only = argc > 5 && std::strcmp(argv[5], "--device-only") == 0;
  if (device_only) goto device_legs;
  {
  std::vector<void*> pinned(K);
  std::vector<uint8_t*> pageable(K);
  for (int k = 0; k < K; ++k) {
    CK(ipls_host_alloc(bytes, &pinned[k]));
    fill_be((uint8_t*)pinned[k], L, k);
    pageable[k] = (uint8_t*)malloc(bytes);
    std::memcpy(pageable[k], pinned[k], bytes);
  }
  void* sum = nullptr;
  CK(ipls_host_alloc(bytes, &sum));
  const double alg = (double)(K + 1) * bytes;
  printf("# L=%lld K=%d REPS=%d  algorithmic bytes/round=%.0f (C-ABI only, no Python)\n", (long long)L, K, REPS, alg);

  auto run = [&](const char* name, const std::function<void()>& round) {
    round();   // warm
    double best = 1e30, tot = 0;
    for (int r = 0; r < REPS; ++r) {
      const double t0 = now();
      round();
      const double dt = now() - t0;
      best = std::min(best, dt);
      tot += dt;
    }
    printf("%-40s mean %7.2f GB/s  best %7.2f GB/s\n", name, alg * REPS / tot / 1e9, alg / best / 1e9);
  };
  run("pinned, per arrival (accumulate)", [&] {
    for (int k = 0; k < K; ++k) CK(ipls_agg_accumulate(h, 0, IPLS_TGT_AGG, pinned[k], L, IPLS_HOST_BE));
    CK(ipls_agg_finalize(h, 0, sum, IPLS_HOST_BE, nullptr));
  });
  run("pinned, per arrival, queued (async)", [&] {
    uint64_t t = 0;
    for (int k = 0; k < K; ++k) CK(ipls_agg_accumulate_async(h, 0, IPLS_TGT_AGG, pinned[k], L, IPLS_HOST_BE, &t));
    CK(ipls_agg_finalize(h, 0, sum, IPLS_HOST_BE, nullptr));
  });
  run("pinned, batched (reduce_batch)", [&] {
    CK(ipls_agg_reduce_batch(h, 0, 1, (const void* const*)pinned.data(), K, IPLS_DEV_BE, IPLS_START_ZERO,
                             IPLS_TGT_AGG));
    CK(ipls_agg_finalize(h, 0, sum, IPLS_HOST_BE, nullptr));
  });
  run("pageable, per arrival (accumulate)", [&] {
    for (int k = 0; k < K; ++k) CK(ipls_agg_accumulate(h, 0, IPLS_TGT_AGG, pageable[k], L, IPLS_HOST_BE));
    CK(ipls_agg_finalize(h, 0, sum, IPLS_HOST_BE, nullptr));
  });
  for (int k = 0; k < K; ++k) {
    ipls_host_free(pinned[k]);
    free(pageable[k]);
  }
  ipls_host_free(sum);
  }
device_legs:
  CK(ipls_agg_close(h));

  // Device-resident buckets, one call per arrival as a native (JNI-like)
  // caller makes them: P partitions x K peers, peers arriving in turn.  The
  // K buckets live in a second handle's AGG arrays (filled by ipls_synth_fill)
  // and are reused for every partition (the timing does not depend on values).
  // Time = wall clock around the P*K calls + the final wait; bytes = the
  // batch's P*(K+1)*L*8.
  if (argc > 4) {
    const int P = atoi(argv[4]);
    ipls_agg* src = nullptr;
    ipls_agg_cfg sc{};
    sc.n_partitions = K;
    sc.bucket_len = L;
    h = nullptr;
    CK(ipls_agg_open(&sc, &src));
    std::vector<const void*> dev(K);
    for (int k = 0; k < K; ++k) {
      void* d = nullptr;
      CK(ipls_agg_device_ptr(src, k, IPLS_TGT_AGG, &d));
      CK(ipls_synth_fill(d, L, 0x1B52026ULL, 0, k, IPLS_DEV_F64, ipls_agg_stream(src)));
      dev[k] = d;
    }
    CK(ipls_agg_sync(src));
    ipls_agg_cfg dc{};
    dc.n_partitions = P;
    dc.bucket_len = L;
    CK(ipls_agg_open(&dc, &h));
    const double algd = (double)P * (K + 1) * bytes;
    printf("# device-resident, one call per arrival: P=%d x K=%d x L=%lld, algorithmic bytes=%.0f\n", P, K,
           (long long)L, algd);
    auto drun = [&](const char* name, const std::function<void()>& round) {
      round();
      double best = 1e30;
      for (int r = 0; r < REPS; ++r) {
        CK(ipls_agg_reset(h, IPLS_ALL_PARTITIONS));
        CK(ipls_agg_sync(h));
        const double t0 = now();
        round();
        best = std::min(best, now() - t0);
      }
      printf("%-40s best %8.3f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", name, best * 1e3, algd / best / 1e9,
             algd / best / 1e9 / 80.0);
    };
    drun("device, one launch per arrival", [&] {
      for (int k = 0; k < K; ++k)
        for (int p = 0; p < P; ++p) CK(ipls_agg_accumulate(h, p, IPLS_TGT_AGG, dev[k], L, IPLS_DEV_F64));
      CK(ipls_agg_sync(h));
    });
    drun("device, queued (accumulate_async)", [&] {
      uint64_t t = 0;
      for (int k = 0; k < K; ++k)
        for (int p = 0; p < P; ++p) CK(ipls_agg_accumulate_async(h, p, IPLS_TGT_AGG, dev[k], L, IPLS_DEV_F64, &t));
      CK(ipls_agg_wait(h, t));
    });
    std::vector<const void*> tab((size_t)P * K);
    for (int p = 0; p < P; ++p)
      for (int k = 0; k < K; ++k) tab[(size_t)p * K + k] = dev[k];
    drun("device, one reduce_batch", [&] {
      CK(ipls_agg_reduce_batch(h, 0, P, tab.data(), K, IPLS_DEV_F64, IPLS_START_ZERO, IPLS_TGT_AGG));
      CK(ipls_agg_sync(h));
    });
    CK(ipls_agg_close(h));
    h = src;
    CK(ipls_agg_close(src));
  }
  return 0;
}
