// host_e2e.cpp -- dev tool: host-inclusive aggregation rate through the C-ABI
// alone (what a JNI caller sees), without the Python/ctypes layer of bench.py.
//
// Usage: host_e2e L K REPS
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
  CK(ipls_agg_close(h));
  return 0;
}
