// ab_sweep.hip -- dev tool: same-process A/B of the shipped k_reduce against a
// previous revision of ipls_kernels.hpp (built from git into namespace
// ipls_old by tools/ab_build.sh), interleaved round-robin so both see the same
// bucket layout (layout moves results by +-5 % across processes).
//
// Usage: ab_sweep P L K PAD REPS
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../ipls-java-api_amd/csrc/ipls_kernels.hpp"
#include AB_OLD_HEADER

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e = (x);                                                                     \
    if (e != hipSuccess) {                                                                  \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));      \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

struct Var {
  std::string name;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};

// Descriptors in the OLD revision's layout: the two revisions' PartDesc may
// differ (a field added), so an old kernel never reads a new-layout table.
static ipls_old::PartDesc* to_old(const std::vector<ipls::PartDesc>& v) {
  std::vector<ipls_old::PartDesc> o(v.size());
  for (size_t i = 0; i < v.size(); ++i) {
    o[i] = ipls_old::PartDesc{};
    o[i].len = v[i].len;
    o[i].dst = v[i].dst;
    o[i].init = v[i].init;
    o[i].rep = v[i].rep;
    o[i].avg = v[i].avg;
  }
  ipls_old::PartDesc* d;
  CK(hipMalloc(&d, o.size() * sizeof(ipls_old::PartDesc)));
  CK(hipMemcpy(d, o.data(), o.size() * sizeof(ipls_old::PartDesc), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 16;
  const int64_t L = argc > 2 ? atoll(argv[2]) : 4194304;
  const int K = argc > 3 ? atoi(argv[3]) : 32;
  const int64_t PAD = argc > 4 ? atoll(argv[4]) : 32;
  const int REPS = argc > 5 ? atoi(argv[5]) : 10;
  const int64_t stride = L + PAD;
  unsigned long long* arena;
  CK(hipMalloc(&arena, (size_t)P * K * stride * 8 + 4096));
  auto* base = (unsigned long long*)(((uintptr_t)arena + 255) / 256 * 256);
  std::vector<const unsigned long long*> ptrs(P * K);
  for (int p = 0; p < P; ++p)
    for (int k = 0; k < K; ++k) {
      unsigned long long* b = base + (int64_t)(p * K + k) * stride;
      ptrs[p * K + k] = b;
      const unsigned long long key = 0x1B52026ULL ^ ((unsigned long long)p << 40) ^ ((unsigned long long)k << 32);
      hipLaunchKernelGGL(ipls::k_synth<false>, dim3(4096), dim3(ipls::kBlock), 0, 0, b, L, key);
    }
  const unsigned long long** d_ptrs;
  CK(hipMalloc(&d_ptrs, ptrs.size() * 8));
  CK(hipMemcpy(d_ptrs, ptrs.data(), ptrs.size() * 8, hipMemcpyHostToDevice));
  const int64_t dl = (L + 31) / 32 * 32;
  unsigned long long* dst;
  CK(hipMalloc(&dst, (size_t)P * dl * 8));
  std::vector<ipls::PartDesc> pd(P);
  for (int p = 0; p < P; ++p) pd[p] = ipls::PartDesc{L, dst + p * dl, nullptr, nullptr, nullptr};
  ipls::PartDesc* d_pd;
  CK(hipMalloc(&d_pd, P * sizeof(ipls::PartDesc)));
  CK(hipMemcpy(d_pd, pd.data(), P * sizeof(ipls::PartDesc), hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  const double alg = (double)P * (K + 1) * L * 8;
  const int64_t tile = 1024 * 2 * 16;
  const int tpp = (int)((L + tile - 1) / tile);
  auto bp = (const unsigned long long* const*)d_ptrs;
  const ipls_old::PartDesc* opd = to_old(pd);
  std::vector<Var> vars;
  vars.push_back({"old k_reduce f64 R=16 MAP=0", [=](hipStream_t s) {
                    hipLaunchKernelGGL((ipls_old::k_reduce<false, false, ipls_old::kZero, 1, 16, true, 0, 1024>),
                                       dim3(tpp * P), dim3(1024), 0, s, bp, opd, K, tpp, P);
                  }});
  vars.push_back({"new k_reduce f64 R=16 MAP=0", [=](hipStream_t s) {
                    hipLaunchKernelGGL((ipls::k_reduce<false, false, ipls::kZero, 1, 16, true, 0, 1024>),
                                       dim3(tpp * P), dim3(1024), 0, s, bp, d_pd, K, tpp, P);
                  }});
  if (L % tile)
    vars.push_back({"new k_reduce f64 R=16 MAP=3 (partial tiles first)", [=](hipStream_t s) {
                      hipLaunchKernelGGL((ipls::k_reduce<false, false, ipls::kZero, 1, 16, true, 3, 1024>),
                                         dim3(tpp * P), dim3(1024), 0, s, bp, d_pd, K, tpp, P);
                    }});
  // fused round (k_round, new kernels only): averages written at the real flat
  // offsets p*(L-1) (mostly not 128-B aligned) vs at 256-B aligned offsets,
  // vs no averages (SWEEP_ROUND=1)
  std::vector<ipls::PartDesc> rpd[3];
  ipls::PartDesc* d_rpd[3] = {nullptr, nullptr, nullptr};
  double* d_cnt = nullptr;
  unsigned long long* avg = nullptr;
  if (getenv("SWEEP_ROUND")) {
    CK(hipMalloc(&avg, (size_t)P * dl * 8 + 4096));
    std::vector<double> cnt(P, (double)K);
    CK(hipMalloc(&d_cnt, P * 8));
    CK(hipMemcpy(d_cnt, cnt.data(), P * 8, hipMemcpyHostToDevice));
    for (int v = 0; v < 3; ++v) {
      rpd[v] = pd;
      for (int p = 0; p < P; ++p) {
        rpd[v][p].init = pd[p].dst;
        rpd[v][p].avg = v == 0 ? avg + (int64_t)p * (L - 1) : v == 1 ? avg + p * dl : nullptr;
      }
      CK(hipMalloc(&d_rpd[v], P * sizeof(ipls::PartDesc)));
      CK(hipMemcpy(d_rpd[v], rpd[v].data(), P * sizeof(ipls::PartDesc), hipMemcpyHostToDevice));
    }
    const char* names[3] = {"k_round, averages at p*(L-1) (real)", "k_round, averages 256-B aligned",
                            "k_round, no averages"};
    {
      const ipls_old::PartDesc* odp = to_old(rpd[0]);
      vars.push_back({"old k_round, averages at p*(L-1) (real)", [=](hipStream_t s) {
                        hipLaunchKernelGGL((ipls_old::k_round<false, ipls_old::kZero, 1, 16, 0, 1024>), dim3(tpp * P),
                                           dim3(1024), 0, s, bp, odp, K, tpp, P, 0, d_cnt);
                      }});
    }
    for (int v = 0; v < 3; ++v) {
      ipls::PartDesc* dp = d_rpd[v];
      vars.push_back({names[v], [=](hipStream_t s) {
                        hipLaunchKernelGGL((ipls::k_round<false, ipls::kZero, 1, 16, 0, 1024>), dim3(tpp * P),
                                           dim3(1024), 0, s, bp, dp, K, tpp, P, 0, d_cnt);
                      }});
    }
  }
  // alignment probes (SWEEP_ALIGN=1): what misaligned 16-B loads/stores cost.
  //  - k_reduce on buckets shifted by one double (every dwordx4 load 8 mod 16)
  //  - k_round with the averages at 8 mod 16 / 16 mod 128 / 128-B aligned for
  //    every partition, and with W (dst) shifted by one double
  std::vector<ipls::PartDesc> apd[5];
  if (getenv("SWEEP_ALIGN")) {
    const unsigned long long** d_ptrs1;
    std::vector<const unsigned long long*> p1(ptrs);
    for (auto& x : p1) x += 1;
    CK(hipMalloc(&d_ptrs1, p1.size() * 8));
    CK(hipMemcpy(d_ptrs1, p1.data(), p1.size() * 8, hipMemcpyHostToDevice));
    auto bp1 = (const unsigned long long* const*)d_ptrs1;
    const int64_t L1 = L - 1;   // the shifted buckets hold L-1 valid doubles before the pad
    std::vector<ipls::PartDesc> pd1(pd);
    for (auto& x : pd1) x.len = L1 - (L1 % tile);   // whole tiles only
    ipls::PartDesc* d_pd1;
    CK(hipMalloc(&d_pd1, P * sizeof(ipls::PartDesc)));
    CK(hipMemcpy(d_pd1, pd1.data(), P * sizeof(ipls::PartDesc), hipMemcpyHostToDevice));
    const int tpp1 = (int)(pd1[0].len / tile);
    ipls::PartDesc* d_pd0;
    std::vector<ipls::PartDesc> pd0(pd1);
    CK(hipMalloc(&d_pd0, P * sizeof(ipls::PartDesc)));
    CK(hipMemcpy(d_pd0, pd0.data(), P * sizeof(ipls::PartDesc), hipMemcpyHostToDevice));
    vars.push_back({"k_reduce, aligned loads (same tiles)", [=](hipStream_t s) {
                      hipLaunchKernelGGL((ipls::k_reduce<false, false, ipls::kZero, 1, 16, true, 0, 1024>),
                                         dim3(tpp1 * P), dim3(1024), 0, s, bp, d_pd0, K, tpp1, P);
                    }});
    const bool mis = getenv("SWEEP_MISALIGNED") != nullptr;   // unaligned 16-B global accesses
    if (mis)
      vars.push_back({"k_reduce, loads 8 mod 16 (misaligned)", [=](hipStream_t s) {
                        hipLaunchKernelGGL((ipls::k_reduce<false, false, ipls::kZero, 1, 16, true, 0, 1024>),
                                           dim3(tpp1 * P), dim3(1024), 0, s, bp1, d_pd1, K, tpp1, P);
                      }});
    double* cnt;
    CK(hipMalloc(&cnt, P * 8));
    std::vector<double> cv(P, (double)K);
    CK(hipMemcpy(cnt, cv.data(), P * 8, hipMemcpyHostToDevice));
    unsigned long long* av;
    CK(hipMalloc(&av, (size_t)P * dl * 8 + 8192));
    auto* avb = (unsigned long long*)(((uintptr_t)av + 255) / 256 * 256);
    unsigned long long* wd;
    CK(hipMalloc(&wd, (size_t)P * dl * 8 + 8192));
    auto* wdb = (unsigned long long*)(((uintptr_t)wd + 255) / 256 * 256);
    const char* names[5] = {"k_round, avg 128-B aligned", "k_round, avg 16 mod 128", "k_round, avg 8 mod 16",
                            "k_round, avg 128-B aligned, W 8 mod 16", "k_round, avg+W 8 mod 16"};
    const int avg_shift[5] = {0, 2, 1, 0, 1}, w_shift[5] = {0, 0, 0, 1, 1};
    for (int v = 0; v < (mis ? 5 : 3); ++v) {
      apd[v] = pd1;
      for (int p = 0; p < P; ++p) {
        apd[v][p].dst = wdb + p * dl + w_shift[v];
        apd[v][p].init = apd[v][p].dst;
        apd[v][p].avg = avb + p * dl + avg_shift[v];
      }
      ipls::PartDesc* dp;
      CK(hipMalloc(&dp, P * sizeof(ipls::PartDesc)));
      CK(hipMemcpy(dp, apd[v].data(), P * sizeof(ipls::PartDesc), hipMemcpyHostToDevice));
      vars.push_back({names[v], [=](hipStream_t s) {
                        hipLaunchKernelGGL((ipls::k_round<false, ipls::kZero, 1, 16, 0, 1024>), dim3(tpp1 * P),
                                           dim3(1024), 0, s, bp, dp, K, tpp1, P, 0, cnt);
                      }});
    }
  }
  // (SWEEP_ROUND2, the tile-shift experiment of profiles/r02/ab_round_line_shift.txt,
  // ran against a kernel revision that was not adopted; see that file.)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vars) v.run(0);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < REPS; ++r)
    for (auto& v : vars) {
      CK(hipEventRecord(e0, 0));
      v.run(0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  printf("# P=%d L=%lld K=%d PAD=%lld REPS=%d  algorithmic bytes/launch=%.0f\n", P, (long long)L, K, (long long)PAD,
         REPS, alg);
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    printf("%-52s median %8.4f ms  min %8.4f ms  %5.1f%% of 8 TB/s\n", v.name.c_str(), med, v.ms[0],
           alg / med / 1e6 / 80.0);
  }
  return 0;
}
