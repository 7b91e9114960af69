// round_sweep.hip -- dev tool: the fused round (k_round, ipls_agg_aggregate_round)
// with a wave-contiguous tile layout, against the shipped kernel, interleaved
// in one process.
//
// Shipped layout: in step r the 16 waves of a 1024-lane block cover 16
// adjacent 1 KiB pieces (off = base + 2*(r*1024 + tid)); a partition whose
// averages start 8 mod 16 (odd p at the flat offsets p*(L-1)) writes them as
// 16-B pairs shifted by one lane, and every wave piece has two single 8-B
// stores at its ends -- partial 128-B lines every 1 KiB.
// Wave-contiguous ("WC"): wave w covers its own contiguous 16 KiB
// (off = base + 2*(w*64*R + r*64 + lane)), so its averages are one run; the
// lane-63 pair of piece r takes lane 0's x of piece r+1 (broadcast), and only
// the run's two ends are single stores.  The bucket loads change pattern too
// (16 streams 16 KiB apart per CU instead of one 16 KiB window), so plain
// k_reduce is timed in both layouts as well.
//
// Usage: round_sweep P L K REPS    (L a multiple of 32768: whole tiles)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../ipls-java-api_amd/csrc/ipls_kernels.hpp"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

using namespace ipls;
typedef unsigned long long u64;

// ZERO start, native doubles, REP logically zero, R = 16, 1024 lanes.
template <bool WC, bool FIN>
__global__ __launch_bounds__(1024) void k_var(const u64* const* __restrict__ bufs, const PartDesc* __restrict__ parts,
                                              int k, int tpp, const double* __restrict__ cnts) {
  constexpr int BS = 1024, R = 16;
  constexpr int64_t kTile = (int64_t)BS * 2 * R;
  const int q = blockIdx.x / tpp, t = blockIdx.x - q * tpp;
  const int64_t L = parts[q].len;
  const int64_t base = (int64_t)t * kTile;
  if (base + kTile > L) return;
  u64* __restrict__ dst = parts[q].dst;
  u64* __restrict__ avg = parts[q].avg;
  const u64* const* __restrict__ pb = bufs + (size_t)q * k;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t lb = WC ? base + 2 * (w * 64 * R + lane) : base + 2 * tid;
  int64_t off[R];
#pragma unroll
  for (int r = 0; r < R; ++r) off[r] = lb + (WC ? 128 : 2 * BS) * r;
  d2 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = d2{0.0, 0.0};
  for (int j = 0; j < k; ++j) {
    const u64* __restrict__ src = pb[j];
    u2 v[R];   // all R loads of a peer, then the adds (the shipped loop's shape)
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = ld16<true>(src + off[r]);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const d2 x = decode2<false>(v[r]);
      acc[r].x = acc[r].x + x.x;
      acc[r].y = acc[r].y + x.y;
    }
  }
  if constexpr (!FIN) {
#pragma unroll
    for (int r = 0; r < R; ++r) __builtin_nontemporal_store(encode2<false>(acc[r]), (gu2)(dst + off[r]));
    return;
  } else {
    const double cnt = cnts[q], den = cnt;
    const bool aligned = !((uintptr_t)avg & 15);
    double ay_prev = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      d2 wv = acc[r];
      wv.x = wv.x + 0.0;
      wv.y = wv.y + 0.0;
      __builtin_nontemporal_store(encode2<false>(wv), (gu2)(dst + off[r]));
      const int64_t e = off[r];
      const double ax = cnt == 0.0 ? wv.x : wv.x / den;
      const double ay = cnt == 0.0 ? wv.y : wv.y / den;
      if (aligned) {
        if (e + 1 < L - 1) __builtin_nontemporal_store(encode2<false>(d2{ax, ay}), (gu2)(avg + e));
        else st8(avg + e, __builtin_bit_cast(u64, ax));
      } else if (!WC) {
        const double nx = __shfl_down(ax, 1);
        if (lane == 0) st8(avg + e, __builtin_bit_cast(u64, ax));
        if (lane < 63) __builtin_nontemporal_store(encode2<false>(d2{ay, nx}), (gu2)(avg + e + 1));
        else if (e + 1 < L - 1) st8(avg + e + 1, __builtin_bit_cast(u64, ay));
      } else {
        const double nx = __shfl_down(ax, 1);
        const double x0 = __shfl(ax, 0);   // lane 0's x: the pair partner of lane 63 of piece r-1
        if (r == 0 && lane == 0) st8(avg + e, __builtin_bit_cast(u64, ax));
        if (r > 0 && lane == 63)
          __builtin_nontemporal_store(encode2<false>(d2{ay_prev, x0}), (gu2)(avg + off[r - 1] + 1));
        if (lane < 63) __builtin_nontemporal_store(encode2<false>(d2{ay, nx}), (gu2)(avg + e + 1));
        ay_prev = ay;
      }
    }
    if (WC && !aligned && lane == 63 && off[R - 1] + 1 < L - 1)
      st8(avg + off[R - 1] + 1, __builtin_bit_cast(u64, ay_prev));
  }
}

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 16;
  const int64_t L = argc > 2 ? atoll(argv[2]) : 4194304;
  const int K = argc > 3 ? atoi(argv[3]) : 32;
  const int REPS = argc > 4 ? atoi(argv[4]) : 20;
  const int64_t PAD = 32, stride = L + PAD;
  const int64_t tile = 32768;
  if (L % tile) {
    fprintf(stderr, "L must be a multiple of %lld\n", (long long)tile);
    return 2;
  }
  const int tpp = (int)(L / tile);
  u64* arena;
  CK(hipMalloc(&arena, (size_t)P * K * stride * 8 + 4096));
  auto* base = (u64*)(((uintptr_t)arena + 255) / 256 * 256);
  std::vector<const u64*> ptrs(P * K);
  for (int p = 0; p < P; ++p)
    for (int k = 0; k < K; ++k) {
      u64* b = base + (int64_t)(p * K + k) * stride;
      ptrs[p * K + k] = b;
      const u64 key = 0x1B52026ULL ^ ((u64)p << 40) ^ ((u64)k << 32);
      hipLaunchKernelGGL(k_synth<false>, dim3(4096), dim3(kBlock), 0, 0, b, L, key);
    }
  const u64** d_ptrs;
  CK(hipMalloc(&d_ptrs, ptrs.size() * 8));
  CK(hipMemcpy(d_ptrs, ptrs.data(), ptrs.size() * 8, hipMemcpyHostToDevice));
  auto bp = (const u64* const*)d_ptrs;
  double* d_cnt;
  std::vector<double> cnt(P, (double)K);
  CK(hipMalloc(&d_cnt, P * 8));
  CK(hipMemcpy(d_cnt, cnt.data(), P * 8, hipMemcpyHostToDevice));
  const int64_t dl = (L + 31) / 32 * 32;

  struct Out {
    u64 *w, *a;
  };
  auto make = [&](Out& o, std::vector<PartDesc>& pd, PartDesc*& d_pd, bool with_avg) {
    CK(hipMalloc(&o.w, (size_t)P * dl * 8 + 4096));
    CK(hipMalloc(&o.a, (size_t)P * L * 8 + 4096));
    CK(hipMemset(o.a, 0xFF, (size_t)P * L * 8 + 4096));
    auto* wb = (u64*)(((uintptr_t)o.w + 255) / 256 * 256);
    auto* ab = (u64*)(((uintptr_t)o.a + 255) / 256 * 256);
    pd.resize(P);
    for (int p = 0; p < P; ++p) pd[p] = PartDesc{L, wb + p * dl, nullptr, nullptr, with_avg ? ab + (int64_t)p * (L - 1) : nullptr};
    CK(hipMalloc(&d_pd, P * sizeof(PartDesc)));
    CK(hipMemcpy(d_pd, pd.data(), P * sizeof(PartDesc), hipMemcpyHostToDevice));
  };
  Out o_ship, o_wc, o_red, o_redwc;
  std::vector<PartDesc> pd_ship, pd_wc, pd_red, pd_redwc;
  PartDesc *d_ship, *d_wc, *d_red, *d_redwc;
  make(o_ship, pd_ship, d_ship, true);
  make(o_wc, pd_wc, d_wc, true);
  make(o_red, pd_red, d_red, false);
  make(o_redwc, pd_redwc, d_redwc, false);
  for (auto* v : {&pd_ship, &pd_wc})
    for (auto& x : *v) x.init = x.dst;

  struct Var {
    std::string name;
    std::function<void()> run;
    std::vector<float> ms;
    double bytes;
  };
  const double red_b = (double)P * (K + 1) * L * 8, round_b = (double)P * (K + 2) * L * 8;
  std::vector<Var> vars;
  vars.push_back({"shipped k_reduce (R=16, 1024 lanes)", [&] {
                    hipLaunchKernelGGL((k_reduce<false, false, kZero, 1, 16, true, 0, 1024>), dim3(tpp * P),
                                       dim3(1024), 0, 0, bp, d_red, K, tpp, P);
                  }, {}, red_b});
  vars.push_back({"WC k_reduce", [&] {
                    hipLaunchKernelGGL((k_var<true, false>), dim3(tpp * P), dim3(1024), 0, 0, bp, d_redwc, K, tpp,
                                       d_cnt);
                  }, {}, red_b});
  vars.push_back({"shipped k_round (avg at p*(L-1))", [&] {
                    hipLaunchKernelGGL((k_round<false, kZero, 1, 16, 0, 1024>), dim3(tpp * P), dim3(1024), 0, 0, bp,
                                       d_ship, K, tpp, P, 0, d_cnt);
                  }, {}, round_b});
  vars.push_back({"WC k_round (avg at p*(L-1))", [&] {
                    hipLaunchKernelGGL((k_var<true, true>), dim3(tpp * P), dim3(1024), 0, 0, bp, d_wc, K, tpp, d_cnt);
                  }, {}, round_b});
  vars.push_back({"tool k_round, shipped layout", [&] {
                    hipLaunchKernelGGL((k_var<false, true>), dim3(tpp * P), dim3(1024), 0, 0, bp, d_wc, K, tpp, d_cnt);
                  }, {}, round_b});

  // correctness: WC round == shipped round (W and averages, whole buffers)
  vars[0].run();
  vars[1].run();
  vars[2].run();
  vars[3].run();
  CK(hipDeviceSynchronize());
  {
    const size_t nw = (size_t)P * dl * 8 + 4096, na = (size_t)P * L * 8 + 4096;
    std::vector<unsigned char> a(std::max(nw, na)), b(std::max(nw, na));
    CK(hipMemcpy(a.data(), o_ship.a, na, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), o_wc.a, na, hipMemcpyDeviceToHost));
    printf("# WC averages vs shipped: %s\n", memcmp(a.data(), b.data(), na) ? "MISMATCH" : "identical");
    CK(hipMemcpy(a.data(), o_ship.w, nw, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), o_wc.w, nw, hipMemcpyDeviceToHost));
    printf("# WC W vs shipped: %s\n", memcmp(a.data(), b.data(), nw) ? "MISMATCH" : "identical");
    CK(hipMemcpy(a.data(), o_red.w, nw, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), o_redwc.w, nw, hipMemcpyDeviceToHost));
    printf("# WC k_reduce vs shipped: %s\n", memcmp(a.data(), b.data(), nw) ? "MISMATCH" : "identical");
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < REPS; ++r)
    for (auto& v : vars) {
      CK(hipEventRecord(e0, 0));
      v.run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  printf("# P=%d L=%lld K=%d PAD=%lld REPS=%d; k_reduce bytes (K+1)*L*8*P, k_round (K+2)*L*8*P\n", P, (long long)L, K,
         (long long)PAD, REPS);
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    printf("%-40s median %8.4f ms  min %8.4f ms  %5.1f%% of 8 TB/s\n", v.name.c_str(), med, v.ms[0],
           v.bytes / med / 1e6 / 80.0);
  }
  return 0;
}
