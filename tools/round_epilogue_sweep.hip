// round_epilogue_sweep.hip -- dev tool: where the fused round's extra time
// goes.  The fused round (k_round) writes two streams after
// the fold: W (Weights, aligned with the buckets) and the averages at the flat
// offsets p*(L-1) of GetPartitions (8 mod 16 for odd p).  This tool keeps the
// shipped fold and tile layout (R = 16, 1024 lanes, config C) and varies only
// the epilogue, interleaved in one process against the shipped kernels:
//   0 tool copy of the shipped epilogue: per vector r, W[r] then avg[r]
//   1 all 16 W stores first, then all 16 averages
//   2 all 16 averages first, then W
//   3 W with plain (cache-resident) stores, averages non-temporal
//   4 W non-temporal, averages plain
//   5 W only (no averages): the cost of the third stream
//   6 averages at 256-B aligned offsets (q*L) instead of p*(L-1): the cost of
//     the 8-mod-16 placement
//   7 as 2 (averages first), and for 8-mod-16 averages no single 8-B stores
//     inside a tile: each wave's last W value goes through LDS to the next
//     wave piece, whose lane 63 stores the pair (previous y, its lane 0's x),
//     so every lane stores one 16-B pair (singles only at the tile's ends)
//   8 wave pairs (round 3): vectors 2m and 2m+1 of a wave are adjacent 1 KiB
//     pieces (the wave owns 2 KiB contiguous per pair, the CU still sweeps one
//     32 KiB window per two vectors), averages first; for 8-mod-16 averages
//     lane 63 of piece 2m stores (its y, piece 2m+1's lane-0 x), so singles
//     fall every 2 KiB instead of every 1 KiB, with no LDS and no barrier
//   9 the wave-pair layout of 8 with the shipped epilogue (the load-pattern cost)
// Every variant that writes the real layout is checked bit-identical to the
// shipped k_round (W and averages).
// Usage: round_epilogue_sweep P L K REPS    (L a multiple of 32768)
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

template <bool NT>
__device__ __forceinline__ void st16(u64* p, d2 v) {
  if constexpr (NT) __builtin_nontemporal_store(encode2<false>(v), (gu2)p);
  else *(gu2)p = encode2<false>(v);
}

// one vector's averages (elements e, e+1) in the shipped placement
template <bool NT>
__device__ __forceinline__ void avg_store(u64* avg, bool aligned, int64_t e, int64_t L, int lane, double ax,
                                          double ay) {
  if (aligned) {
    if (e + 1 < L - 1) st16<NT>(avg + e, d2{ax, ay});
    else st8(avg + e, __builtin_bit_cast(u64, ax));
  } else {
    const double nx = __shfl_down(ax, 1);
    if (lane == 0) st8(avg + e, __builtin_bit_cast(u64, ax));
    if (lane < 63) st16<NT>(avg + e + 1, d2{ay, nx});
    else if (e + 1 < L - 1) st8(avg + e + 1, __builtin_bit_cast(u64, ay));
  }
}

// ZERO start, native doubles, REP logically zero, whole tiles only.
template <int V>
__global__ __launch_bounds__(1024) void k_ep(const u64* const* __restrict__ bufs, const PartDesc* __restrict__ parts,
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
  const int tid = threadIdx.x, lane = tid & 63;
  int64_t off[R];
  if constexpr (V == 8 || V == 9) {
    const int w = tid >> 6;
#pragma unroll
    for (int r = 0; r < R; ++r) off[r] = base + 2 * ((int64_t)(r >> 1) * 2 * BS + w * 128 + (r & 1) * 64 + lane);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) off[r] = base + 2 * ((int64_t)r * BS + tid);
  }
  d2 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = d2{0.0, 0.0};
  for (int j = 0; j < k; ++j) {
    const u64* __restrict__ src = pb[j];
    u2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = ld16<true>(src + off[r]);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const d2 x = decode2<false>(v[r]);
      acc[r].x = acc[r].x + x.x;
      acc[r].y = acc[r].y + x.y;
    }
  }
  const double cnt = cnts[q], den = cnt;
  const bool aligned = !((uintptr_t)avg & 15);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    acc[r].x = acc[r].x + 0.0;
    acc[r].y = acc[r].y + 0.0;
  }
  auto A = [&](int r, double& ax, double& ay) {
    ax = cnt == 0.0 ? acc[r].x : acc[r].x / den;
    ay = cnt == 0.0 ? acc[r].y : acc[r].y / den;
  };
  if constexpr (V == 0 || V == 3 || V == 4 || V == 6 || V == 9) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      st16<V != 3>(dst + off[r], acc[r]);
      double ax, ay;
      A(r, ax, ay);
      avg_store<V != 4>(avg, aligned, off[r], L, lane, ax, ay);
    }
  } else if constexpr (V == 1) {
#pragma unroll
    for (int r = 0; r < R; ++r) st16<true>(dst + off[r], acc[r]);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      double ax, ay;
      A(r, ax, ay);
      avg_store<true>(avg, aligned, off[r], L, lane, ax, ay);
    }
  } else if constexpr (V == 2) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      double ax, ay;
      A(r, ax, ay);
      avg_store<true>(avg, aligned, off[r], L, lane, ax, ay);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) st16<true>(dst + off[r], acc[r]);
  } else if constexpr (V == 7) {
    __shared__ double ylast[16][R];   // W value of lane 63 of wave w at vector r
    const int w = tid >> 6;
    if (lane == 63)
#pragma unroll
      for (int r = 0; r < R; ++r) ylast[w][r] = acc[r].y;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      double ax, ay;
      A(r, ax, ay);
      const int64_t e = off[r];
      if (aligned) {
        if (e + 1 < L - 1) st16<true>(avg + e, d2{ax, ay});
        else st8(avg + e, __builtin_bit_cast(u64, ax));
        continue;
      }
      const double nx = __shfl_down(ax, 1);
      const double x0 = __shfl(ax, 0);
      const bool first = (w == 0 && r == 0), last = (w == 15 && r == R - 1);
      if (lane < 63) {
        st16<true>(avg + e + 1, d2{ay, nx});
      } else {
        // the pair just before this wave piece: (predecessor's y, lane 0's x)
        if (!first) {
          const double py = w > 0 ? ylast[w - 1][r] : ylast[15][r - 1];
          const double pa = cnt == 0.0 ? py : py / den;
          st16<true>(avg + e - 127, d2{pa, x0});
        }
        if (last && e + 1 < L - 1) st8(avg + e + 1, __builtin_bit_cast(u64, ay));
      }
      if (first && lane == 0) st8(avg + e, __builtin_bit_cast(u64, ax));
    }
#pragma unroll
    for (int r = 0; r < R; ++r) st16<true>(dst + off[r], acc[r]);
  } else if constexpr (V == 8) {
#pragma unroll
    for (int m = 0; m < R; m += 2) {
      double ax, ay, bx, by;
      A(m, ax, ay);
      A(m + 1, bx, by);
      const int64_t e = off[m], f = off[m + 1];   // f = e + 128
      if (aligned) {
        st16<true>(avg + e, d2{ax, ay});
        if (f + 1 < L - 1) st16<true>(avg + f, d2{bx, by});
        else st8(avg + f, __builtin_bit_cast(u64, bx));
        continue;
      }
      const double nax = __shfl_down(ax, 1), nbx = __shfl_down(bx, 1);
      const double b0 = __shfl(bx, 0);
      if (lane == 0) st8(avg + e, __builtin_bit_cast(u64, ax));
      st16<true>(avg + e + 1, d2{ay, lane < 63 ? nax : b0});
      if (lane < 63) st16<true>(avg + f + 1, d2{by, nbx});
      else if (f + 1 < L - 1) st8(avg + f + 1, __builtin_bit_cast(u64, by));
    }
#pragma unroll
    for (int r = 0; r < R; ++r) st16<true>(dst + off[r], acc[r]);
  } else {  // 5: W only
#pragma unroll
    for (int r = 0; r < R; ++r) st16<true>(dst + off[r], acc[r]);
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
  const size_t nw = (size_t)P * dl * 8 + 4096, na = (size_t)P * L * 8 + 4096;

  // one W buffer + one averages buffer per variant; avg_stride: (L-1) = the
  // GetPartitions layout, dl = every partition's averages 256-B aligned
  struct Out {
    u64 *w = nullptr, *a = nullptr;
    PartDesc* d = nullptr;
  };
  auto make = [&](Out& o, int64_t avg_stride, bool with_avg) {
    CK(hipMalloc(&o.w, nw));
    CK(hipMalloc(&o.a, na + (size_t)P * 8 * 32));
    CK(hipMemset(o.a, 0xFF, na));
    auto* wb = (u64*)(((uintptr_t)o.w + 255) / 256 * 256);
    auto* ab = (u64*)(((uintptr_t)o.a + 255) / 256 * 256);
    std::vector<PartDesc> pd(P);
    for (int p = 0; p < P; ++p)
      pd[p] = PartDesc{L, wb + p * dl, wb + p * dl, nullptr, with_avg ? ab + (int64_t)p * avg_stride : nullptr};
    CK(hipMalloc(&o.d, P * sizeof(PartDesc)));
    CK(hipMemcpy(o.d, pd.data(), P * sizeof(PartDesc), hipMemcpyHostToDevice));
  };
  Out ship, red, v[10];
  make(ship, L - 1, true);
  make(red, L - 1, false);
  for (int i = 0; i < 10; ++i) make(v[i], i == 6 ? dl : L - 1, i != 5);

  struct Var {
    std::string name;
    std::function<void()> run;
    std::vector<float> ms;
    double bytes;
  };
  const double red_b = (double)P * (K + 1) * L * 8, round_b = (double)P * (K + 2) * L * 8;
  std::vector<Var> vars;
  vars.push_back({"shipped k_reduce", [&] {
                    hipLaunchKernelGGL((k_reduce<false, false, kZero, 1, 16, true, 0, 1024>), dim3(tpp * P),
                                       dim3(1024), 0, 0, bp, red.d, K, tpp, P);
                  }, {}, red_b});
  vars.push_back({"shipped k_round", [&] {
                    hipLaunchKernelGGL((k_round<false, kZero, 1, 16, 0, 1024>), dim3(tpp * P), dim3(1024), 0, 0, bp,
                                       ship.d, K, tpp, P, 0, d_cnt);
                  }, {}, round_b});
  const char* names[10] = {"0 tool copy: W[r], avg[r]", "1 all W, then all avg", "2 all avg, then all W",
                          "3 W plain stores, avg nt", "4 W nt, avg plain stores", "5 W only (no averages)",
                          "6 averages 256-B aligned", "7 avg first, LDS pair at wave ends",
                          "8 wave pairs, avg first, merged pair", "9 wave-pair loads, shipped epilogue"};
#define V(I)                                                                                                 \
  vars.push_back({names[I], [&] {                                                                            \
                    hipLaunchKernelGGL((k_ep<I>), dim3(tpp * P), dim3(1024), 0, 0, bp, v[I].d, K, tpp, d_cnt); \
                  }, {}, I == 5 ? red_b : round_b});
  V(0) V(1) V(2) V(3) V(4) V(5) V(6) V(7) V(8) V(9)
#undef V

  for (auto& x : vars) x.run();
  CK(hipDeviceSynchronize());
  {
    std::vector<unsigned char> a(na), b(na);
    for (int i : {0, 1, 2, 3, 4, 7, 8, 9}) {
      CK(hipMemcpy(a.data(), ship.a, na, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), v[i].a, na, hipMemcpyDeviceToHost));
      const bool avg_ok = !memcmp(a.data(), b.data(), na);
      CK(hipMemcpy(a.data(), ship.w, nw, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), v[i].w, nw, hipMemcpyDeviceToHost));
      const bool w_ok = !memcmp(a.data(), b.data(), nw);
      printf("# variant %d vs shipped k_round: averages %s, W %s\n", i, avg_ok ? "identical" : "MISMATCH",
             w_ok ? "identical" : "MISMATCH");
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < REPS; ++r)
    for (auto& x : vars) {
      CK(hipEventRecord(e0, 0));
      x.run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      x.ms.push_back(ms);
    }
  printf("# P=%d L=%lld K=%d PAD=%lld REPS=%d; bytes (K+1)*L*8*P for k_reduce and W-only, (K+2)*L*8*P otherwise\n",
         P, (long long)L, K, (long long)PAD, REPS);
  for (auto& x : vars) {
    std::sort(x.ms.begin(), x.ms.end());
    const double med = x.ms[x.ms.size() / 2];
    printf("%-34s median %8.4f ms  min %8.4f ms  %5.1f%% of 8 TB/s\n", x.name.c_str(), med, x.ms[0],
           x.bytes / med / 1e6 / 80.0);
  }
  return 0;
}
