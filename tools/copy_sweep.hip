// copy_sweep.hip -- dev tool: block shapes of the two copy-shaped kernels of a
// round, k_finalize (AggregatePartition, W = AGG + REP, IPLS.java:1248-1274)
// and k_divide (GetPartitions, IPLS.java:1159-1174), timed in one process
// round-robin so every variant sees the same physical pages.
// The fold found that the contiguous bytes each CU streams are the lever
// (16 KiB -> 256 KiB: 67-85 % -> 84-89 %); this asks the same
// of the copies, which ship at 256 lanes x 4 vectors = 16 KiB per block.
//
// Usage: copy_sweep P L REPS      (default: config C, 16 x 4194304, 20)
// Algorithmic bytes: finalize 16 per element (read AGG, write W; REP
// logically zero), divide 16 per output element (read W, write the model).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

namespace ipls {
// The round-4 A/B form of k_divide (not shipped): ALIGNED = true reads W with
// 16-B loads whatever its alignment to the output; false is the shipped form.
// SWZ (round 5): blocks that share an XCD (b % 8) take a contiguous run of
// tiles (the guide's bijective T1 remap), so the W line a tile boundary splits
// is read by two blocks on one L2 instead of two L2s.
// WC (round 5): wave-contiguous steps -- a wave's V steps cover V adjacent
// KiB of the output instead of every wave of the block taking one KiB per
// step -- so that, with ALIGNED, the last lane's w[i+1] is lane 0's low half
// of the wave's NEXT step (a broadcast shuffle), and only the wave's last step
// reads one extra double: one shared line per V KiB instead of one per KiB.
template <bool OUT_BE, bool SECURE, int BS = kBlock, int V = kDivV, bool ALIGNED = false, bool SWZ = false,
          bool WC = false>
__global__ __launch_bounds__(BS) void k_divide_ab(const DivDesc* __restrict__ parts,
                                               const double* __restrict__ arena,
                                               unsigned long long* __restrict__ out,
                                               int tiles_per_part) {
  // The flat output offset p*chunk is arbitrary, so the tiles are laid over
  // the OUTPUT: block 0 first writes the `head` elements up to the first 128-B
  // line boundary of this partition's output, then every wave stores whole
  // lines (64 lanes x 16 B = 8 lines), and each lane reads its two W values
  // with 8-B loads (W's alignment relative to the output is arbitrary; reads
  // of partial lines cost little, partial-line writes do).
  // ALIGNED (the round-4 A/B): W read with 16-B loads whatever
  // its alignment to the output -- with the output's line boundary on an odd
  // W index, each lane loads the aligned pair [i-1, i], keeps its high half
  // and takes w[i+1] from the next lane's pair (__shfl_down; the wave's last
  // lane loads it itself).  The shipped two 8-B loads show 1.5 % more read
  // traffic than W's bytes (PMC), but the 16-B form reads 3.9 % more and
  // runs 6-8 % slower (tools/copy_sweep.hip, profiles/r04/d/).
  constexpr int kBlock = BS;
  constexpr int kV = V;
  constexpr int64_t kTile = (int64_t)kBlock * 2 * kV;
  unsigned b = blockIdx.x;
  if constexpr (SWZ) {
    const unsigned nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = b % 8;
    b = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
  }
  const int q = (int)b / tiles_per_part;
  const int t = (int)b - q * tiles_per_part;
  const DivDesc d = parts[q];
  const int64_t n = d.len - 1;
  const double* w = arena + d.w_off;
  const double cnt = w[d.len - 1];
  // Math.pow(10,12) * W[last] (IPLS.java:1167): 1e12 is exact, product rounded once.
  const double den = SECURE ? 1e12 * cnt : cnt;
  auto f = [&](double x) -> unsigned long long {
    const double y = (cnt == 0.0) ? x : x / den;
    unsigned long long bits = __builtin_bit_cast(unsigned long long, y);
    if constexpr (OUT_BE) {
      if (y != y) bits = 0x7ff8000000000000ULL;
      bits = __builtin_bswap64(bits);
    }
    return bits;
  };
  unsigned long long* o = out + d.out_off;
  const int64_t to_line = (16 - (int64_t)(((uintptr_t)o >> 3) & 15)) & 15;   // elements to a 128-B boundary
  const int64_t head = to_line < n ? to_line : n;
  if (t == 0 && threadIdx.x < head) o[threadIdx.x] = f(w[threadIdx.x]);
  const int64_t base = (int64_t)t * kTile + head;
  if (base >= n) return;
  // element index of lane threadIdx.x's pair at step v
  const int64_t wave_base = base + (int64_t)(threadIdx.x >> 6) * 128 * kV + 2 * (threadIdx.x & 63);
  auto idx = [&](int v) -> int64_t {
    if constexpr (WC) return wave_base + (int64_t)v * 128;
    return base + 2 * ((int64_t)v * kBlock + threadIdx.x);
  };
  if (base + kTile <= n) {
    double x[kV][2];
    if constexpr (ALIGNED && WC) {
      if ((((uintptr_t)(w + base)) & 15) == 0) {   // uniform per block
#pragma unroll
        for (int v = 0; v < kV; ++v) {
          const d2 a = __builtin_bit_cast(d2, __builtin_nontemporal_load((gcu2)(w + idx(v))));
          x[v][0] = a.x;
          x[v][1] = a.y;
        }
      } else {
        u2 a[kV];
#pragma unroll
        for (int v = 0; v < kV; ++v) a[v] = __builtin_nontemporal_load((gcu2)(w + idx(v) - 1));   // [i-1, i]
        const bool last = (threadIdx.x & 63) == 63;
        unsigned long long tail = 0;
        if (last) tail = __builtin_nontemporal_load((const __attribute__((address_space(1))) unsigned long long*)(w + idx(kV - 1) + 1));
#pragma unroll
        for (int v = 0; v < kV; ++v) {
          const unsigned long long lo = a[v].x;
          unsigned long long nx = __shfl_down(lo, 1, 64);          // w[i+1] = next lane's low half
          if (v + 1 < kV) {
            const unsigned long long first = __shfl((unsigned long long)a[v + 1].x, 0, 64);   // next step's lane 0
            if (last) nx = first;
          } else if (last) {
            nx = tail;
          }
          x[v][0] = __builtin_bit_cast(double, (unsigned long long)a[v].y);
          x[v][1] = __builtin_bit_cast(double, nx);
        }
      }
    } else if constexpr (ALIGNED) {
      if ((((uintptr_t)(w + base)) & 15) == 0) {   // uniform per block
#pragma unroll
        for (int v = 0; v < kV; ++v) {
          const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
          const d2 a = __builtin_bit_cast(d2, __builtin_nontemporal_load((gcu2)(w + i)));
          x[v][0] = a.x;
          x[v][1] = a.y;
        }
      } else {
        u2 a[kV];
#pragma unroll
        for (int v = 0; v < kV; ++v) {
          const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
          a[v] = __builtin_nontemporal_load((gcu2)(w + i - 1));   // [i-1, i]
        }
        const bool last = (threadIdx.x & 63) == 63;
#pragma unroll
        for (int v = 0; v < kV; ++v) {
          const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
          const unsigned long long lo = a[v].x;
          unsigned long long nx = __shfl_down(lo, 1, 64);          // w[i+1] = next lane's low half
          if (last) nx = *(const __attribute__((address_space(1))) unsigned long long*)(w + i + 1);
          x[v][0] = __builtin_bit_cast(double, (unsigned long long)a[v].y);
          x[v][1] = __builtin_bit_cast(double, nx);
        }
      }
    } else {
#pragma unroll
      for (int v = 0; v < kV; ++v) {
        const int64_t i = idx(v);
        x[v][0] = __builtin_nontemporal_load((const __attribute__((address_space(1))) double*)(w + i));
        x[v][1] = __builtin_nontemporal_load((const __attribute__((address_space(1))) double*)(w + i + 1));
      }
    }
#pragma unroll
    for (int v = 0; v < kV; ++v) {
      const int64_t i = idx(v);
      u2 v2;
      v2.x = f(x[v][0]);
      v2.y = f(x[v][1]);
      __builtin_nontemporal_store(v2, (gu2)(o + i));
    }
    return;
  }
  for (int64_t i = base + threadIdx.x; i < n; i += kBlock) o[i] = f(w[i]);
}

// k_finalize with wave-contiguous steps (round 5 A/B; REP logically zero, no
// accumulator zeroing: the sweep's shape of the shipped k_finalize<true, false>)
template <int BS = kBlock, int V = kFinV>
__global__ __launch_bounds__(BS) void k_finalize_wc(const FinDesc* __restrict__ parts, double* __restrict__ arena,
                                                    int tiles_per_part) {
  constexpr int64_t kTile = (int64_t)BS * 2 * V;
  const int q = blockIdx.x / tiles_per_part;
  const int t = blockIdx.x - q * tiles_per_part;
  const FinDesc d = parts[q];
  const int64_t base = (int64_t)t * kTile;
  if (base >= d.len) return;
  const int64_t end = (base + kTile < d.len) ? base + kTile : d.len;
  const double* agg = arena + d.agg_off;
  double* w = arena + d.w_off;
  if (end - base == kTile) {
    const int64_t wave_base = base + (int64_t)(threadIdx.x >> 6) * 128 * V + 2 * (threadIdx.x & 63);
    u2 a[V];
#pragma unroll
    for (int v = 0; v < V; ++v) a[v] = __builtin_nontemporal_load((gcu2)(agg + wave_base + (int64_t)v * 128));
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const d2 x = __builtin_bit_cast(d2, a[v]);
      d2 o;
      o.x = x.x + 0.0;
      o.y = x.y + 0.0;
      __builtin_nontemporal_store(__builtin_bit_cast(u2, o), (gu2)(w + wave_base + (int64_t)v * 128));
    }
    return;
  }
  for (int64_t i = base + threadIdx.x; i < end; i += BS) w[i] = agg[i] + 0.0;
}

// ---------------------------------------------------------------------------
}  // namespace ipls

struct Var {
  std::string name;
  double bytes;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 16;
  const int64_t L = argc > 2 ? atoll(argv[2]) : 4194304;
  const int REPS = argc > 3 ? atoi(argv[3]) : 20;
  // arena like the engine's: per partition AGG, REP, W, each 256-B aligned
  const int64_t La = (L + 31) / 32 * 32;
  double* arena;
  CK(hipMalloc(&arena, (size_t)P * 3 * La * 8));
  std::vector<FinDesc> fd(P);
  std::vector<DivDesc> dd(P);
  for (int p = 0; p < P; ++p) {
    fd[p] = FinDesc{L, (int64_t)p * 3 * La, (int64_t)p * 3 * La + La, (int64_t)p * 3 * La + 2 * La};
    dd[p] = DivDesc{L, fd[p].w_off, (int64_t)p * (L - 1)};   // flat model offsets p*chunk
    hipLaunchKernelGGL(k_synth<false>, dim3(4096), dim3(kBlock), 0, 0,
                       (unsigned long long*)(arena + fd[p].agg_off), L, 0x1B52026ULL ^ ((unsigned long long)p << 40));
  }
  unsigned long long* model;
  CK(hipMalloc(&model, (size_t)P * (L - 1) * 8 + 256));
  FinDesc* d_fd;
  DivDesc* d_dd;
  CK(hipMalloc(&d_fd, P * sizeof(FinDesc)));
  CK(hipMalloc(&d_dd, P * sizeof(DivDesc)));
  CK(hipMemcpy(d_fd, fd.data(), P * sizeof(FinDesc), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_dd, dd.data(), P * sizeof(DivDesc), hipMemcpyHostToDevice));
  // W = AGG once, so the divide reads a real model (count slot = synth value)
  hipLaunchKernelGGL((k_finalize<true, false>), dim3((unsigned)((L + kFinTile - 1) / kFinTile) * P), dim3(kBlock), 0,
                     0, d_fd, arena, (int)((L + kFinTile - 1) / kFinTile));
  CK(hipDeviceSynchronize());
  const double fin_bytes = (double)P * L * 16, div_bytes = (double)P * (L - 1) * 16;

  std::vector<Var> vars;
#define FIN(BS, V)                                                                                          \
  vars.push_back({"finalize BS=" #BS " V=" #V, fin_bytes, [=](hipStream_t s) {                              \
                    const int64_t tile = (int64_t)BS * 2 * V;                                                \
                    const int tpp = (int)((L + tile - 1) / tile);                                            \
                    hipLaunchKernelGGL((k_finalize<true, false, BS, V>), dim3((unsigned)tpp * P), dim3(BS), 0, s, \
                                       d_fd, arena, tpp);                                                    \
                  }})
#define DIVX(BS, V, AL, SW, TAG) DIVW(BS, V, AL, SW, false, TAG)
#define DIVW(BS, V, AL, SW, WC, TAG)                                                                            \
  vars.push_back({"divide   BS=" #BS " V=" #V TAG, div_bytes, [=](hipStream_t s) {                          \
                    const int64_t tile = (int64_t)BS * 2 * V;                                                \
                    const int tpp = (int)((L - 1 + tile - 1) / tile);                                        \
                    hipLaunchKernelGGL((k_divide_ab<false, false, BS, V, AL, SW, WC>), dim3((unsigned)tpp * P), dim3(BS), 0, s, \
                                       d_dd, (const double*)arena, model, tpp);                              \
                  }})
#define DIV(BS, V) DIVX(BS, V, false, false, "")
  FIN(256, 8);   // shipped (kFinV = 8)
  FIN(256, 4);
#define FINW(BS, V)                                                                                         \
  vars.push_back({"finalize BS=" #BS " V=" #V " wc", fin_bytes, [=](hipStream_t s) {                         \
                    const int64_t tile = (int64_t)BS * 2 * V;                                                \
                    const int tpp = (int)((L + tile - 1) / tile);                                            \
                    hipLaunchKernelGGL((k_finalize_wc<BS, V>), dim3((unsigned)tpp * P), dim3(BS), 0, s,     \
                                       d_fd, arena, tpp);                                                    \
                  }})
  FINW(256, 8);
  FINW(256, 4);
#undef FINW
  DIVX(256, 4, false, false, " 8B");   // round 4's shipped form: two 8-B loads per lane
  DIVX(256, 4, true, false, " 16B");   // round-4 A/B: 16-B loads whatever the alignment
  DIVW(256, 4, false, false, true, " 8B wc");    // shipped since round 5: wave-contiguous steps
  DIVW(256, 4, true, false, true, " 16B wc");
  DIVW(256, 8, true, false, true, " 16B wc");
  DIVW(256, 16, true, false, true, " 16B wc");
#undef FIN
#undef DIV
#undef DIVX
#undef DIVW
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // warm + check: each variant's whole output (W of every partition, or the
  // flat model) after poisoning it must checksum like the shipped shape's
  unsigned long long* d_sum;
  CK(hipMalloc(&d_sum, 8));
  unsigned long long want[2] = {0, 0};
  bool all_ok = true;
  for (auto& v : vars) {
    const bool fin = v.name[0] == 'f';
    if (fin)
      for (int p = 0; p < P; ++p) CK(hipMemsetAsync(arena + fd[p].w_off, 0xA5, (size_t)L * 8, s));
    else
      CK(hipMemsetAsync(model, 0xA5, (size_t)P * (L - 1) * 8, s));
    v.run(s);
    unsigned long long sum = 0;
    for (int p = 0; p < (fin ? P : 1); ++p) {
      CK(hipMemsetAsync(d_sum, 0, 8, s));
      const unsigned long long* x = fin ? (const unsigned long long*)(arena + fd[p].w_off) : model;
      hipLaunchKernelGGL(k_checksum<false>, dim3(2048), dim3(kBlock), 0, s, x, fin ? L : (int64_t)P * (L - 1), d_sum);
      unsigned long long c = 0;
      CK(hipMemcpyAsync(&c, d_sum, 8, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      sum = sum * 31 + c;
    }
    unsigned long long& w = want[fin ? 0 : 1];
    if (!w) w = sum;
    if (sum != w) {
      all_ok = false;
      printf("MISMATCH %s\n", v.name.c_str());
    }
  }
  printf("# outputs identical across shapes: %s\n", all_ok ? "yes" : "NO");
  for (int r = 0; r < REPS; ++r)
    for (auto& v : vars) {
      CK(hipEventRecord(a, s));
      v.run(s);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      v.ms.push_back(ms);
    }
  CK(hipGetLastError());
  printf("# P=%d L=%lld REPS=%d  finalize %.0f B, divide %.0f B per launch\n", P, (long long)L, REPS, fin_bytes,
         div_bytes);
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    printf("%-24s median %8.4f ms  min %8.4f ms  %8.1f GB/s (median)  %5.1f%% of 8 TB/s\n", v.name.c_str(), med,
           v.ms[0], v.bytes / (med * 1e-3) / 1e9, 100.0 * v.bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
