// elementwise_sweep.hip -- dev tool (round 4): the per-arrival elementwise
// kernels of the -async variants and the replica store, as the engine
// launches them (grid-stride, one 8-B element per lane per step), against
// 16-B-vector tile forms of the same arithmetic, in one process, outputs
// compared bit for bit.
//   k_blend  t = a*t + b*g   (async replica fold Updater.java:57-59; leaving
//                             peer :65-69)                    24 B / element
//   k_scale  d = c*s         (async publish 0.25*W :197-199)  16 B / element
//   k_fold_n dst += src      (Other_Replica_Gradients fold,
//                             Download_Scheduler.java:254-260) 24 B / element
// "product" rows: the shipped kernels' VEC form; "grid-stride": their
// unaligned fallback (round 3's only form).
// Timing: REPS rounds, the variant order rotated by one every round, and
// every timed launch from cold caches (a 1 GiB memset before it).
// Usage: elementwise_sweep N REPS     (default 4194304 = one config-C partition;
// at that size the operands fit the 256 MB Infinity Cache -- 67108864 is HBM)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../ipls-java-api_amd/csrc/ipls_kernels.hpp"

using namespace ipls;

// as engine.hip computes its grids
static unsigned blocks_for(int64_t n, int64_t per_block) { return (unsigned)((n + per_block - 1) / per_block); }

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

// Tile forms: a block of 256 lanes owns 256*2*V consecutive elements, each
// lane V 16-B vectors (lane-contiguous 1 KiB per wave per vector); the last
// partial tile goes element by element.  Operands 16-B aligned (checked on
// the host).  NTS: non-temporal stores.
template <bool BE_IN, int V, bool NTS>
__global__ __launch_bounds__(kBlock) void k_blend_v(double* __restrict__ t, const unsigned long long* __restrict__ g,
                                                    int64_t L, double a, double b) {
  constexpr int64_t kTile = (int64_t)kBlock * 2 * V;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  if (base + kTile <= L) {
    u2 gv[V], tv[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
      gv[v] = __builtin_nontemporal_load((gcu2)(g + i));
      tv[v] = *(gcu2)(t + i);
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
      const d2 x = decode2<BE_IN>(gv[v]);
      const d2 w = __builtin_bit_cast(d2, tv[v]);
      d2 o;
      const double awx = a * w.x, bgx = b * x.x, awy = a * w.y, bgy = b * x.y;
      o.x = awx + bgx;
      o.y = awy + bgy;
      if constexpr (NTS) __builtin_nontemporal_store(__builtin_bit_cast(u2, o), (gu2)(t + i));
      else *(gu2)(t + i) = __builtin_bit_cast(u2, o);
    }
    return;
  }
  for (int64_t i = base + threadIdx.x; i < L; i += kBlock) {
    const double x = decode1<BE_IN>(ld8(g + i));
    const double aw = a * t[i];
    const double bg = b * x;
    t[i] = aw + bg;
  }
}

template <int V>
__global__ __launch_bounds__(kBlock) void k_scale_v(double* __restrict__ d, const double* __restrict__ s, int64_t L,
                                                    double c) {
  constexpr int64_t kTile = (int64_t)kBlock * 2 * V;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  if (base + kTile <= L) {
    u2 sv[V];
#pragma unroll
    for (int v = 0; v < V; ++v) sv[v] = __builtin_nontemporal_load((gcu2)(s + base + 2 * ((int64_t)v * kBlock + threadIdx.x)));
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const d2 x = __builtin_bit_cast(d2, sv[v]);
      const d2 o = {c * x.x, c * x.y};
      __builtin_nontemporal_store(__builtin_bit_cast(u2, o), (gu2)(d + base + 2 * ((int64_t)v * kBlock + threadIdx.x)));
    }
    return;
  }
  for (int64_t i = base + threadIdx.x; i < L; i += kBlock) d[i] = c * s[i];
}

template <bool BE_IN, bool FIRST, int V>
__global__ __launch_bounds__(kBlock) void k_fold_n_v(unsigned long long* __restrict__ dst,
                                                     const unsigned long long* __restrict__ src, int64_t n) {
  constexpr int64_t kTile = (int64_t)kBlock * 2 * V;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  if (base + kTile <= n) {
    u2 sv[V], dv[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
      sv[v] = __builtin_nontemporal_load((gcu2)(src + i));
      if constexpr (!FIRST) dv[v] = *(gcu2)(dst + i);
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
      const d2 x = decode2<BE_IN>(sv[v]);
      d2 o = x;
      if constexpr (!FIRST) {
        const d2 y = __builtin_bit_cast(d2, dv[v]);
        o.x = y.x + x.x;
        o.y = y.y + x.y;
      }
      *(gu2)(dst + i) = __builtin_bit_cast(u2, o);
    }
    return;
  }
  for (int64_t i = base + threadIdx.x; i < n; i += kBlock) {
    const double x = decode1<BE_IN>(ld8(src + i));
    const double y = FIRST ? x : __builtin_bit_cast(double, ld8(dst + i)) + x;
    st8(dst + i, __builtin_bit_cast(unsigned long long, y));
  }
}

struct Var {
  std::string name;
  double bytes;
  std::function<void()> reset;   // restore the in-place operand
  std::function<void()> run;
  std::function<void()> save;    // copy the result for the bit check
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 4194304;
  const int REPS = argc > 2 ? atoi(argv[2]) : 20;
  const size_t B = (size_t)N * 8;
  unsigned long long *g, *t0, *t, *s, *d, *ref;
  CK(hipMalloc(&g, B));
  CK(hipMalloc(&t0, B));
  CK(hipMalloc(&t, B));
  CK(hipMalloc(&s, B));
  CK(hipMalloc(&d, B));
  CK(hipMalloc(&ref, B));
  hipLaunchKernelGGL(k_synth<false>, dim3(4096), dim3(kBlock), 0, 0, g, N, 0x1234ULL);
  hipLaunchKernelGGL(k_synth<false>, dim3(4096), dim3(kBlock), 0, 0, t0, N, 0x5678ULL);
  hipLaunchKernelGGL(k_synth<false>, dim3(4096), dim3(kBlock), 0, 0, s, N, 0x9abcULL);
  CK(hipDeviceSynchronize());
  const unsigned gs = std::min<unsigned>(blocks_for(N, kBlock), 8192), gf = std::min<unsigned>(blocks_for(N, kBlock), 4096);
  auto tiles = [&](int V) { return (unsigned)((N + kBlock * 2 * V - 1) / (kBlock * 2 * V)); };
  const double a = 0.75, bb = 1.0, c = 0.25;
  auto reset_t = [=]() { CK(hipMemcpyAsync(t, t0, B, hipMemcpyDeviceToDevice, 0)); };
  auto none = []() {};
  std::vector<Var> vars;
  // blend
  vars.push_back({"blend grid-stride 8 B (unaligned)", 24.0 * N, reset_t,
                  [=]() { hipLaunchKernelGGL(k_blend<false>, dim3(gs), dim3(kBlock), 0, 0, (double*)t, g, N, a, bb); }, nullptr, {}});
  vars.push_back({"blend product k_blend<VEC>", 24.0 * N, reset_t,
                  [=]() { hipLaunchKernelGGL((k_blend<false, true>), dim3(tiles(kEwV)), dim3(kBlock), 0, 0, (double*)t, g, N, a, bb); }, nullptr, {}});
  vars.push_back({"blend tiles V=4", 24.0 * N, reset_t,
                  [=]() { hipLaunchKernelGGL((k_blend_v<false, 4, false>), dim3(tiles(4)), dim3(kBlock), 0, 0, (double*)t, g, N, a, bb); }, nullptr, {}});
  vars.push_back({"blend tiles V=4 nt stores", 24.0 * N, reset_t,
                  [=]() { hipLaunchKernelGGL((k_blend_v<false, 4, true>), dim3(tiles(4)), dim3(kBlock), 0, 0, (double*)t, g, N, a, bb); }, nullptr, {}});
  vars.push_back({"blend tiles V=8", 24.0 * N, reset_t,
                  [=]() { hipLaunchKernelGGL((k_blend_v<false, 8, false>), dim3(tiles(8)), dim3(kBlock), 0, 0, (double*)t, g, N, a, bb); }, nullptr, {}});
  // scale
  vars.push_back({"scale grid-stride 8 B (unaligned)", 16.0 * N, none,
                  [=]() { hipLaunchKernelGGL(k_scale<false>, dim3(gs), dim3(kBlock), 0, 0, (double*)d, (const double*)s, N, c); }, nullptr, {}});
  vars.push_back({"scale product k_scale<VEC>", 16.0 * N, none,
                  [=]() { hipLaunchKernelGGL(k_scale<true>, dim3(tiles(kEwV)), dim3(kBlock), 0, 0, (double*)d, (const double*)s, N, c); }, nullptr, {}});
  vars.push_back({"scale tiles V=4", 16.0 * N, none,
                  [=]() { hipLaunchKernelGGL((k_scale_v<4>), dim3(tiles(4)), dim3(kBlock), 0, 0, (double*)d, (const double*)s, N, c); }, nullptr, {}});
  // bswap (the codec copy: target reads/writes in big-endian, GetParameters into Gradient_Buff)
  vars.push_back({"bswap grid-stride 8 B (unaligned)", 16.0 * N, none,
                  [=]() { hipLaunchKernelGGL(k_bswap64<false>, dim3(gf), dim3(kBlock), 0, 0, s, d, N); }, nullptr, {}});
  vars.push_back({"bswap product k_bswap64<VEC>", 16.0 * N, none,
                  [=]() { hipLaunchKernelGGL(k_bswap64<true>, dim3(tiles(kEwV)), dim3(kBlock), 0, 0, s, d, N); }, nullptr, {}});
  // own accumulate (UpdateGradient: k_split MODE 1 = AGG += v, MODE 2 = +0.0 + v into a zero AGG)
  const unsigned gl = blocks_for(N, kBlock);
  vars.push_back({"own-acc element per lane (unaligned)", 24.0 * N, reset_t,
                  [=]() { hipLaunchKernelGGL((k_split<false, false, 1, false>), dim3(gl), dim3(kBlock), 0, 0, g, (int64_t)0, N - 1, N, t); }, nullptr, {}});
  vars.push_back({"own-acc product k_split<1, VEC>", 24.0 * N, reset_t,
                  [=]() { hipLaunchKernelGGL((k_split<false, false, 1, true>), dim3(tiles(kEwV)), dim3(kBlock), 0, 0, g, (int64_t)0, N - 1, N, t); }, nullptr, {}});
  vars.push_back({"own-acc zero AGG: memset + fold (old)", 16.0 * N, reset_t,
                  [=]() { (void)hipMemsetAsync(t, 0, B, 0);
                          hipLaunchKernelGGL((k_split<false, false, 1, false>), dim3(gl), dim3(kBlock), 0, 0, g, (int64_t)0, N - 1, N, t); }, nullptr, {}});
  vars.push_back({"own-acc zero AGG: k_split<2, VEC>", 16.0 * N, reset_t,
                  [=]() { hipLaunchKernelGGL((k_split<false, false, 2, true>), dim3(tiles(kEwV)), dim3(kBlock), 0, 0, g, (int64_t)0, N - 1, N, t); }, nullptr, {}});
  // AggregatePartition with REP logically zero: W = AGG + 0.0 (k_finalize<REP_ZERO>, 16 B / element,
  // the shipped kFinV = 8, and 4) against k_scale's tile (the same bytes) -- one arena, offsets 0 / N
  double* arena = nullptr;
  CK(hipMalloc(&arena, 2 * B + 256));
  CK(hipMemcpy(arena, s, B, hipMemcpyDeviceToDevice));
  FinDesc fd{N, 0, 0, N};
  FinDesc* d_fd;
  CK(hipMalloc(&d_fd, sizeof fd));
  CK(hipMemcpy(d_fd, &fd, sizeof fd, hipMemcpyHostToDevice));
  auto fin_tpp = [&](int V) { return (int)((N + kBlock * 2 * V - 1) / (kBlock * 2 * V)); };
  vars.push_back({"finalize REP_ZERO V=8 (shipped)", 16.0 * N, none,
                  [=]() { hipLaunchKernelGGL((k_finalize<true, false, kBlock, 8>), dim3(fin_tpp(8)), dim3(kBlock), 0, 0, d_fd, arena, fin_tpp(8)); }, nullptr, {}});
  vars.push_back({"finalize REP_ZERO V=4", 16.0 * N, none,
                  [=]() { hipLaunchKernelGGL((k_finalize<true, false, kBlock, 4>), dim3(fin_tpp(4)), dim3(kBlock), 0, 0, d_fd, arena, fin_tpp(4)); }, nullptr, {}});
  vars.push_back({"scale tile on the same arena", 16.0 * N, none,
                  [=]() { hipLaunchKernelGGL(k_scale<true>, dim3(tiles(kEwV)), dim3(kBlock), 0, 0, arena + N, (const double*)arena, N, 1.0); }, nullptr, {}});
  // fold_n
  vars.push_back({"fold_n grid-stride 8 B (unaligned)", 24.0 * N, reset_t,
                  [=]() { hipLaunchKernelGGL((k_fold_n<false, false>), dim3(gf), dim3(kBlock), 0, 0, t, g, N); }, nullptr, {}});
  vars.push_back({"fold_n product k_fold_n<VEC>", 24.0 * N, reset_t,
                  [=]() { hipLaunchKernelGGL((k_fold_n<false, false, true>), dim3(tiles(kEwV)), dim3(kBlock), 0, 0, t, g, N); }, nullptr, {}});
  vars.push_back({"fold_n tiles V=4", 24.0 * N, reset_t,
                  [=]() { hipLaunchKernelGGL((k_fold_n_v<false, false, 4>), dim3(tiles(4)), dim3(kBlock), 0, 0, t, g, N); }, nullptr, {}});

  // bit checks: each tile form against the shipped kernel of its group
  auto result = [&](Var& v, unsigned long long* out, std::vector<unsigned long long>& host) {
    v.reset();
    v.run();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(host.data(), out, B, hipMemcpyDeviceToHost));
  };
  std::vector<unsigned long long> want(N), got(N);
  bool ok = true;
  const int groups[][2] = {{0, 5}, {5, 8}, {8, 10}, {10, 12}, {12, 14}, {14, 17}, {17, 20}};
  for (auto& gr : groups) {
    unsigned long long* out = (gr[0] == 5 || gr[0] == 8) ? d : gr[0] == 14 ? (unsigned long long*)(arena + N) : t;
    result(vars[gr[0]], out, want);
    for (int i = gr[0] + 1; i < gr[1]; ++i) {
      result(vars[i], out, got);
      const bool same = !memcmp(got.data(), want.data(), B);
      printf("# check %-32s %s\n", vars[i].name.c_str(), same ? "bit-identical" : "MISMATCH");
      ok = ok && same;
    }
  }
  fflush(stdout);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // Cold caches for every timed run: 1 GiB of memset (untimed) pushes the
  // operands out of the L2s and the 256 MB Infinity Cache first.  Without it
  // a kernel that follows one that read the same input with plain (cache-
  // allocating) loads finds the input's tail in the Infinity Cache and reads
  // up to ~8 points fast -- an artefact of the order, not of the kernel.
  void* flush_buf = nullptr;
  const size_t flush_bytes = (size_t)1 << 30;
  CK(hipMalloc(&flush_buf, flush_bytes));
  for (int r = 0; r < REPS; ++r)
    for (size_t j = 0; j < vars.size(); ++j) {
      Var& v = vars[(j + (size_t)r) % vars.size()];
      v.reset();
      CK(hipMemsetAsync(flush_buf, r & 0xFF, flush_bytes, 0));
      CK(hipEventRecord(e0, 0));
      v.run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  printf("# N=%lld doubles, REPS=%d\n", (long long)N, REPS);
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    printf("%-34s median %8.4f ms  min %8.4f ms  %8.1f GB/s  %5.1f%% of 8 TB/s\n", v.name.c_str(), med, v.ms[0],
           v.bytes / med / 1e6, v.bytes / med / 1e6 / 80.0);
  }
  return ok ? 0 : 1;
}
