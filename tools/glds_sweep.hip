// glds_sweep.hip -- dev tool (round-4 A/B, not shipped): the big-endian fold
// with its bucket bytes moved by LDS-DMA (global_load_lds_dwordx4) instead of
// VGPR loads, against the shipped kernels on the same buckets in one process.
//
// Why: the shipped big-endian fold (k_reduce<BE_IN, SEQF = 3>) runs ~3-4
// points under the native-double fold on the same bytes:
// with the bswap between load and add hipcc hoists loads and spills unless
// the loads are fenced into small groups, which caps the bytes a wave keeps
// in flight.  An LDS-DMA load has no VGPR destination, so a wave can keep D-1
// groups of G vectors in flight through a ring in LDS while it decodes and
// adds the oldest group, with its accumulators the only big register cost.
//
// k_glds keeps the shipped tile (BS lanes x R 16-B vectors, each element
// folded over peers 0..k-1 in order: the same fold, bit for bit) and walks
// the (peer, vector group) steps of its tile in the shipped order, with a
// counted `s_waitcnt vmcnt` per step (all LDS in ONE __shared__ array, no
// ordinary vector loads in the loop: cdna_hip_programming.md §5 traps).
//
// Usage: glds_sweep P L K REPS    (default config D's shape per launch:
// 16 x 4194304 x 32, big-endian in and out).  Checks every variant's output
// bit for bit against the shipped kernel before timing.
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

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Full tiles only (L a multiple of BS*2*R), ZERO start, partition-major.
//   G: vectors per step (one LDS-DMA instruction each); D: ring slots (D-1
//   steps in flight while one is consumed).
template <bool BE_IN, bool BE_OUT, int R, int BS, int G, int D>
__global__ __launch_bounds__(BS) void k_glds(const unsigned long long* const* __restrict__ bufs,
                                             const PartDesc* __restrict__ parts, int k, int tiles_per_part) {
  static_assert(R % G == 0, "groups divide the tile");
  constexpr int W = BS / 64;          // waves
  constexpr int NG = R / G;           // steps per peer
  constexpr int SLOT = W * G * 1024;  // bytes of one ring slot (every wave's G vectors)
  __shared__ __attribute__((aligned(16))) unsigned char lds[D * SLOT];
  const int q = blockIdx.x / tiles_per_part;
  const int t = blockIdx.x - q * tiles_per_part;
  const int64_t base = (int64_t)t * BS * 2 * R;
  const unsigned long long* const* __restrict__ pb = bufs + (size_t)q * k;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int S = k * NG;  // steps

  // step s = (peer s / NG, group s % NG); vector r of this lane = elements
  // base + 2*(r*BS + tid) (the shipped layout), landing at
  // lds[slot][wave][v] + lane*16 (wave-uniform base + lane*16, as LDS-DMA writes)
  auto issue = [&](int s) {
    const int j = s / NG, g = s - j * NG, slot = s % D;
    // wave-uniform base + 32-bit lane offset: the saddr form, no 64-bit
    // address VGPRs per vector
    const char* src = (const char*)(pb[j] + base);
    const unsigned lane16 = (unsigned)tid * 16u;
#pragma unroll
    for (int v = 0; v < G; ++v) {
      const int r = g * G + v;
      __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)r * BS * 16 + lane16),
                                       (__attribute__((address_space(3))) void*)(lds + slot * SLOT + (wave * G + v) * 1024),
                                       16, 0, 2 /* nt */);
    }
  };

  d2 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = d2{0.0, 0.0};
  for (int s = 0; s < D - 1 && s < S; ++s) issue(s);
  for (int j = 0; j < k; ++j) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int s = j * NG + g;
      if (s + D - 1 < S) {
        issue(s + D - 1);
        wait_vm<G * (D - 1)>();   // step s landed; the D-1 newer steps may still be in flight
      } else {
        wait_vm<0>();
      }
      const unsigned char* src = lds + (s % D) * SLOT + wave * G * 1024 + lane * 16;
#pragma unroll
      for (int v = 0; v < G; ++v) {
        const u2 raw = *(const __attribute__((address_space(3))) u2*)(src + v * 1024);
        const d2 x = decode2<BE_IN>(raw);
        acc[g * G + v].x = acc[g * G + v].x + x.x;
        acc[g * G + v].y = acc[g * G + v].y + x.y;
      }
    }
  }
  unsigned long long* dst = parts[q].dst;
#pragma unroll
  for (int r = 0; r < R; ++r)
    __builtin_nontemporal_store(encode2<BE_OUT>(acc[r]), (gu2)(dst + base + 2 * ((int64_t)r * BS + tid)));
}

struct Var {
  std::string name;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 16;
  const int64_t L = argc > 2 ? atoll(argv[2]) : 4194304;
  const int K = argc > 3 ? atoi(argv[3]) : 32;
  const int REPS = argc > 4 ? atoi(argv[4]) : 10;
  // GLDS_NATIVE=1: native doubles in and out (against the shipped native fold)
  const bool native = getenv("GLDS_NATIVE") != nullptr;
  const bool be_out = !native && getenv("GLDS_NATIVE_OUT") == nullptr;
  if (L % (1024 * 2 * 16) != 0) {
    fprintf(stderr, "L must be a multiple of 32768\n");
    return 2;
  }
  const int64_t stride = L + 32;
  unsigned long long* arena;
  CK(hipMalloc(&arena, (size_t)P * K * stride * 8 + 4096));
  unsigned long long* base = (unsigned long long*)(((uintptr_t)arena + 255) / 256 * 256);
  std::vector<const unsigned long long*> ptrs(P * K);
  for (int p = 0; p < P; ++p)
    for (int k = 0; k < K; ++k) {
      unsigned long long* b = base + (int64_t)(p * K + k) * stride;
      ptrs[p * K + k] = b;
      const unsigned long long key = 0x1B52026ULL ^ ((unsigned long long)p << 40) ^ ((unsigned long long)k << 32);
      if (native) hipLaunchKernelGGL(k_synth<false>, dim3(4096), dim3(kBlock), 0, 0, b, L, key);
      else hipLaunchKernelGGL(k_synth<true>, dim3(4096), dim3(kBlock), 0, 0, b, L, key);
    }
  const unsigned long long** d_ptrs;
  CK(hipMalloc(&d_ptrs, ptrs.size() * 8));
  CK(hipMemcpy(d_ptrs, ptrs.data(), ptrs.size() * 8, hipMemcpyHostToDevice));
  const int64_t dstride = (L + 31) / 32 * 32;
  unsigned long long* dst;
  CK(hipMalloc(&dst, (size_t)P * dstride * 8));
  std::vector<PartDesc> pd(P);
  for (int p = 0; p < P; ++p) {
    pd[p].len = L;
    pd[p].dst = dst + (int64_t)p * dstride;
  }
  PartDesc* d_pd;
  CK(hipMalloc(&d_pd, P * sizeof(PartDesc)));
  CK(hipMemcpy(d_pd, pd.data(), P * sizeof(PartDesc), hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  const double alg = (double)P * (K + 1) * L * 8;
  auto bp = (const unsigned long long* const*)d_ptrs;

  std::vector<Var> vars;
  vars.push_back(Var{"shipped R=16 BS=1024 (BE: SEQF=3)", [=](hipStream_t s) {
                       const int tpp = (int)(L / (1024 * 2 * 16));
                       if (native)
                         hipLaunchKernelGGL((k_reduce<false, false, kZero, 1, 16, true, 0, 1024>), dim3(tpp * P),
                                            dim3(1024), 0, s, bp, d_pd, K, tpp, P);
                       else if (be_out)
                         hipLaunchKernelGGL((k_reduce<true, true, kZero, 1, 16, true, 0, 1024, 3>), dim3(tpp * P),
                                            dim3(1024), 0, s, bp, d_pd, K, tpp, P);
                       else
                         hipLaunchKernelGGL((k_reduce<true, false, kZero, 1, 16, true, 0, 1024, 3>), dim3(tpp * P),
                                            dim3(1024), 0, s, bp, d_pd, K, tpp, P);
                     }, {}});
  vars.push_back(Var{"native-double kernel, same bytes", [=](hipStream_t s) {
                       const int tpp = (int)(L / (1024 * 2 * 16));
                       hipLaunchKernelGGL((k_reduce<false, false, kZero, 1, 16, true, 0, 1024>), dim3(tpp * P),
                                          dim3(1024), 0, s, bp, d_pd, K, tpp, P);
                     }, {}});
  const size_t first_glds = vars.size();
#define GL(R, BS, G, D)                                                                                  \
  vars.push_back(Var{"glds R=" #R " BS=" #BS " G=" #G " D=" #D, [=](hipStream_t s) {                     \
                       const int tpp = (int)(L / ((int64_t)BS * 2 * R));                                 \
                       if (native)                                                                       \
                         hipLaunchKernelGGL((k_glds<false, false, R, BS, G, D>), dim3(tpp * P), dim3(BS), 0, s, \
                                            bp, d_pd, K, tpp);                                           \
                       else if (be_out)                                                                  \
                         hipLaunchKernelGGL((k_glds<true, true, R, BS, G, D>), dim3(tpp * P), dim3(BS), 0, s, \
                                            bp, d_pd, K, tpp);                                           \
                       else                                                                              \
                         hipLaunchKernelGGL((k_glds<true, false, R, BS, G, D>), dim3(tpp * P), dim3(BS), 0, s, \
                                            bp, d_pd, K, tpp);                                           \
                     }, {}})
  // (R = 16 at 1024 lanes spills: 128 VGPRs is the 1024-lane cap)
  GL(16, 512, 2, 4);    // 8 waves, 64 KiB ring, 6 KiB in flight per wave
  GL(16, 512, 4, 4);    // 128 KiB, 12 KiB per wave
  GL(8, 1024, 2, 4);    // 16 waves, 128 KiB, 6 KiB per wave
  GL(8, 1024, 1, 8);    // 128 KiB, 7 KiB per wave in 1-KiB steps
  GL(8, 1024, 2, 3);    // 96 KiB, 4 KiB per wave
  GL(8, 512, 2, 4);     // 64 KiB: two blocks per CU
  GL(16, 256, 4, 8);    // 4 waves, 128 KiB, 28 KiB per wave
#undef GL

  // correctness: every variant's output equals the shipped kernel's, bit for bit
  std::vector<unsigned long long> want((size_t)P * dstride), got((size_t)P * dstride);
  CK(hipMemset(dst, 0, (size_t)P * dstride * 8));
  vars[0].run(0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(want.data(), dst, want.size() * 8, hipMemcpyDeviceToHost));
  bool ok = true;
  for (size_t i = first_glds; i < vars.size(); ++i) {
    CK(hipMemset(dst, 0xA5, (size_t)P * dstride * 8));
    vars[i].run(0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), dst, got.size() * 8, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (int p = 0; p < P; ++p)
      for (int64_t e = 0; e < L; ++e)
        bad += got[(size_t)p * dstride + e] != want[(size_t)p * dstride + e];
    printf("# check %-32s %s (%zu differing elements)\n", vars[i].name.c_str(), bad ? "MISMATCH" : "bit-identical", bad);
    ok = ok && !bad;
  }
  fflush(stdout);

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
  printf("# P=%d L=%lld K=%d REPS=%d %s; algorithmic bytes/launch=%.0f\n", P, (long long)L, K, REPS,
         native ? "native doubles in and out" : be_out ? "BE in + out" : "BE in, native out", alg);
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    printf("%-36s median %8.4f ms  min %8.4f ms  %8.1f GB/s  %5.1f%% of 8 TB/s\n", v.name.c_str(), med, mn,
           alg / med / 1e6, alg / med / 1e6 / 80.0);
  }
  return ok ? 0 : 1;
}
