// alloc_sweep.hip -- dev tool (round-4 probe): does the physical placement of
// the bucket pool move the fold?  The same shipped k_reduce over two pools of
// identical buckets in ONE process, interleaved launch by launch:
//   default    hipMalloc
//   contiguous hipExtMallocWithFlags(..., hipDeviceMallocContiguous)
//   churned    hipMalloc after the device memory was carved into 256 MiB
//              pieces and every other one freed (what a long-running process
//              that frees and reallocates tends to get)
// Outputs are compared bit for bit across pools before timing.
//
// Usage: alloc_sweep P L K REPS [be]   (default config C: 16 x 4194304 x 32)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

struct Pool {
  std::string name;
  unsigned long long* mem = nullptr;
  const unsigned long long** d_ptrs = nullptr;
  PartDesc* d_pd = nullptr;
  unsigned long long* dst = nullptr;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 16;
  const int64_t L = argc > 2 ? atoll(argv[2]) : 4194304;
  const int K = argc > 3 ? atoi(argv[3]) : 32;
  const int REPS = argc > 4 ? atoi(argv[4]) : 10;
  const bool be = argc > 5 && !strcmp(argv[5], "be");
  if (L % (1024 * 2 * 16) != 0) {
    fprintf(stderr, "L must be a multiple of 32768\n");
    return 2;
  }
  const int64_t stride = L + 32;
  const size_t bytes = (size_t)P * K * stride * 8 + 4096;
  const int64_t dstride = (L + 31) / 32 * 32;
  std::vector<Pool> pools(3);
  pools[0].name = "default (hipMalloc)";
  pools[1].name = "contiguous (hipDeviceMallocContiguous)";
  pools[2].name = "churned (hipMalloc after fragmenting)";
  CK(hipMalloc(&pools[0].mem, bytes));
  hipError_t ce = hipExtMallocWithFlags((void**)&pools[1].mem, bytes, hipDeviceMallocContiguous);
  if (ce != hipSuccess) {
    fprintf(stderr, "# contiguous allocation of %zu bytes refused: %s\n", bytes, hipGetErrorString(ce));
    (void)hipGetLastError();
    pools[1].mem = nullptr;
  }
  {
    // fragment: 256 MiB pieces up to ~bytes + 8 GiB, free every other one
    std::vector<void*> pieces;
    const size_t piece = (size_t)256 << 20;
    for (size_t got = 0; got < bytes + ((size_t)8 << 30); got += piece) {
      void* q;
      if (hipMalloc(&q, piece) != hipSuccess) { (void)hipGetLastError(); break; }
      pieces.push_back(q);
    }
    for (size_t i = 0; i < pieces.size(); i += 2) CK(hipFree(pieces[i]));
    if (hipMalloc(&pools[2].mem, bytes) != hipSuccess) {
      (void)hipGetLastError();
      pools[2].mem = nullptr;
      fprintf(stderr, "# churned allocation refused\n");
    }
    for (size_t i = 1; i < pieces.size(); i += 2) CK(hipFree(pieces[i]));
  }
  const int tpp = (int)(L / (1024 * 2 * 16));
  for (auto& pl : pools) {
    if (!pl.mem) continue;
    unsigned long long* base = (unsigned long long*)(((uintptr_t)pl.mem + 255) / 256 * 256);
    std::vector<const unsigned long long*> ptrs(P * K);
    for (int p = 0; p < P; ++p)
      for (int k = 0; k < K; ++k) {
        unsigned long long* b = base + (int64_t)(p * K + k) * stride;
        ptrs[p * K + k] = b;
        const unsigned long long key = 0x1B52026ULL ^ ((unsigned long long)p << 40) ^ ((unsigned long long)k << 32);
        if (be) hipLaunchKernelGGL(k_synth<true>, dim3(4096), dim3(kBlock), 0, 0, b, L, key);
        else hipLaunchKernelGGL(k_synth<false>, dim3(4096), dim3(kBlock), 0, 0, b, L, key);
      }
    CK(hipMalloc(&pl.d_ptrs, ptrs.size() * 8));
    CK(hipMemcpy(pl.d_ptrs, ptrs.data(), ptrs.size() * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&pl.dst, (size_t)P * dstride * 8));
    std::vector<PartDesc> pd(P);
    for (int p = 0; p < P; ++p) {
      pd[p].len = L;
      pd[p].dst = pl.dst + (int64_t)p * dstride;
    }
    CK(hipMalloc(&pl.d_pd, P * sizeof(PartDesc)));
    CK(hipMemcpy(pl.d_pd, pd.data(), P * sizeof(PartDesc), hipMemcpyHostToDevice));
  }
  CK(hipDeviceSynchronize());
  auto run = [&](Pool& pl) {
    auto bp = (const unsigned long long* const*)pl.d_ptrs;
    if (be)
      hipLaunchKernelGGL((k_reduce<true, true, kZero, 1, 16, true, 0, 1024, 3>), dim3(tpp * P), dim3(1024), 0, 0, bp,
                         pl.d_pd, K, tpp, P);
    else
      hipLaunchKernelGGL((k_reduce<false, false, kZero, 1, 16, true, 0, 1024>), dim3(tpp * P), dim3(1024), 0, 0, bp,
                         pl.d_pd, K, tpp, P);
  };
  // the same buckets in every pool: the same sums, bit for bit
  std::vector<unsigned long long> want((size_t)P * dstride), got((size_t)P * dstride);
  bool ok = true, have_want = false;
  for (auto& pl : pools) {
    if (!pl.mem) continue;
    run(pl);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(have_want ? got.data() : want.data(), pl.dst, want.size() * 8, hipMemcpyDeviceToHost));
    if (have_want) {
      const bool same = !memcmp(got.data(), want.data(), want.size() * 8);
      printf("# check %-40s %s\n", pl.name.c_str(), same ? "bit-identical" : "MISMATCH");
      ok = ok && same;
    }
    have_want = true;
  }
  fflush(stdout);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < REPS; ++r)
    for (auto& pl : pools) {
      if (!pl.mem) continue;
      CK(hipEventRecord(e0, 0));
      run(pl);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      pl.ms.push_back(ms);
    }
  const double alg = (double)P * (K + 1) * L * 8;
  printf("# P=%d L=%lld K=%d REPS=%d %s; algorithmic bytes/launch=%.0f\n", P, (long long)L, K, REPS,
         be ? "BE in + out (SEQF=3)" : "native doubles", alg);
  for (auto& pl : pools) {
    if (!pl.mem) continue;
    std::sort(pl.ms.begin(), pl.ms.end());
    const double med = pl.ms[pl.ms.size() / 2];
    printf("%-42s median %8.4f ms  min %8.4f ms  %8.1f GB/s  %5.1f%% of 8 TB/s\n", pl.name.c_str(), med, pl.ms[0],
           alg / med / 1e6, alg / med / 1e6 / 80.0);
  }
  return ok ? 0 : 1;
}
