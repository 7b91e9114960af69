// h2d_bench.hip -- dev tool: host->device ceilings for the host-inclusive
// aggregation path.  Measures, for K pinned big-endian
// buckets of L doubles:
//   1. hipMemcpyAsync H2D, one stream (the current ipls_agg_accumulate path)
//   2. the same split over S streams (several SDMA engines)
//   3. zero-copy: a kernel that folds straight from pinned host memory
//      (BE decode + acc += x) -- no staging copy at all.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "../ipls-java-api_amd/csrc/ipls_kernels.hpp"

using namespace ipls;
#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e = (x);                                                                    \
    if (e != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));     \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

// acc[i] = acc[i] + bswap(host[i]) reading host memory directly (PCIe reads).
__global__ __launch_bounds__(256) void k_fold_from_host(const u2* __restrict__ host, u2* __restrict__ acc, int64_t n2) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
    const d2 x = decode2<true>(__builtin_nontemporal_load(host + i));
    d2 a = __builtin_bit_cast(d2, acc[i]);
    a.x = a.x + x.x;
    a.y = a.y + x.y;
    acc[i] = __builtin_bit_cast(u2, a);
  }
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int64_t L = argc > 1 ? atoll(argv[1]) : 4194304;
  const int K = argc > 2 ? atoi(argv[2]) : 32;
  const int REPS = argc > 3 ? atoi(argv[3]) : 3;
  const size_t bytes = (size_t)L * 8;
  std::vector<void*> host(K);
  for (int k = 0; k < K; ++k) {
    CK(hipHostMalloc(&host[k], bytes, hipHostMallocDefault));
    std::memset(host[k], 0x11 * (k + 1), bytes);
  }
  void* dev;
  CK(hipMalloc(&dev, bytes * K));
  void* acc;
  CK(hipMalloc(&acc, bytes));
  CK(hipMemset(acc, 0, bytes));
  hipStream_t st[4];
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  printf("# L=%lld K=%d (%.1f MB per bucket, %.2f GB per round)\n", (long long)L, K, bytes / 1e6, bytes * K / 1e9);
  for (int S : {1, 2, 4}) {
    double best = 1e30;
    for (int r = 0; r < REPS; ++r) {
      CK(hipDeviceSynchronize());
      const double t0 = now();
      for (int k = 0; k < K; ++k)
        CK(hipMemcpyAsync((char*)dev + (size_t)k * bytes, host[k], bytes, hipMemcpyHostToDevice, st[k % S]));
      for (int s = 0; s < S; ++s) CK(hipStreamSynchronize(st[s]));
      best = std::min(best, now() - t0);
    }
    printf("hipMemcpyAsync H2D, %d stream(s): %7.2f GB/s\n", S, bytes * K / best / 1e9);
  }
  for (int grid : {256, 1024, 4096}) {
    double best = 1e30;
    for (int r = 0; r < REPS; ++r) {
      CK(hipDeviceSynchronize());
      const double t0 = now();
      for (int k = 0; k < K; ++k)
        hipLaunchKernelGGL(k_fold_from_host, dim3(grid), dim3(256), 0, st[0], (const u2*)host[k], (u2*)acc,
                           (int64_t)(L / 2));
      CK(hipStreamSynchronize(st[0]));
      best = std::min(best, now() - t0);
    }
    printf("zero-copy fold from pinned host, grid %4d: %7.2f GB/s\n", grid, bytes * K / best / 1e9);
  }
  // the shipped per-arrival kernel (k_fold1, 4 pairs per lane in flight) reading
  // pinned host memory: per-arrival sync (ipls_agg_accumulate) and queued
  // (ipls_agg_accumulate_async), by grid size
  for (int sync_each : {1, 0})
    for (int grid : {128, 256, 512, 1024, 4096}) {
      double best = 1e30;
      for (int r = 0; r < REPS; ++r) {
        CK(hipDeviceSynchronize());
        const double t0 = now();
        for (int k = 0; k < K; ++k) {
          hipLaunchKernelGGL((k_fold1<true, false, kAccum, 4>), dim3(grid), dim3(kBlock), 0, st[0],
                             (unsigned long long*)acc, (const unsigned long long*)host[k], L);
          if (sync_each) CK(hipStreamSynchronize(st[0]));
        }
        CK(hipStreamSynchronize(st[0]));
        best = std::min(best, now() - t0);
      }
      printf("k_fold1 from pinned host, %s, grid %4d: %7.2f GB/s\n", sync_each ? "sync each" : "queued   ", grid,
             bytes * K / best / 1e9);
    }
  // pageable sources (a Java heap byte[] pinned by GetPrimitiveArrayCritical)
  {
    std::vector<char*> pg(K);
    for (int k = 0; k < K; ++k) {
      pg[k] = (char*)malloc(bytes);
      std::memset(pg[k], 0x22, bytes);
    }
    double best = 1e30;
    for (int r = 0; r < REPS; ++r) {
      CK(hipDeviceSynchronize());
      const double t0 = now();
      for (int k = 0; k < K; ++k)
        CK(hipMemcpyAsync((char*)dev + (size_t)k * bytes, pg[k], bytes, hipMemcpyHostToDevice, st[0]));
      CK(hipStreamSynchronize(st[0]));
      best = std::min(best, now() - t0);
    }
    printf("hipMemcpyAsync H2D from pageable (HIP staging): %7.2f GB/s\n", bytes * K / best / 1e9);
    best = 1e30;
    for (int r = 0; r < REPS; ++r) {
      const double t0 = now();
      for (int k = 0; k < K; ++k) std::memcpy(host[k], pg[k], bytes);
      best = std::min(best, now() - t0);
    }
    printf("host memcpy pageable -> pinned, 1 thread: %7.2f GB/s\n", bytes * K / best / 1e9);
    best = 1e30;
    for (int r = 0; r < REPS; ++r) {
      CK(hipDeviceSynchronize());
      const double t0 = now();
      for (int k = 0; k < K; ++k) {
        CK(hipHostRegister(pg[k], bytes, hipHostRegisterDefault));
        void* d = nullptr;
        CK(hipHostGetDevicePointer(&d, pg[k], 0));
        hipLaunchKernelGGL(k_fold_from_host, dim3(256), dim3(256), 0, st[0], (const u2*)d, (u2*)acc, (int64_t)(L / 2));
        CK(hipStreamSynchronize(st[0]));
        CK(hipHostUnregister(pg[k]));
      }
      best = std::min(best, now() - t0);
    }
    printf("register + zero-copy fold + unregister per bucket: %7.2f GB/s\n", bytes * K / best / 1e9);
    for (int k = 0; k < K; ++k) free(pg[k]);
  }
  {
    double best = 1e30;
    for (int r = 0; r < REPS; ++r) {
      CK(hipDeviceSynchronize());
      const double t0 = now();
      for (int k = 0; k < K; ++k)
        CK(hipMemcpyAsync(host[k], (char*)dev + (size_t)k * bytes, bytes, hipMemcpyDeviceToHost, st[k % 2]));
      for (int s = 0; s < 2; ++s) CK(hipStreamSynchronize(st[s]));
      best = std::min(best, now() - t0);
    }
    printf("hipMemcpyAsync D2H, 2 streams: %7.2f GB/s\n", bytes * K / best / 1e9);
  }
  return 0;
}
