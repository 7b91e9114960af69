// pinned_read_probe.hip -- dev tool: how fast the CPU reads (and writes)
// pinned host memory that a DMA copy just filled (or will drain), for the
// staging kinds the chunked calls could use.  The JNI heap natives copy every
// chunk between the library's pinned ring and the Java heap
// (finalizePartition(byte[]) / getPartitions(double[]) read the ring,
// accumulate(double[]) writes it); this says whether the ring's allocation
// flags bound that copy.
//
// Usage: pinned_read_probe [chunk_bytes] [reps]
// Per kind: D2H of one chunk into the buffer, then a memcpy buffer -> heap
// (timed); and memcpy heap -> buffer (timed), then H2D of it.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

using clk = std::chrono::steady_clock;

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? (size_t)atoll(argv[1]) : (size_t)4 << 20;
  const int reps = argc > 2 ? atoi(argv[2]) : 50;
  void* dev;
  CK(hipMalloc(&dev, n));
  CK(hipMemset(dev, 0x3c, n));
  std::vector<char> heap(n);
  std::memset(heap.data(), 1, n);
  struct Kind {
    const char* name;
    unsigned flags;
    int registered;   // 0 hipHostMalloc, 1 aligned_alloc(4 KiB), 2 aligned_alloc(2 MiB) + MADV_HUGEPAGE
  } kinds[] = {{"hipHostMalloc default", hipHostMallocDefault, 0},
               {"hipHostMalloc NonCoherent", hipHostMallocNonCoherent, 0},
               {"hipHostMalloc Coherent", hipHostMallocCoherent, 0},
               {"malloc + hipHostRegister", 0, 1},
               {"2M-aligned THP + Register", 0, 2}};
  hipStream_t s;
  CK(hipStreamCreate(&s));
  printf("# chunk %zu bytes, %d reps; GB/s of the CPU memcpy (median)\n", n, reps);
  for (const auto& k : kinds) {
    void* p = nullptr;
    if (k.registered) {
      const size_t al = k.registered == 2 ? ((size_t)2 << 20) : 4096;
      p = aligned_alloc(al, (n + al - 1) / al * al);
      if (k.registered == 2) madvise(p, (n + al - 1) / al * al, MADV_HUGEPAGE);
      std::memset(p, 0, n);
      CK(hipHostRegister(p, n, hipHostRegisterDefault));
    } else {
      CK(hipHostMalloc(&p, n, k.flags));
    }
    std::vector<double> rd, wr, d2h, h2d;
    for (int r = 0; r < reps; ++r) {
      auto a = clk::now();
      CK(hipMemcpyAsync(p, dev, n, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      d2h.push_back(n / std::chrono::duration<double>(clk::now() - a).count() / 1e9);
      a = clk::now();
      std::memcpy(heap.data(), p, n);
      rd.push_back(n / std::chrono::duration<double>(clk::now() - a).count() / 1e9);
      a = clk::now();
      std::memcpy(p, heap.data(), n);
      wr.push_back(n / std::chrono::duration<double>(clk::now() - a).count() / 1e9);
      a = clk::now();
      CK(hipMemcpyAsync(dev, p, n, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      h2d.push_back(n / std::chrono::duration<double>(clk::now() - a).count() / 1e9);
    }
    for (auto* v : {&rd, &wr, &d2h, &h2d}) std::sort(v->begin(), v->end());
    printf("%-28s read (ring -> heap) %6.1f GB/s   write (heap -> ring) %6.1f GB/s   D2H %5.1f  H2D %5.1f GB/s\n",
           k.name, rd[rd.size() / 2], wr[wr.size() / 2], d2h[d2h.size() / 2], h2d[h2d.size() / 2]);
    if (k.registered) {
      CK(hipHostUnregister(p));
      free(p);
    } else {
      CK(hipHostFree(p));
    }
  }
  return 0;
}
