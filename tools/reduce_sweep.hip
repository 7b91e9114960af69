// reduce_sweep.hip -- dev tool: time k_reduce variants on one MI355X.
//
// Usage: reduce_sweep P L K PAD REPS
// Allocates P*K buckets of L doubles (PAD doubles between buckets), fills them
// with the synthetic generator, then times every variant REPS times,
// interleaved round-robin in one process (cdna_hip_programming.md §5.4 rule 24),
// reporting median/min kernel time (hipEvents) and algorithmic GB/s.
// Also times two HBM reference kernels on the same bytes: a pure streaming
// read (ceiling for this access pattern) and a dwordx4 copy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../ipls-java-api_amd/csrc/ipls_kernels.hpp"

using namespace ipls;

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

// Streaming read of every bucket byte (no fold dependency), one store per lane.
template <int G, int R>
__global__ __launch_bounds__(kBlock) void k_readall(const unsigned long long* const* __restrict__ bufs,
                                                    int n_bufs, int64_t L, unsigned long long* sink) {
  const int64_t base = (int64_t)blockIdx.x * kBlock * 2 * R;
  if (base + (int64_t)kBlock * 2 * R > L) return;
  u2 acc = {0, 0};
  int j = 0;
  for (; j + G <= n_bufs; j += G) {
    u2 v[G][R];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int r = 0; r < R; ++r)
        v[g][r] = ld16<true>(bufs[blockIdx.y * n_bufs + j + g] + base + 2 * (r * kBlock + threadIdx.x));
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int r = 0; r < R; ++r) acc ^= v[g][r];
  }
  if ((acc.x ^ acc.y) == 0x1234567ULL) sink[0] = acc.x;
}

// Experimental fold: uniform bucket base + 32-bit lane offset, and (FORCE)
// scheduling groups that put all R loads of a peer in flight before its adds.
// Full tiles only (L a multiple of BS*2*R); partition-major block order.
template <bool BE, int R, int BS, bool FORCE>
__global__ __launch_bounds__(BS) void k_exp(const unsigned long long* const* __restrict__ bufs,
                                            unsigned long long* __restrict__ dst, int64_t dstride, int k,
                                            int tpp) {
  const int q = blockIdx.x / tpp, t = blockIdx.x - q * tpp;
  const int64_t base = (int64_t)t * BS * 2 * R;
  const unsigned lane16 = threadIdx.x * 16u;
  const unsigned long long* const* pb = bufs + (size_t)q * k;
  d2 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = d2{0.0, 0.0};
  for (int j = 0; j < k; ++j) {
    const char* src = (const char*)(pb[j] + base);
    u2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = __builtin_nontemporal_load((gcu2)(src + (size_t)r * BS * 16 + lane16));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const d2 x = decode2<BE>(v[r]);
      acc[r].x = acc[r].x + x.x;
      acc[r].y = acc[r].y + x.y;
    }
    if constexpr (FORCE) {
      __builtin_amdgcn_sched_group_barrier(0x020, R, 0);     // R VMEM reads
      __builtin_amdgcn_sched_group_barrier(0x002, 1000, 0);  // then the VALU work
    }
  }
  char* d = (char*)(dst + q * dstride + base);
#pragma unroll
  for (int r = 0; r < R; ++r)
    __builtin_nontemporal_store(encode2<false>(acc[r]), (gu2)(d + (size_t)r * BS * 16 + lane16));
}

// Cache-policy probe (SWEEP_CPOL): the same ZERO-start fold, each bucket
// read through a buffer resource with the load's cache-policy bits set
// explicitly (gfx950 CPol: 1 = sc0, 2 = nt, 16 = sc1); full tiles only,
// partition-major.  The shipped kernel's loads are global_load ... nt (2).
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
template <int CPOL, int R, int BS, bool BE = false>
__global__ __launch_bounds__(BS) void k_cpol(const unsigned long long* const* __restrict__ bufs,
                                             unsigned long long* __restrict__ dst, int64_t dstride, int k,
                                             int tpp) {
  const int q = blockIdx.x / tpp, t = blockIdx.x - q * tpp;
  const int64_t base = (int64_t)t * BS * 2 * R;
  const unsigned lane16 = threadIdx.x * 16u;
  const unsigned long long* const* pb = bufs + (size_t)q * k;
  d2 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = d2{0.0, 0.0};
  for (int j = 0; j < k; ++j) {
    __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(pb[j] + base), (short)0, BS * 16 * R, 0x00020000);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(r * BS * 16) + lane16, 0, CPOL);
      const u2 w = u2{(unsigned long long)v.x | ((unsigned long long)v.y << 32),
                      (unsigned long long)v.z | ((unsigned long long)v.w << 32)};
      const d2 x = decode2<BE>(w);
      acc[r].x = acc[r].x + x.x;
      acc[r].y = acc[r].y + x.y;
    }
  }
  char* d = (char*)(dst + q * dstride + base);
#pragma unroll
  for (int r = 0; r < R; ++r)
    __builtin_nontemporal_store(encode2<BE>(acc[r]), (gu2)(d + (size_t)r * BS * 16 + lane16));
}

__global__ __launch_bounds__(kBlock) void k_copy(const u2* __restrict__ in, u2* __restrict__ out, int64_t n2) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n2; i += (int64_t)gridDim.x * kBlock)
    __builtin_nontemporal_store(__builtin_nontemporal_load((gcu2)(in + i)), (gu2)(out + i));
}

struct Var {
  std::string name;
  std::function<void(hipStream_t)> run;
  double bytes;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 16;
  const int64_t L = argc > 2 ? atoll(argv[2]) : 4194304;
  const int K = argc > 3 ? atoi(argv[3]) : 32;
  const int64_t PAD = argc > 4 ? atoll(argv[4]) : 32;
  const int REPS = argc > 5 ? atoi(argv[5]) : 10;
  const bool separate = PAD < 0;
  const int64_t stride = separate ? L : L + PAD;
  unsigned long long* arena = nullptr;
  unsigned long long* base = nullptr;
  if (!separate) {
    CK(hipMalloc(&arena, (size_t)P * K * stride * 8 + 4096));
    base = (unsigned long long*)(((uintptr_t)arena + 255) / 256 * 256);
  }
  std::vector<const unsigned long long*> ptrs(P * K);
  for (int p = 0; p < P; ++p)
    for (int k = 0; k < K; ++k) {
      unsigned long long* b;
      if (separate) CK(hipMalloc(&b, (size_t)L * 8));   // one allocation per bucket (network arrivals)
      else b = base + (int64_t)(p * K + k) * stride;
      ptrs[p * K + k] = b;
      const unsigned long long key = 0x1B52026ULL ^ ((unsigned long long)p << 40) ^ ((unsigned long long)k << 32);
      if (getenv("SWEEP_BE")) hipLaunchKernelGGL(k_synth<true>, dim3(4096), dim3(kBlock), 0, 0, b, L, key);
      else hipLaunchKernelGGL(k_synth<false>, dim3(4096), dim3(kBlock), 0, 0, b, L, key);
    }
  const unsigned long long** d_ptrs;
  CK(hipMalloc(&d_ptrs, ptrs.size() * 8));
  CK(hipMemcpy(d_ptrs, ptrs.data(), ptrs.size() * 8, hipMemcpyHostToDevice));
  // SWEEP_SHIFT=B: a second pointer table with every bucket start moved by B
  // bytes (16-B multiple, < PAD*8), for same-process alignment comparisons.
  const int64_t shift = getenv("SWEEP_SHIFT") ? atoll(getenv("SWEEP_SHIFT")) : 0;
  const unsigned long long** d_ptrs_sh = nullptr;
  if (shift) {
    std::vector<const unsigned long long*> sp(ptrs.size());
    for (size_t i = 0; i < ptrs.size(); ++i) sp[i] = (const unsigned long long*)((const char*)ptrs[i] + shift);
    CK(hipMalloc(&d_ptrs_sh, sp.size() * 8));
    CK(hipMemcpy(d_ptrs_sh, sp.data(), sp.size() * 8, hipMemcpyHostToDevice));
  }
  std::vector<PartDesc> pd(P);
  int64_t off = 0;
  for (int p = 0; p < P; ++p) {
    pd[p].len = L;
    pd[p].dst = nullptr;  // set below, once dst is allocated
    off += (L + 31) / 32 * 32;
  }
  unsigned long long* dst;
  CK(hipMalloc(&dst, (size_t)off * 8));
  for (int p = 0, o = 0; p < P; ++p) {
    pd[p].dst = dst + o;
    o += (int)((L + 31) / 32 * 32);
  }
  PartDesc* d_pd;
  CK(hipMalloc(&d_pd, P * sizeof(PartDesc)));
  CK(hipMemcpy(d_pd, pd.data(), P * sizeof(PartDesc), hipMemcpyHostToDevice));
  unsigned long long* sink;
  CK(hipMalloc(&sink, 64));
  unsigned long long* copy_out;
  const int64_t copy_n2 = (int64_t)P * K * stride / 2;
  const bool do_copy = getenv("SWEEP_COPY") != nullptr && !separate;
  if (do_copy) CK(hipMalloc(&copy_out, copy_n2 * 16));
  CK(hipDeviceSynchronize());

  const double alg = (double)P * (K + 1) * L * 8;
  std::vector<Var> vars;
  const bool be = getenv("SWEEP_BE") != nullptr;
#define ADDC(G, R, MAP, BS)                                                                    \
  vars.push_back(Var{"reduce G=" #G " R=" #R " MAP=" #MAP " BS=" #BS,                            \
                     [=](hipStream_t s) {                                                       \
                       const int64_t tile = (int64_t)BS * 2 * R;                                \
                       const int tpp = (int)((L + tile - 1) / tile);                            \
                       const dim3 grid((unsigned)grid_blocks(MAP, (int64_t)tpp * P));           \
                       auto bp = (const unsigned long long* const*)d_ptrs;                      \
                       if (be && be_out)                                                        \
                         hipLaunchKernelGGL((k_reduce<true, true, kZero, G, R, true, MAP, BS>), grid, dim3(BS), 0, s, bp, d_pd, K, tpp, P); \
                       else if (be)                                                             \
                         hipLaunchKernelGGL((k_reduce<true, false, kZero, G, R, true, MAP, BS>), grid, dim3(BS), 0, s, bp, d_pd, K, tpp, P); \
                       else                                                                     \
                         hipLaunchKernelGGL((k_reduce<false, false, kZero, G, R, true, MAP, BS>), grid, dim3(BS), 0, s, bp, d_pd, K, tpp, P); \
                     },                                                                         \
                     alg, {}})
  const bool be_out = getenv("SWEEP_BE_OUT") != nullptr;
  const bool quick = getenv("SWEEP_QUICK") != nullptr;   // the shipped big shape and its neighbours only
  // SWEEP_LAYOUTS=1: the shipped big kernel over other bucket layouts carved
  // from the SAME arena (same physical pages), so only the virtual placement
  // differs: pads of 0 / 32 / 64 / 512 / 4096 / 32768 doubles between buckets,
  // peer-major slot order, and a random slot permutation (pad 32).
  if (getenv("SWEEP_LAYOUTS") && !separate) {
    const int64_t max_pad = (PAD - 32) > 0 ? PAD - 32 : 0;   // run with PAD >= the largest pad + 32
    struct Lay { const char* name; int64_t pad; int order; };
    static const Lay lays[] = {{"layout pad 0", 0, 0},      {"layout pad 32 (shipped)", 32, 0},
                               {"layout pad 64", 64, 0},    {"layout pad 512", 512, 0},
                               {"layout pad 4096", 4096, 0}, {"layout pad 32768", 32768, 0},
                               {"layout pad 32 peer-major", 32, 1}, {"layout pad 32 shuffled", 32, 2}};
    std::vector<int> perm(P * K);
    for (int i = 0; i < P * K; ++i) perm[i] = i;
    unsigned long long x = 88172645463325252ULL;
    for (int i = P * K - 1; i > 0; --i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      std::swap(perm[i], perm[(int)(x % (unsigned long long)(i + 1))]);
    }
    for (const Lay& ly : lays) {
      if (ly.pad > max_pad) continue;
      std::vector<const unsigned long long*> lp(P * K);
      for (int p = 0; p < P; ++p)
        for (int k = 0; k < K; ++k) {
          const int i = p * K + k;
          const int slot = ly.order == 0 ? i : ly.order == 1 ? k * P + p : perm[i];
          lp[i] = base + (int64_t)slot * (L + ly.pad);
        }
      const unsigned long long** d_lp;
      CK(hipMalloc(&d_lp, lp.size() * 8));
      CK(hipMemcpy(d_lp, lp.data(), lp.size() * 8, hipMemcpyHostToDevice));
      vars.push_back(Var{ly.name,
                         [=](hipStream_t s) {
                           const int64_t tile = (int64_t)1024 * 2 * 16;
                           const int tpp = (int)((L + tile - 1) / tile);
                           hipLaunchKernelGGL((k_reduce<false, false, kZero, 1, 16, true, 0, 1024>), dim3(tpp * P),
                                              dim3(1024), 0, s, (const unsigned long long* const*)d_lp, d_pd, K, tpp, P);
                         },
                         alg, {}});
    }
  }
  ADDC(1, 8, 0, 1024);
  ADDC(1, 16, 0, 1024);
  ADDC(1, 16, 2, 1024);
#define ADDS(R, MAP, F)                                                                           \
  vars.push_back(Var{"reduce R=" #R " MAP=" #MAP " BS=1024 SEQF=" #F,                              \
                     [=](hipStream_t s) {                                                       \
                       const int64_t tile = (int64_t)1024 * 2 * R;                              \
                       const int tpp = (int)((L + tile - 1) / tile);                            \
                       const dim3 grid((unsigned)grid_blocks(MAP, (int64_t)tpp * P));           \
                       auto bp = (const unsigned long long* const*)d_ptrs;                      \
                       if (be && be_out)                                                        \
                         hipLaunchKernelGGL((k_reduce<true, true, kZero, 1, R, true, MAP, 1024, F>), grid, dim3(1024), 0, s, bp, d_pd, K, tpp, P); \
                       else if (be)                                                             \
                         hipLaunchKernelGGL((k_reduce<true, false, kZero, 1, R, true, MAP, 1024, F>), grid, dim3(1024), 0, s, bp, d_pd, K, tpp, P); \
                       else                                                                     \
                         hipLaunchKernelGGL((k_reduce<false, false, kZero, 1, R, true, MAP, 1024, F>), grid, dim3(1024), 0, s, bp, d_pd, K, tpp, P); \
                     },                                                                         \
                     alg, {}})
#define ADDSB(R, BS, F)                                                                           \
  vars.push_back(Var{"reduce R=" #R " MAP=0 BS=" #BS " SEQF=" #F,                                  \
                     [=](hipStream_t s) {                                                       \
                       const int64_t tile = (int64_t)BS * 2 * R;                                \
                       const int tpp = (int)((L + tile - 1) / tile);                            \
                       const dim3 grid((unsigned)grid_blocks(0, (int64_t)tpp * P));             \
                       auto bp = (const unsigned long long* const*)d_ptrs;                      \
                       if (be && be_out)                                                        \
                         hipLaunchKernelGGL((k_reduce<true, true, kZero, 1, R, true, 0, BS, F>), grid, dim3(BS), 0, s, bp, d_pd, K, tpp, P); \
                       else if (be)                                                             \
                         hipLaunchKernelGGL((k_reduce<true, false, kZero, 1, R, true, 0, BS, F>), grid, dim3(BS), 0, s, bp, d_pd, K, tpp, P); \
                       else                                                                     \
                         hipLaunchKernelGGL((k_reduce<false, false, kZero, 1, R, true, 0, BS, F>), grid, dim3(BS), 0, s, bp, d_pd, K, tpp, P); \
                     },                                                                         \
                     alg, {}})
  if (be) {   // the native-double kernel on the same bytes (values do not change the timing)
    vars.push_back(Var{"f64 kernel on the same buckets R=16",
                       [=](hipStream_t s) {
                         const int64_t tile = (int64_t)1024 * 2 * 16;
                         const int tpp = (int)((L + tile - 1) / tile);
                         hipLaunchKernelGGL((k_reduce<false, false, kZero, 1, 16, true, 0, 1024>), dim3(tpp * P),
                                            dim3(1024), 0, s, (const unsigned long long* const*)d_ptrs, d_pd, K, tpp, P);
                       },
                       alg, {}});
  }
  if (getenv("SWEEP_MID")) {   // the mid shape (256 lanes, 1-2 partitions) under the SEQ schedules
    ADDSB(16, 256, 42);
    ADDSB(16, 256, 3);
    ADDSB(16, 256, 2);
    ADDSB(16, 1024, 42);
    ADDSB(16, 1024, 3);
  }
  if (getenv("SWEEP_P1")) {   // one partition (per-partition flushes, the storage merge): shapes that fill 256 CUs
    ADDSB(8, 1024, 0);
    ADDSB(16, 512, 2);
    ADDSB(16, 512, 3);
    ADDSB(8, 512, 0);
    ADDSB(16, 256, 2);
    ADDSB(16, 256, 3);
    ADDSB(8, 256, 0);
    ADDSB(16, 256, 0);
  }
  if (getenv("SWEEP_B")) {   // config B (16 x 1M x 8): lanes x vectors per lane, big vs mid
    ADDSB(16, 1024, 0);       // shipped big shape (512 tiles)
    ADDSB(8, 1024, 0);
    ADDSB(4, 1024, 0);
    ADDSB(16, 512, 0);
    ADDSB(8, 512, 0);
    ADDSB(16, 256, 0);        // shipped mid shape
    ADDSB(8, 256, 0);
    ADDSB(4, 256, 0);
  }
  if (getenv("SWEEP_512")) {   // the big shape at 1024 vs 512 lanes (R = 16; 512 lanes keeps 164 VGPRs, one block per CU)
    if (be) {
      ADDSB(16, 1024, 3);
      ADDSB(16, 512, 3);
      ADDSB(16, 512, 2);
      ADDSB(16, 512, 0);
      ADDSB(8, 256, 0);         // the shipped big-endian mid shape
      ADDSB(8, 512, 0);
      ADDSB(8, 1024, 0);
    } else {
      ADDSB(16, 1024, 0);
      ADDSB(16, 512, 0);
      ADDSB(16, 1024, 0);
      ADDSB(16, 512, 0);
    }
  }
  if (getenv("SWEEP_CPOL_BE") && be && be_out && L % (1024 * 2 * 16) == 0) {   // big-endian through buffer loads
    ADDSB(16, 1024, 3);   // shipped (global_load ... nt, SEQF = 3)
#define CPOLB(R, BS)                                                                              \
    vars.push_back(Var{"cpol 2 BE in+out R=" #R " BS=" #BS,                                        \
                       [=](hipStream_t s) {                                                        \
                         const int tpp = (int)(L / ((int64_t)BS * 2 * R));                         \
                         hipLaunchKernelGGL((k_cpol<2, R, BS, true>), dim3(tpp * P), dim3(BS), 0, s, \
                                            (const unsigned long long* const*)d_ptrs, dst,         \
                                            (L + 31) / 32 * 32, K, tpp);                           \
                       },                                                                          \
                       alg, {}})
    CPOLB(16, 1024);
    CPOLB(16, 512);
    CPOLB(8, 1024);
#undef CPOLB
  }
  if (getenv("SWEEP_CPOL") && !be && L % (1024 * 2 * 16) == 0) {   // cache policy of the bucket loads
    ADDSB(16, 1024, 0);   // shipped (global_load ... nt)
#define CPOLV(C, BS)                                                                              \
    vars.push_back(Var{"cpol " #C " R=16 BS=" #BS,                                                   \
                       [=](hipStream_t s) {                                                        \
                         const int tpp = (int)(L / ((int64_t)BS * 2 * 16));                        \
                         hipLaunchKernelGGL((k_cpol<C, 16, BS>), dim3(tpp * P), dim3(BS), 0, s,    \
                                            (const unsigned long long* const*)d_ptrs, dst,         \
                                            (L + 31) / 32 * 32, K, tpp);                           \
                       },                                                                          \
                       alg, {}})
    CPOLV(2, 1024);
    CPOLV(0, 1024);
    CPOLV(1, 1024);
    CPOLV(3, 1024);
    CPOLV(16, 1024);
    CPOLV(18, 1024);
    CPOLV(17, 1024);
    CPOLV(19, 1024);
#undef CPOLV
  }
  if (getenv("SWEEP_BS")) {   // block size / fence interval of the big-endian fold
    ADDSB(16, 1024, 2);
    ADDSB(16, 512, 2);
    ADDSB(16, 256, 2);
    ADDSB(16, 256, 0);
    ADDSB(16, 512, 0);
    ADDSB(32, 256, 2);
    ADDSB(32, 256, 4);
  }
#undef ADDSB
#define ADDACC(R, BS, F)                                                                          \
  vars.push_back(Var{"ACCUM R=" #R " BS=" #BS " SEQF=" #F,                                          \
                     [=](hipStream_t s) {                                                       \
                       const int64_t tile = (int64_t)BS * 2 * R;                                \
                       const int tpp = (int)((L + tile - 1) / tile);                            \
                       auto bp = (const unsigned long long* const*)d_ptrs;                      \
                       if (be)                                                                  \
                         hipLaunchKernelGGL((k_reduce<true, false, kAccum, 1, R, true, 0, BS, F>), dim3(tpp * P), dim3(BS), 0, s, bp, d_pd, K, tpp, P); \
                       else                                                                     \
                         hipLaunchKernelGGL((k_reduce<false, false, kAccum, 1, R, true, 0, BS, F>), dim3(tpp * P), dim3(BS), 0, s, bp, d_pd, K, tpp, P); \
                     },                                                                         \
                     (double)P * (K + 2) * L * 8, {}})
  if (getenv("SWEEP_ACCUM")) {   // ACCUM start (reads the target): shipped R=8 x 1024 lanes vs R=16 at fewer lanes
    ADDACC(8, 1024, 0);
    ADDACC(16, 512, 0);
    ADDACC(16, 256, 0);
    ADDACC(8, 1024, 42);
    ADDACC(16, 512, 42);
  }
#undef ADDACC
  if (getenv("SWEEP_TAIL")) {   // fence every 2, the last T vectors of a peer unfenced (SEQF = 2 + 10*T)
    ADDS(16, 0, 2);
    ADDS(16, 0, 22);
    ADDS(16, 0, 42);
    ADDS(16, 0, 62);
    ADDS(16, 0, 82);
    ADDS(16, 0, 32);
    ADDS(16, 0, 52);
    ADDS(16, 0, 44);
    ADDS(16, 0, 84);
  }
  if (getenv("SWEEP_TAIL1")) {   // fence every 1 or 3 vectors with a free tail (SEQF = F + 10*T)
    ADDS(16, 0, 42);
    ADDS(16, 0, 41);
    ADDS(16, 0, 71);
    ADDS(16, 0, 91);
    ADDS(16, 0, 3);
    ADDS(16, 0, 43);
    ADDS(16, 0, 73);
  }
  if (getenv("SWEEP_MAP3")) {   // block order under the shipped SEQF = 3 schedule
    ADDS(16, 0, 3);
    ADDS(16, 2, 3);
    ADDS(16, 1, 3);
  }
  if (getenv("SWEEP_TAIL2")) {   // fence periods 3..8 around the SEQF=3 result
    ADDS(16, 0, 42);
    ADDS(16, 0, 3);
    ADDS(16, 0, 13);
    ADDS(16, 0, 5);
    ADDS(16, 0, 6);
    ADDS(16, 0, 7);
    ADDS(16, 0, 8);
  }
  if (quick) {             // fence interval of the SEQ schedule (0 = hipcc's own)
    ADDS(16, 0, 0);
    ADDS(16, 0, 1);
    ADDS(16, 0, 2);
    ADDS(16, 0, 4);
    ADDS(16, 2, 2);
  }
#undef ADDS
  if (shift && !be) {
    // the same big-shape kernels over the shifted buckets: nt vs plain loads
#define ADDSH(NT, tag)                                                                             \
    vars.push_back(Var{"shifted reduce R=16 BS=1024 " tag,                                         \
                       [=](hipStream_t s) {                                                        \
                         const int64_t tile = (int64_t)1024 * 2 * 16;                              \
                         const int tpp = (int)((L - 2 + tile - 1) / tile);                         \
                         hipLaunchKernelGGL((k_reduce<false, false, kZero, 1, 16, NT, 0, 1024>), dim3(tpp * P), \
                                            dim3(1024), 0, s, (const unsigned long long* const*)d_ptrs_sh, d_pd, K, tpp, P); \
                       },                                                                          \
                       alg, {}})
    ADDSH(true, "nt");
    ADDSH(false, "plain loads");
#undef ADDSH
    vars.push_back(Var{"aligned reduce R=16 BS=1024 plain loads",
                       [=](hipStream_t s) {
                         const int64_t tile = (int64_t)1024 * 2 * 16;
                         const int tpp = (int)((L + tile - 1) / tile);
                         hipLaunchKernelGGL((k_reduce<false, false, kZero, 1, 16, false, 0, 1024>), dim3(tpp * P),
                                            dim3(1024), 0, s, (const unsigned long long* const*)d_ptrs, d_pd, K, tpp, P);
                       },
                       alg, {}});
    vars.push_back(Var{"shifted readall G=1 R=16",
                       [=](hipStream_t s) {
                         hipLaunchKernelGGL((k_readall<1, 16>), dim3((unsigned)(L / (2 * kBlock * 16)), P), dim3(kBlock), 0,
                                            s, (const unsigned long long* const*)d_ptrs_sh, K, L - 2, sink);
                       },
                       (double)P * K * (L / (2 * kBlock * 16)) * (2 * kBlock * 16) * 8, {}});
  }
  if (quick) {
  } else {
    ADDC(1, 16, 0, 256);
    ADDC(1, 16, 2, 256);
    ADDC(8, 1, 0, 256);
  }
#undef ADDC
#define EXP(R, BS, FORCE)                                                                       \
  vars.push_back(Var{"exp R=" #R " BS=" #BS " force=" #FORCE,                                    \
                     [=](hipStream_t s) {                                                       \
                       const int tpp = (int)(L / ((int64_t)BS * 2 * R));                        \
                       auto bp = (const unsigned long long* const*)d_ptrs;                      \
                       const int64_t ds = (L + 31) / 32 * 32;                                   \
                       if (be)                                                                  \
                         hipLaunchKernelGGL((k_exp<true, R, BS, FORCE>), dim3(tpp * P), dim3(BS), 0, s, bp, dst, ds, K, tpp); \
                       else                                                                     \
                         hipLaunchKernelGGL((k_exp<false, R, BS, FORCE>), dim3(tpp * P), dim3(BS), 0, s, bp, dst, ds, K, tpp); \
                     },                                                                         \
                     alg, {}})
  if (L % (1024 * 2 * 16) == 0 && !quick) {
    EXP(16, 1024, false);
    EXP(8, 1024, true);
    EXP(16, 1024, true);
    EXP(16, 512, true);
    EXP(8, 512, true);
  }
#undef EXP
#define RA(G, R)                                                                                   \
  vars.push_back(Var{"readall G=" #G " R=" #R " (read ceiling)",                                     \
                     [=](hipStream_t s) {                                                            \
                       hipLaunchKernelGGL((k_readall<G, R>), dim3((unsigned)(L / (2 * kBlock * R)), P), \
                                          dim3(kBlock), 0, s, (const unsigned long long* const*)d_ptrs, K, L, sink); \
                     },                                                                              \
                     (double)P * K * (L / (2 * kBlock * R)) * (2 * kBlock * R) * 8, {}})
  if (!quick) RA(8, 1);
  RA(1, 16);
  RA(2, 16);
#undef RA
  if (do_copy)
    vars.push_back(Var{"copy dwordx4 nt (read+write)",
                       [=](hipStream_t s) {
                         hipLaunchKernelGGL(k_copy, dim3(8192), dim3(kBlock), 0, s, (const u2*)base, (u2*)copy_out, copy_n2);
                       },
                       (double)copy_n2 * 32, {}});

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vars) v.run(0);  // warm
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
  printf("# P=%d L=%lld K=%d PAD=%lld REPS=%d  algorithmic bytes/launch=%.0f\n", P, (long long)L, K,
         (long long)PAD, REPS, alg);
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    printf("%-36s median %8.4f ms  min %8.4f ms  %8.1f GB/s (median)  %5.1f%% of 8 TB/s\n", v.name.c_str(), med,
           mn, v.bytes / med / 1e6, v.bytes / med / 1e6 / 80.0);
  }
  return 0;
}
