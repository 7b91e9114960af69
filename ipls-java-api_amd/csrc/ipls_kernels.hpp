// ipls_kernels.hpp -- gfx950 (CDNA4) HIP kernels of the IPLS aggregation path.
//
// Design:
//  * The hot kernel is a fixed-order elementwise fold over K peer buckets.
//    Each lane owns 16 contiguous bytes (2 doubles) per step and walks the
//    peers in order, so every element is ((+0.0 + b0) + b1) + ... exactly as
//    Updater.java:115-117 / IPLS.java:1740 compute it.  No shuffle or tree
//    reduction touches the peer axis: that would reassociate the sum and
//    break bit parity (SURVEY.md §7 "Order vs. shuffles").
//  * Memory-level parallelism comes from issuing the loads of G peers
//    (G x 16 B per lane) before folding them; bucket base pointers are
//    wave-uniform (scalar loads from a device table).
//  * Wavefront DPP reductions + LDS staging are used where the reduction is
//    order-free: the integer checksum kernel (exact, any association).
//  * Compiled with -ffp-contract=off; double division is the IEEE-correct
//    v_div_scale/v_div_fmas/v_div_fixup sequence (no fast-math).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef IPLS_ROT
#define IPLS_ROT 0
#endif
// IPLS_ROUND_PAIRS=1: the fused round's wave-pair tile layout (reduce_tiles);
// the =0 build (the round-2 layout) is the A/B variant
#ifndef IPLS_ROUND_PAIRS
#define IPLS_ROUND_PAIRS 1
#endif

namespace ipls {

typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
typedef unsigned u4w __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;

enum Start : int { kAccum = 0, kZero = 1, kFirst = 2 };

struct PartDesc {
  int64_t len;                      // L_p incl. count slot
  unsigned long long* dst;          // target: an arena accumulator or a caller buffer
  // fused-round fields (k_round only):
  const unsigned long long* init;   // START_ACCUM source (the AGG accumulator)
  const unsigned long long* rep;    // REP accumulator, or null = logically +0.0
  unsigned long long* avg;          // averaged values out (L-1 doubles), or null
};

// Global-address-space views.  Bucket pointers come from a device table, so
// the compiler cannot infer their address space and would emit flat_load with
// a vmcnt(0)+lgkmcnt(0) wait after EVERY load (fully serialised).  Casting to
// addrspace(1) gives global_load and counted vmcnt waits.
#define IPLS_GLOBAL __attribute__((address_space(1)))
typedef const IPLS_GLOBAL u2* gcu2;
typedef IPLS_GLOBAL u2* gu2;
typedef const IPLS_GLOBAL unsigned long long* gcu64;
typedef IPLS_GLOBAL unsigned long long* gu64;

// NOTE: never __builtin_bit_cast(double, v.y) on an ext_vector element: hipcc
// (ROCm 7.2) lowers it to element 0 (measured in the ISA).  Copy the element
// to a scalar first, or bit_cast the whole vector.
__device__ __forceinline__ double be_to_f64(unsigned long long v) {
  return __builtin_bit_cast(double, __builtin_bswap64(v));
}
__device__ __forceinline__ unsigned long long f64_to_be(double v) {
  return __builtin_bswap64(__builtin_bit_cast(unsigned long long, v));
}

template <bool NT>
__device__ __forceinline__ u2 ld16(const unsigned long long* p) {
  if constexpr (NT) return __builtin_nontemporal_load((gcu2)p);
  else return *(gcu2)p;
}
__device__ __forceinline__ unsigned long long ld8(const unsigned long long* p) { return *(gcu64)p; }
__device__ __forceinline__ void st8(unsigned long long* p, unsigned long long v) { *(gu64)p = v; }

template <bool BE>
__device__ __forceinline__ d2 decode2(u2 raw) {
  if constexpr (BE) {
    const unsigned long long a = raw.x, b = raw.y;
    u2 s;
    s.x = __builtin_bswap64(a);
    s.y = __builtin_bswap64(b);
    return __builtin_bit_cast(d2, s);
  } else {
    return __builtin_bit_cast(d2, raw);
  }
}
template <bool BE>
__device__ __forceinline__ u2 encode2(d2 v) {
  u2 raw = __builtin_bit_cast(u2, v);
  if constexpr (BE) {
    const unsigned long long a = raw.x, b = raw.y;
    raw.x = __builtin_bswap64(a);
    raw.y = __builtin_bswap64(b);
  }
  return raw;
}
template <bool BE>
__device__ __forceinline__ double decode1(unsigned long long raw) {
  if constexpr (BE) return be_to_f64(raw);
  else return __builtin_bit_cast(double, raw);
}

// ---------------------------------------------------------------------------
// k_reduce: target[q] = fold(start; bufs[q*k + 0..k-1]) for the partitions of
// one batch.  Grid = n_parts * tiles_per_part blocks of 256 lanes; a tile is
// 256 * 2 * R doubles.  Full tiles take the vector path; the one partial tile
// per partition takes a scalar path (odd lengths, e.g. ETHModel's 147,869).
//   BE_IN  : buckets hold big-endian doubles (IPFS file bytes) -> bswap fused
//   BE_OUT : write the sum as big-endian bytes (update_file), else doubles
//   G      : peers whose loads are in flight together per lane
//   R      : 16-byte vectors per lane per tile
//   NT     : non-temporal loads (each byte is read exactly once)
//   MAP    : block -> (partition, tile) order.  0 = partition-major;
//            1 = tile-major (consecutive blocks in different partitions);
//            2 = XCD-chunked: blocks b, b+8, b+16.. (one XCD under the observed
//                round-robin dispatch) walk one contiguous 1/8 of the work, so
//                the 8 XCDs stream 8 distant regions (speed only, never
//                correctness: any placement computes the same result).
// ---------------------------------------------------------------------------
//            MAP 2 needs gridDim.x padded to a multiple of 8 (grid_blocks());
//            the padding blocks map past the last tile and exit.
__host__ __device__ constexpr int64_t grid_blocks(int map, int64_t tiles) {
  return map == 2 ? (tiles + 7) / 8 * 8 : tiles;
}

//            3 = partial tiles first: blocks [0, n_parts) take the last tile of
//                each partition (partial when L is not a multiple of the tile),
//                the rest the full tiles partition-major.  With 1 workgroup per
//                CU the short partial blocks then run beside the first round of
//                full tiles instead of pushing full tiles into an extra round
//                (L = 4194305: 2064 blocks = 8 rounds + 15 full tiles alone).
__device__ __forceinline__ void map_block(int map, int nblocks, int tiles_per_part, int n_parts, int& q, int& t) {
  int b = blockIdx.x;
  if (map == 3) {
    if (b < n_parts) {
      q = b;
      t = tiles_per_part - 1;
    } else {
      b -= n_parts;
      q = b / (tiles_per_part - 1);
      t = b - q * (tiles_per_part - 1);
    }
    return;
  }
  if (map == 2) {
    const int per = nblocks >> 3;  // nblocks % 8 == 0 (grid_blocks)
    b = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (b >= tiles_per_part * n_parts) { q = n_parts; t = 0; return; }
  }
  if (map == 1) {
    q = b % n_parts;
    t = b / n_parts;
  } else {
    q = b / tiles_per_part;
    t = b - q * tiles_per_part;
  }
}

//   BS     : lanes per workgroup
//   FIN    : fused round -- dst is Weights[p] and receives fold + REP
//            (AggregatePartition, IPLS.java:1256), and parts[q].avg (if set)
//            the GetPartitions divide (IPLS.java:1159-1174), in the same pass
template <bool BE_IN, bool BE_OUT, int START, int G, int R, bool NT, int MAP, int BS, bool FIN, int SEQF>
__device__ __forceinline__ void reduce_tiles(
    const unsigned long long* const* __restrict__ bufs, const PartDesc* __restrict__ parts,
    int k, int tiles_per_part, int n_parts, int secure, const double* __restrict__ cnts) {
  constexpr int kBlock = BS;   // lanes per workgroup (shadows the namespace default)
  constexpr int64_t kTile = (int64_t)kBlock * 2 * R;
  int q, t;
  map_block(MAP, gridDim.x, tiles_per_part, n_parts, q, t);
  if (q >= n_parts) return;
  const int64_t L = parts[q].len;
  const int64_t base = (int64_t)t * kTile;
  if (base >= L) return;
  unsigned long long* __restrict__ dst = parts[q].dst;
  const unsigned long long* const* __restrict__ pb = bufs + (size_t)q * k;
  const int tid = threadIdx.x;
  const int j0 = (START == kFirst) ? 1 : 0;
  static_assert(!(FIN && BE_OUT), "the fused round writes native Weights");
  // ACCUM source: the target itself, or AGG when the round is fused
  const unsigned long long* __restrict__ init = FIN ? parts[q].init : dst;
  const unsigned long long* __restrict__ rep = FIN ? parts[q].rep : nullptr;
  unsigned long long* __restrict__ avg = FIN ? parts[q].avg : nullptr;
  // count slot W[L-1] (k_round_counts folded it exactly as element L-1 is)
  double den = 0.0, cnt = 0.0;
  if constexpr (FIN) {
    if (avg) {
      cnt = cnts[q];
      den = secure ? 1e12 * cnt : cnt;   // Math.pow(10,12) * W[last] (IPLS.java:1167)
    }
  }
  const bool avg_aligned = FIN && !((uintptr_t)avg & 15);
  // fused epilogue for element e holding fold value a: W = a + REP; avg = W / count
  auto fin1 = [&](int64_t e, double a) {
    const double w = a + (rep ? __builtin_bit_cast(double, ld8(rep + e)) : 0.0);
    st8(dst + e, __builtin_bit_cast(unsigned long long, w));
    if (avg && e < L - 1) st8(avg + e, __builtin_bit_cast(unsigned long long, cnt == 0.0 ? w : w / den));
  };

  if (base + kTile <= L) {
    // ---------------- vector path: R x 16 B per lane ----------------
    // (hipcc, held to 128 VGPRs by the 1024-lane bound, issues a peer's R
    // loads one or two at a time per wave (checked in the ISA); the 16 waves
    // of a CU then sweep one 16 KiB window of the bucket at a time, which is
    // the DRAM pattern that measured best -- forcing all R loads in flight
    // with scheduling barriers was slower.)
    int64_t off[R];
    // IPLS_ROT=1 (A/B builds only): tile t visits its R sub-windows starting
    // at sub-window t mod R, so neighbouring tiles in flight at the same loop
    // step touch different offsets of their chunks (accumulator r always
    // pairs with the same sub-window, so every element's fold is unchanged)
#if IPLS_ROT
    const int rot = t & (R - 1);
#else
    constexpr int rot = 0;
#endif
    // PAIRS (the fused round): a wave's vectors 2m and 2m+1 are adjacent 1 KiB
    // pieces, so a wave owns 2 KiB contiguous per pair (the CU still sweeps one
    // window of each bucket per two vectors), and an averages run at 8 mod 16
    // needs single 8-B stores every 2 KiB instead of every 1 KiB (epilogue).
    // Same elements, same fold: bit-identical; +0.3 to +0.8 points on config
    // C's round in three processes (profiles/r03/an/pairs2_probe.jsonl).
    constexpr bool PAIRS = FIN && IPLS_ROUND_PAIRS && (R % 2 == 0);
    if constexpr (PAIRS) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        off[r] = base + 2 * ((int64_t)(r >> 1) * 2 * kBlock + (tid >> 6) * 128 + (r & 1) * 64 + (tid & 63));
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) off[r] = base + 2 * ((int64_t)((r + rot) & (R - 1)) * kBlock + tid);
    }

    // SEQ: one peer per step, each of its R vectors loaded, decoded and added
    // before the next is issued (a scheduling fence between them).  This is
    // the schedule hipcc picks by itself for native doubles; with the bswap
    // (or the ACCUM read of the target) in between it would hoist the loads
    // instead and spill at R = 16.
    constexpr bool SEQ = SEQF > 0 && G == 1;
    d2 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if constexpr (START == kZero) {
        acc[r] = d2{0.0, 0.0};
      } else if constexpr (START == kFirst) {
        acc[r] = decode2<BE_IN>(ld16<NT>(pb[0] + off[r]));
      } else {  // kAccum: the target holds native doubles (or BE if BE_OUT)
        acc[r] = decode2<BE_OUT>(ld16<false>(init + off[r]));
      }
      if constexpr (SEQ && START != kZero) __builtin_amdgcn_sched_barrier(0);
    }
    int j = j0;
    if constexpr (SEQ) {
      for (; j < k; ++j) {
        const unsigned long long* __restrict__ src = pb[j];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const d2 x = decode2<BE_IN>(ld16<NT>(src + off[r]));
          acc[r].x = acc[r].x + x.x;
          acc[r].y = acc[r].y + x.y;
          // SEQF = F + 10*T: a fence after every F vectors, none among the last T
          if constexpr (SEQF > 0)
            if ((r + 1) % (SEQF % 10) == 0 && r + 1 < R - SEQF / 10) __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else {
    for (; j + G <= k; j += G) {
      u2 v[G][R];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const unsigned long long* __restrict__ src = pb[j + g];
#pragma unroll
        for (int r = 0; r < R; ++r) v[g][r] = ld16<NT>(src + off[r]);
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          d2 x = decode2<BE_IN>(v[g][r]);
          acc[r].x = acc[r].x + x.x;
          acc[r].y = acc[r].y + x.y;
        }
      }
    }
    for (; j < k; ++j) {
      const unsigned long long* __restrict__ src = pb[j];
      u2 v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = ld16<NT>(src + off[r]);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        d2 x = decode2<BE_IN>(v[r]);
        acc[r].x = acc[r].x + x.x;
        acc[r].y = acc[r].y + x.y;
      }
    }
    }  // !SEQ
    if constexpr (FIN) {
      // W = fold + REP (AggregatePartition, IPLS.java:1256), and the averages'
      // R stores before W's: two runs of stores per wave instead of
      // alternating between the two streams every vector
      // (tools/round_epilogue_sweep.hip, profiles/r02/s4/round_epilogue.txt)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (rep) {
          const d2 y = decode2<false>(ld16<true>(rep + off[r]));
          acc[r].x = acc[r].x + y.x;
          acc[r].y = acc[r].y + y.y;
        } else {
          acc[r].x = acc[r].x + 0.0;   // AGG + REP with REP == +0.0, as AggregatePartition computes it
          acc[r].y = acc[r].y + 0.0;
        }
        if (avg) {
          // averages of elements e, e+1 (e + 1 may be the count slot L-1, which is not output)
          const int64_t e = off[r];
          const double ax = cnt == 0.0 ? acc[r].x : acc[r].x / den;
          const double ay = cnt == 0.0 ? acc[r].y : acc[r].y / den;
          if (avg_aligned) {
            if (e + 1 < L - 1) __builtin_nontemporal_store(encode2<false>(d2{ax, ay}), (gu2)(avg + e));
            else st8(avg + e, __builtin_bit_cast(unsigned long long, ax));
          } else if constexpr (PAIRS) {
            // piece r pairs its lane-63 y with piece r+1's lane-0 x (r even);
            // piece r+1 directly follows piece r, so singles fall every 2 KiB
            const int lane = tid & 63;
            const double nx = __shfl_down(ax, 1);
            if ((r & 1) == 0) {
              const double nb = acc[r + 1].x + (rep && lane == 0 ? __builtin_bit_cast(double, ld8(rep + off[r + 1])) : 0.0);
              const double b0 = __shfl(cnt == 0.0 ? nb : nb / den, 0);
              if (lane == 0) st8(avg + e, __builtin_bit_cast(unsigned long long, ax));
              __builtin_nontemporal_store(encode2<false>(d2{ay, lane < 63 ? nx : b0}), (gu2)(avg + e + 1));
            } else {
              if (lane < 63) __builtin_nontemporal_store(encode2<false>(d2{ay, nx}), (gu2)(avg + e + 1));
              else if (e + 1 < L - 1) st8(avg + e + 1, __builtin_bit_cast(unsigned long long, ay));
            }
          } else {
            // avg + e is 8 mod 16: lane t writes the aligned pair (e+1, e+2) =
            // (its y, lane t+1's x); the wave's first x and last y go alone.
            const double nx = __shfl_down(ax, 1);
            const int lane = tid & 63;
            if (lane == 0) st8(avg + e, __builtin_bit_cast(unsigned long long, ax));
            if (lane < 63) __builtin_nontemporal_store(encode2<false>(d2{ay, nx}), (gu2)(avg + e + 1));
            else if (e + 1 < L - 1) st8(avg + e + 1, __builtin_bit_cast(unsigned long long, ay));
          }
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) __builtin_nontemporal_store(encode2<false>(acc[r]), (gu2)(dst + off[r]));
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) __builtin_nontemporal_store(encode2<BE_OUT>(acc[r]), (gu2)(dst + off[r]));
    }
  } else {
    // ------- partial last tile: 2*BS-element vector steps, scalar remainder -------
    constexpr int kPB = 8;
    for (int64_t sb = base; sb < L; sb += 2 * kBlock) {
      const int64_t i = sb + 2 * tid;
      if (sb + 2 * kBlock <= L) {
        d2 acc;
        if constexpr (START == kZero) acc = d2{0.0, 0.0};
        else if constexpr (START == kFirst) acc = decode2<BE_IN>(ld16<NT>(pb[0] + i));
        else acc = decode2<BE_OUT>(ld16<false>(init + i));
        // peers in groups of kPB loads in flight (the fold order is unchanged):
        // a one-at-a-time chain of k dependent loads made this block take longer
        // than a full tile
        int jj = j0;
        for (; jj + kPB <= k; jj += kPB) {
          u2 v[kPB];
#pragma unroll
          for (int g = 0; g < kPB; ++g) v[g] = ld16<NT>(pb[jj + g] + i);
#pragma unroll
          for (int g = 0; g < kPB; ++g) {
            const d2 x = decode2<BE_IN>(v[g]);
            acc.x = acc.x + x.x;
            acc.y = acc.y + x.y;
          }
        }
        for (; jj < k; ++jj) {
          const d2 x = decode2<BE_IN>(ld16<NT>(pb[jj] + i));
          acc.x = acc.x + x.x;
          acc.y = acc.y + x.y;
        }
        if constexpr (FIN) {
          fin1(i, acc.x);
          fin1(i + 1, acc.y);
        } else {
          __builtin_nontemporal_store(encode2<BE_OUT>(acc), (gu2)(dst + i));
        }
      } else {
        for (int64_t e = sb + tid; e < L; e += kBlock) {
          double acc;
          if constexpr (START == kZero) acc = 0.0;
          else if constexpr (START == kFirst) acc = decode1<BE_IN>(ld8(pb[0] + e));
          else acc = decode1<BE_OUT>(ld8(init + e));
          int jj = j0;
          for (; jj + kPB <= k; jj += kPB) {
            unsigned long long v[kPB];
#pragma unroll
            for (int g = 0; g < kPB; ++g) v[g] = ld8(pb[jj + g] + e);
#pragma unroll
            for (int g = 0; g < kPB; ++g) acc = acc + decode1<BE_IN>(v[g]);
          }
          for (; jj < k; ++jj) acc = acc + decode1<BE_IN>(ld8(pb[jj] + e));
          if constexpr (FIN) fin1(e, acc);
          else st8(dst + e, BE_OUT ? f64_to_be(acc) : __builtin_bit_cast(unsigned long long, acc));
        }
      }
    }
  }
}

// The batched fold (the benchmarked kernel) and the fused round are two
// kernels over the same tile code, so profiles name them apart.
template <bool BE_IN, bool BE_OUT, int START, int G, int R, bool NT, int MAP = 0, int BS = kBlock, int SEQF = 0>
__global__ __launch_bounds__(BS) void k_reduce(const unsigned long long* const* __restrict__ bufs,
                                               const PartDesc* __restrict__ parts, int k, int tiles_per_part,
                                               int n_parts) {
  reduce_tiles<BE_IN, BE_OUT, START, G, R, NT, MAP, BS, false, SEQF>(bufs, parts, k, tiles_per_part, n_parts, 0,
                                                                     nullptr);
}

template <bool BE_IN, int START, int G, int R, int MAP = 0, int BS = kBlock, int SEQF = 0>
__global__ __launch_bounds__(BS) void k_round(const unsigned long long* const* __restrict__ bufs,
                                              const PartDesc* __restrict__ parts, int k, int tiles_per_part,
                                              int n_parts, int secure, const double* __restrict__ cnts) {
  reduce_tiles<BE_IN, false, START, G, R, true, MAP, BS, true, SEQF>(bufs, parts, k, tiles_per_part, n_parts, secure,
                                                               cnts);
}

// Shape of the elementwise kernels below (k_fold_n, k_blend, k_scale,
// k_encode_secure) when every operand is 16-B aligned (VEC, decided by the
// host): a block of kBlock lanes owns kEwTile consecutive elements, each lane
// kEwV 16-B vectors, loads first, then the arithmetic and stores; the one
// partial tile goes element by element.  Otherwise (a bucket at an 8 mod 16
// address, e.g. a payload inside a Java-serialised file) the 8-B grid-stride
// loop.  Same per-element expressions, so the same bits either way.  From
// cold caches at 64 Mi elements the tiles take k_blend from 56 to 75 %,
// k_scale from 62 to 79 % and k_fold_n from 59 to 75 % of 8 TB/s
// (tools/elementwise_sweep.hip, profiles/r04/zl/).
constexpr int kEwV = 4;
constexpr int64_t kEwTile = (int64_t)kBlock * 2 * kEwV;

// Elementwise fold of one bucket of n doubles into dst (off the hot path:
// Download_Scheduler's Other_Replica_Gradients and their Collect_Replicas fold).
//   FIRST: dst[i] = decode(src[i])          (GetParameters(Hash): a new array)
//   else : dst[i] = dst[i] + decode(src[i])
template <bool BE_IN, bool FIRST, bool VEC = false>
__global__ __launch_bounds__(kBlock) void k_fold_n(unsigned long long* __restrict__ dst,
                                                   const unsigned long long* __restrict__ src, int64_t n) {
  auto one = [&](int64_t i) {
    const double x = decode1<BE_IN>(ld8(src + i));
    const double y = FIRST ? x : __builtin_bit_cast(double, ld8(dst + i)) + x;
    st8(dst + i, __builtin_bit_cast(unsigned long long, y));
  };
  if constexpr (VEC) {
    const int64_t base = (int64_t)blockIdx.x * kEwTile;
    if (base + kEwTile <= n) {
      u2 sv[kEwV], dv[kEwV];
#pragma unroll
      for (int v = 0; v < kEwV; ++v) {
        const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
        sv[v] = __builtin_nontemporal_load((gcu2)(src + i));
        if constexpr (!FIRST) dv[v] = *(gcu2)(dst + i);
      }
#pragma unroll
      for (int v = 0; v < kEwV; ++v) {
        const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
        d2 o = decode2<BE_IN>(sv[v]);
        if constexpr (!FIRST) {
          const d2 y = __builtin_bit_cast(d2, dv[v]);
          o.x = y.x + o.x;
          o.y = y.y + o.y;
        }
        *(gu2)(dst + i) = __builtin_bit_cast(u2, o);
      }
      return;
    }
    for (int64_t i = base + threadIdx.x; i < n; i += kBlock) one(i);
  } else {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) one(i);
  }
}

// Count slot of a fused round, one wave per partition: the same fold k_round
// applies to element L-1, i.e. W[L-1] =
// (init[L-1] | +0.0) + b_0[L-1] + ... + b_{k-1}[L-1] + (REP[L-1] | +0.0).
// Lane j loads b_j[L-1] (64 independent loads in flight instead of a chain of
// k pointer + value loads), then every lane adds the broadcast values in peer
// order -- the identical expression, so the identical bits.
template <bool BE_IN, int START>
__global__ __launch_bounds__(64) void k_round_counts(const unsigned long long* const* __restrict__ bufs,
                                                     const PartDesc* __restrict__ parts, int k, int n_parts,
                                                     double* __restrict__ cnts) {
  const int q = blockIdx.x;
  if (q >= n_parts) return;
  const int lane = threadIdx.x;
  const PartDesc d = parts[q];
  const int64_t e = d.len - 1;
  const unsigned long long* const* pb = bufs + (size_t)q * k;
  double c = (START == kZero) ? 0.0 : __builtin_bit_cast(double, ld8(d.init + e));
  for (int j0 = 0; j0 < k; j0 += 64) {
    const int j = j0 + lane;
    const double v = j < k ? decode1<BE_IN>(ld8(pb[j] + e)) : 0.0;
    const int m = k - j0 < 64 ? k - j0 : 64;
    for (int t = 0; t < m; ++t) c = c + __shfl(v, t);
  }
  if (lane == 0) cnts[q] = c + (d.rep ? __builtin_bit_cast(double, ld8(d.rep + e)) : 0.0);
}

// Same fold for buckets that are only 8-byte aligned (e.g. a device view into
// a frame payload): one double per lane per step.
template <bool BE_IN, bool BE_OUT, int START>
__global__ __launch_bounds__(kBlock) void k_reduce_scalar(
    const unsigned long long* const* __restrict__ bufs, const PartDesc* __restrict__ parts,
    int k, int tiles_per_part, int64_t tile) {
  const int q = blockIdx.x / tiles_per_part;
  const int t = blockIdx.x - q * tiles_per_part;
  const int64_t L = parts[q].len;
  const int64_t base = (int64_t)t * tile;
  if (base >= L) return;
  unsigned long long* __restrict__ dst = parts[q].dst;
  const unsigned long long* const* __restrict__ pb = bufs + (size_t)q * k;
  const int64_t end = (base + tile < L) ? base + tile : L;
  const int j0 = (START == kFirst) ? 1 : 0;
  for (int64_t i = base + threadIdx.x; i < end; i += kBlock) {
    double acc;
    if constexpr (START == kZero) acc = 0.0;
    else if constexpr (START == kFirst) acc = decode1<BE_IN>(ld8(pb[0] + i));
    else acc = decode1<BE_OUT>(ld8(dst + i));
    for (int j = j0; j < k; ++j) acc = acc + decode1<BE_IN>(ld8(pb[j] + i));
    st8(dst + i, BE_OUT ? f64_to_be(acc) : __builtin_bit_cast(unsigned long long, acc));
  }
}

// ---------------------------------------------------------------------------
// k_fold1: the single-bucket fold of one arrival (Updater._Update,
// Updater.java:115-117), pointers passed as kernel arguments -- no table
// upload, so a per-arrival fold is one launch and nothing else on the stream.
//   dst[i] = start(dst[i]) + decode(src[i]),  start: ZERO +0.0 | ACCUM dst | FIRST none
// 16-B aligned src/dst; R pairs per lane in flight (zero-copy sources are
// read over PCIe, where more outstanding requests per lane pay).
// ---------------------------------------------------------------------------
template <bool BE_IN, bool BE_OUT, int START, int R = 4>
__global__ __launch_bounds__(kBlock) void k_fold1(unsigned long long* __restrict__ dst,
                                                  const unsigned long long* __restrict__ src, int64_t L) {
  const int64_t n2 = L >> 1;   // whole pairs
  const int64_t stride = (int64_t)gridDim.x * kBlock * R;
  auto fold = [&](const u2& v, const u2& t) -> u2 {
    const d2 x = decode2<BE_IN>(v);
    if constexpr (START == kFirst) return encode2<BE_OUT>(x);
    d2 a = (START == kZero) ? d2{0.0, 0.0} : decode2<BE_OUT>(t);
    a.x = a.x + x.x;
    a.y = a.y + x.y;
    return encode2<BE_OUT>(a);
  };
  int64_t b = (int64_t)blockIdx.x * kBlock * R + threadIdx.x;
  for (; b + (int64_t)(R - 1) * kBlock < n2; b += stride) {   // all R pairs in range: loads first
    u2 v[R], t[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = ld16<true>(src + 2 * (b + r * kBlock));
    if constexpr (START == kAccum) {
#pragma unroll
      for (int r = 0; r < R; ++r) t[r] = ld16<false>(dst + 2 * (b + r * kBlock));
    }
#pragma unroll
    for (int r = 0; r < R; ++r) __builtin_nontemporal_store(fold(v[r], t[r]), (gu2)(dst + 2 * (b + r * kBlock)));
  }
  for (int r = 0; r < R; ++r) {   // this lane's last, partial group
    const int64_t i2 = b + r * kBlock;
    if (i2 < n2) {
      const u2 t = (START == kAccum) ? ld16<false>(dst + 2 * i2) : u2{0, 0};
      __builtin_nontemporal_store(fold(ld16<true>(src + 2 * i2), t), (gu2)(dst + 2 * i2));
    }
  }
  if ((L & 1) && blockIdx.x == 0 && threadIdx.x == 0) {   // odd length: the last element
    const int64_t e = L - 1;
    const double x = decode1<BE_IN>(ld8(src + e));
    double a;
    if constexpr (START == kFirst) a = x;
    else a = ((START == kZero) ? 0.0 : decode1<BE_OUT>(ld8(dst + e))) + x;
    st8(dst + e, BE_OUT ? f64_to_be(a) : __builtin_bit_cast(unsigned long long, a));
  }
}

// ---------------------------------------------------------------------------
// k_finalize: AggregatePartition (IPLS.java:1255-1270) over a batch.
//   W[i] = AGG[i] + REP[i]  (REP_ZERO: AGG[i] + 0.0 without reading REP)
//   Weight_Address is the same array as Weights (IPLS.java:1141 aliases them).
//   AGG/REP are zeroed unless the host marks them "logically zero" instead.
// ---------------------------------------------------------------------------
struct FinDesc {
  int64_t len;
  int64_t agg_off, rep_off, w_off;
};

// 16-B vectors per lane of k_finalize / k_divide (tile = kBlock * 2 * kV doubles)
constexpr int kFinV = 8, kDivV = 4;   // tools/copy_sweep.hip, profiles/r02/s3/copy_sweep.txt
constexpr int64_t kFinTile = (int64_t)kBlock * 2 * kFinV, kDivTile = (int64_t)kBlock * 2 * kDivV;

//   BS, V: lanes per workgroup and 16-B vectors per lane (tile = BS * 2 * V
//   doubles); the host launches the defaults (tools/copy_sweep.hip sweeps them)
template <bool REP_ZERO, bool ZERO_ACC, int BS = kBlock, int V = kFinV>
__global__ __launch_bounds__(BS) void k_finalize(const FinDesc* __restrict__ parts,
                                                 double* __restrict__ arena,
                                                 int tiles_per_part) {
  // 16 B per lane per step (arena arrays are 256-B aligned), V steps per lane.
  constexpr int kBlock = BS;
  constexpr int kV = V;
  constexpr int64_t kTile = (int64_t)kBlock * 2 * kV;
  const int q = blockIdx.x / tiles_per_part;
  const int t = blockIdx.x - q * tiles_per_part;
  const FinDesc d = parts[q];
  const int64_t base = (int64_t)t * kTile;
  if (base >= d.len) return;
  const int64_t end = (base + kTile < d.len) ? base + kTile : d.len;
  double* agg = arena + d.agg_off;
  double* rep = arena + d.rep_off;
  double* w = arena + d.w_off;
  if (end - base == kTile) {
    u2 a[kV], r[kV];
#pragma unroll
    for (int v = 0; v < kV; ++v) {
      const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
      a[v] = __builtin_nontemporal_load((gcu2)(agg + i));
      if constexpr (!REP_ZERO) r[v] = __builtin_nontemporal_load((gcu2)(rep + i));
    }
#pragma unroll
    for (int v = 0; v < kV; ++v) {
      const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
      const d2 x = __builtin_bit_cast(d2, a[v]);
      const d2 y = REP_ZERO ? d2{0.0, 0.0} : __builtin_bit_cast(d2, r[v]);
      d2 o;
      o.x = x.x + y.x;
      o.y = x.y + y.y;
      // nt stores: plain ones run this kernel ~5 % faster but leave W dirty in
      // the caches, and the next kernel (the GetPartitions divide reading W)
      // pays the write-back: nt in both is the fastest round
      __builtin_nontemporal_store(__builtin_bit_cast(u2, o), (gu2)(w + i));
      if constexpr (ZERO_ACC) {
        __builtin_nontemporal_store(u2{0, 0}, (gu2)(agg + i));
        if constexpr (!REP_ZERO) __builtin_nontemporal_store(u2{0, 0}, (gu2)(rep + i));
      }
    }
    return;
  }
  for (int64_t i = base + threadIdx.x; i < end; i += kBlock) {
    const double a = agg[i];
    const double r = REP_ZERO ? 0.0 : rep[i];
    w[i] = a + r;
    if constexpr (ZERO_ACC) {
      agg[i] = 0.0;
      if constexpr (!REP_ZERO) rep[i] = 0.0;
    }
  }
}

// ---------------------------------------------------------------------------
// k_divide: GetPartitions (IPLS.java:1159-1174) -> flat model.
//   out[m] = cnt == 0.0 ? W[p][j] : W[p][j] / cnt      (secure: / (1e12*cnt))
//   m = p*chunk + j.  OUT_BE writes DataOutputStream.writeDouble bytes
//   (big-endian, NaN canonicalised, Middleware.java:164-170).
// ---------------------------------------------------------------------------
struct DivDesc {
  int64_t len;    // L_p
  int64_t w_off;  // arena offset of Weights[p]
  int64_t out_off;
};

template <bool OUT_BE, bool SECURE, int BS = kBlock, int V = kDivV>
__global__ __launch_bounds__(BS) void k_divide(const DivDesc* __restrict__ parts,
                                               const double* __restrict__ arena,
                                               unsigned long long* __restrict__ out,
                                               int tiles_per_part) {
  // The flat output offset p*chunk is arbitrary, so the tiles are laid over
  // the OUTPUT: block 0 first writes the `head` elements up to the first 128-B
  // line boundary of this partition's output, then every wave stores whole
  // lines (64 lanes x 16 B = 8 lines), and each lane reads its two W values
  // with 8-B loads (W's alignment relative to the output is arbitrary; reads
  // of partial lines cost little, partial-line writes do).  A wave's V steps
  // cover V adjacent KiB of the output (wave-contiguous), so the W line one
  // step's window shares with the next is read by the same wave back to back:
  // 2-2.5 % faster than every wave of the block taking one KiB per step, with
  // 1.025x read PMC against 1.029x (tools/copy_sweep.hip "8B wc",
  // profiles/r05/m/).
  constexpr int kBlock = BS;
  constexpr int kV = V;
  constexpr int64_t kTile = (int64_t)kBlock * 2 * kV;
  static_assert(BS % 64 == 0, "whole waves");
  const int q = blockIdx.x / tiles_per_part;
  const int t = blockIdx.x - q * tiles_per_part;
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
  if (base + kTile <= n) {
    // element index of this lane's pair at step v: wave (threadIdx.x / 64) owns
    // [base + wave * 128 * V, + 128 * V)
    const int64_t wave_base = base + (int64_t)(threadIdx.x >> 6) * 128 * kV + 2 * (threadIdx.x & 63);
    double x[kV][2];
#pragma unroll
    for (int v = 0; v < kV; ++v) {
      const int64_t i = wave_base + (int64_t)v * 128;
      x[v][0] = __builtin_nontemporal_load((const __attribute__((address_space(1))) double*)(w + i));
      x[v][1] = __builtin_nontemporal_load((const __attribute__((address_space(1))) double*)(w + i + 1));
    }
#pragma unroll
    for (int v = 0; v < kV; ++v) {
      const int64_t i = wave_base + (int64_t)v * 128;
      u2 v2;
      v2.x = f(x[v][0]);
      v2.y = f(x[v][1]);
      __builtin_nontemporal_store(v2, (gu2)(o + i));
    }
    return;
  }
  for (int64_t i = base + threadIdx.x; i < n; i += kBlock) o[i] = f(w[i]);
}

// ---------------------------------------------------------------------------
// k_split: OrganizeGradients (IPLS.java:1018-1040) for one partition:
//   dst[j] = flat[p*chunk + j] for j < min(chunk, n - p*chunk) (guarded),
//   dst[stop] = 1.0, rest 0.0.  Optional fused fold into an accumulator
//   (UpdateGradient own-accumulate, IPLS.java:1737-1743).
// ---------------------------------------------------------------------------
//   MODE 0: dst = v (OrganizeGradients' split; BE_OUT packs big-endian)
//   MODE 1: dst = dst + v (own accumulate into AGG, IPLS.java:1737-1743)
//   MODE 2: dst = +0.0 + v (the same into a logically-zero AGG: the zeros are
//           not read, and the bits equal a fold into a zeroed array)
//   VEC: the elementwise tile shape (see k_fold_n) when flat + lo and dst are
//   16-B aligned; tiles wholly inside [0, ncopy) go 16 B at a time, the tile
//   that holds the count slot element by element.
template <bool BE_IN, bool BE_OUT, int MODE, bool VEC = false>
__global__ __launch_bounds__(kBlock) void k_split(const unsigned long long* __restrict__ flat,
                                                  int64_t lo, int64_t ncopy, int64_t L,
                                                  unsigned long long* __restrict__ dst) {
  static_assert(MODE == 0 || !BE_OUT, "the folds write native doubles");
  auto one = [&](int64_t i) {
    double v;
    if (i < ncopy) v = decode1<BE_IN>(flat[lo + i]);
    else if (i == ncopy) v = 1.0;
    else v = 0.0;
    if constexpr (MODE == 1) {
      const double a = __builtin_bit_cast(double, dst[i]);
      dst[i] = __builtin_bit_cast(unsigned long long, a + v);
    } else if constexpr (MODE == 2) {
      dst[i] = __builtin_bit_cast(unsigned long long, 0.0 + v);
    } else {
      dst[i] = BE_OUT ? f64_to_be(v) : __builtin_bit_cast(unsigned long long, v);
    }
  };
  if constexpr (VEC) {
    const int64_t base = (int64_t)blockIdx.x * kEwTile;
    if (base + kEwTile <= ncopy) {
      const unsigned long long* src = flat + lo;
      u2 sv[kEwV], dv[kEwV];
#pragma unroll
      for (int k = 0; k < kEwV; ++k) {
        const int64_t i = base + 2 * ((int64_t)k * kBlock + threadIdx.x);
        sv[k] = __builtin_nontemporal_load((gcu2)(src + i));
        if constexpr (MODE == 1) dv[k] = *(gcu2)(dst + i);
      }
#pragma unroll
      for (int k = 0; k < kEwV; ++k) {
        const int64_t i = base + 2 * ((int64_t)k * kBlock + threadIdx.x);
        const d2 x = decode2<BE_IN>(sv[k]);
        d2 o;
        if constexpr (MODE == 1) {
          const d2 a = __builtin_bit_cast(d2, dv[k]);
          o = d2{a.x + x.x, a.y + x.y};
        } else if constexpr (MODE == 2) {
          o = d2{0.0 + x.x, 0.0 + x.y};
        } else {
          o = x;
        }
        *(gu2)(dst + i) = encode2<BE_OUT>(o);
      }
      return;
    }
    const int64_t end = base + kEwTile < L ? base + kEwTile : L;
    for (int64_t i = base + threadIdx.x; i < end; i += kBlock) one(i);
  } else {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < L) one(i);
  }
}

// Layout conversion between native and big-endian doubles (pack / unpack).
//   VEC: the 16-B tile shape of the elementwise kernels (kEwTile elements per
//   block, see k_fold_n) when both operands are 16-B aligned
template <bool VEC = false>
__global__ __launch_bounds__(kBlock) void k_bswap64(const unsigned long long* __restrict__ in,
                                                    unsigned long long* __restrict__ out, int64_t n) {
  if constexpr (VEC) {
    const int64_t base = (int64_t)blockIdx.x * kEwTile;
    if (base + kEwTile <= n) {
      u2 v[kEwV];
#pragma unroll
      for (int k = 0; k < kEwV; ++k) v[k] = __builtin_nontemporal_load((gcu2)(in + base + 2 * ((int64_t)k * kBlock + threadIdx.x)));
#pragma unroll
      for (int k = 0; k < kEwV; ++k) {
        const unsigned long long a = v[k].x, b = v[k].y;
        __builtin_nontemporal_store(u2{__builtin_bswap64(a), __builtin_bswap64(b)},
                                    (gu2)(out + base + 2 * ((int64_t)k * kBlock + threadIdx.x)));
      }
      return;
    }
    for (int64_t i = base + threadIdx.x; i < n; i += kBlock) out[i] = __builtin_bswap64(in[i]);
  } else {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
      out[i] = __builtin_bswap64(in[i]);
  }
}

// Strided model load (InitializeWeights(List<Double>), IPLS.java:1880-1901):
// dst[j] = flat[lo + j] for j < ncopy, dst[L-1] = 0.0.
template <bool BE_IN>
__global__ __launch_bounds__(kBlock) void k_load_model(const unsigned long long* __restrict__ flat,
                                                       int64_t lo, int64_t ncopy, int64_t L,
                                                       double* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= L) return;
  dst[i] = (i < ncopy) ? decode1<BE_IN>(flat[lo + i]) : 0.0;
}

// ---------------------------------------------------------------------------
// Synthetic workload and checksum.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long v) {
  unsigned long long z = v + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

template <bool BE_OUT>
__global__ __launch_bounds__(kBlock) void k_synth(unsigned long long* __restrict__ dst, int64_t L,
                                                  unsigned long long key) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < L;
       i += (int64_t)gridDim.x * kBlock) {
    double x;
    if (i == L - 1) {
      x = 1.0;
    } else {
      const double u = (double)(splitmix64(key ^ (unsigned long long)i) >> 11) * 0x1.0p-53;
      double tt = 2.0 * u;
      tt = tt - 1.0;
      x = tt * 1e-2;
    }
    dst[i] = BE_OUT ? f64_to_be(x) : __builtin_bit_cast(unsigned long long, x);
  }
}

// 64-bit wave sum with DPP row shifts + row broadcasts (gfx9 DPP controls):
// inclusive scan inside each 16-lane row, then row_bcast:15 / row_bcast:31
// carry the row totals up; lane 63 ends with the wave total.  The sum is an
// exact integer (mod 2^64), so association does not matter here.
__device__ __forceinline__ unsigned long long dpp_shift(unsigned long long v, int ctrl_id) {
  const int lo = (int)(unsigned)v, hi = (int)(unsigned)(v >> 32);
  int rl, rh;
  switch (ctrl_id) {
    case 0: rl = __builtin_amdgcn_update_dpp(0, lo, 0x111, 0xF, 0xF, true);
            rh = __builtin_amdgcn_update_dpp(0, hi, 0x111, 0xF, 0xF, true); break;  // row_shr:1
    case 1: rl = __builtin_amdgcn_update_dpp(0, lo, 0x112, 0xF, 0xF, true);
            rh = __builtin_amdgcn_update_dpp(0, hi, 0x112, 0xF, 0xF, true); break;  // row_shr:2
    case 2: rl = __builtin_amdgcn_update_dpp(0, lo, 0x114, 0xF, 0xF, true);
            rh = __builtin_amdgcn_update_dpp(0, hi, 0x114, 0xF, 0xF, true); break;  // row_shr:4
    case 3: rl = __builtin_amdgcn_update_dpp(0, lo, 0x118, 0xF, 0xF, true);
            rh = __builtin_amdgcn_update_dpp(0, hi, 0x118, 0xF, 0xF, true); break;  // row_shr:8
    case 4: rl = __builtin_amdgcn_update_dpp(0, lo, 0x142, 0xA, 0xF, false);
            rh = __builtin_amdgcn_update_dpp(0, hi, 0x142, 0xA, 0xF, false); break; // row_bcast:15
    default: rl = __builtin_amdgcn_update_dpp(0, lo, 0x143, 0xC, 0xF, false);
             rh = __builtin_amdgcn_update_dpp(0, hi, 0x143, 0xC, 0xF, false); break; // row_bcast:31
  }
  return ((unsigned long long)(unsigned)rh << 32) | (unsigned)rl;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int c = 0; c < 6; ++c) v += dpp_shift(v, c);
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)v, 63);
  const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(v >> 32), 63);
  return ((unsigned long long)hi << 32) | lo;
}

template <bool BE_IN>
__global__ __launch_bounds__(kBlock) void k_checksum(const unsigned long long* __restrict__ x,
                                                     int64_t n, unsigned long long* __restrict__ out) {
  __shared__ unsigned long long lds[kBlock / 64];
  unsigned long long s = 0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    unsigned long long b = BE_IN ? __builtin_bswap64(x[i]) : x[i];
    s += splitmix64(b + (unsigned long long)i * 0x9E3779B97F4A7C15ULL);
  }
  s = wave_sum_u64(s);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) t += lds[w];
    atomicAdd(out, t);
  }
}

// ---------------------------------------------------------------------------
// k_b64url_decode: java.util.Base64 URL decoding of a batch of messages
// (ThreadReceiver.run / process, IPLS.java:855-859, 399; Utils.java:14-15).
// The host strips and validates the '=' tail; the kernel decodes every full
// 4-char unit (16 chars per lane: one dwordx4 load -> 12 bytes) plus the
// partial last unit, and flags any byte outside A-Z a-z 0-9 - _ (Java's
// IllegalArgumentException) in err[msg].  blockIdx.y = message.
// ---------------------------------------------------------------------------
struct B64Desc {
  int64_t src_off;  // byte offset of the text in src (16-B aligned)
  int64_t units;    // full 4-char units
  int64_t dst_off;  // byte offset of the decoded bytes in dst
  int32_t tail;     // data chars in the partial last unit: 0, 2 or 3
  int32_t pad;
};

__device__ __forceinline__ unsigned b64url_val(unsigned c) {
  // A-Z 0-25, a-z 26-51, 0-9 52-61, '-' 62, '_' 63, else 0x100 (invalid)
  if (c - 'A' < 26u) return c - 'A';
  if (c - 'a' < 26u) return c - 'a' + 26;
  if (c - '0' < 10u) return c - '0' + 52;
  if (c == '-') return 62;
  if (c == '_') return 63;
  return 0x100;
}

// 4 chars (little-endian packed in a dword) -> 24 bits; bit 24+ set if invalid.
__device__ __forceinline__ unsigned b64url_unit(unsigned w) {
  const unsigned a = b64url_val(w & 0xFF), b = b64url_val((w >> 8) & 0xFF);
  const unsigned c = b64url_val((w >> 16) & 0xFF), d = b64url_val(w >> 24);
  return (a << 18) | (b << 12) | (c << 6) | d | ((a | b | c | d) & 0x100 ? 0x1000000u : 0u);
}

__global__ __launch_bounds__(kBlock) void k_b64url_decode(const unsigned char* __restrict__ src,
                                                          const B64Desc* __restrict__ descs,
                                                          unsigned char* __restrict__ dst,
                                                          int* __restrict__ err) {
  const int m = blockIdx.y;
  const B64Desc d = descs[m];
  const unsigned char* s = src + d.src_off;
  unsigned char* o = dst + d.dst_off;
  const int64_t u0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4;   // first unit of this lane
  if (u0 > d.units) return;
  unsigned bad = 0;
  if (u0 + 4 <= d.units) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const u4 w = *(const IPLS_GLOBAL u4*)(s + 4 * u0);
    const unsigned v[4] = {b64url_unit(w.x), b64url_unit(w.y), b64url_unit(w.z), b64url_unit(w.w)};
    bad = (v[0] | v[1] | v[2] | v[3]) & 0x1000000u;
    unsigned char* q = o + 3 * u0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      q[3 * i] = (unsigned char)(v[i] >> 16);
      q[3 * i + 1] = (unsigned char)(v[i] >> 8);
      q[3 * i + 2] = (unsigned char)v[i];
    }
  } else {
    for (int64_t u = u0; u < d.units; ++u) {
      const unsigned char* c = s + 4 * u;
      const unsigned w = c[0] | (c[1] << 8) | (c[2] << 16) | ((unsigned)c[3] << 24);
      const unsigned v = b64url_unit(w);
      bad |= v & 0x1000000u;
      o[3 * u] = (unsigned char)(v >> 16);
      o[3 * u + 1] = (unsigned char)(v >> 8);
      o[3 * u + 2] = (unsigned char)v;
    }
    if (d.tail && u0 + 4 > d.units) {   // the lane that ends the full units does the tail
      const unsigned char* c = s + 4 * d.units;
      unsigned v = 0, inval = 0;
      for (int i = 0; i < d.tail; ++i) {
        const unsigned x = b64url_val(c[i]);
        inval |= x;
        v |= (x & 63u) << (18 - 6 * i);
      }
      bad |= inval & 0x100;
      o[3 * d.units] = (unsigned char)(v >> 16);
      if (d.tail == 3) o[3 * d.units + 1] = (unsigned char)(v >> 8);
    }
  }
  if (bad) atomicOr(err + m, 1);
}

// ---------------------------------------------------------------------------
// k_b64url_encode_frame: Marshall_Packet (MyIPFSClass.java:990-1017) of an
// accumulator, straight from HBM -- the frame
//   [i16 pid][i32 n][i32 a][i32 b][n x f64 big-endian][origin bytes]
// encoded by Base64.getUrlEncoder (with '=' padding, :1016).  Lane g writes
// the 32 chars of frame bytes [24g, 24g+24).  Lanes whose window lies inside
// the payload (all but the first and the last few) load the 4 doubles it
// spans (it starts 2 bytes into one: 24g - 14 = 8(3g-2) + 2), take the
// window's 6 big-endian words by funnel shifts and emit 8 units = 2 x 16 B;
// the others assemble their bytes one at a time.  src == null: the
// accumulator is logically +0.0 (all payload bytes zero).
// ---------------------------------------------------------------------------
struct FrameEnc {
  unsigned char hdr[16];          // 14 header bytes
  int64_t n;                      // doubles in the payload
  int64_t origin_len;
  const unsigned char* origin;    // device copy of the origin bytes
};

__device__ __forceinline__ unsigned b64url_char(unsigned v) {
  return v < 26 ? 'A' + v : v < 52 ? 'a' + (v - 26) : v < 62 ? '0' + (v - 52) : v == 62 ? '-' : '_';
}
// 24 bits -> 4 chars packed little-endian (first char in the low byte)
__device__ __forceinline__ unsigned b64url_quad(unsigned v) {
  return b64url_char((v >> 18) & 63) | (b64url_char((v >> 12) & 63) << 8) | (b64url_char((v >> 6) & 63) << 16) |
         (b64url_char(v & 63) << 24);
}

__device__ __forceinline__ unsigned frame_byte(const FrameEnc& f, const unsigned long long* __restrict__ src,
                                               int64_t j) {
  if (j < 14) return f.hdr[j];
  const int64_t q = j - 14;
  if (q < 8 * f.n) {
    if (!src) return 0;
    const unsigned long long v = ld8(src + (q >> 3));
    return (unsigned)(v >> (8 * (7 - (q & 7)))) & 0xFF;   // putDouble: big-endian
  }
  return f.origin[q - 8 * f.n];
}

// Interior chars come from a 64-byte LDS table, one ds_read_u8 per char: the
// branchy b64url_char mapping made the kernel VALU-bound (~400 integer ops
// per lane for 24 bytes; 30.4 us for a 4M-double partition against 15.8 us
// for a copy of the same bytes).  With the table: 18-20 us.  A 4-chars-per-
// dword SWAR map (v_perm offsets) and staging the wave's input window through
// LDS with coalesced 16-B loads were both slower (tools/publish_sweep.hip,
// profiles/r02/publish_sweep.txt).
__device__ __forceinline__ unsigned b64url_quad_lut(const unsigned char* tab, unsigned v) {
  return (unsigned)tab[(v >> 18) & 63] | ((unsigned)tab[(v >> 12) & 63] << 8) | ((unsigned)tab[(v >> 6) & 63] << 16) |
         ((unsigned)tab[v & 63] << 24);
}

// One text: blocks [0, gridDim.x) of this job walk its groups grid-stride.
// tab = the 64-char table in LDS, stage = 2 * kBlock 16-B rows of LDS.
__device__ __forceinline__ void encode_frame_job(const FrameEnc& f, const unsigned long long* __restrict__ src,
                                                 unsigned char* __restrict__ out, int64_t groups, int64_t text_len,
                                                 const unsigned char* tab, u4w* stage) {
  // Each lane's 32 chars go through a wave-private LDS row so that every wave
  // then stores its 2 KiB of text as two contiguous 1 KiB rows (lane-strided
  // 16-B stores would leave every 128-B line half written per instruction).
  // LDS ops of one wave complete in order: a compiler barrier suffices.
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u4w* ws = stage + 128 * wv;
  const int64_t F = 14 + 8 * f.n + f.origin_len;   // frame bytes
  for (int64_t g0 = (int64_t)blockIdx.x * kBlock; g0 < groups; g0 += (int64_t)gridDim.x * kBlock) {
    const int64_t gw = g0 + 64 * wv;                // this wave's first group
    const int64_t g = gw + lane;
    const int64_t b0 = 24 * g;
    u4w c0 = {0u, 0u, 0u, 0u}, c1 = {0u, 0u, 0u, 0u};
    if (g < groups && g >= 1 && b0 + 24 <= 14 + 8 * f.n && src) {
      const unsigned long long* s = src + (3 * g - 2);
      const unsigned long long v0 = ld8(s), v1 = ld8(s + 1), v2 = ld8(s + 2), v3 = ld8(s + 3);
      // big-endian words of the 32 payload bytes, then the window's 6 (2 bytes in)
      const unsigned W[8] = {(unsigned)(v0 >> 32), (unsigned)v0, (unsigned)(v1 >> 32), (unsigned)v1,
                             (unsigned)(v2 >> 32), (unsigned)v2, (unsigned)(v3 >> 32), (unsigned)v3};
      unsigned O[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) O[k] = (W[k] << 16) | (W[k + 1] >> 16);
      const unsigned long long X0 = ((unsigned long long)O[0] << 32) | O[1];
      const unsigned long long X1 = ((unsigned long long)O[2] << 32) | O[3];
      const unsigned long long X2 = ((unsigned long long)O[4] << 32) | O[5];
      c0.x = b64url_quad_lut(tab, (unsigned)(X0 >> 40) & 0xFFFFFF);
      c0.y = b64url_quad_lut(tab, (unsigned)(X0 >> 16) & 0xFFFFFF);
      c0.z = b64url_quad_lut(tab, (unsigned)((X0 << 8) | (X1 >> 56)) & 0xFFFFFF);
      c0.w = b64url_quad_lut(tab, (unsigned)(X1 >> 32) & 0xFFFFFF);
      c1.x = b64url_quad_lut(tab, (unsigned)(X1 >> 8) & 0xFFFFFF);
      c1.y = b64url_quad_lut(tab, (unsigned)((X1 << 16) | (X2 >> 48)) & 0xFFFFFF);
      c1.z = b64url_quad_lut(tab, (unsigned)(X2 >> 24) & 0xFFFFFF);
      c1.w = b64url_quad_lut(tab, (unsigned)X2 & 0xFFFFFF);
    } else if (g < groups) {
      // header / tail lanes: byte by byte, '=' padding on the last unit
      unsigned q8[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
      for (int u = 0; u < 8; ++u) {
        const int64_t j = b0 + 3 * u;
        if (j >= F) break;
        const int nb = F - j >= 3 ? 3 : (int)(F - j);
        unsigned v = frame_byte(f, src, j) << 16;
        if (nb > 1) v |= frame_byte(f, src, j + 1) << 8;
        if (nb > 2) v |= frame_byte(f, src, j + 2);
        unsigned q = b64url_quad(v);
        if (nb < 3) q = (q & 0x00FFFFFFu) | ((unsigned)'=' << 24);
        if (nb < 2) q = (q & 0xFF00FFFFu) | ((unsigned)'=' << 16);
        q8[u] = q;
      }
      c0 = u4w{q8[0], q8[1], q8[2], q8[3]};
      c1 = u4w{q8[4], q8[5], q8[6], q8[7]};
    }
    ws[2 * lane] = c0;
    ws[2 * lane + 1] = c1;
    __builtin_amdgcn_wave_barrier();
    const int64_t wbase = 32 * gw;                  // this wave's 2 KiB of text
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const u4w v = ws[64 * h + lane];
      const int64_t o = wbase + 1024 * h + 16 * lane;
      if (o + 16 <= text_len) {
        __builtin_nontemporal_store(v, (IPLS_GLOBAL u4w*)(out + o));
      } else if (o < text_len) {   // the text's last partial 16 B
        const unsigned w4[4] = {v.x, v.y, v.z, v.w};
        for (int64_t c = 0; o + c < text_len; ++c) out[o + c] = (unsigned char)(w4[c >> 2] >> (8 * (c & 3)));
      }
    }
    __builtin_amdgcn_wave_barrier();   // the row is rewritten by the next iteration
  }
}

__device__ __forceinline__ void init_b64url_table(unsigned char* tab) {
  if (threadIdx.x < 64) tab[threadIdx.x] = (unsigned char)b64url_char(threadIdx.x);
  __syncthreads();
}

__global__ __launch_bounds__(kBlock) void k_b64url_encode_frame(FrameEnc f, const unsigned long long* __restrict__ src,
                                                               unsigned char* __restrict__ out, int64_t groups,
                                                               int64_t text_len) {
  __shared__ u4w stage[2 * kBlock];
  __shared__ unsigned char tab[64];
  init_b64url_table(tab);
  encode_frame_job(f, src, out, groups, text_len, tab, stage);
}

// Several partitions' texts in one launch (the publish loop over Auth_List,
// IPLS.java:1423-1431): blockIdx.y = job.  Every text starts 16-B aligned.
struct FrameJob {
  FrameEnc f;
  const unsigned long long* src;   // accumulator, or null = logically +0.0
  unsigned char* out;
  int64_t groups;
  int64_t text_len;
};

__global__ __launch_bounds__(kBlock) void k_b64url_encode_frames(const FrameJob* __restrict__ jobs) {
  __shared__ u4w stage[2 * kBlock];
  __shared__ unsigned char tab[64];
  init_b64url_table(tab);
  const FrameJob& j = jobs[blockIdx.y];
  encode_frame_job(j.f, j.src, j.out, j.groups, j.text_len, tab, stage);
}

// ---------------------------------------------------------------------------
// Variants, each product rounded, then the sum rounded
// (Java evaluates a*W + b*g left to right, no FMA; -ffp-contract=off here):
//   k_blend : t[i] = a*t[i] + b*g[i]
//             async replica fold  a=0.75, b=1      (Updater.java:57-59)
//             leaving-peer blend  a=0.6,  b=1-0.6  (Updater.java:65-69)
//   k_scale : d[i] = c*s[i]        async publish 0.25*W (Updater.java:197-199)
//   k_encode_secure : Middleware.Encode (Middleware.java:196-210):
//             x > 10 -> 10*1e12, x < -10 -> -10*1e12, else x*1e12
// ---------------------------------------------------------------------------
//   VEC: the tile shape of kEwV 16-B vectors per lane (see k_fold_n).
template <bool BE_IN, bool VEC = false>
__global__ __launch_bounds__(kBlock) void k_blend(double* __restrict__ t, const unsigned long long* __restrict__ g,
                                                  int64_t L, double a, double b) {
  auto one = [&](int64_t i) {
    const double x = decode1<BE_IN>(ld8(g + i));
    const double aw = a * t[i];
    const double bg = b * x;
    t[i] = aw + bg;
  };
  if constexpr (VEC) {
    const int64_t base = (int64_t)blockIdx.x * kEwTile;
    if (base + kEwTile <= L) {
      u2 gv[kEwV], tv[kEwV];
#pragma unroll
      for (int v = 0; v < kEwV; ++v) {
        const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
        gv[v] = __builtin_nontemporal_load((gcu2)(g + i));
        tv[v] = *(gcu2)(t + i);
      }
#pragma unroll
      for (int v = 0; v < kEwV; ++v) {
        const int64_t i = base + 2 * ((int64_t)v * kBlock + threadIdx.x);
        const d2 x = decode2<BE_IN>(gv[v]);
        const d2 w = __builtin_bit_cast(d2, tv[v]);
        const double awx = a * w.x, bgx = b * x.x, awy = a * w.y, bgy = b * x.y;
        *(gu2)(t + i) = __builtin_bit_cast(u2, d2{awx + bgx, awy + bgy});
      }
      return;
    }
    for (int64_t i = base + threadIdx.x; i < L; i += kBlock) one(i);
  } else {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < L; i += (int64_t)gridDim.x * kBlock) one(i);
  }
}

template <bool VEC = false>
__global__ __launch_bounds__(kBlock) void k_scale(double* __restrict__ d, const double* __restrict__ s, int64_t L,
                                                  double c) {
  if constexpr (VEC) {
    const int64_t base = (int64_t)blockIdx.x * kEwTile;
    if (base + kEwTile <= L) {
      u2 sv[kEwV];
#pragma unroll
      for (int v = 0; v < kEwV; ++v)
        sv[v] = __builtin_nontemporal_load((gcu2)(s + base + 2 * ((int64_t)v * kBlock + threadIdx.x)));
#pragma unroll
      for (int v = 0; v < kEwV; ++v) {
        const d2 x = __builtin_bit_cast(d2, sv[v]);
        __builtin_nontemporal_store(__builtin_bit_cast(u2, d2{c * x.x, c * x.y}),
                                    (gu2)(d + base + 2 * ((int64_t)v * kBlock + threadIdx.x)));
      }
      return;
    }
    for (int64_t i = base + threadIdx.x; i < L; i += kBlock) d[i] = c * s[i];
  } else {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < L; i += (int64_t)gridDim.x * kBlock)
      d[i] = c * s[i];
  }
}

__device__ __forceinline__ double encode_secure1(double x) {
  if (x > 10.0) return 10 * 1e12;
  if (x < -10.0) return -10 * 1e12;
  return x * 1e12;
}

template <bool BE_IN, bool BE_OUT, bool VEC = false>
__global__ __launch_bounds__(kBlock) void k_encode_secure(const unsigned long long* __restrict__ src,
                                                          unsigned long long* __restrict__ dst, int64_t n) {
  auto one = [&](int64_t i) {
    const double y = encode_secure1(decode1<BE_IN>(ld8(src + i)));
    st8(dst + i, BE_OUT ? f64_to_be(y) : __builtin_bit_cast(unsigned long long, y));
  };
  if constexpr (VEC) {
    const int64_t base = (int64_t)blockIdx.x * kEwTile;
    if (base + kEwTile <= n) {
      u2 sv[kEwV];
#pragma unroll
      for (int v = 0; v < kEwV; ++v)
        sv[v] = __builtin_nontemporal_load((gcu2)(src + base + 2 * ((int64_t)v * kBlock + threadIdx.x)));
#pragma unroll
      for (int v = 0; v < kEwV; ++v) {
        const d2 x = decode2<BE_IN>(sv[v]);
        __builtin_nontemporal_store(encode2<BE_OUT>(d2{encode_secure1(x.x), encode_secure1(x.y)}),
                                    (gu2)(dst + base + 2 * ((int64_t)v * kBlock + threadIdx.x)));
      }
      return;
    }
    for (int64_t i = base + threadIdx.x; i < n; i += kBlock) one(i);
  } else {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) one(i);
  }
}

}  // namespace ipls
