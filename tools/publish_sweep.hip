// publish_sweep.hip -- dev tool: variants of the publish-side encoder
// (Marshall_Packet + Base64.getUrlEncoder, MyIPFSClass.java:990-1016, a9),
// timed interleaved in one process against the shipped k_b64url_encode_frame,
// every variant's text checked byte-identical to the shipped one.
//
// Variants:
//   shipped   : ipls::k_b64url_encode_frame (4 strided 8-B loads per lane,
//               branchy per-char mapping, output staged through LDS)
//   lut       : wave loads its 1.5 KiB payload window coalesced (16 B per
//               lane) into LDS; each lane reads its 24-B window back; chars
//               come from a 64-byte LDS table (one ds_read_u8 per char)
//   swar      : same input staging; chars by a 4-chars-per-dword SWAR map
//               (class = #thresholds passed, v_perm picks the offset)
//   lut_direct: the shipped strided loads + the LDS table
//   copy      : read 8n bytes, write the text length (a traffic ceiling)
//
// Usage: publish_sweep N REPS   (N doubles in the partition)
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

// 24 bits -> 4 chars (first char in the low byte), SWAR over the 4 bytes.
__device__ __forceinline__ unsigned quad_swar(unsigned v) {
  const unsigned t = (v >> 18) | ((v >> 4) & 0x3F00u) | ((v << 10) & 0x3F0000u) | ((v << 24) & 0x3F000000u);
  const unsigned M = 0x80808080u;
  // per byte: bit 7 of t + (128 - thr) is (t >= thr); t < 64 so no carries
  const unsigned a = ((t + 0x66666666u) & M) >> 7;   // >= 26
  const unsigned b = ((t + 0x4C4C4C4Cu) & M) >> 7;   // >= 52
  const unsigned c = ((t + 0x42424242u) & M) >> 7;   // >= 62
  const unsigned d = ((t + 0x41414141u) & M) >> 7;   // >= 63
  // offsets by class 0..4: 'A', 'a'-26, '0'-52, '-'-62, '_'-63 (mod 256)
  const unsigned off = __builtin_amdgcn_perm(0x00000020u, 0xEFFC4741u, a + b + c + d);
  return (t + (off & 0x7F7F7F7Fu)) ^ (off & M);   // bytewise add, no carries
}

__device__ __forceinline__ unsigned quad_lut(const unsigned char* tab, unsigned v) {
  return (unsigned)tab[(v >> 18) & 63] | ((unsigned)tab[(v >> 12) & 63] << 8) | ((unsigned)tab[(v >> 6) & 63] << 16) |
         ((unsigned)tab[v & 63] << 24);
}

// The 24 frame bytes of an interior group as 8 quads from its 4 doubles
// (window starts 2 bytes into the first, see k_b64url_encode_frame).
template <int MAP>
__device__ __forceinline__ void encode24(const unsigned long long v0, const unsigned long long v1,
                                         const unsigned long long v2, const unsigned long long v3,
                                         const unsigned char* tab, u4w& c0, u4w& c1) {
  const unsigned W[8] = {(unsigned)(v0 >> 32), (unsigned)v0, (unsigned)(v1 >> 32), (unsigned)v1,
                         (unsigned)(v2 >> 32), (unsigned)v2, (unsigned)(v3 >> 32), (unsigned)v3};
  unsigned O[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) O[k] = (W[k] << 16) | (W[k + 1] >> 16);
  const unsigned long long X0 = ((unsigned long long)O[0] << 32) | O[1];
  const unsigned long long X1 = ((unsigned long long)O[2] << 32) | O[3];
  const unsigned long long X2 = ((unsigned long long)O[4] << 32) | O[5];
  const unsigned u[8] = {(unsigned)(X0 >> 40) & 0xFFFFFF,
                         (unsigned)(X0 >> 16) & 0xFFFFFF,
                         (unsigned)((X0 << 8) | (X1 >> 56)) & 0xFFFFFF,
                         (unsigned)(X1 >> 32) & 0xFFFFFF,
                         (unsigned)(X1 >> 8) & 0xFFFFFF,
                         (unsigned)((X1 << 16) | (X2 >> 48)) & 0xFFFFFF,
                         (unsigned)(X2 >> 24) & 0xFFFFFF,
                         (unsigned)X2 & 0xFFFFFF};
  unsigned q[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = MAP == 0 ? quad_lut(tab, u[i]) : quad_swar(u[i]);
  c0 = u4w{q[0], q[1], q[2], q[3]};
  c1 = u4w{q[4], q[5], q[6], q[7]};
}

// header / tail lanes: byte by byte, '=' padding (as shipped)
__device__ void edge_group(const FrameEnc& f, const unsigned long long* src, int64_t g, int64_t F, u4w& c0, u4w& c1) {
  unsigned q8[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  const int64_t b0 = 24 * g;
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

__device__ __forceinline__ void store_rows(const u4w* ws, int lane, int64_t wbase, unsigned char* out,
                                           int64_t text_len) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const u4w v = ws[64 * h + lane];
    const int64_t o = wbase + 1024 * h + 16 * lane;
    if (o + 16 <= text_len) {
      __builtin_nontemporal_store(v, (IPLS_GLOBAL u4w*)(out + o));
    } else if (o < text_len) {
      const unsigned w4[4] = {v.x, v.y, v.z, v.w};
      for (int64_t c = 0; o + c < text_len; ++c) out[o + c] = (unsigned char)(w4[c >> 2] >> (8 * (c & 3)));
    }
  }
}

__device__ __forceinline__ void init_tab(unsigned char* tab) {
  if (threadIdx.x < 64) tab[threadIdx.x] = (unsigned char)b64url_char(threadIdx.x);
  __syncthreads();
}

// STAGE: 1 = the wave's payload window staged through LDS (coalesced 16-B
// loads), 0 = the shipped 4 strided 8-B loads per lane.  MAP: 0 LUT, 1 SWAR.
template <int STAGE, int MAP>
__global__ __launch_bounds__(kBlock) void k_enc_var(FrameEnc f, const unsigned long long* __restrict__ src,
                                                    unsigned char* __restrict__ out, int64_t groups,
                                                    int64_t text_len) {
  __shared__ u4w ostage[2 * kBlock];
  __shared__ unsigned long long istage[4][200];
  __shared__ unsigned char tab[64];
  if (MAP == 0) init_tab(tab);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u4w* ws = ostage + 128 * wv;
  unsigned long long* is = istage[wv];
  const int64_t F = 14 + 8 * f.n + f.origin_len;
  const int64_t pay_end = 14 + 8 * f.n;
  for (int64_t b0g = (int64_t)blockIdx.x * kBlock; b0g < groups; b0g += (int64_t)gridDim.x * kBlock) {
    const int64_t gw = b0g + 64 * wv;          // this wave's first group
    const int64_t g = gw + lane;
    u4w c0 = {0u, 0u, 0u, 0u}, c1 = {0u, 0u, 0u, 0u};
    const bool wave_inner = src && gw >= 1 && 24 * (gw + 64) <= pay_end;
    if (STAGE && wave_inner) {
      // doubles [3gw-2, 3gw+191) -> LDS (3gw-2 is even: 16-B aligned)
      const int64_t d0 = 3 * gw - 2;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int vi = lane + 64 * r;
        if (vi < 97) {
          const int64_t e = d0 + 2 * vi;
          if (e + 1 < f.n) {
            const u2 x = ld16<true>(src + e);
            is[2 * vi] = x.x;
            is[2 * vi + 1] = x.y;
          } else if (e < f.n) {
            is[2 * vi] = ld8(src + e);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      const unsigned long long* s = is + 3 * lane;
      encode24<MAP>(s[0], s[1], s[2], s[3], tab, c0, c1);
    } else if (g < groups && g >= 1 && 24 * g + 24 <= pay_end && src) {
      const unsigned long long* s = src + (3 * g - 2);
      encode24<MAP>(ld8(s), ld8(s + 1), ld8(s + 2), ld8(s + 3), tab, c0, c1);
    } else if (g < groups) {
      edge_group(f, src, g, F, c0, c1);
    }
    ws[2 * lane] = c0;
    ws[2 * lane + 1] = c1;
    __builtin_amdgcn_wave_barrier();
    store_rows(ws, lane, 32 * gw, out, text_len);
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ void k_copy(const unsigned long long* __restrict__ src, int64_t n, unsigned char* __restrict__ out,
                       int64_t text_len) {
  const int64_t nv = n / 2, tv = text_len / 16;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < std::max(nv, tv);
       i += (int64_t)gridDim.x * blockDim.x) {
    u2 x = {0, 0};
    if (i < nv) x = ld16<true>(src + 2 * i);
    if (i < tv) {
      u4w y = {(unsigned)x.x, (unsigned)(x.x >> 32), (unsigned)x.y, (unsigned)(x.y >> 32)};
      __builtin_nontemporal_store(y, (IPLS_GLOBAL u4w*)(out + 16 * i));
    }
  }
}

static unsigned host_char(unsigned v) {
  return v < 26 ? 'A' + v : v < 52 ? 'a' + (v - 26) : v < 62 ? '0' + (v - 52) : v == 62 ? '-' : '_';
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 4194304;
  const int REPS = argc > 2 ? atoi(argv[2]) : 50;
  const char* origin = "QmPeerOriginId12345";
  const int64_t olen = (int64_t)strlen(origin);
  const int64_t F = 14 + 8 * n + olen;
  const int64_t T = (F + 2) / 3 * 4;
  const int64_t groups = (F + 23) / 24;

  unsigned long long* src;
  CK(hipMalloc(&src, n * 8 + 256));
  hipLaunchKernelGGL(k_synth<false>, dim3(4096), dim3(kBlock), 0, 0, src, n, 0x1B52026ULL);
  unsigned char* dorig;
  CK(hipMalloc(&dorig, 64));
  CK(hipMemcpy(dorig, origin, olen, hipMemcpyHostToDevice));
  FrameEnc fe{};
  const uint32_t hv[3] = {(uint32_t)n, 7u, 33u};
  fe.hdr[0] = 0;
  fe.hdr[1] = 3;
  for (int k = 0; k < 3; ++k)
    for (int i = 0; i < 4; ++i) fe.hdr[2 + 4 * k + i] = (unsigned char)(hv[k] >> (24 - 8 * i));
  fe.n = n;
  fe.origin_len = olen;
  fe.origin = dorig;

  struct Var {
    std::string name;
    std::function<void(unsigned char*)> run;
    std::vector<float> ms;
    unsigned char* out;
  };
  const unsigned blocks = std::max<int64_t>(1, std::min<int64_t>((groups + kBlock - 1) / kBlock, 8192));
  std::vector<Var> vars;
  vars.push_back({"shipped", [&](unsigned char* o) {
                    hipLaunchKernelGGL(k_b64url_encode_frame, dim3(blocks), dim3(kBlock), 0, 0, fe, src, o, groups, T);
                  }});
  vars.push_back({"lut (LDS-staged input)", [&](unsigned char* o) {
                    hipLaunchKernelGGL((k_enc_var<1, 0>), dim3(blocks), dim3(kBlock), 0, 0, fe, src, o, groups, T);
                  }});
  vars.push_back({"swar (LDS-staged input)", [&](unsigned char* o) {
                    hipLaunchKernelGGL((k_enc_var<1, 1>), dim3(blocks), dim3(kBlock), 0, 0, fe, src, o, groups, T);
                  }});
  vars.push_back({"lut, strided input", [&](unsigned char* o) {
                    hipLaunchKernelGGL((k_enc_var<0, 0>), dim3(blocks), dim3(kBlock), 0, 0, fe, src, o, groups, T);
                  }});
  vars.push_back({"swar, strided input", [&](unsigned char* o) {
                    hipLaunchKernelGGL((k_enc_var<0, 1>), dim3(blocks), dim3(kBlock), 0, 0, fe, src, o, groups, T);
                  }});
  const unsigned all_blocks = (unsigned)std::max<int64_t>(1, (groups + kBlock - 1) / kBlock);
  for (unsigned gb : {4096u, 16384u, 1u << 30})
    vars.push_back({"lut (LDS-staged), grid " + std::to_string(std::min(gb, all_blocks)), [&, gb](unsigned char* o) {
                      hipLaunchKernelGGL((k_enc_var<1, 0>), dim3(std::min(gb, all_blocks)), dim3(kBlock), 0, 0, fe, src,
                                         o, groups, T);
                    }});
  for (unsigned gb : {4096u, 16384u, 1u << 30})
    vars.push_back({"lut strided, grid " + std::to_string(std::min(gb, all_blocks)), [&, gb](unsigned char* o) {
                      hipLaunchKernelGGL((k_enc_var<0, 0>), dim3(std::min(gb, all_blocks)), dim3(kBlock), 0, 0, fe, src,
                                         o, groups, T);
                    }});
  const bool with_copy = true;
  for (auto& v : vars) CK(hipMalloc(&v.out, T + 64));

  // correctness: all variants equal the shipped text; shipped == host encoder
  for (auto& v : vars) v.run(v.out);
  CK(hipDeviceSynchronize());
  std::vector<unsigned char> ref(T), got(T);
  CK(hipMemcpy(ref.data(), vars[0].out, T, hipMemcpyDeviceToHost));
  {
    std::vector<unsigned long long> h(n);
    CK(hipMemcpy(h.data(), src, n * 8, hipMemcpyDeviceToHost));
    std::vector<unsigned char> fr(F);
    memcpy(fr.data(), fe.hdr, 14);
    for (int64_t i = 0; i < n; ++i)
      for (int b = 0; b < 8; ++b) fr[14 + 8 * i + b] = (unsigned char)(h[i] >> (56 - 8 * b));
    memcpy(fr.data() + 14 + 8 * n, origin, olen);
    int64_t bad = 0;
    for (int64_t j = 0, o = 0; j < F; j += 3, o += 4) {
      const int nb = (int)std::min<int64_t>(3, F - j);
      unsigned v = fr[j] << 16 | (nb > 1 ? fr[j + 1] << 8 : 0) | (nb > 2 ? fr[j + 2] : 0);
      char c[4] = {(char)host_char((v >> 18) & 63), (char)host_char((v >> 12) & 63),
                   nb > 1 ? (char)host_char((v >> 6) & 63) : '=', nb > 2 ? (char)host_char(v & 63) : '='};
      for (int i = 0; i < 4; ++i) bad += ref[o + i] != (unsigned char)c[i];
    }
    printf("# shipped vs host encoder: %lld mismatching chars\n", (long long)bad);
  }
  for (size_t i = 1; i < vars.size(); ++i) {
    CK(hipMemcpy(got.data(), vars[i].out, T, hipMemcpyDeviceToHost));
    printf("# %-32s %s\n", vars[i].name.c_str(), memcmp(got.data(), ref.data(), T) ? "MISMATCH" : "identical");
  }
  if (with_copy)
    vars.push_back({"copy (8n read, T written)", [&](unsigned char* o) {
                      hipLaunchKernelGGL(k_copy, dim3(4096), dim3(kBlock), 0, 0, src, n, o, T);
                    }});
  CK(hipMalloc(&vars.back().out, T + 64));

  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < REPS; ++r)
    for (auto& v : vars) {
      CK(hipEventRecord(a, 0));
      v.run(v.out);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r > 2) v.ms.push_back(ms);
    }
  const double bytes = 8.0 * n + (double)T;
  printf("# n=%lld doubles, text %lld B, algorithmic bytes %.0f (8n read + text written), REPS=%d\n", (long long)n,
         (long long)T, bytes, REPS);
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    printf("%-34s median %8.2f us  min %8.2f us  %6.1f GB/s  %5.1f%% of 8 TB/s\n", v.name.c_str(), med * 1e3,
           v.ms[0] * 1e3, bytes / (med * 1e-3) / 1e9, 100.0 * bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
