// pubsub_host.cpp -- see pubsub_host.hpp.
#include "pubsub_host.hpp"

#include <algorithm>

#include "../../include/ipls_agg.h"

namespace ipls {
namespace pubsub {

namespace {
uint32_t rd_be32(const uint8_t* b) {
  return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}
}  // namespace

int64_t b64_data_chars(const uint8_t* tail, int64_t k, int64_t n) {
  int64_t pad = 0;
  while (pad < k && pad < 3 && tail[k - 1 - pad] == '=') ++pad;
  const int64_t d = n - pad;
  const int64_t r = d % 4;
  if (r == 1) return -1;                       // dangling single char
  if (pad == 0) return d;
  if (pad == 1 && r == 3) return d;            // "xxx="
  if (pad == 2 && r == 2) return d;            // "xx=="
  return -1;                                   // "=" / "x=" / "xx=" / "===" ...
}

int64_t b64_out_len(int64_t d) { return 3 * (d / 4) + (d % 4 == 2 ? 1 : d % 4 == 3 ? 2 : 0); }

int64_t b64_enc_len(int64_t n) { return 4 * ((n + 2) / 3); }

bool b64_host_bytes(const uint8_t* t, int64_t d, int64_t lo, int64_t hi, uint8_t* out) {
  bool ok = true;
  for (int64_t u = lo / 3; 3 * u < hi; ++u) {
    unsigned v = 0;
    for (int c = 0; c < 4; ++c) {
      const int64_t i = 4 * u + c;
      if (i >= d) break;
      const unsigned ch = t[i];
      unsigned x = ch - 'A' < 26u ? ch - 'A' : ch - 'a' < 26u ? ch - 'a' + 26 : ch - '0' < 10u ? ch - '0' + 52
                 : ch == '-' ? 62u : ch == '_' ? 63u : 0x100u;
      if (x > 63) ok = false;
      v |= (x & 63u) << (18 - 6 * c);
    }
    for (int b = 0; b < 3; ++b) {
      const int64_t j = 3 * u + b;
      if (j >= lo && j < hi) out[j - lo] = (uint8_t)(v >> (16 - 8 * b));
    }
  }
  return ok;
}

Pre precheck(const uint8_t* msg, int64_t len, int layers) {
  Pre r{};
  r.status = IPLS_E_FORMAT;
  if (len < 0 || (len > 0 && !msg) || layers < 1 || layers > 2) return r;
  const int64_t d = b64_data_chars(msg, len, len);
  if (d < 0) return r;
  r.dc = d;
  bool ok = true;
  uint8_t hdr[14];
  if (layers == 2) {
    // the inner text's '=' rules need its last chars: decode the outer text's last bytes
    const int64_t n = b64_out_len(d), k = std::min<int64_t>(4, n);
    uint8_t tail[4];
    ok = b64_host_bytes(msg, d, n - k, n, tail);
    const int64_t t = ok ? b64_data_chars(tail, k, n) : -1;
    if (t < 0) return r;
    r.dc2 = t;
    r.frame_len = b64_out_len(t);
    if (r.frame_len >= 14) {
      uint8_t mid[20];
      const int64_t c = std::min<int64_t>(t, 20);   // 20 inner chars -> frame bytes 0..14
      ok = b64_host_bytes(msg, d, 0, c, mid) && b64_host_bytes(mid, c, 0, 14, hdr);
    }
  } else {
    r.dc2 = d;
    r.frame_len = b64_out_len(d);
    if (r.frame_len >= 14) ok = b64_host_bytes(msg, d, 0, 14, hdr);
  }
  if (!ok || r.frame_len < 14) return r;
  // [i16 pid][i32 n][i32 partition][i32 iteration]: n against the real frame length
  // (MyIPFSClass.java:1437-1446: getInt past the end -> BufferUnderflowException)
  const int32_t n = (int32_t)rd_be32(&hdr[2]);
  if (n < 0 || 14 + 8 * (int64_t)n > r.frame_len) return r;
  r.pid = (int16_t)(((uint16_t)hdr[0] << 8) | hdr[1]);
  r.n = n;
  r.a = (int32_t)rd_be32(&hdr[6]);
  r.b = (int32_t)rd_be32(&hdr[10]);
  r.status = 0;
  return r;
}

}  // namespace pubsub
}  // namespace ipls
