// pubsub_host.hpp -- host side of the pubsub codec: the checks of a pubsub
// text that need only its ends (java.util.Base64 URL '=' rules of both
// layers, the 14-byte GET_GRADIENTS header), done before the text goes to
// the device.  Host C++ with no HIP in it, so it builds and is fuzzed under
// AddressSanitizer/UBSan on the CPU (tests/cpp/fuzz_pubsub.cpp).
//
// Reference: ThreadReceiver.run / process (IPLS.java:851-866, 399-465),
// Utils.getRawMessage (Utils.java:8-17), GET_GRADIENTS (MyIPFSClass.java:
// 1437-1459), Marshall_Packet (MyIPFSClass.java:990-1017).
#pragma once

#include <stdint.h>

namespace ipls {
namespace pubsub {

// Data chars of an n-char java.util.Base64 URL text whose last k >= min(n, 3)
// chars are `tail` (the '=' rules Decoder.decode0 enforces), or -1 where Java
// throws IllegalArgumentException.  The rules hang on the data-char count of
// the WHOLE text, not of the window.
int64_t b64_data_chars(const uint8_t* tail, int64_t k, int64_t n);

// Decoded length of a text with d data chars (d % 4 != 1).
int64_t b64_out_len(int64_t d);

// Decoded bytes [lo, hi) (hi <= b64_out_len(d)) of a text with d data chars,
// as Decoder.decode0 produces them; false if a char of the 4-char units
// touched is outside A-Z a-z 0-9 - _.
bool b64_host_bytes(const uint8_t* t, int64_t d, int64_t lo, int64_t hi, uint8_t* out);

// Base64url-encoded length (with '=' padding, Base64.getUrlEncoder) of n bytes.
int64_t b64_enc_len(int64_t n);

// What the host learns from a text's ends.
struct Pre {
  int32_t status;     // IPLS_E_FORMAT: rejected on the host; 0: decode it on the device
  int64_t dc;         // data chars of the outer text
  int64_t dc2;        // data chars of the inner text (== dc for one layer)
  int64_t frame_len;  // bytes of the frame the text decodes to
  int16_t pid;        // frame header [i16 pid][i32 n][i32 a][i32 b]
  int32_t n;          // doubles in the frame (0: null gradient)
  int32_t a;          // partition field (Marshall_Packet's `Partition`)
  int32_t b;          // iteration field
};

// Host pre-pass of one pubsub text with `layers` (1 or 2) rounds of base64url
// around a GET_GRADIENTS frame: the '=' endings of both layers, the frame
// header and the declared length against the real frame length.  A text that
// passes may still hold a char outside the alphabet in its middle; the device
// decode flags that (status IPLS_E_FORMAT then).
Pre precheck(const uint8_t* msg, int64_t len, int layers);

}  // namespace pubsub
}  // namespace ipls
