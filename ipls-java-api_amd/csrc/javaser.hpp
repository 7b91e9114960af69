// javaser.hpp -- Java Object Serialization (ObjectOutputStream protocol 2)
// for the IPLS partial-update object, org.javatuples.Pair<Integer, double[]>
// (MyIPFSClass.Update_file(String, Pair), MyIPFSClass.java:160-166;
// Download_Partial_Updates, :326-338).  Host code inside libipls_agg.so.
#pragma once
#include <cstdint>

namespace ipls {
namespace javaser {

// Layout of the stream for n doubles: [header][8n BE payload][trailer].
int64_t pair_header_len();
int64_t pair_trailer_len();
// Write the header (ends with the double[] length) / trailer; `out` holds
// pair_header_len() / pair_trailer_len() bytes.
void write_pair_header(uint8_t* out, int32_t workers, int32_t n);
void write_pair_trailer(uint8_t* out);

// Parse a Pair<Integer,double[]> stream.  Returns the number of doubles and
// sets *workers and *payload_off (byte offset of the first BE double), or -1
// for a malformed stream / other types.  Bounded by `n`; never reads past it.
int64_t parse_pair(const uint8_t* buf, int64_t n, int32_t* workers, int64_t* payload_off, const char** why);

}  // namespace javaser
}  // namespace ipls
