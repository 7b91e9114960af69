// fuzz_javaser.cpp -- the partial-update parser (ipls-java-api_amd/csrc/
// javaser.cpp) under AddressSanitizer + UBSan on the host: every prefix of a
// valid stream, random byte mutations of it and of the reference's own
// Scheduler stream, and random bytes behind a valid magic.  Built and run by
// tests/test_host_cpp.py (g++ -fsanitize=address,undefined).
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "javaser.hpp"

using namespace ipls::javaser;

int main(int argc, char** argv) {
  std::vector<uint8_t> sched;
  if (argc > 1) {
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    int c;
    while ((c = std::fgetc(f)) != EOF) sched.push_back(uint8_t(c));
    std::fclose(f);
  }
  const int32_t n = 37;
  std::vector<uint8_t> good(pair_header_len() + 8 * n + pair_trailer_len());
  write_pair_header(good.data(), 9, n);
  for (int i = 0; i < 8 * n; ++i) good[pair_header_len() + i] = uint8_t(i * 13);
  write_pair_trailer(good.data() + pair_header_len() + 8 * n);
  int32_t w = 0;
  int64_t off = 0;
  const char* why = nullptr;
  if (parse_pair(good.data(), (int64_t)good.size(), &w, &off, &why) != n || w != 9 || off != pair_header_len()) {
    std::printf("FAIL valid stream: %s\n", why ? why : "?");
    return 1;
  }
  long accepted = 0, rejected = 0;
  for (size_t cut = 0; cut < good.size(); ++cut) {   // every truncation: heap copy of exactly cut bytes
    std::vector<uint8_t> b(good.begin(), good.begin() + cut);
    (parse_pair(b.data(), (int64_t)b.size(), &w, &off, &why) >= 0 ? accepted : rejected)++;
  }
  std::mt19937_64 rng(12345);
  for (int it = 0; it < 20000; ++it) {
    const std::vector<uint8_t>& src = (sched.empty() || (it & 1)) ? good : sched;
    std::vector<uint8_t> b(src);
    const int flips = 1 + int(rng() % 6);
    for (int k = 0; k < flips; ++k) b[rng() % b.size()] = uint8_t(rng());
    if (rng() % 4 == 0) b.resize(rng() % (b.size() + 1));
    (parse_pair(b.data(), (int64_t)b.size(), &w, &off, &why) >= 0 ? accepted : rejected)++;
  }
  for (int it = 0; it < 5000; ++it) {   // random bodies behind the stream magic
    std::vector<uint8_t> b(4 + rng() % 300);
    b[0] = 0xAC, b[1] = 0xED, b[2] = 0, b[3] = 5;
    for (size_t k = 4; k < b.size(); ++k) b[k] = (rng() % 2) ? uint8_t(0x70 + rng() % 16) : uint8_t(rng());
    (parse_pair(b.data(), (int64_t)b.size(), &w, &off, &why) >= 0 ? accepted : rejected)++;
  }
  std::printf("fuzz ok: %ld accepted, %ld rejected\n", accepted, rejected);
  return 0;
}
