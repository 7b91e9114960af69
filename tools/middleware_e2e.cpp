// middleware_e2e.cpp -- the Middleware loopback socket end to end from native
// code: ipls_host::MiddlewareServer (host/ipls_middleware.hpp, Middleware.main
// over the C-ABI) against a C++ client doing what the Python IPLS API does per
// task (connect, send, read the reply).  bench.py runs it as a child process
// beside the Python server's leg.
//
//   middleware_e2e M P K D [chunk]
//     M model doubles, -pa P, -n K: each round is K task-2 updates (cycling D
//     synthetic update vectors) and one task-3 reply; two rounds (the first
//     cold).  Ceiling: the same client against a server that moves the same
//     bytes into / out of one pinned buffer with no aggregator.
//
// Update vector d is SURVEY.md §8(d)'s counter formula with (p, k) = (200+d, 0)
// over M values (element M-1 = 1.0), the same bytes bench.py's Python leg
// sends, so the reply's checksum (oracle.checksum of the averaged model, i.e.
// sum_i splitmix64(bits(x_i) + i*0x9E3779B97F4A7C15)) is checked by bench.py
// against the oracle; this tool links no oracle code.  Prints one JSON line.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "ipls_middleware.hpp"

using namespace ipls_host;
using clk = std::chrono::steady_clock;

static uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// update vector d as big-endian bytes
static std::vector<uint8_t> synth_be(int64_t M, int p, int k) {
  const uint64_t seed = 0x1B52026ull;
  std::vector<uint8_t> out((size_t)M * 8);
  const uint64_t key0 = seed ^ ((uint64_t)(uint32_t)p << 40) ^ ((uint64_t)(uint32_t)k << 32);
  for (int64_t i = 0; i < M; ++i) {
    double x;
    if (i == M - 1) {
      x = 1.0;
    } else {
      const double u = (double)(splitmix64(key0 ^ (uint64_t)i) >> 11) * 0x1p-53;
      double t = 2.0 * u;
      t = t - 1.0;
      x = t * 1e-2;
    }
    uint64_t b;
    std::memcpy(&b, &x, 8);
    b = __builtin_bswap64(b);
    std::memcpy(&out[(size_t)i * 8], &b, 8);
  }
  return out;
}

struct Round {
  double seconds = 0, task2_ms = 0, task3_ms = 0;
};

// one round: K task 2 (ACK each) + one task 3 (reply into `reply`)
static Round client_round(int port, int K, const std::vector<std::vector<uint8_t>>& ups, std::vector<uint8_t>& reply) {
  Round r;
  const auto t0 = clk::now();
  for (int k = 0; k < K; ++k) {
    const auto a = clk::now();
    const auto& u = ups[(size_t)k % ups.size()];
    MiddlewareClient::update(port, u.data(), u.size());
    r.task2_ms += std::chrono::duration<double, std::milli>(clk::now() - a).count();
  }
  const auto a = clk::now();
  MiddlewareClient::get(port, reply.data(), reply.size());
  r.task3_ms = std::chrono::duration<double, std::milli>(clk::now() - a).count();
  r.seconds = std::chrono::duration<double>(clk::now() - t0).count();
  r.task2_ms /= K;
  return r;
}

static void print_round(const char* name, const Round& r, double nbytes, int K, bool comma) {
  std::printf("\"%s\": {\"seconds\": %.4f, \"GBps\": %.3f, \"task2_ms_mean\": %.3f, \"task2_GBps\": %.3f, "
              "\"task3_ms\": %.3f, \"task3_GBps\": %.3f}%s",
              name, r.seconds, (K + 1) * nbytes / r.seconds / 1e9, r.task2_ms, nbytes / r.task2_ms / 1e6, r.task3_ms,
              nbytes / r.task3_ms / 1e6, comma ? ", " : "");
}

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s M P K D [chunk]\n", argv[0]);
    return 1;
  }
  const int64_t M = std::atoll(argv[1]);
  const int P = std::atoi(argv[2]), K = std::atoi(argv[3]), D = std::atoi(argv[4]);
  const int64_t chunk = argc > 5 ? std::atoll(argv[5]) : (1 << 19);
  const double nbytes = 8.0 * (double)M;
  std::vector<std::vector<uint8_t>> ups;
  for (int d = 0; d < D; ++d) ups.push_back(synth_be(M, 200 + d, 0));
  std::vector<uint8_t> reply((size_t)M * 8);
  std::memset(reply.data(), 0, reply.size());

  // ---- the ceiling: the same socket traffic, no aggregator
  Round c[2];
  {
    void* pin = nullptr;
    if (ipls_host_alloc((size_t)M * 8, &pin) != 0) return 4;
    // a plain accept loop (the aggregator-free server)
    const int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    socklen_t len = sizeof a;
    ::bind(lfd, (sockaddr*)&a, sizeof a);
    ::listen(lfd, 16);
    ::getsockname(lfd, (sockaddr*)&a, &len);
    const int nport = ntohs(a.sin_port);
    std::thread srv([&] {
      for (int i = 0; i < 2 * (K + 1); ++i) {
        const int fd = ::accept(lfd, nullptr, nullptr);
        big_socket_buffers(fd);
        int16_t t = 0;
        read_i16(fd, &t);
        if (t == 2) {
          recv_exact(fd, pin, (size_t)M * 8);
          const uint8_t ack[2] = {0, 'A'};
          send_all(fd, ack, 2);
        } else if (t == 3) {
          send_all(fd, pin, (size_t)M * 8);
        }
        ::close(fd);
      }
    });
    for (auto& r : c) r = client_round(nport, K, ups, reply);
    srv.join();
    ::close(lfd);
    ipls_host_free(pin);
  }

  // ---- the aggregator: MiddlewareServer (-pa P -n K)
  Round g[2];
  MiddlewareServer::Stats st0{}, st1{};
  {
    PeerData opts;
    opts._PARTITIONS = P;
    opts.Min_Members = K;
    MiddlewareServer server(opts, chunk);
    const int port = server.listen(0);
    std::string srv_err;   // an exception must not leave the server thread (std::terminate)
    std::thread srv([&] {
      try {
        server.serve(1 + 2 * (K + 1));
      } catch (const std::exception& e) {
        srv_err = e.what();
      }
    });
    MiddlewareClient::init(port, (int32_t)M, "/ip4/127.0.0.1/tcp/5001", "bench");
    g[0] = client_round(port, K, ups, reply);
    st0 = server.stats();
    g[1] = client_round(port, K, ups, reply);
    st1 = server.stats();
    srv.join();
    if (!srv_err.empty()) {
      std::fprintf(stderr, "server: %s\n", srv_err.c_str());
      return 6;
    }
  }
  // the averaged model's checksum (oracle.checksum's definition) over the reply
  uint64_t sum = 0;
  for (int64_t i = 0; i < M; ++i) {
    uint64_t b;
    std::memcpy(&b, &reply[(size_t)i * 8], 8);
    b = __builtin_bswap64(b);
    sum += splitmix64(b + (uint64_t)i * 0x9E3779B97F4A7C15ull);
  }
  std::printf("{\"M\": %lld, \"P\": %d, \"K\": %d, \"D\": %d, \"chunk\": %lld, ", (long long)M, P, K, D, (long long)chunk);
  print_round("aggregator", g[1], nbytes, K, true);
  print_round("aggregator_cold_round", g[0], nbytes, K, true);
  print_round("socket_ceiling", c[1], nbytes, K, true);
  print_round("socket_ceiling_cold_round", c[0], nbytes, K, true);
  std::printf("\"server_ms_per_task2\": %.3f, \"server_ms_task3\": %.3f, \"reply_checksum\": \"%llu\"}\n",
              1e3 * (st1.update_s - st0.update_s) / K, 1e3 * (st1.reply_s - st0.reply_s), (unsigned long long)sum);
  return 0;
}
