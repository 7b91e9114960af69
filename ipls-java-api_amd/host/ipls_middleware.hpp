// ipls_middleware.hpp -- Middleware.main (Middleware.java:212-268), the
// loopback socket server between the Python IPLS API and the aggregator, over
// the C-ABI.  Header-only, POSIX sockets, C++17.
//
// One connection per task, as the reference serves them (Deserialize,
// Middleware.java:121-162; Send_Ack :188-194; Return_Global_model :178-184):
//   task 1  [i16 1][i16 bootstrapper][i16 n]{[i16 len][bytes]}*n [i16 len][path]
//           [i16 len][file name][i32 model_size]          -> IPLS instance, ACK
//   task 2  [i16 2][model_size x f64 big-endian]           -> UpdateModel, ACK
//   task 3  [i16 3]                                        -> model_size x f64 (writeDouble)
//   ACK     writeChar('A') = 00 41
//
// Where Java reads task 2 one readDouble at a time into a List<Double> and
// writes task 3 one writeDouble at a time on an unbuffered stream, this server
// never holds the model on the host:
//   - task 2 is UpdateGradient over the owned partitions (IPLS.java:1737-1743):
//     partition p's slice of the stream is one ipls_agg_accumulate_chunked
//     call whose source recv()s each chunk straight into the library's pinned
//     ring (the copy engine sends chunk k while chunk k+1 is received; the
//     count slot 1.0 of OrganizeGradients, IPLS.java:1018-1040, is appended);
//   - task 3 is GetPartitions (IPLS.java:1159-1174) through
//     ipls_agg_get_partitions_wire_chunked: the divide kernel writes the
//     writeDouble stream and each chunk is send()-ed from the pinned ring while
//     the next crosses PCIe.
// The aggregator is the loopback one of BASELINE configs[0] ("-pa 3 -n 3
// loopback: the aggregator averages 3 peers"): it owns every partition and a
// round closes after -n updates (AggregatePartition for all, IPLS.java:
// 1248-1274).  The Python server (ipls/middleware.py) does the same.
#pragma once

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "ipls_host.hpp"

namespace ipls_host {

// ---- socket helpers ----------------------------------------------------------
// false on EOF or error (the reference's EOFException / IOException)
inline bool recv_exact(int fd, void* buf, size_t n) {
  char* p = (char*)buf;
  while (n) {
    const ssize_t k = ::recv(fd, p, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}
inline bool send_all(int fd, const void* buf, size_t n) {
  const char* p = (const char*)buf;
  while (n) {
    const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}
inline bool read_i16(int fd, int16_t* v) {
  uint8_t b[2];
  if (!recv_exact(fd, b, 2)) return false;
  *v = (int16_t)((b[0] << 8) | b[1]);
  return true;
}
inline bool read_i32(int fd, int32_t* v) {
  uint8_t b[4];
  if (!recv_exact(fd, b, 4)) return false;
  *v = (int32_t)(((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3]);
  return true;
}
// get_string (Middleware.java:112-119): [i16 len][len bytes]
inline bool read_jstr(int fd, std::string* s) {
  int16_t n;
  if (!read_i16(fd, &n) || n < 0) return false;
  s->assign((size_t)n, '\0');
  return n == 0 || recv_exact(fd, s->data(), (size_t)n);
}
inline void big_socket_buffers(int fd, int bytes = 8 << 20) {
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &bytes, sizeof bytes);
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &bytes, sizeof bytes);
}
// A bound on every blocking recv/send of a connection: a peer that stalls
// mid-task makes that recv/send fail (EAGAIN -> recv_exact / send_all false)
// instead of holding the task forever.  ms <= 0: no bound.
inline void io_timeout(int fd, int ms) {
  if (ms <= 0) return;
  timeval tv{};
  tv.tv_sec = ms / 1000;
  tv.tv_usec = (ms % 1000) * 1000;
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
}

// ---- the server ----------------------------------------------------------------
class MiddlewareServer {
 public:
  struct Init {   // task 1's fields (Middleware.java:128-154)
    bool is_bootstrapper = false;
    std::vector<std::string> bootstrappers;
    std::string path, file_name;
    int32_t model_size = 0;
  };
  struct Stats {
    int64_t updates = 0, replies = 0, rounds = 0, failed = 0;
    double update_s = 0, reply_s = 0;   // inside the task handlers, socket reads/writes included
  };

  // opts: Middleware.parse_arguments' PeerData (-pa, -n, device ...);
  // io_timeout_ms bounds each blocking socket read/write of a connection
  explicit MiddlewareServer(PeerData opts, int64_t chunk = 1 << 19, int io_timeout_ms = 60000)
      : opts_(std::move(opts)), chunk_(chunk), io_timeout_ms_(io_timeout_ms) {}
  ~MiddlewareServer() {
    if (lfd_ >= 0) ::close(lfd_);
  }
  MiddlewareServer(const MiddlewareServer&) = delete;
  MiddlewareServer& operator=(const MiddlewareServer&) = delete;

  // new ServerSocket(port) on 127.0.0.1; port 0 picks a free one.  Returns the port.
  int listen(int port = 0) {
    lfd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (lfd_ < 0) throw IllegalArgumentException(IPLS_E_INVAL, "socket() failed");
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    socklen_t len = sizeof a;
    if (::bind(lfd_, (sockaddr*)&a, sizeof a) != 0 || ::listen(lfd_, 16) != 0 ||
        ::getsockname(lfd_, (sockaddr*)&a, &len) != 0)
      throw IllegalArgumentException(IPLS_E_INVAL, std::string("bind/listen failed: ") + std::strerror(errno));
    return ntohs(a.sin_port);
  }

  // The accept loop of Middleware.main: one task per connection.  Stops after
  // max_connections (< 0: never).  A task that fails (a short read, a library
  // error) throws, as the reference's main ends on its first exception
  // (Middleware.java:262-265); a caller running it on a thread catches there.
  // A task-2 connection that ends mid-update leaves the partitions received
  // before it folded (each partition is one call; the one cut short is not).
  // A client that stalls fails its task after io_timeout_ms, the same way.
  // The library holds no shard lock while a task's socket is read or
  // written (the chunked calls lock for the fold / the snapshot only), so
  // other threads' calls on the same IPLS instance never wait for a client.
  // on_error: when given, a task that fails calls on_error(task, exception)
  // and the server goes on with the next connection instead of throwing (what
  // ipls.middleware.serve does; a server of many peers should not be ended
  // by one bad client).  task is 0 when the connection failed before its
  // task number arrived.
  using OnError = std::function<void(int16_t task, const JavaException& e)>;
  void serve(int max_connections = -1, const OnError& on_error = nullptr) {
    for (int served = 0; max_connections < 0 || served < max_connections; ++served) {
      const int fd = ::accept(lfd_, nullptr, nullptr);
      if (fd < 0) {
        if (errno == EINTR) { --served; continue; }
        throw IllegalArgumentException(IPLS_E_INVAL, "accept failed");
      }
      struct Closer { int fd; ~Closer() { ::close(fd); } } closer{fd};
      big_socket_buffers(fd);
      io_timeout(fd, io_timeout_ms_);
      int16_t task = 0;
      try {
        if (!read_i16(fd, &task)) throw BufferUnderflowException(IPLS_E_FORMAT, "EOFException: no task");
        if (task == 1) task1(fd);
        else if (task == 2) task2(fd);
        else if (task == 3) task3(fd);
        // else: Ipls.terminate (the reference does nothing)
      } catch (const JavaException& e) {
        if (!on_error) throw;
        ++stats_.failed;
        on_error(task, e);
      }
    }
  }

  const Stats& stats() const { return stats_; }
  const Init& init() const { return init_; }
  IPLS* ipls() { return ipls_.get(); }

 private:
  static constexpr uint8_t kAck[2] = {0x00, 0x41};   // writeChar('A')

  void ack(int fd) {
    if (!send_all(fd, kAck, 2)) throw DeviceError(IPLS_E_INVAL, "IOException: ACK not sent");
  }

  // task 1: new IPLS(Path, FileName, Bootstrappers, is_bootstraper, model_size)
  void task1(int fd) {
    Init in;
    int16_t boot = 0, nb = 0;
    if (!read_i16(fd, &boot) || !read_i16(fd, &nb)) throw BufferUnderflowException(IPLS_E_FORMAT, "EOFException in task 1");
    in.is_bootstrapper = boot != 0;
    for (int i = 0; i < nb; ++i) {
      std::string s;
      if (!read_jstr(fd, &s)) throw BufferUnderflowException(IPLS_E_FORMAT, "EOFException in task 1");
      in.bootstrappers.push_back(std::move(s));
    }
    if (!read_jstr(fd, &in.path) || !read_jstr(fd, &in.file_name) || !read_i32(fd, &in.model_size))
      throw BufferUnderflowException(IPLS_E_FORMAT, "EOFException in task 1");
    PeerData pd = opts_;
    pd._MODEL_SIZE = in.model_size;
    std::vector<int32_t> all((size_t)pd._PARTITIONS);
    for (int p = 0; p < pd._PARTITIONS; ++p) all[(size_t)p] = p;
    ipls_.reset();   // a second init replaces the instance, as `ipls = new IPLS(...)` does
    ipls_ = std::make_unique<IPLS>(pd, all);
    init_ = std::move(in);
    pending_ = 0;
    ack(fd);
  }

  // task 2: Deserialize + ipls_daemon.UpdateModel(Updates), streamed (see the file comment)
  void task2(int fd) {
    if (!ipls_) throw IllegalArgumentException(IPLS_E_INVAL, "NullPointerException: task 2 before task 1");
    const auto t0 = std::chrono::steady_clock::now();
    ipls_agg* h = ipls_->handle();
    struct Src {
      int fd;
      int64_t L;
    };
    auto source = [](void* ctx, void* dst, int64_t off, int64_t n) -> int {
      const Src* s = (const Src*)ctx;
      const int64_t wire = std::min(off + n, s->L - 1) - off;   // values of this chunk that come off the socket
      if (wire > 0 && !recv_exact(s->fd, dst, (size_t)wire * 8)) return 1;
      if (off + n == s->L) {   // the count slot: 1.0, big-endian
        static const uint8_t one_be[8] = {0x3f, 0xf0, 0, 0, 0, 0, 0, 0};
        std::memcpy((char*)dst + 8 * (n - 1), one_be, 8);
      }
      return 0;
    };
    for (int32_t p : ipls_->Auth_List) {
      Src s{fd, ipls_->partition_length(p)};
      check(ipls_agg_accumulate_chunked(h, p, IPLS_TGT_AGG, s.L, IPLS_HOST_BE, chunk_, source, &s), h);
    }
    if (++pending_ >= opts_.Min_Members) {   // the loopback round closes after -n updates
      check(ipls_agg_finalize(h, IPLS_ALL_PARTITIONS, nullptr, IPLS_HOST_BE, nullptr), h);
      pending_ = 0;
      ++stats_.rounds;
    }
    check(ipls_agg_sync(h), h);
    stats_.update_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    ++stats_.updates;
    ack(fd);
  }

  // task 3: Return_Global_model(ipls_daemon.Get_Partitions(), clientSocket)
  void task3(int fd) {
    if (!ipls_) throw IllegalArgumentException(IPLS_E_INVAL, "NullPointerException: task 3 before task 1");
    const auto t0 = std::chrono::steady_clock::now();
    ipls_agg* h = ipls_->handle();
    auto sink = [](void* ctx, const double* v, int64_t, int64_t n) -> int {
      return send_all(*(const int*)ctx, v, (size_t)n * 8) ? 0 : 1;
    };
    check(ipls_agg_get_partitions_wire_chunked(h, chunk_, sink, &fd), h);
    stats_.reply_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    ++stats_.replies;
  }

  PeerData opts_;
  int64_t chunk_;
  int io_timeout_ms_;
  int lfd_ = -1;
  std::unique_ptr<IPLS> ipls_;
  Init init_;
  int pending_ = 0;
  Stats stats_;
};

// ---- the other end: what the Python IPLS API does per task ----------------------
// (connect, send the task, read the ACK or the model, close), for native tests
// and benches.  Each throws on a refused connection or a short read.
struct MiddlewareClient {
  static int connect_to(int port) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) throw IllegalArgumentException(IPLS_E_INVAL, "socket() failed");
    big_socket_buffers(fd);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (::connect(fd, (sockaddr*)&a, sizeof a) != 0) {
      ::close(fd);
      throw IllegalArgumentException(IPLS_E_INVAL, std::string("connect failed: ") + std::strerror(errno));
    }
    return fd;
  }
  // task 1 (Middleware.java:128-154)
  static void init(int port, int32_t model_size, const std::string& path = "/ip4/127.0.0.1/tcp/5001",
                   const std::string& file_name = "model", bool bootstrapper = false,
                   const std::vector<std::string>& bootstrappers = {}) {
    std::vector<uint8_t> m = {0, 1, 0, (uint8_t)(bootstrapper ? 1 : 0), (uint8_t)(bootstrappers.size() >> 8),
                              (uint8_t)bootstrappers.size()};
    auto jstr = [&](const std::string& s) {
      m.push_back((uint8_t)(s.size() >> 8));
      m.push_back((uint8_t)s.size());
      m.insert(m.end(), s.begin(), s.end());
    };
    for (const auto& b : bootstrappers) jstr(b);
    jstr(path);
    jstr(file_name);
    for (int sh = 24; sh >= 0; sh -= 8) m.push_back((uint8_t)((uint32_t)model_size >> sh));
    exchange(port, m.data(), m.size(), nullptr, 0, true);
  }
  // task 2 (Middleware.java:156-160): model_size big-endian doubles
  static void update(int port, const void* be, size_t nbytes) {
    const uint8_t h[2] = {0, 2};
    exchange(port, h, 2, be, nbytes, true);
  }
  // task 3 (Middleware.java:164-170): the model back as writeDouble bytes
  static void get(int port, void* out, size_t nbytes) {
    const uint8_t h[2] = {0, 3};
    const int fd = connect_to(port);
    const bool ok = send_all(fd, h, 2) && recv_exact(fd, out, nbytes);
    ::close(fd);
    if (!ok) throw BufferUnderflowException(IPLS_E_FORMAT, "EOFException: short task-3 reply");
  }

 private:
  static void exchange(int port, const void* a, size_t na, const void* b, size_t nb, bool want_ack) {
    const int fd = connect_to(port);
    uint8_t ack[2] = {0, 0};
    bool ok = send_all(fd, a, na) && (nb == 0 || send_all(fd, b, nb));
    if (ok && want_ack) ok = recv_exact(fd, ack, 2) && ack[0] == 0 && ack[1] == 'A';
    ::close(fd);
    if (!ok) throw BufferUnderflowException(IPLS_E_FORMAT, "no ACK from the Middleware");
  }
};

}  // namespace ipls_host
