// test_host_parity.cpp -- parity of the C++ host mirror (ipls_host.hpp) over
// the HIP C-ABI, against the C oracle (oracle/ipls_oracle.c, linked as the
// checker only).  Each TEST reads like the Java flow it mirrors.
//
//   test_host_parity            -> all tests (needs a GPU)
//   test_host_parity --no-gpu   -> the host-only tests (flags, frame codec)
//
// ETHModel (config A) is read from tests/golden/ethmodel.f64be.gz via zlib.
#include <zlib.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "ipls_host.hpp"
#include "ipls_middleware.hpp"
#include "ipls_oracle.h"

using namespace ipls_host;

static int g_fail = 0, g_pass = 0;
#define CHECK(cond, what)                                                        \
  do {                                                                           \
    if (!(cond)) {                                                               \
      std::fprintf(stderr, "  FAIL %s:%d %s\n", __FILE__, __LINE__, what);       \
      throw std::runtime_error(what);                                            \
    }                                                                            \
  } while (0)

static void run(const char* name, const std::function<void()>& f) {
  try {
    f();
    ++g_pass;
    std::printf("PASS %s\n", name);
  } catch (const std::exception& e) {
    ++g_fail;
    std::printf("FAIL %s: %s\n", name, e.what());
  }
}

static bool bits_equal(const double* a, const double* b, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    uint64_t x, y;
    std::memcpy(&x, &a[i], 8);
    std::memcpy(&y, &b[i], 8);
    if (x != y && !(a[i] != a[i] && b[i] != b[i])) {
      std::fprintf(stderr, "  element %zu: %.17g != %.17g\n", i, a[i], b[i]);
      return false;
    }
  }
  return true;
}

static std::vector<double> synth(int64_t L, int p, int k) {
  std::vector<double> v((size_t)L);
  ipls_oracle_synth_fill(v.data(), L, 0x1B52026ULL, p, k);
  return v;
}

// oracle: OrganizeGradients partition p of flat
static std::vector<double> organize(const std::vector<double>& flat, int64_t M, int P, int p) {
  std::vector<double> out((size_t)ipls_oracle_partition_len(M, P, p));
  if (ipls_oracle_organize(flat.data(), (int64_t)flat.size(), M, P, p, out.data()) != 0)
    throw std::runtime_error("oracle organize");
  return out;
}

static std::vector<double> read_ethmodel(const std::string& path) {
  gzFile f = gzopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::vector<unsigned char> raw;
  unsigned char buf[1 << 16];
  int n;
  while ((n = gzread(f, buf, sizeof buf)) > 0) raw.insert(raw.end(), buf, buf + n);
  gzclose(f);
  std::vector<double> m(raw.size() / 8);
  ipls_oracle_be_decode(raw.data(), (int64_t)m.size(), m.data());
  return m;
}

int main(int argc, char** argv) {
  const bool gpu = !(argc > 1 && std::string(argv[1]) == "--no-gpu");
  const std::string golden = argc > 2 ? argv[2] : "tests/golden";

  // ---------------- host-only ----------------
  run("Middleware.parse_arguments", [] {
    auto d = Middleware::parse_arguments({"-p", "5000", "-pa", "3", "-mp", "1", "-n", "3", "-i", "0", "-training",
                                          "60", "-aggr", "1", "-async", "true"});
    CHECK(d.port == 5000 && d._PARTITIONS == 3 && d.Min_Members == 3 && d.Partial_Aggregation && !d.isSynchronous,
          "flag values");
    bool threw = false;
    try {
      Middleware::parse_arguments({"-p", "5000", "-pa", "3"});
    } catch (const IllegalArgumentException&) {
      threw = true;
    }
    CHECK(threw, "missing required flags must throw");
  });
  run("MyIPFSClass.Marshall_Packet/GET_GRADIENTS", [] {
    std::vector<double> g = {1.5, -0.0, 1e300, 5e-324};
    auto fr = MyIPFSClass::Marshall_Packet(g, "QmOrigin", 7, 42, 3);
    std::vector<uint8_t> ref(14 + 8 * g.size() + 8);
    const int64_t nb = ipls_oracle_frame_encode(g.data(), (int32_t)g.size(), 7, 42, 3, (const uint8_t*)"QmOrigin", 8,
                                                ref.data());
    CHECK(nb == (int64_t)fr.size() && std::memcmp(fr.data(), ref.data(), fr.size()) == 0, "frame bytes");
    auto h = MyIPFSClass::GET_GRADIENTS(fr);
    CHECK(h.pid == 3 && h.n == 4 && h.partition == 7 && h.iteration == 42 && h.payload_off == 14, "header");
    bool threw = false;
    try {
      MyIPFSClass::GET_GRADIENTS(std::vector<uint8_t>(fr.begin(), fr.begin() + 20));
    } catch (const BufferUnderflowException&) {
      threw = true;
    }
    CHECK(threw, "truncated frame must throw BufferUnderflowException");
  });

  if (gpu) {
    // ---------------- device path ----------------
    run("IPLS over two GPUs' shards: UpdateGradient + Send_Partial_Updates", [&] {
      const int64_t M = 200003;
      PeerData pd;
      pd._MODEL_SIZE = M;
      pd._PARTITIONS = 4;
      pd.Min_Members = 2;
      pd.devices = {0, 0};   // the one GPU of the test box, as two shards
      IPLS ipls(pd, {3, 0, 1});
      auto g = synth(M, 4, 4);
      ipls.UpdateGradient(&g);
      const std::vector<int32_t> w1 = {4, 2, 7};
      auto texts = ipls.Send_Partial_Updates(11, w1, "QmPeer");
      CHECK(texts.size() == 3, "one text per Auth_List partition");
      for (int i = 0; i < 3; ++i) {
        const int p = ipls.Auth_List[i];
        auto part = organize(g, M, 4, p);
        std::vector<double> agg(part.size());
        for (size_t j = 0; j < part.size(); ++j) agg[j] = 0.0 + part[j];   // fresh accumulator + own bucket
        std::vector<uint8_t> fr(14 + 8 * agg.size() + 6), want(4 * ((fr.size() + 2) / 3));
        ipls_oracle_frame_encode(agg.data(), (int32_t)agg.size(), 11, w1[i], 3, (const uint8_t*)"QmPeer", 6,
                                 fr.data());
        ipls_oracle_b64url_encode(fr.data(), (int64_t)fr.size(), want.data());
        CHECK(texts[i].size() == want.size() && std::memcmp(texts[i].data(), want.data(), want.size()) == 0,
              "publish text == Base64.getUrlEncoder(Marshall_Packet(...))");
      }
      bool threw = false;
      try {
        ipls.Send_Partial_Updates(11, {1, 2}, "QmPeer");
      } catch (const IllegalArgumentException&) {
        threw = true;
      }
      CHECK(threw, "a workers list of the wrong length must throw");
    });
    run("IPLS config A (ETHModel, -pa 3 -n 3)", [&] {
      const auto model = read_ethmodel(golden + "/ethmodel.f64be.gz");
      const int64_t M = (int64_t)model.size();
      PeerData pd;
      pd._MODEL_SIZE = M;
      pd._PARTITIONS = 3;
      pd.Min_Members = 3;
      IPLS ipls(pd, {0, 1, 2});
      Updater updater(ipls);
      Light_IPLS_Daemon daemon(ipls);
      ipls.InitializeWeights(model);
      auto first = ipls.GetPartitions();   // count slot 0.0: model passes through
      CHECK(bits_equal(first.data(), model.data(), model.size()), "initial GetPartitions");
      std::vector<std::vector<double>> peers(3, model);
      for (int k = 0; k < 3; ++k) {
        auto noise = synth(M + 1, 0, k);
        for (int64_t i = 0; i < M; ++i) peers[k][i] = model[i] + noise[i];
      }
      daemon.UpdateModel(peers[0]);                              // own partitions
      for (int k = 1; k < 3; ++k) {
        auto parts = ipls.OrganizeGradients(peers[k]);
        for (int p = 0; p < 3; ++p) updater._Update(&parts[p], p, true);   // arrivals
      }
      auto avg = daemon.Get_Partitions();
      // oracle
      std::vector<double> expect;
      for (int p = 0; p < 3; ++p) {
        const int64_t L = ipls_oracle_partition_len(M, 3, p);
        std::vector<double> s((size_t)L);
        std::vector<std::vector<double>> b;
        for (int k = 0; k < 3; ++k) b.push_back(organize(peers[k], M, 3, p));
        const double* bp[3] = {b[0].data(), b[1].data(), b[2].data()};
        ipls_oracle_reduce(s.data(), bp, 3, L, 1);
        std::vector<double> d((size_t)L - 1);
        ipls_oracle_divide(s.data(), L, 0, d.data());
        expect.insert(expect.end(), d.begin(), d.end());
      }
      CHECK(avg.size() == expect.size() && bits_equal(avg.data(), expect.data(), avg.size()), "averaged model");
    });

    run("Middleware.main over TCP loopback (config A, -pa 3 -n 3), two rounds", [&] {
      // the native server (host/ipls_middleware.hpp) with a chunk of 73,934
      // values: partition 2 (L = 147,869 = 2 x 73,934 + 1) ends with a chunk
      // that is its count slot alone, partitions 0 and 1 with 3 values + the slot
      const auto model = read_ethmodel(golden + "/ethmodel.f64be.gz");
      const int64_t M = (int64_t)model.size();
      PeerData opts = Middleware::parse_arguments({"-p", "0", "-pa", "3", "-mp", "1", "-n", "3", "-i", "0",
                                                   "-training", "60", "-aggr", "0"});
      MiddlewareServer server(opts, 73934);
      const int port = server.listen(0);
      std::string srv_err;   // an exception must not leave the server thread (std::terminate)
      std::thread srv([&] {
        try {
          server.serve(1 + 2 * 4);
        } catch (const std::exception& e) {
          srv_err = e.what();
        }
      });
      std::vector<std::vector<double>> peers(3, model);
      std::vector<std::vector<uint8_t>> wire(3, std::vector<uint8_t>((size_t)M * 8));
      for (int k = 0; k < 3; ++k) {
        auto noise = synth(M + 1, 0, k);
        for (int64_t i = 0; i < M; ++i) peers[k][i] = model[i] + noise[i];
        peers[k][7 * k + 1] = -0.0;
        ipls_oracle_be_encode(peers[k].data(), M, wire[k].data());
      }
      std::vector<uint8_t> want;
      for (int p = 0; p < 3; ++p) {   // oracle: fixed-order sum from +0.0, the divide, writeDouble bytes
        const int64_t L = ipls_oracle_partition_len(M, 3, p);
        std::vector<double> sum((size_t)L), avg((size_t)L - 1);
        std::vector<std::vector<double>> b;
        for (int k = 0; k < 3; ++k) b.push_back(organize(peers[k], M, 3, p));
        const double* bp[3] = {b[0].data(), b[1].data(), b[2].data()};
        ipls_oracle_reduce(sum.data(), bp, 3, L, 1);
        ipls_oracle_divide(sum.data(), L, 0, avg.data());
        std::vector<uint8_t> bytes((size_t)(L - 1) * 8);
        ipls_oracle_be_encode_canonical(avg.data(), L - 1, bytes.data());
        want.insert(want.end(), bytes.begin(), bytes.end());
      }
      try {
        MiddlewareClient::init(port, (int32_t)M, "/ip4/127.0.0.1/tcp/5001", "ETHModel");
        for (int round = 0; round < 2; ++round) {
          for (int k = 0; k < 3; ++k) MiddlewareClient::update(port, wire[k].data(), wire[k].size());
          std::vector<uint8_t> got((size_t)M * 8);
          MiddlewareClient::get(port, got.data(), got.size());
          CHECK(got == want, "task-3 reply == the oracle's writeDouble stream");
        }
      } catch (...) {
        srv.detach();
        throw;
      }
      srv.join();
      CHECK(srv_err.empty(), ("server: " + srv_err).c_str());
      CHECK(server.stats().rounds == 2 && server.stats().updates == 6 && server.init().file_name == "ETHModel",
            "two rounds of three updates");
    });

    run("Middleware.main: a client that stalls in task 2 holds no GPU shard and times out", [&] {
      // the server's chunk source is a blocking recv with
      // no shard lock held and SO_RCVTIMEO on the connection.  A client
      // sends task 2 and 100,000 of partition 0's 147,871 values, then stops:
      // folds into partitions 0 and 1 of the same handle from this thread
      // return at once, and after the timeout the task fails (the server
      // throws, as Middleware.main ends on an exception) with partition 0
      // holding only those folds -- its cut-short slice folded nothing.
      const int64_t M = 443610;
      PeerData opts = Middleware::parse_arguments({"-p", "0", "-pa", "3", "-mp", "1", "-n", "3", "-i", "0",
                                                   "-training", "60", "-aggr", "0"});
      MiddlewareServer server(opts, 73934, 500);
      const int port = server.listen(0);
      std::string srv_err;
      std::atomic<bool> srv_done{false};
      std::thread srv([&] {
        try {
          server.serve(2);
        } catch (const std::exception& e) {
          srv_err = e.what();
        }
        srv_done = true;
      });
      MiddlewareClient::init(port, (int32_t)M, "/ip4/127.0.0.1/tcp/5001", "m");
      const int fd = MiddlewareClient::connect_to(port);
      std::vector<uint8_t> part((size_t)2 + 100000 * 8, 0x3f);
      part[0] = 0;
      part[1] = 2;   // task 2
      CHECK(send_all(fd, part.data(), part.size()), "partial task 2 sent");
      std::this_thread::sleep_for(std::chrono::milliseconds(100));   // the server now waits in recv
      ipls_agg* h = server.ipls()->handle();
      const int64_t L0 = ipls_oracle_partition_len(M, 3, 0), L1 = ipls_oracle_partition_len(M, 3, 1);
      const auto g0 = synth(L0, 0, 91), g1 = synth(L1, 1, 92);
      const auto t0 = std::chrono::steady_clock::now();
      CHECK(ipls_agg_accumulate(h, 0, IPLS_TGT_AGG, g0.data(), L0, IPLS_HOST_F64) == 0 &&
                ipls_agg_accumulate(h, 1, IPLS_TGT_AGG, g1.data(), L1, IPLS_HOST_F64) == 0 && ipls_agg_sync(h) == 0,
            "folds beside the stalled task");
      const double inside = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      CHECK(inside < 0.3, "the folds did not wait for the stalled client");
      for (int i = 0; i < 100 && !srv_done; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(50));
      ::close(fd);
      CHECK(srv_done.load(), "the server gave up on the stalled client");
      srv.join();
      CHECK(!srv_err.empty(), "task 2 failed with an exception");
      std::vector<double> got((size_t)L0);
      CHECK(ipls_agg_read(h, 0, IPLS_TGT_AGG, got.data(), L0, IPLS_HOST_F64) == 0, "read AGG[0]");
      std::vector<double> want((size_t)L0);
      const double* bp[1] = {g0.data()};
      ipls_oracle_reduce(want.data(), bp, 1, L0, 1);
      CHECK(bits_equal(got.data(), want.data(), (size_t)L0), "AGG[0] holds only the direct fold");
    });

    run("Middleware.main with on_error: a failed task ends its connection only", [&] {
      // the same stalled client against serve(n, on_error): the server reports
      // the task and answers the next client's task 3 from the same instance
      const int64_t M = 443610;
      PeerData opts = Middleware::parse_arguments({"-p", "0", "-pa", "3", "-mp", "1", "-n", "3", "-i", "0",
                                                   "-training", "60", "-aggr", "0"});
      MiddlewareServer server(opts, 73934, 300);
      const int port = server.listen(0);
      std::vector<int> failed_tasks;
      std::string srv_err;
      std::thread srv([&] {
        try {
          server.serve(3, [&](int16_t task, const JavaException&) { failed_tasks.push_back(task); });
        } catch (const std::exception& e) {
          srv_err = e.what();
        }
      });
      MiddlewareClient::init(port, (int32_t)M, "/ip4/127.0.0.1/tcp/5001", "m");
      const int fd = MiddlewareClient::connect_to(port);
      const uint8_t head[2] = {0, 2};
      CHECK(send_all(fd, head, 2), "task 2 header sent");   // then nothing: the recv times out
      std::vector<uint8_t> got((size_t)M * 8, 1);
      MiddlewareClient::get(port, got.data(), got.size());   // task 3 on the next connection
      ::close(fd);
      srv.join();
      CHECK(srv_err.empty(), ("server: " + srv_err).c_str());
      CHECK(failed_tasks == std::vector<int>{2} && server.stats().failed == 1 && server.stats().replies == 1,
            "one failed task 2, then the reply");
      bool zeros = true;   // nothing folded, no round closed: the initial (zero) model comes back
      for (uint8_t b : got) zeros = zeros && b == 0;
      CHECK(zeros, "the reply is the untouched model");
    });

    run("Updater file + frame arrivals, replicas, commit bytes", [&] {
      const int64_t L = 70001;
      PeerData pd;
      pd._MODEL_SIZE = 0;
      pd._PARTITIONS = 1;
      // synthetic geometry goes through the C-ABI's bucket_len
      ipls_agg_cfg c{};
      c.n_partitions = 1;
      c.bucket_len = L;
      ipls_agg* h = nullptr;
      check(ipls_agg_open(&c, &h), nullptr);
      std::vector<std::vector<double>> b;
      for (int k = 0; k < 4; ++k) b.push_back(synth(L, 3, k));
      std::vector<uint8_t> be(8 * (size_t)L);
      ipls_oracle_be_encode(b[1].data(), L, be.data());
      auto frame = MyIPFSClass::Marshall_Packet(b[2], "QmPeer2", 0, 1, 3);
      check(ipls_agg_accumulate(h, 0, IPLS_TGT_AGG, b[0].data(), L, IPLS_HOST_F64), h);
      check(ipls_agg_accumulate(h, 0, IPLS_TGT_AGG, be.data(), L, IPLS_HOST_BE), h);
      check(ipls_agg_accumulate(h, 0, IPLS_TGT_AGG, frame.data(), (int64_t)frame.size(), IPLS_HOST_FRAME), h);
      check(ipls_agg_accumulate(h, 0, IPLS_TGT_REP, b[3].data(), L, IPLS_HOST_F64), h);
      std::vector<uint8_t> file(8 * (size_t)L);
      check(ipls_agg_finalize(h, 0, file.data(), IPLS_HOST_BE, nullptr), h);
      ipls_agg_close(h);
      std::vector<double> s((size_t)L), r((size_t)L), w((size_t)L), wa((size_t)L);
      const double* bp[3] = {b[0].data(), b[1].data(), b[2].data()};
      ipls_oracle_reduce(s.data(), bp, 3, L, 1);
      const double* rp[1] = {b[3].data()};
      ipls_oracle_reduce(r.data(), rp, 1, L, 1);
      ipls_oracle_aggregate_partition(s.data(), r.data(), w.data(), wa.data(), L);
      std::vector<uint8_t> ref(8 * (size_t)L);
      ipls_oracle_be_encode(w.data(), L, ref.data());
      CHECK(file == ref, "update_file bytes of AGG + REP");
    });

    run("Other_Replica_Gradients: downloads, a remove, Collect_Replicas in HashMap order", [&] {
      // three other aggregators of partition 0 whose Pair(0, id) hashes fall
      // in bins 13, 7 and 2 of the 16-bin HashMap (found with oracle.JavaHashMap;
      // hashCodes 1951003300, 1951003326, 1951003387): keySet() walks them in
      // reverse insertion order.  The fourth is dropped: its partial arrived
      // (Download_Scheduler.java:329-332).
      PeerData pd;
      pd._MODEL_SIZE = 60001;
      pd._PARTITIONS = 1;
      IPLS ipls(pd, {0});
      const int64_t L = ipls_oracle_partition_len(60001, 1, 0);
      const char* ids[4] = {"QmPeer0006", "QmPeer0011", "QmPeer0030", "QmPeerGone"};
      const double scale[4] = {1e16, 1.0, -1e16, 3.0};
      std::vector<std::vector<double>> g;
      for (int a = 0; a < 4; ++a) {
        g.push_back(synth(L, 0, 20 + a));
        for (auto& x : g.back()) x *= scale[a];
        ipls.Other_Replica_Gradients(0, a, ids[a], g.back());
      }
      int32_t h0 = 0;
      check(ipls_java_pair_hash(0, (const uint8_t*)ids[0], 10, &h0), nullptr);
      CHECK(h0 == 1951003300, "Pair(0, \"QmPeer0006\").hashCode()");
      CHECK(ipls.Other_Replica_Gradients_remove(0, 3) && !ipls.Other_Replica_Gradients_remove(0, 3), "remove once");
      auto parts = ipls.Collect_Replicas();
      CHECK(parts.size() == 1 && parts[0] == (int32_t)(3 * L), "Participants: received x length per key");
      auto file = ipls.AggregatePartition(0);
      std::vector<double> rep((size_t)L, 0.0);
      for (int a : {2, 1, 0})   // keySet() order
        for (int64_t j = 0; j < L; ++j) rep[j] = rep[j] + g[a][j];
      std::vector<double> w((size_t)L);
      for (int64_t j = 0; j < L; ++j) w[j] = 0.0 + rep[j];   // W = AGG (+0.0) + REP
      std::vector<uint8_t> ref(8 * (size_t)L);
      ipls_oracle_be_encode(w.data(), L, ref.data());
      CHECK(file == ref, "W = AGG + REP with REP folded in the HashMap's key order");
      std::vector<double> asc((size_t)L, 0.0);
      for (int a : {0, 1, 2})
        for (int64_t j = 0; j < L; ++j) asc[j] = asc[j] + g[a][j];
      CHECK(!bits_equal(asc.data(), rep.data(), (size_t)L), "(the ascending order gives other bits)");
    });

    run("gradients from the future -> Update_Client_WaitAck_List", [&] {
      PeerData pd;
      pd._MODEL_SIZE = 50001;
      pd._PARTITIONS = 2;
      IPLS ipls(pd, {0, 1});
      Updater u(ipls);
      const int64_t L0 = ipls_oracle_partition_len(50001, 2, 0);
      auto now = synth(L0, 0, 1), later = synth(L0, 0, 2);
      u._Update(&now, 0, true);
      u._Update_from_future(&later, 0);
      auto first = ipls.AggregatePartition(0);          // this round: `now` only
      std::vector<uint8_t> ref(8 * (size_t)L0);
      ipls_oracle_be_encode(now.data(), L0, ref.data());
      CHECK(first == ref, "round before promotion");
      ipls.Update_Client_WaitAck_List();
      auto second = ipls.AggregatePartition(0);         // next round starts from `later`
      ipls_oracle_be_encode(later.data(), L0, ref.data());
      CHECK(second == ref, "promoted future gradients");
    });

    run("UpdaterThread: producers, hash-only files, device buckets, a bad request", [&] {
      PeerData pd;
      pd._MODEL_SIZE = 200003;
      pd._PARTITIONS = 6;
      IPLS ipls(pd, {0, 1, 2, 3, 4, 5});
      IPLS src(pd);   // its AGG arrays stand in for device-resident buckets (e.g. RCCL partials)
      std::vector<int64_t> L(6);
      std::vector<std::vector<double>> dval(6);
      std::vector<const void*> dptr(6);
      for (int p = 0; p < 6; ++p) {
        L[p] = ipls.partition_length(p);
        dval[p] = synth(L[p], p, 9);
        check(ipls_agg_accumulate(src.handle(), p, IPLS_TGT_AGG, dval[p].data(), L[p], IPLS_HOST_F64), src.handle());
        void* d = nullptr;
        check(ipls_agg_device_ptr(src.handle(), p, IPLS_TGT_AGG, &d), src.handle());
        dptr[p] = d;
      }
      check(ipls_agg_sync(src.handle()), src.handle());
      std::vector<std::vector<std::vector<double>>> seq(6);   // per partition, the buckets in fold order
      {
        UpdaterThread ut(ipls);
        auto producer = [&](int t) {
          for (int j = 0; j < 24; ++j) {
            const int p = j % 2 ? t + 3 : t;   // each partition has one producer: a fixed order
            UpdaterThread::Request r;
            r.partition = p;
            const int kind = (j + t) % 3;
            std::vector<double> g = synth(L[p], p, (t * 7 + j) % 5);
            if (kind == 0) {
              r.gradient = g;
            } else if (kind == 1) {
              r.file.resize(8 * (size_t)L[p]);
              ipls_oracle_be_encode(g.data(), L[p], r.file.data());
            } else {
              r.device = dptr[p];
              r.device_n = L[p];
              g = dval[p];
            }
            seq[p].push_back(g);
            ut.put(std::move(r));
            if (j % 7 == 6) std::this_thread::sleep_for(std::chrono::milliseconds(1));   // idle: queued folds start
            if (t == 0 && j == 11) {
              UpdaterThread::Request bad;
              bad.partition = 0;
              bad.gradient.assign(3, 1.0);   // shorter than L_0: dropped, reported
              ut.put(std::move(bad));
            }
          }
        };
        std::vector<std::thread> ths;
        for (int t = 0; t < 3; ++t) ths.emplace_back(producer, t);
        for (auto& th : ths) th.join();
        ut.drain();
        auto fails = ut.failures();
        CHECK(fails.size() == 1, "one dropped request");
      }
      for (int p = 0; p < 6; ++p) {
        std::vector<const double*> bp;
        for (auto& g : seq[p]) bp.push_back(g.data());
        std::vector<double> ref((size_t)L[p]), got((size_t)L[p]);
        ipls_oracle_reduce(ref.data(), bp.data(), (int)bp.size(), L[p], 1);
        check(ipls_agg_read(ipls.handle(), p, IPLS_TGT_AGG, got.data(), L[p], IPLS_HOST_F64), ipls.handle());
        CHECK(bits_equal(got.data(), ref.data(), (size_t)L[p]), "partition folded in its producer's order");
      }
    });

    run("Client_Wait_Ack drained -> the queued folds start (flush hint)", [&] {
      PeerData pd;
      pd._MODEL_SIZE = 120001;
      pd._PARTITIONS = 4;
      IPLS ipls(pd, {0, 1, 2, 3});
      IPLS src(pd);
      check(ipls_agg_set_coalesce(ipls.handle(), 1 << 20), ipls.handle());   // no size-triggered flush
      std::vector<int64_t> L(4);
      std::vector<std::vector<std::vector<double>>> vals(4);
      std::vector<std::vector<double>> dv(4);
      std::vector<const void*> dptr(4);
      for (int p = 0; p < 4; ++p) {
        L[p] = ipls.partition_length(p);
        dv[p] = synth(L[p], p, 5);
        check(ipls_agg_accumulate(src.handle(), p, IPLS_TGT_AGG, dv[p].data(), L[p], IPLS_HOST_F64), src.handle());
        void* d = nullptr;
        check(ipls_agg_device_ptr(src.handle(), p, IPLS_TGT_AGG, &d), src.handle());
        dptr[p] = d;
      }
      check(ipls_agg_sync(src.handle()), src.handle());
      const char* peers[3] = {"QmA", "QmB", "QmC"};
      {
        UpdaterThread ut(ipls, std::chrono::seconds(30));   // an idle flush would take 30 s
        ut.Client_Wait_Ack({peers[0], peers[1], peers[2]});
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < 3; ++k)
          for (int p = 0; p < 4; ++p) {
            UpdaterThread::Request r;
            r.partition = p;
            r.device = dptr[p];
            r.device_n = L[p];
            r.origin = peers[k];
            ut.put(std::move(r));
          }
        ut.Wait_Client_Gradients();
        // the request that cleared the last trainer launched the folds
        for (int i = 0; i < 2000 && ut.hint_flushes() == 0; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        CHECK(ut.hint_flushes() == 1, "one flush at the drain of Client_Wait_Ack");
        CHECK(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10), "not the idle flush");
        ut.drain();
        CHECK(ut.failures().empty(), "no failures");
      }
      for (int p = 0; p < 4; ++p) {
        const double* bp[3] = {dv[p].data(), dv[p].data(), dv[p].data()};
        std::vector<double> ref((size_t)L[p]), got((size_t)L[p]);
        ipls_oracle_reduce(ref.data(), bp, 3, L[p], 1);
        check(ipls_agg_read(ipls.handle(), p, IPLS_TGT_AGG, got.data(), L[p], IPLS_HOST_F64), ipls.handle());
        CHECK(bits_equal(got.data(), ref.data(), (size_t)L[p]), "three queued arrivals per partition");
      }
    });

    run("partial updates (-i 1): commit, replica fold, storage merge", [&] {
      PeerData pd;
      pd._MODEL_SIZE = 20001;
      pd._PARTITIONS = 2;
      IPLS ipls(pd, {0, 1});
      Updater u(ipls);
      const int64_t L0 = ipls_oracle_partition_len(20001, 2, 0);
      auto g = synth(L0, 0, 5);
      u._Update(&g, 0, true);
      auto file = ipls.commit_partial_update(0, 4);
      int32_t w = 0;
      int64_t off = 0;
      CHECK(ipls_pair_parse(file.data(), (int64_t)file.size(), &w, &off) == L0 && w == 4, "Pair header");
      std::vector<double> back((size_t)L0);
      ipls_oracle_be_decode(file.data() + off, L0, back.data());
      std::vector<double> s((size_t)L0);
      const double* bp[1] = {g.data()};
      ipls_oracle_reduce(s.data(), bp, 1, L0, 1);
      CHECK(bits_equal(back.data(), s.data(), (size_t)L0), "Pair payload = AGG");
      u._Update_from_partial(file, 0);                    // as a replica partial -> REP
      auto sum = ipls.AggregatePartition(0);               // W = AGG + REP = 2 * S
      std::vector<double> w2((size_t)L0), zero((size_t)L0, 0.0), wa((size_t)L0);
      std::vector<double> a = s, r = s;
      ipls_oracle_aggregate_partition(a.data(), r.data(), w2.data(), wa.data(), L0);
      std::vector<uint8_t> ref(8 * (size_t)L0);
      ipls_oracle_be_encode(w2.data(), L0, ref.data());
      CHECK(sum == ref, "AGG + REP after the Pair fold");
      Decentralized_Storage_Receiver store(ipls);
      auto merged = store.merge({file, file}, 1);
      std::vector<double> m2((size_t)L0);
      const double* mp[2] = {s.data(), s.data()};
      ipls_oracle_reduce(m2.data(), mp, 2, L0, 2);        // FIRST start: S + S
      ipls_oracle_be_encode(m2.data(), L0, ref.data());
      CHECK(merged == ref, "storage merge of two Pair files");
    });

    run("exceptions", [] {
      PeerData pd;
      pd._MODEL_SIZE = 10;
      pd._PARTITIONS = 7;
      bool neg = false;
      try {
        IPLS bad(pd);
      } catch (const NegativeArraySizeException&) {
        neg = true;
      }
      CHECK(neg, "M=10, -pa 7 -> NegativeArraySizeException");
      pd._PARTITIONS = 2;
      IPLS ok(pd, {0, 1});
      Updater u(ok);
      std::vector<double> shortg(3, 1.0);
      bool aioobe = false;
      try {
        u._Update(&shortg, 0, true);
      } catch (const ArrayIndexOutOfBoundsException&) {
        aioobe = true;
      }
      CHECK(aioobe, "short bucket -> ArrayIndexOutOfBoundsException");
      u._Update(nullptr, 0, true);   // Gradient == null: no-op
    });
  }
  std::printf("%d passed, %d failed\n", g_pass, g_fail);
  return g_fail ? 1 : 0;
}
