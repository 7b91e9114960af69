// ipls_host.hpp -- C++17 host-side mirror of the reference's aggregation path
// over the C-ABI (include/ipls_agg.h).  Header-only.
//
// The reference is Java (no JDK in this image), so the host layer above the
// C-ABI mirrors its classes in C++ under the same names, with the same
// argument meaning and the same exceptions:
//
//   IPLS                 IPLS.java:880-2305  (aggregation methods only)
//   Updater              Updater.java:14-218 (_Update)
//   UpdaterThread        Updater.run, Updater.java:155-216 (the reducer thread
//                        draining PeerData.queue, PeerData.java:117)
//   Light_IPLS_Daemon    Light_IPLS_Daemon.java:9-114 (UpdateModel / Get_Partitions)
//   MyIPFSClass          MyIPFSClass.java codecs used on the path
//   Middleware           Middleware.java:26-210 (flags, wire stream, Encode)
//
// Every arithmetic loop runs in the HIP library; nothing here computes on
// doubles.  Negative C-ABI codes become the Java exception the reference
// throws at the same spot (ArrayIndexOutOfBoundsException, ...).
#pragma once

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "ipls_agg.h"

namespace ipls_host {

// ---- Java exceptions -------------------------------------------------------
struct JavaException : std::runtime_error {
  int code;
  JavaException(int c, const std::string& m) : std::runtime_error(m), code(c) {}
  virtual const char* java_name() const { return "java.lang.RuntimeException"; }
};
#define IPLS_HOST_EXC(NAME, JNAME)                                           \
  struct NAME : JavaException {                                              \
    using JavaException::JavaException;                                      \
    const char* java_name() const override { return JNAME; }                 \
  };
IPLS_HOST_EXC(ArrayIndexOutOfBoundsException, "java.lang.ArrayIndexOutOfBoundsException")
IPLS_HOST_EXC(NegativeArraySizeException, "java.lang.NegativeArraySizeException")
IPLS_HOST_EXC(BufferUnderflowException, "java.nio.BufferUnderflowException")
IPLS_HOST_EXC(IllegalArgumentException, "java.lang.IllegalArgumentException")
IPLS_HOST_EXC(OutOfMemoryError, "java.lang.OutOfMemoryError")
IPLS_HOST_EXC(DeviceError, "ipls.DeviceError")
#undef IPLS_HOST_EXC

[[noreturn]] inline void raise(int rc, const ipls_agg* h) {
  (void)h;
  const std::string msg = ipls_agg_last_error(nullptr);   // this thread's failure
  switch (rc) {
    case IPLS_E_RANGE: throw ArrayIndexOutOfBoundsException(rc, msg);
    case IPLS_E_NEGSIZE: throw NegativeArraySizeException(rc, msg);
    case IPLS_E_FORMAT: throw BufferUnderflowException(rc, msg);
    case IPLS_E_INVAL: throw IllegalArgumentException(rc, msg);
    case IPLS_E_NOMEM: throw OutOfMemoryError(rc, msg);
    default: throw DeviceError(rc, msg);
  }
}
inline int64_t check(int64_t rc, const ipls_agg* h) {
  if (rc < 0) raise((int)rc, h);
  return rc;
}

// ---- PeerData: the configuration the path reads (PeerData.java) -------------
struct PeerData {
  int64_t _MODEL_SIZE = 0;          // IPLS(..., long model_size)
  int _PARTITIONS = 1;              // -pa
  int _MIN_PARTITIONS = 1;          // -mp
  int Min_Members = 1;              // -n
  bool Indirect_Communication = false;  // -i
  bool Partial_Aggregation = false;     // -aggr
  bool IPNS_Enable = false;             // -IPNS
  bool isSynchronous = true;            // -async
  int Training_time = 0;                // -training
  int port = 0;                         // -p
  bool secure_ipls = false;             // PeerData.java:62 (hard-coded false)
  int device = 0;                       // HIP device ordinal
  std::vector<int32_t> devices;         // several GPUs: the -pa segments sharded over them (cfg.devices)
};

// ---- Middleware (Middleware.java) ------------------------------------------
struct Middleware {
  // parse_arguments (Middleware.java:26-110): required -p -pa -mp -n -i
  // -training -aggr; optional -IPNS -async.  Missing/invalid -> throws
  // IllegalArgumentException (Middleware prints help and exits 1).
  static PeerData parse_arguments(const std::vector<std::string>& args) {
    struct Flag { const char* s; const char* l; bool req; };
    static const Flag flags[] = {{"p", "port_number", true}, {"pa", "partitions", true},
                                 {"mp", "minimum_partitions", true}, {"n", "min_peers", true},
                                 {"i", "indirect_communication", true}, {"training", "training", true},
                                 {"aggr", "partial_aggregation", true}, {"IPNS", "IPNS", false},
                                 {"async", "Async", false}};
    std::map<std::string, std::string> v;
    for (size_t i = 0; i < args.size(); ++i) {
      std::string a = args[i];
      if (a.empty() || a[0] != '-') continue;
      a = a.substr(a.find_first_not_of('-'));
      const Flag* f = nullptr;
      for (const auto& fl : flags)
        if (a == fl.s || a == fl.l) f = &fl;
      if (!f || i + 1 >= args.size()) throw IllegalArgumentException(IPLS_E_INVAL, "Unrecognized option: " + args[i]);
      v[f->s] = args[++i];
    }
    for (const auto& fl : flags)
      if (fl.req && !v.count(fl.s)) throw IllegalArgumentException(IPLS_E_INVAL, std::string("Missing required option: ") + fl.s);
    auto num = [&](const char* k) {
      try {
        size_t pos = 0;
        const int x = std::stoi(v[k], &pos);
        if (pos != v[k].size()) throw std::invalid_argument(k);
        return x;
      } catch (const std::exception&) {
        throw IllegalArgumentException(IPLS_E_INVAL, std::string("NumberFormatException for -") + k);
      }
    };
    PeerData d;
    d.port = num("p");
    d._PARTITIONS = num("pa");
    d._MIN_PARTITIONS = num("mp");
    d.Min_Members = num("n");
    d.Indirect_Communication = num("i") > 0;
    d.Training_time = num("training");
    d.Partial_Aggregation = num("aggr") > 0;
    d.IPNS_Enable = v.count("IPNS") && v["IPNS"] == "true";
    d.isSynchronous = !(v.count("async") && v["async"] == "true");
    return d;
  }

  // Serialize (Middleware.java:164-170): the task-3 writeDouble stream.
  static std::vector<uint8_t> Serialize_wire_from(ipls_agg* h, int64_t model_size) {
    std::vector<uint8_t> out(8 * (size_t)model_size);
    check(ipls_agg_get_partitions(h, out.data(), model_size, IPLS_HOST_BE_CANON), h);
    return out;
  }
};

// ---- MyIPFSClass codecs on the path ---------------------------------------------
struct MyIPFSClass {
  // Marshall_Packet(double[], origin, partition, iteration, pid) before base64
  // (MyIPFSClass.java:990-1017).
  static std::vector<uint8_t> Marshall_Packet(const std::vector<double>& g, const std::string& origin,
                                              int partition, int iteration, int16_t pid) {
    std::vector<uint8_t> out(14 + 8 * g.size() + origin.size());
    check(ipls_frame_encode(g.data(), (int64_t)g.size(), IPLS_HOST_F64, partition, iteration, pid,
                            (const uint8_t*)origin.data(), (int32_t)origin.size(), out.data(), (int64_t)out.size()),
          nullptr);
    return out;
  }
  struct Frame { int16_t pid; int64_t n; int32_t partition, iteration; int64_t payload_off, origin_off; };
  // GET_GRADIENTS header (MyIPFSClass.java:1437-1446) -- the payload is
  // folded on the device, never decoded here.
  static Frame GET_GRADIENTS(const std::vector<uint8_t>& frame) {
    Frame f{};
    f.n = check(ipls_frame_parse(frame.data(), (int64_t)frame.size(), &f.pid, &f.partition, &f.iteration,
                                 &f.payload_off, &f.origin_off),
                nullptr);
    return f;
  }
};

// ---- IPLS: the aggregation methods of IPLS.java ----------------------------------
class IPLS {
 public:
  explicit IPLS(const PeerData& pd, std::vector<int> auth_list = {}) : cfg_(pd), Auth_List(std::move(auth_list)) {
    ipls_agg_cfg c{};
    c.model_size = pd._MODEL_SIZE;
    c.n_partitions = pd._PARTITIONS;
    c.max_peers = pd.Min_Members;
    c.partial_aggregation = pd.Partial_Aggregation;
    c.secure = pd.secure_ipls;
    c.device = pd.device;
    if (!pd.devices.empty()) {
      c.devices = pd.devices.data();
      c.n_devices = (int32_t)pd.devices.size();
    }
    ipls_agg* h = nullptr;
    const int rc = ipls_agg_open(&c, &h);   // init() -> InitializeWeights() (IPLS.java:1860)
    if (rc < 0) raise(rc, nullptr);
    h_.reset(h);
  }
  ipls_agg* handle() const { return h_.get(); }
  int64_t partition_length(int p) const {
    int64_t L = 0;
    check(ipls_agg_partition_len(h_.get(), p, &L), h_.get());
    return L;
  }

  // InitializeWeights(List<Double> Model) -- IPLS.java:1880-1901
  void InitializeWeights(const std::vector<double>& Model) {
    check(ipls_agg_load_model(h_.get(), Model.data(), (int64_t)Model.size(), IPLS_HOST_F64), h_.get());
  }

  // OrganizeGradients -- IPLS.java:1018-1040
  std::map<int, std::vector<double>> OrganizeGradients(const std::vector<double>& Gradients) const {
    std::map<int, std::vector<double>> out;
    for (int p = 0; p < cfg_._PARTITIONS; ++p) {
      std::vector<double> part((size_t)partition_length(p));
      check(ipls_agg_split(h_.get(), Gradients.data(), (int64_t)Gradients.size(), IPLS_HOST_F64, p, part.data(),
                           IPLS_HOST_F64),
            h_.get());
      out.emplace(p, std::move(part));
    }
    return out;
  }

  // UpdateGradient (IPLS.java:1703): the own-partition accumulate of
  // 1737-1743.  nullptr = "did not train in time" (Gradients == null).
  void UpdateGradient(const std::vector<double>* Gradients) {
    if (!Gradients) return;
    check(ipls_agg_update_gradient(h_.get(), Gradients->data(), (int64_t)Gradients->size(), IPLS_HOST_F64,
                                   Auth_List.data(), (int)Auth_List.size()),
          h_.get());
  }

  // Download_Scheduler.download_gradients (:245-268): a bucket another
  // aggregator of Partition will fold, kept in Other_Replica_Gradients.
  // Aggregator is the int the caller maps 1:1 from the aggregator's peer ID;
  // AggregatorId is that ID, whose Pair<>(Partition, AggregatorId).hashCode()
  // fixes the key's place in the HashMap and so the Collect_Replicas order
  // (IPLS.java:1218).
  void Other_Replica_Gradients(int Partition, int32_t Aggregator, const std::string& AggregatorId,
                               const std::vector<double>& gradients) {
    int32_t key_hash = 0;
    check(ipls_java_pair_hash(Partition, (const uint8_t*)AggregatorId.data(), (int64_t)AggregatorId.size(),
                              &key_hash),
          nullptr);
    check(ipls_agg_other_replica_keyed(h_.get(), Partition, Aggregator, key_hash, gradients.data(),
                                       (int64_t)gradients.size(), IPLS_HOST_F64),
          h_.get());
  }

  // Other_Replica_Gradients.remove(new Pair<>(Partition, Aggregator)) and the
  // _Received count (Download_Scheduler.java:215-217, 329-332, 438-440): the
  // aggregator's own partial arrived.  True if the key was stored.
  bool Other_Replica_Gradients_remove(int Partition, int32_t Aggregator) {
    return check(ipls_agg_other_replica_drop(h_.get(), Partition, Aggregator), h_.get()) == 1;
  }

  // Collect_Replicas (IPLS.java:1217-1241): fold every stored array into
  // Replicas_Gradients and clear the store; returns the per-partition
  // increments of PeerData.Participants (received x length per key, :1229-1234).
  std::vector<int32_t> Collect_Replicas() {
    std::vector<int32_t> participants((size_t)cfg_._PARTITIONS);
    check(ipls_agg_collect_replicas(h_.get(), participants.data()), h_.get());
    return participants;
  }

  // AggregatePartition (IPLS.java:1248-1274); returns the update_file bytes
  // commit_update publishes (IPLS_Comm.java:27-37).
  std::vector<uint8_t> AggregatePartition(int Partition) {
    std::vector<uint8_t> file(8 * (size_t)partition_length(Partition));
    check(ipls_agg_finalize(h_.get(), Partition, file.data(), IPLS_HOST_BE, nullptr), h_.get());
    return file;
  }

  // IPLS_Comm.commit_partial_update (IPLS_Comm.java:51-61): the file bytes of
  // new Pair<>(workers, Aggregated_Gradients[Partition]) (ObjectOutputStream).
  std::vector<uint8_t> commit_partial_update(int Partition, int32_t workers) {
    const int64_t n = ipls_agg_commit_partial(h_.get(), Partition, workers, nullptr, 0);
    if (n < 0) raise((int)n, h_.get());
    std::vector<uint8_t> out((size_t)n);
    const int64_t m = ipls_agg_commit_partial(h_.get(), Partition, workers, out.data(), n);
    if (m < 0) raise((int)m, h_.get());
    return out;
  }

  // Wait_Client_Gradients' publish loop (IPLS.java:1423-1431, direct
  // communication): for every partition i of Auth_List, ipfsClass.send(topic,
  // Marshall_Packet(Aggregated_Gradients[i], id, middleware_iteration,
  // workers[i].size() + 1, 3)) -- the texts, encoded on the GPU in one launch
  // per device, in Auth_List order.
  std::vector<std::string> Send_Partial_Updates(int32_t middleware_iteration,
                                                const std::vector<int32_t>& workers_plus_one,
                                                const std::string& id) {
    const int n = (int)Auth_List.size();
    if ((int)workers_plus_one.size() != n) throw IllegalArgumentException(IPLS_E_INVAL, "one workers count per partition");
    std::vector<int64_t> lens((size_t)std::max(1, n)), offs((size_t)std::max(1, n));
    const int64_t total = ipls_agg_publish_partials(h_.get(), Auth_List.data(), n, IPLS_TGT_AGG,
                                                    middleware_iteration, workers_plus_one.data(), 3,
                                                    (const uint8_t*)id.data(), (int32_t)id.size(), nullptr, 0,
                                                    IPLS_HOST_TEXT, lens.data(), offs.data());
    if (total < 0) raise((int)total, h_.get());
    std::string buf((size_t)std::max<int64_t>(1, total), '\0');
    const int64_t rc = ipls_agg_publish_partials(h_.get(), Auth_List.data(), n, IPLS_TGT_AGG, middleware_iteration,
                                                 workers_plus_one.data(), 3, (const uint8_t*)id.data(),
                                                 (int32_t)id.size(), buf.data(), total, IPLS_HOST_TEXT, nullptr,
                                                 nullptr);
    if (rc < 0) raise((int)rc, h_.get());
    std::vector<std::string> out;
    for (int i = 0; i < n; ++i) out.push_back(buf.substr((size_t)offs[i], (size_t)lens[i]));
    return out;
  }

  // Tail of Update_Client_WaitAck_List (IPLS.java:1556-1562): for p in
  // Auth_List, Aggregated_Gradients[p] = from_future[p], from_future[p] = 0.
  void Update_Client_WaitAck_List() {
    check(ipls_agg_promote_future(h_.get(), Auth_List.data(), (int)Auth_List.size()), h_.get());
  }

  // Download_Scheduler.cache_partition (:752-754): Weight_Address[p] = GetParameters(hash)
  void cache_partition(int Partition, const std::vector<uint8_t>& file_bytes) {
    check(ipls_agg_set_weights(h_.get(), Partition, file_bytes.data(), (int64_t)file_bytes.size() / 8, IPLS_HOST_BE),
          h_.get());
  }

  // AggregatePartition for every partition + GetPartitions, fused
  // (ipls_agg_aggregate_round with no further buckets).
  std::vector<double> AggregateRound() {
    std::vector<double> out((size_t)cfg_._MODEL_SIZE);
    check(ipls_agg_aggregate_round(h_.get(), 0, cfg_._PARTITIONS, nullptr, 0, IPLS_DEV_F64, out.data(),
                                   IPLS_HOST_F64),
          h_.get());
    return out;
  }

  // GetPartitions (IPLS.java:1080-1178), the synchronous steady-state branch.
  std::vector<double> GetPartitions() const {
    std::vector<double> out((size_t)cfg_._MODEL_SIZE);
    check(ipls_agg_get_partitions(h_.get(), out.data(), (int64_t)out.size(), IPLS_HOST_F64), h_.get());
    return out;
  }

  const PeerData& peer_data() const { return cfg_; }

 private:
  struct Closer {
    void operator()(ipls_agg* h) const { ipls_agg_close(h); }
  };
  PeerData cfg_;
  std::unique_ptr<ipls_agg, Closer> h_;

 public:
  std::vector<int32_t> Auth_List;   // PeerData.Auth_List: partitions this peer aggregates
};

// ---- Updater (Updater.java) -----------------------------------------------------
class Updater {
 public:
  explicit Updater(IPLS& ipls) : ipls_(ipls) {}
  // _Update(double[] Gradient, int Partition, List<String> Origin, int
  // iteration, boolean from_clients) -- the synchronous folds
  // (Updater.java:40-44 replicas, 115-117 clients).
  void _Update(const std::vector<double>* Gradient, int Partiton, bool from_clients) {
    if (!Gradient) return;   // `&& Gradient != null` in every loop
    check(ipls_agg_accumulate(ipls_.handle(), Partiton, from_clients ? IPLS_TGT_AGG : IPLS_TGT_REP,
                              Gradient->data(), (int64_t)Gradient->size(), IPLS_HOST_F64),
          ipls_.handle());
  }
  // run(): a queue item with a hash and no payload -- GetParameters(hash,
  // Gradient_Buff) then _Update (Updater.java:176-187).  The BE decode is
  // fused into the device fold.
  // Like Java, the bytes go through the one reusable Gradient_Buff.
  void _Update_from_file(const std::vector<uint8_t>& ipfs_cat_bytes, int Partiton, bool from_clients) {
    check(ipls_agg_update_indirect(ipls_.handle(), Partiton, from_clients ? IPLS_TGT_AGG : IPLS_TGT_REP,
                                   ipfs_cat_bytes.data(), (int64_t)ipfs_cat_bytes.size()),
          ipls_.handle());
  }
  // The "gradients from the future" branch (Updater.java:91-101): a client's
  // bucket for a later iteration folds into Aggregated_Gradients_from_future.
  void _Update_from_future(const std::vector<double>* Gradient, int Partiton) {
    if (!Gradient) return;
    check(ipls_agg_accumulate(ipls_.handle(), Partiton, IPLS_TGT_FUTURE, Gradient->data(),
                              (int64_t)Gradient->size(), IPLS_HOST_F64),
          ipls_.handle());
  }
  // Download_Scheduler.java:324: a replica's Pair<Integer,double[]> partial
  // update (Download_Partial_Updates) queued with from_clients = false.
  void _Update_from_partial(const std::vector<uint8_t>& pair_file, int Partiton) {
    check(ipls_agg_accumulate(ipls_.handle(), Partiton, IPLS_TGT_REP, pair_file.data(), (int64_t)pair_file.size(),
                              IPLS_HOST_PAIR),
          ipls_.handle());
  }
  // ThreadReceiver pid 3 -> queue -> _Update (IPLS.java:453-465): a decoded frame.
  void _Update_from_frame(const std::vector<uint8_t>& frame, int Partiton, bool from_clients) {
    check(ipls_agg_accumulate(ipls_.handle(), Partiton, from_clients ? IPLS_TGT_AGG : IPLS_TGT_REP, frame.data(),
                              (int64_t)frame.size(), IPLS_HOST_FRAME),
          ipls_.handle());
  }

 private:
  IPLS& ipls_;
};

// ---- Updater.run (Updater.java:155-216): the reducer thread ----------------------
// One consumer drains the request queue (PeerData.queue, PeerData.java:117) in
// arrival order: a request with a payload folds through _Update; a hash-only
// request reads the `ipfs cat` bytes into the one Gradient_Buff and folds that
// (Updater.java:176-187).  Device-resident payloads are queued on the handle
// (ipls_agg_accumulate_async), so a burst of arrivals folds in one launch per
// partition.  Producers (ThreadReceiver, GGP_Receiver, Download_Scheduler) call
// put() from any thread; the daemon calls drain() before AggregatePartition.
// Java's thread dies on the first exception (the catch sits outside
// while(true), :168-215); here the request is dropped, its exception message
// kept in failures(), and the loop goes on.
class UpdaterThread {
 public:
  // Sextet<origins, partition, iteration, from_clients, double[], hash>
  struct Request {
    int partition = 0;
    bool from_clients = true;
    std::vector<double> gradient;   // value4 (the payload); empty and no file/device -> null, no fold
    std::vector<uint8_t> file;      // a hash-only request: the `ipfs cat` bytes of value5
    const void* device = nullptr;   // or a device-resident bucket, kept alive by the caller until drain()
    int64_t device_n = 0;
    bool device_big_endian = false;
    std::string origin;             // value0: the sending peer (a client's request clears its Client_Wait_Ack)
  };

  // idle_flush: when no request arrives for this long, the queued device
  // buckets are folded (ipls_agg_flush) instead of waiting for the queues to fill.
  explicit UpdaterThread(IPLS& ipls, std::chrono::microseconds idle_flush = std::chrono::microseconds(200))
      : ipls_(ipls), idle_flush_(idle_flush), th_([this] { loop(); }) {}
  ~UpdaterThread() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  UpdaterThread(const UpdaterThread&) = delete;
  UpdaterThread& operator=(const UpdaterThread&) = delete;

  // PeerData.queue.put
  void put(Request r) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(r));
      ++put_n_;
    }
    cv_.notify_one();
  }
  // Block until every request put so far has been folded on the device.
  void drain() {
    std::unique_lock<std::mutex> lk(mu_);
    idle_.wait(lk, [this] { return done_n_ == put_n_; });
    lk.unlock();
    check(ipls_agg_sync(ipls_.handle()), ipls_.handle());   // folds queued device buckets, waits
  }
  std::vector<std::string> failures() {
    std::lock_guard<std::mutex> lk(mu_);
    return failures_;
  }

  // The round's PeerData.Client_Wait_Ack: the trainers this aggregator
  // waits for (IPLS.java:1402-1404 spins until the list is empty).  The
  // request that clears the last one is the flush hint: the queued device
  // folds start at once instead of after the idle timeout or at the daemon's
  // AggregatePartition.
  void Client_Wait_Ack(std::set<std::string> peers) {
    std::lock_guard<std::mutex> lk(mu_);
    wait_ack_ = std::move(peers);
  }
  // Wait_Client_Gradients (IPLS.java:1402-1404): block until every expected
  // trainer's request has been taken by the Updater.
  void Wait_Client_Gradients() {
    std::unique_lock<std::mutex> lk(mu_);
    idle_.wait(lk, [this] { return wait_ack_.empty(); });
  }
  uint64_t hint_flushes() {
    std::lock_guard<std::mutex> lk(mu_);
    return hint_flushes_;
  }

 private:
  void loop() {
    Updater u(ipls_);
    for (;;) {
      Request r;
      {
        std::unique_lock<std::mutex> lk(mu_);
        auto ready = [this] { return stop_ || !q_.empty(); };
        if (!cv_.wait_for(lk, idle_flush_, ready)) {
          if (queued_) {   // the queue ran dry: start the queued folds
            queued_ = false;
            lk.unlock();
            const int rc = ipls_agg_flush(ipls_.handle());
            lk.lock();
            if (rc < 0) failures_.push_back(ipls_agg_last_error(nullptr));
          }
          cv_.wait(lk, ready);
        }
        if (q_.empty()) return;   // stop_ and nothing left
        r = std::move(q_.front());
        q_.pop_front();
      }
      bool hint = false;
      try {
        if (r.device) {
          uint64_t t = 0;
          check(ipls_agg_accumulate_async(ipls_.handle(), r.partition, r.from_clients ? IPLS_TGT_AGG : IPLS_TGT_REP,
                                          r.device, r.device_n, r.device_big_endian ? IPLS_DEV_BE : IPLS_DEV_F64, &t),
                ipls_.handle());
          std::lock_guard<std::mutex> lk(mu_);
          queued_ = true;
        } else if (!r.gradient.empty()) {
          u._Update(&r.gradient, r.partition, r.from_clients);
        } else if (!r.file.empty()) {
          u._Update_from_file(r.file, r.partition, r.from_clients);
        }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(mu_);
        failures_.push_back(e.what());
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (r.from_clients && !wait_ack_.empty() && wait_ack_.erase(r.origin) && wait_ack_.empty() && queued_) {
          hint = true;   // Client_Wait_Ack drained: every expected bucket of the round is queued
          queued_ = false;
        }
      }
      if (hint) {
        const int rc = ipls_agg_flush(ipls_.handle());
        std::lock_guard<std::mutex> lk(mu_);
        ++hint_flushes_;
        if (rc < 0) failures_.push_back(ipls_agg_last_error(nullptr));
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        ++done_n_;
      }
      idle_.notify_all();
    }
  }

  IPLS& ipls_;
  std::chrono::microseconds idle_flush_;
  std::mutex mu_;
  std::condition_variable cv_, idle_;
  std::deque<Request> q_;
  bool stop_ = false, queued_ = false;
  uint64_t put_n_ = 0, done_n_ = 0, hint_flushes_ = 0;
  std::set<std::string> wait_ack_;
  std::vector<std::string> failures_;
  std::thread th_;   // last: starts after every member above exists
};

// ---- Decentralized_Storage_Receiver (storage node, -aggr 1) ----------------------
// The merge of the files one request names (Decentralized_Storage_Receiver.java:
// 239-258): status 0 -> raw gradient files, otherwise Pair partial updates;
// returns the `<p>_partial_aggregation` file bytes.
class Decentralized_Storage_Receiver {
 public:
  explicit Decentralized_Storage_Receiver(IPLS& node) : node_(node) {}
  std::vector<uint8_t> merge(const std::vector<std::vector<uint8_t>>& files, int status) {
    std::vector<const uint8_t*> ptrs;
    std::vector<int64_t> lens;
    for (const auto& f : files) ptrs.push_back(f.data()), lens.push_back((int64_t)f.size());
    const int kind = status == 0 ? IPLS_HOST_BE : IPLS_HOST_PAIR;
    int64_t cap = files.empty() ? 0 : (int64_t)(files[0].size() / 8) * 8;
    if (status != 0 && !files.empty()) {
      int32_t w;
      int64_t off;
      const int64_t n0 = ipls_pair_parse(files[0].data(), (int64_t)files[0].size(), &w, &off);
      if (n0 < 0) raise((int)n0, nullptr);
      cap = 8 * n0;
    }
    std::vector<uint8_t> out((size_t)std::max<int64_t>(cap, 1));
    const int64_t nb = ipls_agg_merge_files(node_.handle(), ptrs.data(), lens.data(), (int)files.size(), kind,
                                            out.data(), cap);
    if (nb < 0) raise((int)nb, node_.handle());
    out.resize((size_t)nb);
    return out;
  }

 private:
  IPLS& node_;
};

// ---- Light_IPLS_Daemon (Light_IPLS_Daemon.java) -----------------------------------
// The blocking API pair the Middleware calls.  One round here = the daemon
// loop's UpdateGradient for this peer's own partitions, the arrivals the
// Updater folded, then AggregatePartition for Auth_List and GetPartitions.
class Light_IPLS_Daemon {
 public:
  explicit Light_IPLS_Daemon(IPLS& ipls) : ipls_(ipls) {}
  void UpdateModel(const std::vector<double>& Gradients) { ipls_.UpdateGradient(&Gradients); }
  std::vector<double> Get_Partitions() {
    // Responsible for every partition: AggregatePartition for all of them and
    // the divide are one fused launch (the update_file bytes are not needed here).
    std::vector<int> sorted = ipls_.Auth_List;
    std::sort(sorted.begin(), sorted.end());
    bool all = (int)sorted.size() == ipls_.peer_data()._PARTITIONS;
    for (int i = 0; all && i < (int)sorted.size(); ++i) all = sorted[i] == i;
    if (all) return ipls_.AggregateRound();
    for (int p : ipls_.Auth_List) ipls_.AggregatePartition(p);
    return ipls_.GetPartitions();
  }

 private:
  IPLS& ipls_;
};

}  // namespace ipls_host
