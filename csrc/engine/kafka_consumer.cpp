// Native Kafka consumer: Metadata v1 -> one TCP connection per partition leader ->
// Fetch v4 -> RecordBatch v2 (CRC-32C checked; uncompressed or gzip) -> rows written
// straight into the engine's pinned partition rings (SURVEY.md §2.4 H1 "C++ Kafka ingest ...
// writes directly into ring slots").
//
// One consumer thread per rank serves that rank's partitions of one topic.  Each round it
// sends one Fetch to EVERY leader broker first and then reads the responses, so brokers
// serve in parallel (the reference's consumers dial the 3-broker service,
// deploy/router.yaml:55-56, deploy/frauddetection_cr.yaml:75-77).  Partition errors:
//   NOT_LEADER_FOR_PARTITION / UNKNOWN_TOPIC_OR_PARTITION / LEADER_NOT_AVAILABLE /
//   REPLICA_NOT_AVAILABLE, or a dead connection -> metadata refresh, reconnect, continue
//   from the same offset (nothing skipped, nothing duplicated downstream);
//   OFFSET_OUT_OF_RANGE -> ListOffsets reset per policy (earliest / latest / none = stop
//   the partition and report);
//   anything else -> counted and reported through ccfd_kc_last_error (never silently).
// Each record value is either a TXB1 columnar batch (contracts/transaction.py: ids,
// customers and f32 rows are copied / W64-encoded row-block by row-block) or one JSON
// transaction (parsed by the native parser, ingest.cpp).  Offsets: after the rows of a
// record are committed to the ring, (ring rows written, next offset) is queued;
// ccfd_kc_committable() returns the highest offset whose rows the engine has already
// released (scored), so the caller commits consumer-group offsets only for scored data
// (at-least-once).
//
// Sinks: an engine ring (production) or a flat array (tests; no GPU needed).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../include/ccfd_abi.h"
#include "binenc.h"

extern "C" uint32_t ccfd_crc32c(const void* data, size_t n, uint32_t seed);

namespace ccfd {
void set_error(const std::string& e);
bool parse_json_row(const char* s, const char* e, float* f, uint64_t* id, uint32_t* cust);
void encode_w64_row(const float* x, uint8_t* out);
void encode_bins_row(const BinPlan& plan, const float* x, uint8_t* out);
void encode_bins_rows(const BinPlan& plan, const float* x, int64_t n, int64_t ld, uint8_t* out, float* amount_out);
bool g32_table_ok(const float* edges, const int32_t* offsets, int32_t stamp);
bool g20_table_ok(const float* edges, const int32_t* offsets, int32_t stamp);
}  // namespace ccfd

namespace {

// ---------------------------------------------------------------- big-endian buffer I/O
struct Out {
  std::vector<uint8_t> b;
  void i8(int8_t v) { b.push_back((uint8_t)v); }
  void i16(int16_t v) { uint16_t x = htons((uint16_t)v); put(&x, 2); }
  void i32(int32_t v) { uint32_t x = htonl((uint32_t)v); put(&x, 4); }
  void i64(int64_t v) { i32((int32_t)((uint64_t)v >> 32)); i32((int32_t)(uint32_t)v); }
  void str(const std::string& s) { i16((int16_t)s.size()); put(s.data(), s.size()); }
  void put(const void* p, size_t n) { const uint8_t* c = (const uint8_t*)p; b.insert(b.end(), c, c + n); }
};

struct In {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  bool need(size_t n) { if ((size_t)(e - p) < n) { ok = false; return false; } return true; }
  int8_t i8() { if (!need(1)) return 0; return (int8_t)*p++; }
  int16_t i16() { if (!need(2)) return 0; uint16_t x; std::memcpy(&x, p, 2); p += 2; return (int16_t)ntohs(x); }
  int32_t i32() { if (!need(4)) return 0; uint32_t x; std::memcpy(&x, p, 4); p += 4; return (int32_t)ntohl(x); }
  uint32_t u32() { return (uint32_t)i32(); }
  int64_t i64() { uint64_t hi = (uint32_t)i32(); uint64_t lo = (uint32_t)i32(); return (int64_t)((hi << 32) | lo); }
  void skip(size_t n) { if (need(n)) p += n; }
  int64_t varlong() {           // zig-zag varint
    uint64_t v = 0;
    int sh = 0;
    while (ok) {
      if (!need(1)) return 0;
      const uint8_t c = *p++;
      v |= (uint64_t)(c & 0x7F) << sh;
      if (!(c & 0x80)) break;
      sh += 7;
      if (sh > 63) { ok = false; return 0; }
    }
    return (int64_t)((v >> 1) ^ (~(v & 1) + 1));
  }
};

// ---------------------------------------------------------------- sinks
struct Sink {
  // ring-like contiguous acquire/commit of rows of a partition
  virtual int64_t acquire(int p, int64_t want, int64_t* row) = 0;
  // origin_ns: producer send time of these rows on the engine's steady clock (0 = unknown)
  virtual void commit(int p, int64_t n, int64_t origin_ns) = 0;
  virtual uint8_t* feats(int p) = 0;
  virtual uint64_t* ids(int p) = 0;
  virtual uint32_t* cust(int p) = 0;
  virtual float* amount(int p) = 0;         // G32: host-side Amount column (may be NULL)
  virtual int64_t released(int p) = 0;      // rows consumed downstream (for offset commits)
  virtual ~Sink() = default;
};

struct EngineSink : Sink {
  void* eng;
  std::vector<ccfd_kc_partition> parts;
  int64_t acquire(int p, int64_t want, int64_t* row) override {
    return ccfd_engine_ring_acquire(eng, parts[p].engine_partition, want, row);
  }
  void commit(int p, int64_t n, int64_t origin_ns) override {
    ccfd_engine_ring_commit_at(eng, parts[p].engine_partition, n, origin_ns);
  }
  uint8_t* feats(int p) override { return (uint8_t*)parts[p].feats; }
  uint64_t* ids(int p) override { return parts[p].ids; }
  uint32_t* cust(int p) override { return parts[p].customer; }
  float* amount(int p) override { return parts[p].amount; }
  int64_t released(int p) override { return ccfd_engine_cursor(eng, parts[p].engine_partition); }
};

struct ArraySink : Sink {                  // tests: flat arrays, no wrap, "released" = written
  std::vector<ccfd_kc_partition> parts;
  std::vector<int64_t> used;
  int64_t acquire(int p, int64_t want, int64_t* row) override {
    const int64_t k = std::min<int64_t>(want, parts[p].capacity - used[p]);
    *row = used[p];
    return k;
  }
  void commit(int p, int64_t n, int64_t origin_ns) override {
    used[p] += n;
    last_origin = origin_ns;
  }
  int64_t last_origin = 0;
  uint8_t* feats(int p) override { return (uint8_t*)parts[p].feats; }
  uint64_t* ids(int p) override { return parts[p].ids; }
  uint32_t* cust(int p) override { return parts[p].customer; }
  float* amount(int p) override { return parts[p].amount; }
  int64_t released(int p) override { return used[p]; }
};

struct PState {
  int32_t kafka_partition = 0;
  int64_t next_offset = 0;
  int64_t rows_in = 0;
  int32_t leader = -1;          // broker node id (-1: unknown -> metadata refresh)
  bool stopped = false;         // OFFSET_OUT_OF_RANGE under policy "none"
  bool reset = false;           // OFFSET_OUT_OF_RANGE seen: ListOffsets before the next fetch
  std::deque<std::pair<int64_t, int64_t>> pending;   // (rows_in after record, next offset)
};

// Kafka error codes handled by the consumer
constexpr int16_t kErrOffsetOutOfRange = 1, kErrUnknownTopicOrPartition = 3, kErrLeaderNotAvailable = 5,
                  kErrNotLeader = 6, kErrReplicaNotAvailable = 9;

struct Conn {                   // one broker connection
  std::string host;
  int port = 0;
  int fd = -1;
  int32_t corr = 0;
  int32_t expect = 0;           // correlation id of the request in flight (0: none)
};

class Consumer {
 public:
  std::vector<std::pair<std::string, int>> seeds;   // bootstrap list
  std::string topic, client = "ccfd-native";
  int wire = 0;                 // sink row format: 0 = f32[30], 1 = W64, 2 = G32, 3 = G20
  ccfd::BinPlan bins;                               // G32 / G20 bin table (ccfd_kc_set_bins), SIMD plan
  std::vector<float> scratch;                       // aligned copy of a TXB1 block being binned
  int32_t g32_stamp = 0;
  int reset_policy = CCFD_KC_RESET_EARLIEST;
  Sink* sink = nullptr;
  std::vector<PState> ps;
  std::mutex mu;                // guards ps[*].pending / next_offset / last_err reads from other threads
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> n_records{0}, n_rows{0}, n_bytes{0}, n_errors{0}, n_fetches{0};
  std::atomic<uint64_t> n_meta{0}, n_resets{0}, n_leaders{0};
  std::atomic<uint64_t> t_io{0}, t_handle{0}, t_encode{0}, t_ring_wait{0};   // ns, see ccfd_kc_stats
  // producer send time of the batch being ingested, on the steady clock: from the ccfd-ts
  // header of its first record (ingest/kafka_wire.py with_produce_time), 0 when absent
  int64_t cur_origin = 0;
  // send -> the fetch response carrying the batch was received (broker + network + fetch
  // wait), ns, 4 buckets per octave: splits the engine's produce -> scored into the broker
  // side and parse (including earlier batches of the same response) + ring + scoring
  std::atomic<uint64_t> fetch_age_hist[256] = {};
  int64_t fetch_real = 0;                           // wall clock the current response arrived
  static int64_t real_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch())
        .count();
  }
  static int64_t mono_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  std::thread th;
  std::map<int32_t, Conn> brokers;                  // node id -> connection
  bool meta_stale = true;
  int max_wait_ms = 5;
  std::string last_err;
  std::vector<uint8_t> inflated;                    // gzip scratch (consumer thread only)

  ~Consumer() {
    stop.store(true);
    if (th.joinable()) th.join();
    for (auto& kv : brokers) if (kv.second.fd >= 0) ::close(kv.second.fd);
    delete sink;
  }

  void error(const std::string& e) {
    n_errors.fetch_add(1);
    std::lock_guard<std::mutex> lk(mu);
    last_err = e;
  }

  static int dial(const std::string& host, int port) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) return -1;
    int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
    if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) != 0) { ::close(fd); fd = -1; }
    freeaddrinfo(res);
    if (fd < 0) return -1;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int rcv = 8 << 20;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &rcv, sizeof(rcv));
    timeval tv{5, 0};                                // a broker that stops answering is a dead broker
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    return fd;
  }

  static bool send_all(int fd, const uint8_t* p, size_t n) {
    while (n) {
      const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
      if (k <= 0) return false;
      p += k;
      n -= (size_t)k;
    }
    return true;
  }
  static bool recv_all(int fd, uint8_t* p, size_t n) {
    while (n) {
      const ssize_t k = ::recv(fd, p, n, 0);
      if (k <= 0) return false;
      p += k;
      n -= (size_t)k;
    }
    return true;
  }

  // frame = [size][api key][version][corr][client id][body]
  bool send_request(Conn& c, int16_t api, int16_t ver, const Out& body) {
    Out h;
    h.i16(api);
    h.i16(ver);
    h.i32(++c.corr);
    h.str(client);
    Out frame;
    frame.i32((int32_t)(h.b.size() + body.b.size()));
    frame.put(h.b.data(), h.b.size());
    frame.put(body.b.data(), body.b.size());
    c.expect = c.corr;
    return send_all(c.fd, frame.b.data(), frame.b.size());
  }
  // response body after the correlation id
  bool recv_response(Conn& c, std::vector<uint8_t>& resp) {
    uint8_t hdr[4];
    if (!recv_all(c.fd, hdr, 4)) return false;
    uint32_t len;
    std::memcpy(&len, hdr, 4);
    len = ntohl(len);
    if (len < 4 || len > (1u << 30)) return false;
    resp.resize(len);
    if (!recv_all(c.fd, resp.data(), len)) return false;
    int32_t corr;
    std::memcpy(&corr, resp.data(), 4);
    if ((int32_t)ntohl((uint32_t)corr) != c.expect) return false;
    c.expect = 0;
    resp.erase(resp.begin(), resp.begin() + 4);
    return true;
  }
  void close_conn(Conn& c) {
    if (c.fd >= 0) ::close(c.fd);
    c.fd = -1;
    c.expect = 0;
  }

  // Metadata v1 for our topic from any reachable broker (known brokers first, then seeds):
  // broker table + the leader of every partition we consume.
  bool refresh_metadata() {
    n_meta.fetch_add(1, std::memory_order_relaxed);
    std::vector<std::pair<std::string, int>> cands;
    for (auto& kv : brokers) cands.emplace_back(kv.second.host, kv.second.port);
    for (auto& sd : seeds) cands.push_back(sd);
    Out body;
    body.i32(1);
    body.str(topic);
    std::vector<uint8_t> resp;
    for (auto& hp : cands) {
      Conn c;
      c.host = hp.first;
      c.port = hp.second;
      c.fd = dial(c.host, c.port);
      if (c.fd < 0) continue;
      const bool ok = send_request(c, 3, 1, body) && recv_response(c, resp);
      close_conn(c);
      if (!ok) continue;
      In in{resp.data(), resp.data() + resp.size()};
      std::map<int32_t, std::pair<std::string, int>> nodes;
      const int32_t nb = in.i32();
      for (int32_t i = 0; i < nb && in.ok; ++i) {
        const int32_t id = in.i32();
        const int16_t hl = in.i16();
        std::string h;
        if (hl > 0 && in.need((size_t)hl)) { h.assign((const char*)in.p, (size_t)hl); in.p += hl; }
        const int32_t port = in.i32();
        const int16_t rl = in.i16();
        if (rl > 0) in.skip((size_t)rl);
        nodes[id] = {h, port};
      }
      in.i32();                                       // controller
      const int32_t nt = in.i32();
      std::map<int32_t, int32_t> leader;              // partition -> node
      bool topic_ok = false;
      for (int32_t t = 0; t < nt && in.ok; ++t) {
        const int16_t terr = in.i16();
        const int16_t sl = in.i16();
        std::string name;
        if (sl > 0 && in.need((size_t)sl)) { name.assign((const char*)in.p, (size_t)sl); in.p += sl; }
        in.i8();                                      // internal
        const int32_t np = in.i32();
        for (int32_t q = 0; q < np && in.ok; ++q) {
          const int16_t perr = in.i16();
          const int32_t idx = in.i32();
          const int32_t lead = in.i32();
          const int32_t nr = in.i32();
          for (int32_t k = 0; k < nr && in.ok; ++k) in.i32();
          const int32_t ni = in.i32();
          for (int32_t k = 0; k < ni && in.ok; ++k) in.i32();
          if (name == topic && perr == 0) leader[idx] = lead;
        }
        if (name == topic && terr == 0) topic_ok = true;
      }
      if (!in.ok) continue;
      if (!topic_ok) { error("metadata: topic " + topic + " unavailable"); return false; }
      // reconnect only brokers whose address changed or that disappeared
      for (auto it = brokers.begin(); it != brokers.end();) {
        auto nd = nodes.find(it->first);
        if (nd == nodes.end() || nd->second.first != it->second.host || nd->second.second != it->second.port) {
          close_conn(it->second);
          it = brokers.erase(it);
        } else {
          ++it;
        }
      }
      for (auto& kv : nodes)
        if (!brokers.count(kv.first)) { Conn c2; c2.host = kv.second.first; c2.port = kv.second.second; brokers[kv.first] = c2; }
      bool all = true;
      for (auto& s : ps) {
        auto l = leader.find(s.kafka_partition);
        s.leader = (l != leader.end() && brokers.count(l->second)) ? l->second : -1;
        all = all && s.leader >= 0;
      }
      meta_stale = !all;                              // a leaderless partition: ask again soon
      return true;
    }
    error("metadata: no broker reachable");
    return false;
  }

  Conn* leader_conn(int32_t node) {
    auto it = brokers.find(node);
    if (it == brokers.end()) return nullptr;
    Conn& c = it->second;
    if (c.fd < 0) c.fd = dial(c.host, c.port);
    return c.fd >= 0 ? &c : nullptr;
  }

  // Fetch v4 for this leader's partitions
  // wait_ms: the broker holds an empty fetch this long for data (long poll).  Only used when
  // every partition of this thread has one leader: responses are read in send order, so a
  // long-polling leader would delay another leader's data
  Out fetch_body(const std::vector<int>& pis, int wait_ms) {
    Out body;
    body.i32(-1);           // replica id
    body.i32(wait_ms);
    body.i32(1);            // min bytes
    body.i32(64 << 20);     // max bytes
    body.i8(0);             // isolation: read uncommitted
    body.i32(1);            // one topic
    body.str(topic);
    std::lock_guard<std::mutex> lk(mu);
    body.i32((int32_t)pis.size());
    for (int pi : pis) {
      body.i32(ps[pi].kafka_partition);
      body.i64(ps[pi].next_offset);
      body.i32(16 << 20);
    }
    return body;
  }

  // ListOffsets v1 on the partition's leader: earliest (-2) or latest (-1)
  bool reset_offset(int pi) {
    PState& s = ps[pi];
    Conn* c = leader_conn(s.leader);
    if (!c) { meta_stale = true; return false; }
    Out body;
    body.i32(-1);
    body.i32(1);
    body.str(topic);
    body.i32(1);
    body.i32(s.kafka_partition);
    body.i64(reset_policy == CCFD_KC_RESET_LATEST ? -1 : -2);
    std::vector<uint8_t> resp;
    if (!send_request(*c, 2, 1, body) || !recv_response(*c, resp)) { close_conn(*c); meta_stale = true; return false; }
    In in{resp.data(), resp.data() + resp.size()};
    in.i32();
    const int16_t sl = in.i16();
    in.skip(sl > 0 ? (size_t)sl : 0);
    in.i32();
    in.i32();                                         // partition
    const int16_t err = in.i16();
    in.i64();                                         // timestamp
    const int64_t off = in.i64();
    if (!in.ok || err != 0) {
      if (err == kErrNotLeader || err == kErrUnknownTopicOrPartition || err == kErrLeaderNotAvailable) meta_stale = true;
      else error("list offsets error " + std::to_string(err) + " on partition " + std::to_string(s.kafka_partition));
      return false;
    }
    std::lock_guard<std::mutex> lk(mu);
    s.next_offset = off;
    s.reset = false;
    n_resets.fetch_add(1);
    return true;
  }

  // ring write of n rows given per-row writer; handles wrap + back-pressure
  template <class RowFn>
  bool write_rows(int pi, int64_t n, RowFn&& fn) {
    int64_t done = 0;
    while (done < n) {
      int64_t row = 0;
      const int64_t k = sink->acquire(pi, n - done, &row);
      if (k < 0) return false;
      if (k == 0) {                                   // ring full: wait for the engine
        if (stop.load(std::memory_order_relaxed)) return false;
        const int64_t tw = mono_ns();
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        t_ring_wait.fetch_add((uint64_t)(mono_ns() - tw), std::memory_order_relaxed);
        continue;
      }
      const int64_t te = mono_ns();
      fn(row, done, k);
      t_encode.fetch_add((uint64_t)(mono_ns() - te), std::memory_order_relaxed);
      sink->commit(pi, k, cur_origin);
      done += k;
    }
    return true;
  }

  int row_bytes() const {
    return wire == 3 ? CCFD_G20_ROW_BYTES : wire == 2 ? CCFD_G32_ROW_BYTES : wire ? CCFD_WIRE_ROW_BYTES
                                                                                : CCFD_N_FEATURES * 4;
  }

  // one canonical f32 row into the sink's row format at ring row `row`
  void put_row(int pi, const float* x, uint8_t* dst, int64_t row) {
    if (wire >= 2) {
      ccfd::encode_bins_row(bins, x, dst);
      if (float* am = sink->amount(pi)) am[row] = x[CCFD_N_FEATURES - 1];
    } else if (wire) {
      ccfd::encode_w64_row(x, dst);
    } else {
      std::memcpy(dst, x, CCFD_N_FEATURES * sizeof(float));
    }
  }

  bool ingest_value(int pi, const uint8_t* v, int32_t vlen, int64_t* rows_out) {
    *rows_out = 0;
    if (vlen >= 32 && std::memcmp(v, "TXB1", 4) == 0) {
      uint32_t n, nf;
      std::memcpy(&n, v + 8, 4);
      std::memcpy(&nf, v + 12, 4);
      if (nf != CCFD_N_FEATURES) return false;
      const size_t off_ids = 32, off_cu = off_ids + 8ull * n;
      const size_t off_f = (off_cu + 4ull * n + 15) & ~(size_t)15;
      if (off_f + 120ull * n > (size_t)vlen) return false;
      const uint8_t* ids = v + off_ids;
      const uint8_t* cu = v + off_cu;
      // 16-B aligned within the TXB1 value, but the value itself sits at an arbitrary offset
      // of the fetch buffer: address rows as bytes (UBSan caught the typed-pointer version)
      const uint8_t* f = v + off_f;
      constexpr size_t kRow = CCFD_N_FEATURES * sizeof(float);
      const int rb = row_bytes();
      const bool ok = write_rows(pi, n, [&](int64_t row, int64_t s, int64_t k) {
        std::memcpy(sink->ids(pi) + row, ids + 8 * s, 8 * k);
        std::memcpy(sink->cust(pi) + row, cu + 4 * s, 4 * k);
        uint8_t* dst = sink->feats(pi) + row * rb;
        if (wire >= 2) {
          // binned rows: the block goes through the SIMD plan (16 rows at a time with
          // AVX-512) from an aligned copy (the value sits at any offset of the fetch buffer)
          scratch.resize((size_t)k * CCFD_N_FEATURES);
          std::memcpy(scratch.data(), f + (size_t)s * kRow, (size_t)k * kRow);
          float* am = sink->amount(pi);
          ccfd::encode_bins_rows(bins, scratch.data(), k, CCFD_N_FEATURES, dst, am ? am + row : nullptr);
        } else if (wire) {
          float tmp[CCFD_N_FEATURES];
          for (int64_t i = 0; i < k; ++i) {
            std::memcpy(tmp, f + (size_t)(s + i) * kRow, sizeof(tmp));
            put_row(pi, tmp, dst + i * rb, row + i);
          }
        } else {
          std::memcpy(dst, f + (size_t)s * kRow, (size_t)k * rb);
        }
      });
      *rows_out = ok ? n : 0;
      return ok;
    }
    // one JSON transaction
    float x[CCFD_N_FEATURES];
    uint64_t id;
    uint32_t cust;
    if (!ccfd::parse_json_row(reinterpret_cast<const char*>(v), reinterpret_cast<const char*>(v) + vlen, x, &id, &cust))
      return false;
    const int rb = row_bytes();
    const bool ok = write_rows(pi, 1, [&](int64_t row, int64_t, int64_t) {
      sink->ids(pi)[row] = id;
      sink->cust(pi)[row] = cust;
      put_row(pi, x, sink->feats(pi) + row * rb, row);
    });
    *rows_out = ok ? 1 : 0;
    return ok;
  }

  // ---- parallel JSON parse (CCFD_KC_PARSE_THREADS > 1): one batch's messages are parsed on
  // a small pool into scratch rows, then written to the ring in order by this thread.  A
  // 4096-message batch costs ~5 ms of serial parse; the batch's last row waited for all of it.
  struct Rec { const uint8_t* val; int32_t vlen; int64_t off; };
  static constexpr int64_t kParMin = 256;
  static constexpr int64_t kParChunk = 1024;
  std::vector<Rec> recs;
  // 4 by default: in the deployed topology (JSON 1.2e6/s, 4096-message produce requests) the
  // engine's share of produce -> scored p50 fell from 3.2 to 1.4 ms on the same box
  // (profiles/r4/final_tree_v2/json_durable{,_p4}.json); CCFD_KC_PARSE_THREADS=1 is the serial path
  int parse_threads = 4;
  std::vector<float> pfeat;
  std::vector<uint64_t> pid;
  std::vector<uint32_t> pcust;
  std::vector<uint8_t> pok;
  struct Pool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv, done;
    uint64_t gen = 0;
    int left = 0;
    bool quit = false;
    std::function<void(int)> job;
    explicit Pool(int helpers) {
      for (int k = 0; k < helpers; ++k)
        th.emplace_back([this, k] {
          uint64_t seen = 0;
          for (;;) {
            std::function<void(int)> f;
            {
              std::unique_lock<std::mutex> lk(m);
              cv.wait(lk, [&] { return quit || gen != seen; });
              if (quit) return;
              seen = gen;
              f = job;
            }
            f(k + 1);
            std::lock_guard<std::mutex> lk(m);
            if (--left == 0) done.notify_one();
          }
        });
    }
    // run f(0) here and f(1..helpers) on the pool; returns when all are done
    void run(const std::function<void(int)>& f) {
      {
        std::lock_guard<std::mutex> lk(m);
        job = f;
        left = (int)th.size();
        ++gen;
      }
      cv.notify_all();
      f(0);
      std::unique_lock<std::mutex> lk(m);
      done.wait(lk, [&] { return left == 0; });
    }
    ~Pool() {
      {
        std::lock_guard<std::mutex> lk(m);
        quit = true;
      }
      cv.notify_all();
      for (auto& t : th) t.join();
    }
  };
  std::unique_ptr<Pool> pool;

  // records [c0, c1) of recs, split over the parse pool (results at their record index)
  void parse_parallel(int64_t c0, int64_t c1) {
    const int64_t n = (int64_t)recs.size();
    if (c0 == 0) {
      pfeat.resize((size_t)n * CCFD_N_FEATURES);
      pid.resize((size_t)n);
      pcust.resize((size_t)n);
      pok.assign((size_t)n, 0);
    }
    if (!pool) pool.reset(new Pool(parse_threads - 1));
    const int T = parse_threads;
    const int64_t m = c1 - c0;
    pool->run([this, c0, m, T](int k) {
      const int64_t lo = c0 + m * k / T, hi = c0 + m * (k + 1) / T;
      for (int64_t i = lo; i < hi; ++i) {
        const Rec& rc = recs[(size_t)i];
        if (rc.vlen <= 0) continue;
        const char* v = reinterpret_cast<const char*>(rc.val);
        pok[(size_t)i] = ccfd::parse_json_row(v, v + rc.vlen, &pfeat[(size_t)i * CCFD_N_FEATURES], &pid[(size_t)i],
                                              &pcust[(size_t)i]) ? 1 : 0;
      }
    });
  }

  // record i of the last parse_parallel() into the ring (the sequential half of ingest_value)
  bool put_parsed(int pi, size_t i, int64_t* rows_out) {
    *rows_out = 0;
    const float* x = &pfeat[i * CCFD_N_FEATURES];
    const int rb = row_bytes();
    const bool ok = write_rows(pi, 1, [&](int64_t row, int64_t, int64_t) {
      sink->ids(pi)[row] = pid[i];
      sink->cust(pi)[row] = pcust[i];
      put_row(pi, x, sink->feats(pi) + row * rb, row);
    });
    *rows_out = ok ? 1 : 0;
    return ok;
  }

  // gzip (codec 1) records section -> `inflated`; false on a corrupt stream
  bool gunzip(const uint8_t* p, size_t n) {
    z_stream zs{};
    if (inflateInit2(&zs, 32 + MAX_WBITS) != Z_OK) return false;   // gzip or zlib header
    inflated.resize(std::max<size_t>(inflated.capacity(), n * 4 + 4096));
    zs.next_in = const_cast<Bytef*>(p);
    zs.avail_in = (uInt)n;
    size_t out = 0;
    int rc = Z_OK;
    while (rc == Z_OK) {
      if (out == inflated.size()) {
        if (inflated.size() >= (size_t)1 << 30) { rc = Z_MEM_ERROR; break; }
        inflated.resize(inflated.size() * 2);
      }
      zs.next_out = inflated.data() + out;
      zs.avail_out = (uInt)std::min<size_t>(inflated.size() - out, UINT_MAX);
      rc = inflate(&zs, Z_NO_FLUSH);
      out = inflated.size() - zs.avail_out;
      if (rc == Z_BUF_ERROR && zs.avail_in == 0) break;
    }
    inflateEnd(&zs);
    if (rc != Z_STREAM_END) return false;
    inflated.resize(out);
    return true;
  }

  // RecordBatch v2 records of one partition's record set
  void ingest_record_set(int pi, const uint8_t* p, const uint8_t* e) {
    while (e - p >= 61) {                            // batch header
      In h{p, e};
      const int64_t base = h.i64();
      const int32_t blen = h.i32();
      if (blen < 49 || e - p < 12 + (int64_t)blen) break;   // partial trailing batch
      const uint8_t* bend = p + 12 + blen;
      h.i32();                                       // leader epoch
      const int8_t magic = h.i8();
      const uint32_t crc = h.u32();
      if (magic != 2 || ccfd_crc32c(h.p, (size_t)(bend - h.p), 0) != crc) {
        error("bad record batch (magic/crc)");
        return;
      }
      const int16_t attrs = h.i16();
      h.i32();                                       // last offset delta
      h.i64(); h.i64(); h.i64(); h.i16(); h.i32();    // timestamps, producer id/epoch, base seq
      const int32_t count = h.i32();
      const int codec = attrs & 0x7;
      In r{h.p, bend};
      if (codec == 1) {
        // a batch that passes its CRC but does not inflate is never skipped: a later batch would
        // move next_offset past its records and commit them unread (at-least-once broken) --
        // the partition stalls on it, like an unsupported codec below
        if (!gunzip(h.p, (size_t)(bend - h.p))) { error("corrupt gzip record batch"); return; }
        r = In{inflated.data(), inflated.data() + inflated.size()};
      } else if (codec != 0) {
        static const char* names[] = {"none", "gzip", "snappy", "lz4", "zstd"};
        error(std::string("unsupported compression codec ") + (codec <= 4 ? names[codec] : "?"));
        return;                                      // never skip data silently: the partition stalls
      }
      cur_origin = 0;
      recs.clear();
      bool all_json = true;
      for (int32_t i = 0; i < count && r.ok; ++i) {
        const int64_t rlen = r.varlong();
        if (!r.ok || rlen < 0 || rlen > r.e - r.p) { r.ok = false; break; }
        const uint8_t* rend = r.p + rlen;
        In rec{r.p, rend};
        rec.i8();                                    // attributes
        rec.varlong();                               // timestamp delta
        const int64_t od = rec.varlong();
        const int64_t klen = rec.varlong();
        if (klen > 0) rec.skip((size_t)klen);
        const int64_t vlen = rec.varlong();
        const uint8_t* val = rec.p;
        if (vlen > 0) rec.skip((size_t)vlen);
        // a value (or key) that runs past its record is a malformed batch (CRC only detects
        // corruption, any producer can build one): stop processing this batch
        if (!rec.ok || vlen > INT32_MAX || (vlen > 0 && val + vlen > rend)) { r.ok = false; break; }
        if (i == 0) {                                // the first record may carry the send time
          const int64_t hc = rec.varlong();
          for (int64_t h = 0; rec.ok && h < hc && h < 64; ++h) {
            const int64_t hk = rec.varlong();
            if (!rec.ok || hk < 0 || hk > rend - rec.p) break;
            const uint8_t* key = rec.p;
            rec.skip((size_t)hk);
            const int64_t hv = rec.varlong();
            if (!rec.ok || hv > rend - rec.p) break;
            if (hk == 7 && hv == 8 && std::memcmp(key, "ccfd-ts", 7) == 0) {
              uint64_t ts = 0;
              for (int b = 0; b < 8; ++b) ts = (ts << 8) | rec.p[b];
              const int64_t age = real_ns() - (int64_t)ts;       // send -> now (same host clock)
              if (age >= 0 && age < 3600ll * 1000000000ll) {
                cur_origin = mono_ns() - age;
                const int64_t fa = fetch_real > 0 ? std::max<int64_t>(0, fetch_real - (int64_t)ts) : age;
                const int bk = fa > 0 ? std::min(255, (int)(4.0 * std::log2((double)fa))) : 0;
                fetch_age_hist[bk].fetch_add(1, std::memory_order_relaxed);
              }
            }
            if (hv > 0) rec.skip((size_t)hv);
          }
        }
        r.p = rend;                                  // (other) headers skipped
        if (vlen >= 4 && std::memcmp(val, "TXB1", 4) == 0) all_json = false;
        recs.push_back({val, (int32_t)std::max<int64_t>(vlen, 0), base + od});
      }
      // the records, in order: JSON messages of a large batch are parsed on the parse pool
      // (CCFD_KC_PARSE_THREADS) kParChunk at a time, each chunk written / booked sequentially
      // before the next is parsed -- the batch's first rows reach the scoring ring after one
      // chunk's parse instead of the whole batch's (a 4096-message produce request: ~0.7 ms)
      const bool par = all_json && parse_threads > 1 && (int64_t)recs.size() >= kParMin;
      const size_t nrec = recs.size();
      const size_t step = par ? (size_t)kParChunk : nrec;
      for (size_t i = 0; i < nrec; ++i) {
        if (par && i % step == 0) parse_parallel((int64_t)i, (int64_t)std::min(nrec, i + step));
        const Rec& rc = recs[i];
        PState& s = ps[pi];
        if (rc.off < s.next_offset) continue;        // already consumed (batch starts below the fetch offset)
        int64_t rows = 0;
        bool ok;
        if (rc.vlen <= 0) ok = true;
        else if (par) ok = pok[i] && put_parsed(pi, i, &rows);
        else ok = ingest_value(pi, rc.val, rc.vlen, &rows);
        if (!ok) {
          if (stop.load()) return;
          n_errors.fetch_add(1);                     // malformed message: skip it
        }
        n_records.fetch_add(1, std::memory_order_relaxed);
        n_rows.fetch_add((uint64_t)rows, std::memory_order_relaxed);
        std::lock_guard<std::mutex> lk(mu);
        s.rows_in += rows;
        s.next_offset = rc.off + 1;
        s.pending.emplace_back(s.rows_in, rc.off + 1);
      }
      if (!r.ok) { error("malformed record in batch at offset " + std::to_string(base)); return; }
      p = bend;
    }
  }

  // one Fetch v4 response of one broker
  bool handle_fetch(const std::vector<uint8_t>& resp) {
    In in{resp.data(), resp.data() + resp.size()};
    in.i32();                                        // throttle
    const int32_t nt = in.i32();
    bool any = false;
    for (int32_t t = 0; t < nt && in.ok; ++t) {
      const int16_t sl = in.i16();
      in.skip(sl > 0 ? (size_t)sl : 0);
      const int32_t np = in.i32();
      for (int32_t q = 0; q < np && in.ok; ++q) {
        const int32_t part = in.i32();
        const int16_t err = in.i16();
        in.i64(); in.i64();                          // high watermark, last stable offset
        const int32_t na = in.i32();
        for (int32_t a = 0; a < na && in.ok; ++a) { in.i64(); in.i64(); }
        const int32_t rl = in.i32();
        const uint8_t* rs = in.p;
        if (rl > 0) in.skip((size_t)rl);
        if (!in.ok) break;
        int pi = -1;
        for (size_t k = 0; k < ps.size(); ++k)
          if (ps[k].kafka_partition == part) { pi = (int)k; break; }
        if (pi < 0) continue;
        if (err == kErrNotLeader || err == kErrUnknownTopicOrPartition || err == kErrLeaderNotAvailable ||
            err == kErrReplicaNotAvailable) {
          meta_stale = true;                         // leadership moved: refresh, same offset
          ps[pi].leader = -1;
          continue;
        }
        if (err == kErrOffsetOutOfRange) {
          if (reset_policy == CCFD_KC_RESET_NONE) {
            ps[pi].stopped = true;
            error("offset out of range on partition " + std::to_string(part) + " (reset policy none)");
          } else {
            ps[pi].reset = true;
          }
          continue;
        }
        if (err != 0) {
          error("fetch error " + std::to_string(err) + " on partition " + std::to_string(part));
          continue;
        }
        if (rl <= 0) continue;
        any = true;
        ingest_record_set(pi, rs, rs + rl);
      }
    }
    if (!in.ok) error("truncated fetch response");
    return any;
  }

  void loop() {
    std::vector<uint8_t> resp;
    std::map<int32_t, std::vector<int>> by_leader;
    while (!stop.load()) {
      if (meta_stale && !refresh_metadata()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
        continue;
      }
      for (size_t pi = 0; pi < ps.size(); ++pi)
        if (ps[pi].reset && !ps[pi].stopped) reset_offset((int)pi);
      by_leader.clear();
      for (size_t pi = 0; pi < ps.size(); ++pi)
        if (ps[pi].leader >= 0 && !ps[pi].stopped && !ps[pi].reset) by_leader[ps[pi].leader].push_back((int)pi);
      if (by_leader.empty()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(ps.empty() ? 100 : 5));
        if (std::all_of(ps.begin(), ps.end(), [](const PState& s) { return s.leader < 0; })) meta_stale = true;
        continue;
      }
      // send to every leader, then read every response: brokers work in parallel
      std::vector<int32_t> sent;
      int64_t ti = mono_ns();
      for (auto& kv : by_leader) {
        Conn* c = leader_conn(kv.first);
        if (!c) { meta_stale = true; continue; }
        if (!send_request(*c, 1, 4, fetch_body(kv.second, by_leader.size() == 1 ? max_wait_ms : 0))) {
          close_conn(*c);
          meta_stale = true;
          continue;
        }
        sent.push_back(kv.first);
      }
      n_leaders.store(sent.size(), std::memory_order_relaxed);
      bool any = false;
      for (int32_t node : sent) {
        Conn& c = brokers[node];
        const bool ok = recv_response(c, resp);
        t_io.fetch_add((uint64_t)(mono_ns() - ti), std::memory_order_relaxed);
        if (!ok) {                                   // broker died or stalled: reconnect via metadata
          close_conn(c);
          meta_stale = true;
          ti = mono_ns();
          continue;
        }
        n_fetches.fetch_add(1, std::memory_order_relaxed);
        n_bytes.fetch_add(resp.size(), std::memory_order_relaxed);
        fetch_real = real_ns();                      // the fetch-age histogram's "fetched"
        const int64_t th = mono_ns();
        any = handle_fetch(resp) || any;
        ti = mono_ns();
        t_handle.fetch_add((uint64_t)(ti - th), std::memory_order_relaxed);
      }
      if (!any) std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  }

  int64_t committable(int pi) {
    const int64_t rel = sink->released(pi);
    std::lock_guard<std::mutex> lk(mu);
    PState& s = ps[pi];
    int64_t last = -1;
    while (!s.pending.empty() && s.pending.front().first <= rel) {
      last = s.pending.front().second;
      s.pending.pop_front();
    }
    return last;
  }
};

Consumer* make(const char* host, int port, const char* topic, const ccfd_kc_partition* parts, int n, int wire) {
  auto* c = new Consumer();
  // bootstrap list: "h1:p1,h2:p2" or a bare host (then `port`)
  std::string all = host;
  size_t pos = 0;
  while (pos <= all.size()) {
    size_t q = all.find(',', pos);
    if (q == std::string::npos) q = all.size();
    std::string item = all.substr(pos, q - pos);
    pos = q + 1;
    if (item.empty()) continue;
    const size_t colon = item.rfind(':');
    if (colon != std::string::npos) c->seeds.emplace_back(item.substr(0, colon), std::atoi(item.c_str() + colon + 1));
    else c->seeds.emplace_back(item, port);
  }
  c->topic = topic;
  c->wire = wire;
  if (const char* e = std::getenv("CCFD_KC_PARSE_THREADS")) c->parse_threads = std::max(1, std::min(16, std::atoi(e)));
  c->ps.resize(n);
  for (int i = 0; i < n; ++i) {
    c->ps[i].kafka_partition = parts[i].kafka_partition;
    c->ps[i].next_offset = parts[i].start_offset;
  }
  return c;
}

}  // namespace

extern "C" {

void* ccfd_kc_create_engine(void* engine, const char* host, int port, const char* topic,
                            const ccfd_kc_partition* parts, int n_parts, int wire) {
  if (!engine || !host || !topic || !parts || n_parts <= 0) { ccfd::set_error("kc: bad arguments"); return nullptr; }
  Consumer* c = make(host, port, topic, parts, n_parts, wire);
  auto* s = new EngineSink();
  s->eng = engine;
  s->parts.assign(parts, parts + n_parts);
  c->sink = s;
  return c;
}

void* ccfd_kc_create_array(const char* host, int port, const char* topic, const ccfd_kc_partition* parts,
                           int n_parts, int wire) {
  if (!host || !topic || !parts || n_parts <= 0) { ccfd::set_error("kc: bad arguments"); return nullptr; }
  Consumer* c = make(host, port, topic, parts, n_parts, wire);
  auto* s = new ArraySink();
  s->parts.assign(parts, parts + n_parts);
  s->used.assign(n_parts, 0);
  c->sink = s;
  return c;
}

int ccfd_kc_set_bins(void* kc, const float* edges, const int32_t* offsets, int32_t stamp) {
  auto* c = static_cast<Consumer*>(kc);
  if (c->th.joinable()) { ccfd::set_error("kc: set_bins after start"); return -1; }
  if (!(c->wire == 3 ? ccfd::g20_table_ok : ccfd::g32_table_ok)(edges, offsets, stamp)) {
    ccfd::set_error(c->wire == 3 ? "kc: bad G20 bin table" : "kc: bad G32 bin table");
    return -1;
  }
  if (!c->bins.build(edges, offsets, stamp, c->wire == 3)) { ccfd::set_error("kc: bin plan allocation failed"); return -1; }
  c->g32_stamp = stamp;
  return 0;
}

int ccfd_kc_start(void* kc) {
  auto* c = static_cast<Consumer*>(kc);
  if (c->th.joinable()) return 0;
  if (c->wire >= 2 && c->g32_stamp == 0) { ccfd::set_error("kc: G32/G20 sink without a bin table"); return -1; }
  c->stop.store(false);
  c->th = std::thread([c] { c->loop(); });
  return 0;
}

void ccfd_kc_stop(void* kc) {
  auto* c = static_cast<Consumer*>(kc);
  c->stop.store(true);
  if (c->th.joinable()) c->th.join();
}

void ccfd_kc_destroy(void* kc) { delete static_cast<Consumer*>(kc); }

int64_t ccfd_kc_committable(void* kc, int part_index) {
  auto* c = static_cast<Consumer*>(kc);
  if (part_index < 0 || part_index >= (int)c->ps.size()) return -1;
  return c->committable(part_index);
}

void ccfd_kc_get_stats(void* kc, ccfd_kc_stats* out) {
  auto* c = static_cast<Consumer*>(kc);
  out->records = c->n_records.load();
  out->rows = c->n_rows.load();
  out->bytes = c->n_bytes.load();
  out->errors = c->n_errors.load();
  out->fetches = c->n_fetches.load();
  out->io_ns = c->t_io.load();
  out->handle_ns = c->t_handle.load();
  out->encode_ns = c->t_encode.load();
  out->ring_wait_ns = c->t_ring_wait.load();
  out->metadata_refreshes = c->n_meta.load();
  out->offset_resets = c->n_resets.load();
  out->leaders = c->n_leaders.load();
}

const char* ccfd_kc_last_error(void* kc) {
  auto* c = static_cast<Consumer*>(kc);
  static thread_local std::string copy;               // stable while the consumer thread runs
  std::lock_guard<std::mutex> lk(c->mu);
  copy = c->last_err;
  return copy.c_str();
}

int ccfd_kc_set_offset_reset(void* kc, int policy) {
  auto* c = static_cast<Consumer*>(kc);
  if (policy < CCFD_KC_RESET_EARLIEST || policy > CCFD_KC_RESET_NONE || c->th.joinable()) return -1;
  c->reset_policy = policy;
  return 0;
}

int64_t ccfd_kc_position(void* kc, int part_index) {
  auto* c = static_cast<Consumer*>(kc);
  if (part_index < 0 || part_index >= (int)c->ps.size()) return -1;
  std::lock_guard<std::mutex> lk(c->mu);
  return c->ps[part_index].next_offset;
}

// The producer send time (engine steady clock, ns) of the last ingested batch: 0 when it had
// no ccfd-ts header (tests; the engine reads it through ccfd_engine_ring_commit_at).
int64_t ccfd_kc_last_origin(void* kc) {
  return kc ? static_cast<Consumer*>(kc)->cur_origin : -1;
}

void ccfd_kc_fetch_age_hist(void* kc, uint64_t* out256) {
  auto* c = static_cast<Consumer*>(kc);
  for (int i = 0; i < 256; ++i) out256[i] = c ? c->fetch_age_hist[i].load(std::memory_order_relaxed) : 0;
}

// Fuzz / unit entry: feed raw bytes as partition 0's record set of an array-sink consumer
// (no socket).  Returns records accepted.  Used by tests/test_native_cpu.py under ASan.
int64_t ccfd_kc_feed_record_set(void* kc, const uint8_t* data, int64_t n) {
  auto* c = static_cast<Consumer*>(kc);
  if (!c || c->ps.empty() || !data || n < 0) return -1;
  const uint64_t before = c->n_records.load();
  c->ingest_record_set(0, data, data + n);
  return (int64_t)(c->n_records.load() - before);
}

}  // extern "C"
