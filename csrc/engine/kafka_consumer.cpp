// Native Kafka consumer: Fetch v4 over one TCP connection -> RecordBatch v2 (CRC-32C
// checked) -> rows written straight into the engine's pinned partition rings (SURVEY.md
// §2.4 H1 "C++ Kafka ingest ... writes directly into ring slots").
//
// One consumer thread per rank serves that rank's partitions of one topic.  Each record
// value is either a TXB1 columnar batch (contracts/transaction.py: ids, customers and f32
// rows are copied / W64-encoded row-block by row-block) or one JSON transaction (parsed by
// the native parser, ingest.cpp).  Offsets: after the rows of a record are committed to
// the ring, (ring rows written, next offset) is queued; ccfd_kc_committable() returns the
// highest offset whose rows the engine has already released (scored), so the caller
// commits consumer-group offsets only for scored data (at-least-once).
//
// Sinks: an engine ring (production) or a flat array (tests; no GPU needed).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../include/ccfd_abi.h"

extern "C" uint32_t ccfd_crc32c(const void* data, size_t n, uint32_t seed);

namespace ccfd {
void set_error(const std::string& e);
bool parse_json_row(const char* s, const char* e, float* f, uint64_t* id, uint32_t* cust);
void encode_w64_row(const float* x, uint8_t* out);
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
  virtual void commit(int p, int64_t n) = 0;
  virtual uint8_t* feats(int p) = 0;
  virtual uint64_t* ids(int p) = 0;
  virtual uint32_t* cust(int p) = 0;
  virtual int64_t released(int p) = 0;      // rows consumed downstream (for offset commits)
  virtual ~Sink() = default;
};

struct EngineSink : Sink {
  void* eng;
  std::vector<ccfd_kc_partition> parts;
  int64_t acquire(int p, int64_t want, int64_t* row) override {
    return ccfd_engine_ring_acquire(eng, parts[p].engine_partition, want, row);
  }
  void commit(int p, int64_t n) override { ccfd_engine_ring_commit(eng, parts[p].engine_partition, n); }
  uint8_t* feats(int p) override { return (uint8_t*)parts[p].feats; }
  uint64_t* ids(int p) override { return parts[p].ids; }
  uint32_t* cust(int p) override { return parts[p].customer; }
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
  void commit(int p, int64_t n) override { used[p] += n; }
  uint8_t* feats(int p) override { return (uint8_t*)parts[p].feats; }
  uint64_t* ids(int p) override { return parts[p].ids; }
  uint32_t* cust(int p) override { return parts[p].customer; }
  int64_t released(int p) override { return used[p]; }
};

struct PState {
  int32_t kafka_partition = 0;
  int64_t next_offset = 0;
  int64_t rows_in = 0;
  std::deque<std::pair<int64_t, int64_t>> pending;   // (rows_in after record, next offset)
};

class Consumer {
 public:
  std::string host, topic, client = "ccfd-native";
  int port = 9092;
  int wire = 0;                 // sink row format: 0 = f32[30], 1 = W64
  Sink* sink = nullptr;
  std::vector<PState> ps;
  std::mutex mu;                // guards ps[*].pending / next_offset reads from other threads
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> n_records{0}, n_rows{0}, n_bytes{0}, n_errors{0}, n_fetches{0};
  std::thread th;
  int fd = -1;
  int32_t corr = 0;
  int max_wait_ms = 5;
  std::string last_err;

  ~Consumer() {
    stop.store(true);
    if (th.joinable()) th.join();
    if (fd >= 0) ::close(fd);
    delete sink;
  }

  bool connect_broker() {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
      last_err = "resolve " + host;
      return false;
    }
    fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
    if (fd < 0 || ::connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
      freeaddrinfo(res);
      last_err = "connect " + host + ":" + std::to_string(port);
      return false;
    }
    freeaddrinfo(res);
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int rcv = 8 << 20;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &rcv, sizeof(rcv));
    return true;
  }

  bool send_all(const uint8_t* p, size_t n) {
    while (n) {
      const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
      if (k <= 0) return false;
      p += k;
      n -= (size_t)k;
    }
    return true;
  }
  bool recv_all(uint8_t* p, size_t n) {
    while (n) {
      const ssize_t k = ::recv(fd, p, n, 0);
      if (k <= 0) return false;
      p += k;
      n -= (size_t)k;
    }
    return true;
  }

  // Fetch v4 for every partition; returns the response body (after correlation id)
  bool fetch(std::vector<uint8_t>& resp) {
    Out body;
    body.i16(1);            // api key Fetch
    body.i16(4);            // version
    body.i32(++corr);
    body.str(client);
    body.i32(-1);           // replica id
    body.i32(max_wait_ms);
    body.i32(1);            // min bytes
    body.i32(64 << 20);     // max bytes
    body.i8(0);             // isolation: read uncommitted
    body.i32(1);            // one topic
    body.str(topic);
    {
      std::lock_guard<std::mutex> lk(mu);
      body.i32((int32_t)ps.size());
      for (auto& s : ps) {
        body.i32(s.kafka_partition);
        body.i64(s.next_offset);
        body.i32(16 << 20);
      }
    }
    Out frame;
    frame.i32((int32_t)body.b.size());
    frame.put(body.b.data(), body.b.size());
    if (!send_all(frame.b.data(), frame.b.size())) { last_err = "send"; return false; }
    uint8_t hdr[4];
    if (!recv_all(hdr, 4)) { last_err = "recv"; return false; }
    uint32_t len;
    std::memcpy(&len, hdr, 4);
    len = ntohl(len);
    resp.resize(len);
    if (!recv_all(resp.data(), len)) { last_err = "recv body"; return false; }
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
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        continue;
      }
      fn(row, done, k);
      sink->commit(pi, k);
      done += k;
    }
    return true;
  }

  const int row_bytes() const { return wire ? CCFD_WIRE_ROW_BYTES : CCFD_N_FEATURES * 4; }

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
        if (wire) {
          float tmp[CCFD_N_FEATURES];
          for (int64_t i = 0; i < k; ++i) {
            std::memcpy(tmp, f + (size_t)(s + i) * kRow, sizeof(tmp));
            ccfd::encode_w64_row(tmp, dst + i * rb);
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
      uint8_t* dst = sink->feats(pi) + row * rb;
      if (wire) ccfd::encode_w64_row(x, dst);
      else std::memcpy(dst, x, rb);
    });
    *rows_out = ok ? 1 : 0;
    return ok;
  }

  // RecordBatch v2 records of one partition's record set
  void ingest_record_set(int pi, const uint8_t* p, const uint8_t* e) {
    while (e - p >= 61) {                            // batch header
      In h{p, e};
      const int64_t base = h.i64();
      const int32_t blen = h.i32();
      if (blen < 49 || e - p < 12 + blen) break;     // partial trailing batch
      const uint8_t* bend = p + 12 + blen;
      h.i32();                                       // leader epoch
      const int8_t magic = h.i8();
      const uint32_t crc = h.u32();
      if (magic != 2 || ccfd_crc32c(h.p, (size_t)(bend - h.p), 0) != crc) {
        n_errors.fetch_add(1);
        std::lock_guard<std::mutex> lk(mu);
        last_err = "bad record batch (magic/crc)";
        return;
      }
      const int16_t attrs = h.i16();
      h.i32();                                       // last offset delta
      h.i64(); h.i64(); h.i64(); h.i16(); h.i32();    // timestamps, producer id/epoch, base seq
      const int32_t count = h.i32();
      if ((attrs & 0x7) != 0) {                      // compressed batches are not produced here
        n_errors.fetch_add(1);
        std::lock_guard<std::mutex> lk(mu);
        last_err = "compressed record batch";
        return;
      }
      In r{h.p, bend};
      for (int32_t i = 0; i < count && r.ok; ++i) {
        const int64_t rlen = r.varlong();
        const uint8_t* rend = r.p + rlen;
        if (rlen < 0 || rend > bend) { r.ok = false; break; }
        r.i8();                                      // attributes
        r.varlong();                                 // timestamp delta
        const int64_t od = r.varlong();
        const int64_t klen = r.varlong();
        if (klen > 0) r.skip((size_t)klen);
        const int64_t vlen = r.varlong();
        const uint8_t* val = r.p;
        if (vlen > 0) r.skip((size_t)vlen);
        r.p = rend;                                  // headers skipped
        const int64_t off = base + od;
        PState& s = ps[pi];
        if (off < s.next_offset) continue;           // already consumed (re-fetch overlap)
        int64_t rows = 0;
        if (vlen > 0 && !ingest_value(pi, val, (int32_t)vlen, &rows)) {
          if (stop.load()) return;
          n_errors.fetch_add(1);                     // malformed message: skip it
        }
        n_records.fetch_add(1, std::memory_order_relaxed);
        n_rows.fetch_add((uint64_t)rows, std::memory_order_relaxed);
        std::lock_guard<std::mutex> lk(mu);
        s.rows_in += rows;
        s.next_offset = off + 1;
        s.pending.emplace_back(s.rows_in, off + 1);
      }
      p = bend;
    }
  }

  void loop() {
    std::vector<uint8_t> resp;
    while (!stop.load()) {
      if (fd < 0 && !connect_broker()) {
        n_errors.fetch_add(1);
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
        continue;
      }
      if (!fetch(resp)) {
        n_errors.fetch_add(1);
        ::close(fd);
        fd = -1;
        continue;
      }
      n_fetches.fetch_add(1, std::memory_order_relaxed);
      n_bytes.fetch_add(resp.size(), std::memory_order_relaxed);
      In in{resp.data(), resp.data() + resp.size()};
      in.i32();                                      // correlation id
      in.i32();                                      // throttle
      const int32_t nt = in.i32();
      bool any = false;
      for (int32_t t = 0; t < nt && in.ok; ++t) {
        const int16_t sl = in.i16();
        in.skip(sl > 0 ? sl : 0);
        const int32_t np = in.i32();
        for (int32_t q = 0; q < np && in.ok; ++q) {
          const int32_t part = in.i32();
          const int16_t err = in.i16();
          in.i64(); in.i64();                        // high watermark, last stable offset
          const int32_t na = in.i32();
          for (int32_t a = 0; a < na && in.ok; ++a) { in.i64(); in.i64(); }
          const int32_t rl = in.i32();
          const uint8_t* rs = in.p;
          if (rl > 0) in.skip((size_t)rl);
          if (err != 0 || rl <= 0 || !in.ok) continue;
          int pi = -1;
          for (size_t k = 0; k < ps.size(); ++k)
            if (ps[k].kafka_partition == part) { pi = (int)k; break; }
          if (pi < 0) continue;
          any = true;
          ingest_record_set(pi, rs, rs + rl);
        }
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
  c->host = host;
  c->port = port;
  c->topic = topic;
  c->wire = wire;
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

int ccfd_kc_start(void* kc) {
  auto* c = static_cast<Consumer*>(kc);
  if (c->th.joinable()) return 0;
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
}

const char* ccfd_kc_last_error(void* kc) { return static_cast<Consumer*>(kc)->last_err.c_str(); }

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
