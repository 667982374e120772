// Native ingest: JSON-per-transaction parser for the compat path of topic `odh-demo`.
//
// The reference producer puts one `creditcard.csv` row per Kafka message
// (README.md:547-548); the router "extracts the features needed for the model"
// (README.md:549).  This parser does that extraction for a whole fetch of messages at
// once, straight into a (pinned) [n][30] feature block the engine can hand to the GPU.
// Accepted shapes (contracts/transaction.py): named columns {"Time","V1".."V28","Amount"}
// with optional "id"/"customer_id", or {"features":[30 numbers]}.
#include <cctype>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <thread>
#include <vector>

#include "../include/ccfd_abi.h"
#include "json_num.h"
#include "binenc.h"

namespace {

struct Cur {
  const char* p;
  const char* e;
  void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; }
  bool eat(char c) { ws(); if (p < e && *p == c) { ++p; return true; } return false; }
};

// feature column of a key, or -1 (ids: -2 = id, -3 = customer_id)
int key_col(const char* k, int n) {
  if (n == 4 && !std::memcmp(k, "Time", 4)) return 0;
  if (n == 6 && !std::memcmp(k, "Amount", 6)) return 29;
  if ((n == 2 || n == 3) && k[0] == 'V') {
    int v = 0;
    for (int i = 1; i < n; ++i) { if (!isdigit((unsigned char)k[i])) return -1; v = v * 10 + (k[i] - '0'); }
    return (v >= 1 && v <= 28) ? v : -1;
  }
  if ((n == 2 && !std::memcmp(k, "id", 2)) || (n == 5 && !std::memcmp(k, "tx_id", 5))) return -2;
  if ((n == 11 && !std::memcmp(k, "customer_id", 11)) || (n == 8 && !std::memcmp(k, "customer", 8))) return -3;
  if (n == 8 && !std::memcmp(k, "features", 8)) return -4;
  return -1;
}

bool parse_number(Cur& c, double* out) {
  c.ws();
  return ccfd::json::parse_number(c.p, c.e, out);
}

bool skip_value(Cur& c);

bool skip_string(Cur& c) {
  if (!c.eat('"')) return false;
  while (c.p < c.e) {
    if (*c.p == '\\') { c.p += 2; continue; }
    if (*c.p++ == '"') return true;
  }
  return false;
}

bool skip_value(Cur& c) {
  c.ws();
  if (c.p >= c.e) return false;
  char ch = *c.p;
  if (ch == '"') return skip_string(c);
  if (ch == '{' || ch == '[') {
    char close = ch == '{' ? '}' : ']';
    ++c.p;
    if (c.eat(close)) return true;
    for (;;) {
      if (ch == '{') { if (!skip_string(c) || !c.eat(':')) return false; }
      if (!skip_value(c)) return false;
      if (c.eat(',')) continue;
      return c.eat(close);
    }
  }
  // length first: the input is not NUL-terminated
  if (c.e - c.p >= 4 && !std::memcmp(c.p, "true", 4)) { c.p += 4; return true; }
  if (c.e - c.p >= 5 && !std::memcmp(c.p, "false", 5)) { c.p += 5; return true; }
  if (c.e - c.p >= 4 && !std::memcmp(c.p, "null", 4)) { c.p += 4; return true; }
  double d;
  return parse_number(c, &d);
}

bool parse_one(const char* s, const char* e, float* f, uint64_t* id, uint32_t* cust) {
  Cur c{s, e};
  for (int k = 0; k < CCFD_N_FEATURES; ++k) f[k] = 0.f;
  *id = 0; *cust = 0;
  if (!c.eat('{')) return false;
  if (c.eat('}')) return false;
  int seen = 0;
  for (;;) {
    c.ws();
    if (c.p >= c.e || *c.p != '"') return false;
    const char* k0 = ++c.p;
    if (c.e - c.p >= 8) {                    // short keys ("V17", "Amount"): find the quote 8 bytes at a time
      uint64_t w;
      std::memcpy(&w, c.p, 8);
      const uint64_t x = w ^ 0x2222222222222222ull;
      const uint64_t z = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
      if (z) c.p += __builtin_ctzll(z) >> 3;
      else while (c.p < c.e && *c.p != '"') ++c.p;
    } else {
      while (c.p < c.e && *c.p != '"') ++c.p;
    }
    if (c.p >= c.e) return false;
    const int kn = (int)(c.p - k0);
    ++c.p;
    if (!c.eat(':')) return false;
    const int col = key_col(k0, kn);
    if (col >= 0) {
      double d;
      if (!parse_number(c, &d)) return false;
      f[col] = (float)d;
      ++seen;
    } else if (col == -2 || col == -3) {
      double d;
      c.ws();
      bool quoted = c.eat('"');
      if (!parse_number(c, &d)) return false;
      if (quoted && !c.eat('"')) return false;
      // ids are non-negative integers: anything else (negative, NaN, beyond the type) is a
      // malformed message, never an undefined float->int conversion
      if (col == -2) {
        if (!(d >= 0.0 && d < 18446744073709551616.0)) return false;
        *id = (uint64_t)d;
      } else {
        if (!(d >= 0.0 && d < 4294967296.0)) return false;
        *cust = (uint32_t)d;
      }
    } else if (col == -4) {
      if (!c.eat('[')) return false;
      for (int k = 0; k < CCFD_N_FEATURES; ++k) {
        double d;
        if (!parse_number(c, &d)) return false;
        f[k] = (float)d;
        if (k + 1 < CCFD_N_FEATURES && !c.eat(',')) return false;
      }
      if (!c.eat(']')) return false;
      seen = CCFD_N_FEATURES;
    } else {
      if (!skip_value(c)) return false;
    }
    if (c.eat(',')) continue;
    if (!c.eat('}')) return false;
    break;
  }
  return seen > 0;
}

}  // namespace

extern "C" int64_t ccfd_parse_json_batch(const char* buf, const int64_t* offsets, int64_t n_msgs,
                                         float* feats, uint64_t* ids, uint32_t* customer) {
  for (int64_t i = 0; i < n_msgs; ++i) {
    const char* s = buf + offsets[i];
    const char* e = buf + offsets[i + 1];
    if (!parse_one(s, e, feats + i * CCFD_N_FEATURES, ids + i, customer + i)) return -(i + 1);
  }
  return n_msgs;
}

// ---------------------------------------------------------------------------------------
// W64 wire rows (contracts/transaction.py encode_wire): V1..V28 -> bf16 (round to nearest
// even), Time and Amount stay f32.  `ld` = f32 stride of the source rows.
namespace {
inline uint16_t bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7FFFFFFFu) > 0x7F800000u) return (uint16_t)((u >> 16) | 0x0040u);   // NaN stays a (quiet) NaN
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline void encode_row_w64(const float* x, uint8_t* out) {
  uint16_t* h = reinterpret_cast<uint16_t*>(out);
  for (int k = 0; k < 28; ++k) h[k] = bf16_rne(x[1 + k]);
  std::memcpy(out + 56, &x[0], 4);
  std::memcpy(out + 60, &x[CCFD_N_FEATURES - 1], 4);
}
}  // namespace

extern "C" int64_t ccfd_encode_w64(const float* x, int64_t n, int64_t ld, uint8_t* out) {
  if (ld < CCFD_N_FEATURES) return -1;
  for (int64_t i = 0; i < n; ++i) encode_row_w64(x + i * ld, out + i * CCFD_WIRE_ROW_BYTES);
  return n;
}

// JSON messages straight into W64 rows (the ingest path of a wire-format engine ring).
extern "C" int64_t ccfd_parse_json_batch_w64(const char* buf, const int64_t* offsets, int64_t n_msgs,
                                             uint8_t* rows, uint64_t* ids, uint32_t* customer) {
  float f[CCFD_N_FEATURES];
  for (int64_t i = 0; i < n_msgs; ++i) {
    const char* s = buf + offsets[i];
    const char* e = buf + offsets[i + 1];
    if (!parse_one(s, e, f, ids + i, customer + i)) return -(i + 1);
    encode_row_w64(f, rows + i * CCFD_WIRE_ROW_BYTES);
  }
  return n_msgs;
}

// ---------------------------------------------------------------------------------------
// G32 rows (GBDT; ccfd_abi.h, contracts/transaction.py encode_g32): byte j = #{edges_j < x_j}
// (lower_bound; NaN compares false everywhere -> 0), byte 30 = amount bucket with the
// device's bounds (common.h amount_bucket), byte 31 = bin-table stamp.  G20 rows: the same
// bins, 5 bits each, little-endian over 160 bits; the amount bucket at bit 150 and the 6-bit
// stamp at bit 154.  Encoded by the branch-free SIMD BinPlan (binenc.h); the scalar
// binary-search encoders stay as `_ref` entry points (oracle for tests and the microbench).
namespace {
using ccfd::amount_bucket_host;
using ccfd::bin_of_ref;

inline void encode_row_g32_ref(const float* r, uint8_t* o, const float* edges, const int32_t* offsets, int32_t stamp) {
  for (int j = 0; j < CCFD_N_FEATURES; ++j)
    o[j] = bin_of_ref(edges + offsets[j], offsets[j + 1] - offsets[j], r[j]);
  o[30] = amount_bucket_host(r[CCFD_N_FEATURES - 1]);
  o[31] = (uint8_t)stamp;
}

inline void encode_row_g20_ref(const float* r, uint8_t* o, const float* edges, const int32_t* offsets, int32_t stamp) {
  uint32_t w[6] = {0, 0, 0, 0, 0, 0};  // 5 dwords + one spill dword for the funnel below
  auto put = [&](int bit, uint32_t v) {   // v < 2^6
    w[bit >> 5] |= v << (bit & 31);
    if ((bit & 31) + 6 > 32) w[(bit >> 5) + 1] |= v >> (32 - (bit & 31));
  };
  for (int j = 0; j < CCFD_N_FEATURES; ++j)
    put(5 * j, bin_of_ref(edges + offsets[j], offsets[j + 1] - offsets[j], r[j]));
  put(150, amount_bucket_host(r[CCFD_N_FEATURES - 1]));
  w[4] |= (uint32_t)(stamp & 63) << (154 - 128);
  memcpy(o, w, CCFD_G20_ROW_BYTES);
}

int64_t encode_plan(const float* x, int64_t n, int64_t ld, const ccfd::BinPlan& plan, uint8_t* out,
                    float* amount_out) {
  plan.encode_rows(x, n, ld, out, amount_out);
  return n;
}
}  // namespace

namespace ccfd {
bool g32_table_ok(const float* edges, const int32_t* offsets, int32_t stamp) {
  if (stamp < 1 || stamp > 255 || !edges || !offsets) return false;
  for (int j = 0; j < CCFD_N_FEATURES; ++j) {
    const int ne = offsets[j + 1] - offsets[j];
    if (offsets[j] < 0 || ne < 0 || ne > 255) return false;
  }
  return true;
}
bool g20_table_ok(const float* edges, const int32_t* offsets, int32_t stamp) {
  if (stamp > 63 || !g32_table_ok(edges, offsets, stamp)) return false;
  for (int j = 0; j < CCFD_N_FEATURES; ++j)
    if (offsets[j + 1] - offsets[j] > CCFD_G20_MAX_EDGES) return false;
  return true;
}
}  // namespace ccfd

extern "C" int64_t ccfd_encode_g32(const float* x, int64_t n, int64_t ld, const float* edges,
                                   const int32_t* offsets, int32_t stamp, uint8_t* out, float* amount_out) {
  if (ld < CCFD_N_FEATURES || n < 0 || !out || !ccfd::g32_table_ok(edges, offsets, stamp)) return -1;
  ccfd::BinPlan plan;
  if (!plan.build(edges, offsets, stamp, false)) return -1;
  return encode_plan(x, n, ld, plan, out, amount_out);
}

extern "C" int64_t ccfd_encode_g20(const float* x, int64_t n, int64_t ld, const float* edges,
                                   const int32_t* offsets, int32_t stamp, uint8_t* out, float* amount_out) {
  if (ld < CCFD_N_FEATURES || n < 0 || !out || !ccfd::g20_table_ok(edges, offsets, stamp)) return -1;
  ccfd::BinPlan plan;
  if (!plan.build(edges, offsets, stamp, true)) return -1;
  return encode_plan(x, n, ld, plan, out, amount_out);
}

// The pre-SIMD encoders (scalar binary search a feature), kept as the exactness oracle and
// the microbench baseline (bench/encode_bench.py).
extern "C" int64_t ccfd_encode_g32_ref(const float* x, int64_t n, int64_t ld, const float* edges,
                                       const int32_t* offsets, int32_t stamp, uint8_t* out, float* amount_out) {
  if (ld < CCFD_N_FEATURES || n < 0 || !out || !ccfd::g32_table_ok(edges, offsets, stamp)) return -1;
  for (int64_t i = 0; i < n; ++i) {
    const float* r = x + i * ld;
    encode_row_g32_ref(r, out + i * CCFD_G32_ROW_BYTES, edges, offsets, stamp);
    if (amount_out) amount_out[i] = r[CCFD_N_FEATURES - 1];
  }
  return n;
}

extern "C" int64_t ccfd_encode_g20_ref(const float* x, int64_t n, int64_t ld, const float* edges,
                                       const int32_t* offsets, int32_t stamp, uint8_t* out, float* amount_out) {
  if (ld < CCFD_N_FEATURES || n < 0 || !out || !ccfd::g20_table_ok(edges, offsets, stamp)) return -1;
  for (int64_t i = 0; i < n; ++i) {
    const float* r = x + i * ld;
    encode_row_g20_ref(r, out + i * CCFD_G20_ROW_BYTES, edges, offsets, stamp);
    if (amount_out) amount_out[i] = r[CCFD_N_FEATURES - 1];
  }
  return n;
}

// Multi-threaded encode of a large block (log fill, bench attribution): rows split over
// `threads` std::threads.  Returns n or -1.
extern "C" int64_t ccfd_encode_bins_mt(const float* x, int64_t n, int64_t ld, const float* edges,
                                       const int32_t* offsets, int32_t stamp, int32_t g20, uint8_t* out,
                                       float* amount_out, int32_t threads) {
  if (ld < CCFD_N_FEATURES || n < 0 || !out || threads < 1 || threads > 256) return -1;
  if (!(g20 ? ccfd::g20_table_ok : ccfd::g32_table_ok)(edges, offsets, stamp)) return -1;
  ccfd::BinPlan plan;
  if (!plan.build(edges, offsets, stamp, g20 != 0)) return -1;
  const int rb = g20 ? CCFD_G20_ROW_BYTES : CCFD_G32_ROW_BYTES;
  const int64_t per = (n + threads - 1) / threads;
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) {
    const int64_t a = (int64_t)t * per, b = std::min<int64_t>(n, a + per);
    if (a >= b) break;
    th.emplace_back([=, &plan] {
      encode_plan(x + a * ld, b - a, ld, plan, out + a * rb, amount_out ? amount_out + a : nullptr);
    });
  }
  for (auto& t : th) t.join();
  return n;
}

// Which encoder a G20 / G32 BinPlan runs on this host: 2 = AVX-512 16-row (G20 only),
// 1 = AVX2 compare + popcount, 0 = scalar (CCFD_ENCODE_NO_AVX512 honoured).
extern "C" int32_t ccfd_encode_isa(int32_t g20) {
  const float e = 0.f;
  const int32_t offs[CCFD_N_FEATURES + 1] = {};
  ccfd::BinPlan plan;
  if (!plan.build(&e, offs, 1, g20 != 0)) return -1;
  return plan.avx512 ? 2 : plan.simd ? 1 : 0;
}

// Internal entry points for the native Kafka consumer (kafka_consumer.cpp).
namespace ccfd {
bool parse_json_row(const char* s, const char* e, float* f, uint64_t* id, uint32_t* cust) {
  return parse_one(s, e, f, id, cust);
}
void encode_w64_row(const float* x, uint8_t* out) { encode_row_w64(x, out); }
void encode_bins_row(const BinPlan& plan, const float* x, uint8_t* out) { plan.encode(x, out); }
void encode_bins_rows(const BinPlan& plan, const float* x, int64_t n, int64_t ld, uint8_t* out, float* amount_out) {
  plan.encode_rows(x, n, ld, out, amount_out);
}
}  // namespace ccfd
