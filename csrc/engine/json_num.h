// Decimal number reader shared by the native JSON front ends (ingest.cpp: one transaction
// per Kafka message; seldon_http.cpp: Seldon predict() bodies).  Bit-identical to strtod:
// the common short decimals take an exact fast path (8 digits per SWAR step + Clinger's
// single correctly rounded multiply/divide); everything else falls back to strtod.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>

namespace ccfd {
namespace json {

// Exact powers of ten in double (10^0 .. 10^22).
inline constexpr double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                      1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

inline bool parse_number_slow(const char*& p, const char* e, double* out) {
  // strtod needs a terminator; numbers in JSON are short, copy to a small buffer
  char buf[64];
  int n = 0;
  while (p < e && n < 63 && (((unsigned)(*p - '0') < 10u) || *p == '-' || *p == '+' || *p == '.' ||
                              *p == 'e' || *p == 'E'))
    buf[n++] = *p++;
  if (n == 0) return false;
  buf[n] = 0;
  char* end = nullptr;
  *out = std::strtod(buf, &end);
  return end == buf + n;
}

// Up to 8 ASCII digits at p (8 readable bytes): k = how many lead the word, *val = their value
// (SWAR: one 8-byte load instead of a branch per digit; fast_float-style 8-digit reduction).
inline int swar_digits(const char* p, uint64_t* val) {
  uint64_t w;
  std::memcpy(&w, p, 8);
  const uint64_t d = w ^ 0x3030303030303030ull;                      // digits -> 0..9 per byte
  const uint64_t nd = (((d & 0x7F7F7F7F7F7F7F7Full) + 0x7676767676767676ull) | d) & 0x8080808080808080ull;
  const int k = nd ? __builtin_ctzll(nd) >> 3 : 8;
  if (k == 0) { *val = 0; return 0; }
  uint64_t v = d << (8 * (8 - k));                                   // leading zeros pad to 8 digits
  v = (v * 10) + (v >> 8);
  v = (((v & 0x000000FF000000FFull) * (100 + (1000000ull << 32))) +
       (((v >> 16) & 0x000000FF000000FFull) * (1 + (10000ull << 32)))) >> 32;
  *val = v;
  return k;
}

inline constexpr uint64_t kPow10u[9] = {1, 10, 100, 1000, 10000, 100000, 1000000, 10000000, 100000000};

// Clinger's fast path: a mantissa m <= 2^53 with a decimal exponent within +-22 is exact in
// double, as is 10^|e|, so ONE correctly rounded multiply or divide gives the same double
// strtod returns.  Anything else (long mantissas, big exponents, malformed input) takes
// strtod.  Integer and fraction digits are read 8 at a time when the message has 8 more
// bytes (the common case); the tail of a message falls back to the per-digit loop.
inline bool parse_number(const char*& cp, const char* ce, double* out) {
  if (cp >= ce) return false;
  const char* const start = cp;
  const char* p = cp;
  const bool neg = *p == '-';
  if (neg || *p == '+') ++p;
  uint64_t m = 0;
  int ndig = 0, exp10 = 0;
  bool any = false;
  // integer part
  for (;;) {
    if (ce - p >= 8) {
      uint64_t v;
      const int k = swar_digits(p, &v);
      if (ndig + k > 19) goto slow;
      m = m * kPow10u[k] + v;
      ndig += k;
      p += k;
      any = any || k > 0;
      if (k == 8) continue;
      break;
    }
    while (p < ce && (unsigned)(*p - '0') < 10u) {
      if (++ndig > 19) goto slow;
      m = m * 10 + (uint64_t)(*p++ - '0');
      any = true;
    }
    break;
  }
  if (p < ce && *p == '.') {
    ++p;
    for (;;) {
      if (ce - p >= 8) {
        uint64_t v;
        const int k = swar_digits(p, &v);
        if (ndig + k > 19) goto slow;
        m = m * kPow10u[k] + v;
        ndig += k;
        exp10 -= k;
        p += k;
        any = any || k > 0;
        if (k == 8) continue;
        break;
      }
      while (p < ce && (unsigned)(*p - '0') < 10u) {
        if (++ndig > 19) goto slow;
        m = m * 10 + (uint64_t)(*p++ - '0');
        --exp10;
        any = true;
      }
      break;
    }
  }
  if (!any) return false;
  if (p < ce && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < ce && (*p == '-' || *p == '+')) eneg = *p++ == '-';
    const char* e0 = p;
    int ev = 0;
    while (p < ce && (unsigned)(*p - '0') < 10u) { if (ev < 10000) ev = ev * 10 + (*p - '0'); ++p; }
    if (p == e0) return false;
    exp10 += eneg ? -ev : ev;
  }
  if (m <= (1ull << 53) && exp10 >= -22 && exp10 <= 22) {
    double v = (double)m;
    v = exp10 < 0 ? v / kPow10[-exp10] : v * kPow10[exp10];
    *out = neg ? -v : v;
    cp = p;
    return true;
  }
slow:
  cp = start;
  return parse_number_slow(cp, ce, out);
}

}  // namespace json
}  // namespace ccfd
