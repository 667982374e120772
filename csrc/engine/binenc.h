// Branch-free G32 / G20 row encoder (GBDT ingest binning).
//
// A G32/G20 row stores, per feature j, bin_j = #{edges_j < x_j} against the ensemble's
// sorted split thresholds (contracts/transaction.py; exact for oblivious trees: the tree test
// `x > thr_k` is `bin > k`).  The reference op is the `x_f > thr` half of the model's predict
// (deploy/model/modelfull.json:37-44, BASELINE.json configs[3]); at 1e9 rows/s it is the ingest
// cost of the GBDT path, so it is vectorised instead of a per-feature binary search (5-8
// unpredictable branches a feature):
//
//   * `BinPlan` pads every feature's edges to a multiple of 8 with +inf, 32-byte aligned;
//   * a row broadcasts x_j and compares it against 8 edges per AVX2 `vcmpltps` (ordered,
//     quiet: NaN compares false everywhere -> bin 0, +inf padding never counts), the 8-bit
//     movemask is popcounted and summed -- `ceil(ne_j / 8)` compares a feature, no branches
//     on data (G20: every feature padded to 32 lanes, 4 compares, unrolled);
//   * G20 with AVX-512 (`encode_rows`, 16 rows at a time): each feature's 32 padded edges sit
//     in two zmm registers and the 16 rows' values are gathered into one; a 5-step branch-free
//     binary search (`vpermt2ps` picks edge lo + s - 1 per lane, `vcmpltps`, masked add) gives
//     all 16 bins in 20 instructions, and the 5-bit fields are packed vertically into three
//     64-bit words a row and scattered -- no per-row scalar work.
//
// Exact against the scalar lower_bound (`bin_of_ref`) for every input incl. NaN / +-inf /
// denormals (tests/test_native_cpu.py::test_simd_encoder_matches_reference).
#pragma once

#include <immintrin.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ccfd_abi.h"

namespace ccfd {

inline uint8_t bin_of_ref(const float* e, int ne, float x) {
  int lo = 0, hi = ne;                 // first edge >= x  ==  #edges < x  (edges ascending)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (e[mid] < x) lo = mid + 1; else hi = mid;
  }
  return (uint8_t)lo;
}

constexpr float kAmountBoundsHost[CCFD_N_AMOUNT_BUCKETS - 1] = {1.f, 5.f, 10.f, 25.f, 50.f, 100.f, 250.f,
                                                                500.f, 1000.f, 2500.f, 5000.f, 10000.f, 25000.f};
inline uint8_t amount_bucket_host(float a) {
  int b = 0;
  for (float bound : kAmountBoundsHost) b += a > bound ? 1 : 0;
  return (uint8_t)b;
}

struct BinPlan {
  float* pad = nullptr;                // 64-byte aligned, per feature nv[j] * 8 floats
  int32_t base[CCFD_N_FEATURES] = {};  // float offset of feature j in `pad`
  int32_t nv[CCFD_N_FEATURES] = {};    // 8-wide vectors of feature j
  int32_t stamp = 0;
  bool g20 = false;
  bool simd = false;
  bool avx512 = false;                 // 16-row vertical G20 encoder (encode_rows)

  BinPlan() = default;
  BinPlan(const BinPlan&) = delete;
  BinPlan& operator=(const BinPlan&) = delete;
  ~BinPlan() { std::free(pad); }

  // edges/offsets: the BinSpec flat table (offsets[30] = total edges); false on a bad table
  bool build(const float* edges, const int32_t* offsets, int32_t stamp_, bool g20_) {
    std::free(pad);
    pad = nullptr;
    int total = 0;
    for (int j = 0; j < CCFD_N_FEATURES; ++j) {
      const int ne = offsets[j + 1] - offsets[j];
      if (offsets[j] < 0 || ne < 0 || ne > (g20_ ? CCFD_G20_MAX_EDGES : 255)) return false;
      base[j] = total;
      nv[j] = g20_ ? 4 : (ne + 7) / 8;   // G20 (<= 31 edges): a fixed 32-lane compare, no loop
      total += nv[j] * 8;
    }
    const size_t bytes = ((size_t)std::max(total, 16) * sizeof(float) + 63) & ~(size_t)63;
    pad = static_cast<float*>(std::aligned_alloc(64, bytes));      // zmm-aligned rows of edges
    if (!pad) return false;
    const float inf = __builtin_inff();
    for (size_t i = 0; i < bytes / sizeof(float); ++i) pad[i] = inf;
    for (int j = 0; j < CCFD_N_FEATURES; ++j)
      std::memcpy(pad + base[j], edges + offsets[j], sizeof(float) * (size_t)(offsets[j + 1] - offsets[j]));
    stamp = stamp_;
    g20 = g20_;
    simd = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("popcnt");
    avx512 = g20 && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq");
    if (const char* e = std::getenv("CCFD_ENCODE_NO_AVX512")) if (std::atoi(e)) avx512 = false;
    return true;
  }

  // scalar fallback over the padded table (same result; +inf padding never counts)
  uint8_t bin_scalar(int j, float x) const {
    const float* e = pad + base[j];
    int c = 0;
    for (int k = 0; k < nv[j] * 8; ++k) c += e[k] < x ? 1 : 0;
    return (uint8_t)c;
  }

  __attribute__((target("avx2,popcnt"))) void bins_avx2(const float* x, uint8_t* b) const {
    if (g20) {                         // every feature padded to 32 lanes: 4 compares, unrolled
      for (int j = 0; j < CCFD_N_FEATURES; ++j) {
        const __m256 xv = _mm256_set1_ps(x[j]);
        const float* e = pad + base[j];
        const unsigned m0 = (unsigned)_mm256_movemask_ps(_mm256_cmp_ps(_mm256_load_ps(e), xv, _CMP_LT_OQ));
        const unsigned m1 = (unsigned)_mm256_movemask_ps(_mm256_cmp_ps(_mm256_load_ps(e + 8), xv, _CMP_LT_OQ));
        const unsigned m2 = (unsigned)_mm256_movemask_ps(_mm256_cmp_ps(_mm256_load_ps(e + 16), xv, _CMP_LT_OQ));
        const unsigned m3 = (unsigned)_mm256_movemask_ps(_mm256_cmp_ps(_mm256_load_ps(e + 24), xv, _CMP_LT_OQ));
        b[j] = (uint8_t)__builtin_popcount(m0 | (m1 << 8) | (m2 << 16) | (m3 << 24));
      }
      return;
    }
    for (int j = 0; j < CCFD_N_FEATURES; ++j) {
      const __m256 xv = _mm256_set1_ps(x[j]);
      const float* e = pad + base[j];
      int c = 0;
      for (int v = 0; v < nv[j]; ++v) {
        const __m256 m = _mm256_cmp_ps(_mm256_load_ps(e + 8 * v), xv, _CMP_LT_OQ);
        c += __builtin_popcount((unsigned)_mm256_movemask_ps(m));
      }
      b[j] = (uint8_t)c;
    }
  }

  void bins(const float* x, uint8_t* b) const {
    if (simd) { bins_avx2(x, b); return; }
    for (int j = 0; j < CCFD_N_FEATURES; ++j) b[j] = bin_scalar(j, x[j]);
  }

  // OR 16 fields (u32 lanes, < 64) at bit `bit` into the rows' 3 x 64-bit words
  // (w[word][half]: half 0 = rows 0..7, 1 = rows 8..15)
  __attribute__((target("avx512f,avx512dq"))) static void put_field(__m512i (*w)[2], __m512i v16, int bit) {
    const __m512i v[2] = {_mm512_cvtepu32_epi64(_mm512_castsi512_si256(v16)),
                          _mm512_cvtepu32_epi64(_mm512_extracti64x4_epi64(v16, 1))};
    const int wd = bit >> 6, sh = bit & 63;
    for (int h = 0; h < 2; ++h) {
      w[wd][h] = _mm512_or_si512(w[wd][h], _mm512_sll_epi64(v[h], _mm_cvtsi32_si128(sh)));
      if (sh + 6 > 64) w[wd + 1][h] = _mm512_or_si512(w[wd + 1][h], _mm512_srl_epi64(v[h], _mm_cvtsi32_si128(64 - sh)));
    }
  }

  // 16 G20 rows (row stride `ld` floats) -> out[16][20]; Amount column -> amount_out[16]
  __attribute__((target("avx512f,avx512dq"))) void encode16_g20_avx512(const float* x, int64_t ld, uint8_t* out,
                                                                      float* amount_out) const {
    const __m512i iota = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    const __m512i vidx = _mm512_mullo_epi32(iota, _mm512_set1_epi32((int)ld));
    __m512i w[3][2];
    for (int a = 0; a < 3; ++a) w[a][0] = w[a][1] = _mm512_setzero_si512();
    __m512 xa = _mm512_setzero_ps();
    for (int j = 0; j < CCFD_N_FEATURES; ++j) {
      const __m512 xv = _mm512_i32gather_ps(vidx, x + j, 4);
      if (j == CCFD_N_FEATURES - 1) xa = xv;
      const float* e = pad + base[j];
      const __m512 e0 = _mm512_loadu_ps(e), e1 = _mm512_loadu_ps(e + 16);
      __m512i lo = _mm512_setzero_si512();
      for (int st = 16; st >= 1; st >>= 1) {           // branch-free lower_bound over 32 lanes
        const __m512i idx = _mm512_add_epi32(lo, _mm512_set1_epi32(st - 1));
        const __m512 ec = _mm512_permutex2var_ps(e0, idx, e1);
        const __mmask16 m = _mm512_cmp_ps_mask(ec, xv, _CMP_LT_OQ);
        lo = _mm512_mask_add_epi32(lo, m, lo, _mm512_set1_epi32(st));
      }
      put_field(w, lo, 5 * j);
    }
    __m512i amt = _mm512_setzero_si512();
    for (float bound : kAmountBoundsHost) {
      const __mmask16 m = _mm512_cmp_ps_mask(xa, _mm512_set1_ps(bound), _CMP_GT_OQ);
      amt = _mm512_mask_add_epi32(amt, m, amt, _mm512_set1_epi32(1));
    }
    put_field(w, amt, 150);
    put_field(w, _mm512_set1_epi32(stamp & 63), 154);
    const __m512i off8 = _mm512_mullo_epi64(_mm512_setr_epi64(0, 1, 2, 3, 4, 5, 6, 7), _mm512_set1_epi64(CCFD_G20_ROW_BYTES));
    for (int h = 0; h < 2; ++h) {
      uint8_t* o = out + (size_t)h * 8 * CCFD_G20_ROW_BYTES;
      _mm512_i64scatter_epi64(o, off8, w[0][h], 1);
      _mm512_i64scatter_epi64(o + 8, off8, w[1][h], 1);
      _mm512_i64scatter_epi32(o + 16, off8, _mm512_cvtepi64_epi32(w[2][h]), 1);
    }
    if (amount_out) _mm512_storeu_ps(amount_out, xa);
  }

  // n rows (stride `ld` floats) -> n encoded rows; Amount column -> amount_out (optional)
  void encode_rows(const float* x, int64_t n, int64_t ld, uint8_t* out, float* amount_out) const {
    const int rb = g20 ? CCFD_G20_ROW_BYTES : CCFD_G32_ROW_BYTES;
    int64_t i = 0;
    if (avx512) {
      float amt[16];
      for (; i + 16 <= n; i += 16) {
        encode16_g20_avx512(x + i * ld, ld, out + i * rb, amount_out ? amount_out + i : amt);
      }
    }
    for (; i < n; ++i) {
      encode(x + i * ld, out + i * rb);
      if (amount_out) amount_out[i] = x[i * ld + CCFD_N_FEATURES - 1];
    }
  }

  // one G32 (32 B) or G20 (20 B) row
  void encode(const float* x, uint8_t* o) const {
    uint8_t b[CCFD_N_FEATURES];
    bins(x, b);
    const uint8_t amt = amount_bucket_host(x[CCFD_N_FEATURES - 1]);
    if (!g20) {
      std::memcpy(o, b, CCFD_N_FEATURES);
      o[30] = amt;
      o[31] = (uint8_t)stamp;
      return;
    }
    // 5 bits a feature, little-endian over 160 bits; amount bucket at bit 150, stamp at 154
    uint64_t w0 = 0, w1 = 0, w2 = 0;   // bits [0,64), [64,128), [128,192)
    for (int j = 0; j < 12; ++j) w0 |= (uint64_t)b[j] << (5 * j);                     // bits 0..59
    w0 |= (uint64_t)(b[12] & 0xF) << 60;                                              // bits 60..63
    w1 = (uint64_t)(b[12] >> 4);                                                      // bit 64
    for (int j = 13; j < 25; ++j) w1 |= (uint64_t)b[j] << (5 * j - 64);               // bits 65..124
    w1 |= (uint64_t)(b[25] & 0x7) << 61;                                              // bits 125..127
    w2 = (uint64_t)(b[25] >> 3);                                                      // bits 128..129
    for (int j = 26; j < CCFD_N_FEATURES; ++j) w2 |= (uint64_t)b[j] << (5 * j - 128); // bits 130..149
    w2 |= (uint64_t)amt << (150 - 128);
    w2 |= (uint64_t)(stamp & 63) << (154 - 128);
    std::memcpy(o, &w0, 8);
    std::memcpy(o + 8, &w1, 8);
    std::memcpy(o + 16, &w2, 4);
  }
};

}  // namespace ccfd
