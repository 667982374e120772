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

// 16 G20 rows as five 32-bit word vectors (lane = row) -> row-major 16 x 5 dwords: output
// register m holds flat dwords 16m + i = (row (16m + i) / 5, word (16m + i) % 5)
struct G20OutTable {
  alignas(64) int32_t idx[5][16];
  uint16_t mask[5][5];
  constexpr G20OutTable() : idx(), mask() {
    for (int m = 0; m < 5; ++m)
      for (int i = 0; i < 16; ++i) {
        const int f = 16 * m + i;
        idx[m][i] = f / 5;
        mask[m][f % 5] = (uint16_t)(mask[m][f % 5] | (1u << i));
      }
  }
};
inline constexpr G20OutTable kG20Out{};

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

  // OR 16 fields (u32 lanes, < 64) at bit `bit` of the rows' five 32-bit words (lane = row)
  __attribute__((target("avx512f"))) static void put_field(__m512i* w, __m512i v16, int bit) {
    const int wd = bit >> 5, sh = bit & 31;
    w[wd] = _mm512_or_si512(w[wd], _mm512_slli_epi32(v16, (unsigned)sh));
    if (sh + 6 > 32) w[wd + 1] = _mm512_or_si512(w[wd + 1], _mm512_srli_epi32(v16, (unsigned)(32 - sh)));
  }

  // In-register 16x16 transpose: r[i] = row i (16 floats) -> r[j] = column j of the 16 rows.
  // 64 shuffles (32-bit unpack, 64-bit shuffle, two 128-bit lane shuffles) instead of 16
  // gathers: a zmm gather is ~20 uops on both Zen 4/5 and Golden Cove.
  __attribute__((target("avx512f"))) static void transpose16(__m512* r) {
    __m512 t[16];
    for (int i = 0; i < 16; i += 2) {
      t[i] = _mm512_unpacklo_ps(r[i], r[i + 1]);
      t[i + 1] = _mm512_unpackhi_ps(r[i], r[i + 1]);
    }
    for (int i = 0; i < 16; i += 4) {              // r[i + q], lane k: rows i..i+3 of column 4k + q
      r[i] = _mm512_shuffle_ps(t[i], t[i + 2], _MM_SHUFFLE(1, 0, 1, 0));
      r[i + 1] = _mm512_shuffle_ps(t[i], t[i + 2], _MM_SHUFFLE(3, 2, 3, 2));
      r[i + 2] = _mm512_shuffle_ps(t[i + 1], t[i + 3], _MM_SHUFFLE(1, 0, 1, 0));
      r[i + 3] = _mm512_shuffle_ps(t[i + 1], t[i + 3], _MM_SHUFFLE(3, 2, 3, 2));
    }
    for (int q = 0; q < 4; ++q) {
      t[q] = _mm512_shuffle_f32x4(r[q], r[4 + q], 0x88);          // columns q, 8+q of rows 0..7
      t[4 + q] = _mm512_shuffle_f32x4(r[q], r[4 + q], 0xdd);      // columns 4+q, 12+q
      t[8 + q] = _mm512_shuffle_f32x4(r[8 + q], r[12 + q], 0x88); // same, rows 8..15
      t[12 + q] = _mm512_shuffle_f32x4(r[8 + q], r[12 + q], 0xdd);
    }
    for (int q = 0; q < 4; ++q) {
      r[q] = _mm512_shuffle_f32x4(t[q], t[8 + q], 0x88);
      r[8 + q] = _mm512_shuffle_f32x4(t[q], t[8 + q], 0xdd);
      r[4 + q] = _mm512_shuffle_f32x4(t[4 + q], t[12 + q], 0x88);
      r[12 + q] = _mm512_shuffle_f32x4(t[4 + q], t[12 + q], 0xdd);
    }
  }

  // 16 G20 rows (row stride `ld` >= 30 floats) -> out[16][20]; Amount column -> amount_out[16].
  // The rows are read with two overlapping 16-float loads each (features 0..15 and 14..29, no
  // read past feature 29) and transposed in registers; the packed words go out with plain
  // stores (a zmm scatter is microcoded on Zen 4/5).
  __attribute__((target("avx512f,avx512dq"))) void encode16_g20_avx512(const float* x, int64_t ld, uint8_t* out,
                                                                      float* amount_out) const {
    __m512 lo16[16], hi16[16];
    for (int r = 0; r < 16; ++r) {
      lo16[r] = _mm512_loadu_ps(x + r * ld);
      hi16[r] = _mm512_loadu_ps(x + r * ld + (CCFD_N_FEATURES - 16));
    }
    transpose16(lo16);
    transpose16(hi16);
    __m512i w[5];
    for (int a = 0; a < 5; ++a) w[a] = _mm512_setzero_si512();
    const __m512 xa = hi16[15];
    for (int j = 0; j < CCFD_N_FEATURES; ++j) {
      const __m512 xv = j < 16 ? lo16[j] : hi16[j - (CCFD_N_FEATURES - 16)];
      const float* e = pad + base[j];
      // branch-free lower_bound over 32 lanes: the first two steps pick between broadcast
      // edges (15; 7 / 23), the last three permute (vpermt2ps) the two edge registers
      const __mmask16 m16 = _mm512_cmp_ps_mask(_mm512_set1_ps(e[15]), xv, _CMP_LT_OQ);
      const __m512 e8 = _mm512_mask_blend_ps(m16, _mm512_set1_ps(e[7]), _mm512_set1_ps(e[23]));
      const __mmask16 m8 = _mm512_cmp_ps_mask(e8, xv, _CMP_LT_OQ);
      __m512i lo = _mm512_maskz_mov_epi32(m16, _mm512_set1_epi32(16));
      lo = _mm512_mask_add_epi32(lo, m8, lo, _mm512_set1_epi32(8));
      const __m512 e0 = _mm512_load_ps(e), e1 = _mm512_load_ps(e + 16);
      for (int st = 4; st >= 1; st >>= 1) {
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
    // five word vectors (lane = row) -> 16 rows x 5 dwords, row-major: output register m holds
    // flat dwords 16m..16m+15 = (row, word) = divmod(16m + i, 5), gathered by masked permutes
    for (int m = 0; m < 5; ++m) {
      const __m512i ix = _mm512_load_si512(kG20Out.idx[m]);
      __m512i o = _mm512_maskz_permutexvar_epi32(kG20Out.mask[m][0], ix, w[0]);
      for (int k = 1; k < 5; ++k) o = _mm512_mask_permutexvar_epi32(o, kG20Out.mask[m][k], ix, w[k]);
      _mm512_storeu_si512(out + 64 * m, o);
    }
    if (amount_out) _mm512_storeu_ps(amount_out, xa);
  }

  // n rows (stride `ld` floats) -> n encoded rows; Amount column -> amount_out (optional)
  void encode_rows(const float* x, int64_t n, int64_t ld, uint8_t* out, float* amount_out) const {
    const int rb = g20 ? CCFD_G20_ROW_BYTES : CCFD_G32_ROW_BYTES;
    int64_t i = 0;
    if (avx512 && ld >= CCFD_N_FEATURES) {
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
