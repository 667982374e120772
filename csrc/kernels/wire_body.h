// Streaming body shared by the W64 wire kernels (MLP, LR): 16-row tiles per wave with a
// branch-free prefetch ring, the per-tile epilogue (outputs, counters, lane-spread amount
// histogram, compacted fraud list) and the workgroup flush.  The model math is a Scorer:
//   static constexpr int kLds;                       LDS bytes the scorer stages (blob copy)
//   void stage(const ccfd_score_args&, char* lds, int tid, int nthreads);   before the barrier
//   void lanes(const char* lds, const ccfd_score_args&, int g);            after the barrier
//   float tile(const char* lds, const WireRegs&, int g, int lane) const;   proba_1 of row lane&15
// and, for the four-tile epilogue (kQuad, kPf == 4, no routing rules):
//   float logit(const char* lds, const WireRegs&, int g, int lane) const;  logit of row lane&15
//   float proba(float z) const;                                            sigmoid of a logit
#pragma once
#include "common.h"
#include "rules.h"

namespace ccfd {

// One wave scores 16-row tiles with kPf tiles in flight -- a tile's slot is refilled as
// soon as its operand is consumed, so a wave keeps kPf-1 1-KB requests outstanding while it
// computes.  Loads are branch-free (rows clamped into the batch; clamped rows are never
// scored) and the steady-state loop is unrolled kPf times over static ring slots, so no
// register copy of an in-flight load -- which would force an s_waitcnt vmcnt(0) -- is ever
// needed; only the < kPf-tile tail rotates the ring.
// kR: the launch carries a routing rule program (a.rules); instantiated separately so the
// threshold-only kernels keep their register allocation.
template <class Scorer, int kWaves, int kPf, bool kR = false>
__device__ __forceinline__ void wire_stream_body(const ccfd_score_args& a, int blk, int nblk) {
  __shared__ __attribute__((aligned(16))) char lds[Scorer::kLds > 0 ? Scorer::kLds : 16];
  __shared__ EpilogueLds epi;
  __shared__ unsigned flbuf[kWaves][128];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  stamp_start(a, blk);
  const int n = a.n;
  const int ntiles = (n + kTileRows - 1) / kTileRows;
  const int tstride = nblk * kWaves;
  int tile = blk * kWaves + wave;
  const unsigned char* xw = reinterpret_cast<const unsigned char*>(a.x) + 16 * g;
  auto issue = [&](int t, WireRegs& r) __attribute__((always_inline)) {
    const int row = min(t * kTileRows + c, n - 1);
    r.v = *reinterpret_cast<const uint4*>(xw + (size_t)row * CCFD_WIRE_ROW_BYTES);
  };
  WireRegs ring[kPf];
#pragma unroll
  for (int k = 0; k < kPf; ++k) issue(tile + k * tstride, ring[k]);
  Scorer sc;
  sc.stage(a, lds, tid, 64 * kWaves);
  epi_init(epi);
  __syncthreads();
  sc.lanes(lds, a, g);

  const float thr = a.threshold;
  FlagStage fls{flbuf[wave], 0u};
  unsigned fraud = 0, rows = 0;
  unsigned long long psum = 0;
  HistLanes hl;
  hist_lanes_init(hl, g);
  // routing rules (when configured) read the tile's features, so they are evaluated while
  // the tile's registers are still live -- before its ring slot is refilled
  const ccfd_rule_prog* rules = a.rules;
  auto rule_of = [&](const WireRegs& r, float p) __attribute__((always_inline)) {
    if constexpr (kR) {
      float xv[8];
      wire_features(r, g, xv);
      return rule_route(rules, __shfl(p, c), [&](int j) { return lane_feature<true>(xv, j, c); });
    } else {
      return false;
    }
  };
  auto finish = [&](float p, float amount, int t, bool rf) __attribute__((always_inline)) {
    const int row = t * kTileRows + c;
    const bool valid = row < n;
    const bool fr = valid && (kR ? rf : (p >= thr));
    if (valid && g == 0) {
      if (a.proba) st_g(a.proba + row, p);
      if (a.route) st_g(a.route + row, (uint8_t)(fr ? 1 : 0));
      psum += (unsigned)(p * 1e6f + 0.5f);
    }
    const unsigned long long frm = __ballot(fr && g == 3);     // same rows as the g == 0 lanes
    fraud += __popcll(frm);
    rows += (unsigned)min(kTileRows, n - t * kTileRows);
    const float am_g3 = (valid && g == 3) ? amount : -__builtin_inff();
    hist_lanes_add(hl, __shfl(am_g3, 48 + c));
    if (frm) {                                                   // rare: fraud rows' buckets
      if (fr && g == 3) atomicAdd(&epi.hist[kNB + amount_bucket_fast(amount)], 1u);
      if (a.flags & CCFD_ARG_FLAG_DIRECT) emit_flagged(a, fr && g == 3, row);
      else flag_push(a, fls, frm, fr && g == 3, row, lane);
    }
  };
  // steady state: the kPf strided tiles of a round all exist
  const int full_end = ntiles - (kPf - 1) * tstride;
  // Four-tile epilogue: every lane's proba_1 / logit is replicated over the 4 lane groups, so
  // lane group g finishes tile g of the round -- one sigmoid, one threshold, one 64-lane store,
  // one ballot per counter for 64 rows instead of four 16-lane passes.  The amount histogram
  // becomes 13 wave-uniform "amount > bound" ballot popcounts (SALU) per 64 rows.
  unsigned hgt[kNB - 1];
#pragma unroll
  for (int j = 0; j < kNB - 1; ++j) hgt[j] = 0;
  constexpr bool kQuadPath = Scorer::kQuad && kPf == 4 && !kR;
  if constexpr (kQuadPath) {
    constexpr float kB[kNB - 1] = {1.f, 5.f, 10.f, 25.f, 50.f, 100.f, 250.f, 500.f, 1000.f, 2500.f,
                                   5000.f, 10000.f, 25000.f};
    while (tile < full_end) {
      float z[4], am[4];
      if constexpr (Scorer::kPair) {
        sc.logit2(lds, ring[0], ring[1], g, lane, z[0], z[1]);
        sc.logit2(lds, ring[2], ring[3], g, lane, z[2], z[3]);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) z[k] = sc.logit(lds, ring[k], g, lane);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        am[k] = __shfl(__uint_as_float(ring[k].v.w), 48 + c);     // Amount of row c of tile k
        issue(tile + (4 + k) * tstride, ring[k]);
      }
      const float zs = g == 0 ? z[0] : g == 1 ? z[1] : g == 2 ? z[2] : z[3];
      const float ams = g == 0 ? am[0] : g == 1 ? am[1] : g == 2 ? am[2] : am[3];
      const float p = sc.proba(zs);
      const int row = (tile + g * tstride) * kTileRows + c;
      const bool valid = row < n;
      const bool fr = valid && p >= thr;
      if (valid) {
        if (a.proba) st_g(a.proba + row, p);
        if (a.route) st_g(a.route + row, (uint8_t)(fr ? 1 : 0));
        psum += (unsigned)(p * 1e6f + 0.5f);
      }
      const unsigned long long frm = __ballot(fr);
      fraud += __popcll(frm);
      rows += __popcll(__ballot(valid));
      const float amv = valid ? ams : -__builtin_inff();
#pragma unroll
      for (int j = 0; j < kNB - 1; ++j) hgt[j] += __popcll(__ballot(amv > kB[j]));
      if (frm) {                                                  // rare: fraud rows' buckets
        if (fr) atomicAdd(&epi.hist[kNB + amount_bucket_fast(ams)], 1u);
        if (a.flags & CCFD_ARG_FLAG_DIRECT) emit_flagged(a, fr, row);
        else flag_push(a, fls, frm, fr, row, lane);
      }
      tile += 4 * tstride;
    }
  }
  while (!kQuadPath && tile < full_end) {
    if constexpr (Scorer::kPair && kPf % 2 == 0) {
#pragma unroll
      for (int k = 0; k < kPf; k += 2) {             // two tiles per scorer call (shared weight reads)
        const float am0 = __uint_as_float(ring[k].v.w), am1 = __uint_as_float(ring[k + 1].v.w);
        float p0, p1;
        sc.tile2(lds, ring[k], ring[k + 1], g, lane, p0, p1);
        const bool rf0 = rule_of(ring[k], p0);
        const bool rf1 = rule_of(ring[k + 1], p1);
        issue(tile + kPf * tstride, ring[k]);
        issue(tile + (kPf + 1) * tstride, ring[k + 1]);
        finish(p0, am0, tile, rf0);
        finish(p1, am1, tile + tstride, rf1);
        tile += 2 * tstride;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPf; ++k) {
        const float amount = __uint_as_float(ring[k].v.w);
        const float p = sc.tile(lds, ring[k], g, lane);
        const bool rf = rule_of(ring[k], p);
        issue(tile + kPf * tstride, ring[k]);
        finish(p, amount, tile, rf);
        tile += tstride;
      }
    }
  }
  // tail: fewer than kPf tiles left, already in flight in ring[0..]
#pragma unroll 1
  for (int k = 0; k < kPf && tile < ntiles; ++k) {
    const WireRegs cur = ring[0];
#pragma unroll
    for (int q = 0; q + 1 < kPf; ++q) ring[q] = ring[q + 1];
    const float p = sc.tile(lds, cur, g, lane);
    finish(p, __uint_as_float(cur.v.w), tile, rule_of(cur, p));
    tile += tstride;
  }
  if (a.flag_idx != nullptr) flag_flush(a, fls, lane);
  psum = wave_sum_u64(psum);
  hist_lanes_commit(epi, hl, g, c);
  if constexpr (kQuadPath) {
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < kNB - 1; ++j)
        if (hgt[j]) atomicAdd(&epi.hgt[j], hgt[j]);
    }
  }
  if (lane == 0) {
    atomicAdd(&epi.fraud, fraud);
    atomicAdd(&epi.rows, rows);
    atomicAdd(&epi.psum_e6, psum);
  }
  epi_flush_ballot(epi, a.counters);
  signal_done(a, (unsigned)nblk);
}

}  // namespace ccfd
