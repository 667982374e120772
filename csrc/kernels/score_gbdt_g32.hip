// Oblivious-GBDT scorer over G32 rows (BASELINE.json configs[3]: 100 trees x depth 6,
// batch 65536) -- the exact low-byte wire for tree ensembles.
//
// A tree only ever asks `x_f > thr`.  With the sorted split thresholds of feature f as bin
// edges, bin_f(x) = #{edges_f < x} and `x_f > edges_f[k]` <=> `bin_f(x) > k` for every float
// x (NaN -> bin 0 -> every test false, like the f32 compare).  So the ingest side stores one
// byte per feature (contracts/transaction.py G32: 30 bins, the amount bucket, a bin-table
// stamp) and the kernel compares bytes against per-split bin indices: 32 B per row instead
// of 120, i.e. 3.75x the rows per second through the same PCIe link, with bit-identical
// leaf choices (the leaf sums differ from the f32 kernel only in summation order).
//
// Layout: 256-thread workgroups; each wave owns 64-row chunks (one row per lane, grid-
// stride).  A chunk arrives as two contiguous 1 KB wave loads and is transposed through a
// wave-private LDS tile so that lane l holds row l; the next chunk is in flight while the
// current one is evaluated.  The 30 bins are lifted into 30 VGPRs once per row;
// a tree level is then v_movrel (wave-uniform feature id from an SGPR), v_sub against the
// SGPR bin index and v_alignbit (shift + bit), and the leaf value is gathered from the
// LDS-resident leaf tables.
#include <cstdlib>
#include <cstring>

#include <type_traits>

#include "common.h"
#include "persist_core.h"
#include "rules.h"

namespace ccfd {

constexpr int kG32Rows = 64;        // rows per wave chunk (one per lane)
constexpr int kG32Waves = 4;
constexpr int kG32LeafLds = 16384;  // floats: leaf tables up to 64 KB are staged in LDS, larger ones read from L2
#ifndef CCFD_G32_TREE_BLOCK
#define CCFD_G32_TREE_BLOCK 4
#endif
constexpr int kG32Tb = CCFD_G32_TREE_BLOCK;   // trees whose split parameters load together

struct G32Row { uint4 lo, hi; };

// One 64-row chunk is 2 KB.  Lane l fetches bytes [16l, 16l+16) and [1024+16l, 1024+16l+16):
// each load instruction is ONE contiguous 1 KB wave request (a row-per-lane load -- 32 B at
// a 32 B lane stride -- splits every instruction over the whole 2 KB and measured 0.6 of the
// zero-copy PCIe rate; the W64 kernels' contiguous tiles reach 0.99).  Bytes past the batch
// are clamped to its last 16 B (never scored; a score() tensor ends exactly there).
__device__ __forceinline__ void g32_fetch(const unsigned char* __restrict__ x, int n, int chunk, int lane,
                                          G32Row& r) {
  const long last = (long)n * CCFD_G32_ROW_BYTES - 16;
  const long b0 = (long)chunk * (kG32Rows * CCFD_G32_ROW_BYTES) + 16 * lane;
  r.lo = *reinterpret_cast<const uint4*>(x + min(b0, last));
  r.hi = *reinterpret_cast<const uint4*>(x + min(b0 + 1024, last));
}

// Wave-private LDS transpose: after it, lane l holds row l of the chunk (lo = bytes 0..15,
// hi = bytes 16..31).
__device__ __forceinline__ void g32_rows(uint4* __restrict__ t, int lane, G32Row& r) {
  t[lane] = r.lo;
  t[64 + lane] = r.hi;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  r.lo = t[2 * lane];
  r.hi = t[2 * lane + 1];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__device__ __forceinline__ unsigned g32_byte(const G32Row& r, int j) {   // j compile-time
  const unsigned w = j < 4 ? r.lo.x : j < 8 ? r.lo.y : j < 12 ? r.lo.z : j < 16 ? r.lo.w
                   : j < 20 ? r.hi.x : j < 24 ? r.hi.y : j < 28 ? r.hi.z : r.hi.w;
  return (w >> (8 * (j & 3))) & 0xffu;
}

typedef const __attribute__((address_space(4))) int* g32_cint_p;   // split params -> s_load

// Sum of the T trees' leaves for R row chains whose bins are lifted into b0 (/ b1).  Per
// level: the row's bin (v_movrel with the wave-uniform feature id), then
//   idx = (idx << 1) | (k - bin < 0)   ==   v_sub_u32 + v_alignbit_b32(idx, k - bin, 31)
// (bins and k are <= 255, so the sign bit of k - bin is exactly `bin > k`).  Plain C with
// no VCC / inline asm: the compiler interleaves the independent chains of the trees of a
// block, where a v_cmp + v_addc chain serialises every level on VCC.  Split parameters of
// kG32Tb trees are loaded per batch of scalar loads: one s_waitcnt per block.
template <int D, int R>
__device__ __forceinline__ void g32_trees(const unsigned (&b0)[kF], const unsigned (&b1)[kF],
                                          const float* __restrict__ lv, g32_cint_p feat, g32_cint_p kbin, int T,
                                          float (&acc)[R]) {
  constexpr int L = 1 << D;
#pragma unroll
  for (int q = 0; q < R; ++q) acc[q] = 0.f;
  auto tree = [&](int t, const int* fs, const int* ks) __attribute__((always_inline)) {
    unsigned i0 = 0, i1 = 0;
#pragma unroll
    for (int d = D - 1; d >= 0; --d) {                       // MSB first: bit d lands at position d
      const int f = fs[d];
      const unsigned k = (unsigned)ks[d];
      i0 = __builtin_amdgcn_alignbit(i0, k - b0[f], 31);
      if constexpr (R == 2) i1 = __builtin_amdgcn_alignbit(i1, k - b1[f], 31);
    }
    acc[0] += lv[t * L + (int)i0];
    if constexpr (R == 2) acc[R - 1] += lv[t * L + (int)i1];
  };
  int t = 0;
  for (; t + kG32Tb <= T; t += kG32Tb) {
    int fb[kG32Tb * D], kb[kG32Tb * D];
#pragma unroll
    for (int j = 0; j < kG32Tb * D; ++j) { fb[j] = feat[t * D + j]; kb[j] = kbin[t * D + j]; }
#pragma unroll
    for (int k = 0; k < kG32Tb; ++k) tree(t + k, fb + k * D, kb + k * D);
  }
  for (; t < T; ++t) {
    int fb[D], kb[D];
#pragma unroll
    for (int j = 0; j < D; ++j) { fb[j] = feat[t * D + j]; kb[j] = kbin[t * D + j]; }
    tree(t, fb, kb);
  }
}

// Lift a transposed row's 30 bins into registers; returns bytes 30..31 (bucket | stamp << 8).
__device__ __forceinline__ unsigned g32_lift(const G32Row& r, unsigned (&b)[kF]) {
#pragma unroll
  for (int j = 0; j < kF; ++j) b[j] = g32_byte(r, j);
  return r.hi.w >> 16;
}

// Stage the T * 2^D leaf table (blob section after feat / kbin) into LDS.
template <int D>
__device__ __forceinline__ void g32_stage_leaves(const char* blob, int T, float* lv, int tid, int nthreads) {
  constexpr int L = 1 << D;
  const int tdw = ((4 * T * D + 15) & ~15) / 4;
  const float* src = reinterpret_cast<const float*>(blob + kHeader + 8 * tdw);
  const float4* s4 = reinterpret_cast<const float4*>(src);
  float4* d4 = reinterpret_cast<float4*>(lv);
  const int nl = T * L;
  for (int i = tid; i < nl / 4; i += nthreads) d4[i] = s4[i];
  for (int i = (nl & ~3) + tid; i < nl; i += nthreads) lv[i] = src[i];
}

// Leaf tables of T * 2^D floats up to kG32LeafLds are staged in LDS; larger ensembles
// (kGL: e.g. CatBoost's default 1000 x depth 6 = 250 KB) gather their leaves straight from
// the blob in global memory -- read-only and L2-resident, one gather per tree and row chain.
__device__ __forceinline__ const float* g32_leaves_global(const char* blob, int T, int D) {
  const int tdw = ((4 * T * D + 15) & ~15) / 4;
  return reinterpret_cast<const float*>(blob + kHeader + 8 * tdw);
}

template <int D, int R, bool kR, bool kGL>
__global__ __launch_bounds__(256) void score_gbdt_g32_kernel(ccfd_score_args a) {
  extern __shared__ __attribute__((aligned(16))) float lv[];   // T * L floats
  __shared__ uint4 xt[kG32Waves][128];                         // per-wave chunk transpose
  __shared__ EpilogueLds epi;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = a.n;
  const int nchunks = (n + kG32Rows - 1) / kG32Rows;
  const int ngroups = (nchunks + R - 1) / R;                  // R chunks per wave step
  const int gstride = gridDim.x * kG32Waves;
  int grp = blockIdx.x * kG32Waves + wave;
  const unsigned char* __restrict__ xb = reinterpret_cast<const unsigned char*>(a.x);

  // rows first: the host-memory latency overlaps the leaf staging below
  G32Row pre[R];
#pragma unroll
  for (int q = 0; q < R; ++q) g32_fetch(xb, n, grp * R + q, lane, pre[q]);

  epi_init(epi);
  stamp_start(a, blockIdx.x);
  const char* blob = reinterpret_cast<const char*>(a.blob);
  const int T = a.gbdt_trees;
  const float base = *reinterpret_cast<const float*>(blob + 16);
  const unsigned stamp = (unsigned)*reinterpret_cast<const int*>(blob + 20);
  const int tdw = ((4 * T * D + 15) & ~15) / 4;
  // split parameters through the CONSTANT address space: wave-uniform indices compile to
  // s_load into SGPRs (the model blob is immutable for the kernel's lifetime)
  const g32_cint_p feat = (g32_cint_p)(blob + kHeader);
  const g32_cint_p kbin = (g32_cint_p)(blob + kHeader + 4 * tdw);
  const float* leaves = lv;
  if constexpr (kGL) leaves = g32_leaves_global(blob, T, D);
  else g32_stage_leaves<D>(blob, T, lv, tid, 256);
  __syncthreads();                                              // leaves staged, epi initialised

  const bool store_out = !(a.flags & CCFD_ARG_ABLATE_OUTPUTS);
  unsigned fraud = 0, rows = 0, stale = 0;
  unsigned long long psum = 0;
  for (; grp < ngroups; grp += gstride) {
    // separate 1-D arrays per row chain: indexed by a runtime (wave-uniform) feature id they
    // stay in VGPRs (v_movrel); a 2-D array would be demoted to scratch
    unsigned b0[kF], b1[kF];
    unsigned meta[R];                                           // bytes 30, 31: bucket, stamp
    G32Row cur = pre[0];
    g32_rows(xt[wave], lane, cur);
    meta[0] = g32_lift(cur, b0);
    if constexpr (R == 2) {
      cur = pre[1];
      g32_rows(xt[wave], lane, cur);
      meta[1] = g32_lift(cur, b1);
    }
    const int nxt = grp + gstride;
    if (nxt < ngroups) {
#pragma unroll
      for (int q = 0; q < R; ++q) g32_fetch(xb, n, nxt * R + q, lane, pre[q]);
    }
    float acc[R];
    g32_trees<D, R>(b0, b1, leaves, feat, kbin, T, acc);
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int row = (grp * R + q) * kG32Rows + lane;
      const bool valid = row < n;
      const bool fresh = ((meta[q] >> 8) & 0xffu) == stamp;
      const float p = fresh ? sigmoid(base + acc[q]) : __builtin_nanf("");
      bool fr;
      if constexpr (kR) fr = valid && fresh && rule_route(a.rules, p, [](int) { return 0.f; });
      else fr = valid && fresh && (p >= a.threshold);
      if (valid) {
        if (store_out) {
          if (a.proba) a.proba[row] = p;
          if (a.route) a.route[row] = fr ? 1 : 0;
        }
        if (fresh) psum += (unsigned)(p * 1e6f + 0.5f);
        atomicAdd(&epi.hist[(fr ? kNB : 0) + min((int)(meta[q] & 0xffu), kNB - 1)], 1u);
      }
      fraud += __popcll(__ballot(fr));
      rows += __popcll(__ballot(valid));
      stale += __popcll(__ballot(valid && !fresh));
      emit_flagged(a, fr, row);
    }
  }
  psum = wave_sum_u64(psum);
  if (lane == 0) {
    atomicAdd(&epi.fraud, fraud);
    atomicAdd(&epi.rows, rows);
    atomicAdd(&epi.psum_e6, psum);
  }
  unsigned long long* cnt = (a.flags & CCFD_ARG_ABLATE_COUNTERS) ? nullptr : a.counters;
  if (cnt != nullptr && lane == 0 && stale) atomicAdd(&cnt[CCFD_CNT_WIRE_STALE], (unsigned long long)stale);
  epi_flush(epi, cnt);
  signal_done(a, gridDim.x);
}

// ---------------------------------------------------------------------------------------
// Persistent variant (engine exec_mode = 1; protocol in persist_core.h).  The leaf tables
// are staged into LDS ONCE per resident workgroup (a launch per micro-batch re-stages them
// in every workgroup), and a claimed item is 4 waves x `cpw` 64-row chunks, the next chunk
// of a wave in flight while the current one is evaluated.
// ---------------------------------------------------------------------------------------
template <int D, bool kR, bool kGL>
__global__ __launch_bounds__(256) void persist_gbdt_g32_kernel(ccfd_persist_args a) {
  extern __shared__ __attribute__((aligned(16))) float lv[];   // T * L floats
  __shared__ uint4 xt[kG32Waves][128];
  __shared__ EpilogueLds epi;
  __shared__ ccfd_persist_desc sdesc;
  __shared__ unsigned long long s_item;
  __shared__ int s_cmd;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int C = a.items_per_batch;
  const int cpw = a.tiles_per_wave;                       // 64-row chunks per wave per item
  if (blockIdx.x == 0) {                                  // doorbell (persist_core.h)
    if (wave == 0) persist_doorbell(a, lane);
    return;                                               // no barrier is ever used by WG 0
  }
  const char* blob = reinterpret_cast<const char*>(a.blob);
  const int T = a.gbdt_trees;
  const float base = *reinterpret_cast<const float*>(blob + 16);
  const unsigned stamp = (unsigned)*reinterpret_cast<const int*>(blob + 20);
  const int tdw = ((4 * T * D + 15) & ~15) / 4;
  const g32_cint_p feat = (g32_cint_p)(blob + kHeader);
  const g32_cint_p kbin = (g32_cint_p)(blob + kHeader + 4 * tdw);
  const float* leaves = lv;
  if constexpr (kGL) leaves = g32_leaves_global(blob, T, D);
  else g32_stage_leaves<D>(blob, T, lv, tid, 256);
  epi_init(epi);
  __syncthreads();
  unsigned long long posted_cache = 0;                    // thread 0 only

  for (;;) {
    if (tid == 0) persist_claim(a, C, posted_cache, sdesc, s_item, s_cmd);
    __syncthreads();
    if (s_cmd) break;
    const int item = (int)(s_item % (unsigned long long)C);
    const int slot = (int)(sdesc.seq % (unsigned long long)a.ring);
    const int n = sdesc.n;
    const unsigned char* xb = reinterpret_cast<const unsigned char*>(sdesc.x);
    if (item == 0 && tid == 0)                            // K7: micro-batch start (item 0 claimed first)
      __hip_atomic_store(&a.dev->tstart[slot], wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int c0 = item * (kG32Waves * cpw) + wave;       // this wave's chunks: c0 + 4k
    unsigned fraud = 0, rows = 0, stale = 0;
    unsigned long long psum = 0;
    auto score_chunk = [&](int chunk, G32Row& cur) __attribute__((always_inline)) {
      g32_rows(xt[wave], lane, cur);
      unsigned b0[kF];
      const unsigned meta = g32_lift(cur, b0);
      float acc[1];
      g32_trees<D, 1>(b0, b0, leaves, feat, kbin, T, acc);
      const int row = chunk * kG32Rows + lane;
      const bool valid = row < n;
      const bool fresh = ((meta >> 8) & 0xffu) == stamp;
      const float p = fresh ? sigmoid(base + acc[0]) : __builtin_nanf("");
      bool fr;
      if constexpr (kR) fr = valid && fresh && rule_route(a.rules, p, [](int) { return 0.f; });
      else fr = valid && fresh && (p >= a.threshold);
      if (valid) {
        if (sdesc.proba) sdesc.proba[row] = p;
        if (sdesc.route) sdesc.route[row] = fr ? 1 : 0;
        if (fresh) psum += (unsigned)(p * 1e6f + 0.5f);
        atomicAdd(&epi.hist[(fr ? kNB : 0) + min((int)(meta & 0xffu), kNB - 1)], 1u);
      }
      const unsigned long long m = __ballot(fr);
      fraud += __popcll(m);
      rows += __popcll(__ballot(valid));
      stale += __popcll(__ballot(valid && !fresh));
      persist_emit_flagged(a, sdesc, slot, m, fr, row, lane);
    };
    // CCFD_G32_INFLIGHT=1: every chunk of the wave's share of the item in flight at once
    // (static registers: no copy of a pending load, so no vmcnt(0) between chunks)
    auto full_item = [&](auto kC) __attribute__((always_inline)) {
      constexpr int CPW = decltype(kC)::value;
      G32Row r[CPW];
#pragma unroll
      for (int k = 0; k < CPW; ++k) {
        const int chunk = c0 + kG32Waves * k;
        if (chunk * kG32Rows < n) g32_fetch(xb, n, chunk, lane, r[k]);
      }
#pragma unroll
      for (int k = 0; k < CPW; ++k) {
        const int chunk = c0 + kG32Waves * k;
        if (chunk * kG32Rows >= n) break;                 // wave-uniform
        score_chunk(chunk, r[k]);
      }
    };
    if (a.flags & CCFD_ARG_CHUNK_RING) {                  // default: one chunk ahead
      G32Row pre;
      if (c0 * kG32Rows < n) g32_fetch(xb, n, c0, lane, pre);
#pragma unroll 1
      for (int k = 0; k < cpw; ++k) {
        const int chunk = c0 + kG32Waves * k;
        if (chunk * kG32Rows >= n) break;                 // wave-uniform
        G32Row cur = pre;
        if (k + 1 < cpw && (chunk + kG32Waves) * kG32Rows < n) g32_fetch(xb, n, chunk + kG32Waves, lane, pre);
        score_chunk(chunk, cur);
      }
    } else if (cpw == 1) {
      full_item(std::integral_constant<int, 1>{});
    } else if (cpw == 2) {
      full_item(std::integral_constant<int, 2>{});
    } else {
      full_item(std::integral_constant<int, 4>{});        // 1024-row items (engine accepts 256/512/1024)
    }
    psum = wave_sum_u64(psum);
    if (lane == 0 && rows) {
      atomicAdd(&epi.fraud, fraud);
      atomicAdd(&epi.rows, rows);
      atomicAdd(&epi.psum_e6, psum);
      unsigned long long* cnt = a.counters[sdesc.epoch & 1];
      if (stale && cnt) atomicAdd(&cnt[CCFD_CNT_WIRE_STALE], (unsigned long long)stale);
    }
    persist_item_done(a, epi, sdesc, slot, C, tid);
  }
}

template <int D>
static int launch_persist_g32_d(const ccfd_persist_args& a0, int grid, hipStream_t s) {
  ccfd_persist_args a = a0;
  // one-chunk prefetch ring by default: at BASELINE config 4 (65536-row batches) it measured
  // 1.67e9 tx/s at p50 107 us (depth 3) vs 1.64e9 with the whole item in flight (VALU-heavy
  // trees overlap the next chunk's load better); CCFD_G32_INFLIGHT=1 selects the latter.
  // Read per launch: sweepable in-process (profiles/r2/persist_full_item/g32_inflight_ab.jsonl)
  const char* e = getenv("CCFD_G32_INFLIGHT");
  if (!e || atoi(e) == 0) a.flags |= CCFD_ARG_CHUNK_RING;
  const char* eg = getenv("CCFD_G32_GLOBAL_LEAVES");              // A/B knob: force the L2 path
  const bool gl = ((long)a.gbdt_trees << D) > kG32LeafLds || (eg && atoi(eg) == 1);
  const size_t lds = gl ? 0 : (size_t)a.gbdt_trees * (1 << D) * sizeof(float);
  if (gl) {
    if (a.rules) hipLaunchKernelGGL((persist_gbdt_g32_kernel<D, true, true>), dim3(grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((persist_gbdt_g32_kernel<D, false, true>), dim3(grid), dim3(256), 0, s, a);
  } else {
    if (a.rules) hipLaunchKernelGGL((persist_gbdt_g32_kernel<D, true, false>), dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL((persist_gbdt_g32_kernel<D, false, false>), dim3(grid), dim3(256), lds, s, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_persist_gbdt_g32(const ccfd_persist_args& a, int grid, hipStream_t s) {
  if (a.gbdt_trees <= 0 || a.gbdt_depth < 1 || a.gbdt_depth > 8) return -2;
  switch (a.gbdt_depth) {
    case 1: return launch_persist_g32_d<1>(a, grid, s);
    case 2: return launch_persist_g32_d<2>(a, grid, s);
    case 3: return launch_persist_g32_d<3>(a, grid, s);
    case 4: return launch_persist_g32_d<4>(a, grid, s);
    case 5: return launch_persist_g32_d<5>(a, grid, s);
    case 6: return launch_persist_g32_d<6>(a, grid, s);
    case 7: return launch_persist_g32_d<7>(a, grid, s);
    default: return launch_persist_g32_d<8>(a, grid, s);
  }
}

// Grid: one wave per R-chunk group, capped at CCFD_G32_WGS_PER_CU workgroups per CU (grid-
// stride beyond).  A 65536-row micro-batch is 1024 chunks = 256 workgroups at R = 1: every
// CU has its rows in flight at once.  CCFD_G32_R: 64-row chunks per wave step (1 | 2).
static int g32_env(const char* name, int dflt, int lo, int hi) {
  const char* e = getenv(name);
  if (!e) return dflt;
  const int v = atoi(e);
  return v < lo || v > hi ? dflt : v;
}

template <int D, int R>
static void launch_g32_r(const ccfd_score_args& a, hipStream_t s) {
  constexpr int L = 1 << D;
  const int wgs_per_cu = g32_env("CCFD_G32_WGS_PER_CU", 4, 1, 8);   // read per launch: sweepable in-process
  const int nchunks = (a.n + kG32Rows - 1) / kG32Rows;
  const int ngroups = (nchunks + R - 1) / R;
  int grid = (ngroups + kG32Waves - 1) / kG32Waves;
  const int cap = 256 * wgs_per_cu;
  grid = grid < 1 ? 1 : (grid > cap ? cap : grid);
  // a launch re-stages the leaves in every workgroup: past 32 KB of leaves the L2 gather wins
  // (250 x 6 at 1 M rows: 5.3 vs 4.0 G rows/s; 100 x 6: LDS 14.2 vs 13.1 at 16 M rows,
  // profiles/r2/g32_large_ensembles/lds_vs_global_*.jsonl)
  const bool gl = ((long)a.gbdt_trees << D) > kG32LeafLds / 2 || g32_env("CCFD_G32_GLOBAL_LEAVES", 0, 0, 1);
  const size_t lds = gl ? 0 : (size_t)a.gbdt_trees * L * sizeof(float);
  if (gl) {
    if (a.rules) hipLaunchKernelGGL((score_gbdt_g32_kernel<D, R, true, true>), dim3(grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((score_gbdt_g32_kernel<D, R, false, true>), dim3(grid), dim3(256), 0, s, a);
  } else {
    if (a.rules) hipLaunchKernelGGL((score_gbdt_g32_kernel<D, R, true, false>), dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL((score_gbdt_g32_kernel<D, R, false, false>), dim3(grid), dim3(256), lds, s, a);
  }
}

template <int D>
static void launch_g32_d(const ccfd_score_args& a, hipStream_t s) {
  const int r = g32_env("CCFD_G32_R", 1, 1, 2);
  if (r == 2) launch_g32_r<D, 2>(a, s);
  else launch_g32_r<D, 1>(a, s);
}

int launch_gbdt_g32(const ccfd_score_args& a, hipStream_t s) {
  if (a.gbdt_trees <= 0 || a.gbdt_depth < 1 || a.gbdt_depth > 8) return -2;
  if (a.n <= 0) return 0;
  switch (a.gbdt_depth) {
    case 1: launch_g32_d<1>(a, s); break;
    case 2: launch_g32_d<2>(a, s); break;
    case 3: launch_g32_d<3>(a, s); break;
    case 4: launch_g32_d<4>(a, s); break;
    case 5: launch_g32_d<5>(a, s); break;
    case 6: launch_g32_d<6>(a, s); break;
    case 7: launch_g32_d<7>(a, s); break;
    default: launch_g32_d<8>(a, s); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace ccfd
