// Oblivious-GBDT scorer (BASELINE.json configs[3]: 100 trees x depth 6, batch 65536).
//
// In an oblivious tree every level tests one (feature, threshold) pair, identical for
// every row, so for a wave walking the SAME tree the split parameters are wave-uniform:
// they come from scalar loads into SGPRs, and a row's leaf index is D compares + shifts.
// Layout per 256-thread workgroup:
//   * 64 rows staged FEATURE-MAJOR in LDS (xs[30][64]): lane r reads xs[f][r] with f
//     uniform -> consecutive lanes hit consecutive banks (conflict-free ds_read_b32);
//   * the leaf tables of a chunk of trees staged in LDS (<= 64 KB per chunk; once per
//     workgroup when they fit);
//   * each workgroup walks several 64-row chunks with the next chunk prefetched (below);
//   * the 4 waves split the trees (wave w takes trees w, w+4, ...) over the same 64 rows,
//     so each SIMD has independent leaf-gather chains in flight; partial sums are reduced
//     through LDS, then sigmoid + threshold + counters as in the other scorers.
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "rules.h"

namespace ccfd {

constexpr int kGbRows = 64;
constexpr int kGbWaves = 4;
constexpr int kLeafLds = 16384;     // floats of leaf table per chunk (64 KB)
constexpr int kGbF4 = kGbRows * kF / 4;   // 480 float4 per 64-row chunk

// Register-staged copy of one 64-row chunk (contiguous rows): thread t owns float4 t and
// t + 256 of the chunk's 7680 bytes.
struct GbRegs { float4 v[2]; };

__device__ __forceinline__ void gb_issue(const float* __restrict__ x, int row0, int nrows, int tid, GbRegs& r) {
  const int avail = nrows * kF * 4;
  const float4* src = reinterpret_cast<const float4*>(x + (size_t)row0 * kF);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = tid + 256 * k;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < kGbF4) {
      if (i * 16 + 16 <= avail) v = src[i];
      else if (i * 16 + 8 <= avail) { const float2 h = reinterpret_cast<const float2*>(src)[2 * i]; v.x = h.x; v.y = h.y; }
    }
    r.v[k] = v;
  }
}

__device__ __forceinline__ void gb_store(float (*xs)[kGbRows], int tid, const GbRegs& r) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = tid + 256 * k;
    if (i < kGbF4) {
      const int e = 4 * i;
      const float vv[4] = {r.v[k].x, r.v[k].y, r.v[k].z, r.v[k].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) { const int ee = e + q; xs[ee % kF][ee / kF] = vv[q]; }
    }
  }
}

// Each workgroup scores `cpw` consecutive 64-row chunks.  Chunk c+1's rows are fetched into
// registers while chunk c is evaluated, so a workgroup always has host reads in flight, and
// a grid of ~2 workgroups per CU leaves room for the next micro-batch's kernel to start
// fetching before this one drains (one workgroup per chunk filled every CU slot with
// workgroups waiting on PCIe and serialised consecutive batches).  The leaf tables are
// staged into LDS once per workgroup when they fit (T * 2^D <= 16384 floats).
template <int D, bool kContig, bool kR>
__global__ __launch_bounds__(256) void score_gbdt_kernel(ccfd_score_args a, int cpw) {
  constexpr int L = 1 << D;
  __shared__ __attribute__((aligned(16))) float xs[kF][kGbRows];
  extern __shared__ __attribute__((aligned(16))) float lv[];   // min(T, kLeafLds/L) * L floats
  __shared__ float part[kGbWaves][kGbRows];
  __shared__ EpilogueLds epi;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nchunks = (a.n + kGbRows - 1) / kGbRows;
  const int c_begin = blockIdx.x * cpw;
  const int c_end = min(nchunks, c_begin + cpw);
  epi_init(epi);
  stamp_start(a, blockIdx.x);

  const char* blob = reinterpret_cast<const char*>(a.blob);
  const int T = a.gbdt_trees;
  const float base = *reinterpret_cast<const float*>(blob + 16);
  const int* __restrict__ feat = reinterpret_cast<const int*>(blob + kHeader);
  const int tdw = ((4 * T * D + 15) & ~15) / 4;
  const float* __restrict__ thr = reinterpret_cast<const float*>(blob + kHeader) + tdw;
  const float* __restrict__ leaves = thr + tdw;
  const int kChunk = min(T, kLeafLds / L);
  const bool resident = kChunk == T;

  GbRegs cur, nxt;
  if constexpr (kContig)
    if (c_begin < c_end) gb_issue(a.x, c_begin * kGbRows, min(kGbRows, a.n - c_begin * kGbRows), tid, cur);

  auto stage_leaves = [&](int c0, int c1) {
    const int nl = (c1 - c0) * L;
    if constexpr (L >= 4) {
      const float4* s4 = reinterpret_cast<const float4*>(leaves + (size_t)c0 * L);
      float4* d4 = reinterpret_cast<float4*>(lv);
      for (int i = tid; i < nl / 4; i += 256) d4[i] = s4[i];
    } else {
      for (int i = tid; i < nl; i += 256) lv[i] = leaves[(size_t)c0 * L + i];
    }
  };
  if (resident) stage_leaves(0, T);    // made visible by the first loop barrier

  for (int c = c_begin; c < c_end; ++c) {
    const int row0 = c * kGbRows;
    const int nrows = min(kGbRows, a.n - row0);
    __syncthreads();   // previous chunk's xs / part readers are done
    if constexpr (kContig) {
      if (c + 1 < c_end) gb_issue(a.x, row0 + kGbRows, min(kGbRows, a.n - row0 - kGbRows), tid, nxt);
      gb_store(xs, tid, cur);
    } else {
      for (int e = tid; e < kGbRows * kF; e += 256) {
        const int r = e / kF, f = e % kF;
        xs[f][r] = (r < nrows) ? a.x[(size_t)(row0 + r) * a.ld + f] : 0.f;
      }
    }

    float acc = 0.f;
    for (int c0 = 0; c0 < T; c0 += kChunk) {
      const int c1 = min(T, c0 + kChunk);
      if (!resident) {
        __syncthreads();   // previous tree chunk consumed
        stage_leaves(c0, c1);
      }
      __syncthreads();     // rows (and leaves) staged
      for (int t = c0 + wave; t < c1; t += kGbWaves) {
        int idx = 0;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const int f = feat[t * D + d];          // wave-uniform -> s_load
          const float th = thr[t * D + d];
          idx |= (xs[f][lane] > th ? 1 : 0) << d;
        }
        acc += lv[(t - c0) * L + idx];
      }
    }
    part[wave][lane] = acc;
    __syncthreads();

    if (wave == 0) {
      const float z = base + part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
      const float p = sigmoid(z);
      const bool valid = lane < nrows;
      // configurable routing rules: row = lane, its features are column xs[*][lane]
      bool fr;
      if constexpr (kR) fr = valid && rule_route(a.rules, p, [&](int j) { return xs[j][lane]; });
      else fr = valid && (p >= a.threshold);
      const int row = row0 + lane;
      if (valid) {
        if (a.proba) st_g(a.proba + row, p);
        if (a.route) st_g(a.route + row, (uint8_t)(fr ? 1 : 0));
        atomicAdd(&epi.hist[(fr ? kNB : 0) + amount_bucket(xs[kAmountCol][lane])], 1u);
      }
      unsigned long long ps = valid ? (unsigned long long)(p * 1e6f + 0.5f) : 0ull;
      ps = wave_sum_u64(ps);
      const unsigned nf = __popcll(__ballot(fr));
      if (lane == 0) { epi.fraud += nf; epi.rows += nrows; epi.psum_e6 += ps; }
      emit_flagged(a, fr, row);
    }
    if constexpr (kContig) cur = nxt;
  }
  epi_flush(epi, a.counters);
  signal_done(a, gridDim.x);
}


// ---------------------------------------------------------------------------------------
// v2: rows in registers (contiguous rows whose leaf tables fit in LDS -- the common case).
// Each WAVE owns its own 64-row chunks (R chunks at a time, R = 2 -> two independent row
// chains per lane): the chunk is fetched with coalesced float4 loads (also right for a
// host-mapped log over PCIe), transposed through a wave-private LDS tile, and every lane
// lifts ITS row's 30 features into VGPRs once.  A tree level is then three VALU -- the
// wave-uniform feature id indexes the register file (s_set_gpr_idx + v_mov), one compare
// against the SGPR threshold, one add-with-carry that shifts the leaf index and adds the
// bit -- instead of an LDS read per level; only the leaf value is gathered from LDS.  All
// trees run in every wave (no cross-wave partial sums).  The next chunk group is prefetched
// into registers while the current one is scored.  (v1 above is kept for strided rows and
// for ensembles whose leaves exceed 64 KB.)
// ---------------------------------------------------------------------------------------
constexpr int kGb2Waves = 4;
#ifndef CCFD_GBDT_TREE_BLOCK
#define CCFD_GBDT_TREE_BLOCK 4
#endif
constexpr int kGbTb = CCFD_GBDT_TREE_BLOCK;    // trees whose split parameters are loaded together

template <int D, int R, bool kR>
__global__ __launch_bounds__(256) void score_gbdt_v2_kernel(ccfd_score_args a) {
  constexpr int L = 1 << D;
  __shared__ __attribute__((aligned(16))) float xs[kGb2Waves][kF][kGbRows + 1];
  extern __shared__ __attribute__((aligned(16))) float lv[];   // T * L floats
  __shared__ EpilogueLds epi;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = a.n;
  const int nchunks = (n + kGbRows - 1) / kGbRows;
  const int ngroups = (nchunks + R - 1) / R;                  // R chunks per wave step
  const int gstride = gridDim.x * kGb2Waves;
  int grp = blockIdx.x * kGb2Waves + wave;
  epi_init(epi);
  stamp_start(a, blockIdx.x);

  const char* blob = reinterpret_cast<const char*>(a.blob);
  const int T = a.gbdt_trees;
  const float base = *reinterpret_cast<const float*>(blob + 16);
  const int tdw = ((4 * T * D + 15) & ~15) / 4;
  // split parameters through the CONSTANT address space: wave-uniform indices then compile
  // to s_load into SGPRs (the model blob is immutable for the kernel's lifetime)
  typedef const __attribute__((address_space(4))) int* cint_p;
  typedef const __attribute__((address_space(4))) float* cflt_p;
  const cint_p feat = (cint_p)(blob + kHeader);
  const cflt_p thr = (cflt_p)(blob + kHeader + 4 * tdw);
  const float* __restrict__ leaves = reinterpret_cast<const float*>(blob + kHeader) + 2 * tdw;
  {
    const float4* s4 = reinterpret_cast<const float4*>(leaves);
    float4* d4 = reinterpret_cast<float4*>(lv);
    for (int i = tid; i < T * L / 4; i += 256) d4[i] = s4[i];
  }

  // one 64-row chunk = 480 float4; lane l holds float4 l + 64k (k < 8)
  auto fetch = [&](int chunk, float4 (&r)[8]) __attribute__((always_inline)) {
    const int row0 = chunk * kGbRows;
    const int avail = max(0, min(kGbRows, n - row0)) * kF * 4;
    const float4* src = reinterpret_cast<const float4*>(a.x + (size_t)row0 * kF);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = lane + 64 * k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < kGbF4) {
        if (i * 16 + 16 <= avail) v = src[i];
        else if (i * 16 + 8 <= avail) { const float2 h = reinterpret_cast<const float2*>(src)[2 * i]; v.x = h.x; v.y = h.y; }
      }
      r[k] = v;
    }
  };
  auto lift = [&](const float4 (&r)[8], float (&x)[kF]) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = lane + 64 * k;
      if (i < kGbF4) {
        const float vv[4] = {r[k].x, r[k].y, r[k].z, r[k].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) { const int e = 4 * i + q; xs[wave][e % kF][e / kF] = vv[q]; }
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int f = 0; f < kF; ++f) x[f] = xs[wave][f][lane];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  };

  float4 pre[R][8];
#pragma unroll
  for (int q = 0; q < R; ++q) fetch(grp * R + q, pre[q]);
  __syncthreads();                                            // leaves staged

  unsigned fraud = 0, rows = 0;
  unsigned long long psum = 0;
  for (; grp < ngroups; grp += gstride) {
    // separate arrays per row chain: a 2-D register array indexed by a runtime feature id
    // is demoted to scratch, two 1-D ones stay in VGPRs (s_set_gpr_idx)
    float x0[kF], x1[kF];
    lift(pre[0], x0);
    if constexpr (R == 2) lift(pre[1], x1);
    const int nxt = grp + gstride;
    if (nxt < ngroups) {
#pragma unroll
      for (int q = 0; q < R; ++q) fetch(nxt * R + q, pre[q]);
    }
    float acc[R];
#pragma unroll
    for (int q = 0; q < R; ++q) acc[q] = 0.f;
    // one tree: D levels of (s_set_gpr_idx + v_mov, v_cmp, v_addc) per row chain, then the
    // leaf gathered from LDS
    auto tree = [&](int t, const int* fs, const float* ths) __attribute__((always_inline)) {
      unsigned i0 = 0, i1 = 0;
#pragma unroll
      for (int d = D - 1; d >= 0; --d) {                       // MSB first: bit d lands at position d
        const int f = fs[d];
        const float th = ths[d];
        const float v0 = x0[f];                                 // s_set_gpr_idx + v_mov
        asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2\n"
                     "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
                     : "+v"(i0) : "s"(th), "v"(v0) : "vcc");
        if constexpr (R == 2) {
          const float v1 = x1[f];
          asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2\n"
                       "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
                       : "+v"(i1) : "s"(th), "v"(v1) : "vcc");
        }
      }
      acc[0] += lv[t * L + (int)i0];
      if constexpr (R == 2) acc[R - 1] += lv[t * L + (int)i1];
    };
    // Split parameters of kGbTb trees at a time: one batch of s_load_dwordx8/x16 and ONE
    // s_waitcnt per block instead of two scalar-load round trips per tree (scalar loads
    // return out of order, so every wait is lgkmcnt(0) and nothing else hides it at the
    // 2 waves/SIMD this kernel's LDS footprint allows).
    int t = 0;
    for (; t + kGbTb <= T; t += kGbTb) {
      int fb[kGbTb * D];
      float tb[kGbTb * D];
#pragma unroll
      for (int j = 0; j < kGbTb * D; ++j) { fb[j] = feat[t * D + j]; tb[j] = thr[t * D + j]; }
#pragma unroll
      for (int k = 0; k < kGbTb; ++k) tree(t + k, fb + k * D, tb + k * D);
    }
    for (; t < T; ++t) {
      int fb[D];
      float tb[D];
#pragma unroll
      for (int j = 0; j < D; ++j) { fb[j] = feat[t * D + j]; tb[j] = thr[t * D + j]; }
      tree(t, fb, tb);
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int row = (grp * R + q) * kGbRows + lane;
      const bool valid = row < n;
      const float p = sigmoid(base + acc[q]);
      bool fr;
      if constexpr (kR) fr = valid && rule_route(a.rules, p, [&](int j) { return q == 0 ? x0[j] : x1[j]; });
      else fr = valid && (p >= a.threshold);
      if (valid) {
        if (a.proba) st_g(a.proba + row, p);
        if (a.route) st_g(a.route + row, (uint8_t)(fr ? 1 : 0));
        psum += (unsigned)(p * 1e6f + 0.5f);
        atomicAdd(&epi.hist[(fr ? kNB : 0) + amount_bucket_fast(q == 0 ? x0[kAmountCol] : x1[kAmountCol])], 1u);
      }
      fraud += __popcll(__ballot(fr));
      rows += __popcll(__ballot(valid));
      emit_flagged(a, fr, row);
    }
  }
  psum = wave_sum_u64(psum);
  if (lane == 0) {
    atomicAdd(&epi.fraud, fraud);
    atomicAdd(&epi.rows, rows);
    atomicAdd(&epi.psum_e6, psum);
  }
  epi_flush(epi, a.counters);
  signal_done(a, gridDim.x);
}

// Kernel choice.  v2 wins on large launches (HBM-resident bulk scoring: 2.6 -> 8.8 G rows/s
// at 16M rows, profiles/r1/gbdt_v2_sweep.jsonl); on streaming micro-batches (<= 64K rows read
// zero-copy over PCIe) v1's smaller LDS footprint keeps more workgroups -- i.e. more PCIe
// reads -- in flight (408 vs 345 M tx/s), so v1 stays the default below kGbV2MinRows.
// CCFD_GBDT_KERNEL=v1|v2 forces one; CCFD_GBDT_R: 64-row chunks per wave step (1|2).
constexpr int kGbV2MinRows = 262144;
static int gbdt_v2_rows() {
  static const int r = [] {
    const char* e = getenv("CCFD_GBDT_R");
    return (e && atoi(e) == 1) ? 1 : 2;          // R = 2 measured best (8.8 vs 7.1 G rows/s)
  }();
  return r;
}
static int gbdt_forced_kernel() {   // 0 = by size, 1 = v1, 2 = v2
  static const int v = [] {
    const char* e = getenv("CCFD_GBDT_KERNEL");
    return !e ? 0 : strcmp(e, "v1") == 0 ? 1 : strcmp(e, "v2") == 0 ? 2 : 0;
  }();
  return v;
}

template <int D, int R, bool kR>
static void launch_v2(const ccfd_score_args& a, hipStream_t s) {
  constexpr int L = 1 << D;
  const int nchunks = (a.n + kGbRows - 1) / kGbRows;
  const int ngroups = (nchunks + R - 1) / R;
  int grid = (ngroups + kGb2Waves - 1) / kGb2Waves;
  const int cap = 256 * 2;                 // two resident workgroups per CU (LDS: staging + leaves)
  grid = grid < 1 ? 1 : (grid > cap ? cap : grid);
  const size_t lds = (size_t)a.gbdt_trees * L * sizeof(float);
  hipLaunchKernelGGL((score_gbdt_v2_kernel<D, R, kR>), dim3(grid), dim3(256), lds, s, a);
}

template <int D>
static void launch_d2(const ccfd_score_args& a, hipStream_t s) {
  const bool r = a.rules != nullptr;
  if (gbdt_v2_rows() == 1) { if (r) launch_v2<D, 1, true>(a, s); else launch_v2<D, 1, false>(a, s); }
  else { if (r) launch_v2<D, 2, true>(a, s); else launch_v2<D, 2, false>(a, s); }
}

// CCFD_GBDT_CPW: 64-row chunks per workgroup.  Default: a ~256-workgroup grid (one per CU;
// 4 chunks each on a 65536-row micro-batch).  Measured on MI355X, 100x6 trees, 65536-row
// batches (profiles/r1/gbdt_sweep.txt): 1 chunk/WG 348M tx/s, 2 -> 368M, 4 -> 412M,
// 8 -> 408M, 16 -> 395M.
static int gbdt_chunks_per_wg(int nchunks) {
  static const int env = [] {
    const char* e = getenv("CCFD_GBDT_CPW");
    return e ? atoi(e) : 0;
  }();
  if (env > 0) return env;
  const int target_wgs = 256;
  return max(1, (nchunks + target_wgs - 1) / target_wgs);
}

template <int D>
static void launch_d(const ccfd_score_args& a, hipStream_t s, bool contig) {
  constexpr int L = 1 << D;
  const int nchunks = (a.n + kGbRows - 1) / kGbRows;
  const int cpw = gbdt_chunks_per_wg(nchunks);
  const int grid = (nchunks + cpw - 1) / cpw;
  const size_t lds = (size_t)min(a.gbdt_trees, kLeafLds / L) * L * sizeof(float);
  const bool r = a.rules != nullptr;    // routing rules: separate instantiation (register budget)
  if (contig && r)
    hipLaunchKernelGGL((score_gbdt_kernel<D, true, true>), dim3(grid), dim3(256), lds, s, a, cpw);
  else if (contig)
    hipLaunchKernelGGL((score_gbdt_kernel<D, true, false>), dim3(grid), dim3(256), lds, s, a, cpw);
  else if (r)
    hipLaunchKernelGGL((score_gbdt_kernel<D, false, true>), dim3(grid), dim3(256), lds, s, a, cpw);
  else
    hipLaunchKernelGGL((score_gbdt_kernel<D, false, false>), dim3(grid), dim3(256), lds, s, a, cpw);
}

int launch_gbdt(const ccfd_score_args& a, hipStream_t s) {
  const bool contig = a.ld == kF && (reinterpret_cast<uintptr_t>(a.x) & 15) == 0;
  if (a.gbdt_trees <= 0) return -2;
  if (a.n <= 0) return 0;
  const int forced = gbdt_forced_kernel();
  const bool want_v2 = forced == 2 || (forced == 0 && a.n >= kGbV2MinRows);
  if (want_v2 && contig && a.gbdt_depth >= 1 && a.gbdt_depth <= 8 &&
      ((long)a.gbdt_trees << a.gbdt_depth) <= kLeafLds) {
    switch (a.gbdt_depth) {
      case 1: launch_d2<1>(a, s); break;
      case 2: launch_d2<2>(a, s); break;
      case 3: launch_d2<3>(a, s); break;
      case 4: launch_d2<4>(a, s); break;
      case 5: launch_d2<5>(a, s); break;
      case 6: launch_d2<6>(a, s); break;
      case 7: launch_d2<7>(a, s); break;
      default: launch_d2<8>(a, s); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
  }
  switch (a.gbdt_depth) {
    case 1: launch_d<1>(a, s, contig); break;
    case 2: launch_d<2>(a, s, contig); break;
    case 3: launch_d<3>(a, s, contig); break;
    case 4: launch_d<4>(a, s, contig); break;
    case 5: launch_d<5>(a, s, contig); break;
    case 6: launch_d<6>(a, s, contig); break;
    case 7: launch_d<7>(a, s, contig); break;
    case 8: launch_d<8>(a, s, contig); break;
    default: return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace ccfd
