// G32 / G20 oblivious-GBDT scorer, one launch per micro-batch (engine exec_mode = 0, score_sync).
// Row format, level form and layout: g32_core.h; persistent variant: score_gbdt_g32_persist.hip.
#include "g32_core.h"

namespace ccfd {

template <int D, int R, bool kR, bool kGL, bool kG20>
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
  for (int q = 0; q < R; ++q) gx_fetch<kG20>(xb, n, grp * R + q, lane, pre[q]);

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

  unsigned fraud = 0, rows = 0, stale = 0;
  unsigned long long psum = 0;
  for (; grp < ngroups; grp += gstride) {
    // separate 1-D arrays per row chain: indexed by a runtime (wave-uniform) feature id they
    // stay in VGPRs (v_movrel); a 2-D array would be demoted to scratch
    unsigned b0[kF], b1[kF];
    unsigned meta[R];                                           // bucket | stamp << 8
    G32Row cur = pre[0];
    gx_rows<kG20>(xt[wave], lane, cur);
    meta[0] = gx_lift<kG20>(cur, b0);
    if constexpr (R == 2) {
      cur = pre[1];
      gx_rows<kG20>(xt[wave], lane, cur);
      meta[1] = gx_lift<kG20>(cur, b1);
    }
    const int nxt = grp + gstride;
    if (nxt < ngroups) {
#pragma unroll
      for (int q = 0; q < R; ++q) gx_fetch<kG20>(xb, n, nxt * R + q, lane, pre[q]);
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
        if (a.proba) st_g(a.proba + row, p);
        if (a.route) st_g(a.route + row, (uint8_t)(fr ? 1 : 0));
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
  unsigned long long* cnt = a.counters;
  if (cnt != nullptr && lane == 0 && stale) atomicAdd(&cnt[CCFD_CNT_WIRE_STALE], (unsigned long long)stale);
  epi_flush(epi, cnt);
  signal_done(a, gridDim.x);
}

// Grid: one wave per R-chunk group, capped at CCFD_G32_WGS_PER_CU workgroups per CU (grid-
// stride beyond).  A 65536-row micro-batch is 1024 chunks = 256 workgroups at R = 1: every
// CU has its rows in flight at once.  CCFD_G32_R: 64-row chunks per wave step (1 | 2).
template <int D, int R, bool kG20>
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
    if (a.rules) hipLaunchKernelGGL((score_gbdt_g32_kernel<D, R, true, true, kG20>), dim3(grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((score_gbdt_g32_kernel<D, R, false, true, kG20>), dim3(grid), dim3(256), 0, s, a);
  } else {
    if (a.rules) hipLaunchKernelGGL((score_gbdt_g32_kernel<D, R, true, false, kG20>), dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL((score_gbdt_g32_kernel<D, R, false, false, kG20>), dim3(grid), dim3(256), lds, s, a);
  }
}

template <int D>
static void launch_g32_d(const ccfd_score_args& a, hipStream_t s) {
  if (a.flags & CCFD_ARG_WIRE_G20) {             // G20: one chunk per wave step
    launch_g32_r<D, 1, true>(a, s);
    return;
  }
  const int r = g32_env("CCFD_G32_R", 1, 1, 2);
  if (r == 2) launch_g32_r<D, 2, false>(a, s);
  else launch_g32_r<D, 1, false>(a, s);
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
