// G32 / G20 oblivious-GBDT scorer, persistent variant (engine exec_mode = 1; protocol in
// persist_core.h; row format and level form in g32_core.h).  The leaf tables
// are staged into LDS ONCE per resident workgroup (a launch per micro-batch re-stages them
// in every workgroup), and a claimed item is 4 waves x `cpw` 64-row chunks, the next chunk
// of a wave in flight while the current one is evaluated.
#include "g32_core.h"
#include "persist_core.h"

namespace ccfd {

template <int D, bool kR, bool kGL, bool kG20>
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

  // per-item accumulators of this wave (flushed by item_flush)
  unsigned fraud = 0, rows = 0, stale = 0;
  unsigned long long psum = 0;
  auto score_chunk = [&](const ccfd_persist_desc& d, int slot, int n, int chunk, G32Row& cur)
      __attribute__((always_inline)) {
    gx_rows<kG20>(xt[wave], lane, cur);
    unsigned b0[kF];
    const unsigned meta = gx_lift<kG20>(cur, b0);
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
      if (d.proba) st_g(d.proba + row, p);
      if (d.route) st_g(d.route + row, (uint8_t)(fr ? 1 : 0));
      if (fresh) psum += (unsigned)(p * 1e6f + 0.5f);
      atomicAdd(&epi.hist[(fr ? kNB : 0) + min((int)(meta & 0xffu), kNB - 1)], 1u);
    }
    const unsigned long long m = __ballot(fr);
    fraud += __popcll(m);
    rows += __popcll(__ballot(valid));
    stale += __popcll(__ballot(valid && !fresh));
    persist_emit_flagged(a, d, slot, m, fr, row, lane);
  };
  auto item_flush = [&](const ccfd_persist_desc& d, int slot) __attribute__((always_inline)) {
    psum = wave_sum_u64(psum);
    if (lane == 0 && rows) {
      atomicAdd(&epi.fraud, fraud);
      atomicAdd(&epi.rows, rows);
      atomicAdd(&epi.psum_e6, psum);
      unsigned long long* cnt = a.counters[d.epoch & 1];
      if (stale && cnt) atomicAdd(&cnt[CCFD_CNT_WIRE_STALE], (unsigned long long)stale);
    }
    fraud = rows = stale = 0;
    psum = 0;
    persist_item_done(a, epi, d, slot, C, tid);
  };
  auto k7_start = [&](unsigned long long it, int slot) __attribute__((always_inline)) {
    if (it % (unsigned long long)C == 0 && tid == 0)      // K7: micro-batch start (item 0 claimed first)
      __hip_atomic_store(&a.dev->tstart[slot], wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  for (;;) {
    if (tid == 0) persist_claim(a, C, posted_cache, sdesc, s_item, s_cmd);
    __syncthreads();
    if (s_cmd) break;
    const ccfd_persist_desc d = sdesc;                     // registers: no LDS wait in the epilogue
    const int item = (int)(s_item % (unsigned long long)C);
    const int slot = (int)(d.seq % (unsigned long long)a.ring);
    const int n = d.n;
    const unsigned char* xb = reinterpret_cast<const unsigned char*>(d.x);
    k7_start(s_item, slot);
    const int c0 = item * (kG32Waves * cpw) + wave;       // this wave's chunks: c0 + 4k
    // CCFD_G32_INFLIGHT=1: every chunk of the wave's share of the item in flight at once
    // (static registers: no copy of a pending load, so no vmcnt(0) between chunks)
    auto full_item = [&](auto kC) __attribute__((always_inline)) {
      constexpr int CPW = decltype(kC)::value;
      G32Row r[CPW];
#pragma unroll
      for (int k = 0; k < CPW; ++k) {
        const int chunk = c0 + kG32Waves * k;
        if (chunk * kG32Rows < n) gx_fetch<kG20>(xb, n, chunk, lane, r[k]);
      }
#pragma unroll
      for (int k = 0; k < CPW; ++k) {
        const int chunk = c0 + kG32Waves * k;
        if (chunk * kG32Rows >= n) break;                 // wave-uniform
        score_chunk(d, slot, n, chunk, r[k]);
      }
    };
    if (a.flags & CCFD_ARG_CHUNK_RING) {                  // default: one chunk ahead
      G32Row pre;
      if (c0 * kG32Rows < n) gx_fetch<kG20>(xb, n, c0, lane, pre);
#pragma unroll 1
      for (int k = 0; k < cpw; ++k) {
        const int chunk = c0 + kG32Waves * k;
        if (chunk * kG32Rows >= n) break;                 // wave-uniform
        G32Row cur_row = pre;
        if (k + 1 < cpw && (chunk + kG32Waves) * kG32Rows < n) gx_fetch<kG20>(xb, n, chunk + kG32Waves, lane, pre);
        score_chunk(d, slot, n, chunk, cur_row);
      }
    } else if (cpw == 1) {
      full_item(std::integral_constant<int, 1>{});
    } else if (cpw == 2) {
      full_item(std::integral_constant<int, 2>{});
    } else {
      full_item(std::integral_constant<int, 4>{});        // 1024-row items (engine accepts 256/512/1024)
    }
    item_flush(d, slot);
  }
}

template <int D, bool kG20>
static int launch_persist_g32_f(const ccfd_persist_args& a0, int grid, hipStream_t s) {
  ccfd_persist_args a = a0;
  // one-chunk prefetch ring by default: at BASELINE config 4 (65536-row batches) it measured
  // 1.67e9 tx/s at p50 107 us (depth 3) vs 1.64e9 with the whole item in flight (VALU-heavy
  // trees overlap the next chunk's load better); CCFD_G32_INFLIGHT=1 selects the latter.
  // Read per launch: sweepable in-process (profiles/r2/persist_full_item/g32_inflight_ab.jsonl)
  if (g32_env("CCFD_G32_INFLIGHT", 0, 0, 1) == 0) a.flags |= CCFD_ARG_CHUNK_RING;
  const bool gl = ((long)a.gbdt_trees << D) > kG32LeafLds || g32_env("CCFD_G32_GLOBAL_LEAVES", 0, 0, 1);
  const size_t lds = gl ? 0 : (size_t)a.gbdt_trees * (1 << D) * sizeof(float);
  if (gl) {
    if (a.rules) hipLaunchKernelGGL((persist_gbdt_g32_kernel<D, true, true, kG20>), dim3(grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((persist_gbdt_g32_kernel<D, false, true, kG20>), dim3(grid), dim3(256), 0, s, a);
  } else {
    if (a.rules) hipLaunchKernelGGL((persist_gbdt_g32_kernel<D, true, false, kG20>), dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL((persist_gbdt_g32_kernel<D, false, false, kG20>), dim3(grid), dim3(256), lds, s, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

template <int D>
static int launch_persist_g32_d(const ccfd_persist_args& a, int grid, hipStream_t s) {
  return (a.flags & CCFD_ARG_WIRE_G20) ? launch_persist_g32_f<D, true>(a, grid, s)
                                       : launch_persist_g32_f<D, false>(a, grid, s);
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

}  // namespace ccfd
