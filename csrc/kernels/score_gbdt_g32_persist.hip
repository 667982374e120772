// G32 / G20 oblivious-GBDT scorer, persistent variant (engine exec_mode = 1; protocol in
// persist_core.h; row format and level form in g32_core.h).  The leaf tables
// are staged into LDS ONCE per resident workgroup (a launch per micro-batch re-stages them
// in every workgroup), and a claimed item is 4 waves x `cpw` 64-row chunks, the next chunk
// of a wave in flight while the current one is evaluated.
//
// Measured against it in round 6 (config 4, depth 4; profiles/r6/pass_c, pass_d; the code is
// in commit 95a7cf0): both chunks of a wave walked through the trees as a pair (R = 2: two
// row chains a lane) 2.540 vs 2.545e9 tx/s -- the tree walk's ILP is not the limit; a
// wave-specialised workgroup (a loader wave filling LDS item stages, 4 scorer waves reading
// only LDS) 1.78-2.05e9 in every variant (claim-ahead, two loaders, double-buffered without
// claim-ahead): queued items raise the micro-batch latency, and at a fixed ring depth the
// rate falls with it (Little's law: 4 x 65536 rows / batch latency).
#include <cstdio>
#include <vector>

#include "g32_core.h"
#include "persist_core.h"

namespace ccfd {

#ifdef CCFD_EXP_ITEM_TRACE
// Experiment build only (scripts/build_ab.py -D CCFD_EXP_ITEM_TRACE; never in the default
// library): thread 0 stamps each claimed item's phases -- claim atomic, wait for the posting +
// descriptor, first chunk's load, scoring, release + ticket -- into a device ring that the
// engine dumps at teardown (engine.cpp persist_free; bench/experiments/item_trace.py reads it).
struct ItemTrace {
  unsigned long long item, wg, t_claim, t_claimed, t_seen, t_desc, t_load, t_scored, t_done;
};
constexpr unsigned kItemTraceCap = 1u << 17;
__device__ ItemTrace g_item_trace[kItemTraceCap];
__device__ unsigned long long g_item_trace_n;
#define CCFD_ITRACE(stmt) stmt
#else
#define CCFD_ITRACE(stmt)
#endif

// kW waves per workgroup: 4 (default), or 8 in an experiment build (CCFD_EXP_G20_WAVES8: two
// waves per SIMD, each scoring half as many chunks of an item, so one wave's tree-walk
// latency hides behind the other's)
template <int D, bool kR, bool kGL, bool kG20, int kW = kG32Waves>
__global__ __launch_bounds__(64 * kW) void persist_gbdt_g32_kernel(ccfd_persist_args a) {
  extern __shared__ __attribute__((aligned(16))) float lv[];   // T * L floats
  __shared__ uint4 xt[kW][128];
  __shared__ EpilogueLds epi;
  __shared__ ccfd_persist_desc sdesc;
  __shared__ unsigned long long s_item;
  __shared__ int s_cmd;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int C = a.items_per_batch;
  const int cpw = a.tiles_per_wave * kG32Waves / kW;      // 64-row chunks per wave per item
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
  else g32_stage_leaves<D>(blob, T, lv, tid, 64 * kW);
  epi_init(epi);
  __syncthreads();
  unsigned long long posted_cache = 0;                    // thread 0 only

  // per-item accumulators of this wave (flushed by item_flush)
  unsigned fraud = 0, rows = 0, stale = 0;
  unsigned long long psum = 0;
  // sigmoid, route, outputs, histogram and flag list of one scored 64-row chunk
  auto chunk_epilogue = [&](const ccfd_persist_desc& d, int slot, int n, int chunk, unsigned meta, float acc)
      __attribute__((always_inline)) {
    const int row = chunk * kG32Rows + lane;
    const bool valid = row < n;
    const bool fresh = ((meta >> 8) & 0xffu) == stamp;
    const float p = fresh ? sigmoid(base + acc) : __builtin_nanf("");
    bool fr;
    if constexpr (kR) fr = valid && fresh && rule_route(a.rules, p, [](int) { return 0.f; });
    else fr = valid && fresh && (p >= a.threshold);
    if (valid) {
#ifndef CCFD_EXP_NO_OUTPUTS                                // experiment build only: cost of the output stream
      if (d.proba) st_g(d.proba + row, p);
      if (d.route) st_g(d.route + row, (uint8_t)(fr ? 1 : 0));
#endif
      if (fresh) psum += (unsigned)(p * 1e6f + 0.5f);
      atomicAdd(&epi.hist[(fr ? kNB : 0) + min((int)(meta & 0xffu), kNB - 1)], 1u);
    }
    const unsigned long long m = __ballot(fr);
    fraud += __popcll(m);
    rows += __popcll(__ballot(valid));
    stale += __popcll(__ballot(valid && !fresh));
    persist_emit_flagged(a, d, slot, m, fr, row, lane);
  };
  auto score_chunk = [&](const ccfd_persist_desc& d, int slot, int n, int chunk, G32Row& cur)
      __attribute__((always_inline)) {
    gx_rows<kG20>(xt[wave], lane, cur);
    unsigned b0[kF];
    const unsigned meta = gx_lift<kG20>(cur, b0);
    float acc[1];
#ifdef CCFD_EXP_READ_ONLY
    // experiment build only: the same items, loads, outputs and protocol with the trees replaced
    // by a use of the bins -- what the persistent read + completion path alone sustains
    acc[0] = (float)(b0[0] + b0[kF - 1]) * 1e-3f;
#else
    g32_trees<D, 1>(b0, b0, leaves, feat, kbin, T, acc);
#endif
    chunk_epilogue(d, slot, n, chunk, meta, acc[0]);
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
#ifdef CCFD_EXP_ITEM_TRACE
    unsigned long long t_claim = 0, t_claimed = 0, t_seen = 0, t_desc = 0, t_load = 0, t_scored = 0;
    if (tid == 0) {
      t_claim = wall_clock64();
      const unsigned long long it =
          __hip_atomic_fetch_add(&a.dev->work_next, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the claim's value is back (not just issued)
      t_claimed = wall_clock64();
      // persist_wait_item, split: the wait for the posting, then the descriptor read
      const unsigned long long b = it / (unsigned long long)C;
      s_cmd = 0;
      unsigned sleep_n = 1;
      while (posted_cache <= b) {
        posted_cache = __hip_atomic_load(&a.dev->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (posted_cache > b) break;
        if (__hip_atomic_load(&a.dev->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { s_cmd = 1; break; }
        for (unsigned k = 0; k < sleep_n; ++k) __builtin_amdgcn_s_sleep(1);
        sleep_n = sleep_n < 8 ? sleep_n * 2 : 8;
      }
      t_seen = wall_clock64();
      if (!s_cmd) persist_read_desc(a, b, sdesc);
      s_item = it;
      t_desc = wall_clock64();
    }
#else
    if (tid == 0) persist_claim(a, C, posted_cache, sdesc, s_item, s_cmd);
#endif
    __syncthreads();
    if (s_cmd) break;
    const ccfd_persist_desc d = sdesc;                     // registers: no LDS wait in the epilogue
    const int item = (int)(s_item % (unsigned long long)C);
    const int slot = (int)(d.seq % (unsigned long long)a.ring);
    const int n = d.n;
    const unsigned char* xb = reinterpret_cast<const unsigned char*>(d.x);
    k7_start(s_item, slot);
    const int c0 = item * (kW * cpw) + wave;              // this wave's chunks: c0 + kW*k
    // CCFD_G32_INFLIGHT=1: every chunk of the wave's share of the item in flight at once
    // (static registers: no copy of a pending load, so no vmcnt(0) between chunks)
    auto full_item = [&](auto kC) __attribute__((always_inline)) {
      constexpr int CPW = decltype(kC)::value;
      G32Row r[CPW];
#pragma unroll
      for (int k = 0; k < CPW; ++k) {
        const int chunk = c0 + kW * k;
        if (chunk * kG32Rows < n) gx_fetch<kG20>(xb, n, chunk, lane, r[k]);
      }
#pragma unroll
      for (int k = 0; k < CPW; ++k) {
        const int chunk = c0 + kW * k;
        if (chunk * kG32Rows >= n) break;                 // wave-uniform
        score_chunk(d, slot, n, chunk, r[k]);
      }
    };
    if (a.flags & CCFD_ARG_CHUNK_RING) {                  // default: one chunk ahead
      G32Row pre;
      if (c0 * kG32Rows < n) gx_fetch<kG20>(xb, n, c0, lane, pre);
#pragma unroll 1
      for (int k = 0; k < cpw; ++k) {
        const int chunk = c0 + kW * k;
        if (chunk * kG32Rows >= n) break;                 // wave-uniform
        G32Row cur_row = pre;
        CCFD_ITRACE(if (k == 0) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); if (tid == 0) t_load = wall_clock64(); })
        if (k + 1 < cpw && (chunk + kW) * kG32Rows < n) gx_fetch<kG20>(xb, n, chunk + kW, lane, pre);
        score_chunk(d, slot, n, chunk, cur_row);
      }
    } else if (cpw == 1) {
      full_item(std::integral_constant<int, 1>{});
    } else if (cpw == 2) {
      full_item(std::integral_constant<int, 2>{});
    } else {
      full_item(std::integral_constant<int, 4>{});        // 1024-row items (engine accepts 256/512/1024)
    }
    CCFD_ITRACE(if (tid == 0) t_scored = wall_clock64();)
    item_flush(d, slot);
#ifdef CCFD_EXP_ITEM_TRACE
    if (tid == 0) {
      const unsigned long long k =
          __hip_atomic_fetch_add(&g_item_trace_n, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      g_item_trace[k % kItemTraceCap] = ItemTrace{s_item, blockIdx.x, t_claim, t_claimed, t_seen, t_desc, t_load, t_scored,
                                                  (unsigned long long)wall_clock64()};
    }
#endif
  }
}

// Pipelined static items (engine persist_items = pipelined / CCFD_PERSIST_PIPE=1; VERDICT r4
// item 6).  The claimed kernel above ends every item with its outputs' release, a ticket and
// then -- only then -- the next claim, descriptor read and first loads: a 512-row G20 item is
// 10 KB, so at ~18 us of loaded PCIe read latency a workgroup has nothing in flight for a
// large share of each item (profiles/r4/g20/README.md).  Here, as in persist_pipe_kernel
// (score_persist.hip) for W64 rows:
//   * worker w (workgroup 1 + w of W) takes items base + w, base + w + W, ... -- no claim
//     atomic, the next item is known;
//   * the next item's rows are issued BEFORE the current item is scored, so its PCIe round
//     trip overlaps the current item's evaluation, output stores, release and ticket (the
//     release's vmcnt drain then waits on loads that are needed next anyway);
//   * leaves in LDS only (kGL = false: BASELINE's 100 x 6 is 25.6 KB); 512-row items (CPW 2).
// Unlike round 4's rejected two-item CLAIM pipeline, nothing is claimed early: the static
// assignment already fixes which workgroup scores which item.
template <int D, bool kR, bool kG20, int CPW>
__global__ __launch_bounds__(256) void persist_gbdt_pipe_kernel(ccfd_persist_args a) {
  extern __shared__ __attribute__((aligned(16))) float lv[];
  __shared__ uint4 xt[kG32Waves][128];
  __shared__ EpilogueLds epi;
  __shared__ ccfd_persist_desc sdesc[2];
  __shared__ int s_pre, s_cmd;                            // rewritten by thread 0 after a barrier only

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int C = a.items_per_batch;
  if (blockIdx.x == 0) {                                  // doorbell (persist_core.h)
    if (wave == 0) persist_doorbell(a, lane);
    return;
  }
  const char* blob = reinterpret_cast<const char*>(a.blob);
  const int T = a.gbdt_trees;
  const float base = *reinterpret_cast<const float*>(blob + 16);
  const unsigned stamp = (unsigned)*reinterpret_cast<const int*>(blob + 20);
  const int tdw = ((4 * T * D + 15) & ~15) / 4;
  const g32_cint_p feat = (g32_cint_p)(blob + kHeader);
  const g32_cint_p kbin = (g32_cint_p)(blob + kHeader + 4 * tdw);
  g32_stage_leaves<D>(blob, T, lv, tid, 256);
  const float* leaves = lv;
  epi_init(epi);
  __syncthreads();
  const unsigned long long W = gridDim.x - 1;
  unsigned long long item = __hip_atomic_load(&a.dev->work_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
                            (unsigned long long)(blockIdx.x - 1);
  unsigned long long posted_cache = 0;                    // thread 0 only

  unsigned fraud = 0, rows = 0, stale = 0;
  unsigned long long psum = 0;
  auto k7 = [&](const ccfd_persist_desc& d, unsigned long long it) __attribute__((always_inline)) {
    if (it % (unsigned long long)C == 0)                  // K7: micro-batch start
      __hip_atomic_store(&a.dev->tstart[d.seq % (unsigned long long)a.ring], wall_clock64(), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  };
  auto issue = [&](const ccfd_persist_desc& d, unsigned long long it, G32Row (&r)[CPW]) __attribute__((always_inline)) {
    const int c0 = (int)(it % (unsigned long long)C) * (kG32Waves * CPW) + wave;
    const unsigned char* xb = reinterpret_cast<const unsigned char*>(d.x);
#pragma unroll
    for (int k = 0; k < CPW; ++k) {
      const int chunk = c0 + kG32Waves * k;
      if (chunk * kG32Rows < d.n) gx_fetch<kG20>(xb, d.n, chunk, lane, r[k]);
    }
  };
  auto score = [&](const ccfd_persist_desc& d, unsigned long long it, G32Row (&r)[CPW]) __attribute__((always_inline)) {
    const int slot = (int)(d.seq % (unsigned long long)a.ring);
    const int n = d.n;
    const int c0 = (int)(it % (unsigned long long)C) * (kG32Waves * CPW) + wave;
#pragma unroll
    for (int k = 0; k < CPW; ++k) {
      const int chunk = c0 + kG32Waves * k;
      if (chunk * kG32Rows >= n) break;                   // wave-uniform
      gx_rows<kG20>(xt[wave], lane, r[k]);
      unsigned b0[kF];
      const unsigned meta = gx_lift<kG20>(r[k], b0);
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
    }
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
    persist_item_done(a, epi, d, slot, C, tid);           // barriers, release, ticket
  };
  // score `it` from (dc, rc) while item it + W is fetched into (dn, rn); true = host stopped
  auto stage = [&](ccfd_persist_desc& dc, G32Row (&rc)[CPW], ccfd_persist_desc& dn, G32Row (&rn)[CPW],
                   unsigned long long it) __attribute__((always_inline)) {
    const unsigned long long nx = it + W;
    if (tid == 0) {
      s_pre = persist_try_item(a, C, posted_cache, nx, dn);
      if (s_pre) k7(dn, nx);
    }
    __syncthreads();
    const bool pre = s_pre != 0;
    const ccfd_persist_desc d = dc;                       // registers: no LDS reads in the epilogue
    if (pre) issue(dn, nx, rn);                           // next item's rows in flight now
    score(d, it, rc);                                     // ends with barriers (persist_item_done)
    if (!pre) {
      if (tid == 0) {
        s_cmd = persist_wait_far(a, C, posted_cache, nx, dn);
        if (!s_cmd) k7(dn, nx);
      }
      __syncthreads();
      if (s_cmd) return true;
      issue(dn, nx, rn);
    }
    return false;
  };

  if (tid == 0) {
    s_cmd = persist_wait_far(a, C, posted_cache, item, sdesc[0]);
    if (!s_cmd) k7(sdesc[0], item);
  }
  __syncthreads();
  if (s_cmd) return;
  G32Row ra[CPW], rb[CPW];
  issue(sdesc[0], item, ra);
  for (;;) {
    if (stage(sdesc[0], ra, sdesc[1], rb, item)) break;
    item += W;
    if (stage(sdesc[1], rb, sdesc[0], ra, item)) break;
    item += W;
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
  if (a.flags & CCFD_ARG_PIPE_ITEMS) {                    // pipelined static 512-row items
    if (gl || a.tiles_per_wave != 2 || grid < 2) return -2;
    if (a.rules) hipLaunchKernelGGL((persist_gbdt_pipe_kernel<D, true, kG20, 2>), dim3(grid), dim3(256), lds, s, a);
    else hipLaunchKernelGGL((persist_gbdt_pipe_kernel<D, false, kG20, 2>), dim3(grid), dim3(256), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
  }
#ifdef CCFD_EXP_G20_WAVES8
  if (!gl && a.tiles_per_wave % 2 == 0) {
    if (a.rules) hipLaunchKernelGGL((persist_gbdt_g32_kernel<D, true, false, kG20, 8>), dim3(grid), dim3(512), lds, s, a);
    else hipLaunchKernelGGL((persist_gbdt_g32_kernel<D, false, false, kG20, 8>), dim3(grid), dim3(512), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
  }
#endif
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

#ifdef CCFD_EXP_ITEM_TRACE
// host: the item ring -> <path> as {u64 n, ItemTrace[kItemTraceCap]} (record k at k % cap), then the
// doorbell ring (persist_core.h)
int item_trace_dump(const char* path) {
  unsigned long long n = 0;
  std::vector<ItemTrace> v(kItemTraceCap);
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_item_trace_n), sizeof(n)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(g_item_trace), sizeof(ItemTrace) * v.size()) != hipSuccess) return -1;
  FILE* f = std::fopen(path, "wb");
  if (!f) return -1;
  std::fwrite(&n, sizeof(n), 1, f);
  std::fwrite(v.data(), sizeof(ItemTrace), v.size(), f);
  // then the doorbell ring: {u64 n, DoorbellTrace[kDoorbellTraceCap]}
  std::vector<DoorbellTrace> db(kDoorbellTraceCap);
  unsigned long long ndb = 0;
  if (hipMemcpyFromSymbol(&ndb, HIP_SYMBOL(g_db_trace_n), sizeof(ndb)) == hipSuccess &&
      hipMemcpyFromSymbol(db.data(), HIP_SYMBOL(g_db_trace), sizeof(DoorbellTrace) * db.size()) == hipSuccess) {
    std::fwrite(&ndb, sizeof(ndb), 1, f);
    std::fwrite(db.data(), sizeof(DoorbellTrace), db.size(), f);
  }
  std::fclose(f);
  return 0;
}
#endif

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
