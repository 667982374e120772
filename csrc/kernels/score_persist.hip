// Persistent streaming scorer (engine exec_mode = 1), MLP and LR; protocol helpers in
// persist_core.h (the GBDT G32 persistent kernel shares them, score_gbdt_g32_persist.hip).
//
// One launch lives as long as the engine.  Every resident workgroup loops:
//   claim work item i (one agent-scope atomic)      -> micro-batch b = i / C, chunk c = i % C
//   wait until b is posted                          (thread 0 polls the DEVICE mirror kept by
//                                                   the doorbell workgroup 0, which alone
//                                                   polls host memory with relaxed system-
//                                                   scope loads; s_sleep back-off)
//   read descriptor b % R from the device mirror    -> LDS
//   4 waves x T tiles x 16 rows (item = 64T rows, CCFD_PERSIST_ITEM_ROWS; engine defaults
//   T = 8 for the MLP on W64 rows, 4 otherwise): W64 items of 4 / 8 tiles issue every tile
//   at once and score them in pairs, other sizes prefetch the next tile while the current
//   one computes (f32 rows via a wave-private LDS tile); the same fused math as the
//   per-batch kernels (mlp_core.h), outputs written straight to host-mapped memory,
//   fraud rows appended to the descriptor's compacted flag list
//   counters + amount histogram -> counters[desc.epoch] (one atomic set per item)
//   release (system scope) + ticket on remaining[b % R]; the last ticket publishes
//   ctl->done[b % R] = {b + 1, #flagged, t_start, t_end}
// A workgroup only waits for the HOST (never for another workgroup), so residency of the
// whole grid is not required and nothing can deadlock; it exits when the host sets `stop`
// while it waits for an unposted batch.  The host never posts batch b into ring slot
// b % R before observing done for b - R, which is what makes the slot-local state
// (remaining/nflag reset by the last ticket) safe to reuse.
#include <type_traits>

#include "mlp_core.h"
#include "persist_core.h"
#include "rules.h"

namespace ccfd {

int launch_persist_gbdt_g32(const ccfd_persist_args& a, int grid, hipStream_t s);   // score_gbdt_g32_persist.hip

namespace {

template <int kModel, bool kR>
__global__ __launch_bounds__(256) void persist_kernel(ccfd_persist_args a) {
  __shared__ __attribute__((aligned(16))) char sblob[kMlpBlobWire];
  __shared__ __attribute__((aligned(16))) float sx[4][kTileRows * kF + 4];
  __shared__ EpilogueLds epi;
  __shared__ ccfd_persist_desc sdesc;
  __shared__ unsigned long long s_item;
  __shared__ int s_cmd;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int C = a.items_per_batch;

  if (kModel == CCFD_MODEL_MLP)
    mlp_stage(a.blob, sblob, tid, 256, (a.flags & CCFD_ARG_WIRE_W64) ? kMlpBlobWire : kMlpBlob);
  else for (int i = tid; i < 448 / 16; i += 256) reinterpret_cast<int4*>(sblob)[i] = reinterpret_cast<const int4*>(a.blob)[i];
  epi_init(epi);
  __syncthreads();

  MlpLane L{};
  MlpWireLane LW{};
  float wm[8];
  if (kModel == CCFD_MODEL_MLP) {
    L = mlp_lane(sblob, g);
    LW = mlp_wire_lane(sblob);
  } else {
    const unsigned flags = *reinterpret_cast<const unsigned*>(sblob + 4);
    L.b3 = *reinterpret_cast<const float*>(sblob + 8);
    L.log_amount = (flags & 1u) != 0;
    const float* mu = reinterpret_cast<const float*>(sblob + 64) + 8 * g;
    const float* isg = reinterpret_cast<const float*>(sblob + 192) + 8 * g;
    const float* w = reinterpret_cast<const float*>(sblob + 320) + 8 * g;
#pragma unroll
    for (int j = 0; j < 8; ++j) { L.mu[j] = mu[j]; L.isg[j] = isg[j]; wm[j] = w[j]; }
  }
  float* tile_lds = sx[wave];
  unsigned long long posted_cache = 0;     // thread 0 only

  // Workgroup 0 is the DOORBELL (persist_core.h): its first wave alone polls host memory.
  if (blockIdx.x == 0) {
    if (wave == 0) persist_doorbell(a, lane);
    return;                                              // no barrier is ever used by WG 0
  }

  for (;;) {
    if (tid == 0) persist_claim(a, C, posted_cache, sdesc, s_item, s_cmd);
    __syncthreads();
    if (s_cmd) break;

    const unsigned long long item = s_item;
    // the item's descriptor in registers: the epilogue reads its pointers with no LDS wait
    const ccfd_persist_desc dsc = sdesc;
    const int chunk = (int)(item % (unsigned long long)C);
    const int slot = (int)(dsc.seq % (unsigned long long)a.ring);
    const int n = dsc.n;
    const float* x = dsc.x;
    const int kTilesPerWave = a.tiles_per_wave;
    const int tile0 = chunk * (4 * kTilesPerWave) + wave;      // wave w: tiles tile0 + 4k
    if (chunk == 0 && tid == 0)                                // K7: micro-batch start (item 0 claimed first)
      __hip_atomic_store(&a.dev->tstart[slot], wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    auto avail = [&](int t) { return min(kTileRows, n - t * kTileRows) * kF * 4; };
    const bool wire = (a.flags & CCFD_ARG_WIRE_W64) != 0;       // uniform per launch
    const unsigned char* xw = reinterpret_cast<const unsigned char*>(x);
    unsigned nf_w = 0, nv_w = 0;
    unsigned long long ps_w = 0;
    // LR on one lane group's 8 features (the g == 3 group also carries Time / Amount)
    auto lr_p = [&](float (&xv)[8]) __attribute__((always_inline)) {
      if (g == 3) { xv[6] = 0.f; xv[7] = 0.f; if (L.log_amount) xv[5] = log1pf(fmaxf(xv[5], 0.f)); }
      float z = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) z = fmaf((xv[j] - L.mu[j]) * L.isg[j], wm[j], z);
      z += __shfl_xor(z, 16);
      z += __shfl_xor(z, 32);
      return sigmoid(z + L.b3);
    };
    // per-tile epilogue: outputs, route, counters, amount histogram, compacted fraud list;
    // xr = the tile's raw features (routing rules only)
    auto finish = [&](float p, float amount, int tile, float (&xr)[8]) __attribute__((always_inline)) {
      const int row = tile * kTileRows + c;
      const bool valid = row < n;
      bool fr;
      if constexpr (kR) {                               // configurable routing rules (rules.h)
        const float pr = __shfl(p, c);
        fr = valid && (wire ? rule_route(a.rules, pr, [&](int j) { return lane_feature<true>(xr, j, c); })
                            : rule_route(a.rules, pr, [&](int j) { return lane_feature<false>(xr, j, c); }));
      } else {
        fr = valid && (p >= a.threshold);
      }
      if (valid && g == 0) {
        if (dsc.proba) st_g(dsc.proba + row, p);
        if (dsc.route) st_g(dsc.route + row, (uint8_t)(fr ? 1 : 0));
        ps_w += (unsigned long long)(p * 1e6f + 0.5f);
      }
      const unsigned long long m = __ballot(fr && g == 0);
      nf_w += __popcll(m);
      nv_w += __popcll(__ballot(valid && g == 0));
      if (valid && g == 3) atomicAdd(&epi.hist[(fr ? kNB : 0) + amount_bucket(amount)], 1u);
      persist_emit_flagged(a, dsc, slot, m, fr && g == 0, row, lane);
    };
    // W64 items of 2, 4 or 8 tiles per wave (128 / 256 / 512 rows): every tile
    // of the item in flight at once -- the item costs one PCIe round trip instead of one per
    // tile, so fewer rows in flight keep the link busy (lower p50 at the same rate) -- and
    // scored in pairs (mlp_tile_w64_x2: one LDS weight read feeds two MFMAs)
    auto full_item = [&](auto kT) __attribute__((always_inline)) {
      constexpr int T = decltype(kT)::value;
      WireRegs r[T];
#pragma unroll
      for (int k = 0; k < T; ++k) wire_issue(xw, n, tile0 + 4 * k, c, g, r[k]);
#pragma unroll
      for (int k = 0; k < T; k += 2) {
        const int ta = tile0 + 4 * k;
        if (ta * kTileRows >= n) break;                    // wave-uniform
        float pa, pb;
        float xa[8], xb[8];
        if (kModel == CCFD_MODEL_MLP) {
          mlp_tile_w64_x2(sblob, LW, r[k], r[k + 1], g, lane, pa, pb);
          if constexpr (kR) { wire_features(r[k], g, xa); wire_features(r[k + 1], g, xb); }
        } else {
          wire_features(r[k], g, xa);
          wire_features(r[k + 1], g, xb);
          float la[8], lb[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) { la[j] = xa[j]; lb[j] = xb[j]; }
          pa = lr_p(la);
          pb = lr_p(lb);
        }
        finish(pa, __uint_as_float(r[k].v.w), ta, xa);
        finish(pb, __uint_as_float(r[k + 1].v.w), ta + 4, xb);   // rows >= n: no-op epilogue
      }
    };
    if (wire && kTilesPerWave == 2) {
      full_item(std::integral_constant<int, 2>{});
    } else if (wire && kTilesPerWave == 4) {
      full_item(std::integral_constant<int, 4>{});
    } else if (wire && kTilesPerWave == 8) {
      full_item(std::integral_constant<int, 8>{});
    } else {
      TileRegs pre;
      WireRegs wpre;
      if (tile0 * kTileRows < n) {
        if (wire) wire_issue(xw, n, tile0, c, g, wpre);
        else tile_issue(x + (size_t)tile0 * kTileRows * kF, avail(tile0), lane, pre);
      }
#pragma unroll 1
      for (int k = 0; k < kTilesPerWave; ++k) {
        const int tile = tile0 + 4 * k;
        const int row0 = tile * kTileRows;
        if (row0 >= n) break;                                // wave-uniform
        const int nxt = tile + 4;
        float xv[8];
        WireRegs cur_w;
        if (wire) {
          cur_w = wpre;
          if (k + 1 < kTilesPerWave && nxt * kTileRows < n) wire_issue(xw, n, nxt, c, g, wpre);
          if (kModel != CCFD_MODEL_MLP || kR) wire_features(cur_w, g, xv);
        } else {
          tile_store(tile_lds, lane, pre);
          if (k + 1 < kTilesPerWave && nxt * kTileRows < n) tile_issue(x + (size_t)nxt * kTileRows * kF, avail(nxt), lane, pre);
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          tile_features(tile_lds, c, g, xv);
        }
        float xr[8];                                         // raw features for the rules
        if constexpr (kR) {
#pragma unroll
          for (int j = 0; j < 8; ++j) xr[j] = xv[j];
        }
        float p, amount;
        if (kModel == CCFD_MODEL_MLP) {
          if (wire) {        // W64 blob: raw bf16 operands, folded normalisation (mlp_core.h)
            amount = __uint_as_float(cur_w.v.w);
            p = mlp_tile_w64(sblob, LW, cur_w, g, lane);
          } else {
            p = mlp_tile(sblob, L, xv, g, lane, amount);
            if (kR && g == 3) xr[5] = amount;              // the model replaced Amount by its log1p
          }
        } else {
          amount = xv[5];
          p = lr_p(xv);
        }
        finish(p, amount, tile, xr);
      }
    }
    ps_w = wave_sum_u64(ps_w);
    if (lane == 0 && nv_w) {
      atomicAdd(&epi.fraud, nf_w);
      atomicAdd(&epi.rows, nv_w);
      atomicAdd(&epi.psum_e6, ps_w);
    }
    persist_item_done(a, epi, dsc, slot, C, tid);
  }
}

// Pipelined static work items (CCFD_ARG_PIPE_ITEMS; MLP on W64 rows).  A CU reading host
// memory sustains only ~2 GB/s (a few KB of requests outstanding over a ~2 us PCIe round
// trip), so a micro-batch finishes soonest when its 256 KB is spread over many CUs: small
// items (64 / 128 rows, one per workgroup).  The claim-score-release chain of one item is
// ~9 us of latency, though (atomic claim, descriptor read, PCIe round trip, output release,
// ticket), which with one item per workgroup at a time capped small items far below the link
// (profiles/r3/latency/latency_sweep_workgroup_items.jsonl).  Here:
//   * items are assigned statically -- worker w (workgroup 1 + w of W) takes items
//     base + w, base + w + W, ... -- so there is no claim atomic and a worker knows its next
//     item without asking;
//   * while item i is scored, the descriptor of item i + W is read and its rows are already
//     in flight (when its micro-batch is posted), so one item's release / ticket overlaps the
//     next item's PCIe round trip;
//   * a worker waiting for a batch several batches ahead of the posted count sleeps longer,
//     so idle workers do not hammer the device `posted` word.
// T = tiles per wave per item (1: 64-row items, 2: 128-row items).
template <bool kR, int T>
__global__ __launch_bounds__(256) void persist_pipe_kernel(ccfd_persist_args a) {
  static_assert(T == 1 || T == 2, "64- or 128-row items");
  __shared__ __attribute__((aligned(16))) char sblob[kMlpBlobWire];
  __shared__ EpilogueLds epi;
  __shared__ ccfd_persist_desc sdesc[2];
  // two flags: s_pre (next item prefetched) and s_cmd (stop) are each rewritten by thread 0
  // only after a barrier that every thread passes after reading the previous value
  __shared__ int s_pre, s_cmd;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int C = a.items_per_batch;
  mlp_stage(a.blob, sblob, tid, 256, kMlpBlobWire);
  epi_init(epi);
  __syncthreads();
  if (blockIdx.x == 0) {                                 // the DOORBELL (persist_core.h)
    if (wave == 0) persist_doorbell(a, lane);
    return;
  }
  const MlpWireLane LW = mlp_wire_lane(sblob);
  const unsigned long long W = gridDim.x - 1;
  unsigned long long item = __hip_atomic_load(&a.dev->work_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
                            (unsigned long long)(blockIdx.x - 1);
  unsigned long long posted_cache = 0;                   // thread 0 only

  auto stamp = [&](const ccfd_persist_desc& d, unsigned long long it) __attribute__((always_inline)) {
    if (it % (unsigned long long)C == 0)                // K7: micro-batch start
      __hip_atomic_store(&a.dev->tstart[d.seq % (unsigned long long)a.ring], wall_clock64(), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  };
  auto issue = [&](const ccfd_persist_desc& d, unsigned long long it, WireRegs (&r)[T]) __attribute__((always_inline)) {
    const int tile0 = (int)(it % (unsigned long long)C) * (4 * T) + wave;   // wave w: tiles tile0 + 4k
    const unsigned char* xw = reinterpret_cast<const unsigned char*>(d.x);
#pragma unroll
    for (int k = 0; k < T; ++k) wire_issue(xw, d.n, tile0 + 4 * k, c, g, r[k]);
  };
  // score item `it` (rows in r), counters into LDS, outputs to the host, then release + ticket
  auto score = [&](const ccfd_persist_desc& d, unsigned long long it, const WireRegs (&r_in)[T]) __attribute__((always_inline)) {
    const int slot = (int)(d.seq % (unsigned long long)a.ring);
    const int n = d.n;
    const int tile0 = (int)(it % (unsigned long long)C) * (4 * T) + wave;
    WireRegs r[T];
#pragma unroll
    for (int k = 0; k < T; ++k) r[k] = r_in[k];
    unsigned nf_w = 0, nv_w = 0;
    unsigned long long ps_w = 0;
    auto finish = [&](float p, const WireRegs& rr, int tile) __attribute__((always_inline)) {
      const int row = tile * kTileRows + c;
      const bool valid = row < n;
      bool fr;
      if constexpr (kR) {
        float xr[8];
        wire_features(rr, g, xr);
        fr = valid && rule_route(a.rules, __shfl(p, c), [&](int j) { return lane_feature<true>(xr, j, c); });
      } else {
        fr = valid && (p >= a.threshold);
      }
      if (valid && g == 0) {
        if (d.proba) st_g(d.proba + row, p);
        if (d.route) st_g(d.route + row, (uint8_t)(fr ? 1 : 0));
        ps_w += (unsigned long long)(p * 1e6f + 0.5f);
      }
      const unsigned long long m = __ballot(fr && g == 0);
      nf_w += __popcll(m);
      nv_w += __popcll(__ballot(valid && g == 0));
      const float amount = __uint_as_float(rr.v.w);
      if (valid && g == 3) atomicAdd(&epi.hist[(fr ? kNB : 0) + amount_bucket_fast(amount)], 1u);
      persist_emit_flagged(a, d, slot, m, fr && g == 0, row, lane);
    };
    if (tile0 * kTileRows < n) {
      if constexpr (T == 2) {
        float pa, pb;
        mlp_tile_w64_x2(sblob, LW, r[0], r[1], g, lane, pa, pb);
        finish(pa, r[0], tile0);
        finish(pb, r[1], tile0 + 4);                     // rows >= n: no-op epilogue
      } else {
        finish(mlp_tile_w64(sblob, LW, r[0], g, lane), r[0], tile0);
      }
    }
    ps_w = wave_sum_u64(ps_w);
    if (lane == 0 && nv_w) {
      atomicAdd(&epi.fraud, nf_w);
      atomicAdd(&epi.rows, nv_w);
      atomicAdd(&epi.psum_e6, ps_w);
    }
    persist_item_done(a, epi, d, slot, C, tid);
  };
  // one pipeline stage: score `it` from (dc, rc) while item it + W is fetched into (dn, rn);
  // returns true when the host stopped the kernel
  auto stage = [&](ccfd_persist_desc& dc, const WireRegs (&rc)[T], ccfd_persist_desc& dn, WireRegs (&rn)[T],
                   unsigned long long it) __attribute__((always_inline)) {
    const unsigned long long nx = it + W;
    if (tid == 0) {
      s_pre = persist_try_item(a, C, posted_cache, nx, dn);
      if (s_pre) stamp(dn, nx);
    }
    __syncthreads();
    const bool pre = s_pre != 0;
    if (pre) issue(dn, nx, rn);                          // next item's rows in flight now
    score(dc, it, rc);                                   // ends with barriers (persist_item_done)
    if (!pre) {
      if (tid == 0) {
        s_cmd = persist_wait_far(a, C, posted_cache, nx, dn);
        if (!s_cmd) stamp(dn, nx);
      }
      __syncthreads();
      if (s_cmd) return true;
      issue(dn, nx, rn);
    }
    return false;
  };

  if (tid == 0) {
    s_cmd = persist_wait_far(a, C, posted_cache, item, sdesc[0]);
    if (!s_cmd) stamp(sdesc[0], item);
  }
  __syncthreads();
  if (s_cmd) return;
  WireRegs ra[T], rb[T];
  issue(sdesc[0], item, ra);
  for (;;) {
    if (stage(sdesc[0], ra, sdesc[1], rb, item)) break;
    item += W;
    if (stage(sdesc[1], rb, sdesc[0], ra, item)) break;
    item += W;
  }
}

}  // namespace

}  // namespace ccfd

extern "C" int ccfd_persist_launch(const ccfd_persist_args* a, int grid, void* stream) {
  using namespace ccfd;
  if (!a || !a->ctl || !a->desc || !a->dev || !a->blob) return -1;
  if (a->ring <= 0 || a->ring > CCFD_PERSIST_MAX_RING || a->items_per_batch <= 0 || a->tiles_per_wave <= 0) return -2;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // routing rules: separate instantiations, so threshold-only kernels keep their registers
  if (a->model == CCFD_MODEL_MLP && (a->flags & CCFD_ARG_PIPE_ITEMS)) {
    if (!(a->flags & CCFD_ARG_WIRE_W64) || grid < 2) return -2;
    const bool r = a->rules != nullptr;
    switch (a->tiles_per_wave) {
      case 1: if (r) hipLaunchKernelGGL((persist_pipe_kernel<true, 1>), dim3(grid), dim3(256), 0, s, *a);
              else hipLaunchKernelGGL((persist_pipe_kernel<false, 1>), dim3(grid), dim3(256), 0, s, *a); break;
      case 2: if (r) hipLaunchKernelGGL((persist_pipe_kernel<true, 2>), dim3(grid), dim3(256), 0, s, *a);
              else hipLaunchKernelGGL((persist_pipe_kernel<false, 2>), dim3(grid), dim3(256), 0, s, *a); break;
      default: return -2;
    }
  } else if (a->model == CCFD_MODEL_MLP) {
    if (a->rules) hipLaunchKernelGGL((persist_kernel<CCFD_MODEL_MLP, true>), dim3(grid), dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((persist_kernel<CCFD_MODEL_MLP, false>), dim3(grid), dim3(256), 0, s, *a);
  } else if (a->model == CCFD_MODEL_LR) {
    if (a->rules) hipLaunchKernelGGL((persist_kernel<CCFD_MODEL_LR, true>), dim3(grid), dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((persist_kernel<CCFD_MODEL_LR, false>), dim3(grid), dim3(256), 0, s, *a);
  } else if (a->model == CCFD_MODEL_GBDT && (a->flags & CCFD_ARG_WIRE_G32)) {
    return launch_persist_gbdt_g32(*a, grid, s);
  } else {
    return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
