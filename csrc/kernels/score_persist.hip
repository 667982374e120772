// Persistent streaming scorer (engine exec_mode = 1).
//
// One launch lives as long as the engine.  Every resident workgroup loops:
//   claim work item i (one agent-scope atomic)      -> micro-batch b = i / C, chunk c = i % C
//   wait until b is posted                          (thread 0 polls the DEVICE mirror kept by
//                                                   the doorbell workgroup 0, which alone
//                                                   polls host memory with relaxed system-
//                                                   scope loads; s_sleep back-off)
//   read descriptor b % R from the device mirror    -> LDS
//   4 waves x T tiles x 16 rows (item = 64T rows; default T = 8, CCFD_PERSIST_ITEM_ROWS),
//   next tile prefetched while the current one computes (f32 rows via a wave-private LDS
//   tile, W64 rows straight into registers), scored with the same fused math as the
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
#include "mlp_core.h"
#include "rules.h"

namespace ccfd {

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

  // Workgroup 0 is the DOORBELL: its first wave alone polls host memory (ctl->posted/stop)
  // and mirrors new descriptors + the posted count into device memory.  Every other
  // workgroup polls only the device mirror: hundreds of workgroups polling host memory
  // would each hold PCIe read requests and starve the feature stream (measured: 2x grid
  // -> 3x slower before this split).
  if (blockIdx.x == 0) {
    // The whole first wave mirrors: lane l copies word l % W of descriptor (mirrored + l / W),
    // so up to 10 newly posted descriptors cost ONE PCIe round trip instead of one per word
    // (a thread-0 copy loop serialised ~11 us per micro-batch: profiles/r1/persist_sweep.txt).
    if (wave == 0) {
      constexpr int kW = (int)(sizeof(ccfd_persist_desc) / 8);
      constexpr int kPer = 64 / kW;                     // descriptors per wave step
      unsigned long long mirrored = __hip_atomic_load(&a.dev->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned sleep_n = 1;
      for (;;) {
        unsigned long long p = 0;
        if (lane == 0) p = __hip_atomic_load(&a.ctl->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        p = __shfl(p, 0);
        if (p > mirrored) {
          const unsigned long long nb = min(p - mirrored, (unsigned long long)kPer);
          const int bi = lane / kW, wi = lane % kW;
          if (bi < (int)nb) {
            const unsigned long long b = mirrored + bi;
            const unsigned long long* src =
                reinterpret_cast<const unsigned long long*>(a.desc + (b % (unsigned long long)a.ring));
            unsigned long long* dst = reinterpret_cast<unsigned long long*>(a.dev->desc + (b % (unsigned long long)a.ring));
            __hip_atomic_store(dst + wi, __hip_atomic_load(src + wi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          // every lane's descriptor store is ordered before the new posted count
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          mirrored += nb;
          if (lane == 0) __hip_atomic_store(&a.dev->posted, mirrored, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          sleep_n = 1;
          continue;
        }
        int stop = 0;
        if (lane == 0) stop = __hip_atomic_load(&a.ctl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        if (__shfl(stop, 0)) {
          if (lane == 0) {
            __hip_atomic_store(&a.dev->stop, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&a.ctl->exited, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          break;
        }
        for (unsigned k = 0; k < sleep_n; ++k) __builtin_amdgcn_s_sleep(1);   // ~64..1024 cycles
        sleep_n = sleep_n < 8 ? sleep_n * 2 : 8;
      }
    }
    return;                                              // no barrier is ever used by WG 0
  }

  for (;;) {
    if (tid == 0) {
      const unsigned long long item =
          __hip_atomic_fetch_add(&a.dev->work_next, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long b = item / (unsigned long long)C;
      int cmd = 0;
      unsigned sleep_n = 1;
      while (posted_cache <= b) {
        // relaxed poll; the acquire fence below runs once the item's batch is posted
        posted_cache = __hip_atomic_load(&a.dev->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (posted_cache > b) break;
        if (__hip_atomic_load(&a.dev->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { cmd = 1; break; }
        for (unsigned k = 0; k < sleep_n; ++k) __builtin_amdgcn_s_sleep(1);
        sleep_n = sleep_n < 8 ? sleep_n * 2 : 8;
      }
      if (!cmd) {
        // one acquire per claimed item (not per poll): invalidates this XCD's L2 copies of
        // non-coherent inputs (a reused ring slot / DMA staging buffer) before they are read
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const unsigned long long* d = reinterpret_cast<const unsigned long long*>(a.dev->desc + (b % (unsigned long long)a.ring));
        sdesc.x = reinterpret_cast<const float*>(__hip_atomic_load(d + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        sdesc.proba = reinterpret_cast<float*>(__hip_atomic_load(d + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        sdesc.route = reinterpret_cast<uint8_t*>(__hip_atomic_load(d + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        sdesc.flag_idx = reinterpret_cast<unsigned int*>(__hip_atomic_load(d + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const unsigned long long ne = __hip_atomic_load(d + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sdesc.n = (int32_t)(ne & 0xffffffffull);
        sdesc.epoch = (int32_t)(ne >> 32);
        sdesc.seq = b;
      }
      s_item = item;
      s_cmd = cmd;
    }
    __syncthreads();
    if (s_cmd) break;

    const unsigned long long item = s_item;
    const int chunk = (int)(item % (unsigned long long)C);
    const int slot = (int)(sdesc.seq % (unsigned long long)a.ring);
    const int n = sdesc.n;
    const float* x = sdesc.x;
    const int kTilesPerWave = a.tiles_per_wave;
    const int tile0 = chunk * (4 * kTilesPerWave) + wave;      // wave w: tiles tile0 + 4k
    if (chunk == 0 && tid == 0)                                // K7: micro-batch start (item 0 claimed first)
      __hip_atomic_store(&a.dev->tstart[slot], wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    auto avail = [&](int t) { return min(kTileRows, n - t * kTileRows) * kF * 4; };
    TileRegs pre;
    WireRegs wpre;
    const bool wire = (a.flags & CCFD_ARG_WIRE_W64) != 0;       // uniform per launch
    const unsigned char* xw = reinterpret_cast<const unsigned char*>(x);
    if (tile0 * kTileRows < n) {
      if (wire) wire_issue(xw, n, tile0, c, g, wpre);
      else tile_issue(x + (size_t)tile0 * kTileRows * kF, avail(tile0), lane, pre);
    }
    unsigned nf_w = 0, nv_w = 0;
    unsigned long long ps_w = 0;
#pragma unroll 1
    for (int k = 0; k < kTilesPerWave; ++k) {
      const int tile = tile0 + 4 * k;
      const int row0 = tile * kTileRows;
      if (row0 >= n) break;                                // wave-uniform
      const int row = row0 + c;
      const bool valid = row < n;
      const int nxt = tile + 4;
      float xv[8];
      WireRegs cur_w;
      if (wire) {
        cur_w = wpre;
        if (k + 1 < kTilesPerWave && nxt * kTileRows < n) wire_issue(xw, n, nxt, c, g, wpre);
        if (kModel != CCFD_MODEL_MLP) wire_features(cur_w, g, xv);
      } else {
        tile_store(tile_lds, lane, pre);
        if (k + 1 < kTilesPerWave && nxt * kTileRows < n) tile_issue(x + (size_t)nxt * kTileRows * kF, avail(nxt), lane, pre);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        tile_features(tile_lds, c, g, xv);
      }
      float p, amount;
      if (kModel == CCFD_MODEL_MLP) {
        if (wire) {        // W64 blob: raw bf16 operands, folded normalisation (mlp_core.h)
          amount = __uint_as_float(cur_w.v.w);
          p = mlp_tile_w64(sblob, LW, cur_w, g, lane);
        } else {
          p = mlp_tile(sblob, L, xv, g, lane, amount);
        }
      } else {
        amount = xv[5];
        if (g == 3) { xv[6] = 0.f; xv[7] = 0.f; if (L.log_amount) xv[5] = log1pf(fmaxf(xv[5], 0.f)); }
        float z = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) z = fmaf((xv[j] - L.mu[j]) * L.isg[j], wm[j], z);
        z += __shfl_xor(z, 16);
        z += __shfl_xor(z, 32);
        p = sigmoid(z + L.b3);
      }
      bool fr;
      if constexpr (kR) {                               // configurable routing rules (rules.h)
        float xr[8];
        if (wire) {
          wire_features(cur_w, g, xr);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) xr[j] = xv[j];
          if (g == 3) xr[5] = amount;                   // the model replaced Amount by its log1p
        }
        const float pr = __shfl(p, c);
        fr = valid && (wire ? rule_route(a.rules, pr, [&](int j) { return lane_feature<true>(xr, j, c); })
                            : rule_route(a.rules, pr, [&](int j) { return lane_feature<false>(xr, j, c); }));
      } else {
        fr = valid && (p >= a.threshold);
      }
      if (valid && g == 0) {
        if (sdesc.proba) sdesc.proba[row] = p;
        if (sdesc.route) sdesc.route[row] = fr ? 1 : 0;
        ps_w += (unsigned long long)(p * 1e6f + 0.5f);
      }
      const unsigned long long m = __ballot(fr && g == 0);
      nf_w += __popcll(m);
      nv_w += __popcll(__ballot(valid && g == 0));
      if (valid && g == 3) atomicAdd(&epi.hist[(fr ? kNB : 0) + amount_bucket(amount)], 1u);
      // compacted flag list (reservation on the slot's device counter)
      if (m && sdesc.flag_idx) {
        const int leader = __builtin_ffsll((long long)m) - 1;
        unsigned base = 0;
        if (lane == leader)
          base = __hip_atomic_fetch_add(&a.dev->nflag[slot], (unsigned)__popcll(m), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
        base = __shfl(base, leader);
        if (fr && g == 0) sdesc.flag_idx[base + __popcll(m & ((1ull << lane) - 1ull))] = (unsigned)row;
      }
    }
    ps_w = wave_sum_u64(ps_w);
    if (lane == 0 && nv_w) {
      atomicAdd(&epi.fraud, nf_w);
      atomicAdd(&epi.rows, nv_w);
      atomicAdd(&epi.psum_e6, ps_w);
    }
    // per-item epilogue: counters of this item into the epoch's buffer, reset LDS state
    __syncthreads();
    unsigned long long* cnt = a.counters[sdesc.epoch & 1];
    if (tid < 2 * kNB) {
      const unsigned h = epi.hist[tid];
      if (h && cnt) atomicAdd(&cnt[(tid < kNB ? CCFD_CNT_HIST_STD : CCFD_CNT_HIST_FRAUD - kNB) + tid],
                              (unsigned long long)h);
      epi.hist[tid] = 0;
    } else if (tid == 64) {
      if (cnt && epi.rows) {
        atomicAdd(&cnt[CCFD_CNT_INCOMING], (unsigned long long)epi.rows);
        atomicAdd(&cnt[CCFD_CNT_FRAUD], (unsigned long long)epi.fraud);
        atomicAdd(&cnt[CCFD_CNT_STANDARD], (unsigned long long)(epi.rows - epi.fraud));
        atomicAdd(&cnt[CCFD_CNT_PROBA_E6], epi.psum_e6);
      }
      epi.rows = 0; epi.fraud = 0; epi.psum_e6 = 0;
    }
    // completion: publish this item's outputs, take a ticket, last ticket signals the host
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      // system-scope release of this item's outputs, relaxed ticket (see common.h signal_done)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned left =
          __hip_atomic_fetch_sub(&a.dev->remaining[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - 1u;
      if (left == 0) {
        const unsigned nflag = __hip_atomic_load(&a.dev->nflag[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.dev->nflag[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.dev->remaining[slot], (unsigned)C, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.ctl->done[slot][1], (unsigned long long)nflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&a.ctl->done[slot][2],
                           __hip_atomic_load(&a.dev->tstart[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&a.ctl->done[slot][3], wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&a.ctl->done[slot][0], sdesc.seq + 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
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
  if (a->model == CCFD_MODEL_MLP) {
    if (a->rules) hipLaunchKernelGGL((persist_kernel<CCFD_MODEL_MLP, true>), dim3(grid), dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((persist_kernel<CCFD_MODEL_MLP, false>), dim3(grid), dim3(256), 0, s, *a);
  } else if (a->model == CCFD_MODEL_LR) {
    if (a->rules) hipLaunchKernelGGL((persist_kernel<CCFD_MODEL_LR, true>), dim3(grid), dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((persist_kernel<CCFD_MODEL_LR, false>), dim3(grid), dim3(256), 0, s, *a);
  } else {
    return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
