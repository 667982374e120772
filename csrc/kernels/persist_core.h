// Protocol of the persistent streaming kernels (engine exec_mode = 1), shared by the MLP/LR
// kernel (score_persist.hip) and the GBDT G32 kernel (score_gbdt_g32_persist.hip):
//   * workgroup 0's first wave is the DOORBELL: it alone polls host memory and mirrors newly
//     posted descriptors + the posted count into device memory;
//   * every other workgroup claims work items with one agent-scope atomic, waits for the
//     item's micro-batch to be posted (device mirror only), reads its descriptor;
//   * after scoring an item: counters of the item into the epoch's buffer, system-scope
//     release of its outputs, ticket on remaining[slot]; the last ticket publishes
//     ctl->done[slot] = {seq + 1, #flagged, t_start, t_end}.
// A workgroup only waits for the HOST (never for another workgroup), so residency of the
// whole grid is not required and nothing can deadlock; it exits when the host sets `stop`
// while it waits for an unposted batch.
#pragma once
#include "common.h"

namespace ccfd {

#ifdef CCFD_EXP_ITEM_TRACE
// Experiment build only: one record per doorbell cycle that found new postings -- poll issued,
// poll returned, posted count seen, count mirrored before, mirror published (wall clock).
struct DoorbellTrace {
  unsigned long long t_poll, t_polled, posted, mirrored, t_mirrored, pad0, pad1, pad2;
};
constexpr unsigned kDoorbellTraceCap = 1u << 16;
static __device__ DoorbellTrace g_db_trace[kDoorbellTraceCap];
static __device__ unsigned long long g_db_trace_n;
#endif

// Workgroup 0, wave 0: mirror host descriptors into device memory until `stop`.  The whole
// wave copies: lane l copies word l % W of descriptor (mirrored + l / W), so up to 10 newly
// posted descriptors cost ONE PCIe round trip instead of one per word (a thread-0 copy loop
// serialised ~11 us per micro-batch: profiles/r1/persist_sweep.txt).  Hundreds of
// workgroups polling host memory would each hold PCIe read requests and starve the
// feature stream (measured: 2x grid -> 3x slower before this split).
__device__ __forceinline__ void persist_doorbell(const ccfd_persist_args& a, int lane) {
  constexpr int kW = (int)(sizeof(ccfd_persist_desc) / 8);
  constexpr int kPer = 64 / kW;                     // descriptors per wave step
  unsigned long long mirrored = __hip_atomic_load(&a.dev->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned sleep_n = 1;
  for (;;) {
    unsigned long long p = 0;
#ifdef CCFD_EXP_ITEM_TRACE
    const unsigned long long t_poll = wall_clock64();
#endif
    if (lane == 0) p = __hip_atomic_load(&a.ctl->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    p = __shfl(p, 0);
    if (p > mirrored) {
#ifdef CCFD_EXP_ITEM_TRACE
      const unsigned long long t_polled = wall_clock64(), m0 = mirrored;
#endif
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
#ifdef CCFD_EXP_ITEM_TRACE
      if (lane == 0) {
        const unsigned long long k =
            __hip_atomic_fetch_add(&g_db_trace_n, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        g_db_trace[k % kDoorbellTraceCap] =
            DoorbellTrace{t_poll, t_polled, p, m0, (unsigned long long)wall_clock64(), 0, 0, 0};
      }
#endif
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

// Thread 0: read the descriptor of posted micro-batch b into `sdesc` (one acquire per item,
// not per poll: it invalidates this XCD's L2 copies of non-coherent inputs -- a reused ring
// slot / DMA staging buffer -- before they are read).
__device__ __forceinline__ void persist_read_desc(const ccfd_persist_args& a, unsigned long long b,
                                                  ccfd_persist_desc& sdesc) {
#ifndef CCFD_EXP_NO_ACQUIRE                  // experiment build only: cost of the per-item acquire
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
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

// Thread 0: wait until claimed item `item`'s micro-batch is posted, then read its descriptor;
// returns 1 (and reads nothing) when the host stopped the kernel instead.
__device__ __forceinline__ int persist_wait_item(const ccfd_persist_args& a, int C, unsigned long long& posted_cache,
                                                 unsigned long long item, ccfd_persist_desc& sdesc) {
  const unsigned long long b = item / (unsigned long long)C;
  unsigned sleep_n = 1;
  while (posted_cache <= b) {
    // relaxed poll; the acquire fence in persist_read_desc runs once the batch is posted
    posted_cache = __hip_atomic_load(&a.dev->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (posted_cache > b) break;
    if (__hip_atomic_load(&a.dev->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return 1;
    for (unsigned k = 0; k < sleep_n; ++k) __builtin_amdgcn_s_sleep(1);
    sleep_n = sleep_n < 8 ? sleep_n * 2 : 8;
  }
  persist_read_desc(a, b, sdesc);
  return 0;
}

// Thread 0: claim the next work item, wait for its micro-batch, read its descriptor into
// `sdesc`.  Sets cmd = 1 when the host stopped the kernel instead.
__device__ __forceinline__ void persist_claim(const ccfd_persist_args& a, int C, unsigned long long& posted_cache,
                                              ccfd_persist_desc& sdesc, unsigned long long& s_item, int& s_cmd) {
  const unsigned long long item =
      __hip_atomic_fetch_add(&a.dev->work_next, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  s_cmd = persist_wait_item(a, C, posted_cache, item, sdesc);
  s_item = item;
}

// Static-item pipelines (persist_pipe_kernel, persist_gbdt_pipe_kernel): thread 0 reads item
// `item`'s descriptor if its micro-batch is already posted (1) or reports that it is not yet (0)
// without waiting; persist_wait_far waits for it (napping longer when it is >= 2 batches
// ahead) and returns 1 when the host stopped the kernel instead.
__device__ __forceinline__ int persist_try_item(const ccfd_persist_args& a, int C, unsigned long long& posted_cache,
                                                unsigned long long item, ccfd_persist_desc& sdesc) {
  const unsigned long long b = item / (unsigned long long)C;
  if (posted_cache <= b)
    posted_cache = __hip_atomic_load(&a.dev->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (posted_cache <= b) return 0;
  persist_read_desc(a, b, sdesc);
  return 1;
}

__device__ __forceinline__ int persist_wait_far(const ccfd_persist_args& a, int C, unsigned long long& posted_cache,
                                                unsigned long long item, ccfd_persist_desc& sdesc) {
  const unsigned long long b = item / (unsigned long long)C;
  unsigned sleep_n = 1;
  while (posted_cache <= b) {
    posted_cache = __hip_atomic_load(&a.dev->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (posted_cache > b) break;
    if (__hip_atomic_load(&a.dev->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return 1;
    if (b - posted_cache >= 2) {                 // >= 2 batches ahead: ~1 us naps
      for (int k = 0; k < 4; ++k) __builtin_amdgcn_s_sleep(8);
    } else {
      for (unsigned k = 0; k < sleep_n; ++k) __builtin_amdgcn_s_sleep(1);
      sleep_n = sleep_n < 8 ? sleep_n * 2 : 8;
    }
  }
  persist_read_desc(a, b, sdesc);
  return 0;
}

// Append this wave's fraud-routed rows (fr_lane; m = __ballot(fr_lane)) to the slot's
// compacted flag list (reservation on the slot's device counter).
__device__ __forceinline__ void persist_emit_flagged(const ccfd_persist_args& a, const ccfd_persist_desc& sdesc,
                                                     int slot, unsigned long long m, bool fr_lane, int row,
                                                     int lane) {
  if (m == 0 || sdesc.flag_idx == nullptr) return;
  const int leader = __builtin_ffsll((long long)m) - 1;
  unsigned base = 0;
  if (lane == leader)
    base = __hip_atomic_fetch_add(&a.dev->nflag[slot], (unsigned)__popcll(m), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
  base = __shfl(base, leader);
  if (fr_lane) st_g(sdesc.flag_idx + base + __popcll(m & ((1ull << lane) - 1ull)), (unsigned)row);
}

// One thread: system-scope release of this item's outputs, then a ticket on the slot; the last
// ticket publishes ctl->done[slot] = {seq + 1, #flagged, t_start, t_end} for the host.
__device__ __forceinline__ void persist_ticket(const ccfd_persist_args& a, const ccfd_persist_desc& sdesc, int slot,
                                               int C) {
  // system-scope release of this item's outputs, relaxed ticket (see common.h signal_done)
#ifdef CCFD_EXP_AGENT_RELEASE
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // experiment build only: cost of the system scope
#else
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
#endif
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

// All threads, after the item's rows are scored: flush the item's counters (LDS state is
// reset for the next item) and drain every wave's output stores; the item is then ready for
// its ticket (persist_ticket, one thread).
__device__ __forceinline__ void persist_item_close(const ccfd_persist_args& a, EpilogueLds& epi,
                                                   const ccfd_persist_desc& sdesc, int tid) {
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
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// persist_item_close, then the ticket: publish this item's outputs, the last ticket of the
// micro-batch signals the host.
__device__ __forceinline__ void persist_item_done(const ccfd_persist_args& a, EpilogueLds& epi,
                                                  const ccfd_persist_desc& sdesc, int slot, int C, int tid) {
  persist_item_close(a, epi, sdesc, tid);
  if (tid == 0) persist_ticket(a, sdesc, slot, C);
}

}  // namespace ccfd
