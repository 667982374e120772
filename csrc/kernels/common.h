// Shared device helpers for the fused scoring kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../include/ccfd_abi.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace ccfd {

constexpr int kF = CCFD_N_FEATURES;          // 30 raw features
constexpr int kAmountCol = kF - 1;           // "Amount"
constexpr int kNB = CCFD_N_AMOUNT_BUCKETS;   // 13 finite bounds + Inf
constexpr int kTileRows = 16;                // rows per 16x16x32 MFMA tile (one wave)
constexpr int kTileBytes = kTileRows * kF * 4;   // 1920: contiguous when ld == 30
constexpr int kHeader = 64;

// Row loads and output stores through the GLOBAL address space.  A generic pointer (every
// pointer read from a descriptor or struct) compiles to FLAT instructions, and a FLAT
// load / store counts on LGKM_CNT as well as VM_CNT: each `s_waitcnt lgkmcnt(0)` that an
// LDS or scalar read of the epilogue needs then also waited for the wave's outstanding
// host-memory traffic -- a proba store over PCIe before the next tile's weight reads, a
// prefetched row chunk before the current chunk's LDS transpose.  Global instructions count
// on VM_CNT only.  Every pointer handed to these is device memory or host memory mapped
// into the GPU's address space, never LDS.
#define CCFD_GAS __attribute__((address_space(1)))
typedef unsigned ccfd_u32x4 __attribute__((ext_vector_type(4)));

template <class T>
__device__ __forceinline__ void st_g(T* p, T v) { *(CCFD_GAS T*)p = v; }
template <class T>
__device__ __forceinline__ T ld_g(const T* p) { return *(const CCFD_GAS T*)p; }
__device__ __forceinline__ uint4 ld_g16(const void* p) {            // 16-byte aligned
  const ccfd_u32x4 v = *(const CCFD_GAS ccfd_u32x4*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 ld_g16f(const void* p) {
  const uint4 v = ld_g16(p);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// Must match contracts/metric_names.py AMOUNT_BUCKETS.
__device__ __forceinline__ int amount_bucket(float a) {
  int b = 0;
  b += a > 1.f;    b += a > 5.f;    b += a > 10.f;   b += a > 25.f;
  b += a > 50.f;   b += a > 100.f;  b += a > 250.f;  b += a > 500.f;
  b += a > 1000.f; b += a > 2500.f; b += a > 5000.f; b += a > 10000.f;
  b += a > 25000.f;
  return b;   // 0..13, bucket b holds bound[b-1] < a <= bound[b]
}

// Same bucket as amount_bucket in 26 VALU: one compare + add-with-carry per bound (the
// compiler's select/shift/add3 form of the sum costs ~4 per bound).  NaN -> bucket 0 like
// amount_bucket (every ordered compare is false).
__device__ __forceinline__ int amount_bucket_fast(float a) {
  int b = 0;
  asm volatile(
      "v_cmp_lt_f32_e32 vcc, 0x3f800000, %1\n"   /* 1 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x40a00000, %1\n"   /* 5 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x41200000, %1\n"   /* 10 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x41c80000, %1\n"   /* 25 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x42480000, %1\n"   /* 50 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x42c80000, %1\n"   /* 100 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x437a0000, %1\n"   /* 250 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x43fa0000, %1\n"   /* 500 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x447a0000, %1\n"   /* 1000 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x451c4000, %1\n"   /* 2500 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x459c4000, %1\n"   /* 5000 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x461c4000, %1\n"   /* 10000 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      "v_cmp_lt_f32_e32 vcc, 0x46c35000, %1\n"   /* 25000 < a */
      "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
      : "+v"(b) : "v"(a) : "vcc");
  return b;
}

__device__ __forceinline__ float sigmoid(float z) { return 1.f / (1.f + __expf(-z)); }

// Per-workgroup epilogue accumulators in LDS.
struct EpilogueLds {
  unsigned int hist[2 * kNB];
  unsigned int fraud;
  unsigned int rows;
  unsigned long long psum_e6;
  unsigned int hgt[kNB - 1];   // rows with amount > bound i (HistLanes)
};

__device__ __forceinline__ void epi_init(EpilogueLds& s) {
  const int t = threadIdx.x;
  if (t < 2 * kNB) s.hist[t] = 0;
  if (t >= 32 && t < 32 + kNB - 1) s.hgt[t - 32] = 0;
  if (t == 0) { s.fraud = 0; s.rows = 0; s.psum_e6 = 0; }
}

// Amount histogram without per-row atomics or per-row bucket search.  The 13 bucket
// bounds are spread over the 4 lane groups (lane group g owns bounds g, 4+g, 8+g, 12+g):
// every lane sees the amount of row (lane & 15) -- broadcast from lane group 3 with one
// ds_bpermute -- and keeps 4 per-lane counters of "amount > its bounds" (4 compares + 4
// adds per 16-row tile instead of a 13-compare search + an LDS atomic per row).  At the
// end the 16 lanes of each group are summed, and bucket counts follow from differences of
// consecutive "greater-than" counts; the standard-route histogram is all rows minus the
// fraud-route histogram, which fraud rows (~0.2 %) still add per row into
// epi.hist[kNB + b].  `am` must be -inf for a row that is not valid.
struct HistLanes {
  unsigned cnt[4];
  float bound[4];
};

__device__ __forceinline__ void hist_lanes_init(HistLanes& h, int g) {
  constexpr float kB[16] = {1.f, 5.f, 10.f, 25.f, 50.f, 100.f, 250.f, 500.f, 1000.f, 2500.f,
                            5000.f, 10000.f, 25000.f, __builtin_inff(), __builtin_inff(), __builtin_inff()};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h.cnt[j] = 0;
    h.bound[j] = kB[4 * j + g];
  }
}

// `am_row`: amount of row (lane & 15) in EVERY lane (or -inf when that row is not valid).
__device__ __forceinline__ void hist_lanes_add(HistLanes& h, float am_row) {
#pragma unroll
  for (int j = 0; j < 4; ++j) h.cnt[j] += am_row > h.bound[j] ? 1u : 0u;
}

__device__ __forceinline__ void hist_lanes_commit(EpilogueLds& e, const HistLanes& h, int g, int c) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    unsigned v = h.cnt[j];
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    const int i = 4 * j + g;
    if (c == 0 && i < kNB - 1 && v) atomicAdd(&e.hgt[i], v);
  }
}

// Flush of a workgroup that built its amount histogram with HistLanes (all rows) plus
// per-row fraud atomics: standard bucket b = (rows in bucket b) - (fraud rows in bucket b).
__device__ __forceinline__ void epi_flush_ballot(EpilogueLds& s, unsigned long long* cnt) {
  __syncthreads();
  if (cnt == nullptr) return;
  const int t = threadIdx.x;
  if (t < kNB) {
    const unsigned above = t == 0 ? s.rows : s.hgt[t - 1];
    const unsigned all = above - (t == kNB - 1 ? 0u : s.hgt[t]);
    const unsigned h = all - s.hist[kNB + t];
    if (h) atomicAdd(&cnt[CCFD_CNT_HIST_STD + t], (unsigned long long)h);
  } else if (t < 2 * kNB) {
    const unsigned h = s.hist[t];
    if (h) atomicAdd(&cnt[CCFD_CNT_HIST_FRAUD - kNB + t], (unsigned long long)h);
  } else if (t == 2 * kNB) {
    atomicAdd(&cnt[CCFD_CNT_INCOMING], (unsigned long long)s.rows);
    atomicAdd(&cnt[CCFD_CNT_FRAUD], (unsigned long long)s.fraud);
    atomicAdd(&cnt[CCFD_CNT_STANDARD], (unsigned long long)(s.rows - s.fraud));
    atomicAdd(&cnt[CCFD_CNT_PROBA_E6], s.psum_e6);
  }
}

// Flush the workgroup's LDS accumulators into the global u64 counters (one atomic per slot).
__device__ __forceinline__ void epi_flush(EpilogueLds& s, unsigned long long* cnt) {
  __syncthreads();
  if (cnt == nullptr) return;
  const int t = threadIdx.x;
  if (t < 2 * kNB) {
    const unsigned h = s.hist[t];
    if (h) atomicAdd(&cnt[(t < kNB ? CCFD_CNT_HIST_STD : CCFD_CNT_HIST_FRAUD - kNB) + t],
                     (unsigned long long)h);
  } else if (t == 2 * kNB) {        // lane 28: valid for 1-wave workgroups too
    atomicAdd(&cnt[CCFD_CNT_INCOMING], (unsigned long long)s.rows);
    atomicAdd(&cnt[CCFD_CNT_FRAUD], (unsigned long long)s.fraud);
    atomicAdd(&cnt[CCFD_CNT_STANDARD], (unsigned long long)(s.rows - s.fraud));
    atomicAdd(&cnt[CCFD_CNT_PROBA_E6], s.psum_e6);
  }
}

// Append the fraud-routed rows of this wave to the slot's compacted flag list: one agent-
// scope atomic per wave that has any (fraud is ~0.2 % of traffic), then one 4-byte store
// per flagged row into host-mapped memory.  `fr_lane`: this lane owns a fraud-routed row.
__device__ __forceinline__ void emit_flagged(const ccfd_score_args& a, bool fr_lane, int row) {
  if (a.flag_idx == nullptr) return;
  const unsigned long long m = __ballot(fr_lane);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __builtin_ffsll((long long)m) - 1;
  unsigned base = 0;
  if (lane == leader)
    base = __hip_atomic_fetch_add(&a.slot_ctl[1], (unsigned)__popcll(m), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
  base = __shfl(base, leader);
  if (fr_lane) st_g(a.flag_idx + base + __popcll(m & ((1ull << lane) - 1ull)), (unsigned)row);
}

// Per-wave LDS staging of fraud-routed row indices for the streaming bodies.  Appending
// costs LDS writes only: emit_flagged's reservation is a global atomic WITH return, and the
// wait for its result (s_waitcnt vmcnt(0)) drains every row load the wave has in flight --
// at a 1 % fraud rate half the four-tile rounds of the W64 kernels paid that.  The wave
// reserves space in the batch's flag list once per >= 64 flagged rows and once at the end.
struct FlagStage {
  unsigned* buf;      // this wave's 128 LDS entries
  unsigned n;         // staged rows (wave-uniform)
};

__device__ __forceinline__ void flag_flush(const ccfd_score_args& a, FlagStage& f, int lane) {
  if (f.n == 0) return;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");       // this wave's LDS writes first
  unsigned base = 0;
  if (lane == 0) base = __hip_atomic_fetch_add(&a.slot_ctl[1], f.n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  base = __shfl(base, 0);
  for (unsigned i = (unsigned)lane; i < f.n; i += 64) st_g(a.flag_idx + base + i, f.buf[i]);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");       // reads done before reuse
  f.n = 0;
}

// m = __ballot(fr_lane), known non-zero by the caller
__device__ __forceinline__ void flag_push(const ccfd_score_args& a, FlagStage& f, unsigned long long m, bool fr_lane,
                                          int row, int lane) {
  if (a.flag_idx == nullptr) return;
  if (fr_lane) f.buf[f.n + __popcll(m & ((1ull << lane) - 1ull))] = (unsigned)row;
  f.n += (unsigned)__popcll(m);
  if (f.n > 64) flag_flush(a, f, lane);           // room for one more 64-row ballot
}

// Completion hand-off to the host, executed by EVERY thread as the kernel's last action
// (cdna_hip_programming.md §6 Guideline 16 publish recipe, system scope): each storing wave
// drains its stores, the workgroup barrier, lane 0 releases at system scope and takes a
// ticket; the last ticket resets the slot and publishes {#flagged, done_seq} to the host.
// `nblk`: workgroups that score this micro-batch (gridDim.x for a plain launch, the
// per-sub-batch share for a coalesced one).
__device__ __forceinline__ void signal_done(const ccfd_score_args& a, unsigned nblk) {
  if (a.slot_ctl == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    // system-scope release: this workgroup's host-visible stores (proba/route/flag list)
    // are complete at system scope before its ticket -- required across XCDs even for
    // fine-grained outputs (an s_waitcnt alone only means "accepted by this XCD's L2").
    // The ticket itself is relaxed: no agent-scope acquire, i.e. no L2 invalidate per
    // workgroup (the last workgroup reads only atomics).
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned ticket = __hip_atomic_fetch_add(&a.slot_ctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ticket == nblk - 1) {
      // K7: device-clock execution window of this micro-batch
      const unsigned long long t_end = wall_clock64();
      const unsigned long long t_start = __hip_atomic_load(
          reinterpret_cast<unsigned long long*>(a.slot_ctl + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.done_rec[2], t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&a.done_rec[3], t_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const unsigned nflag = __hip_atomic_load(&a.slot_ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.slot_ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.slot_ctl[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.done_rec[1], (unsigned long long)nflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&a.done_rec[0], a.done_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// K7: workgroup 0 of a micro-batch stamps its start on the device wall clock.
__device__ __forceinline__ void stamp_start(const ccfd_score_args& a, int blk) {
  if (a.slot_ctl != nullptr && blk == 0 && threadIdx.x == 0)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.slot_ctl + 2), wall_clock64(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Wave-level reduction of a u64 over the 64 lanes.
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// One 16-row tile of a packed [n][30] f32 matrix is 1920 contiguous bytes = 120 float4:
// lane l fetches float4 l and l+64 (full-width coalesced requests, also over PCIe for a
// host-mapped log).  Split into issue (global -> registers) and store (registers ->
// wave-private LDS tile) so the next tile's fetch is in flight while this one computes.
// `avail` = valid bytes in the tile (multiple of 8); bytes past it are zero-filled.
struct TileRegs { float4 v[2]; };

__device__ __forceinline__ void tile_issue(const float* __restrict__ xt, int avail, int lane, TileRegs& r) {
  const float4* src = reinterpret_cast<const float4*>(xt);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = lane + 64 * it;
    const int off = i * 16;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < kTileBytes / 16) {
      if (off + 16 <= avail) {
        v = ld_g16f(src + i);
      } else if (off + 8 <= avail) {
        v.x = ld_g(xt + 4 * i);
        v.y = ld_g(xt + 4 * i + 1);
      }
    }
    r.v[it] = v;
  }
}

__device__ __forceinline__ void tile_store(float* lds_tile, int lane, const TileRegs& r) {
  float4* dst = reinterpret_cast<float4*>(lds_tile);
  dst[lane] = r.v[0];
  if (lane + 64 < kTileBytes / 16) dst[lane + 64] = r.v[1];
}

// W64 wire rows (contracts/transaction.py WIRE_ROW_BYTES): 16 B per lane -- lane (g, c)
// owns bytes [16g, 16g+16) of row c of the tile, which in wire order are exactly its 8
// features (g < 3: eight bf16 V-components; g == 3: V25..V28 bf16, Time f32, Amount f32).
// A 16-row tile is one contiguous 1 KB wave request; no LDS staging is needed.
struct WireRegs { uint4 v; };

__device__ __forceinline__ void wire_issue(const unsigned char* __restrict__ x, int n, int tile, int c, int g,
                                           WireRegs& r) {
  const int row = tile * kTileRows + c;
  r.v = row < n ? ld_g16(x + (size_t)row * CCFD_WIRE_ROW_BYTES + 16 * g) : make_uint4(0u, 0u, 0u, 0u);
}

__device__ __forceinline__ void wire_features(const WireRegs& r, int g, float xv[8]) {
  const unsigned w0 = r.v.x, w1 = r.v.y, w2 = r.v.z, w3 = r.v.w;
  xv[0] = __uint_as_float(w0 << 16); xv[1] = __uint_as_float(w0 & 0xffff0000u);
  xv[2] = __uint_as_float(w1 << 16); xv[3] = __uint_as_float(w1 & 0xffff0000u);
  const bool tail = g == 3;
  xv[4] = tail ? __uint_as_float(w2) : __uint_as_float(w2 << 16);
  xv[5] = tail ? __uint_as_float(w3) : __uint_as_float(w2 & 0xffff0000u);
  xv[6] = tail ? 0.f : __uint_as_float(w3 << 16);
  xv[7] = tail ? 0.f : __uint_as_float(w3 & 0xffff0000u);
}

// Read this lane's 8 features of row c from a wave-private LDS tile [16][30].
__device__ __forceinline__ void tile_features(const float* tile_lds, int c, int g, float xv[8]) {
  const float2* r2 = reinterpret_cast<const float2*>(tile_lds + c * kF + 8 * g);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float2 v = (g < 3 || j < 3) ? r2[j] : make_float2(0.f, 0.f);
    xv[2 * j] = v.x; xv[2 * j + 1] = v.y;
  }
}

__device__ __forceinline__ void load_tile_contig(const float* __restrict__ xt, int avail,
                                                 float* lds_tile, int lane) {
  TileRegs r;
  tile_issue(xt, avail, lane, r);
  tile_store(lds_tile, lane, r);
}

// Per-micro-batch view of a coalesced launch: sub-batch j of `m` as plain score args.
// `m` must be addressable memory (the kernarg segment, see score_mlp_multi_kernel).
__device__ __forceinline__ ccfd_score_args sub_args(const ccfd_multi_args& m, int j) {
  ccfd_score_args a = m.base;
  const int64_t r0 = (int64_t)j * m.sub_rows;
  a.x = m.base.x + r0 * m.base.ld;
  a.n = (int)min((int64_t)m.sub_rows, (int64_t)m.base.n - r0);
  const ccfd_sub_batch& sb = m.sub[j];
  a.proba = sb.proba;
  a.route = sb.route;
  a.slot_ctl = sb.slot_ctl;
  a.flag_idx = sb.flag_idx;
  a.done_rec = sb.done_rec;
  a.done_seq = sb.done_seq;
  return a;
}

}  // namespace ccfd
