// Fused MLP fraud scorer: normalize -> 30x128 -> relu -> 128x64 -> relu -> 64x1 ->
// sigmoid -> FRAUD_THRESHOLD route -> counters + amount histogram.  One launch per
// micro-batch; replaces the reference's per-transaction Seldon REST predict()
// (deploy/model/modelfull.json:37-44, README.md:549-550) and the router's Drools
// threshold rule (deploy/router.yaml:69-70).
//
// CDNA4 mapping (see models/mlp.py for the packing derivation):
//  * one wave owns a 16-row tile; activations are computed TRANSPOSED (H^T = W . X^T) so
//    each mfma_f32_16x16x32_bf16 accumulator is the next layer's B operand in place --
//    no LDS round trip and no cross-lane shuffles between layers;
//  * the 25.9 KB packed weight blob is staged once per workgroup in LDS and read as
//    16-B fragments (ds_read_b128, lane-linear, conflict-free);
//  * the input tile (16 rows x 120 B, contiguous) is fetched with 16-B loads into a
//    wave-private LDS tile, so host-mapped (zero-copy, over PCIe) and HBM inputs are both
//    read with full-width coalesced requests;
//  * layer 3 is a 64-term dot product: 16 FMAs per lane + two xor-shuffles.
//  24 MFMAs (16x16x32) per 16 rows: compute is ~1% of the kernel; it is a latency /
//  bandwidth kernel, so fusion (one launch, one pass over x) is what matters.
#include <cstdlib>
#include <string>

#include "mlp_core.h"
#include "rules.h"
#include "wire_body.h"

namespace ccfd {

// Waves per workgroup is a template parameter (CCFD_MLP_WAVES=1/2/4): a 4096-row
// micro-batch is 256 tiles, so 4-wave workgroups occupy 64 CUs per launch; several launches
// run concurrently on separate streams.  Smaller workgroups spread one launch wider but pay
// the weight staging and completion ticket more often (profiles/r1/waves_sweep.txt).
// f32 rows (kMode: 0 = strided [n][ld], 1 = contiguous [n][30] through LDS-staged tiles;
// +4 = weights read from global instead of an LDS copy).  W64 wire rows take the separate
// wire_stream_body (wire_body.h, MlpWireScorer).  Body shared by the plain and the
// coalesced launch: workgroup `blk` of the `nblk` that score micro-batch `a`.  Entry points
// ask for >= 4 waves per SIMD (<= 128 VGPRs): occupancy (outstanding zero-copy loads) beats
// hoisting the 24 weight fragments into registers.
template <int kMode, int kWaves, bool kR>
__device__ __forceinline__ void mlp_body(const ccfd_score_args& a, int blk, int nblk) {
  constexpr bool kContig = (kMode & 3) == 1;
  constexpr bool kGW = (kMode & 4) != 0;     // weights read from global (L1/L2), no LDS copy
  static_assert((kMode & 3) != 2, "W64 rows use wire_stream_body");
  __shared__ __attribute__((aligned(16))) char sblob[kGW ? 16 : kMlpBlob];
  __shared__ __attribute__((aligned(16))) float sx[kWaves][kTileRows * kF + 4];
  __shared__ EpilogueLds epi;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  stamp_start(a, blk);
  const int ntiles = (a.n + kTileRows - 1) / kTileRows;
  const int tstride = nblk * kWaves;
  int tile = blk * kWaves + wave;

  // Issue this wave's first input tile BEFORE staging the weights: the (possibly PCIe)
  // fetch latency of x overlaps the L2 fetch of the model blob.
  TileRegs pre;
  auto tile_avail = [&](int t) { return min(kTileRows, a.n - t * kTileRows) * kF * 4; };
  if constexpr (kContig) {
    if (tile < ntiles) tile_issue(a.x + (size_t)tile * kTileRows * kF, tile_avail(tile), lane, pre);
  }
  if constexpr (!kGW) mlp_stage(a.blob, sblob, tid, 64 * kWaves);
  const char* W = kGW ? reinterpret_cast<const char*>(a.blob) : sblob;
  epi_init(epi);
  __syncthreads();

  const MlpLane L = mlp_lane(W, g);
  const float thr = a.threshold;
  unsigned fraud = 0, rows = 0;
  unsigned long long psum = 0;
  float* tile_lds = sx[wave];

  for (; tile < ntiles; tile += tstride) {
    const int row = tile * kTileRows + c;
    const bool valid = row < a.n;
    float xv[8];
    if constexpr (kContig) {
      tile_store(tile_lds, lane, pre);
      // prefetch the next tile of this wave while this one computes
      const int nxt = tile + tstride;
      if (nxt < ntiles) tile_issue(a.x + (size_t)nxt * kTileRows * kF, tile_avail(nxt), lane, pre);
      // wave-private tile: LDS ops of one wave complete in order
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      tile_features(tile_lds, c, g, xv);
    } else {
      // compiler barrier: keep the weight fragments as per-tile LDS reads (not hoisted into
      // ~100 loop-invariant VGPRs, which would spill under the 128-VGPR occupancy cap)
      asm volatile("" ::: "memory");
      const float* xr = a.x + (size_t)row * a.ld + 8 * g;
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[j] = (valid && (8 * g + j) < kF) ? xr[j] : 0.f;
    }
    float amount;
    const float p = mlp_tile(W, L, xv, g, lane, amount);
    bool fr;
    if constexpr (kR) {                                 // configurable routing rules (rules.h)
      if (g == 3) xv[5] = amount;                       // mlp_tile replaced Amount by its log1p
      fr = valid && rule_route(a.rules, __shfl(p, c), [&](int j) { return lane_feature<false>(xv, j, c); });
    } else {
      fr = valid && (p >= thr);
    }

    if (valid && g == 0) {
      if (a.proba) st_g(a.proba + row, p);
      if (a.route) st_g(a.route + row, (uint8_t)(fr ? 1 : 0));
      psum += (unsigned)(p * 1e6f + 0.5f);              // p in [0,1]: u32 convert, u64 sum
    }
    fraud += __popcll(__ballot(fr && g == 0));
    rows += __popcll(__ballot(valid && g == 0));
    if (valid && g == 3) atomicAdd(&epi.hist[(fr ? kNB : 0) + amount_bucket_fast(amount)], 1u);
    emit_flagged(a, fr && g == 0, row);
  }
  psum = wave_sum_u64(psum);
  if (lane == 0) {
    atomicAdd(&epi.fraud, fraud);
    atomicAdd(&epi.rows, rows);
    atomicAdd(&epi.psum_e6, psum);
  }
  epi_flush(epi, a.counters);
  signal_done(a, (unsigned)nblk);
}

template <int kMode, int kWaves, bool kR>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(4)))
void score_mlp_kernel(ccfd_score_args a) {
  mlp_body<kMode, kWaves, kR>(a, blockIdx.x, gridDim.x);
}

template <int kWaves, int kPf, bool kR>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(4)))
void score_mlp_wire_kernel(ccfd_score_args a) {
  wire_stream_body<MlpWireScorer, kWaves, kPf, kR>(a, blockIdx.x, gridDim.x);
}

template <int kWaves, int kPf, bool kR>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(2)))
void score_mlp_wire_reg_kernel(ccfd_score_args a) {
  wire_stream_body<MlpWireRegScorer, kWaves, kPf, kR>(a, blockIdx.x, gridDim.x);
}

// Coalesced launch: workgroups [j*wpb, (j+1)*wpb) score sub-batch j.
template <int kMode, int kWaves, bool kR>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(4)))
void score_mlp_multi_kernel(ccfd_multi_args m) {
  // read the table through the kernarg segment pointer: indexing the by-value parameter
  // with the (workgroup-uniform) sub index would make the compiler spill it to scratch
  (void)m;
  const ccfd_multi_args& mk = *(const ccfd_multi_args*)__builtin_amdgcn_kernarg_segment_ptr();
  const int wpb = gridDim.x / mk.nsub;                 // workgroups per sub-batch
  const int j = blockIdx.x / wpb;
  mlp_body<kMode, kWaves, kR>(sub_args(mk, j), blockIdx.x - j * wpb, wpb);
}

template <int kWaves, int kPf, bool kR>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(4)))
void score_mlp_wire_multi_kernel(ccfd_multi_args m) {
  (void)m;
  const ccfd_multi_args& mk = *(const ccfd_multi_args*)__builtin_amdgcn_kernarg_segment_ptr();
  const int wpb = gridDim.x / mk.nsub;
  const int j = blockIdx.x / wpb;
  wire_stream_body<MlpWireScorer, kWaves, kPf, kR>(sub_args(mk, j), blockIdx.x - j * wpb, wpb);
}

// CCFD_MLP_PF: W64 tiles in flight per wave (1, 2, 4).  LDS-weight kernels (coalesced
// launches): default 2 = one tile pair (32.0 vs 31.0 G rows/s at 4,
// profiles/r1/kernel_sol_mlp_pair_sweep.jsonl).  Register-weight kernel (single launches):
// default 4, which takes the four-tile epilogue of wire_body.h (30.1 -> 36.9 G rows/s at 16M
// HBM-resident rows, profiles/r3/kernel_sol/).
static int mlp_wire_prefetch(int dflt = 2) {
  static const int forced = [] {                   // read once: this runs per launch
    const char* e = std::getenv("CCFD_MLP_PF");
    const int x = e ? std::atoi(e) : 0;
    return (x == 1 || x == 2 || x == 4) ? x : 0;
  }();
  return forced ? forced : dflt;
}

// CCFD_MLP_REGW (default 1): W64 weights resident in VGPRs at 2 waves/SIMD
// (MlpWireRegScorer); 0 = per-tile LDS fragment reads at 4 waves/SIMD (MlpWireScorer).
// Measured with 8-wave workgroups (profiles/r1/kernel_sol_mlp_wg_regw_sweep.txt).
static bool mlp_reg_weights() {
  static const bool v = [] {
    const char* e = std::getenv("CCFD_MLP_REGW");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return v;
}

template <int kW, bool kR>
static void launch_wire(dim3 grid, hipStream_t s, const ccfd_score_args& a) {
  if (kW <= 8 && mlp_reg_weights()) {     // 2 waves/SIMD: at most 8 waves per workgroup
    const int cap = 256 * 8 / kW;          // 2 waves/SIMD residency
    if ((int)grid.x > cap) grid.x = cap;
    switch (mlp_wire_prefetch(4)) {
      case 4: hipLaunchKernelGGL((score_mlp_wire_reg_kernel<kW, 4, kR>), grid, dim3(64 * kW), 0, s, a); break;
      default: hipLaunchKernelGGL((score_mlp_wire_reg_kernel<kW, 2, kR>), grid, dim3(64 * kW), 0, s, a); break;
    }
    return;
  }
  switch (mlp_wire_prefetch()) {
    case 1: hipLaunchKernelGGL((score_mlp_wire_kernel<kW, 1, kR>), grid, dim3(64 * kW), 0, s, a); break;
    default: hipLaunchKernelGGL((score_mlp_wire_kernel<kW, 2, kR>), grid, dim3(64 * kW), 0, s, a); break;
    case 4: hipLaunchKernelGGL((score_mlp_wire_kernel<kW, 4, kR>), grid, dim3(64 * kW), 0, s, a); break;
  }
}

// CCFD_MLP_WEIGHTS=global: MFMA weight fragments read straight from the (L1/L2-resident)
// blob instead of a per-workgroup LDS copy -- no staging on the critical path and no LDS
// occupancy limit.  Default: lds.
// CCFD_MLP_TPW: 16-row tiles per wave (1, 2, 4, 8; default 8).  More tiles per wave = fewer workgroups per
// micro-batch, i.e. fewer weight-staging copies and completion releases (each wave keeps
// one tile of prefetch in flight).
int mlp_tiles_per_wave_policy();
static int mlp_tiles_per_wave() { return mlp_tiles_per_wave_policy(); }
int mlp_tiles_per_wave_policy() {
  static const int t = [] {
    const char* e = std::getenv("CCFD_MLP_TPW");
    const int v = e ? std::atoi(e) : 8;     // measured best (profiles/r1/launch_sweep.txt)
    return (v == 1 || v == 2 || v == 4 || v == 8) ? v : 8;
  }();
  return t;
}

static bool mlp_global_weights() {
  static const bool gw = [] {
    const char* e = std::getenv("CCFD_MLP_WEIGHTS");
    return e != nullptr && std::string(e) == "global";
  }();
  return gw;
}

template <int kW, bool kR>
static void launch_w(const ccfd_score_args& a, int ntiles, bool contig, hipStream_t s) {
  const int per_wg = kW * mlp_tiles_per_wave();
  int grid = (ntiles + per_wg - 1) / per_wg;
  // cap: one full residency of the chip (256 CUs x 16 waves at the 128-VGPR cap); a
  // grid-stride loop covers the rest, so large HBM-resident launches do not pay a second
  // round of weight staging and counter flushes
  const int cap = 256 * 16 / kW;
  grid = grid < 1 ? 1 : (grid > cap ? cap : grid);
  const bool gw = mlp_global_weights();
  if (a.flags & CCFD_ARG_WIRE_W64) {
    launch_wire<kW, kR>(dim3(grid), s, a);
  } else if (contig) {
    if (gw) hipLaunchKernelGGL((score_mlp_kernel<5, kW, kR>), dim3(grid), dim3(64 * kW), 0, s, a);
    else hipLaunchKernelGGL((score_mlp_kernel<1, kW, kR>), dim3(grid), dim3(64 * kW), 0, s, a);
  } else {
    hipLaunchKernelGGL((score_mlp_kernel<0, kW, kR>), dim3(grid), dim3(64 * kW), 0, s, a);
  }
}

int mlp_waves_for(int ntiles) {
  static const int forced = [] {
    const char* e = std::getenv("CCFD_MLP_WAVES");
    return e ? std::atoi(e) : 0;
  }();
  if (forced == 1 || forced == 2 || forced == 4 || forced == 8 || forced == 16) return forced;
  (void)ntiles;
  return 4;   // measured: 1-wave workgroups lose (per-workgroup weight staging + completion)
}

template <bool kR>
static int launch_mlp_multi_t(const ccfd_multi_args& m, hipStream_t s) {
  constexpr int kW = 4;
  const int rows_per_wg = kTileRows * kW * mlp_tiles_per_wave();
  const int wpb = (m.sub_rows + rows_per_wg - 1) / rows_per_wg;
  const dim3 grid(wpb * m.nsub), block(64 * kW);
  const bool gw = mlp_global_weights();
  if (m.base.flags & CCFD_ARG_WIRE_W64) {
    switch (mlp_wire_prefetch()) {
      case 1: hipLaunchKernelGGL((score_mlp_wire_multi_kernel<kW, 1, kR>), grid, block, 0, s, m); break;
      default: hipLaunchKernelGGL((score_mlp_wire_multi_kernel<kW, 2, kR>), grid, block, 0, s, m); break;
      case 4: hipLaunchKernelGGL((score_mlp_wire_multi_kernel<kW, 4, kR>), grid, block, 0, s, m); break;
    }
  } else {
    if (gw) hipLaunchKernelGGL((score_mlp_multi_kernel<5, kW, kR>), grid, block, 0, s, m);
    else hipLaunchKernelGGL((score_mlp_multi_kernel<1, kW, kR>), grid, block, 0, s, m);
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_mlp_multi(const ccfd_multi_args& m, hipStream_t s) {
  return m.base.rules ? launch_mlp_multi_t<true>(m, s) : launch_mlp_multi_t<false>(m, s);
}

// Waves per workgroup of the W64 single launch: CCFD_MLP_WAVES when set, else 8 -- half the
// blob stagings and counter flushes of 4-wave groups, and the widest group the 2-waves/SIMD
// register-weight kernel allows (+47 % at 256K-1M rows, same at 16M).
static int mlp_wire_waves(int ntiles) {
  static const bool forced = std::getenv("CCFD_MLP_WAVES") != nullptr;
  return forced ? mlp_waves_for(ntiles) : 8;
}

template <bool kR>
static int launch_mlp_t(const ccfd_score_args& a, hipStream_t s) {
  const int ntiles = (a.n + kTileRows - 1) / kTileRows;
  const bool contig = a.ld == kF && (reinterpret_cast<uintptr_t>(a.x) & 15) == 0;
  const int w = (a.flags & CCFD_ARG_WIRE_W64) ? mlp_wire_waves(ntiles) : mlp_waves_for(ntiles);
  if ((a.flags & CCFD_ARG_WIRE_W64) && (w == 8 || w == 16)) {
    // wider workgroups for the W64 path: one blob staging, flush and completion release per
    // 8 or 16 waves instead of per 4
    const int per_wg = w * mlp_tiles_per_wave();
    int grid = (ntiles + per_wg - 1) / per_wg;
    const int cap = 256 * 16 / w;
    grid = grid < 1 ? 1 : (grid > cap ? cap : grid);
    if (w == 8) launch_wire<8, kR>(dim3(grid), s, a);
    else launch_wire<16, kR>(dim3(grid), s, a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
  }
  switch (w) {
    case 1: launch_w<1, kR>(a, ntiles, contig, s); break;
    case 2: launch_w<2, kR>(a, ntiles, contig, s); break;
    default: launch_w<4, kR>(a, ntiles, contig, s); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_mlp(const ccfd_score_args& a, hipStream_t s) {
  return a.rules ? launch_mlp_t<true>(a, s) : launch_mlp_t<false>(a, s);
}

}  // namespace ccfd
