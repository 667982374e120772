// Fused logistic-regression scorer: normalize -> w.x + b -> sigmoid -> threshold ->
// counters.  Same 16-row tile / 4-lanes-per-row layout as score_mlp.hip so the input is
// read with full-width coalesced loads; the 30-term dot product is 8 FMAs per lane plus
// two xor-shuffles.  GPU counterpart of the config-1 LR model (BASELINE.json configs[0]).
// Launch structure mirrors score_mlp.hip: a plain and a coalesced (multi-micro-batch) entry
// over one body, tiles-per-wave with a one-tile prefetch.
#include <cstdlib>

#include "common.h"
#include "wire_body.h"

namespace ccfd {

int mlp_waves_for(int ntiles);     // score_mlp.hip (same policy and CCFD_MLP_WAVES override)
int mlp_tiles_per_wave_policy();   // score_mlp.hip (CCFD_MLP_TPW)

// f32 rows, kMode as in score_mlp.hip: 0 strided, 1 contiguous (W64 rows: LrWireScorer below)
template <int kMode, int kLrWaves, bool kR>
__device__ __forceinline__ void lr_body(const ccfd_score_args& a, int blk, int nblk) {
  constexpr bool kContig = kMode == 1;
  static_assert(kMode != 2, "W64 rows use wire_stream_body");
  __shared__ __attribute__((aligned(16))) float sx[kContig ? kLrWaves : 1][kTileRows * kF + 4];
  __shared__ EpilogueLds epi;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  stamp_start(a, blk);
  const int ntiles = (a.n + kTileRows - 1) / kTileRows;
  const int tstride = nblk * kLrWaves;
  int tile = blk * kLrWaves + wave;

  TileRegs pre;
  auto tile_avail = [&](int t) { return min(kTileRows, a.n - t * kTileRows) * kF * 4; };
  if constexpr (kContig) {
    if (tile < ntiles) tile_issue(a.x + (size_t)tile * kTileRows * kF, tile_avail(tile), lane, pre);
  }
  epi_init(epi);

  const char* blob = reinterpret_cast<const char*>(a.blob);
  const unsigned flags = *reinterpret_cast<const unsigned*>(blob + 4);
  const float b = *reinterpret_cast<const float*>(blob + 8);
  const float* mu = reinterpret_cast<const float*>(blob + 64) + 8 * g;
  const float* isg = reinterpret_cast<const float*>(blob + 192) + 8 * g;
  const float* w = reinterpret_cast<const float*>(blob + 320) + 8 * g;
  float wm[8], ws[8], wmu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { wmu[j] = mu[j]; ws[j] = isg[j]; wm[j] = w[j]; }
  const bool log_amount = (flags & 1u) != 0;
  __syncthreads();

  unsigned fraud = 0, rows = 0;
  unsigned long long psum = 0;
  float* tile_lds = sx[kContig ? wave : 0];
  for (; tile < ntiles; tile += tstride) {
    const int row = tile * kTileRows + c;
    const bool valid = row < a.n;
    const int nxt = tile + tstride;
    float xv[8];
    if constexpr (kContig) {
      tile_store(tile_lds, lane, pre);
      if (nxt < ntiles) tile_issue(a.x + (size_t)nxt * kTileRows * kF, tile_avail(nxt), lane, pre);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      tile_features(tile_lds, c, g, xv);
    } else {
      const float* xr = a.x + (size_t)row * a.ld + 8 * g;
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[j] = (valid && (8 * g + j) < kF) ? xr[j] : 0.f;
    }
    const float amount = xv[5];
    if (g == 3) {
      xv[6] = 0.f; xv[7] = 0.f;
      if (log_amount) xv[5] = log1pf(fmaxf(xv[5], 0.f));
    }
    float z = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) z = fmaf((xv[j] - wmu[j]) * ws[j], wm[j], z);
    z += __shfl_xor(z, 16);
    z += __shfl_xor(z, 32);
    const float p = sigmoid(z + b);
    bool fr;
    if constexpr (kR) {                                 // configurable routing rules (rules.h)
      if (g == 3) xv[5] = amount;
      fr = valid && rule_route(a.rules, __shfl(p, c), [&](int j) { return lane_feature<false>(xv, j, c); });
    } else {
      fr = valid && (p >= a.threshold);
    }
    if (valid && g == 0) {
      if (a.proba) st_g(a.proba + row, p);
      if (a.route) st_g(a.route + row, (uint8_t)(fr ? 1 : 0));
      psum += (unsigned)(p * 1e6f + 0.5f);
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

template <int kMode, int kLrWaves, bool kR>
__global__ __launch_bounds__(64 * kLrWaves) void score_lr_kernel(ccfd_score_args a) {
  lr_body<kMode, kLrWaves, kR>(a, blockIdx.x, gridDim.x);
}

template <int kMode, int kLrWaves, bool kR>
__global__ __launch_bounds__(64 * kLrWaves) void score_lr_multi_kernel(ccfd_multi_args m) {
  (void)m;   // table read through the kernarg segment (see score_mlp_multi_kernel)
  const ccfd_multi_args& mk = *(const ccfd_multi_args*)__builtin_amdgcn_kernarg_segment_ptr();
  const int wpb = gridDim.x / mk.nsub;
  const int j = blockIdx.x / wpb;
  lr_body<kMode, kLrWaves, kR>(sub_args(mk, j), blockIdx.x - j * wpb, wpb);
}


// W64 wire rows: the blob (models/lr.py pack(wire=True)) has the normaliser folded into w/b,
// so the dot product runs on the raw row values -- bf16 V-columns widened by one shift/mask,
// Time as f32, Amount as log2(1 + a) with ln 2 folded into its weight -- through the shared
// prefetch-ring streaming body (wire_body.h).
struct LrWireScorer {
  static constexpr int kLds = 0;
  float w[8];
  float b;
  bool log_amount;
  __device__ __forceinline__ void stage(const ccfd_score_args&, char*, int, int) {}
  __device__ __forceinline__ void lanes(const char*, const ccfd_score_args& a, int g) {
    const char* blob = reinterpret_cast<const char*>(a.blob);
    const unsigned flags = *reinterpret_cast<const unsigned*>(blob + 4);
    b = *reinterpret_cast<const float*>(blob + 8);
    log_amount = (flags & 1u) != 0;
    const float* wp = reinterpret_cast<const float*>(blob + 320) + 8 * g;
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = wp[j];
    if (g == 3 && log_amount) w[5] *= 0.693147180559945f;
  }
  __device__ __forceinline__ float tile(const char* lds, const WireRegs& r, int g, int lane) const {
    return proba(logit(lds, r, g, lane));
  }
  __device__ __forceinline__ float proba(float z) const { return __builtin_amdgcn_rcpf(1.f + __expf(-z)); }
  __device__ __forceinline__ float logit(const char*, const WireRegs& r, int g, int) const {
    const bool g3 = g == 3;
    const uint4 v = r.v;
    float am = __uint_as_float(v.w);
    if (log_amount) am = __log2f(1.f + __builtin_amdgcn_fmed3f(am, 0.f, 3.4e38f));
    float x[8];
    x[0] = __uint_as_float(v.x << 16); x[1] = __uint_as_float(v.x & 0xffff0000u);
    x[2] = __uint_as_float(v.y << 16); x[3] = __uint_as_float(v.y & 0xffff0000u);
    x[4] = g3 ? __uint_as_float(v.z) : __uint_as_float(v.z << 16);
    x[5] = g3 ? am : __uint_as_float(v.z & 0xffff0000u);
    x[6] = g3 ? 0.f : __uint_as_float(v.w << 16);
    x[7] = g3 ? 0.f : __uint_as_float(v.w & 0xffff0000u);
    float z = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) z = fmaf(w[j], x[j], z);
    z += __shfl_xor(z, 16);
    z += __shfl_xor(z, 32);
    return z + b;
  }
  static constexpr bool kPair = false;
  static constexpr bool kQuad = true;
  __device__ __forceinline__ void logit2(const char* lds, const WireRegs& r0, const WireRegs& r1, int g, int lane,
                                         float& z0, float& z1) const {
    z0 = logit(lds, r0, g, lane);
    z1 = logit(lds, r1, g, lane);
  }
  __device__ __forceinline__ void tile2(const char* lds, const WireRegs& r0, const WireRegs& r1, int g, int lane,
                                        float& p0, float& p1) const {
    p0 = tile(lds, r0, g, lane);
    p1 = tile(lds, r1, g, lane);
  }
};

template <int kLrWaves, int kPf, bool kR>
__global__ __launch_bounds__(64 * kLrWaves) void score_lr_wire_kernel(ccfd_score_args a) {
  wire_stream_body<LrWireScorer, kLrWaves, kPf, kR>(a, blockIdx.x, gridDim.x);
}

template <int kLrWaves, int kPf, bool kR>
__global__ __launch_bounds__(64 * kLrWaves) void score_lr_wire_multi_kernel(ccfd_multi_args m) {
  (void)m;
  const ccfd_multi_args& mk = *(const ccfd_multi_args*)__builtin_amdgcn_kernarg_segment_ptr();
  const int wpb = gridDim.x / mk.nsub;
  const int j = blockIdx.x / wpb;
  wire_stream_body<LrWireScorer, kLrWaves, kPf, kR>(sub_args(mk, j), blockIdx.x - j * wpb, wpb);
}

// CCFD_LR_PF: W64 tiles in flight per wave (2, 4, 8; default 4).  CCFD_LR_OCC: resident
// waves per SIMD the wire grid is sized for (4 or 8; default 4).  The LR scorer stages no
// LDS and needs few VGPRs, so both only trade bytes in flight against grid-stride overhead.
static int lr_env(const char* name, int def, int a, int b, int c) {
  const char* e = std::getenv(name);
  const int x = e ? std::atoi(e) : def;
  return (x == a || x == b || x == c) ? x : def;
}
static int lr_wire_prefetch() {
  static const int v = lr_env("CCFD_LR_PF", 4, 2, 4, 8);
  return v;
}
static int lr_wire_occupancy() {
  static const int v = lr_env("CCFD_LR_OCC", 4, 4, 8, 4);
  return v;
}

template <int kW, bool kR>
static void launch_lr_wire(dim3 grid, hipStream_t s, const ccfd_score_args& a) {
  switch (lr_wire_prefetch()) {
    case 2: hipLaunchKernelGGL((score_lr_wire_kernel<kW, 2, kR>), grid, dim3(64 * kW), 0, s, a); break;
    default: hipLaunchKernelGGL((score_lr_wire_kernel<kW, 4, kR>), grid, dim3(64 * kW), 0, s, a); break;
    case 8: hipLaunchKernelGGL((score_lr_wire_kernel<kW, 8, kR>), grid, dim3(64 * kW), 0, s, a); break;
  }
}

template <int kW, bool kR>
static void launch_lr_w(const ccfd_score_args& a, int ntiles, bool contig, hipStream_t s) {
  const int per_wg = kW * mlp_tiles_per_wave_policy();
  int grid = (ntiles + per_wg - 1) / per_wg;
  if (a.flags & CCFD_ARG_WIRE_W64) {
    const int cap = 256 * 4 * lr_wire_occupancy() / kW;   // one chip residency, grid-stride beyond
    grid = grid < 1 ? 1 : (grid > cap ? cap : grid);
    launch_lr_wire<kW, kR>(dim3(grid), s, a);
    return;
  }
  grid = grid < 1 ? 1 : (grid > 2048 ? 2048 : grid);
  if (contig)
    hipLaunchKernelGGL((score_lr_kernel<1, kW, kR>), dim3(grid), dim3(64 * kW), 0, s, a);
  else
    hipLaunchKernelGGL((score_lr_kernel<0, kW, kR>), dim3(grid), dim3(64 * kW), 0, s, a);
}

// CCFD_LR_WAVES: waves per workgroup of the W64 single launch (4, 8, 16; default 16 -- one
// counter flush per 16 waves; G rows/s at 1M / 4M / 16M rows: 16.3 / 44.4 / 61.1 with 4,
// 35.5 / 67.9 / 66.1 with 16, profiles/r1/kernel_sol_lr_wg_sweep.txt).
static int lr_wire_waves() {
  static const int v = lr_env("CCFD_LR_WAVES", 16, 4, 8, 16);
  return v;
}

template <bool kR>
static int launch_lr_t(const ccfd_score_args& a, hipStream_t s) {
  const int ntiles = (a.n + kTileRows - 1) / kTileRows;
  const bool contig = a.ld == kF && (reinterpret_cast<uintptr_t>(a.x) & 15) == 0;
  if (a.flags & CCFD_ARG_WIRE_W64) {
    switch (lr_wire_waves()) {
      case 4: launch_lr_w<4, kR>(a, ntiles, contig, s); break;
      case 8: launch_lr_w<8, kR>(a, ntiles, contig, s); break;
      default: launch_lr_w<16, kR>(a, ntiles, contig, s); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
  }
  switch (mlp_waves_for(ntiles)) {
    case 1: launch_lr_w<1, kR>(a, ntiles, contig, s); break;
    case 2: launch_lr_w<2, kR>(a, ntiles, contig, s); break;
    default: launch_lr_w<4, kR>(a, ntiles, contig, s); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_lr(const ccfd_score_args& a, hipStream_t s) {
  return a.rules ? launch_lr_t<true>(a, s) : launch_lr_t<false>(a, s);
}

template <bool kR>
static int launch_lr_multi_t(const ccfd_multi_args& m, hipStream_t s) {
  constexpr int kW = 4;
  const int rows_per_wg = kTileRows * kW * mlp_tiles_per_wave_policy();
  const int wpb = (m.sub_rows + rows_per_wg - 1) / rows_per_wg;
  const dim3 grid(wpb * m.nsub), block(64 * kW);
  if (m.base.flags & CCFD_ARG_WIRE_W64)
    hipLaunchKernelGGL((score_lr_wire_multi_kernel<kW, 4, kR>), grid, block, 0, s, m);
  else
    hipLaunchKernelGGL((score_lr_multi_kernel<1, kW, kR>), grid, block, 0, s, m);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_lr_multi(const ccfd_multi_args& m, hipStream_t s) {
  return m.base.rules ? launch_lr_multi_t<true>(m, s) : launch_lr_multi_t<false>(m, s);
}

}  // namespace ccfd
