// Fused logistic-regression scorer: normalize -> w.x + b -> sigmoid -> threshold ->
// counters.  Same 16-row tile / 4-lanes-per-row layout as score_mlp.hip so the input is
// read with full-width coalesced loads; the 30-term dot product is 8 FMAs per lane plus
// two xor-shuffles.  GPU counterpart of the config-1 LR model (BASELINE.json configs[0]).
#include "common.h"

namespace ccfd {

constexpr int kLrBlob = 64 + 3 * 32 * 4;   // models/lr.py BLOB_BYTES

// waves per workgroup: see score_mlp.hip (small micro-batches use 1-wave workgroups so the
// grid covers every CU)
// kMode as in score_mlp.hip: 0 strided f32, 1 contiguous f32, 2 W64 wire rows
template <int kMode, int kLrWaves>
__global__ __launch_bounds__(64 * kLrWaves) void score_lr_kernel(ccfd_score_args a) {
  constexpr bool kContig = kMode == 1;
  constexpr bool kWire = kMode == 2;
  __shared__ __attribute__((aligned(16))) float sx[kLrWaves][kTileRows * kF + 4];
  __shared__ EpilogueLds epi;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
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
  const int ntiles = (a.n + kTileRows - 1) / kTileRows;
  float* tile_lds = sx[wave];
  for (int tile = blockIdx.x * kLrWaves + wave; tile < ntiles; tile += gridDim.x * kLrWaves) {
    const int row = tile * kTileRows + c;
    const bool valid = row < a.n;
    float xv[8];
    if constexpr (kContig) {
      const int rows_here = min(kTileRows, a.n - tile * kTileRows);
      load_tile_contig(a.x + (size_t)tile * kTileRows * kF, rows_here * kF * 4, tile_lds, lane);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      const float2* r2 = reinterpret_cast<const float2*>(tile_lds + c * kF + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float2 v = (g < 3 || j < 3) ? r2[j] : make_float2(0.f, 0.f);
        xv[2 * j] = v.x; xv[2 * j + 1] = v.y;
      }
    } else if constexpr (kWire) {
      WireRegs r;
      wire_issue(reinterpret_cast<const unsigned char*>(a.x), a.n, tile, c, g, r);
      wire_features(r, g, xv);
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
    const bool fr = valid && (p >= a.threshold);
    if (valid && g == 0) {
      if (a.proba) a.proba[row] = p;
      if (a.route) a.route[row] = fr ? 1 : 0;
      psum += (unsigned long long)(p * 1e6f + 0.5f);
    }
    fraud += __popcll(__ballot(fr && g == 0));
    rows += __popcll(__ballot(valid && g == 0));
    if (valid && g == 3) atomicAdd(&epi.hist[(fr ? kNB : 0) + amount_bucket(amount)], 1u);
    emit_flagged(a, fr && g == 0, row);
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

int mlp_waves_for(int ntiles);   // score_mlp.hip (same policy and CCFD_MLP_WAVES override)

template <int kW>
static void launch_lr_w(const ccfd_score_args& a, int ntiles, bool contig, hipStream_t s) {
  int grid = (ntiles + kW - 1) / kW;
  grid = grid < 1 ? 1 : (grid > 2048 ? 2048 : grid);
  if (a.flags & CCFD_ARG_WIRE_W64)
    hipLaunchKernelGGL((score_lr_kernel<2, kW>), dim3(grid), dim3(64 * kW), 0, s, a);
  else if (contig)
    hipLaunchKernelGGL((score_lr_kernel<1, kW>), dim3(grid), dim3(64 * kW), 0, s, a);
  else
    hipLaunchKernelGGL((score_lr_kernel<0, kW>), dim3(grid), dim3(64 * kW), 0, s, a);
}

int launch_lr(const ccfd_score_args& a, hipStream_t s) {
  const int ntiles = (a.n + kTileRows - 1) / kTileRows;
  const bool contig = a.ld == kF && (reinterpret_cast<uintptr_t>(a.x) & 15) == 0;
  switch (mlp_waves_for(ntiles)) {
    case 1: launch_lr_w<1>(a, ntiles, contig, s); break;
    case 2: launch_lr_w<2>(a, ntiles, contig, s); break;
    default: launch_lr_w<4>(a, ntiles, contig, s); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace ccfd
