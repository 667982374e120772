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
#include "common.h"

namespace ccfd {

constexpr int kMlpBlob = 25920;           // models/mlp.py BLOB_BYTES
constexpr int kOffNorm = 64;
constexpr int kOffW1 = kOffNorm + 256;
constexpr int kOffW2 = kOffW1 + 8 * 64 * 16;
constexpr int kOffB1 = kOffW2 + 16 * 64 * 16;
constexpr int kOffB2 = kOffB1 + 8 * 4 * 16;
constexpr int kOffW3 = kOffB2 + 4 * 4 * 16;
static_assert(kOffW3 + 4 * 4 * 16 == kMlpBlob, "blob layout");
constexpr int kWaves = 4;

template <bool kContig>
__global__ __launch_bounds__(256) void score_mlp_kernel(ccfd_score_args a) {
  __shared__ __attribute__((aligned(16))) char sblob[kMlpBlob];
  __shared__ __attribute__((aligned(16))) float sx[kWaves][kTileRows * kF + 4];
  __shared__ EpilogueLds epi;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int ntiles = (a.n + kTileRows - 1) / kTileRows;
  const int tstride = gridDim.x * kWaves;
  int tile = blockIdx.x * kWaves + wave;

  // Issue this wave's first input tile BEFORE staging the weights: the (possibly PCIe)
  // fetch latency of x overlaps the L2 fetch of the model blob.
  TileRegs pre;
  auto tile_avail = [&](int t) { return min(kTileRows, a.n - t * kTileRows) * kF * 4; };
  if constexpr (kContig) {
    if (tile < ntiles) tile_issue(a.x + (size_t)tile * kTileRows * kF, tile_avail(tile), lane, pre);
  }
  {  // stage the packed model: 1620 x 16 B
    const int4* src = reinterpret_cast<const int4*>(a.blob);
    int4* dst = reinterpret_cast<int4*>(sblob);
    for (int i = tid; i < kMlpBlob / 16; i += 256) dst[i] = src[i];
  }
  epi_init(epi);
  __syncthreads();

  const unsigned flags = *reinterpret_cast<const unsigned*>(sblob + 4);
  const float b3 = *reinterpret_cast<const float*>(sblob + 8);
  float mu[8], isg[8];
  {
    const f32x4* m4 = reinterpret_cast<const f32x4*>(sblob + kOffNorm) + 2 * g;
    const f32x4* s4 = reinterpret_cast<const f32x4*>(sblob + kOffNorm + 128) + 2 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mu[j] = m4[0][j]; mu[4 + j] = m4[1][j];
      isg[j] = s4[0][j]; isg[4 + j] = s4[1][j];
    }
  }
  const bf16x8* W1f = reinterpret_cast<const bf16x8*>(sblob + kOffW1);
  const bf16x8* W2f = reinterpret_cast<const bf16x8*>(sblob + kOffW2);
  const f32x4* b1f = reinterpret_cast<const f32x4*>(sblob + kOffB1);
  const f32x4* b2f = reinterpret_cast<const f32x4*>(sblob + kOffB2);
  const f32x4* w3f = reinterpret_cast<const f32x4*>(sblob + kOffW3);
  const bool log_amount = (flags & 1u) != 0;
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
      const float2* r2 = reinterpret_cast<const float2*>(tile_lds + c * kF + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float2 v = (g < 3 || j < 3) ? r2[j] : make_float2(0.f, 0.f);
        xv[2 * j] = v.x; xv[2 * j + 1] = v.y;
      }
    } else {
      const float* xr = a.x + (size_t)row * a.ld + 8 * g;
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[j] = (valid && (8 * g + j) < kF) ? xr[j] : 0.f;
    }
    const float amount = xv[5];               // raw Amount (valid in lane group 3)
    if (g == 3) {
      xv[6] = 0.f; xv[7] = 0.f;
      if (log_amount) xv[5] = log1pf(fmaxf(xv[5], 0.f));
    }
    bf16x8 xb;
#pragma unroll
    for (int j = 0; j < 8; ++j) xb[j] = (__bf16)((xv[j] - mu[j]) * isg[j]);

    // ---- layer 1: H1^T = W1 . Xn^T  (+ b1 as accumulator init)
    f32x4 acc1[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      acc1[t] = b1f[t * 4 + g];
      acc1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W1f[t * 64 + lane], xb, acc1[t], 0, 0, 0);
    }
    // ---- relu + bf16: accumulator tiles (2s, 2s+1) are K-step s of layer 2 (k order pi)
    bf16x8 hb[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hb[s][r] = (__bf16)fmaxf(acc1[2 * s][r], 0.f);
        hb[s][4 + r] = (__bf16)fmaxf(acc1[2 * s + 1][r], 0.f);
      }
    }
    // ---- layer 2 + layer 3 partial dot
    float z = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x4 acc = b2f[u * 4 + g];
#pragma unroll
      for (int s = 0; s < 4; ++s)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W2f[(u * 4 + s) * 64 + lane], hb[s], acc, 0, 0, 0);
      const f32x4 w3v = w3f[u * 4 + g];
#pragma unroll
      for (int r = 0; r < 4; ++r) z = fmaf(fmaxf(acc[r], 0.f), w3v[r], z);
    }
    z += __shfl_xor(z, 16);
    z += __shfl_xor(z, 32);
    const float p = sigmoid(z + b3);
    const bool fr = valid && (p >= thr);

    if (valid && g == 0) {
      if (a.proba) a.proba[row] = p;
      if (a.route) a.route[row] = fr ? 1 : 0;
      psum += (unsigned long long)(p * 1e6f + 0.5f);
    }
    const unsigned long long mf = __ballot(fr && g == 0);
    const unsigned long long mv = __ballot(valid && g == 0);
    fraud += __popcll(mf);
    rows += __popcll(mv);
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
  signal_done(a);
}

template __global__ void score_mlp_kernel<true>(ccfd_score_args);
template __global__ void score_mlp_kernel<false>(ccfd_score_args);

int launch_mlp(const ccfd_score_args& a, hipStream_t s) {
  const int ntiles = (a.n + kTileRows - 1) / kTileRows;
  int grid = (ntiles + kWaves - 1) / kWaves;
  grid = grid < 1 ? 1 : (grid > 2048 ? 2048 : grid);
  const bool contig = a.ld == kF && (reinterpret_cast<uintptr_t>(a.x) & 15) == 0;
  if (contig)
    hipLaunchKernelGGL(score_mlp_kernel<true>, dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(score_mlp_kernel<false>, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace ccfd
