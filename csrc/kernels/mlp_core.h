// MLP 30->128->64->1 per-16-row-tile math shared by the per-batch kernel (score_mlp.hip)
// and the persistent streaming kernel (score_persist.hip).  Layout derivation of the
// packed blob and of the transposed-activation MFMA chain: models/mlp.py.
#pragma once
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

// Stage the packed model (1620 x 16 B) into LDS; caller synchronises.
__device__ __forceinline__ void mlp_stage(const void* blob, char* sblob, int tid, int nthreads) {
  const int4* src = reinterpret_cast<const int4*>(blob);
  int4* dst = reinterpret_cast<int4*>(sblob);
  for (int i = tid; i < kMlpBlob / 16; i += nthreads) dst[i] = src[i];
}

// Per-lane constants (lane group g = lane >> 4 owns features 8g..8g+7).
struct MlpLane {
  float mu[8], isg[8];
  float b3;
  bool log_amount;
};

__device__ __forceinline__ MlpLane mlp_lane(const char* sblob, int g) {
  MlpLane L;
  const unsigned flags = *reinterpret_cast<const unsigned*>(sblob + 4);
  L.b3 = *reinterpret_cast<const float*>(sblob + 8);
  L.log_amount = (flags & 1u) != 0;
  const f32x4* m4 = reinterpret_cast<const f32x4*>(sblob + kOffNorm) + 2 * g;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(sblob + kOffNorm + 128) + 2 * g;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    L.mu[j] = m4[0][j]; L.mu[4 + j] = m4[1][j];
    L.isg[j] = s4[0][j]; L.isg[4 + j] = s4[1][j];
  }
  return L;
}

// proba_1 of row (lane & 15) of the tile; identical in all four lane groups.
// xv: raw features (consumed); amount_out: raw Amount (valid in lane group 3).
__device__ __forceinline__ float mlp_tile(const char* sblob, const MlpLane& L, float xv[8], int g, int lane,
                                          float& amount_out) {
  amount_out = xv[5];
  if (g == 3) {
    xv[6] = 0.f; xv[7] = 0.f;
    if (L.log_amount) xv[5] = log1pf(fmaxf(xv[5], 0.f));
  }
  bf16x8 xb;
#pragma unroll
  for (int j = 0; j < 8; ++j) xb[j] = (__bf16)((xv[j] - L.mu[j]) * L.isg[j]);

  const bf16x8* W1f = reinterpret_cast<const bf16x8*>(sblob + kOffW1);
  const bf16x8* W2f = reinterpret_cast<const bf16x8*>(sblob + kOffW2);
  const f32x4* b1f = reinterpret_cast<const f32x4*>(sblob + kOffB1);
  const f32x4* b2f = reinterpret_cast<const f32x4*>(sblob + kOffB2);
  const f32x4* w3f = reinterpret_cast<const f32x4*>(sblob + kOffW3);

  // layer 1: H1^T = W1 . Xn^T  (+ b1 as accumulator init)
  f32x4 acc1[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    acc1[t] = b1f[t * 4 + g];
    acc1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W1f[t * 64 + lane], xb, acc1[t], 0, 0, 0);
  }
  // relu + bf16: accumulator tiles (2s, 2s+1) are K-step s of layer 2 (k order pi)
  bf16x8 hb[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      hb[s][r] = (__bf16)fmaxf(acc1[2 * s][r], 0.f);
      hb[s][4 + r] = (__bf16)fmaxf(acc1[2 * s + 1][r], 0.f);
    }
  }
  // layer 2 + layer-3 partial dot
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
  return sigmoid(z + L.b3);
}

}  // namespace ccfd
