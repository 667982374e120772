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
// W64 wire blobs append layer 3 as MFMA A-fragments (models/mlp.py WIRE_BLOB_BYTES)
constexpr int kOffW3F = kMlpBlob;
constexpr int kMlpBlobWire = kOffW3F + 2 * 64 * 16;

// Stage the packed model (bytes / 16 int4) into LDS; caller synchronises.
__device__ __forceinline__ void mlp_stage(const void* blob, char* sblob, int tid, int nthreads,
                                          int bytes = kMlpBlob) {
  const int4* src = reinterpret_cast<const int4*>(blob);
  int4* dst = reinterpret_cast<int4*>(sblob);
  for (int i = tid; i < bytes / 16; i += nthreads) dst[i] = src[i];
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

// ---------------------------------------------------------------------------------------
// W64 wire rows (blob from models/mlp.py pack(wire=True)).  A lane's 16-B chunk of the row
// IS its layer-1 B fragment: the bf16 V-columns enter the MFMA as raw bits (their
// normalisation is folded into W1/b1 at pack time), b1 rides in K-columns 30/31 against
// constant-1 inputs, and only Time/Amount (lane group 3) are normalised here -- ~10 VALU
// instead of unpack + 8 x normalise + convert per lane.
// ---------------------------------------------------------------------------------------
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  // one v_cvt_pk_bf16_f32 (RNE); a pair of scalar (__bf16) casts is emitted as two
  // single-lane converts + v_perm
  const f32x2 f = {lo, hi};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f, bf16x2));
}

// relu on two packed bf16: a negative bf16 is a negative int16 (sign bit), so one
// v_pk_max_i16 against 0 is the ReLU of both halves (relu commutes with RNE rounding).
__device__ __forceinline__ unsigned relu_pack_bf16x2(float lo, float hi) {
  s16x2 v = __builtin_bit_cast(s16x2, pack_bf16x2(lo, hi));
  v = __builtin_elementwise_max(v, (s16x2){0, 0});
  return __builtin_bit_cast(unsigned, v);
}

struct MlpWireLane {
  float t_scale, t_shift;   // Time (wire K 28):   bf16(t * isg - mu * isg)
  float a_scale, a_shift;   // Amount (wire K 29): log1p as log2 with ln 2 folded into the scale
  float b3;
  bool log_amount;
};

__device__ __forceinline__ MlpWireLane mlp_wire_lane(const char* sblob) {
  MlpWireLane L;
  const unsigned flags = *reinterpret_cast<const unsigned*>(sblob + 4);
  L.b3 = *reinterpret_cast<const float*>(sblob + 8);
  L.log_amount = (flags & 1u) != 0;
  const float* mu = reinterpret_cast<const float*>(sblob + kOffNorm);
  const float* isg = mu + 32;
  L.t_scale = isg[28];
  L.t_shift = -mu[28] * isg[28];
  L.a_scale = isg[29] * (L.log_amount ? 0.693147180559945f : 1.f);
  L.a_shift = -mu[29] * isg[29];
  return L;
}

__device__ __forceinline__ bf16x8 wire_operand(const WireRegs& r, bool g3, const MlpWireLane& L) {
  const float t = __uint_as_float(r.v.z);
  float am = __uint_as_float(r.v.w);
  if (L.log_amount) am = __log2f(1.f + __builtin_amdgcn_fmed3f(am, 0.f, 3.4e38f));   // v_med3 + v_log_f32
  const unsigned pk = pack_bf16x2(fmaf(t, L.t_scale, L.t_shift), fmaf(am, L.a_scale, L.a_shift));
  uint4 u = r.v;
  u.z = g3 ? pk : u.z;
  u.w = g3 ? 0x3F803F80u : u.w;                         // bf16 1.0, 1.0: the b1 hi/lo inputs
  return __builtin_bit_cast(bf16x8, u);
}

// proba_1 of row (lane & 15) of the tile from its W64 lane chunk; identical in all four
// lane groups.  Layer 1 needs no accumulator init (b1 is inside the MFMA), layer-1 ReLU +
// bf16 pack is 2 VALU per pair, the sigmoid uses the hardware reciprocal.
__device__ __forceinline__ float mlp_tile_w64(const char* sblob, const MlpWireLane& L, const WireRegs& r,
                                              int g, int lane) {
  const bf16x8 xb = wire_operand(r, g == 3, L);
  const bf16x8* W1f = reinterpret_cast<const bf16x8*>(sblob + kOffW1);
  const bf16x8* W2f = reinterpret_cast<const bf16x8*>(sblob + kOffW2);
  const f32x4* b2f = reinterpret_cast<const f32x4*>(sblob + kOffB2);
  const f32x4* w3f = reinterpret_cast<const f32x4*>(sblob + kOffW3);
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4 acc1[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W1f[t * 64 + lane], xb, zero, 0, 0, 0);
  bf16x8 hb[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const uint4 u = make_uint4(relu_pack_bf16x2(acc1[2 * s][0], acc1[2 * s][1]),
                               relu_pack_bf16x2(acc1[2 * s][2], acc1[2 * s][3]),
                               relu_pack_bf16x2(acc1[2 * s + 1][0], acc1[2 * s + 1][1]),
                               relu_pack_bf16x2(acc1[2 * s + 1][2], acc1[2 * s + 1][3]));
    hb[s] = __builtin_bit_cast(bf16x8, u);
  }
  // layer 2, then layer 3 as two more MFMAs: relu(H2^T) packed to bf16 exactly like layer 1's
  // output (K-step s' = M-tiles 2s', 2s'+1) against W3pad, whose rows 0/4/8/12 hold w3 -- so
  // register 0 of EVERY lane group receives z of row (lane & 15): no cross-lane reduction
  f32x4 acc2[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f32x4 acc = b2f[u * 4 + g];
#pragma unroll
    for (int s = 0; s < 4; ++s)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W2f[(u * 4 + s) * 64 + lane], hb[s], acc, 0, 0, 0);
    acc2[u] = acc;
  }
  const bf16x8* W3f = reinterpret_cast<const bf16x8*>(sblob + kOffW3F);
  f32x4 acc3 = zero;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const uint4 u4 = make_uint4(relu_pack_bf16x2(acc2[2 * s][0], acc2[2 * s][1]),
                                relu_pack_bf16x2(acc2[2 * s][2], acc2[2 * s][3]),
                                relu_pack_bf16x2(acc2[2 * s + 1][0], acc2[2 * s + 1][1]),
                                relu_pack_bf16x2(acc2[2 * s + 1][2], acc2[2 * s + 1][3]));
    acc3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W3f[s * 64 + lane], __builtin_bit_cast(bf16x8, u4), acc3, 0, 0, 0);
  }
  (void)w3f;
  return __builtin_amdgcn_rcpf(1.f + __expf(-(acc3[0] + L.b3)));
}

// Two independent tiles per call: every weight fragment read from LDS feeds two MFMAs (half
// the LDS traffic per row) and the two dependency chains interleave (ILP 2 per wave).
__device__ __forceinline__ float mlp_proba_of_logit(float z) { return __builtin_amdgcn_rcpf(1.f + __expf(-z)); }

__device__ __forceinline__ void mlp_logit_w64_x2(const char* sblob, const MlpWireLane& L, const WireRegs& r0,
                                                 const WireRegs& r1, int g, int lane, float& z0, float& z1) {
  const bf16x8 xa = wire_operand(r0, g == 3, L);
  const bf16x8 xb = wire_operand(r1, g == 3, L);
  const bf16x8* W1f = reinterpret_cast<const bf16x8*>(sblob + kOffW1);
  const bf16x8* W2f = reinterpret_cast<const bf16x8*>(sblob + kOffW2);
  const f32x4* b2f = reinterpret_cast<const f32x4*>(sblob + kOffB2);
  const bf16x8* W3f = reinterpret_cast<const bf16x8*>(sblob + kOffW3F);
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  bf16x8 ha[4], hb[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const bf16x8 w0 = W1f[(2 * s) * 64 + lane], w1 = W1f[(2 * s + 1) * 64 + lane];
    const f32x4 a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, xa, zero, 0, 0, 0);
    const f32x4 b0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, xb, zero, 0, 0, 0);
    const f32x4 a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, xa, zero, 0, 0, 0);
    const f32x4 b1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, xb, zero, 0, 0, 0);
    ha[s] = __builtin_bit_cast(bf16x8, make_uint4(relu_pack_bf16x2(a0[0], a0[1]), relu_pack_bf16x2(a0[2], a0[3]),
                                                  relu_pack_bf16x2(a1[0], a1[1]), relu_pack_bf16x2(a1[2], a1[3])));
    hb[s] = __builtin_bit_cast(bf16x8, make_uint4(relu_pack_bf16x2(b0[0], b0[1]), relu_pack_bf16x2(b0[2], b0[3]),
                                                  relu_pack_bf16x2(b1[0], b1[1]), relu_pack_bf16x2(b1[2], b1[3])));
  }
  f32x4 a2[4], b2[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f32x4 aa = b2f[u * 4 + g], bb = aa;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 w = W2f[(u * 4 + s) * 64 + lane];
      aa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, ha[s], aa, 0, 0, 0);
      bb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, hb[s], bb, 0, 0, 0);
    }
    a2[u] = aa;
    b2[u] = bb;
  }
  f32x4 za = zero, zb = zero;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bf16x8 w = W3f[s * 64 + lane];
    const uint4 ua = make_uint4(relu_pack_bf16x2(a2[2 * s][0], a2[2 * s][1]), relu_pack_bf16x2(a2[2 * s][2], a2[2 * s][3]),
                                relu_pack_bf16x2(a2[2 * s + 1][0], a2[2 * s + 1][1]),
                                relu_pack_bf16x2(a2[2 * s + 1][2], a2[2 * s + 1][3]));
    const uint4 ub = make_uint4(relu_pack_bf16x2(b2[2 * s][0], b2[2 * s][1]), relu_pack_bf16x2(b2[2 * s][2], b2[2 * s][3]),
                                relu_pack_bf16x2(b2[2 * s + 1][0], b2[2 * s + 1][1]),
                                relu_pack_bf16x2(b2[2 * s + 1][2], b2[2 * s + 1][3]));
    za = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, __builtin_bit_cast(bf16x8, ua), za, 0, 0, 0);
    zb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, __builtin_bit_cast(bf16x8, ub), zb, 0, 0, 0);
  }
  z0 = za[0] + L.b3;
  z1 = zb[0] + L.b3;
}

__device__ __forceinline__ void mlp_tile_w64_x2(const char* sblob, const MlpWireLane& L, const WireRegs& r0,
                                                const WireRegs& r1, int g, int lane, float& p0, float& p1) {
  float z0, z1;
  mlp_logit_w64_x2(sblob, L, r0, r1, g, lane, z0, z1);
  p0 = mlp_proba_of_logit(z0);
  p1 = mlp_proba_of_logit(z1);
}

// wire_body.h scorer for the MLP
struct MlpWireScorer {
  static constexpr int kLds = kMlpBlobWire;
  MlpWireLane L;
  __device__ __forceinline__ void stage(const ccfd_score_args& a, char* lds, int tid, int nthreads) {
    mlp_stage(a.blob, lds, tid, nthreads, kMlpBlobWire);
  }
  __device__ __forceinline__ void lanes(const char* lds, const ccfd_score_args&, int) { L = mlp_wire_lane(lds); }
  __device__ __forceinline__ float tile(const char* lds, const WireRegs& r, int g, int lane) const {
    return mlp_tile_w64(lds, L, r, g, lane);
  }
  static constexpr bool kPair = true;
  static constexpr bool kQuad = true;
  __device__ __forceinline__ void tile2(const char* lds, const WireRegs& r0, const WireRegs& r1, int g, int lane,
                                        float& p0, float& p1) const {
    mlp_tile_w64_x2(lds, L, r0, r1, g, lane, p0, p1);
  }
  __device__ __forceinline__ void logit2(const char* lds, const WireRegs& r0, const WireRegs& r1, int g, int lane,
                                         float& z0, float& z1) const {
    mlp_logit_w64_x2(lds, L, r0, r1, g, lane, z0, z1);
  }
  __device__ __forceinline__ float proba(float z) const { return mlp_proba_of_logit(z); }
};

// Same math with every weight fragment held in VGPRs for the kernel's lifetime (26 bf16x8
// A-fragments + the lane group's 4 b2 quads = 120 VGPRs): no LDS read or lgkmcnt wait on the
// MFMA chain.  Needs the 256-VGPR budget of 2 waves/SIMD (score_mlp_wire_reg_kernel).
struct MlpWireRegScorer {
  static constexpr int kLds = kMlpBlobWire;
  MlpWireLane L;
  bf16x8 w1[8], w2[16], w3[2];
  f32x4 b2[4];
  __device__ __forceinline__ void stage(const ccfd_score_args& a, char* lds, int tid, int nthreads) {
    mlp_stage(a.blob, lds, tid, nthreads, kMlpBlobWire);
  }
  __device__ __forceinline__ void lanes(const char* lds, const ccfd_score_args&, int g) {
    L = mlp_wire_lane(lds);
    const int lane = threadIdx.x & 63;
    const bf16x8* W1f = reinterpret_cast<const bf16x8*>(lds + kOffW1);
    const bf16x8* W2f = reinterpret_cast<const bf16x8*>(lds + kOffW2);
    const bf16x8* W3f = reinterpret_cast<const bf16x8*>(lds + kOffW3F);
    const f32x4* b2f = reinterpret_cast<const f32x4*>(lds + kOffB2);
#pragma unroll
    for (int t = 0; t < 8; ++t) w1[t] = W1f[t * 64 + lane];
#pragma unroll
    for (int t = 0; t < 16; ++t) w2[t] = W2f[t * 64 + lane];
#pragma unroll
    for (int t = 0; t < 2; ++t) w3[t] = W3f[t * 64 + lane];
#pragma unroll
    for (int u = 0; u < 4; ++u) b2[u] = b2f[u * 4 + g];
  }
  __device__ __forceinline__ void logit2(const char*, const WireRegs& r0, const WireRegs& r1, int g, int,
                                         float& z0, float& z1) const {
    const bf16x8 xa = wire_operand(r0, g == 3, L);
    const bf16x8 xb = wire_operand(r1, g == 3, L);
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    bf16x8 ha[4], hb[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const f32x4 a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[2 * s], xa, zero, 0, 0, 0);
      const f32x4 b0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[2 * s], xb, zero, 0, 0, 0);
      const f32x4 a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[2 * s + 1], xa, zero, 0, 0, 0);
      const f32x4 b1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[2 * s + 1], xb, zero, 0, 0, 0);
      ha[s] = __builtin_bit_cast(bf16x8, make_uint4(relu_pack_bf16x2(a0[0], a0[1]), relu_pack_bf16x2(a0[2], a0[3]),
                                                    relu_pack_bf16x2(a1[0], a1[1]), relu_pack_bf16x2(a1[2], a1[3])));
      hb[s] = __builtin_bit_cast(bf16x8, make_uint4(relu_pack_bf16x2(b0[0], b0[1]), relu_pack_bf16x2(b0[2], b0[3]),
                                                    relu_pack_bf16x2(b1[0], b1[1]), relu_pack_bf16x2(b1[2], b1[3])));
    }
    f32x4 a2[4], b2v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x4 aa = b2[u], bb = b2[u];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        aa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2[u * 4 + s], ha[s], aa, 0, 0, 0);
        bb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2[u * 4 + s], hb[s], bb, 0, 0, 0);
      }
      a2[u] = aa;
      b2v[u] = bb;
    }
    f32x4 za = zero, zb = zero;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint4 ua = make_uint4(relu_pack_bf16x2(a2[2 * s][0], a2[2 * s][1]), relu_pack_bf16x2(a2[2 * s][2], a2[2 * s][3]),
                                  relu_pack_bf16x2(a2[2 * s + 1][0], a2[2 * s + 1][1]),
                                  relu_pack_bf16x2(a2[2 * s + 1][2], a2[2 * s + 1][3]));
      const uint4 ub = make_uint4(relu_pack_bf16x2(b2v[2 * s][0], b2v[2 * s][1]), relu_pack_bf16x2(b2v[2 * s][2], b2v[2 * s][3]),
                                  relu_pack_bf16x2(b2v[2 * s + 1][0], b2v[2 * s + 1][1]),
                                  relu_pack_bf16x2(b2v[2 * s + 1][2], b2v[2 * s + 1][3]));
      za = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w3[s], __builtin_bit_cast(bf16x8, ua), za, 0, 0, 0);
      zb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w3[s], __builtin_bit_cast(bf16x8, ub), zb, 0, 0, 0);
    }
    z0 = za[0] + L.b3;
    z1 = zb[0] + L.b3;
  }
  __device__ __forceinline__ void tile2(const char* lds, const WireRegs& r0, const WireRegs& r1, int g, int lane,
                                        float& p0, float& p1) const {
    float z0, z1;
    logit2(lds, r0, r1, g, lane, z0, z1);
    p0 = mlp_proba_of_logit(z0);
    p1 = mlp_proba_of_logit(z1);
  }
  __device__ __forceinline__ float proba(float z) const { return mlp_proba_of_logit(z); }
  __device__ __forceinline__ float tile(const char* lds, const WireRegs& r, int g, int lane) const {
    float p0, p1;
    tile2(lds, r, r, g, lane, p0, p1);
    return p0;
  }
  static constexpr bool kPair = true;
  static constexpr bool kQuad = true;
};

}  // namespace ccfd
