// Shared device code of the G32 oblivious-GBDT kernels (score_gbdt_g32.hip: one launch per
// micro-batch; score_gbdt_g32_persist.hip: the persistent variant).  Two translation units
// so the many (depth x rules x leaf-placement) instantiations compile in parallel.
//
// Oblivious-GBDT scorer over G32 rows (BASELINE.json configs[3]: 100 trees x depth 6,
// batch 65536) -- the exact low-byte wire for tree ensembles.
//
// A tree only ever asks `x_f > thr`.  With the sorted split thresholds of feature f as bin
// edges, bin_f(x) = #{edges_f < x} and `x_f > edges_f[k]` <=> `bin_f(x) > k` for every float
// x (NaN -> bin 0 -> every test false, like the f32 compare).  So the ingest side stores one
// byte per feature (contracts/transaction.py G32: 30 bins, the amount bucket, a bin-table
// stamp) and the kernel compares bytes against per-split bin indices: 32 B per row instead
// of 120, i.e. 3.75x the rows per second through the same PCIe link, with bit-identical
// leaf choices (the leaf sums differ from the f32 kernel only in summation order).
//
// Layout: 256-thread workgroups; each wave owns 64-row chunks (one row per lane, grid-
// stride).  A chunk arrives as two contiguous 1 KB wave loads and is transposed through a
// wave-private LDS tile so that lane l holds row l; the next chunk is in flight while the
// current one is evaluated.  The 30 bins are lifted into 30 VGPRs once per row;
// a tree level is then v_movrel (wave-uniform feature id from an SGPR), v_sub against the
// SGPR bin index and v_alignbit (shift + bit), and the leaf value is gathered from the
// LDS-resident leaf tables.
#pragma once

#include <cstdlib>
#include <cstring>

#include <type_traits>

#include "common.h"
#include "rules.h"

#ifndef CCFD_G32_TREE_BLOCK
#define CCFD_G32_TREE_BLOCK 4
#endif

namespace ccfd {

constexpr int kG32Rows = 64;        // rows per wave chunk (one per lane)
constexpr int kG32Waves = 4;
constexpr int kG32LeafLds = 16384;  // floats: leaf tables up to 64 KB are staged in LDS, larger ones read from L2
constexpr int kG32Tb = CCFD_G32_TREE_BLOCK;   // trees whose split parameters load together

struct G32Row { uint4 lo, hi; };

// One 64-row chunk is 2 KB.  Lane l fetches bytes [16l, 16l+16) and [1024+16l, 1024+16l+16):
// each load instruction is ONE contiguous 1 KB wave request (a row-per-lane load -- 32 B at
// a 32 B lane stride -- splits every instruction over the whole 2 KB and measured 0.6 of the
// zero-copy PCIe rate; the W64 kernels' contiguous tiles reach 0.99).  Bytes past the batch
// are clamped to its last 16 B (never scored; a score() tensor ends exactly there).
__device__ __forceinline__ void g32_fetch(const unsigned char* __restrict__ x, int n, int chunk, int lane,
                                          G32Row& r) {
  const long last = (long)n * CCFD_G32_ROW_BYTES - 16;
  const long b0 = (long)chunk * (kG32Rows * CCFD_G32_ROW_BYTES) + 16 * lane;
  r.lo = ld_g16(x + min(b0, last));
  r.hi = ld_g16(x + min(b0 + 1024, last));
}

// Wave-private LDS transpose: after it, lane l holds row l of the chunk (lo = bytes 0..15,
// hi = bytes 16..31).
__device__ __forceinline__ void g32_rows(uint4* __restrict__ t, int lane, G32Row& r) {
  t[lane] = r.lo;
  t[64 + lane] = r.hi;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  r.lo = t[2 * lane];
  r.hi = t[2 * lane + 1];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__device__ __forceinline__ unsigned g32_byte(const G32Row& r, int j) {   // j compile-time
  const unsigned w = j < 4 ? r.lo.x : j < 8 ? r.lo.y : j < 12 ? r.lo.z : j < 16 ? r.lo.w
                   : j < 20 ? r.hi.x : j < 24 ? r.hi.y : j < 28 ? r.hi.z : r.hi.w;
  return (w >> (8 * (j & 3))) & 0xffu;
}

// G20 rows (ccfd_abi.h: 30 bins of 5 bits, amount bucket at bit 150, 6-bit stamp at bit
// 154) -- 5 dwords a row, a 64-row chunk is 1280 B.  Lane l fetches dwords 64k + l (k < 5):
// every load instruction is one contiguous 256 B wave request, and only 4-byte alignment is
// needed wherever a micro-batch starts in the log.  Dwords past the batch are clamped to
// its last dword (never scored).  The row lands in r.lo.xyzw, r.hi.x.  (Dword lanes are
// the fast form here: zero-copy reads run at 57.5 GB/s with 4-byte lanes vs 55.5 with
// 16-byte lanes, and a 16-byte-lane G20 fetch measured 2.43e9 vs 2.47e9 tx/s --
// profiles/r3/load_width/.)
constexpr int kG20Words = CCFD_G20_ROW_BYTES / 4;

__device__ __forceinline__ void g20_fetch(const unsigned char* __restrict__ x, int n, int chunk, int lane,
                                          G32Row& r) {
  const unsigned* __restrict__ xw = reinterpret_cast<const unsigned*>(x);
  const long last = (long)n * kG20Words - 1;
  const long w0 = (long)chunk * (kG32Rows * kG20Words) + lane;
  r.lo.x = ld_g(xw + min(w0, last));
  r.lo.y = ld_g(xw + min(w0 + 64, last));
  r.lo.z = ld_g(xw + min(w0 + 128, last));
  r.lo.w = ld_g(xw + min(w0 + 192, last));
  r.hi.x = ld_g(xw + min(w0 + 256, last));
}

// Wave-private LDS transpose of a G20 chunk: dword 64k + l is written by lane l, lane l then
// reads its row's dwords 5l .. 5l+4 (stride 5: conflict-free over the 32 banks).
__device__ __forceinline__ void g20_rows(uint4* __restrict__ t4, int lane, G32Row& r) {
  unsigned* t = reinterpret_cast<unsigned*>(t4);
  t[lane] = r.lo.x;
  t[64 + lane] = r.lo.y;
  t[128 + lane] = r.lo.z;
  t[192 + lane] = r.lo.w;
  t[256 + lane] = r.hi.x;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const unsigned* q = t + kG20Words * lane;
  r.lo.x = q[0];
  r.lo.y = q[1];
  r.lo.z = q[2];
  r.lo.w = q[3];
  r.hi.x = q[4];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// Lift a transposed G20 row's 30 five-bit bins (compile-time offsets: one v_bfe, or a
// v_alignbit + v_and where a field straddles two dwords); returns bucket | stamp << 8.
__device__ __forceinline__ unsigned g20_lift(const G32Row& r, unsigned (&b)[kF]) {
  const unsigned w[kG20Words + 1] = {r.lo.x, r.lo.y, r.lo.z, r.lo.w, r.hi.x, 0u};
#pragma unroll
  for (int j = 0; j < kF; ++j) {
    const int bit = 5 * j, wi = bit >> 5, sh = bit & 31;
    b[j] = (sh + 5 <= 32 ? (w[wi] >> sh) : __builtin_amdgcn_alignbit(w[wi + 1], w[wi], sh)) & 31u;
  }
  return ((r.hi.x >> 22) & 0xfu) | ((r.hi.x >> 26) << 8);
}

typedef const __attribute__((address_space(4))) int* g32_cint_p;   // split params -> s_load

// Sum of the T trees' leaves for R row chains whose bins are lifted into b0 (/ b1).  Per
// level: the row's bin (v_movrel with the wave-uniform feature id), then
//   idx = (idx << 1) | (k - bin < 0)   ==   v_sub_u32 + v_alignbit_b32(idx, k - bin, 31)
// (bins and k are <= 255, so the sign bit of k - bin is exactly `bin > k`).  Plain C with
// no VCC / inline asm: the compiler interleaves the independent chains of the trees of a
// block, where a v_cmp + v_addc chain serialises every level on VCC.  Split parameters of
// kG32Tb trees are loaded per batch of scalar loads: one s_waitcnt per block.
template <int D, int R>
__device__ __forceinline__ void g32_trees(const unsigned (&b0)[kF], const unsigned (&b1)[kF],
                                          const float* __restrict__ lv, g32_cint_p feat, g32_cint_p kbin, int T,
                                          float (&acc)[R]) {
  constexpr int L = 1 << D;
#pragma unroll
  for (int q = 0; q < R; ++q) acc[q] = 0.f;
  auto tree = [&](int t, const int* fs, const int* ks) __attribute__((always_inline)) {
    unsigned i0 = 0, i1 = 0;
#pragma unroll
    for (int d = D - 1; d >= 0; --d) {                       // MSB first: bit d lands at position d
      const int f = fs[d];
      const unsigned k = (unsigned)ks[d];
      i0 = __builtin_amdgcn_alignbit(i0, k - b0[f], 31);
      if constexpr (R == 2) i1 = __builtin_amdgcn_alignbit(i1, k - b1[f], 31);
    }
    acc[0] += lv[t * L + (int)i0];
    if constexpr (R == 2) acc[R - 1] += lv[t * L + (int)i1];
  };
  int t = 0;
  for (; t + kG32Tb <= T; t += kG32Tb) {
    int fb[kG32Tb * D], kb[kG32Tb * D];
#pragma unroll
    for (int j = 0; j < kG32Tb * D; ++j) { fb[j] = feat[t * D + j]; kb[j] = kbin[t * D + j]; }
#pragma unroll
    for (int k = 0; k < kG32Tb; ++k) tree(t + k, fb + k * D, kb + k * D);
  }
  for (; t < T; ++t) {
    int fb[D], kb[D];
#pragma unroll
    for (int j = 0; j < D; ++j) { fb[j] = feat[t * D + j]; kb[j] = kbin[t * D + j]; }
    tree(t, fb, kb);
  }
}

// Lift a transposed row's 30 bins into registers; returns bytes 30..31 (bucket | stamp << 8).
__device__ __forceinline__ unsigned g32_lift(const G32Row& r, unsigned (&b)[kF]) {
#pragma unroll
  for (int j = 0; j < kF; ++j) b[j] = g32_byte(r, j);
  return r.hi.w >> 16;
}

// Row-format policy of the binned-row kernels: G32 (u8 bins) or G20 (5-bit bins).
template <bool kG20>
__device__ __forceinline__ void gx_fetch(const unsigned char* __restrict__ x, int n, int chunk, int lane, G32Row& r) {
  if constexpr (kG20) g20_fetch(x, n, chunk, lane, r);
  else g32_fetch(x, n, chunk, lane, r);
}
template <bool kG20>
__device__ __forceinline__ void gx_rows(uint4* __restrict__ t, int lane, G32Row& r) {
  if constexpr (kG20) g20_rows(t, lane, r);
  else g32_rows(t, lane, r);
}
template <bool kG20>
__device__ __forceinline__ unsigned gx_lift(const G32Row& r, unsigned (&b)[kF]) {
  if constexpr (kG20) return g20_lift(r, b);
  else return g32_lift(r, b);
}

// Stage the T * 2^D leaf table (blob section after feat / kbin) into LDS.
template <int D>
__device__ __forceinline__ void g32_stage_leaves(const char* blob, int T, float* lv, int tid, int nthreads) {
  constexpr int L = 1 << D;
  const int tdw = ((4 * T * D + 15) & ~15) / 4;
  const float* src = reinterpret_cast<const float*>(blob + kHeader + 8 * tdw);
  const float4* s4 = reinterpret_cast<const float4*>(src);
  float4* d4 = reinterpret_cast<float4*>(lv);
  const int nl = T * L;
  for (int i = tid; i < nl / 4; i += nthreads) d4[i] = s4[i];
  for (int i = (nl & ~3) + tid; i < nl; i += nthreads) lv[i] = src[i];
}

// Leaf tables of T * 2^D floats up to kG32LeafLds are staged in LDS; larger ensembles
// (kGL: e.g. CatBoost's default 1000 x depth 6 = 250 KB) gather their leaves straight from
// the blob in global memory -- read-only and L2-resident, one gather per tree and row chain.
__device__ __forceinline__ const float* g32_leaves_global(const char* blob, int T, int D) {
  const int tdw = ((4 * T * D + 15) & ~15) / 4;
  return reinterpret_cast<const float*>(blob + kHeader + 8 * tdw);
}

// read per launch, so in-process sweeps can vary it
inline int g32_env(const char* name, int dflt, int lo, int hi) {
  const char* e = getenv(name);
  if (!e) return dflt;
  const int v = atoi(e);
  return v < lo || v > hi ? dflt : v;
}

}  // namespace ccfd
