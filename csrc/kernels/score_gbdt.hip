// Oblivious-GBDT scorer (BASELINE.json configs[3]: 100 trees x depth 6, batch 65536).
//
// In an oblivious tree every level tests one (feature, threshold) pair, identical for
// every row, so for a wave walking the SAME tree the split parameters are wave-uniform:
// they come from scalar loads into SGPRs, and a row's leaf index is D compares + shifts.
// Layout per 256-thread workgroup:
//   * 64 rows staged FEATURE-MAJOR in LDS (xs[30][64]): lane r reads xs[f][r] with f
//     uniform -> consecutive lanes hit consecutive banks (conflict-free ds_read_b32);
//   * the leaf tables of a chunk of trees staged in LDS (<= 64 KB per chunk; once per
//     workgroup when they fit);
//   * each workgroup walks several 64-row chunks with the next chunk prefetched (below);
//   * the 4 waves split the trees (wave w takes trees w, w+4, ...) over the same 64 rows,
//     so each SIMD has independent leaf-gather chains in flight; partial sums are reduced
//     through LDS, then sigmoid + threshold + counters as in the other scorers.
#include <cstdlib>
#include <cstring>

#include "common.h"

namespace ccfd {

constexpr int kGbRows = 64;
constexpr int kGbWaves = 4;
constexpr int kLeafLds = 16384;     // floats of leaf table per chunk (64 KB)
constexpr int kGbF4 = kGbRows * kF / 4;   // 480 float4 per 64-row chunk

// Register-staged copy of one 64-row chunk (contiguous rows): thread t owns float4 t and
// t + 256 of the chunk's 7680 bytes.
struct GbRegs { float4 v[2]; };

__device__ __forceinline__ void gb_issue(const float* __restrict__ x, int row0, int nrows, int tid, GbRegs& r) {
  const int avail = nrows * kF * 4;
  const float4* src = reinterpret_cast<const float4*>(x + (size_t)row0 * kF);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = tid + 256 * k;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < kGbF4) {
      if (i * 16 + 16 <= avail) v = src[i];
      else if (i * 16 + 8 <= avail) { const float2 h = reinterpret_cast<const float2*>(src)[2 * i]; v.x = h.x; v.y = h.y; }
    }
    r.v[k] = v;
  }
}

__device__ __forceinline__ void gb_store(float (*xs)[kGbRows], int tid, const GbRegs& r) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = tid + 256 * k;
    if (i < kGbF4) {
      const int e = 4 * i;
      const float vv[4] = {r.v[k].x, r.v[k].y, r.v[k].z, r.v[k].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) { const int ee = e + q; xs[ee % kF][ee / kF] = vv[q]; }
    }
  }
}

// Each workgroup scores `cpw` consecutive 64-row chunks.  Chunk c+1's rows are fetched into
// registers while chunk c is evaluated, so a workgroup always has host reads in flight, and
// a grid of ~2 workgroups per CU leaves room for the next micro-batch's kernel to start
// fetching before this one drains (one workgroup per chunk filled every CU slot with
// workgroups waiting on PCIe and serialised consecutive batches).  The leaf tables are
// staged into LDS once per workgroup when they fit (T * 2^D <= 16384 floats).
template <int D, bool kContig>
__global__ __launch_bounds__(256) void score_gbdt_kernel(ccfd_score_args a, int cpw) {
  constexpr int L = 1 << D;
  __shared__ __attribute__((aligned(16))) float xs[kF][kGbRows];
  extern __shared__ __attribute__((aligned(16))) float lv[];   // min(T, kLeafLds/L) * L floats
  __shared__ float part[kGbWaves][kGbRows];
  __shared__ EpilogueLds epi;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nchunks = (a.n + kGbRows - 1) / kGbRows;
  const int c_begin = blockIdx.x * cpw;
  const int c_end = min(nchunks, c_begin + cpw);
  epi_init(epi);
  stamp_start(a, blockIdx.x);

  const char* blob = reinterpret_cast<const char*>(a.blob);
  const int T = a.gbdt_trees;
  const float base = *reinterpret_cast<const float*>(blob + 16);
  const int* __restrict__ feat = reinterpret_cast<const int*>(blob + kHeader);
  const int tdw = ((4 * T * D + 15) & ~15) / 4;
  const float* __restrict__ thr = reinterpret_cast<const float*>(blob + kHeader) + tdw;
  const float* __restrict__ leaves = thr + tdw;
  const int kChunk = min(T, kLeafLds / L);
  const bool resident = kChunk == T;

  GbRegs cur, nxt;
  if constexpr (kContig)
    if (c_begin < c_end) gb_issue(a.x, c_begin * kGbRows, min(kGbRows, a.n - c_begin * kGbRows), tid, cur);

  auto stage_leaves = [&](int c0, int c1) {
    const int nl = (c1 - c0) * L;
    if constexpr (L >= 4) {
      const float4* s4 = reinterpret_cast<const float4*>(leaves + (size_t)c0 * L);
      float4* d4 = reinterpret_cast<float4*>(lv);
      for (int i = tid; i < nl / 4; i += 256) d4[i] = s4[i];
    } else {
      for (int i = tid; i < nl; i += 256) lv[i] = leaves[(size_t)c0 * L + i];
    }
  };
  if (resident) stage_leaves(0, T);    // made visible by the first loop barrier

  for (int c = c_begin; c < c_end; ++c) {
    const int row0 = c * kGbRows;
    const int nrows = min(kGbRows, a.n - row0);
    __syncthreads();   // previous chunk's xs / part readers are done
    if constexpr (kContig) {
      if (c + 1 < c_end) gb_issue(a.x, row0 + kGbRows, min(kGbRows, a.n - row0 - kGbRows), tid, nxt);
      gb_store(xs, tid, cur);
    } else {
      for (int e = tid; e < kGbRows * kF; e += 256) {
        const int r = e / kF, f = e % kF;
        xs[f][r] = (r < nrows) ? a.x[(size_t)(row0 + r) * a.ld + f] : 0.f;
      }
    }

    float acc = 0.f;
    for (int c0 = 0; c0 < T; c0 += kChunk) {
      const int c1 = min(T, c0 + kChunk);
      if (!resident) {
        __syncthreads();   // previous tree chunk consumed
        stage_leaves(c0, c1);
      }
      __syncthreads();     // rows (and leaves) staged
      for (int t = c0 + wave; t < c1; t += kGbWaves) {
        int idx = 0;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const int f = feat[t * D + d];          // wave-uniform -> s_load
          const float th = thr[t * D + d];
          idx |= (xs[f][lane] > th ? 1 : 0) << d;
        }
        acc += lv[(t - c0) * L + idx];
      }
    }
    part[wave][lane] = acc;
    __syncthreads();

    if (wave == 0) {
      const float z = base + part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
      const float p = sigmoid(z);
      const bool valid = lane < nrows;
      const bool fr = valid && (p >= a.threshold);
      const int row = row0 + lane;
      if (valid) {
        if (a.proba) a.proba[row] = p;
        if (a.route) a.route[row] = fr ? 1 : 0;
        atomicAdd(&epi.hist[(fr ? kNB : 0) + amount_bucket(xs[kAmountCol][lane])], 1u);
      }
      unsigned long long ps = valid ? (unsigned long long)(p * 1e6f + 0.5f) : 0ull;
      ps = wave_sum_u64(ps);
      const unsigned nf = __popcll(__ballot(fr));
      if (lane == 0) { epi.fraud += nf; epi.rows += nrows; epi.psum_e6 += ps; }
      emit_flagged(a, fr, row);
    }
    if constexpr (kContig) cur = nxt;
  }
  epi_flush(epi, a.counters);
  signal_done(a, gridDim.x);
}

// CCFD_GBDT_CPW: 64-row chunks per workgroup.  Default: a ~256-workgroup grid (one per CU;
// 4 chunks each on a 65536-row micro-batch).  Measured on MI355X, 100x6 trees, 65536-row
// batches (profiles/r1/gbdt_sweep.txt): 1 chunk/WG 348M tx/s, 2 -> 368M, 4 -> 412M,
// 8 -> 408M, 16 -> 395M.
static int gbdt_chunks_per_wg(int nchunks) {
  static const int env = [] {
    const char* e = getenv("CCFD_GBDT_CPW");
    return e ? atoi(e) : 0;
  }();
  if (env > 0) return env;
  const int target_wgs = 256;
  return max(1, (nchunks + target_wgs - 1) / target_wgs);
}

template <int D>
static void launch_d(const ccfd_score_args& a, hipStream_t s, bool contig) {
  constexpr int L = 1 << D;
  const int nchunks = (a.n + kGbRows - 1) / kGbRows;
  const int cpw = gbdt_chunks_per_wg(nchunks);
  const int grid = (nchunks + cpw - 1) / cpw;
  const size_t lds = (size_t)min(a.gbdt_trees, kLeafLds / L) * L * sizeof(float);
  if (contig)
    hipLaunchKernelGGL((score_gbdt_kernel<D, true>), dim3(grid), dim3(256), lds, s, a, cpw);
  else
    hipLaunchKernelGGL((score_gbdt_kernel<D, false>), dim3(grid), dim3(256), lds, s, a, cpw);
}

int launch_gbdt(const ccfd_score_args& a, hipStream_t s) {
  const bool contig = a.ld == kF && (reinterpret_cast<uintptr_t>(a.x) & 15) == 0;
  if (a.gbdt_trees <= 0) return -2;
  if (a.n <= 0) return 0;
  switch (a.gbdt_depth) {
    case 1: launch_d<1>(a, s, contig); break;
    case 2: launch_d<2>(a, s, contig); break;
    case 3: launch_d<3>(a, s, contig); break;
    case 4: launch_d<4>(a, s, contig); break;
    case 5: launch_d<5>(a, s, contig); break;
    case 6: launch_d<6>(a, s, contig); break;
    case 7: launch_d<7>(a, s, contig); break;
    case 8: launch_d<8>(a, s, contig); break;
    default: return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace ccfd
