// Roofline probes for the streaming path: how fast can one MI355X pull bytes from pinned
// host memory (a) with an SDMA H2D copy, (b) with zero-copy kernel loads over PCIe, and
// (c) from HBM.  The scoring engine's ceiling is bytes/transaction (120 B of f32
// features) divided by the best of these, so bench numbers are quoted against them.
#include <hip/hip_runtime.h>

#include <sys/mman.h>

#include <chrono>
#include <cstdlib>
#include <cstring>

#include "../include/ccfd_abi.h"

namespace {

__global__ __launch_bounds__(256) void read_sum_kernel(const float4* __restrict__ src, size_t n4, float* out) {
  float acc = 0.f;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = src[i];
    acc += v.x + v.y + v.z + v.w;
  }
  // keep the loads live; one store per thread that is never read back
  if (acc == 1234.5678f) out[threadIdx.x] = acc;
}

// Workgroup b reads whole `blk`-byte blocks in a scattered order (odd multiplicative hash of
// the block index, a permutation when the block count is a power of two): every workgroup on
// its own page-sized stretch at a time, like the persistent kernel's small items.
__global__ __launch_bounds__(256) void read_blocks_kernel(const char* __restrict__ src, size_t nblk, size_t blk,
                                                          float* out) {
  float acc = 0.f;
  for (size_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const size_t pb = (b * 2654435761ull) & (nblk - 1);
    const float4* p = reinterpret_cast<const float4*>(src + pb * blk);
    for (size_t i = threadIdx.x; i < blk / 16; i += blockDim.x) {
      const float4 v = p[i];
      acc += v.x + v.y + v.z + v.w;
    }
  }
  if (acc == 1234.5678f) out[threadIdx.x] = acc;
}

// Same stream as read_sum_kernel with a `W`-byte load per lane (4: one dword, 8, 16): how
// the wave instruction's width (256 B / 512 B / 1 KB contiguous) sets the zero-copy rate.
template <int W>
__global__ __launch_bounds__(256) void read_sum_width_kernel(const unsigned* __restrict__ src, size_t nw, float* out) {
  constexpr int K = W / 4;
  unsigned acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw / K; i += stride) {
    if constexpr (K == 1) {
      acc += src[i];
    } else if constexpr (K == 2) {
      const uint2 v = reinterpret_cast<const uint2*>(src)[i];
      acc += v.x + v.y;
    } else {
      const uint4 v = reinterpret_cast<const uint4*>(src)[i];
      acc += v.x + v.y + v.z + v.w;
    }
  }
  if (acc == 0x12345678u) out[threadIdx.x] = (float)acc;
}

}  // namespace

// Zero-copy read GB/s of `bytes` of pinned host memory with `width`-byte loads per lane
// (4, 8 or 16), `grid` x 256 threads, `iters` passes (events around the timed passes).
extern "C" double ccfd_bw_probe_width(const void* src_host, size_t bytes, int width, int grid, int iters,
                                      void* dev_scratch) {
  if (!src_host || !dev_scratch || bytes < 16 || grid < 1 || iters < 1 || (width != 4 && width != 8 && width != 16))
    return -1.0;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void*>(src_host), 0) != hipSuccess) return -2.0;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -4.0;
  bool ok = true;
  const size_t nw = bytes / 4;
  auto once = [&]() {
    const unsigned* p = static_cast<const unsigned*>(d);
    float* o = static_cast<float*>(dev_scratch);
    if (width == 4) hipLaunchKernelGGL(read_sum_width_kernel<4>, dim3(grid), dim3(256), 0, s, p, nw, o);
    else if (width == 8) hipLaunchKernelGGL(read_sum_width_kernel<8>, dim3(grid), dim3(256), 0, s, p, nw, o);
    else hipLaunchKernelGGL(read_sum_width_kernel<16>, dim3(grid), dim3(256), 0, s, p, nw, o);
    ok = ok && hipGetLastError() == hipSuccess;
  };
  hipEvent_t e0, e1;
  ok = ok && hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess;
  float ms = 0.f;
  if (ok) {
    once();
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    ok = ok && hipEventRecord(e0, s) == hipSuccess;
    for (int i = 0; i < iters && ok; ++i) once();
    ok = ok && hipEventRecord(e1, s) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
         hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  (void)hipStreamDestroy(s);
  if (!ok) return -4.0;
  return ms > 0 ? (double)(nw / (width / 4)) * width * iters / (ms * 1e-3) / 1e9 : -3.0;
}

// Pinned host memory backed by transparent huge pages where the kernel grants them
// (2 MB-aligned anonymous mapping, MADV_HUGEPAGE, faulted in, then hipHostRegister): fewer
// GPU / IOMMU translations per byte for zero-copy reads.  NULL on failure.
extern "C" void* ccfd_host_alloc_huge(size_t bytes) {
  const size_t align = (size_t)2 << 20;
  bytes = (bytes + align - 1) & ~(align - 1);
  void* p = mmap(nullptr, bytes + align, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return nullptr;
  char* a = reinterpret_cast<char*>(((uintptr_t)p + align - 1) & ~(uintptr_t)(align - 1));
  (void)madvise(a, bytes, MADV_HUGEPAGE);
  std::memset(a, 0, bytes);
  if (hipHostRegister(a, bytes, hipHostRegisterMapped | hipHostRegisterPortable) != hipSuccess) {
    munmap(p, bytes + align);
    return nullptr;
  }
  return a;
}

// Zero-copy read GB/s of `bytes` at `src_host` in `blk`-byte blocks (power-of-two count),
// `grid` workgroups of 256 threads, `iters` passes (host wall clock after one warm pass).
extern "C" double ccfd_bw_probe_blocks(const void* src_host, size_t bytes, size_t blk, int grid, int iters,
                                       void* dev_scratch) {
  if (!src_host || !dev_scratch || blk < 256 || (blk & 15) || grid < 1 || iters < 1) return -1.0;
  size_t nblk = 1;
  while (nblk * 2 * blk <= bytes) nblk *= 2;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void*>(src_host), 0) != hipSuccess) return -2.0;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -4.0;
  bool ok = true;
  auto once = [&]() {
    hipLaunchKernelGGL(read_blocks_kernel, dim3(grid), dim3(256), 0, s, static_cast<const char*>(d), nblk, blk,
                       static_cast<float*>(dev_scratch));
    ok = ok && hipGetLastError() == hipSuccess;
  };
  once();
  ok = ok && hipStreamSynchronize(s) == hipSuccess;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters && ok; ++i) once();
  ok = ok && hipStreamSynchronize(s) == hipSuccess;
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  (void)hipStreamDestroy(s);
  if (!ok) return -4.0;
  return sec > 0 ? (double)(nblk * blk) * iters / sec / 1e9 : -3.0;
}

extern "C" double ccfd_bw_probe(const void* src, size_t bytes, int mode, int iters, void* dev_scratch) {
  // mode 0: hipMemcpyAsync H2D (src pinned host) into dev_scratch (>= bytes)
  // mode 1: zero-copy kernel read of host-mapped src
  // mode 2: kernel read of device memory src
  // returns GB/s, or < 0 on a bad argument (-1), pointer (-2), timing (-3) or HIP error (-4)
  if (!src || !dev_scratch || bytes < 16 || iters < 1 || mode < 0 || mode > 2) return -1.0;
  bool ok = true;
  auto chk = [&](hipError_t e) { ok = ok && e == hipSuccess; };
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -4.0;
  hipEvent_t e0, e1;
  chk(hipEventCreate(&e0));
  chk(hipEventCreate(&e1));
  const float4* p = static_cast<const float4*>(src);
  if (mode == 1) {
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, const_cast<void*>(src), 0) != hipSuccess) ok = false;
    p = static_cast<const float4*>(d);
  }
  const size_t n4 = bytes / 16;
  auto once = [&]() {
    if (mode == 0) {
      chk(hipMemcpyAsync(dev_scratch, src, bytes, hipMemcpyHostToDevice, s));
    } else {
      hipLaunchKernelGGL(read_sum_kernel, dim3(2048), dim3(256), 0, s, p, n4, static_cast<float*>(dev_scratch));
      chk(hipGetLastError());
    }
  };
  float ms = 0.f;
  if (ok) {
    once();
    chk(hipStreamSynchronize(s));
    chk(hipEventRecord(e0, s));
    for (int i = 0; i < iters && ok; ++i) once();
    chk(hipEventRecord(e1, s));
    chk(hipEventSynchronize(e1));
    chk(hipEventElapsedTime(&ms, e0, e1));
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamDestroy(s);
  if (!ok) return -4.0;
  return ms > 0 ? (double)bytes * iters / (ms * 1e-3) / 1e9 : -3.0;
}

// Chunked zero-copy probe: the streaming engine's access pattern -- back-to-back kernels
// each reading one `chunk`-byte micro-batch of host-mapped memory, round-robin over
// `nstreams` streams, with `grid` x `block` threads per kernel.  Returns GB/s over `bytes`
// (walked chunk by chunk, `iters` passes).  Tells how much of the large-kernel zero-copy
// roofline survives at micro-batch granularity.
extern "C" double ccfd_bw_probe_chunked(const void* src_host, size_t bytes, size_t chunk, int grid, int block,
                                        int nstreams, int iters, void* dev_scratch) {
  if (nstreams < 1 || nstreams > 16 || chunk < 16 || grid < 1 || block < 64 || block > 256 || iters < 1 ||
      bytes < chunk)
    return -1.0;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void*>(src_host), 0) != hipSuccess) return -2.0;
  bool ok = true;
  auto chk = [&](hipError_t e) { ok = ok && e == hipSuccess; };
  const char* base = static_cast<const char*>(d);
  hipStream_t ss[16] = {};
  for (int i = 0; i < nstreams; ++i) chk(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
  const size_t nchunks = bytes / chunk;
  auto pass = [&]() {
    for (size_t c = 0; c < nchunks && ok; ++c) {
      hipLaunchKernelGGL(read_sum_kernel, dim3(grid), dim3(block), 0, ss[c % nstreams],
                         reinterpret_cast<const float4*>(base + c * chunk), chunk / 16,
                         static_cast<float*>(dev_scratch));
      chk(hipGetLastError());
    }
  };
  auto sync = [&]() { for (int i = 0; i < nstreams; ++i) chk(hipStreamSynchronize(ss[i])); };
  double sec = 0.0;
  if (ok) {
    pass();
    sync();
    // time on the host: several streams run concurrently, so bracket all of them
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters && ok; ++i) pass();
    sync();
    sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  for (int i = 0; i < nstreams; ++i)
    if (ss[i]) (void)hipStreamDestroy(ss[i]);
  if (!ok) return -4.0;
  return sec > 0 ? (double)(nchunks * chunk) * iters / sec / 1e9 : -3.0;
}

// Mixed feed: can the H2D link carry more than one feeder alone?  A fraction `zc_frac` of
// `bytes` is read by a zero-copy kernel while `n_sdma` streams copy the rest (equal slices)
// with SDMA, all concurrently; returns the aggregate GB/s over host wall time.  (Roofline
// question behind the W64 headline: 55.3 GB/s zero-copy vs 57.2 GB/s SDMA alone.)
extern "C" double ccfd_bw_probe_mix(const void* src_host, size_t bytes, int n_sdma, double zc_frac, int iters,
                                    void* dev_scratch) {
  if (n_sdma < 0 || n_sdma > 8 || zc_frac < 0.0 || zc_frac > 1.0 || iters < 1) return -1.0;
  if (n_sdma == 0 && zc_frac < 1.0) return -1.0;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void*>(src_host), 0) != hipSuccess) return -2.0;
  bool ok = true;
  auto chk = [&](hipError_t e) { ok = ok && e == hipSuccess; };
  const size_t zc = ((size_t)(zc_frac * (double)bytes)) & ~(size_t)4095;
  const size_t rest = bytes - zc;
  hipStream_t ks = nullptr, ss[8] = {};
  chk(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
  for (int i = 0; i < n_sdma; ++i) chk(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
  const char* hsrc = static_cast<const char*>(src_host);
  char* dst = static_cast<char*>(dev_scratch);
  auto pass = [&]() {
    if (zc) {
      hipLaunchKernelGGL(read_sum_kernel, dim3(2048), dim3(256), 0, ks, reinterpret_cast<const float4*>(d), zc / 16,
                         reinterpret_cast<float*>(dst));
      chk(hipGetLastError());
    }
    if (n_sdma > 0 && rest) {
      const size_t slice = (rest / n_sdma) & ~(size_t)4095;
      for (int i = 0; i < n_sdma; ++i) {
        const size_t off = zc + (size_t)i * slice;
        const size_t len = i + 1 == n_sdma ? bytes - off : slice;
        chk(hipMemcpyAsync(dst + off, hsrc + off, len, hipMemcpyHostToDevice, ss[i]));
      }
    }
  };
  auto sync = [&]() {
    chk(hipStreamSynchronize(ks));
    for (int i = 0; i < n_sdma; ++i) chk(hipStreamSynchronize(ss[i]));
  };
  double s = 0.0;
  if (ok) {
    pass();
    sync();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters && ok; ++i) pass();
    sync();
    s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  if (ks) (void)hipStreamDestroy(ks);
  for (int i = 0; i < n_sdma; ++i)
    if (ss[i]) (void)hipStreamDestroy(ss[i]);
  if (!ok) return -4.0;
  return s > 0 ? (double)bytes * iters / s / 1e9 : -3.0;
}
