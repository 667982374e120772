// Host-DRAM read-bandwidth probe (CPU side).
//
// The zero-copy scoring path streams every row from pinned host memory over PCIe: at N GPUs
// a socket's DRAM serves the reads of every rank placed on it (8 ranks x ~55 GB/s = 440 GB/s
// on a 2-socket node, ~220 GB/s a socket).  The per-rank GPU probe (probe.hip) cannot see
// that ceiling from one GPU; this one measures what the socket's memory controllers deliver
// to streaming reads, with `threads` CPU threads inheriting the caller's affinity (bench.py
// binds each rank to its GPU's NUMA node first), over a pinned buffer the caller allocated on
// that node.  Non-temporal-style wide loads, reduced so the compiler cannot elide them.
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <thread>
#include <vector>

namespace {

__attribute__((target("avx2"))) uint64_t sweep(const uint8_t* p, size_t n) {
  __m256i acc0 = _mm256_setzero_si256(), acc1 = _mm256_setzero_si256();
  __m256i acc2 = _mm256_setzero_si256(), acc3 = _mm256_setzero_si256();
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    acc0 = _mm256_xor_si256(acc0, _mm256_load_si256(reinterpret_cast<const __m256i*>(p + i)));
    acc1 = _mm256_xor_si256(acc1, _mm256_load_si256(reinterpret_cast<const __m256i*>(p + i + 32)));
    acc2 = _mm256_xor_si256(acc2, _mm256_load_si256(reinterpret_cast<const __m256i*>(p + i + 64)));
    acc3 = _mm256_xor_si256(acc3, _mm256_load_si256(reinterpret_cast<const __m256i*>(p + i + 96)));
  }
  __m256i a = _mm256_xor_si256(_mm256_xor_si256(acc0, acc1), _mm256_xor_si256(acc2, acc3));
  alignas(32) uint64_t w[4];
  _mm256_store_si256(reinterpret_cast<__m256i*>(w), a);
  uint64_t r = w[0] ^ w[1] ^ w[2] ^ w[3];
  for (; i < n; ++i) r += p[i];
  return r;
}

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// GB/s of streaming reads of [buf, buf + bytes) by `threads` threads for ~`seconds`
// (each thread sweeps its own 128-byte-aligned slice; whole passes only).  buf must be
// 32-byte aligned.  Returns < 0 on bad arguments.
extern "C" double ccfd_host_read_bw(const void* buf, size_t bytes, int threads, double seconds) {
  if (!buf || bytes < (1u << 20) || threads < 1 || threads > 256 ||
      (reinterpret_cast<uintptr_t>(buf) & 31))
    return -1.0;
  const auto* base = static_cast<const uint8_t*>(buf);
  const size_t slice = (bytes / (size_t)threads) & ~(size_t)127;
  if (slice < 4096) return -1.0;
  std::atomic<bool> go{false}, stop{false};
  std::atomic<uint64_t> sink{0};
  std::vector<uint64_t> done((size_t)threads, 0);
  std::vector<std::thread> th;
  th.reserve((size_t)threads);
  for (int t = 0; t < threads; ++t) {
    th.emplace_back([&, t] {
      const uint8_t* p = base + (size_t)t * slice;
      uint64_t s = 0, passes = 0;
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      do {
        s += sweep(p, slice);
        ++passes;
      } while (!stop.load(std::memory_order_relaxed));
      done[(size_t)t] = passes;
      sink.fetch_add(s, std::memory_order_relaxed);
    });
  }
  const double t0 = now_s();
  go.store(true, std::memory_order_release);
  std::this_thread::sleep_for(std::chrono::duration<double>(std::max(0.01, seconds)));
  stop.store(true, std::memory_order_relaxed);
  for (auto& x : th) x.join();
  const double dt = now_s() - t0;
  uint64_t passes = 0;
  for (uint64_t d : done) passes += d;
  (void)sink.load();
  return dt > 0 ? (double)passes * (double)slice / dt / 1e9 : -1.0;
}
