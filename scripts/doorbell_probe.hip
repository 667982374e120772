// Doorbell latency probe: host -> GPU ping-pong, two placements of the doorbell word.
//   host: the word lives in pinned host memory; one GPU wave polls it over PCIe (the
//         persistent kernel's current doorbell, persist_core.h);
//   vram: the word lives in fine-grained device memory (hipDeviceMallocFinegrained) that the
//         CPU writes through the BAR; the wave polls it locally.
// Each round: host stores k to the doorbell, the wave sees k and stores k to a pinned host
// "pong" word (system scope), the host spins until it reads k.  Prints one JSON line per
// placement with the round-trip p50 / p99 in microseconds.  Every wave exits after `rounds`
// pongs or ~2 s without a ping (device clock), so the grid always drains.
//
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/doorbell_probe scripts/doorbell_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void pong_kernel(const unsigned long long* ping, unsigned long long* pong, int rounds) {
  if (threadIdx.x != 0) return;
  unsigned long long last = 0;
  const unsigned long long t_limit = 200000000ull;    // ~2 s of the 100 MHz wall clock
  unsigned long long t0 = wall_clock64();
  for (int r = 0; r < rounds;) {
    const unsigned long long v = __hip_atomic_load(ping, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v != last) {
      last = v;
      __hip_atomic_store(pong, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      ++r;
      t0 = wall_clock64();
    } else if (wall_clock64() - t0 > t_limit) {
      break;                                          // host gone: exit
    }
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int run(const char* name, unsigned long long* ping_host_view, const unsigned long long* ping_dev,
               unsigned long long* pong_host, unsigned long long* pong_dev, int rounds) {
  *ping_host_view = 0;
  *pong_host = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(pong_kernel, dim3(1), dim3(64), 0, s, ping_dev, pong_dev, rounds);
  CK(hipGetLastError());
  std::vector<double> rt;
  rt.reserve(rounds);
  volatile unsigned long long* pong = pong_host;
  volatile unsigned long long* ping = ping_host_view;
  for (int k = 1; k <= rounds; ++k) {
    const double t0 = now_us();
    *ping = (unsigned long long)k;
    while (*pong != (unsigned long long)k) {
      if (now_us() - t0 > 1e6) { std::printf("{\"error\": \"%s: no pong for round %d\"}\n", name, k); goto done; }
    }
    rt.push_back(now_us() - t0);
  }
done:
  CK(hipStreamSynchronize(s));
  CK(hipStreamDestroy(s));
  if (rt.size() > 100) {
    std::sort(rt.begin() + 100, rt.end());                     // drop warm-up rounds
    const size_t n = rt.size() - 100;
    std::printf("{\"doorbell\": \"%s\", \"rounds\": %zu, \"rtt_p50_us\": %.3f, \"rtt_p99_us\": %.3f, \"rtt_min_us\": %.3f}\n",
                name, n, rt[100 + n / 2], rt[100 + (n * 99) / 100], rt[100]);
  }
  return 0;
}

int main() {
  const int rounds = 20000;
  unsigned long long *pong_h = nullptr, *pong_d = nullptr, *ping_h = nullptr, *ping_hd = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pong_h), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&pong_d), pong_h, 0));
  CK(hipHostMalloc(reinterpret_cast<void**>(&ping_h), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ping_hd), ping_h, 0));
  if (run("host", ping_h, ping_hd, pong_h, pong_d, rounds)) return 1;
  // fine-grained VRAM: the same pointer is valid on the host (large BAR) when the runtime
  // maps it; hipPointerGetAttributes says whether it has a host address
  unsigned long long* v = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&v), 4096, hipDeviceMallocFinegrained));
  hipPointerAttribute_t at{};
  CK(hipPointerGetAttributes(&at, v));
  std::printf("{\"vram_alloc\": \"ok\", \"hostPointer\": %s, \"devicePointer\": %s, \"type\": %d}\n",
              at.hostPointer ? "\"set\"" : "null", at.devicePointer ? "\"set\"" : "null", (int)at.type);
  unsigned long long* hv = static_cast<unsigned long long*>(at.hostPointer ? at.hostPointer : nullptr);
  if (!hv) { std::printf("{\"doorbell\": \"vram\", \"skipped\": \"no host mapping\"}\n"); return 0; }
  if (run("vram", hv, v, pong_h, pong_d, rounds)) return 1;
  return 0;
}
