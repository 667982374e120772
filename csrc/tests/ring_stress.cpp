// Race/ordering stress test of the engine's SPSC row ring (csrc/engine/spsc_ring.h).
// Built by tests/test_native_cpu.py with -fsanitize=thread (and separately with
// address,undefined): a producer thread writes rows carrying their global sequence number,
// a consumer thread takes variable-size "micro-batches", checks every row it reads, and
// releases them after a random delay (the GPU completing out of the producer's sight).
// Randomised sleeps on both sides shake the interleavings.  Exit code 0 = no lost,
// duplicated, reordered or torn row.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "../engine/spsc_ring.h"

int main(int argc, char** argv) {
  const int64_t total = argc > 1 ? std::atoll(argv[1]) : 2000000;
  const int64_t cap = argc > 2 ? std::atoll(argv[2]) : 4093;   // prime: wraps at odd offsets
  constexpr int kW = 8;                                          // words per row
  std::vector<int64_t> rows(cap * kW);
  ccfd::RowRing ring;
  ring.reset(cap);
  std::atomic<bool> failed{false};

  std::thread producer([&] {
    std::mt19937_64 rng(1);
    int64_t next = 0;
    while (next < total && !failed.load()) {
      int64_t phys = 0;
      const int64_t want = 1 + (int64_t)(rng() % 700);
      const int64_t k = ring.acquire(std::min<int64_t>(want, total - next), &phys);
      if (k == 0) { std::this_thread::yield(); continue; }
      for (int64_t i = 0; i < k; ++i)
        for (int w = 0; w < kW; ++w) rows[(phys + i) * kW + w] = (next + i) * kW + w;
      ring.commit(k);
      next += k;
      if (rng() % 64 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 50));
    }
  });

  std::thread consumer([&] {
    std::mt19937_64 rng(2);
    int64_t expect = 0;
    std::vector<int64_t> inflight;     // batch sizes taken but not yet released
    while (expect < total && !failed.load()) {
      int64_t avail = ring.available();
      if (avail > 0) {
        const int64_t phys = ring.take_pos();
        const int64_t n = std::min<int64_t>({avail, 1 + (int64_t)(rng() % 1024), cap - phys});
        for (int64_t i = 0; i < n; ++i)
          for (int w = 0; w < kW; ++w)
            if (rows[(phys + i) * kW + w] != (expect + i) * kW + w) {
              std::fprintf(stderr, "row %lld word %d: got %lld\n", (long long)(expect + i), w,
                           (long long)rows[(phys + i) * kW + w]);
              failed.store(true);
              return;
            }
        ring.take(n);
        expect += n;
        inflight.push_back(n);
      }
      // release completed batches in order, sometimes holding several in flight
      while (!inflight.empty() && (rng() % 3 != 0 || avail <= 0)) {
        ring.release_rows(inflight.front());
        inflight.erase(inflight.begin());
      }
      if (rng() % 128 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 50));
    }
    for (int64_t n : inflight) ring.release_rows(n);
    if (!failed.load() && ring.released_count() != total) failed.store(true);
  });

  producer.join();
  consumer.join();
  if (failed.load()) { std::fprintf(stderr, "ring stress FAILED\n"); return 1; }
  std::printf("ring stress ok: %lld rows through a %lld-row ring\n", (long long)total, (long long)cap);
  return 0;
}
