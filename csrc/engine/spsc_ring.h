// Single-producer / single-consumer row ring used by the engine's streaming (ring) mode.
//
// Producer (ingest thread):  acquire() contiguous free rows -> write them -> commit(n)
// Consumer (engine thread):  available() -> take(n) when a micro-batch is submitted ->
//                            release_rows(n) when that micro-batch has COMPLETED
// Rows are only overwritten after release, i.e. after the GPU has finished reading them.
// Header-only and HIP-free so tests/test_native_cpu.py can hammer it under ThreadSanitizer
// (csrc/tests/ring_stress.cpp).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>

namespace ccfd {

class RowRing {
 public:
  void reset(int64_t capacity) {
    cap_ = capacity;
    head_.store(0, std::memory_order_relaxed);
    released_.store(0, std::memory_order_relaxed);
    taken_ = 0;
  }
  int64_t capacity() const { return cap_; }

  // ---- producer side
  // Contiguous free rows (<= want) starting at physical row *row; 0 when full.
  int64_t acquire(int64_t want, int64_t* row) const {
    const int64_t h = head_.load(std::memory_order_relaxed);
    const int64_t free_rows = cap_ - (h - released_.load(std::memory_order_acquire));
    const int64_t phys = h % cap_;
    *row = phys;
    return std::max<int64_t>(0, std::min<int64_t>(std::min<int64_t>(want, free_rows), cap_ - phys));
  }
  int64_t head_count() const { return head_.load(std::memory_order_relaxed); }
  void commit(int64_t n) { head_.store(head_.load(std::memory_order_relaxed) + n, std::memory_order_release); }

  // ---- consumer side
  int64_t available() const { return head_.load(std::memory_order_acquire) - taken_; }
  int64_t taken() const { return taken_; }
  int64_t take_pos() const { return taken_ % cap_; }
  void take(int64_t n) { taken_ += n; }
  void release_rows(int64_t n) {
    released_.store(released_.load(std::memory_order_relaxed) + n, std::memory_order_release);
  }
  int64_t released_count() const { return released_.load(std::memory_order_acquire); }

 private:
  int64_t cap_ = 0;
  std::atomic<int64_t> head_{0};       // rows committed by the producer (monotonic)
  std::atomic<int64_t> released_{0};   // rows released by the consumer (monotonic)
  int64_t taken_ = 0;                  // rows handed to the GPU (consumer-private)
};

}  // namespace ccfd
