// Streaming scoring engine: the GPU-resident micro-batcher.
//
// Replaces the reference's per-transaction hot loop (router consumes one Kafka message,
// POSTs it to Seldon, applies Drools, starts a KIE process: SURVEY.md §3.1,
// deploy/router.yaml:45-70) with:
//
//   partition log (pinned host, written by the ingest side)
//     -> micro-batch of B rows (pointer arithmetic, no copy)
//     -> [input_mode=DMA]      hipMemcpyAsync H2D into an HBM staging slot
//        [input_mode=zerocopy] the kernel reads the pinned log over PCIe directly
//     -> ONE fused kernel (normalize + model + sigmoid + threshold + counters + histogram)
//     -> proba/route written straight into pinned host result slots (or D2H copy)
//     -> completion (event) -> flagged transactions pushed to the hand-off ring
//
// `depth` micro-batches are in flight over `n_streams` HIP streams, so the H2D copy of
// batch i+1 overlaps the kernel of batch i and the completion handling of batch i-1.
// Counters accumulate on the device into one of two epoch buffers; flip_epoch() lets a
// side stream all-reduce the closed epoch over RCCL while scoring continues (X2).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include <sys/prctl.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "../include/ccfd_abi.h"
#include "spsc_ring.h"

namespace ccfd {
void set_error(const std::string& e);
#ifdef CCFD_EXP_ITEM_TRACE
int item_trace_dump(const char* path);     // score_gbdt_g32_persist.hip, experiment build only
#endif
}

namespace {

using ccfd::set_error;

// persistent engines alive in this process, per device: hardware queues belong to a device,
// so the GPU_MAX_HW_QUEUES bound is per device, not per process
constexpr int kMaxDevices = 64;
std::atomic<int> g_persist_engines[kMaxDevices];

inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define HIPCHK(expr)                                                          \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) {                                                   \
      set_error(std::string(#expr ": ") + hipGetErrorString(_e));             \
      return -4;                                                              \
    }                                                                         \
  } while (0)

struct Partition {
  const float* feats = nullptr;      // host pointer
  const float* feats_dev = nullptr;  // device-visible alias (zero-copy)
  const uint64_t* ids = nullptr;
  const uint32_t* cust = nullptr;
  const float* amount = nullptr;     // G32 rows: host-side Amount column (flagged records)
  int64_t n = 0;
  int64_t cursor = 0;
  // ring (streaming) mode: SPSC ring of n rows; producer = ingest thread, consumer = run()
  bool ring = false;
  ccfd::RowRing rr;                  // SPSC row ring (csrc/engine/spsc_ring.h)
  std::mutex arr_mu;
  struct Arrival { int64_t head, t, origin; };       // head after commit, commit time, producer send time
  std::deque<Arrival> arrivals;

  Arrival arrival_of(int64_t row) {   // commit (and origin) time of `row`
    std::lock_guard<std::mutex> lk(arr_mu);
    // heads increase monotonically: binary search (a JSON feed commits one entry per message,
    // so tens of thousands of entries are in flight and a linear scan held arr_mu -- and the
    // ingest thread's next commit -- for tens of microseconds)
    auto it = std::upper_bound(arrivals.begin(), arrivals.end(), row,
                               [](int64_t r, const Arrival& a) { return r < a.head; });
    if (it != arrivals.end()) return *it;
    return arrivals.empty() ? Arrival{0, 0, 0} : arrivals.back();
  }
  void forget_before(int64_t row) {
    std::lock_guard<std::mutex> lk(arr_mu);
    while (!arrivals.empty() && arrivals.front().head <= row) arrivals.pop_front();
  }
};

struct Slot {
  bool busy = false;
  int part = 0;
  int64_t start = 0;
  int32_t rows = 0;
  int64_t t_submit = 0;
  int64_t t_arrival = 0;           // ring mode: commit time of the batch's first row
  int64_t t_origin = 0;            // ring mode: producer send time of that row (0 = unknown)
  float* d_x = nullptr;
  float* d_proba = nullptr;
  uint8_t* d_route = nullptr;
  float* h_proba = nullptr;        // pinned host
  uint8_t* h_route = nullptr;
  float* h_proba_dev = nullptr;    // device alias of the pinned host slot
  uint8_t* h_route_dev = nullptr;
  hipEvent_t ev = nullptr;
  // kernel-published completion (flag mode): device ticket counters, compacted flagged
  // row indices and the {seq, #flagged} record the last workgroup stores to host memory
  unsigned int* d_ctl = nullptr;
  unsigned int* h_flag = nullptr;
  unsigned int* h_flag_dev = nullptr;
  volatile unsigned long long* h_done = nullptr;
  unsigned long long* h_done_dev = nullptr;
  unsigned long long expect = 0;
  volatile unsigned long long* done_ptr = nullptr;   // h_done, or the persistent ctl record
  bool use_flag = false;
  int64_t seq_no = 0;
};

inline void cpu_relax() {
#if defined(__x86_64__)
  _mm_pause();
#endif
}

class Engine {
 public:
  ccfd_engine_config cfg{};
  std::vector<hipStream_t> streams;
  std::vector<hipEvent_t> flip_ev;
  std::vector<Slot> slots;
  std::vector<std::unique_ptr<Partition>> parts;
  uint64_t seq = 0;
  int next_part = 0;
  int epoch = 0;
  // flagged hand-off ring (producer: pump thread; consumer: drain, any thread)
  std::vector<ccfd_flagged> ring;
  uint64_t ring_head = 0, ring_tail = 0;
  std::mutex ring_mu;
  uint64_t dropped = 0;              // must stay 0: complete() reserves room first (lossless)
  uint64_t flag_full_events = 0;     // completions deferred because the ring was full
  // opt-in scored-record ring (every row; ccfd_engine_scored_enable), same producer/consumer
  std::vector<ccfd_scored> sring;
  uint64_t s_head = 0, s_tail = 0, s_dropped = 0;
  std::mutex s_mu;
  std::atomic<bool> scored_on{false};
  // per-batch latency: O(1) memory however long the engine runs (a long-lived service
  // scores ~2e5 batches/s): count/sum/max, a 0.25-us linear histogram up to 4 ms for the
  // reported quantiles, and the 4-buckets-per-octave log histogram merged over ranks (X3)
  static constexpr int kFineBuckets = 16384;
  static constexpr double kFineUs = 0.25;
  uint64_t lat_n = 0, lat_over = 0;
  double lat_sum_us = 0.0, lat_max_us = 0.0;
  std::vector<uint64_t> lat_fine = std::vector<uint64_t>(kFineBuckets, 0u);   // u64: never wraps
  uint64_t lat_hist[256] = {};
  uint64_t t_submit_ns = 0, t_wait_ns = 0, t_complete_ns = 0;
  uint64_t dev_batches = 0, dev_exec_ns = 0, dev_hist[256] = {};
  uint64_t lat_hist_rows[256] = {}, dev_hist_rows[256] = {};   // row-weighted (Seldon histograms)
  uint64_t origin_batches = 0, origin_hist[256] = {}, origin_hist_rows[256] = {};   // produce -> scored
  // last completed transaction (model "last request" gauges)
  uint64_t last_seq = 0, last_tx_id = 0;
  float last_proba = 0.f, last_amount = 0.f;
  int32_t last_partition = -1;
  uint8_t last_row[128] = {};
  std::vector<ccfd_batch_trace> trace;     // per-batch stage trace ring (ccfd_engine_trace_enable)
  uint64_t trace_n = 0;                    // entries ever written
  std::mutex trace_mu;                     // the ring may be read from another thread
  std::atomic<bool> trace_on{false};       // fast check on the completion path
  double wall_ns_per_tick = 0.0;   // device wall clock (s_memrealtime) period
  unsigned long long done_counter = 0;

  // Completion stamper (CCFD_COMPLETION_THREAD, default on): a host thread that watches the
  // kernel-published completion records of the in-flight micro-batches and stamps the host
  // time each one lands, so a batch's latency ends when its results are in host memory, not
  // when the pump thread next looks (between pump() calls the caller runs the router
  // hand-off and the X2 tick: without the stamper those milliseconds were charged to every
  // batch that completed meanwhile -- the p99 tail).  One packed word per slot: the low 16
  // bits of the awaited sequence number << 48 | ns since the engine started (48 bits), so a
  // stamp can never be attributed to another use of the slot.
  bool stamper_on = false;
  int64_t stamp_base_ns = 0;
  std::unique_ptr<std::atomic<unsigned long long>[]> st_armed;            // awaited seq (0 = idle)
  std::unique_ptr<std::atomic<const volatile unsigned long long*>[]> st_ptr;
  std::unique_ptr<std::atomic<uint64_t>[]> st_word;                       // tag << 48 | t
  std::thread stamper;
  std::atomic<bool> stamper_stop{false};

  static constexpr uint64_t kStampMask = (1ull << 48) - 1;

  void stamper_loop() {
    prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
    const int D = (int)slots.size();
    while (!stamper_stop.load(std::memory_order_relaxed)) {
      bool any = false;
      for (int i = 0; i < D; ++i) {
        const unsigned long long e = st_armed[i].load(std::memory_order_acquire);
        if (!e) continue;
        any = true;
        const uint64_t tag = (uint64_t)(e & 0xffffull) << 48;
        if ((st_word[i].load(std::memory_order_relaxed) & ~kStampMask) == tag) continue;   // stamped
        const volatile unsigned long long* p = st_ptr[i].load(std::memory_order_relaxed);
        if (p && p[0] == e) {
          st_word[i].store(tag | ((uint64_t)(now_ns() - stamp_base_ns) & kStampMask), std::memory_order_release);
          stamps_written.fetch_add(1, std::memory_order_relaxed);
        }
      }
      stamper_iters.fetch_add(1, std::memory_order_relaxed);
      if (any) cpu_relax();
      else std::this_thread::sleep_for(std::chrono::microseconds(2));
    }
  }

  // after s.done_ptr / s.expect are set for a kernel-published completion
  void arm(Slot& s) {
    if (!stamper_on) return;
    const size_t i = (size_t)(&s - slots.data());
    st_ptr[i].store(s.done_ptr, std::memory_order_relaxed);
    st_armed[i].store(s.expect, std::memory_order_release);
  }

  // host time the completion record of `s` landed (stamper), else `fallback`
  uint64_t stamp_used = 0, stamp_missed = 0, stamp_rejected = 0;   // CCFD_STAMPER_DEBUG report
  std::atomic<uint64_t> stamps_written{0}, stamper_iters{0};

  int64_t landed_ns(Slot& s, int64_t fallback) {
    if (!stamper_on || !s.use_flag) return fallback;
    const size_t i = (size_t)(&s - slots.data());
    const uint64_t w = st_word[i].load(std::memory_order_acquire);
    st_armed[i].store(0, std::memory_order_relaxed);
    if ((w >> 48) != (s.expect & 0xffffull)) { ++stamp_missed; return fallback; }
    const int64_t t = stamp_base_ns + (int64_t)(w & kStampMask);
    if (t <= fallback && t >= s.t_submit) { ++stamp_used; return t; }
    ++stamp_rejected;
    return fallback;
  }

  int init(const ccfd_engine_config& c) {
    cfg = c;
    if (cfg.max_batch <= 0 || cfg.depth <= 0 || cfg.n_streams <= 0) {
      set_error("max_batch, depth and n_streams must be > 0");
      return -1;
    }
    if (cfg.blob == nullptr) { set_error("null model blob"); return -1; }
    if (cfg.wire < 0 || cfg.wire > 3) { set_error("wire must be 0 (f32), 1 (W64), 2 (G32) or 3 (G20)"); return -1; }
    if (cfg.wire == 1 && cfg.model == CCFD_MODEL_GBDT) { set_error("W64 wire rows: MLP and LR only"); return -1; }
    if (cfg.wire >= 2 && cfg.model != CCFD_MODEL_GBDT) { set_error("G32 / G20 rows: GBDT only"); return -1; }
    rowf = cfg.wire == 3 ? CCFD_G20_ROW_BYTES / 4 : cfg.wire == 2 ? CCFD_G32_ROW_BYTES / 4
         : cfg.wire ? CCFD_WIRE_ROW_BYTES / 4 : CCFD_N_FEATURES;
    amount_f = cfg.wire >= 2 ? -1 : cfg.wire ? CCFD_WIRE_ROW_BYTES / 4 - 1 : CCFD_N_FEATURES - 1;
    wire_flag = cfg.wire == 3 ? (CCFD_ARG_WIRE_G32 | CCFD_ARG_WIRE_G20) : cfg.wire == 2 ? CCFD_ARG_WIRE_G32
              : cfg.wire ? CCFD_ARG_WIRE_W64 : 0;
    HIPCHK(hipSetDevice(cfg.device));
    {
      int khz = 0;
      if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, cfg.device) == hipSuccess && khz > 0)
        wall_ns_per_tick = 1e6 / (double)khz;
    }
    streams.resize(cfg.n_streams);
    flip_ev.resize(cfg.n_streams);
    for (int i = 0; i < cfg.n_streams; ++i) {
      HIPCHK(hipStreamCreateWithFlags(&streams[i], hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&flip_ev[i], hipEventDisableTiming));
    }
    slots.resize(cfg.depth);
    const size_t B = (size_t)cfg.max_batch;
    // zero-copy outputs in fine-grained (coherent) pinned memory: kernels stream them over
    // PCIe without parking dirty lines in the XCD L2s (the per-workgroup system-scope release
    // at completion stays: it is what orders the outputs before the completion record across
    // XCDs).  CCFD_COHERENT_OUT=0 allocates non-coherent outputs instead (A/B switch).
    if (const char* e = std::getenv("CCFD_COHERENT_OUT")) coherent_out = std::atoi(e) != 0;
    // HIP_LAUNCH_BLOCKING-style debug mode: synchronise after every launch so a kernel fault
    // is reported against the micro-batch that caused it (SURVEY.md §5 race detection)
    if (const char* e = std::getenv("CCFD_DEBUG_SYNC")) debug_sync = std::atoi(e) != 0;
    if (const char* e = std::getenv("CCFD_SYNC_ZC_ROWS")) sync_zc_rows = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("CCFD_IDLE_FLUSH_US")) idle_flush_ns = (int64_t)std::atoi(e) * 1000;
    sync_zc_rows = std::min(sync_zc_rows, cfg.max_batch);
    const unsigned out_flags = hipHostMallocMapped | hipHostMallocPortable |
                               (coherent_out ? hipHostMallocCoherent : 0u);
    for (auto& s : slots) {
      // HBM staging slot: used by input_mode=DMA and always by score_sync (caller memory
      // may be pageable, which the GPU must never dereference directly)
      HIPCHK(hipMalloc(&s.d_x, B * rowf * sizeof(float)));
      if (cfg.output_mode == 1) {
        HIPCHK(hipMalloc(&s.d_proba, B * sizeof(float)));
        HIPCHK(hipMalloc(&s.d_route, B));
      }
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&s.h_proba), B * sizeof(float), out_flags));
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&s.h_route), B, out_flags));
      HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.h_proba_dev), s.h_proba, 0));
      HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.h_route_dev), s.h_route, 0));
      HIPCHK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
      HIPCHK(hipMalloc(reinterpret_cast<void**>(&s.d_ctl), 4 * sizeof(unsigned int)));
      HIPCHK(hipMemsetAsync(s.d_ctl, 0, 4 * sizeof(unsigned int), streams[0]));
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&s.h_flag), B * sizeof(unsigned int), out_flags));
      HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.h_flag_dev), s.h_flag, 0));
      void* hd = nullptr;
      HIPCHK(hipHostMalloc(&hd, 64, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent));
      std::memset(hd, 0, 64);
      s.h_done = static_cast<volatile unsigned long long*>(hd);
      HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.h_done_dev), hd, 0));
    }
    // never hipDeviceSynchronize here: another engine's persistent kernel may be resident
    HIPCHK(hipStreamSynchronize(streams[0]));
    // one micro-batch must always fit (a batch is handed off whole or not at all)
    ring.resize(std::max({1024, cfg.flag_capacity, cfg.max_batch}));
    stamper_on = true;
    if (const char* e = std::getenv("CCFD_COMPLETION_THREAD")) stamper_on = std::atoi(e) != 0;
    if (stamper_on) {
      const size_t D = slots.size();
      st_armed.reset(new std::atomic<unsigned long long>[D]);
      st_ptr.reset(new std::atomic<const volatile unsigned long long*>[D]);
      st_word.reset(new std::atomic<uint64_t>[D]);
      for (size_t i = 0; i < D; ++i) { st_armed[i] = 0; st_ptr[i] = nullptr; st_word[i] = 0; }
      stamp_base_ns = now_ns();
      stamper = std::thread([this] { stamper_loop(); });
    }
    if (cfg.exec_mode == 1) return persist_init();
    return 0;
  }

  // ------------------------------------------------------------------ persistent mode
  bool persistent = false;
  bool persist_counted = false;            // holds one of the process's persistent-queue slots
  bool coherent_out = true;
  uint64_t launches = 0;        // coalesced launches issued (stream round-robin)
  int rowf = CCFD_N_FEATURES;   // f32 words per log row: 30, 16 for W64, 8 for G32, 5 for G20 rows
  int amount_f = CCFD_N_FEATURES - 1;   // word of Amount in a row (-1: G32, host-side column)
  int wire_flag = 0;            // CCFD_ARG_WIRE_* of the row format
  bool debug_sync = false;
  // score_sync of small pageable batches (the REST front end: 1..~50 rows per call) copies
  // the rows into this pinned, mapped buffer and the kernel reads them zero-copy, instead of
  // a staged pageable hipMemcpy before the launch (CCFD_SYNC_ZC_ROWS, default 512; 0 = off)
  float* sync_stage = nullptr;
  const float* sync_stage_dev = nullptr;
  int sync_zc_rows = 512;
  // run(): a partial batch goes out once its oldest row is idle_flush_ns old if nothing is in
  // flight (CCFD_IDLE_FLUSH_US; < 0 = off: partial batches wait for the flush deadline)
  int64_t idle_flush_ns = 20'000;
  ccfd_persist_ctl* pctl = nullptr;       // host (coherent pinned)
  ccfd_persist_desc* pdesc = nullptr;      // host (coherent pinned)
  ccfd_persist_dev* pdev = nullptr;        // device
  hipStream_t pstream = nullptr;
  bool prunning = false;
  int persist_C = 0;
  int persist_tpw = 1;
  bool persist_pipe = false;
  int64_t completed_upto = 0;              // batches completed in order (seq count)
  std::vector<int64_t> flip_seq;           // seq at each epoch flip

  int persist_init() {
    const bool g32 = cfg.model == CCFD_MODEL_GBDT && cfg.wire >= 2;     // G32 or G20 rows
    if (cfg.model != CCFD_MODEL_MLP && cfg.model != CCFD_MODEL_LR && !g32) {
      set_error("persistent exec_mode supports the MLP and LR models, and GBDT on G32 / G20 rows");
      return -1;
    }
    if (cfg.output_mode != 0 || cfg.depth > CCFD_PERSIST_MAX_RING) {
      set_error("persistent exec_mode needs zero-copy outputs and depth <= 64");
      return -1;
    }
    // take this device's persistent-queue slot before allocating anything, so a refusal
    // leaks nothing (see the stream-priority note below)
    if (cfg.device < 0 || cfg.device >= kMaxDevices) { set_error("device index out of range"); return -1; }
    {
      int max_q = 4;
      if (const char* e = std::getenv("GPU_MAX_HW_QUEUES")) max_q = std::max(1, std::atoi(e));
      if (g_persist_engines[cfg.device].fetch_add(1) >= max_q) {
        g_persist_engines[cfg.device].fetch_sub(1);
        set_error("more persistent engines on one device than GPU_MAX_HW_QUEUES in one process: their "
                  "kernels would share a hardware queue");
        return -1;
      }
      persist_counted = true;
    }
    void* p = nullptr;
    HIPCHK(hipHostMalloc(&p, sizeof(ccfd_persist_ctl), hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent));
    std::memset(p, 0, sizeof(ccfd_persist_ctl));
    pctl = static_cast<ccfd_persist_ctl*>(p);
    HIPCHK(hipHostMalloc(&p, sizeof(ccfd_persist_desc) * cfg.depth,
                         hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent));
    std::memset(p, 0, sizeof(ccfd_persist_desc) * cfg.depth);
    pdesc = static_cast<ccfd_persist_desc*>(p);
    // work-item size: 64 rows (one 16-row tile per wave) by default; CCFD_PERSIST_ITEM_ROWS
    // = 128/256 gives each wave 2/4 tiles with a one-tile prefetch (fewer claims per batch)
    // GBDT on G32 rows: items of 4 waves x 64-row chunks (256 / 512 / 1024 rows, default 512)
    // W64 rows on 64 workgroups, every tile of an item in flight at once (score_persist.hip):
    // MLP 512-row items -- 8.63e8 tx/s at p50 53 us and depth 12 vs 8.56e8 at 72 us for
    // 256-row items on 128 workgroups at depth 16; LR 256-row items (8.47e8 at 56 us; 512:
    // 7.3e8) -- profiles/r2/persist_full_item/
    const bool w64 = (wire_flag & CCFD_ARG_WIRE_W64) != 0;
    // G32 ensembles far beyond BASELINE's 100 x 6 (> 1200 tree levels a row) are VALU-bound:
    // 256-row items on 512 workgroups spread them over more waves (700 x 6 at depth 6:
    // 1.01e9 tx/s vs 7.3e8 with 512-row items on 256, profiles/r2/g32_large_ensembles/)
    const bool big_trees = g32 && cfg.gbdt_trees * cfg.gbdt_depth > 1200;
    int item_rows = big_trees ? 256 : (g32 || (w64 && cfg.model == CCFD_MODEL_MLP)) ? 512 : CCFD_PERSIST_ITEM_ROWS;
    if (const char* e = std::getenv("CCFD_PERSIST_ITEM_ROWS")) {
      const int v = std::atoi(e);
      if (v == 256 || v == 512 || v == 1024 || (!g32 && (v == 64 || v == 128))) item_rows = v;
    }
    persist_tpw = g32 ? item_rows / 256 : item_rows / 64;
    // Pipelined static items (MLP on W64 rows, score_persist.hip persist_pipe_kernel): a
    // micro-batch spread over 32 workgroups / CUs, the next item's rows fetched while the
    // current one is scored -- 19 us unloaded latency vs 29 us for claimed 512-row items,
    // better up to ~4 batches in flight, capped near 6.5e8 tx/s beyond
    // (profiles/r3/latency/).  cfg.persist_items: 2 = pipelined, 1 = claimed, 0 = env
    // CCFD_PERSIST_PIPE (default claimed).  CCFD_PERSIST_ITEM_ROWS = 64 / 128 (default 128).
    persist_pipe = false;
    // GBDT on G32 / G20 rows: the same pipelined static items, 512-row items, leaves in LDS
    // (score_gbdt_g32_persist.hip persist_gbdt_pipe_kernel)
    const bool g32_pipe_ok = g32 && !big_trees && ((long)cfg.gbdt_trees << cfg.gbdt_depth) <= 16384;   // kG32LeafLds
    if ((w64 && cfg.model == CCFD_MODEL_MLP) || g32_pipe_ok) {
      if (cfg.persist_items == 2) persist_pipe = true;
      else if (cfg.persist_items == 0)
        if (const char* e = std::getenv("CCFD_PERSIST_PIPE")) persist_pipe = std::atoi(e) != 0;
    }
    if (persist_pipe && g32) {
      item_rows = 512;
      persist_tpw = 2;
    } else if (persist_pipe) {
      item_rows = 128;
      if (const char* e = std::getenv("CCFD_PERSIST_ITEM_ROWS")) if (std::atoi(e) == 64) item_rows = 64;
      persist_tpw = item_rows / 64;
    }
    const int C = (cfg.max_batch + item_rows - 1) / item_rows;
    ccfd_persist_dev init{};
    for (int i = 0; i < CCFD_PERSIST_MAX_RING; ++i) init.remaining[i] = (unsigned)C;
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&pdev), sizeof(ccfd_persist_dev)));
    HIPCHK(hipMemcpy(pdev, &init, sizeof(init), hipMemcpyHostToDevice));
    // The persistent kernel never ends, and the HIP runtime multiplexes streams onto
    // GPU_MAX_HW_QUEUES hardware queues PER PRIORITY LEVEL: any stream that shares the
    // kernel's queue sits behind it forever (measured: the 4th normal-priority torch stream
    // created after the engine stalled; tests/helpers/queue_probe.py).  The kernel's stream
    // therefore takes the LEAST priority level, which neither torch (0 / -1) nor RCCL use,
    // and at most GPU_MAX_HW_QUEUES persistent engines may exist per process.
    {
      int least = 0, greatest = 0;
      HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIPCHK(hipStreamCreateWithPriority(&pstream, hipStreamNonBlocking, least));
    }
    persist_C = C;
    persistent = true;
    return 0;
  }

  // Launch the persistent kernel (lazily, at the first post after a halt).  Device state is
  // re-based on the host's `posted` count: every posted batch has completed (halt drains).
  int persist_launch() {
    ccfd_persist_dev init{};
    init.work_next = (unsigned long long)pctl->posted * (unsigned long long)persist_C;
    init.posted = pctl->posted;
    init.stop = 0;
    for (int i = 0; i < CCFD_PERSIST_MAX_RING; ++i) init.remaining[i] = (unsigned)persist_C;
    HIPCHK(hipMemcpyAsync(pdev, &init, sizeof(init), hipMemcpyHostToDevice, pstream));
    HIPCHK(hipStreamSynchronize(pstream));
    __atomic_store_n(&pctl->stop, 0ull, __ATOMIC_RELEASE);
    ccfd_persist_args a{};
    void* d = nullptr;
    HIPCHK(hipHostGetDevicePointer(&d, pctl, 0));
    a.ctl = static_cast<ccfd_persist_ctl*>(d);
    HIPCHK(hipHostGetDevicePointer(&d, pdesc, 0));
    a.desc = static_cast<const ccfd_persist_desc*>(d);
    a.dev = pdev;
    a.ring = cfg.depth;
    a.items_per_batch = persist_C;
    a.tiles_per_wave = persist_tpw;
    a.flags = (coherent_out ? CCFD_ARG_FENCE_COHERENT : CCFD_ARG_FENCE_SYS) | wire_flag |
              (persist_pipe ? CCFD_ARG_PIPE_ITEMS : 0);
    a.model = cfg.model;
    a.threshold = cfg.threshold;
    a.rules = cfg.rules;
    a.blob = cfg.blob;
    a.counters[0] = cfg.counters[0];
    a.counters[1] = cfg.counters[1];
    a.gbdt_trees = cfg.gbdt_trees;
    a.gbdt_depth = cfg.gbdt_depth;
    // resident workgroups (+ the doorbell): 128 for GBDT G32 (1.68e9 tx/s vs 1.62e9 at 256 and
    // 1.34e9 at 768, profiles/r2/gbdt_g32_persist_sweep.jsonl) and f32 rows; 64 for W64 rows
    // (their 512-row items keep 32 KB per workgroup in flight)
    // G32 ensembles well beyond BASELINE's 100 x 6 are VALU-bound, not PCIe-bound: two
    // workgroups per CU (see persist_init; 700 x 6: 3.8e8 tx/s at 128, 7.3e8 at 256 and
    // 1.01e9 at 512 with 256-row items, profiles/r2/g32_large_ensembles/)
    // G20 rows carry 1.6x the rows of G32 per PCIe byte, so more resident workgroups keep
    // up: 216 (2.56-2.57e9 tx/s at p50 91 us, depth 4, 512-row items) vs 2.52e9 at 192,
    // 2.53e9 at 240 and 2.45e9 at 249 (profiles/r5/pass_w/; r2: 2.18e9 at 128, g20/sweep.txt)
    const bool big_trees = (wire_flag & CCFD_ARG_WIRE_G32) && cfg.gbdt_trees * cfg.gbdt_depth > 1200;
    const int grid = cfg.persist_grid > 0 ? cfg.persist_grid
                     : persist_pipe ? CCFD_PERSIST_GRID
                     : (wire_flag & CCFD_ARG_WIRE_W64) ? CCFD_PERSIST_GRID_W64
                     : big_trees ? 4 * CCFD_PERSIST_GRID
                     : (wire_flag & CCFD_ARG_WIRE_G20) ? CCFD_PERSIST_GRID_G20 : CCFD_PERSIST_GRID;
    int rc = ccfd_persist_launch(&a, grid, pstream);
    if (rc) { set_error("persistent kernel launch failed"); return rc; }
    prunning = true;
    return 0;
  }

  // Stop the persistent kernel: every posted batch must be complete (callers drain first);
  // all workgroups then wait on an unposted batch, see `stop` and exit.  Bounded wait.
  int persist_halt() {
    if (!prunning) return 0;
    __atomic_store_n(&pctl->stop, 1ull, __ATOMIC_RELEASE);
    const int64_t t0 = now_ns();
    hipError_t q;
    while ((q = hipStreamQuery(pstream)) == hipErrorNotReady) {
      if (now_ns() - t0 > 20ll * 1000000000ll) { set_error("persistent kernel did not stop"); return -6; }
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    prunning = false;
    if (q != hipSuccess) { set_error(std::string("persistent kernel: ") + hipGetErrorString(q)); return -4; }
    return 0;
  }

  void persist_free() {
    if (!persistent) {                       // refused or failed part-way through persist_init
      if (pstream) (void)hipStreamDestroy(pstream);
      if (pdev) (void)hipFree(pdev);
      if (pdesc) (void)hipHostFree(pdesc);
      if (pctl) (void)hipHostFree(pctl);
      pstream = nullptr; pdev = nullptr; pdesc = nullptr; pctl = nullptr;
      if (persist_counted) g_persist_engines[cfg.device].fetch_sub(1);
      persist_counted = false;
      return;
    }
    // a completed batch the host never retired (scored-ring back-pressure, a held hand-off,
    // an exception before the drain) stays busy: wait for it here and mark it retired -- its
    // completion record lives in pctl, which is freed below (the slot loop in ~Engine must
    // not read it afterwards)
    for (auto& s : slots) {
      if (s.busy) wait_done(s);
      if (s.use_flag) { s.busy = false; s.use_flag = false; s.done_ptr = nullptr; }
    }
    persist_halt();
#ifdef CCFD_EXP_ITEM_TRACE
    if (const char* out = std::getenv("CCFD_ITEM_TRACE_OUT")) {   // experiment build only
      static int k = 0;
      const std::string path = std::string(out) + "." + std::to_string(k++);
      ccfd::item_trace_dump(path.c_str());
    }
#endif
    // teardown: nothing useful can be done about a failed release, so results are dropped
    (void)hipStreamDestroy(pstream);
    (void)hipFree(pdev);
    (void)hipHostFree(pdesc);
    (void)hipHostFree(pctl);
    if (persist_counted) g_persist_engines[cfg.device].fetch_sub(1);
    persist_counted = false;
    persistent = false;
  }

  // post micro-batch `s` (already filled: part/start/rows) to the persistent kernel
  void persist_post(Slot& s, const float* x_dev) {
    const uint64_t sq = seq;                       // caller increments seq after submit
    ccfd_persist_desc& d = pdesc[sq % cfg.depth];
    d.x = x_dev;
    d.proba = s.h_proba_dev;
    d.route = s.h_route_dev;
    d.flag_idx = s.h_flag_dev;
    d.n = s.rows;
    d.epoch = epoch & 1;
    d.seq = sq;
    s.expect = sq + 1;
    s.use_flag = true;
    s.done_ptr = reinterpret_cast<volatile unsigned long long*>(pctl->done[sq % cfg.depth]);
    arm(s);
    __atomic_store_n(&pctl->posted, sq + 1, __ATOMIC_RELEASE);
  }

  ~Engine() {
    stamper_stop.store(true);
    if (stamper.joinable()) stamper.join();
    if (std::getenv("CCFD_STAMPER_DEBUG"))
      std::fprintf(stderr, "[engine] completion stamps used %llu missed %llu rejected %llu written %llu iters %llu\n",
                   (unsigned long long)stamp_used, (unsigned long long)stamp_missed,
                   (unsigned long long)stamp_rejected, (unsigned long long)stamps_written.load(),
                   (unsigned long long)stamper_iters.load());
    (void)hipSetDevice(cfg.device);
    persist_free();
    if (sync_stage) (void)hipHostFree(sync_stage);
    for (auto& s : slots) {
      if (s.busy) wait_done(s);
      if (s.d_x) (void)hipFree(s.d_x);
      if (s.d_proba) (void)hipFree(s.d_proba);
      if (s.d_route) (void)hipFree(s.d_route);
      if (s.h_proba) (void)hipHostFree(s.h_proba);
      if (s.h_route) (void)hipHostFree(s.h_route);
      if (s.ev) (void)hipEventDestroy(s.ev);
      if (s.d_ctl) (void)hipFree(s.d_ctl);
      if (s.h_flag) (void)hipHostFree(s.h_flag);
      if (s.h_done) (void)hipHostFree(const_cast<unsigned long long*>(s.h_done));
    }
    for (auto e : flip_ev) if (e) (void)hipEventDestroy(e);
    for (auto st : streams) if (st) (void)hipStreamDestroy(st);
  }

  int set_log(int p, const float* feats, const uint64_t* ids, const uint32_t* cust, int64_t n, int64_t cursor) {
    if (p < 0 || p > 4096) { set_error("bad partition index"); return -1; }
    if (n < cfg.max_batch) { set_error("partition log shorter than one micro-batch"); return -1; }
    if (reinterpret_cast<uintptr_t>(feats) & 15) { set_error("log must be 16-byte aligned"); return -1; }
    { int rc = drain_all(); if (rc) return rc; }
    while ((int)parts.size() <= p) parts.emplace_back(new Partition());
    Partition& P = *parts[p];
    P.ring = false;
    P.feats = feats; P.ids = ids; P.cust = cust; P.n = n; P.cursor = cursor % n;
    P.amount = nullptr;
    P.feats_dev = feats;
    if (cfg.input_mode == 1) {
      void* d = nullptr;
      HIPCHK(hipHostGetDevicePointer(&d, const_cast<float*>(feats), 0));
      P.feats_dev = static_cast<const float*>(d);
    }
    return 0;
  }

  void push_flagged_idx(const Slot& s, uint64_t nf) {
    const Partition& P = *parts[s.part];
    std::lock_guard<std::mutex> lk(ring_mu);
    const uint64_t cap = ring.size();
    for (uint64_t k = 0; k < nf; ++k) emit(P, s, (int)s.h_flag[k], cap);
  }

  void push_flagged(const Slot& s) {
    const Partition& P = *parts[s.part];
    const uint8_t* r = s.h_route;
    const int n = s.rows;
    std::lock_guard<std::mutex> lk(ring_mu);
    const uint64_t cap = ring.size();
    int i = 0;
    for (; i + 8 <= n; i += 8) {
      uint64_t w;
      std::memcpy(&w, r + i, 8);
      if (w == 0) continue;
      for (int k = 0; k < 8; ++k) if (r[i + k]) emit(P, s, i + k, cap);
    }
    for (; i < n; ++i) if (r[i]) emit(P, s, i, cap);
  }

  // free records in the flagged ring (drainers only ever grow it)
  uint64_t flag_room() {
    std::lock_guard<std::mutex> lk(ring_mu);
    return ring.size() - (ring_tail - ring_head);
  }

  // fraud-routed rows of a finished batch: the kernel-published count, or the route bytes
  uint64_t nflag_of(const Slot& s) const {
    if (s.use_flag) return s.done_ptr[1];
    uint64_t nf = 0;
    for (int i = 0; i < s.rows; ++i) nf += s.h_route[i];
    return nf;
  }

  // complete() found the batch's flagged records do not fit: nothing was retired
  static constexpr int kFlagFull = CCFD_ENGINE_FLAG_FULL;

  inline void emit(const Partition& P, const Slot& s, int i, uint64_t cap) {
    // complete() reserved room for the whole batch before calling in; reaching this is a bug
    if (ring_tail - ring_head >= cap) { ++dropped; return; }
    const int64_t row = s.start + i;
    ccfd_flagged& f = ring[ring_tail % cap];
    f.tx_id = P.ids ? P.ids[row] : (uint64_t)row;
    f.customer = P.cust ? P.cust[row] : 0u;
    f.proba = s.h_proba[i];
    f.amount = amount_f >= 0 ? P.feats[row * rowf + amount_f] : (P.amount ? P.amount[row] : __builtin_nanf(""));
    f.partition = (uint32_t)s.part;
    ++ring_tail;
  }

  uint64_t scored_room() {
    std::lock_guard<std::mutex> lk(s_mu);
    return sring.size() - (s_tail - s_head);
  }

  // every row of the completed batch `s` -> the scored ring (route from the kernel's route
  // byte, proba_1 from its output slot; both written by the epilogue before the completion
  // record); rows that do not fit are counted, never overwrite unread records
  void push_scored(const Slot& s) {
    const Partition& P = *parts[s.part];
    std::lock_guard<std::mutex> lk(s_mu);
    const uint64_t cap = sring.size();
    const int n = s.rows;
    const uint64_t room = cap - (s_tail - s_head);
    const int take = (int)std::min<uint64_t>(room, (uint64_t)n);
    s_dropped += (uint64_t)(n - take);
    for (int i = 0; i < take; ++i) {
      const int64_t row = s.start + i;
      ccfd_scored& r = sring[s_tail % cap];
      r.tx_id = P.ids ? P.ids[row] : (uint64_t)row;
      r.customer = P.cust ? P.cust[row] : 0u;
      r.proba = s.h_proba[i];
      r.amount = amount_f >= 0 ? P.feats[row * rowf + amount_f] : (P.amount ? P.amount[row] : __builtin_nanf(""));
      r.partition = (uint16_t)s.part;
      r.route = s.h_route[i] ? 1 : 0;
      r.pad = 0;
      ++s_tail;
    }
  }

  int64_t drain_scored(ccfd_scored* out, int64_t max) {
    std::lock_guard<std::mutex> lk(s_mu);
    const uint64_t cap = sring.size();
    int64_t k = 0;
    while (s_head < s_tail && k < max) out[k++] = sring[s_head++ % cap];
    return k;
  }

  bool is_done(const Slot& s) {
    if (s.use_flag) return s.done_ptr[0] == s.expect;
    return hipEventQuery(s.ev) == hipSuccess;
  }

  int wait_done(Slot& s) {
    if (!s.use_flag) {
      HIPCHK(hipEventSynchronize(s.ev));
      return 0;
    }
    // spin on the pinned completion record; every 64K spins check the device for errors
    // and give up after 60 s so a faulted kernel can never hang the host thread
    const int64_t t0 = now_ns();
    for (uint64_t it = 0; s.done_ptr[0] != s.expect; ++it) {
      cpu_relax();
      if ((it & 0xFFFF) == 0xFFFF) {
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) { set_error(std::string("kernel error: ") + hipGetErrorString(e)); return -4; }
        if (now_ns() - t0 > 60ll * 1000000000ll) { set_error("timeout waiting for micro-batch completion"); return -6; }
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return 0;
  }

  void record_trace(const Slot& s, int64_t t_landed, uint64_t nf) {
    std::lock_guard<std::mutex> lk(trace_mu);
    if (trace.empty()) return;
    ccfd_batch_trace& e = trace[trace_n++ % trace.size()];
    e.seq = s.seq_no;
    e.partition = s.part;
    e.rows = s.rows;
    e.t_arrival = s.t_arrival;
    e.t_submit = s.t_submit;
    e.t_landed = t_landed;
    e.t_complete = now_ns();
    const bool dev = s.use_flag && wall_ns_per_tick > 0 && s.done_ptr[3] > s.done_ptr[2];
    e.dev_start = dev ? (int64_t)((double)s.done_ptr[2] * wall_ns_per_tick) : 0;
    e.dev_end = dev ? (int64_t)((double)s.done_ptr[3] * wall_ns_per_tick) : 0;
    e.flagged = (int32_t)nf;
    e.pad = 0;
  }

  // Retire finished batch `s`.  Lossless hand-off: when the flagged ring lacks room for the
  // batch's fraud-routed rows, nothing is retired (the batch stays busy, its ring rows stay
  // unreleased, so back-pressure reaches ingest) and kFlagFull asks the caller to drain.
  int complete(Slot& s, ccfd_engine_stats* st) {
    const int64_t tw = now_ns();
    { int rc = wait_done(s); if (rc) return rc; }
    const int64_t t = now_ns();
    t_wait_ns += t - tw;
    const uint64_t nf_need = nflag_of(s);
    if (nf_need && flag_room() < nf_need) { ++flag_full_events; return kFlagFull; }
    const int64_t t0 = s.t_arrival ? s.t_arrival : s.t_submit;   // ring: end-to-end from commit
    const int64_t t_landed = landed_ns(s, t);                   // results in host memory
    const double us = (t_landed - t0) * 1e-3;

    ++lat_n;
    lat_sum_us += us;
    lat_max_us = std::max(lat_max_us, us);
    {
      const double fb = us / kFineUs;
      if (fb < kFineBuckets) ++lat_fine[(size_t)fb]; else ++lat_over;
    }
    const double ns = (double)std::max<int64_t>(1, t_landed - t0);
    {
      const int b = std::min(255, (int)std::floor(4.0 * std::log2(ns)));
      lat_hist[b]++;
      lat_hist_rows[b] += (uint64_t)s.rows;
    }
    if (s.t_origin > 0 && t_landed > s.t_origin) {        // producer send -> results in host memory
      const int b = std::min(255, (int)std::floor(4.0 * std::log2((double)(t_landed - s.t_origin))));
      ++origin_batches;
      origin_hist[b]++;
      origin_hist_rows[b] += (uint64_t)s.rows;
    }
    const uint64_t nf = nf_need;
    if (s.use_flag) {
      if (nf) push_flagged_idx(s, nf);
      {                                                // K7: device-clock execution window
        const uint64_t t0d = s.done_ptr[2], t1d = s.done_ptr[3];
        if (t1d > t0d && wall_ns_per_tick > 0) {
          const double dns = (double)(t1d - t0d) * wall_ns_per_tick;
          dev_exec_ns += (uint64_t)dns;
          ++dev_batches;
          const int b = std::min(255, (int)std::floor(4.0 * std::log2(std::max(1.0, dns))));
          dev_hist[b]++;
          dev_hist_rows[b] += (uint64_t)s.rows;
        }
      }
    } else if (nf) {
      push_flagged(s);
    }
    if (scored_on.load(std::memory_order_relaxed)) push_scored(s);
    if (st) { st->batches++; st->rows += s.rows; st->fraud_rows += nf; }
    if (trace_on.load(std::memory_order_relaxed)) record_trace(s, t_landed, nf);
    Partition& P = *parts[s.part];
    if (s.rows > 0 && P.feats) {                     // "last request" record (still unreleased)
      const int64_t row = s.start + s.rows - 1;
      std::memcpy(last_row, P.feats + row * rowf, (size_t)rowf * sizeof(float));
      last_tx_id = P.ids ? P.ids[row] : (uint64_t)row;
      last_proba = s.h_proba[s.rows - 1];
      last_amount = amount_f >= 0 ? P.feats[row * rowf + amount_f] : (P.amount ? P.amount[row] : __builtin_nanf(""));
      last_partition = s.part;
      ++last_seq;
    }
    if (P.ring) {
      // batches of one partition complete in submission order: release in order
      P.rr.release_rows(s.rows);
      P.forget_before(P.rr.released_count());
    }
    s.busy = false;
    s.t_arrival = 0;
    s.t_origin = 0;
    completed_upto = std::max<int64_t>(completed_upto, s.seq_no + 1);
    t_complete_ns += now_ns() - t;
    return 0;
  }

  int drain_all(ccfd_engine_stats* st = nullptr) {
    // complete in submission order
    const int D = (int)slots.size();
    for (int k = 0; k < D; ++k) {
      Slot& s = slots[(seq + k) % D];
      if (s.busy) { int rc = complete(s, st); if (rc) return rc; }   // kFlagFull: drain, call again
    }
    // fully drained: let the persistent kernel exit so the device is idle (and a
    // device-wide synchronize by the caller can never wait on a resident kernel)
    if (persistent) return persist_halt();
    return 0;
  }

  // force_dma: x is pageable, stage it through the slot's device buffer; force_zc: x is a
  // device pointer of mapped host memory the kernel reads directly, whatever the input mode
  int submit(Slot& s, const float* x_dev_or_host, const float* x_host, int rows, hipStream_t stream,
             bool force_dma = false, bool force_zc = false) {
    s.t_submit = now_ns();
    s.seq_no = (int64_t)seq;
    struct Acc { uint64_t& a; int64_t t0; ~Acc() { a += now_ns() - t0; } } acc{t_submit_ns, s.t_submit};
    const float* xk = x_dev_or_host;
    if (persistent) {
      if ((cfg.input_mode == 0 || force_dma) && !force_zc) {
        HIPCHK(hipMemcpy(s.d_x, x_host, (size_t)rows * rowf * sizeof(float), hipMemcpyHostToDevice));
        xk = s.d_x;
      }
      if (!prunning) { int rc = persist_launch(); if (rc) return rc; }
      s.rows = rows;                    // the descriptor's row count (score_sync does not set it)
      persist_post(s, xk);
      s.busy = true;
      return 0;
    }
    if ((cfg.input_mode == 0 || force_dma) && !force_zc) {
      HIPCHK(hipMemcpyAsync(s.d_x, x_host, (size_t)rows * rowf * sizeof(float),
                            hipMemcpyHostToDevice, stream));
      xk = s.d_x;
    }
    ccfd_score_args a{};
    a.x = xk; a.ld = rowf; a.n = rows; a.model = cfg.model; a.blob = cfg.blob;
    a.threshold = cfg.threshold; a.gbdt_trees = cfg.gbdt_trees; a.gbdt_depth = cfg.gbdt_depth;
    a.rules = cfg.rules;
    a.proba = cfg.output_mode == 1 ? s.d_proba : s.h_proba_dev;
    a.route = cfg.output_mode == 1 ? s.d_route : s.h_route_dev;
    a.counters = cfg.counters[epoch & 1];
    s.use_flag = cfg.output_mode == 0;
    if (s.use_flag) {
      s.expect = ++done_counter;
      a.slot_ctl = s.d_ctl;
      a.flag_idx = s.h_flag_dev;
      a.done_rec = s.h_done_dev;
      a.done_seq = s.expect;
      s.done_ptr = s.h_done;
      arm(s);
      a.flags = (coherent_out ? CCFD_ARG_FENCE_COHERENT : CCFD_ARG_FENCE_SYS);
    }
    a.flags |= wire_flag;
    int rc = ccfd_score_launch(&a, stream);
    if (rc) return rc;
    if (debug_sync) HIPCHK(hipStreamSynchronize(stream));   // CCFD_DEBUG_SYNC: fault -> this batch
    if (cfg.output_mode == 1) {
      HIPCHK(hipMemcpyAsync(s.h_proba, s.d_proba, (size_t)rows * sizeof(float), hipMemcpyDeviceToHost, stream));
      HIPCHK(hipMemcpyAsync(s.h_route, s.d_route, (size_t)rows, hipMemcpyDeviceToHost, stream));
    }
    if (!s.use_flag) HIPCHK(hipEventRecord(s.ev, stream));
    s.busy = true;
    return 0;
  }

  // Coalesced launches (launch mode, zero-copy in/out, MLP/LR): K >= 2 ready micro-batches
  // that are contiguous in one partition's log go out as ONE kernel launch; each keeps its
  // own slot, outputs, flag list and kernel-published completion record.
  int coalesce_max() const {
    if (persistent || cfg.input_mode != 1 || cfg.output_mode != 0 ||
        (cfg.model != CCFD_MODEL_MLP && cfg.model != CCFD_MODEL_LR)) return 1;
    return std::max(1, std::min({cfg.coalesce, CCFD_MAX_SUB, (int)slots.size()}));
  }

  int submit_multi(int p, int64_t start, int32_t rows, int K) {
    Partition& P = *parts[p];
    const int D = (int)slots.size();
    const int64_t t = now_ns();
    struct Acc { uint64_t& a; int64_t t0; ~Acc() { a += now_ns() - t0; } } acc{t_submit_ns, t};
    ccfd_multi_args m{};
    ccfd_score_args& a = m.base;
    a.x = P.feats_dev + (size_t)start * rowf;
    a.ld = rowf; a.n = K * rows; a.model = cfg.model; a.blob = cfg.blob;
    a.threshold = cfg.threshold;
    a.rules = cfg.rules;
    a.counters = cfg.counters[epoch & 1];
    a.flags = (coherent_out ? CCFD_ARG_FENCE_COHERENT : CCFD_ARG_FENCE_SYS) | wire_flag;
    m.nsub = K;
    m.sub_rows = rows;
    for (int k = 0; k < K; ++k) {
      Slot& s = slots[(seq + k) % D];
      s.t_submit = t;
      s.seq_no = (int64_t)(seq + k);
      s.part = p; s.start = start + (int64_t)k * rows; s.rows = rows;
      s.use_flag = true;
      s.expect = ++done_counter;
      s.done_ptr = s.h_done;
      arm(s);
      s.busy = true;
      m.sub[k] = ccfd_sub_batch{s.h_proba_dev, s.h_route_dev, s.d_ctl, s.h_flag_dev, s.h_done_dev, s.expect};
    }
    hipStream_t stream = streams[(launches++) % streams.size()];
    const int rc = ccfd_score_launch_multi(&m, stream);
    if (rc == 0 && debug_sync) HIPCHK(hipStreamSynchronize(stream));
    return rc;
  }

  int pump(int64_t n_batches, int32_t batch_rows, bool drain, ccfd_engine_stats* st) {
    HIPCHK(hipSetDevice(cfg.device));
    if (parts.empty()) { set_error("no partition log registered"); return -1; }
    if (batch_rows <= 0 || batch_rows > cfg.max_batch) { set_error("bad batch_rows"); return -1; }
    const int64_t t0 = now_ns();
    const int D = (int)slots.size();
    const int kmax = coalesce_max();
    int64_t b = 0;
    // every exit reports the batches submitted by this call: a kFlagFull return is resumed by
    // the caller (after draining the flagged ring) with n_batches - submitted
    auto finish = [&](int rc) {
      if (st) {
        st->submitted += (uint64_t)b;
        st->wall_s += (now_ns() - t0) * 1e-9;
        st->flagged_dropped = dropped;
        st->flag_full_events = flag_full_events;
        fill_latency(st);
      }
      return rc;
    };
    while (b < n_batches) {
      int p = next_part;
      for (int k = 0; k < (int)parts.size() && (parts[p]->feats == nullptr || parts[p]->ring); ++k)
        p = (p + 1) % parts.size();
      next_part = (p + 1) % (int)parts.size();
      Partition& P = *parts[p];
      if (P.ring || P.feats == nullptr) { set_error("pump() needs a replay log partition"); return -1; }
      if (P.cursor + batch_rows > P.n) P.cursor = 0;
      // coalesce up to kmax consecutive micro-batches of this partition into one launch
      const int K = (int)std::min<int64_t>({(int64_t)kmax, n_batches - b, (P.n - P.cursor) / batch_rows});
      for (int k = 0; k < K; ++k) {
        Slot& s = slots[(seq + k) % D];
        if (s.busy) { int rc = complete(s, st); if (rc) return finish(rc); }
      }
      if (K > 1) {
        int rc = submit_multi(p, P.cursor, batch_rows, K);
        if (rc) return finish(rc);
        P.cursor += (int64_t)K * batch_rows;
        seq += K;
        b += K;
        continue;
      }
      Slot& s = slots[seq % D];
      s.part = p; s.start = P.cursor; s.rows = batch_rows;
      P.cursor += batch_rows;
      const size_t off = (size_t)s.start * rowf;
      hipStream_t stream = streams[seq % streams.size()];
      int rc = submit(s, P.feats_dev + off, P.feats + off, batch_rows, stream);
      if (rc) return finish(rc);
      ++seq;
      ++b;
    }
    return finish(drain ? drain_all(st) : 0);
  }

  // nearest-rank quantile from the fine histogram (bucket midpoint); samples beyond its
  // range report the max
  double fine_quantile(double q) const {
    const uint64_t k = (uint64_t)std::floor(q * (double)(lat_n - 1) + 0.5);
    uint64_t c = 0;
    for (int i = 0; i < kFineBuckets; ++i) {
      c += lat_fine[i];
      if (c > k) return (i + 0.5) * kFineUs;
    }
    return lat_max_us;
  }

  void reset_latency() {
    lat_n = lat_over = 0;
    lat_sum_us = lat_max_us = 0.0;
    std::fill(lat_fine.begin(), lat_fine.end(), 0ull);
    std::memset(lat_hist, 0, sizeof(lat_hist));
    std::memset(lat_hist_rows, 0, sizeof(lat_hist_rows));
    origin_batches = 0;
    std::memset(origin_hist, 0, sizeof(origin_hist));
    std::memset(origin_hist_rows, 0, sizeof(origin_hist_rows));
  }

  void fill_latency(ccfd_engine_stats* st) {
    std::memcpy(st->lat_hist, lat_hist, sizeof(lat_hist));
    st->host_submit_ns = t_submit_ns;
    st->host_wait_ns = t_wait_ns;
    st->host_complete_ns = t_complete_ns;
    st->dev_batches = dev_batches;
    st->dev_exec_ns = dev_exec_ns;
    std::memcpy(st->dev_hist, dev_hist, sizeof(dev_hist));
    std::memcpy(st->lat_hist_rows, lat_hist_rows, sizeof(lat_hist_rows));
    std::memcpy(st->dev_hist_rows, dev_hist_rows, sizeof(dev_hist_rows));
    st->last_seq = last_seq;
    st->last_tx_id = last_tx_id;
    st->last_proba = last_proba;
    st->last_amount = last_amount;
    st->last_partition = last_partition;
    st->last_row_bytes = rowf * (int32_t)sizeof(float);
    std::memcpy(st->last_row, last_row, sizeof(last_row));
    st->origin_batches = origin_batches;
    std::memcpy(st->origin_hist, origin_hist, sizeof(origin_hist));
    std::memcpy(st->origin_hist_rows, origin_hist_rows, sizeof(origin_hist_rows));
    if (lat_n == 0) return;
    st->lat_p50_us = fine_quantile(0.50);
    st->lat_p99_us = fine_quantile(0.99);
    st->lat_max_us = lat_max_us;
    st->lat_mean_us = lat_sum_us / (double)lat_n;
  }

  int score_sync(const float* x, int32_t n, float* proba_out, uint8_t* route_out) {
    HIPCHK(hipSetDevice(cfg.device));
    int rc = drain_all();
    if (rc) return rc;
    const int D = (int)slots.size();
    for (int32_t off = 0; off < n; off += cfg.max_batch) {
      const int rows = std::min<int32_t>(cfg.max_batch, n - off);
      Slot& s = slots[seq % D];
      hipStream_t stream = streams[seq % streams.size()];
      const float* xh = x + (size_t)off * rowf;
      if (rows <= sync_zc_rows) {
        if (!sync_stage) {
          void* p = nullptr;
          HIPCHK(hipHostMalloc(&p, (size_t)sync_zc_rows * rowf * sizeof(float),
                               hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent));
          sync_stage = static_cast<float*>(p);
          void* d = nullptr;
          HIPCHK(hipHostGetDevicePointer(&d, p, 0));
          sync_stage_dev = static_cast<const float*>(d);
        }
        // the previous batch has completed (wait_done below), so the stage is free
        std::memcpy(sync_stage, xh, (size_t)rows * rowf * sizeof(float));
        rc = submit(s, sync_stage_dev, sync_stage, rows, stream, /*force_dma=*/false, /*force_zc=*/true);
      } else {
        rc = submit(s, xh, xh, rows, stream, /*force_dma=*/true);
      }
      if (rc) return rc;
      ++seq;
      rc = wait_done(s);
      if (rc) return rc;
      landed_ns(s, 0);                                 // disarm the stamper
      s.busy = false;
      completed_upto = std::max<int64_t>(completed_upto, s.seq_no + 1);
      if (proba_out) std::memcpy(proba_out + off, s.h_proba, rows * sizeof(float));
      if (route_out) std::memcpy(route_out + off, s.h_route, rows);
    }
    return persistent ? persist_halt() : 0;
  }

  // Model hot swap (X1 at runtime): every in-flight micro-batch completes with the old
  // weights (and a resident persistent kernel halts), then later submissions read `blob`.
  // The caller keeps the old blob alive until this returns.
  int set_blob(const void* blob) {
    if (blob == nullptr) { set_error("null model blob"); return -1; }
    HIPCHK(hipSetDevice(cfg.device));
    int rc = drain_all();
    if (rc) return rc;
    if (persistent && prunning) { rc = persist_halt(); if (rc) return rc; }
    cfg.blob = blob;
    return 0;
  }

  int flip_epoch(void* side_stream) {
    HIPCHK(hipSetDevice(cfg.device));
    const int closed = epoch & 1;
    if (!persistent) {
      for (size_t i = 0; i < streams.size(); ++i) {
        HIPCHK(hipEventRecord(flip_ev[i], streams[i]));
        if (side_stream) HIPCHK(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(side_stream), flip_ev[i], 0));
      }
    }
    flip_seq.push_back((int64_t)seq);
    ++epoch;
    return closed;
  }

  int epoch_complete(int64_t flip_count) {
    if (flip_count <= 0 || flip_count > (int64_t)flip_seq.size()) return -1;
    return completed_upto >= flip_seq[flip_count - 1] ? 1 : 0;
  }

  // ------------------------------------------------------------------ ring (streaming) mode
  int set_ring(int p, float* feats, uint64_t* ids, uint32_t* cust, int64_t cap) {
    if (p < 0 || p > 4096 || cap < cfg.max_batch) { set_error("bad ring partition/capacity"); return -1; }
    if (reinterpret_cast<uintptr_t>(feats) & 15) { set_error("ring must be 16-byte aligned"); return -1; }
    int rc = drain_all();
    if (rc) return rc;
    while ((int)parts.size() <= p) parts.emplace_back(new Partition());
    Partition& P = *parts[p];
    P.ring = true;
    P.feats = feats; P.ids = ids; P.cust = cust; P.n = cap; P.cursor = 0;
    P.amount = nullptr;
    P.rr.reset(cap);
    P.feats_dev = feats;
    if (cfg.input_mode == 1) {
      void* d = nullptr;
      HIPCHK(hipHostGetDevicePointer(&d, feats, 0));
      P.feats_dev = static_cast<const float*>(d);
    }
    return 0;
  }

  // Producer side: contiguous free rows starting at physical *row (0 if the ring is full).
  int64_t ring_acquire(int p, int64_t want, int64_t* row) {
    if (p < 0 || p >= (int)parts.size() || !parts[p]->ring) return -1;
    return parts[p]->rr.acquire(want, row);
  }

  int ring_commit(int p, int64_t n, int64_t origin_ns = 0) {
    if (p < 0 || p >= (int)parts.size() || !parts[p]->ring) return -1;
    Partition& P = *parts[p];
    {
      std::lock_guard<std::mutex> lk(P.arr_mu);
      const int64_t t = now_ns();
      P.arrivals.push_back(Partition::Arrival{P.rr.head_count() + n, t, origin_ns > 0 && origin_ns <= t ? origin_ns : 0});
    }
    P.rr.commit(n);                    // publish after the arrival stamp exists
    return 0;
  }

  // Consumer loop for `budget_us`: submit every full micro-batch (and partial ones whose
  // first row has waited >= flush_us: deadline flush bounds latency at low load), complete
  // finished batches; returns the number of batches submitted.
  bool nothing_in_flight() const {
    for (const Slot& s : slots)
      if (s.busy) return false;
    return true;
  }

  int run(int64_t budget_us, int64_t flush_us, ccfd_engine_stats* st) {
    HIPCHK(hipSetDevice(cfg.device));
    // the default 50 us timer slack would turn every idle 5 us sleep into ~55 us of added
    // latency; the scoring thread asks for 1 us (per-thread setting, set once)
    static thread_local bool slack_set = false;
    if (!slack_set) { prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0); slack_set = true; }
    int64_t t_progress = now_ns();
    const int64_t t0 = now_ns();
    const int64_t t_end = t0 + budget_us * 1000;
    const int D = (int)slots.size();
    int submitted = 0;
    for (;;) {
      bool progress = false;
      // 1) retire completed batches (oldest first) without blocking
      for (int k = 0; k < D; ++k) {
        Slot& s = slots[(seq + k) % D];
        if (!s.busy) continue;
        if (!is_done(s)) break;
        // scored ring full: leave the batch (and its ring rows) in place until the consumer
        // drains -- back-pressure reaches ingest instead of losing standard-route records
        if (scored_on.load(std::memory_order_relaxed) && scored_room() < (uint64_t)s.rows) break;
        // flagged ring full: the same -- the batch waits for the hand-off consumer (never dropped)
        int rc = complete(s, st);
        if (rc == kFlagFull) break;
        if (rc) return rc;
        progress = true;
      }
      // 2) submit eligible batches round-robin over ring partitions
      const int64_t now = now_ns();
      for (size_t q = 0; q < parts.size(); ++q) {
        Partition& P = *parts[q];
        if (!P.ring) continue;
        int64_t avail = P.rr.available();
        while (avail > 0) {
          Slot& s = slots[seq % D];
          if (s.busy) break;                               // all slots in flight
          const int64_t phys = P.rr.take_pos();
          // several full micro-batches ready and contiguous in the ring: one coalesced launch
          int K = (int)std::min<int64_t>({(int64_t)coalesce_max(), avail / cfg.max_batch,
                                          (P.n - phys) / cfg.max_batch});
          for (int k = 1; k < K; ++k)
            if (slots[(seq + k) % D].busy) { K = k; break; }
          if (K >= 2) {
            int rc = submit_multi((int)q, phys, cfg.max_batch, K);
            if (rc) return rc;
            for (int k = 0; k < K; ++k) {
              const Partition::Arrival a = P.arrival_of(P.rr.taken() + (int64_t)k * cfg.max_batch);
              slots[(seq + k) % D].t_arrival = a.t;
              slots[(seq + k) % D].t_origin = a.origin;
            }
            seq += K;
            submitted += K;
            P.rr.take((int64_t)K * cfg.max_batch);
            avail -= (int64_t)K * cfg.max_batch;
            progress = true;
            continue;
          }
          int64_t rows = std::min<int64_t>({avail, (int64_t)cfg.max_batch, P.n - phys});
          const bool full = rows == cfg.max_batch || rows == P.n - phys;
          const Partition::Arrival arr_rec = P.arrival_of(P.rr.taken());
          const int64_t arr = arr_rec.t;
          // a partial batch waits for more rows until its deadline -- unless the GPU has
          // nothing in flight (work-conserving: at low / moderate arrival rates a row is
          // scored right away instead of after flush_us; under load the in-flight batches
          // give the ring time to fill, so batches grow back to max_batch)
          if (!full && now - arr < flush_us * 1000 &&
              !(idle_flush_ns >= 0 && now - arr >= idle_flush_ns && nothing_in_flight()))
            break;
          s.part = (int)q; s.start = phys; s.rows = (int32_t)rows;
          const size_t off = (size_t)phys * rowf;
          hipStream_t stream = streams[seq % streams.size()];
          int rc = submit(s, P.feats_dev + off, P.feats + off, (int)rows, stream);
          if (rc) return rc;
          s.t_arrival = arr;
          s.t_origin = arr_rec.origin;
          ++seq;
          ++submitted;
          P.rr.take(rows);
          avail -= rows;
          progress = true;
        }
      }
      if (now_ns() >= t_end) break;
      if (progress) {
        t_progress = now_ns();
      } else if (now_ns() - t_progress < 50'000) {
        cpu_relax();                                   // poll: in-flight batches complete in ~20 us
      } else {
        std::this_thread::sleep_for(std::chrono::microseconds(5));
      }
    }
    if (st) {
      st->wall_s += (now_ns() - t0) * 1e-9;
      st->flagged_dropped = dropped;
      st->flag_full_events = flag_full_events;
      st->submitted += (uint64_t)submitted;
      fill_latency(st);
    }
    return submitted;
  }

  // ------------------------------------------------------------------ native serving thread
  // ccfd_engine_serve_start: a C++ thread calls run() back to back, so scoring latency never
  // waits on the host language's scheduler (the round-3 deployed-topology tail: the Python
  // scoring thread had to win the GIL between run() calls, profiles/r4/tail/).  Every other
  // entry point that touches engine state takes api_mu, which the serving thread holds for one
  // run() call at a time and yields as soon as a caller is waiting (api_waiters), so flips,
  // hot swaps and stats reads interleave between run() calls on the caller's thread.  The
  // flagged / scored rings and the ingest rings have their own locks and never take api_mu.
  std::mutex api_mu;
  std::atomic<int> api_waiters{0};
  std::thread serve_th;
  std::atomic<bool> serve_stop{false};
  std::atomic<bool> serving{false};
  std::atomic<int> serve_hold{0};
  std::atomic<int> serve_rc{0};
  int64_t serve_budget_us = 200, serve_flush_us = 500;
  ccfd_engine_stats serve_st{};            // cumulative (under api_mu)
  uint64_t serve_iters = 0;

  void serve_loop() {
    prctl(PR_SET_NAME, "ccfd-serve", 0, 0, 0);
    (void)hipSetDevice(cfg.device);
    while (!serve_stop.load(std::memory_order_relaxed)) {
      if (api_waiters.load(std::memory_order_acquire) > 0) { std::this_thread::yield(); continue; }
      if (serve_hold.load(std::memory_order_relaxed)) {       // hand-off back-pressure
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        continue;
      }
      std::lock_guard<std::mutex> lk(api_mu);
      const int rc = run(serve_budget_us, serve_flush_us, &serve_st);
      ++serve_iters;
      if (rc < 0) { serve_rc.store(rc); break; }             // error text: ccfd_last_error
    }
  }

  int serve_start(int64_t budget_us, int64_t flush_us) {
    if (serving.load()) { set_error("engine already serving"); return -1; }
    if (budget_us <= 0 || flush_us < 0) { set_error("bad serve budget / flush"); return -1; }
    serve_budget_us = budget_us;
    serve_flush_us = flush_us;
    serve_stop.store(false);
    serve_rc.store(0);
    serving.store(true);
    serve_th = std::thread([this] { serve_loop(); });
    return 0;
  }

  int serve_stop_join() {
    if (!serving.load()) return 0;
    serve_stop.store(true);
    if (serve_th.joinable()) serve_th.join();
    serving.store(false);
    return serve_rc.load();
  }

  int64_t drain_flagged(ccfd_flagged* out, int64_t max) {
    std::lock_guard<std::mutex> lk(ring_mu);
    const uint64_t cap = ring.size();
    int64_t k = 0;
    while (ring_head < ring_tail && k < max) out[k++] = ring[ring_head++ % cap];
    return k;
  }
};

// engine state guard for every API entry point except the ingest rings, the flagged / scored
// drains and the watchdog paths (see the serving-thread note in Engine)
struct ApiLock {
  Engine* e;
  explicit ApiLock(Engine* e_) : e(e_) {
    e->api_waiters.fetch_add(1, std::memory_order_acq_rel);
    e->api_mu.lock();
    e->api_waiters.fetch_sub(1, std::memory_order_acq_rel);
  }
  ~ApiLock() { e->api_mu.unlock(); }
  ApiLock(const ApiLock&) = delete;
  ApiLock& operator=(const ApiLock&) = delete;
};

}  // namespace

extern "C" {

int ccfd_crash_report_install();          // crash_report.cpp

void* ccfd_engine_create(const ccfd_engine_config* cfg) {
  if (!cfg) { set_error("null config"); return nullptr; }
  ccfd_crash_report_install();              // a native fault prints its stack (then faulthandler's)
  auto* e = new Engine();
  if (e->init(*cfg) != 0) { delete e; return nullptr; }
  return e;
}

void ccfd_engine_destroy(void* eng) {
  auto* e = static_cast<Engine*>(eng);
  if (!e) return;
  ccfd_crash_report_install();              // in front of any handler a runtime added since
  e->serve_stop_join();
  delete e;
}

int ccfd_engine_serve_start(void* eng, int64_t budget_us, int64_t flush_us) {
  auto* e = static_cast<Engine*>(eng);
  ApiLock lk(e);
  return e->serve_start(budget_us, flush_us);
}

int ccfd_engine_serve_stop(void* eng) {
  return static_cast<Engine*>(eng)->serve_stop_join();
}

int ccfd_engine_serve_hold(void* eng, int hold) {
  static_cast<Engine*>(eng)->serve_hold.store(hold ? 1 : 0, std::memory_order_relaxed);
  return 0;
}

int ccfd_engine_serve_collect(void* eng, ccfd_engine_stats* out, ccfd_flagged* flagged, int64_t max_flagged,
                              int64_t* n_flagged, ccfd_scored* scored, int64_t max_scored, int64_t* n_scored) {
  auto* e = static_cast<Engine*>(eng);
  if (!out || !n_flagged || (max_flagged > 0 && !flagged)) return -1;
  ApiLock lk(e);                       // no batch completes while the three are read
  *out = e->serve_st;
  e->fill_latency(out);
  out->flagged_dropped = e->dropped;
  out->flag_full_events = e->flag_full_events;
  *n_flagged = e->drain_flagged(flagged, max_flagged);
  if (n_scored) *n_scored = (scored && max_scored > 0) ? e->drain_scored(scored, max_scored) : 0;
  return e->serve_rc.load();
}

int ccfd_engine_serve_stats(void* eng, ccfd_engine_stats* out, int64_t* iters) {
  auto* e = static_cast<Engine*>(eng);
  if (!out) return -1;
  ApiLock lk(e);
  *out = e->serve_st;
  e->fill_latency(out);
  out->flagged_dropped = e->dropped;
  out->flag_full_events = e->flag_full_events;
  if (iters) *iters = (int64_t)e->serve_iters;
  return e->serve_rc.load();
}

int ccfd_engine_set_log(void* eng, int partition, const float* feats, const uint64_t* ids,
                        const uint32_t* customer, int64_t n_rows, int64_t cursor) {
  ApiLock lk(static_cast<Engine*>(eng));
  return static_cast<Engine*>(eng)->set_log(partition, feats, ids, customer, n_rows, cursor);
}

int ccfd_engine_pump(void* eng, int64_t n_batches, int32_t batch_rows, int32_t drain,
                     ccfd_engine_stats* st) {
  ApiLock lk(static_cast<Engine*>(eng));
  return static_cast<Engine*>(eng)->pump(n_batches, batch_rows, drain != 0, st);
}

int ccfd_engine_score_sync(void* eng, const float* x, int32_t n, float* proba_out, uint8_t* route_out) {
  ApiLock lk(static_cast<Engine*>(eng));
  return static_cast<Engine*>(eng)->score_sync(x, n, proba_out, route_out);
}

int ccfd_engine_flip_epoch(void* eng, void* side_stream) {
  ApiLock lk(static_cast<Engine*>(eng));
  return static_cast<Engine*>(eng)->flip_epoch(side_stream);
}

int ccfd_engine_epoch_complete(void* eng, int64_t flip_count) {
  ApiLock lk(static_cast<Engine*>(eng));
  return static_cast<Engine*>(eng)->epoch_complete(flip_count);
}

int ccfd_engine_set_blob(void* eng, const void* blob) {
  ApiLock lk(static_cast<Engine*>(eng));
  return static_cast<Engine*>(eng)->set_blob(blob);
}

int64_t ccfd_engine_drain_flagged(void* eng, ccfd_flagged* out, int64_t max) {
  return static_cast<Engine*>(eng)->drain_flagged(out, max);
}

int ccfd_engine_scored_enable(void* eng, int64_t capacity) {
  auto* e = static_cast<Engine*>(eng);
  if (!e || capacity < 0 || capacity > (int64_t(1) << 28)) { set_error("bad scored-ring capacity"); return -1; }
  ApiLock lk(e);
  int rc = e->drain_all();
  if (rc) return rc;
  std::lock_guard<std::mutex> slk(e->s_mu);
  e->sring.assign((size_t)capacity, ccfd_scored{});
  e->s_head = e->s_tail = e->s_dropped = 0;
  e->scored_on.store(capacity > 0, std::memory_order_relaxed);
  return 0;
}

int64_t ccfd_engine_drain_scored(void* eng, ccfd_scored* out, int64_t max) {
  if (!eng || (!out && max > 0) || max < 0) return -1;
  return static_cast<Engine*>(eng)->drain_scored(out, max);
}

int64_t ccfd_engine_scored_dropped(void* eng) {
  auto* e = static_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->s_mu);
  return (int64_t)e->s_dropped;
}

int64_t ccfd_engine_cursor(void* eng, int partition) {
  auto* e = static_cast<Engine*>(eng);
  if (partition < 0 || partition >= (int)e->parts.size()) return -1;
  Partition& P = *e->parts[partition];
  return P.ring ? P.rr.released_count() : P.cursor;
}

// Watchdog diagnostics (racy reads of plain counters; never blocks): out[0] = micro-batches
// submitted, out[1] = completed in order, out[2] = persistent descriptors posted (-1 when not
// persistent), out[3] = persistent kernel resident (0/1), out[4] = batches in flight.
int ccfd_engine_progress(void* eng, int64_t* out) {
  auto* e = static_cast<Engine*>(eng);
  if (!out) return -1;
  out[0] = (int64_t)e->seq;
  out[1] = e->completed_upto;
  out[2] = e->persistent && e->pctl ? (int64_t)__atomic_load_n(&e->pctl->posted, __ATOMIC_RELAXED) : -1;
  out[3] = e->prunning ? 1 : 0;
  int64_t busy = 0;
  for (const auto& s : e->slots) busy += s.busy ? 1 : 0;
  out[4] = busy;
  return 0;
}

// Watchdog exit path: ask a resident persistent kernel to leave (the stop word every
// waiting workgroup polls) and wait up to `timeout_ms` for its grid to drain, so a process
// that is about to _exit never leaves a resident kernel behind.  Touches only the host
// control record and queries the kernel's stream.  0 = no kernel resident / drained.
int ccfd_engine_emergency_stop(void* eng, int timeout_ms) {
  auto* e = static_cast<Engine*>(eng);
  if (!e->persistent || !e->pctl || !e->prunning) return 0;
  __atomic_store_n(&e->pctl->stop, 1ull, __ATOMIC_RELEASE);
  const int64_t t0 = now_ns();
  while (hipStreamQuery(e->pstream) == hipErrorNotReady) {
    if (now_ns() - t0 > (int64_t)timeout_ms * 1000000ll) return -6;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  return 0;
}

int ccfd_engine_set_amount(void* eng, int partition, const float* amount) {
  auto* e = static_cast<Engine*>(eng);
  ApiLock lk(e);
  if (partition < 0 || partition >= (int)e->parts.size()) { set_error("bad partition index"); return -1; }
  int rc = e->drain_all();
  if (rc) return rc;
  e->parts[partition]->amount = amount;
  return 0;
}

int ccfd_engine_set_ring(void* eng, int partition, float* feats, uint64_t* ids, uint32_t* customer,
                         int64_t capacity) {
  ApiLock lk(static_cast<Engine*>(eng));
  return static_cast<Engine*>(eng)->set_ring(partition, feats, ids, customer, capacity);
}

int64_t ccfd_engine_ring_acquire(void* eng, int partition, int64_t want, int64_t* row) {
  return static_cast<Engine*>(eng)->ring_acquire(partition, want, row);
}

int ccfd_engine_ring_commit(void* eng, int partition, int64_t n) {
  return static_cast<Engine*>(eng)->ring_commit(partition, n);
}

int ccfd_engine_ring_commit_at(void* eng, int partition, int64_t n, int64_t origin_ns) {
  return static_cast<Engine*>(eng)->ring_commit(partition, n, origin_ns);
}

int ccfd_engine_run(void* eng, int64_t budget_us, int64_t flush_us, ccfd_engine_stats* st) {
  auto* e = static_cast<Engine*>(eng);
  if (e->serving.load()) { ccfd::set_error("engine is serving (ccfd_engine_serve_start): run() is its thread's"); return -1; }
  ApiLock lk(e);
  return static_cast<Engine*>(eng)->run(budget_us, flush_us, st);
}

int ccfd_engine_trace_enable(void* eng, int32_t capacity) {
  if (!eng || capacity < 0 || capacity > (1 << 24)) return -1;
  Engine* e = static_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->trace_mu);
  e->trace.assign((size_t)capacity, ccfd_batch_trace{});
  e->trace_n = 0;
  e->trace_on.store(capacity > 0, std::memory_order_relaxed);
  return 0;
}

int ccfd_engine_trace_read(void* eng, ccfd_batch_trace* out, int32_t max) {
  if (!eng || (!out && max > 0) || max < 0) return -1;
  Engine* e = static_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->trace_mu);
  const uint64_t cap = e->trace.size();
  if (cap == 0) return 0;
  const uint64_t have = std::min<uint64_t>(e->trace_n, cap);
  const uint64_t n = std::min<uint64_t>(have, (uint64_t)max);
  const uint64_t first = e->trace_n - n;                 // the newest n, oldest first
  for (uint64_t i = 0; i < n; ++i) out[i] = e->trace[(first + i) % cap];
  return (int)n;
}

void ccfd_engine_reset_stats(void* eng) {
  auto* e = static_cast<Engine*>(eng);
  ApiLock lk(e);
  e->reset_latency();
  e->t_submit_ns = e->t_wait_ns = e->t_complete_ns = 0;
  e->dev_batches = e->dev_exec_ns = 0;
  std::memset(e->dev_hist, 0, sizeof(e->dev_hist));
  std::memset(e->dev_hist_rows, 0, sizeof(e->dev_hist_rows));
}

}  // extern "C"
