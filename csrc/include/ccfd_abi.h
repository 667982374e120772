// C ABI of libccfd_hip.so -- the MI355X-native compute + streaming runtime.
//
// Python binds this with ctypes (ccfd_demo_summit_amd/ops/_lib.py); every struct here
// has a ctypes mirror there, keep them in sync (test_abi_layout checks sizes/offsets).
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum ccfd_model_kind { CCFD_MODEL_LR = 0, CCFD_MODEL_MLP = 1, CCFD_MODEL_GBDT = 2 };

// Cumulative u64 counter slots written by the scoring kernels' epilogue (device side)
// and all-reduced across ranks (X2 in SURVEY.md §2.4).  Mirrors ops/layout.py.
enum ccfd_counter_slot {
  CCFD_CNT_INCOMING = 0,      // transaction.incoming
  CCFD_CNT_FRAUD = 1,         // transaction.outgoing{type=fraud}
  CCFD_CNT_STANDARD = 2,      // transaction.outgoing{type=standard}
  CCFD_CNT_PROBA_E6 = 3,      // sum(round(proba_1 * 1e6))
  CCFD_CNT_WIRE_STALE = 4,    // G32 / G20 rows whose bin stamp != the model's (proba NaN, standard route)
  CCFD_CNT_HIST_STD = 8,      // 14 amount buckets, standard route
  CCFD_CNT_HIST_FRAUD = 24,   // 14 amount buckets, fraud route
  CCFD_CNT_SLOTS = 64
};
#define CCFD_N_AMOUNT_BUCKETS 14
#define CCFD_N_FEATURES 30

// ccfd_score_args.flags / ccfd_persist_args.flags: reserved (0).  Completion ordering is
// fixed: each workgroup releases at system scope, then takes a relaxed ticket.
#define CCFD_ARG_FENCE_SYS 0
#define CCFD_ARG_FENCE_COHERENT 1   // outputs live in fine-grained pinned memory (informational)
#define CCFD_ARG_WIRE_W64 2           // x holds W64 rows (64 B: bf16 V1..V28, f32 Time, f32 Amount)
#define CCFD_WIRE_ROW_BYTES 64
// G32 rows (GBDT only, 32 B): byte j < 30 = bin of feature j against the model's split
// table (#edges_j < x_j, so `x_j > thr` == `bin_j > k(thr)` exactly), byte 30 = amount
// bucket (K6), byte 31 = bin-table stamp (1..255; rows encoded for another table are
// counted in CCFD_CNT_WIRE_STALE and not scored).  Amount itself stays host-side.
#define CCFD_ARG_WIRE_G32 4
#define CCFD_G32_ROW_BYTES 32
// G20 rows (GBDT only, 20 B; flags carry WIRE_G32 | WIRE_G20): the same bins packed 5 bits
// each for bin tables of <= 31 edges per feature -- bits [5j, 5j+5) = bin of feature j,
// bits [150, 154) = amount bucket, bits [154, 160) = bin-table stamp (1..63).  Little-endian
// bit order over the 5 dwords of the row.  0.625x the bytes of a G32 row, equally exact.
#define CCFD_ARG_WIRE_G20 8
#define CCFD_G20_ROW_BYTES 20
#define CCFD_G20_MAX_EDGES 31
#define CCFD_ARG_CHUNK_RING 128       // persistent G32: one-chunk prefetch ring (default) instead of the whole item in flight
#define CCFD_ARG_FLAG_DIRECT 1024      // W64 launch kernels: reserve flag-list slots per ballot (A/B of the LDS staging)
#define CCFD_ARG_PIPE_ITEMS 256       // persistent W64 MLP: statically assigned 64/128-row items, the next
                                      // item's rows fetched while the current one is scored

// Routing rule program (router/rules.py RuleSet.device_program): the configurable routing
// rules (reference "Drools rules", README.md:427) evaluated per row in the scoring
// kernels' epilogue instead of the plain `proba >= threshold` test.  Postfix code over a
// <= CCFD_RULE_MAX_STACK-deep f32 stack; rules are tried in order, the first whose
// condition holds decides the route, DEFAULT applies otherwise.  Variables: 0 = proba_1,
// 1 + j = feature j in reference column order (Time, V1..V28, Amount).
#define CCFD_RULE_MAX_OPS 48
#define CCFD_RULE_MAX_STACK 8
enum ccfd_rule_opcode {
  CCFD_RULE_END = 0,     // pop cond; first true rule sets route = arg
  CCFD_RULE_VAR = 1,     // push variable arg
  CCFD_RULE_CONST = 2,   // push imm
  CCFD_RULE_ADD = 3, CCFD_RULE_SUB = 4, CCFD_RULE_MUL = 5, CCFD_RULE_DIV = 6,
  CCFD_RULE_NEG = 7, CCFD_RULE_ABS = 8, CCFD_RULE_LOG1P = 9, CCFD_RULE_MIN = 10, CCFD_RULE_MAX = 11,
  CCFD_RULE_GT = 12, CCFD_RULE_GE = 13, CCFD_RULE_LT = 14, CCFD_RULE_LE = 15, CCFD_RULE_EQ = 16,
  CCFD_RULE_NE = 17, CCFD_RULE_AND = 18, CCFD_RULE_OR = 19, CCFD_RULE_NOT = 20
};
typedef struct ccfd_rule_op {
  int16_t op;
  int16_t arg;
  float imm;
} ccfd_rule_op;
typedef struct ccfd_rule_prog {   // device memory
  int32_t n_ops;
  int32_t default_route;          // 1 = fraud, 0 = standard
  int32_t n_rules;
  int32_t max_stack;
  ccfd_rule_op ops[CCFD_RULE_MAX_OPS];
} ccfd_rule_prog;

typedef struct ccfd_score_args {
  const float* x;        // features, row-major [n][ld] (device or host-mapped pointer)
  int64_t ld;            // row stride in floats (fast path: 30)
  int32_t n;             // rows
  int32_t model;         // ccfd_model_kind
  const void* blob;      // packed model (device memory), see models/*.py pack()
  float threshold;       // FRAUD_THRESHOLD
  int32_t gbdt_trees;    // GBDT only
  int32_t gbdt_depth;    // GBDT only
  int32_t flags;         // CCFD_ARG_* (informational)
  float* proba;          // out [n] proba_1 (device or host-mapped), may be NULL
  uint8_t* route;        // out [n] 1 = fraud route, may be NULL
  unsigned long long* counters;  // device [CCFD_CNT_SLOTS] accumulated atomically, may be NULL
  // Launch-completion protocol (engine slots; all NULL for a plain launch):
  //   every workgroup publishes its outputs (system-scope release) and bumps slot_ctl[0];
  //   fraud-routed rows append their row index to flag_idx (reserved via slot_ctl[1]);
  //   the LAST workgroup resets slot_ctl, stores done_rec[1] = #flagged and then
  //   done_rec[0] = done_seq (system-scope release) -> the host polls done_rec[0] in pinned
  //   memory instead of recording/synchronising a HIP event per micro-batch.
  unsigned int* slot_ctl;        // device [4]: ticket, #flagged, u64 start timestamp (K7)
  unsigned int* flag_idx;        // host-mapped [n] row indices of fraud-routed rows
  unsigned long long* done_rec;  // host-mapped coherent [4]: seq, #flagged, t_start, t_end
  unsigned long long done_seq;
  const ccfd_rule_prog* rules;   // device; NULL = route by `proba >= threshold`
} ccfd_score_args;

// Coalesced launch: `nsub` consecutive micro-batches of `sub_rows` rows (contiguous in x,
// base.n rows in total) scored by ONE launch; every micro-batch keeps its own outputs,
// flag list and completion record, and its workgroups signal it independently.  Cuts the
// per-launch host + dispatch cost by nsub while the unit of completion stays the micro-batch.
#define CCFD_MAX_SUB 8
typedef struct ccfd_sub_batch {
  float* proba;
  uint8_t* route;
  unsigned int* slot_ctl;
  unsigned int* flag_idx;
  unsigned long long* done_rec;
  unsigned long long done_seq;
} ccfd_sub_batch;   // 48 bytes

typedef struct ccfd_multi_args {
  ccfd_score_args base;            // x, n (total), model, blob, threshold, flags, counters
  int32_t nsub;
  int32_t sub_rows;
  ccfd_sub_batch sub[CCFD_MAX_SUB];
} ccfd_multi_args;

int ccfd_score_launch_multi(const ccfd_multi_args* m, void* stream);

// Enqueue one fused scoring launch (normalize -> model -> sigmoid -> threshold ->
// counters/histogram) on `stream` (a hipStream_t; NULL = legacy default stream).
// Returns 0 or a negative error code (shape/alignment checks happen on the host).
int ccfd_score_launch(const ccfd_score_args* a, void* stream);

// ---------------------------------------------------------------------------
// Persistent streaming kernel (exec_mode = 1): ONE long-running launch per engine; the
// host publishes micro-batch descriptors into a ring in coherent pinned memory and bumps
// `posted`; resident workgroups claim 64..256-row work items with one device atomic, wait for
// the descriptor to be posted, score, and the last workgroup of a micro-batch publishes
// its completion record.  No per-batch launch, event or copy on the host.
#define CCFD_PERSIST_MAX_RING 64
#define CCFD_PERSIST_ITEM_ROWS 256   // default item of f32 rows: 4 waves x 4 tiles x 16 rows (W64: 512, G32: 512)
#define CCFD_PERSIST_GRID 128        // default resident workgroups (+ the doorbell workgroup 0)
#define CCFD_PERSIST_GRID_W64 64     // ... for W64 rows (512-row items, every tile in flight)
#define CCFD_PERSIST_GRID_G20 216    // ... for G20 rows (GBDT, BASELINE-size ensembles)

typedef struct ccfd_persist_desc {   // host-coherent pinned, written before `posted`
  const float* x;          // device-visible rows [n][30]
  float* proba;            // host-mapped out [n] (may be NULL)
  uint8_t* route;          // host-mapped out [n] (may be NULL)
  unsigned int* flag_idx;  // host-mapped out: compacted fraud-routed row indices
  int32_t n;
  int32_t epoch;           // counter buffer index (0/1) for the X2 epoch flip
  uint64_t seq;            // 0-based micro-batch sequence number
} ccfd_persist_desc;

typedef struct ccfd_persist_ctl {    // host-coherent pinned
  uint64_t posted;         // host -> GPU: number of descriptors published
  uint64_t stop;           // host -> GPU: exit once every posted batch is claimed
  uint64_t done[CCFD_PERSIST_MAX_RING][4];   // GPU -> host: {seq + 1, #flagged, t_start, t_end} per ring slot
  uint64_t exited;         // GPU -> host: workgroups that left the loop
} ccfd_persist_ctl;

typedef struct ccfd_persist_dev {    // device memory
  unsigned long long work_next;                   // next work item to claim
  unsigned long long posted;                      // device mirror of ctl->posted (doorbell WG)
  unsigned long long stop;                        // device mirror of ctl->stop
  unsigned long long _pad;
  unsigned int remaining[CCFD_PERSIST_MAX_RING];  // items left per ring slot
  unsigned int nflag[CCFD_PERSIST_MAX_RING];      // flagged rows per ring slot
  ccfd_persist_desc desc[CCFD_PERSIST_MAX_RING];  // device mirror of the descriptor ring
  unsigned long long tstart[CCFD_PERSIST_MAX_RING];  // K7: device clock when item 0 was claimed
} ccfd_persist_dev;

typedef struct ccfd_persist_args {
  ccfd_persist_ctl* ctl;           // device alias of the host control block
  const ccfd_persist_desc* desc;   // device alias of the host descriptor ring
  ccfd_persist_dev* dev;
  int32_t ring;                    // R ring slots (<= CCFD_PERSIST_MAX_RING)
  int32_t items_per_batch;         // ceil(max_batch / item_rows)
  int32_t model;                   // MLP, LR, or GBDT on G32 rows
  float threshold;
  int32_t tiles_per_wave;          // item_rows = 4 waves x tiles_per_wave x 16 rows
  int32_t flags;                   // CCFD_ARG_* (informational)
  const void* blob;
  unsigned long long* counters[2];
  const ccfd_rule_prog* rules;     // device; NULL = threshold route
  int32_t gbdt_trees, gbdt_depth;  // GBDT (G32 rows): tiles_per_wave = 64-row chunks per wave per item
} ccfd_persist_args;

int ccfd_persist_launch(const ccfd_persist_args* a, int grid, void* stream);

// ---------------------------------------------------------------------------
// Host memory (pinned, device-mapped; used for partition logs and result rings)
void* ccfd_host_alloc(size_t bytes);                 // hipHostMalloc(mapped|portable|NumaUser)
int ccfd_host_free(void* p);
void* ccfd_host_device_ptr(void* host_ptr);          // hipHostGetDevicePointer

// ---------------------------------------------------------------------------
// Streaming engine: a GPU-resident micro-batcher over a pinned host partition log.
typedef struct ccfd_engine_config {
  int32_t device;
  int32_t model;
  const void* blob;            // device pointer (owned by caller)
  int32_t gbdt_trees, gbdt_depth;
  float threshold;
  int32_t max_batch;           // rows per micro-batch (4096)
  int32_t depth;               // micro-batches in flight
  int32_t n_streams;           // HIP streams used round-robin
  int32_t input_mode;          // 0 = DMA H2D into HBM staging, 1 = zero-copy host reads
  int32_t output_mode;         // 0 = zero-copy host writes, 1 = device + D2H copy
  int32_t flag_capacity;       // flagged-transaction ring capacity (records)
  int32_t exec_mode;           // 0 = one fused launch per micro-batch, 1 = persistent kernel
  int32_t persist_grid;        // workgroups of the persistent kernel (0 = 256)
  int32_t wire;                // 0 = f32 rows [30]; 1 = W64 rows (64 B); 2 = G32 rows (32 B, GBDT); 3 = G20 (20 B, GBDT)
  int32_t coalesce;            // launch mode: up to this many ready micro-batches per launch (<= 8)
  int32_t persist_items;       // persistent MLP on W64 rows: 0 = env (CCFD_PERSIST_PIPE), 1 = claimed
                               // 512-row items (throughput), 2 = pipelined 128-row items (latency)
  unsigned long long* counters[2];  // device counter buffers, alternated per epoch
  const ccfd_rule_prog* rules;      // device rule program (owned by caller); NULL = threshold
} ccfd_engine_config;

typedef struct ccfd_flagged {
  uint64_t tx_id;
  uint32_t customer;
  float proba;
  float amount;
  uint32_t partition;
} ccfd_flagged;   // 24 bytes

// Opt-in per-row scored record (ccfd_engine_scored_enable): every completed row, fraud- and
// standard-routed, with its proba_1 and route -- what the reference router needs to start a
// standard OR a fraud process per transaction (README.md:549-552).
typedef struct ccfd_scored {
  uint64_t tx_id;
  uint32_t customer;
  float proba;
  float amount;
  uint16_t partition;
  uint8_t route;               // 1 = fraud (the kernel's route byte), 0 = standard
  uint8_t pad;
} ccfd_scored;    // 24 bytes

typedef struct ccfd_engine_stats {
  uint64_t batches, rows, fraud_rows, flagged_dropped;
  double wall_s;
  double lat_p50_us, lat_p99_us, lat_max_us, lat_mean_us;
  uint64_t lat_hist[256];      // batch latency histogram in ns, 4 buckets per octave:
                               // bucket i holds [2^(i/4), 2^((i+1)/4))
  // host-side time accounting of the submission/completion thread (cumulative ns)
  uint64_t host_submit_ns;     // H2D enqueue + kernel launch + event record
  uint64_t host_wait_ns;       // blocked in hipEventSynchronize (GPU not done yet)
  uint64_t host_complete_ns;   // route scan + flagged hand-off + bookkeeping
  // K7 stream_stats: per-micro-batch device execution time measured on the GPU's constant
  // wall clock (s_memrealtime, first workgroup start -> last workgroup completion)
  uint64_t dev_batches;
  uint64_t dev_exec_ns;        // sum
  uint64_t dev_hist[256];      // same bucketing as lat_hist
  // row-weighted twins of lat_hist / dev_hist (each batch adds its row count): per-transaction
  // latency distributions, exported as the Seldon engine's server / client request histograms
  // (deploy/grafana/SeldonCore.json:119-531; one scored transaction = one reference request)
  uint64_t lat_hist_rows[256];
  uint64_t dev_hist_rows[256];
  // the last scored transaction (the reference model's "last request" gauges proba_1 / Amount /
  // V17 / V10, deploy/grafana/ModelPrediction.json:96-322): its raw log row in the engine's row
  // format (f32[30], W64, G32 or G20), proba, Amount and id; last_seq = 0 until one completed
  uint64_t last_seq;
  uint64_t last_tx_id;
  float last_proba;
  float last_amount;
  int32_t last_partition;
  int32_t last_row_bytes;
  uint8_t last_row[128];
  // producer send -> scored (results in host memory) per ring micro-batch whose rows carried a
  // send time (ccfd_engine_ring_commit_at: the ccfd-ts record header); same bucketing as lat_hist
  uint64_t origin_batches;
  uint64_t origin_hist[256];
  uint64_t origin_hist_rows[256];
  // lossless hand-off (round 6): micro-batches submitted by the call(s) that filled this record,
  // and completions deferred so far because the flagged ring had no room for a batch's records
  uint64_t submitted;
  uint64_t flag_full_events;
} ccfd_engine_stats;

// ccfd_engine_pump / drain paths: a finished micro-batch's fraud-routed records do not fit in
// the flagged ring.  Nothing was retired or lost; drain the ring (ccfd_engine_drain_flagged) and
// call again (pump: with n_batches - stats.submitted).  ccfd_engine_run() never returns it: it
// leaves such batches in flight until a later call finds room.
#define CCFD_ENGINE_FLAG_FULL 1

void* ccfd_engine_create(const ccfd_engine_config* cfg);
void ccfd_engine_destroy(void* eng);
const char* ccfd_last_error(void);

// Register partition log p: pinned host features [n_rows][30] (+ optional ids/customer/
// amount columns).  Rows are consumed from `cursor` and wrap around.
int ccfd_engine_set_log(void* eng, int partition, const float* feats, const uint64_t* ids,
                        const uint32_t* customer, int64_t n_rows, int64_t cursor);
// Score `n_batches` micro-batches of `batch_rows` rows round-robin over the registered
// partitions.  With drain != 0 it blocks until every submitted batch is complete;
// otherwise up to `depth` batches stay in flight across calls (no pipeline bubble between
// steps).  Counts of completed batches accumulate into *st; latency percentiles cover all
// batches completed since the last ccfd_engine_reset_stats().  Returns CCFD_ENGINE_FLAG_FULL
// (after submitting stats.submitted batches) when the flagged ring cannot take a finished
// batch's records: the hand-off is lossless, so the caller drains and resumes.
int ccfd_engine_pump(void* eng, int64_t n_batches, int32_t batch_rows, int32_t drain,
                     ccfd_engine_stats* st);
// Score one caller-provided batch (pinned host or device pointer) synchronously; proba/route
// are copied to the caller's host arrays.  Used by predict() serving and tests.
int ccfd_engine_score_sync(void* eng, const float* x, int32_t n, float* proba_out, uint8_t* route_out);
// Epoch flip for the X2 all-reduce: subsequent batches accumulate into the other counter
// buffer; `side_stream` (hipStream_t) is made to wait for every batch of the closed epoch.
// Returns the index (0/1) of the closed buffer.
int ccfd_engine_flip_epoch(void* eng, void* side_stream);
// 1 once every micro-batch submitted before the flip that closed `epoch_index` (the value
// returned by flip) has completed.  Required before reducing a closed epoch buffer in
// exec_mode 1 (the persistent kernel has no per-batch events a stream could wait on).
int ccfd_engine_epoch_complete(void* eng, int64_t flip_count);
// Hot swap: drain in-flight micro-batches, then score later ones with `blob` (same kind/shape).
int ccfd_engine_set_blob(void* eng, const void* blob);
// Drain up to `max` flagged records (fraud route) into `out`; returns count.
int64_t ccfd_engine_drain_flagged(void* eng, ccfd_flagged* out, int64_t max);
int64_t ccfd_engine_cursor(void* eng, int partition);
// Scored-record ring of `capacity` rows (0 = off, the default).  Records are assembled when a
// micro-batch completes, from the per-row proba_1 / route the kernel's epilogue wrote into the
// batch's pinned output slots (the same epilogue that compacts the flag list) and the log's
// id / customer / Amount columns.  ccfd_engine_run() does not retire a batch while the ring
// lacks room for it (back-pressure to ingest, nothing is lost); pump() / drain paths count
// rows that do not fit in ccfd_engine_scored_dropped().
int ccfd_engine_scored_enable(void* eng, int64_t capacity);
int64_t ccfd_engine_drain_scored(void* eng, ccfd_scored* out, int64_t max);
int64_t ccfd_engine_scored_dropped(void* eng);
// Watchdog diagnostics: submitted, completed, persistent posted (-1), kernel resident, in flight.
int ccfd_engine_progress(void* eng, int64_t* out5);
// Watchdog exit path: stop a resident persistent kernel, wait <= timeout_ms for it to drain.
int ccfd_engine_emergency_stop(void* eng, int timeout_ms);
// G32 logs/rings: host-side Amount column of partition p (the flagged-record amount; the
// rows themselves carry only its bucket).  Call after set_log / set_ring.
int ccfd_engine_set_amount(void* eng, int partition, const float* amount);

// Streaming (ring) mode: partition p is an SPSC ring of `capacity` rows in pinned memory.
// Producer (ingest thread): ring_acquire -> write rows at [row, row+n) -> ring_commit(n).
// Consumer: ccfd_engine_run() submits full micro-batches, flushes partial ones whose first
// row has waited `flush_us`, completes finished ones and frees their ring space.
int ccfd_engine_set_ring(void* eng, int partition, float* feats, uint64_t* ids, uint32_t* customer,
                         int64_t capacity);
int64_t ccfd_engine_ring_acquire(void* eng, int partition, int64_t want, int64_t* row);
int ccfd_engine_ring_commit(void* eng, int partition, int64_t n);
// ... with the producer send time of these rows on the engine's steady clock (ns, 0 = unknown):
// feeds the produce -> scored histogram (ccfd_engine_stats.origin_hist)
int ccfd_engine_ring_commit_at(void* eng, int partition, int64_t n, int64_t origin_ns);
int ccfd_engine_run(void* eng, int64_t budget_us, int64_t flush_us, ccfd_engine_stats* st);
void ccfd_engine_reset_stats(void* eng);
// Native serving thread: a C++ thread calls ccfd_engine_run(budget_us, flush_us) back to back
// (the deployed engine's consumer loop, free of the host language's scheduler).  While it
// serves, ccfd_engine_run() from another thread is refused; every other call is serialised with
// it between two run() calls.  hold != 0 pauses scoring (hand-off back-pressure).  serve_stats
// copies the cumulative counters / latency histograms since serve start (reset_stats zeroes the
// latencies), returns the serving thread's error code (0 = running or stopped cleanly).
int ccfd_engine_serve_start(void* eng, int64_t budget_us, int64_t flush_us);
int ccfd_engine_serve_stop(void* eng);
int ccfd_engine_serve_hold(void* eng, int hold);
int ccfd_engine_serve_stats(void* eng, ccfd_engine_stats* out, int64_t* iters);
// One consistent cut while serving: the cumulative stats AND every flagged (and, if `scored`,
// scored) record of the batches those stats count, drained together between two run() calls
// (a commit snapshot taken BEFORE this call never covers a row whose records it misses).
int ccfd_engine_serve_collect(void* eng, ccfd_engine_stats* out, ccfd_flagged* flagged, int64_t max_flagged,
                              int64_t* n_flagged, ccfd_scored* scored, int64_t max_scored, int64_t* n_scored);

// Per-micro-batch stage trace (SURVEY.md §5 "per-stage timestamps in a ring buffer"): the
// last `capacity` completed batches, host times in ns of the engine's monotonic clock, device
// times in ns of the GPU wall clock (its own epoch; tools align the two).  capacity 0 = off.
typedef struct {
  int64_t seq;          // submission number
  int32_t partition;    // partition (log / ring) index; score() batches are not traced
  int32_t rows;
  int64_t t_arrival;    // oldest row committed to the ring (0: pre-filled log / score())
  int64_t t_submit;     // descriptor posted / kernel launched
  int64_t t_landed;     // completion record seen in host memory (completion stamper)
  int64_t t_complete;   // retired by the engine thread (flagged rows handed off)
  int64_t dev_start;    // first item claimed / first workgroup started (device clock, ns)
  int64_t dev_end;      // last item done (device clock, ns); 0 when outputs went by DMA
  int32_t flagged;
  int32_t pad;
} ccfd_batch_trace;
int ccfd_engine_trace_enable(void* eng, int32_t capacity);
// copies the retained entries, oldest first; returns the number written (<= max)
int ccfd_engine_trace_read(void* eng, ccfd_batch_trace* out, int32_t max);

// ---------------------------------------------------------------------------
// Native ingest helpers (JSON transaction parser, TXB1 batch codec)
// Parse `n_msgs` JSON transactions (concatenated, offsets[i]..offsets[i+1]) into
// feats[n][30], ids[n], customer[n].  Returns number parsed or -(index+1) on error.
int64_t ccfd_parse_json_batch(const char* buf, const int64_t* offsets, int64_t n_msgs,
                              float* feats, uint64_t* ids, uint32_t* customer);
// Same, straight into W64 wire rows (64 B each).
int64_t ccfd_parse_json_batch_w64(const char* buf, const int64_t* offsets, int64_t n_msgs,
                                  uint8_t* rows, uint64_t* ids, uint32_t* customer);
// f32 rows (stride ld >= 30) -> W64 wire rows; returns n or -1.
int64_t ccfd_encode_w64(const float* x, int64_t n, int64_t ld, uint8_t* out);
// f32 rows -> G32 rows against a bin table: `edges` = the sorted split thresholds of every
// feature back to back, feature j owning edges[offsets[j] .. offsets[j+1]) (<= 255 each);
// `stamp` in 1..255.  amount_out (may be NULL) receives the raw Amount column.  Returns n or -1.
int64_t ccfd_encode_g32(const float* x, int64_t n, int64_t ld, const float* edges, const int32_t* offsets,
                        int32_t stamp, uint8_t* out, float* amount_out);
// Same table -> G20 rows (<= 31 edges per feature, stamp 1..63); returns n or -1.
int64_t ccfd_encode_g20(const float* x, int64_t n, int64_t ld, const float* edges, const int32_t* offsets,
                        int32_t stamp, uint8_t* out, float* amount_out);

// ---------------------------------------------------------------------------
// Native Kafka consumer (csrc/engine/kafka_consumer.cpp): Metadata v1 -> one connection
// per partition leader -> Fetch v4 -> RecordBatch v2 (uncompressed or gzip) -> TXB1 / JSON
// values -> rows in the engine's pinned partition rings.  `host` may be a bootstrap list
// "h1:p1,h2:p2" (then `port` is only the default for entries without one).
typedef struct ccfd_kc_partition {
  int32_t kafka_partition;   // partition id in the topic
  int32_t engine_partition;  // ring index in the engine (engine sink)
  int64_t start_offset;      // first offset to fetch (committed offset)
  void* feats;               // ring rows (f32[30] or W64), array sink: [capacity] rows
  uint64_t* ids;
  uint32_t* customer;
  int64_t capacity;          // array sink only
  float* amount;             // G32 rows: host-side Amount column ([capacity] rows), may be NULL
} ccfd_kc_partition;

typedef struct ccfd_kc_stats {
  uint64_t records, rows, bytes, errors, fetches;
  uint64_t metadata_refreshes;   // leader / broker changes seen (NOT_LEADER, dead connection, ...)
  uint64_t offset_resets;        // OFFSET_OUT_OF_RANGE handled by the reset policy
  uint64_t leaders;              // broker connections used by the last fetch round
  // time attribution of the consumer thread (ns, cumulative): waiting on brokers (send +
  // receive of Fetch), handling responses (RecordBatch / TXB1 / JSON parsing + the two
  // below), writing rows into the ring (copy / W64 / G20 / G32 encoding), and blocked on a
  // full ring (engine back-pressure)
  uint64_t io_ns, handle_ns, encode_ns, ring_wait_ns;
} ccfd_kc_stats;

// offset reset policy on OFFSET_OUT_OF_RANGE (auto.offset.reset)
#define CCFD_KC_RESET_EARLIEST 0
#define CCFD_KC_RESET_LATEST 1
#define CCFD_KC_RESET_NONE 2     // stop the partition and report the error

void* ccfd_kc_create_engine(void* engine, const char* host, int port, const char* topic,
                            const ccfd_kc_partition* parts, int n_parts, int wire);
void* ccfd_kc_create_array(const char* host, int port, const char* topic, const ccfd_kc_partition* parts,
                           int n_parts, int wire);
int ccfd_kc_start(void* kc);
void ccfd_kc_stop(void* kc);
void ccfd_kc_destroy(void* kc);
// highest offset whose rows have all been consumed downstream (-1: nothing new)
int64_t ccfd_kc_committable(void* kc, int part_index);
void ccfd_kc_get_stats(void* kc, ccfd_kc_stats* out);
const char* ccfd_kc_last_error(void* kc);
int64_t ccfd_kc_feed_record_set(void* kc, const uint8_t* data, int64_t n);   // tests / fuzzing
void ccfd_kc_fetch_age_hist(void* kc, uint64_t* out256);   // batches by send -> fetched age (ns, 4 buckets/octave)
int64_t ccfd_kc_last_origin(void* kc);         // send time (steady ns) of the last batch's ccfd-ts header, 0 = none
int ccfd_kc_set_offset_reset(void* kc, int policy);                           // before start
int64_t ccfd_kc_position(void* kc, int part_index);                           // next offset to fetch
// G32 / G20 sinks (wire = 2 / 3): the bin table rows are encoded against (ccfd_encode_g32 layout);
// required before ccfd_kc_start.  The table is copied.
int ccfd_kc_set_bins(void* kc, const float* edges, const int32_t* offsets, int32_t stamp);

#ifdef __cplusplus
}
#endif
