// Transaction-id -> process-instance-id index for the KIE tier's idempotent process starts
// (process/engine.py ProcessEngine.start_standard_array).
// Two modes: a count window (the oldest key leaves when `window` keys are held), or gated: a
// fixed capacity the caller drains with ccfd_dedupe_erase once the engine has committed the
// Kafka offsets behind those keys -- a key whose transaction can still be re-delivered never
// leaves, however many other keys arrive meanwhile.
//
// At the reference's semantics every transaction starts a process (README.md:552), so at
// 1e6 tx/s a KIE shard admits ~2.5e5 standard starts a second: a Python set/dict over a
// 1M-entry window cost ~1 us a row.  This is an open-addressing table (linear probing,
// backward-shift deletion, no tombstones) with a FIFO ring of the admitted keys: the oldest
// key leaves the table when the window is full.  One call admits a whole hand-off batch:
// a key already present (a re-delivered batch, or a transaction twice in one batch) answers
// its stored instance id; a new key gets the next id of the caller's arithmetic sequence
// (first_id + k * stride -- shard-encoded ids, iid = shard + K * n) and is returned in
// new_keys in admission order, which is what the journal records.
// Not thread-safe: the caller (the process engine) holds its own lock.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

namespace {

constexpr int64_t kEmpty = INT64_MIN;       // tx ids are non-negative (uint63 on the wire)

inline uint64_t mix(uint64_t x) {           // splitmix64 finaliser
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27; x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

struct Slot {
  int64_t key, val;
};

struct Index {
  std::vector<Slot> t;                      // table: key + id in one line (one miss a probe)
  std::vector<int64_t> ring;                // FIFO of admitted keys
  uint64_t mask = 0;
  int64_t window = 0, head = 0, count = 0;  // ring: oldest at head, `count` live
  // gated (commit-watermark) mode: `window` is a hard capacity, nothing leaves by itself -- the
  // caller erases keys once the offsets behind them are committed (ccfd_dedupe_erase, in any
  // order: no FIFO ring), and an admission that could overflow the capacity is refused (-2:
  // back-pressure, never an eviction)
  bool gated = false;

  explicit Index(int64_t w, bool g = false) : window(w), gated(g) {
    uint64_t cap = 16;
    while (cap < (uint64_t)w * 2 + 16) cap <<= 1;   // load factor <= 0.5
    t.assign(cap, Slot{kEmpty, 0});
    if (!gated) ring.assign((size_t)w, 0);
    mask = cap - 1;
  }

  int64_t find(int64_t k) const {
    for (uint64_t i = mix((uint64_t)k) & mask;; i = (i + 1) & mask) {
      if (t[i].key == k) return (int64_t)i;
      if (t[i].key == kEmpty) return -1;
    }
  }

  void erase_slot(uint64_t i) {             // backward-shift deletion
    for (uint64_t j = (i + 1) & mask;; j = (j + 1) & mask) {
      if (t[j].key == kEmpty) break;
      const uint64_t home = mix((uint64_t)t[j].key) & mask;
      // move j into the hole at i when j's home is not in the cyclic range (i, j]
      const bool in_range = (i <= j) ? (home > i && home <= j) : (home > i || home <= j);
      if (!in_range) {
        t[i] = t[j];
        i = j;
      }
    }
    t[i].key = kEmpty;
  }

  void prefetch(int64_t k) const { __builtin_prefetch(&t[mix((uint64_t)k) & mask]); }

  void evict_oldest() {
    const int64_t old = ring[(size_t)head];
    const int64_t s = find(old);
    if (s >= 0) erase_slot((uint64_t)s);
    if (++head == window) head = 0;
    --count;
  }

  void insert_new(int64_t k, int64_t v) {   // k known absent (gated: and room checked)
    if (!gated && count == window) evict_oldest();
    uint64_t i = mix((uint64_t)k) & mask;
    while (t[i].key != kEmpty) i = (i + 1) & mask;
    t[i] = Slot{k, v};
    if (gated) { ++count; return; }
    int64_t tail = head + count;
    if (tail >= window) tail -= window;
    ring[(size_t)tail] = k;
    ++count;
  }
};

}  // namespace

extern "C" {

void* ccfd_dedupe_new(int64_t window) {
  if (window < 1) return nullptr;
  return new (std::nothrow) Index(window);
}

// Gated index of `capacity` keys: no automatic eviction (see Index::gated).
void* ccfd_dedupe_new_gated(int64_t capacity) {
  if (capacity < 1) return nullptr;
  return new (std::nothrow) Index(capacity, true);
}

// Count-window mode: evict the `k` oldest admitted keys.  Returns the number evicted.
int64_t ccfd_dedupe_evict(void* h, int64_t k) {
  Index* ix = static_cast<Index*>(h);
  if (!ix || k < 0 || ix->gated) return -1;
  int64_t n = 0;
  for (; n < k && ix->count > 0; ++n) ix->evict_oldest();
  return n;
}

// Gated mode: erase these keys (their offsets were committed).  Returns the number erased.
int64_t ccfd_dedupe_erase(void* h, const int64_t* keys, int64_t n) {
  Index* ix = static_cast<Index*>(h);
  if (!ix || n < 0 || (n && !keys) || !ix->gated) return -1;
  int64_t erased = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (keys[i] < 0) continue;
    const int64_t s = ix->find(keys[i]);
    if (s < 0) continue;
    ix->erase_slot((uint64_t)s);
    --ix->count;
    ++erased;
  }
  return erased;
}

void ccfd_dedupe_free(void* h) { delete static_cast<Index*>(h); }

int64_t ccfd_dedupe_size(const void* h) { return h ? static_cast<const Index*>(h)->count : -1; }

// Admit a batch.  out_ids[i]: the instance id of tx[i] (existing or new); new_keys[0..ret):
// the newly admitted keys in admission order (ids first_id, first_id + stride, ...).
// Returns the number of new keys, -1 on a bad argument (a negative tx id), or -2 (gated mode)
// when the batch could overflow the capacity: nothing was admitted.
int64_t ccfd_dedupe_assign(void* h, const int64_t* tx, int64_t n, int64_t first_id, int64_t stride,
                           int64_t* out_ids, int64_t* new_keys) {
  Index* ix = static_cast<Index*>(h);
  if (!ix || n < 0 || (n && (!tx || !out_ids || !new_keys)) || stride < 1) return -1;
  for (int64_t i = 0; i < n; ++i)
    if (tx[i] < 0) return -1;
  if (ix->gated && ix->count + n > ix->window) return -2;
  int64_t nn = 0, next = first_id;
  constexpr int64_t kAhead = 12;            // table lines in flight (a 1M window is ~64 MB)
  for (int64_t i = 0; i < n && i < kAhead; ++i) ix->prefetch(tx[i]);
  for (int64_t i = 0; i < n; ++i) {
    if (i + kAhead < n) ix->prefetch(tx[i + kAhead]);
    // the key this row (or one kAhead rows later) evicts once the window is full
    if (ix->count == ix->window) {
      int64_t e = ix->head + kAhead;
      if (e >= ix->window) e %= ix->window;
      ix->prefetch(ix->ring[(size_t)e]);
    }
    const int64_t s = ix->find(tx[i]);
    if (s >= 0) {
      out_ids[i] = ix->t[(size_t)s].val;
      continue;
    }
    ix->insert_new(tx[i], next);
    out_ids[i] = next;
    new_keys[nn++] = tx[i];
    next += stride;
  }
  return nn;
}

// Recovery: insert (key, id) pairs in admission order (a key already present keeps its id).
// A gated index refuses (-2, nothing inserted) a batch that could overflow its capacity.
int64_t ccfd_dedupe_insert(void* h, const int64_t* tx, const int64_t* ids, int64_t n) {
  Index* ix = static_cast<Index*>(h);
  if (!ix || n < 0) return -1;
  if (ix->gated && ix->count + n > ix->window) return -2;
  int64_t added = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (tx[i] < 0) return -1;
    if (ix->find(tx[i]) >= 0) continue;
    ix->insert_new(tx[i], ids[i]);
    ++added;
  }
  return added;
}

// out_ids[i] = the stored id of tx[i], or -1 when absent.
int64_t ccfd_dedupe_lookup(const void* h, const int64_t* tx, int64_t n, int64_t* out_ids) {
  const Index* ix = static_cast<const Index*>(h);
  if (!ix || n < 0) return -1;
  int64_t hits = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = tx[i] < 0 ? -1 : ix->find(tx[i]);
    out_ids[i] = s >= 0 ? ix->t[(size_t)s].val : -1;
    hits += s >= 0;
  }
  return hits;
}

}  // extern "C"
