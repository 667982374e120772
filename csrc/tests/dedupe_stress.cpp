// Randomised stress of the KIE tier's windowed dedupe index (csrc/engine/dedupe.cpp) against a
// reference model (std::unordered_map + FIFO window), built with -fsanitize by
// tests/test_native_cpu.py: batches with repeats inside a batch and across batches, keys
// re-admitted after they left the window, recovery inserts, lookups of present / evicted /
// never-seen keys, and a table that wraps many times (backward-shift deletion).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <random>
#include <unordered_map>
#include <vector>

extern "C" {
void* ccfd_dedupe_new(int64_t window);
void ccfd_dedupe_free(void* h);
int64_t ccfd_dedupe_size(const void* h);
int64_t ccfd_dedupe_assign(void* h, const int64_t* tx, int64_t n, int64_t first_id, int64_t stride,
                           int64_t* out_ids, int64_t* new_keys);
int64_t ccfd_dedupe_insert(void* h, const int64_t* tx, const int64_t* ids, int64_t n);
int64_t ccfd_dedupe_lookup(const void* h, const int64_t* tx, int64_t n, int64_t* out_ids);
}

struct Ref {
  int64_t window;
  std::unordered_map<int64_t, int64_t> map;
  std::deque<int64_t> fifo;
  void admit(int64_t k, int64_t id) {
    map[k] = id;
    fifo.push_back(k);
    while ((int64_t)fifo.size() > window) { map.erase(fifo.front()); fifo.pop_front(); }
  }
};

static int fail(const char* what, long a, long b) {
  std::fprintf(stderr, "dedupe stress FAILED: %s (%ld vs %ld)\n", what, a, b);
  return 1;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int64_t window = argc > 2 ? std::atoll(argv[2]) : 1000;
  std::mt19937_64 rng(42);
  void* h = ccfd_dedupe_new(window);
  if (!h) return fail("new", 0, 0);
  Ref ref{window, {}, {}};
  int64_t next_id = 7;
  const int64_t stride = 3;
  std::vector<int64_t> tx, out, nk, look;
  for (int r = 0; r < rounds; ++r) {
    const int n = (int)(rng() % 300) + 1;
    tx.resize(n); out.resize(n); nk.resize(n); look.resize(n);
    const int64_t span = (rng() % 4 == 0) ? 50 : 20 * window;     // dense batches repeat a lot
    for (int i = 0; i < n; ++i) tx[i] = (int64_t)(rng() % span) + (r % 7 == 0 ? 0 : r * 13);
    if (r % 11 == 0) {                                             // recovery: insert given ids
      for (int i = 0; i < n; ++i) out[i] = 1000000 + i;
      ccfd_dedupe_insert(h, tx.data(), out.data(), n);
      for (int i = 0; i < n; ++i) if (!ref.map.count(tx[i])) ref.admit(tx[i], out[i]);
    } else {
      const int64_t k = ccfd_dedupe_assign(h, tx.data(), n, next_id, stride, out.data(), nk.data());
      int64_t expect_new = 0;
      for (int i = 0; i < n; ++i) {
        auto it = ref.map.find(tx[i]);
        int64_t id;
        if (it != ref.map.end()) {
          id = it->second;
        } else {
          id = next_id + expect_new * stride;
          if (nk[expect_new] != tx[i]) return fail("new key order", (long)nk[expect_new], (long)tx[i]);
          ++expect_new;
          ref.admit(tx[i], id);
        }
        if (out[i] != id) return fail("assigned id", (long)out[i], (long)id);
      }
      if (k != expect_new) return fail("new count", (long)k, (long)expect_new);
      next_id += k * stride;
    }
    if (ccfd_dedupe_size(h) != (int64_t)ref.map.size()) return fail("size", (long)ccfd_dedupe_size(h), (long)ref.map.size());
    for (int i = 0; i < n; ++i) tx[i] = (int64_t)(rng() % (30 * window));
    ccfd_dedupe_lookup(h, tx.data(), n, look.data());
    for (int i = 0; i < n; ++i) {
      auto it = ref.map.find(tx[i]);
      const int64_t want = it == ref.map.end() ? -1 : it->second;
      if (look[i] != want) return fail("lookup", (long)look[i], (long)want);
    }
  }
  int64_t neg = -5;
  if (ccfd_dedupe_assign(h, &neg, 1, 0, 1, out.data(), nk.data()) != -1) return fail("negative key", 0, 0);
  ccfd_dedupe_free(h);
  std::printf("dedupe stress ok\n");
  return 0;
}
