// CRC-32C (Castagnoli) for Kafka RecordBatch v2 framing (ingest/kafka_wire.py).
// SSE4.2 `crc32` instruction, 8 bytes per step; table fallback for CPUs without it.
#include <cstddef>
#include <cstdint>
#include <cstring>

#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

namespace {

uint32_t table[256];
bool table_ready = false;

void init_table() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    table[i] = c;
  }
  table_ready = true;
}

uint32_t crc_table(uint32_t crc, const uint8_t* p, size_t n) {
  if (!table_ready) init_table();
  for (size_t i = 0; i < n; ++i) crc = table[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
  return crc;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32;
}
#endif

}  // namespace

extern "C" uint32_t ccfd_crc32c(const void* data, size_t n, uint32_t seed) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t crc = ~seed;
#if defined(__x86_64__)
  if (__builtin_cpu_supports("sse4.2")) return ~crc_hw(crc, p, n);
#endif
  return ~crc_table(crc, p, n);
}
