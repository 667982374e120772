// Native RecordBatch v2 encoder for producers (ingest/kafka_wire.py encode_record_batch).
//
// The reference's producer publishes one JSON transaction per Kafka message
// (README.md:547-549); at ~1e6 messages/s per rank a Python per-record varint loop is the
// ceiling, so the batch framing is built here: n values (NULL keys, no headers) ->
// [baseOffset 0][batchLength][leaderEpoch 0][magic 2][crc32c][attributes][lastOffsetDelta]
// [first/max timestamp][producerId -1][producerEpoch -1][baseSequence -1][count][records].
#include <climits>
#include <cstdint>
#include <cstring>

extern "C" uint32_t ccfd_crc32c(const void* data, size_t n, uint32_t seed);

namespace {

inline uint8_t* put_be16(uint8_t* p, uint16_t v) { p[0] = v >> 8; p[1] = (uint8_t)v; return p + 2; }
inline uint8_t* put_be32(uint8_t* p, uint32_t v) {
  p[0] = v >> 24; p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v; return p + 4;
}
inline uint8_t* put_be64(uint8_t* p, uint64_t v) { p = put_be32(p, (uint32_t)(v >> 32)); return put_be32(p, (uint32_t)v); }

inline int varint_len(int64_t v) {
  uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
  int n = 1;
  while (z >= 0x80) { z >>= 7; ++n; }
  return n;
}
inline uint8_t* put_varint(uint8_t* p, int64_t v) {
  uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
  while (z >= 0x80) { *p++ = (uint8_t)(z | 0x80); z >>= 7; }
  *p++ = (uint8_t)z;
  return p;
}

int64_t finish_batch_impl(uint8_t* out, uint8_t* p, int64_t n, int64_t ts_ms);
// RecordBatch v2 header + CRC over the records written at out + 61 .. p
inline int64_t finish_batch(uint8_t* out, uint8_t* p, int64_t n, int64_t ts_ms) {
  return finish_batch_impl(out, p, n, ts_ms);
}

}  // namespace

extern "C" {

// Bytes needed for n values of total payload `payload` (upper bound, exact enough to size
// the output buffer: 61-byte header + per record <= 5 varints + attributes).
int64_t ccfd_kafka_batch_bound(int64_t n, int64_t payload) { return 61 + payload + n * (1 + 5 * 10); }

// values[i] = buf[off[i] .. off[i+1]); returns bytes written, or -1 on bad arguments /
// insufficient capacity.
int64_t ccfd_kafka_encode_batch(const uint8_t* buf, const int64_t* off, int64_t n, int64_t ts_ms, uint8_t* out,
                                int64_t cap) {
  if (!buf || !off || !out || n <= 0 || n > INT32_MAX || cap < 61) return -1;
  uint8_t* p = out + 61;
  uint8_t* const end = out + cap;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t vlen = off[i + 1] - off[i];
    if (vlen < 0) return -1;
    // record body: attributes, timestamp delta 0, offset delta i, key -1 (null), value, 0 headers
    const int64_t body = 1 + 1 + varint_len(i) + 1 + varint_len(vlen) + vlen + 1;
    if (end - p < varint_len(body) + body) return -1;
    p = put_varint(p, body);
    *p++ = 0;
    *p++ = 0;                                        // varint(0)
    p = put_varint(p, i);
    *p++ = 1;                                        // varint(-1): zig-zag 1
    p = put_varint(p, vlen);
    std::memcpy(p, buf + off[i], (size_t)vlen);
    p += vlen;
    *p++ = 0;
  }
  return finish_batch(out, p, n, ts_ms);
}

// The producer's hot path for the reference wire format (one JSON transaction per message,
// README.md:547-548): message i = `{"id":<id0 + i>` + tail[(start + i) % n_pool], the tails
// being pre-rendered `,"customer_id":..,"Time":..,...,"Amount":..}` bodies
// (ingest/producer.py json_tail) -- the id is formatted here, so a RecordBatch of n
// messages is built without a Python object per message.  Returns bytes written or -1.
int64_t ccfd_kafka_encode_json_batch(const uint8_t* pool, const int64_t* pool_off, int64_t n_pool, int64_t start,
                                     int64_t n, uint64_t id0, int64_t ts_ms, uint8_t* out, int64_t cap) {
  if (!pool || !pool_off || !out || n <= 0 || n > INT32_MAX || n_pool <= 0 || start < 0 || cap < 61) return -1;
  uint8_t* p = out + 61;
  uint8_t* const end = out + cap;
  char idbuf[32];
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = (start + i) % n_pool;
    const int64_t tlen = pool_off[k + 1] - pool_off[k];
    if (tlen < 0) return -1;
    // decimal id
    uint64_t v = id0 + (uint64_t)i;
    int nd = 0;
    do { idbuf[31 - nd++] = (char)('0' + v % 10); v /= 10; } while (v);
    const int64_t vlen = 6 + nd + tlen;                // {"id": + digits + tail
    const int64_t body = 1 + 1 + varint_len(i) + 1 + varint_len(vlen) + vlen + 1;
    if (end - p < varint_len(body) + body) return -1;
    p = put_varint(p, body);
    *p++ = 0;
    *p++ = 0;
    p = put_varint(p, i);
    *p++ = 1;
    p = put_varint(p, vlen);
    std::memcpy(p, "{\"id\":", 6);
    p += 6;
    std::memcpy(p, idbuf + 32 - nd, (size_t)nd);
    p += nd;
    std::memcpy(p, pool + pool_off[k], (size_t)tlen);
    p += tlen;
    *p++ = 0;
  }
  return finish_batch(out, p, n, ts_ms);
}

}  // extern "C"

namespace {
int64_t finish_batch_impl(uint8_t* out, uint8_t* p, int64_t n, int64_t ts_ms) {
  const int64_t total = p - out;
  uint8_t* h = out;
  h = put_be64(h, 0);                                // base offset (the broker assigns it)
  h = put_be32(h, (uint32_t)(total - 12));           // batch length
  h = put_be32(h, 0);                                // partition leader epoch
  *h++ = 2;                                          // magic
  uint8_t* crc_at = h;
  h += 4;
  h = put_be16(h, 0);                                // attributes: no compression, create time
  h = put_be32(h, (uint32_t)(n - 1));                // last offset delta
  h = put_be64(h, (uint64_t)ts_ms);
  h = put_be64(h, (uint64_t)ts_ms);
  h = put_be64(h, ~0ull);                            // producer id -1
  h = put_be16(h, 0xFFFF);                           // producer epoch -1
  h = put_be32(h, 0xFFFFFFFFu);                      // base sequence -1
  h = put_be32(h, (uint32_t)n);
  put_be32(crc_at, ccfd_crc32c(out + 21, (size_t)(total - 21), 0));
  return total;
}
}  // namespace
