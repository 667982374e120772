"""Kafka wire protocol (subset) -- client side, no third-party Kafka library.

The reference's services talk to a Strimzi Kafka cluster at ``BROKER_URL``
(``odh-message-bus-kafka-brokers:9092``, deploy/router.yaml:55-56).  There is no Kafka
client in this image, so the framework speaks the protocol itself:

  ApiVersions v0, Metadata v1, Produce v3, Fetch v4, ListOffsets v1, FindCoordinator v0,
  OffsetCommit v2, OffsetFetch v1, CreateTopics v0   (all non-flexible encodings)

Records use RecordBatch v2 (magic 2) with CRC-32C computed by the native library
(csrc/engine/crc32c.cpp, SSE4.2) or a table fallback; gzip-compressed batches (codec 1)
are decoded and can be produced, other codecs are refused explicitly.  ``KafkaBroker``
exposes the same interface as ``InProcBroker`` (produce / fetch / offsets / commit /
consumer), so every service runs unchanged against either.  It takes a comma-separated
bootstrap list, routes Produce / Fetch / ListOffsets to each partition's leader from
Metadata, and on NOT_LEADER / UNKNOWN_TOPIC_OR_PARTITION / LEADER_NOT_AVAILABLE or a dead
connection refreshes metadata and retries (leader moves and broker failover); offsets are
committed to the group coordinator (FindCoordinator).  Static consumers (``consumer``) use
the engine's ``p % world == rank`` sharding; group membership (JoinGroup / SyncGroup /
Heartbeat) lives in ``kafka_group.py``.
"""
from __future__ import annotations

import collections
import itertools
import socket
import struct
import threading
import time
import zlib
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from .broker import BrokerError, Record

# --------------------------------------------------------------------------- api keys
PRODUCE, FETCH, LIST_OFFSETS, METADATA, OFFSET_COMMIT, OFFSET_FETCH, FIND_COORDINATOR = 0, 1, 2, 3, 8, 9, 10
API_VERSIONS, CREATE_TOPICS, INIT_PRODUCER_ID = 18, 19, 22
JOIN_GROUP, HEARTBEAT, LEAVE_GROUP, SYNC_GROUP = 11, 12, 13, 14       # ingest/kafka_group.py
SUPPORTED = {PRODUCE: 3, FETCH: 4, LIST_OFFSETS: 1, METADATA: 1, OFFSET_COMMIT: 2, OFFSET_FETCH: 1,
             FIND_COORDINATOR: 0, API_VERSIONS: 0, CREATE_TOPICS: 0,
             JOIN_GROUP: 1, HEARTBEAT: 0, LEAVE_GROUP: 0, SYNC_GROUP: 0, INIT_PRODUCER_ID: 0}

ERR_NONE, ERR_OFFSET_OUT_OF_RANGE, ERR_UNKNOWN_TOPIC, ERR_CORRUPT = 0, 1, 3, 2
ERR_LEADER_NOT_AVAILABLE, ERR_NOT_LEADER, ERR_NOT_COORDINATOR = 5, 6, 16
RETRIABLE = (ERR_UNKNOWN_TOPIC, ERR_LEADER_NOT_AVAILABLE, ERR_NOT_LEADER, ERR_NOT_COORDINATOR)
ERR_UNSUPPORTED_VERSION, ERR_TOPIC_EXISTS, ERR_INVALID_REQUEST = 35, 36, 42
ERR_OUT_OF_ORDER_SEQUENCE = 45
# idempotent-producer sequence numbers are int32 and wrap from 2^31 - 1 to 0 (Kafka semantics)
SEQ_MASK = 0x7FFFFFFF

# --------------------------------------------------------------------------- crc32c
_CRC_TABLE = None


def _crc32c_py(data: bytes, crc: int = 0) -> int:
    global _CRC_TABLE
    if _CRC_TABLE is None:
        t = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
            t.append(c)
        _CRC_TABLE = t
    crc ^= 0xFFFFFFFF
    for b in data:
        crc = _CRC_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def _codec_lib():
    """The host-only codec library (ops/_hostlib.py: no HIP runtime, no GPU); the engine
    library as a fallback where the host one cannot be built."""
    try:
        from ..ops._hostlib import hostlib
        return hostlib()
    except Exception:
        from ..ops._lib import lib
        return lib()


_native_crc = None


def crc32c(data: bytes) -> int:
    global _native_crc
    if _native_crc is None:
        try:
            import ctypes as C
            f = _codec_lib().ccfd_crc32c
            f.argtypes = [C.c_char_p, C.c_size_t, C.c_uint32]
            f.restype = C.c_uint32
            _native_crc = f
        except Exception:
            _native_crc = False
    if _native_crc:
        if isinstance(data, memoryview) and not data.readonly and data.contiguous:
            import ctypes as C                    # zero-copy: a writable buffer's address
            n = data.nbytes
            buf = (C.c_char * n).from_buffer(data)
            try:
                return int(_native_crc(C.cast(buf, C.c_char_p), n, 0))
            finally:
                del buf
        return int(_native_crc(bytes(data), len(data), 0))
    return _crc32c_py(data)


def warm_native() -> float:
    """Load the native CRC-32C / RecordBatch codecs now (seconds taken).  They used to be
    loaded from the engine's library, whose first load also brings up the HIP runtime (~0.3 s
    with the GIL held): a service that loaded it lazily on its first produce stalled its event
    loop right when traffic began -- the KIE server's 270-450 ms event-loop lag at the start of
    every deployed run, the whole scored -> process-started p99 (profiles/r4/kie_handoff/).
    They now come from the host-only library (ops/_hostlib.py); services still load it before
    they start serving."""
    t0 = time.perf_counter()
    crc32c(b"ccfd")
    _native_encoder()
    return time.perf_counter() - t0


# --------------------------------------------------------------------------- primitives
class Writer:
    __slots__ = ("parts",)

    def __init__(self):
        self.parts: List[bytes] = []

    def i8(self, v):
        self.parts.append(struct.pack(">b", v)); return self

    def i16(self, v):
        self.parts.append(struct.pack(">h", v)); return self

    def i32(self, v):
        self.parts.append(struct.pack(">i", v)); return self

    def u32(self, v):
        self.parts.append(struct.pack(">I", v)); return self

    def i64(self, v):
        self.parts.append(struct.pack(">q", v)); return self

    def string(self, s: Optional[str]):
        if s is None:
            return self.i16(-1)
        b = s.encode()
        self.i16(len(b)); self.parts.append(b); return self

    def bytes_(self, b: Optional[bytes]):
        if b is None:
            return self.i32(-1)
        self.i32(len(b)); self.parts.append(bytes(b)); return self

    def array(self, items, fn):
        if items is None:
            return self.i32(-1)
        items = list(items)
        self.i32(len(items))
        for it in items:
            fn(self, it)
        return self

    def raw(self, b: bytes):
        self.parts.append(b); return self

    def build(self) -> bytes:
        return b"".join(self.parts)


class Reader:
    __slots__ = ("b", "o")

    def __init__(self, b: bytes, o: int = 0):
        self.b = memoryview(b)
        self.o = o

    def _u(self, fmt, n):
        v = struct.unpack_from(fmt, self.b, self.o)[0]
        self.o += n
        return v

    def i8(self): return self._u(">b", 1)
    def i16(self): return self._u(">h", 2)
    def i32(self): return self._u(">i", 4)
    def u32(self): return self._u(">I", 4)
    def i64(self): return self._u(">q", 8)

    def string(self) -> Optional[str]:
        n = self.i16()
        if n < 0:
            return None
        s = bytes(self.b[self.o:self.o + n]).decode()
        self.o += n
        return s

    def bytes_(self) -> Optional[bytes]:
        n = self.i32()
        if n < 0:
            return None
        v = bytes(self.b[self.o:self.o + n])
        self.o += n
        return v

    def view_(self) -> Optional[memoryview]:
        """Like ``bytes_`` without the copy: a view into the request buffer, valid only while
        the request is being handled (kafka-lite copies a produce request's batches once,
        into its log)."""
        n = self.i32()
        if n < 0:
            return None
        v = self.b[self.o:self.o + n]
        self.o += n
        return v

    def array(self, fn) -> Optional[list]:
        n = self.i32()
        if n < 0:
            return None
        return [fn(self) for _ in range(n)]

    def remaining(self) -> int:
        return len(self.b) - self.o


def _zigzag(v: int) -> int:
    return (v << 1) ^ (v >> 63)


def _varint(v: int) -> bytes:
    v = _zigzag(v) & 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    while True:
        if v < 0x80:
            out.append(v)
            return bytes(out)
        out.append((v & 0x7F) | 0x80)
        v >>= 7


def _read_varint(mv, o: int) -> Tuple[int, int]:
    shift = 0
    v = 0
    while True:
        b = mv[o]
        o += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            break
        shift += 7
    return (v >> 1) ^ -(v & 1), o


# --------------------------------------------------------------------------- RecordBatch v2
CODEC_NONE, CODEC_GZIP = 0, 1
_CODEC_NAMES = {1: "gzip", 2: "snappy", 3: "lz4", 4: "zstd"}


_native_enc = None


def _native_encoder():
    global _native_enc
    if _native_enc is None:
        try:
            import ctypes as C
            L = _codec_lib()
            L.ccfd_kafka_encode_batch.argtypes = [C.c_char_p, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_int64]
            L.ccfd_kafka_encode_batch.restype = C.c_int64
            L.ccfd_kafka_batch_bound.argtypes = [C.c_int64, C.c_int64]
            L.ccfd_kafka_batch_bound.restype = C.c_int64
            _native_enc = L
        except Exception:
            _native_enc = False
    return _native_enc


def encode_record_batch(values: Sequence[bytes], keys: Optional[Sequence[Optional[bytes]]] = None,
                        base_offset: int = 0, timestamp_ms: Optional[int] = None,
                        compression: int = CODEC_NONE) -> bytes:
    ts = int(time.time() * 1000) if timestamp_ms is None else timestamp_ms
    n = len(values)
    if (n >= 8 and compression == CODEC_NONE and base_offset == 0 and (keys is None or all(k is None for k in keys))
            and all(v is not None for v in values)):
        L = _native_encoder()
        if L:                                   # native framing (csrc/engine/kafka_codec.cpp)
            import numpy as np
            buf = b"".join(values)
            off = np.zeros(n + 1, np.int64)
            np.cumsum([len(v) for v in values], out=off[1:])
            out = bytearray(L.ccfd_kafka_batch_bound(n, len(buf)))
            import ctypes as C
            ob = (C.c_char * len(out)).from_buffer(out)
            k = L.ccfd_kafka_encode_batch(buf, off.ctypes.data, n, ts, C.addressof(ob), len(out))
            if k > 0:
                del ob
                del out[k:]                       # a bytearray: producers stamp it in place
                return out
    recs = []
    for i, v in enumerate(values):
        k = keys[i] if keys is not None else None
        body = b"".join([b"\x00", _varint(0), _varint(i),
                         _varint(-1) if k is None else _varint(len(k)) + k,
                         _varint(-1) if v is None else _varint(len(v)) + bytes(v), _varint(0)])
        recs.append(_varint(len(body)) + body)
    n = len(values)
    records = b"".join(recs)
    if compression == CODEC_GZIP:
        import gzip
        records = gzip.compress(records, compresslevel=1)
    elif compression != CODEC_NONE:
        raise BrokerError(f"unsupported compression codec {compression}")
    after_crc = struct.pack(">hiqqqhii", compression, max(n - 1, 0), ts, ts, -1, -1, -1, n) + records
    crc = crc32c(after_crc)
    head = struct.pack(">ibI", 0, 2, crc)                 # partitionLeaderEpoch, magic, crc
    batch_len = len(head) + len(after_crc)
    out = bytearray(struct.pack(">qi", base_offset, batch_len))   # mutable: stamped in place by
    out += head                                                    # idempotent producers
    out += after_crc
    return out


PRODUCE_TS_HEADER = b"ccfd-ts"          # record header: producer send time, u64 BE ns (CLOCK_REALTIME)


def with_produce_time(record_set, ts_ns: int) -> bytearray:
    """``record_set`` with a ``ccfd-ts`` header (the send time, ns since the epoch) added to the
    FIRST record of every uncompressed batch -- the origin stamp behind the engine's
    produce -> scored latency (csrc/engine/kafka_consumer.cpp reads it).  Batch lengths are
    fixed up; CRCs are NOT (the caller re-seals them, see ``seal_batches``)."""
    src = memoryview(record_set)
    out = bytearray()
    o = 0
    hdr = _varint(len(PRODUCE_TS_HEADER)) + PRODUCE_TS_HEADER + _varint(8) + struct.pack(">Q", ts_ns)
    while o + 61 <= len(src):
        blen = struct.unpack_from(">i", src, o + 8)[0]
        end = o + 12 + blen
        attrs, count = struct.unpack_from(">h", src, o + 21)[0], struct.unpack_from(">i", src, o + 57)[0]
        if attrs & 0x7 or count <= 0:                       # compressed / empty: left as it is
            out += src[o:end]
            o = end
            continue
        q = o + 61
        rlen, q1 = _read_varint(src, q)
        rend = q1 + rlen
        p = q1 + 1                                          # attributes
        for _ in range(3):                                  # timestamp delta, offset delta, key length
            v, p = _read_varint(src, p)
        if v > 0:
            p += v
        vl, p = _read_varint(src, p)
        p += max(vl, 0)
        hc, ph = _read_varint(src, p)                       # header count
        body = bytes(src[q1:p]) + _varint(hc + 1) + bytes(src[ph:rend]) + hdr
        first = _varint(len(body)) + body
        start = len(out)
        out += src[o:o + 61]
        out += first
        out += src[rend:end]
        struct.pack_into(">i", out, start + 8, len(out) - start - 12)
        o = end
    return out


def seal_batches(b: bytearray) -> None:
    """Recompute the CRC-32C of every batch of ``b`` in place."""
    mv = memoryview(b)
    o = 0
    while o + 61 <= len(b):
        blen = struct.unpack_from(">i", b, o + 8)[0]
        struct.pack_into(">I", b, o + 17, crc32c(mv[o + 21:o + 12 + blen]))
        o += 12 + blen
    del mv


def decode_record_batches(data: bytes, topic: str = "", partition: int = 0,
                          verify_crc: bool = True) -> List[Record]:
    out: List[Record] = []
    mv = memoryview(data)
    o = 0
    while o + 12 <= len(data):
        base_offset, batch_len = struct.unpack_from(">qi", mv, o)
        end = o + 12 + batch_len
        if end > len(data):
            break                                          # partial batch at the end of a fetch
        _epoch, magic, crc = struct.unpack_from(">ibI", mv, o + 12)
        if magic != 2:
            raise BrokerError(f"unsupported record batch magic {magic}")
        body = mv[o + 21:end]
        if verify_crc and crc32c(bytes(body)) != crc:
            raise BrokerError("record batch CRC mismatch")
        (attrs, _lod, base_ts, _max_ts, _pid, _pep, _bseq, count) = struct.unpack_from(">hiqqqhii", body, 0)
        codec = attrs & 0x7
        q = o + 61                                         # first record
        rmv = mv
        if codec == CODEC_GZIP:
            rmv = memoryview(zlib.decompress(bytes(mv[q:end]), 47))   # gzip or zlib header
            q = 0
        elif codec:
            raise BrokerError(f"unsupported compression codec {_CODEC_NAMES.get(codec, codec)}")
        mv_outer, mv = mv, rmv
        for _ in range(count):
            ln, q = _read_varint(mv, q)
            rend = q + ln
            q += 1                                         # record attributes
            tsd, q = _read_varint(mv, q)
            od, q = _read_varint(mv, q)
            kl, q = _read_varint(mv, q)
            key = None if kl < 0 else bytes(mv[q:q + kl])
            q += max(kl, 0)
            vl, q = _read_varint(mv, q)
            val = None if vl < 0 else bytes(mv[q:q + vl])
            q += max(vl, 0)
            hdrs = ()
            hc, q = _read_varint(mv, q)
            if hc > 0:
                hl = []
                for _h in range(hc):
                    hk, q = _read_varint(mv, q)
                    k_ = bytes(mv[q:q + hk]).decode("utf-8", "replace")
                    q += hk
                    hv, q = _read_varint(mv, q)
                    hl.append((k_, None if hv < 0 else bytes(mv[q:q + hv])))
                    q += max(hv, 0)
                hdrs = tuple(hl)
            q = rend
            out.append(Record(topic, partition, base_offset + od, key, val, (base_ts + tsd) / 1000.0, hdrs))
        mv = mv_outer
        o = end
    return out


# --------------------------------------------------------------------------- framing
def encode_request(api_key: int, version: int, corr: int, client_id: str, body: bytes) -> bytes:
    hdr = Writer().i16(api_key).i16(version).i32(corr).string(client_id).build()
    msg = hdr + body
    return struct.pack(">i", len(msg)) + msg


def _sendall_parts(sock: socket.socket, parts: Sequence) -> None:
    """sendall over a list of buffers without joining them (scatter-gather ``sendmsg``): a
    produce request's RecordBatch goes to the socket straight from where it was encoded."""
    views = [memoryview(p).cast("B") for p in parts if len(p)]
    while views:
        n = sock.sendmsg(views[:64])
        while n:
            if n >= len(views[0]):
                n -= len(views[0])
                views.pop(0)
            else:
                views[0] = views[0][n:]
                n = 0


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("kafka connection closed")
        buf += chunk
    return bytes(buf)


class Connection:
    def __init__(self, host: str, port: int, client_id: str = "ccfd-mi355x", timeout: float = 10.0,
                 connect_wait_s: float = 0.0):
        """``connect_wait_s``: keep retrying a refused connection this long (services start in
        any order, like pods waiting for the broker)."""
        deadline = time.monotonic() + connect_wait_s
        while True:
            try:
                self.sock = socket.create_connection((host, port), timeout=timeout)
                break
            except (ConnectionRefusedError, socket.timeout, OSError):
                if time.monotonic() >= deadline:
                    raise
                time.sleep(0.25)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.client_id = client_id
        self._corr = itertools.count(1)
        self._lock = threading.Lock()

    def request(self, api_key: int, version: int, body) -> Reader:
        """``body``: bytes, or a list of buffers sent as they are (no concatenation)."""
        with self._lock:
            corr = self._send(api_key, version, body)
            return self._recv(corr)

    def _send(self, api_key: int, version: int, body) -> int:
        corr = next(self._corr)
        if isinstance(body, list):
            hdr = Writer().i16(api_key).i16(version).i32(corr).string(self.client_id).build()
            n = len(hdr) + sum(len(b) for b in body)
            _sendall_parts(self.sock, [struct.pack(">i", n) + hdr] + body)
        else:
            self.sock.sendall(encode_request(api_key, version, corr, self.client_id, body))
        return corr

    def _recv(self, corr: int) -> Reader:
        size = struct.unpack(">i", _recv_exact(self.sock, 4))[0]
        r = Reader(_recv_exact(self.sock, size))
        got = r.i32()
        if got != corr:
            raise BrokerError(f"correlation id mismatch {got} != {corr}")
        return r

    # pipelining (one owner thread): requests sent back to back, answered in order
    def send(self, api_key: int, version: int, body) -> int:
        with self._lock:
            return self._send(api_key, version, body)

    def recv(self, corr: int) -> Reader:
        with self._lock:
            return self._recv(corr)

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass


# --------------------------------------------------------------------------- client
class KafkaBroker:
    """Kafka-protocol implementation of the InProcBroker interface.  ``bootstrap`` is
    ``host:port[,host:port...]``; partition leaders come from Metadata and are connected
    lazily; leader moves and broker failures are recovered by refresh + retry."""

    RETRIES = 8

    def __init__(self, bootstrap: str, client_id: str = "ccfd-mi355x", timeout: float = 10.0,
                 connect_wait_s: float = 0.0, compression: int = CODEC_NONE, idempotent: bool = False):
        """``idempotent``: Kafka's idempotent producer -- InitProducerId once, then every
        produced batch carries (producer id, epoch, base sequence per partition), so a batch
        re-sent after a lost ack or a broker restart is stored once (the broker answers a
        duplicate with its original offset)."""
        self.idempotent = bool(idempotent)
        # stamp_time: the ccfd-ts send-time header on the first record of every batch (the
        # engine's produce -> scored latency); set by the transaction producer
        self.stamp_time = False
        self.stamp_every = 8                # every 8th batch: a sampled latency, a fraction of the copies
        self._stamp_n: Dict[Tuple[str, int], int] = {}
        self._pid: Optional[Tuple[int, int]] = None
        self._seq: Dict[Tuple[str, int], int] = {}
        self._seq_locks: Dict[Tuple[str, int], threading.Lock] = {}
        self._seq_guard = threading.Lock()
        self.timeout = timeout
        self.client_id = client_id
        self.compression = compression
        self._seeds = [(h, int(pt)) for h, pt in (x.strip().rsplit(":", 1) for x in bootstrap.split(",") if x.strip())]
        self._bootstrap = self._seeds[0]
        self._conns: Dict[int, Connection] = {}
        self._nodes: Dict[int, Tuple[str, int]] = {}
        self._leaders: Dict[Tuple[str, int], int] = {}
        self._partitions: Dict[str, int] = {}
        self._coord: Dict[str, int] = {}
        # produce defaults: acks (1 = leader, -1 = all in-sync replicas) and the requests kept in
        # flight per producer (max.in.flight; > 1 pipelines produce_raw, flush() drains)
        self.default_acks = 1
        self.max_in_flight = 1
        self._pconns: Dict[int, Connection] = {}
        self._inflight: "collections.deque" = collections.deque()
        self.connect_wait_s = float(connect_wait_s)
        self._boot = self._connect_any(connect_wait_s)
        self._rr = itertools.count()
        self.retries_done = 0                               # refresh-and-retry count (tests, metrics)
        self.api_versions = self._api_versions()

    def _connect_any(self, wait_s: float = 0.0) -> Connection:
        cands = self._seeds + [a for a in self._nodes.values() if a not in self._seeds]
        deadline = time.monotonic() + wait_s
        while True:
            for host, port in cands:
                try:
                    return Connection(host, port, self.client_id, self.timeout)
                except OSError:
                    continue
            if time.monotonic() >= deadline:
                raise BrokerError(f"no reachable broker in {cands}")
            time.sleep(0.25)

    def _boot_request(self, api: int, ver: int, body: bytes) -> Reader:
        # a broker that dies (or is being killed) right as we reconnect to it resets the new
        # connection too: try a few bootstrap connections before giving up
        for attempt in range(4):
            try:
                return self._boot.request(api, ver, body)
            except (OSError, ConnectionError):
                self._boot.close()
                if attempt == 3:
                    raise
                time.sleep(0.05 * attempt)
                self._boot = self._connect_any(self.timeout)
        raise AssertionError("unreachable")

    def _api_versions(self) -> Dict[int, Tuple[int, int]]:
        r = self._boot_request(API_VERSIONS, 0, b"")
        err = r.i16()
        if err:
            raise BrokerError(f"ApiVersions error {err}")
        return {k: (lo, hi) for k, lo, hi in r.array(lambda x: (x.i16(), x.i16(), x.i16()))}

    def _conn(self, node: int) -> Connection:
        if node not in self._conns:
            if node not in self._nodes:
                raise BrokerError(f"unknown broker node {node}")
            self._conns[node] = Connection(*self._nodes[node], self.client_id, self.timeout)
        return self._conns[node]

    def _drop(self, node: int) -> None:
        c = self._conns.pop(node, None)
        if c is not None:
            c.close()

    def metadata(self, topics: Optional[Sequence[str]] = None) -> Dict[str, int]:
        body = Writer().array(topics, lambda w, t: w.string(t)).build()
        r = self._boot_request(METADATA, 1, body)
        brokers = r.array(lambda x: (x.i32(), x.string(), x.i32(), x.string()))
        nodes = {nid: (host, port) for nid, host, port, _rack in brokers}
        for nid in list(self._conns):
            if nodes.get(nid) != self._nodes.get(nid):
                self._drop(nid)                             # broker gone or moved
        self._nodes = nodes
        r.i32()                                             # controller id

        def part(x):
            return x.i16(), x.i32(), x.i32(), x.array(lambda y: y.i32()), x.array(lambda y: y.i32())
        out = {}
        for err, name, _internal, parts in r.array(lambda x: (x.i16(), x.string(), x.i8(), x.array(part))):
            if err:
                continue
            out[name] = len(parts)
            self._partitions[name] = len(parts)
            for _e, idx, leader, _rep, _isr in parts:
                self._leaders[(name, idx)] = leader
        return out

    def create_topic(self, name: str, partitions: Optional[int] = None) -> None:
        if name in self._partitions or name in self.metadata([name]):
            return
        body = (Writer().array([name], lambda w, t: w.string(t).i32(partitions or 1).i16(1)
                               .array([], None).array([], None)).i32(int(self.timeout * 1000)).build())
        # a replicated cluster creates topics once every broker has registered: LEADER_NOT_AVAILABLE
        # until then, retried for up to connect_wait_s (at least 30 s)
        t_end = time.monotonic() + max(30.0, self.connect_wait_s)
        while True:
            r = self._boot_request(CREATE_TOPICS, 0, body)
            errs = r.array(lambda x: (x.string(), x.i16()))
            if not any(err == ERR_LEADER_NOT_AVAILABLE for _t, err in errs) or time.monotonic() > t_end:
                break
            time.sleep(0.2)
        for tname, err in errs:
            if err not in (ERR_NONE, ERR_TOPIC_EXISTS):
                raise BrokerError(f"CreateTopics {tname}: error {err}")
        self.metadata([name])

    def partitions(self, topic: str) -> int:
        if topic not in self._partitions:
            self.metadata([topic])
        if topic not in self._partitions:
            self.create_topic(topic)
        return self._partitions[topic]

    def leader_of(self, topic: str, partition: int) -> int:
        if (topic, partition) not in self._leaders:
            self.metadata([topic])
        return self._leaders.get((topic, partition), -1)

    def _on_leader(self, topic: str, partition: int, api: int, ver: int, body: bytes, parse):
        """Send to the partition leader; ``parse(reader) -> (error code, result)``.  Retriable
        errors and dead connections refresh metadata and retry with back-off."""
        last = None
        for attempt in range(self.RETRIES):
            node = self.leader_of(topic, partition)
            try:
                if node < 0:
                    raise BrokerError(f"{topic}[{partition}] has no leader")
                err, res = parse(self._conn(node).request(api, ver, body))
            except (OSError, ConnectionError, BrokerError) as e:
                last = e
                self._drop(node)
                err = ERR_LEADER_NOT_AVAILABLE
            if err not in RETRIABLE:
                if err:
                    raise BrokerError(f"{topic}[{partition}] api {api} error {err}")
                return res
            self.retries_done += 1
            self._leaders.pop((topic, partition), None)
            time.sleep(min(0.5, 0.01 * (2 ** attempt)))
            try:
                self.metadata([topic])
            except (OSError, ConnectionError, BrokerError) as e:
                last = e
        raise BrokerError(f"{topic}[{partition}]: leader not reachable after {self.RETRIES} tries ({last})")

    # ---------------------------------------------------------------- produce
    def produce_batch(self, topic: str, partition: int, values: Sequence[bytes],
                      keys: Optional[Sequence[Optional[bytes]]] = None, acks: Optional[int] = None) -> int:
        rb = encode_record_batch(values, keys, compression=self.compression)
        return self.produce_raw(topic, partition, rb, acks)

    def init_producer_id(self) -> Tuple[int, int]:
        """InitProducerId v0 (no transactional id): (producer id, epoch)."""
        body = Writer().string(None).i32(60000).build()
        r = self._boot_request(INIT_PRODUCER_ID, 0, body)
        r.i32()                                             # throttle
        err, pid, epoch = r.i16(), r.i64(), r.i16()
        if err:
            raise BrokerError(f"InitProducerId error {err}")
        return pid, epoch

    def _stamp_sequence(self, topic: str, partition: int, b: bytearray) -> int:
        """Write (producer id, epoch, base sequence) into every batch of ``b`` (in place, CRC
        not re-sealed); returns the records in it."""
        if self._pid is None:
            self._pid = self.init_producer_id()
        pid, epoch = self._pid
        seq = self._seq.get((topic, partition), 0)
        o = n_total = 0
        while o + 61 <= len(b):
            blen = struct.unpack_from(">i", b, o + 8)[0]
            count = struct.unpack_from(">i", b, o + 57)[0]
            struct.pack_into(">qhi", b, o + 43, pid, epoch, seq)
            seq = (seq + count) & SEQ_MASK        # wraps at 2^31 like Kafka's sequences
            n_total += count
            o += 12 + blen
        return n_total

    def produce_raw(self, topic: str, partition: int, record_set: bytes, acks: Optional[int] = None) -> int:
        """Produce an already encoded RecordBatch (e.g. from the native encoder).  With
        ``max_in_flight`` > 1 the request is pipelined: it returns -1 (the base offset arrives
        later) and ``flush()`` waits for every answer."""
        acks = self.default_acks if acks is None else acks
        stamp = False
        if self.stamp_time:                 # a sample of the batches carries its send time:
            # every stamp_every-th batch OF EACH PARTITION -- one counter over round-robin
            # partitions stamped only partition 0 when stamp_every divided their count, so
            # the ranks owning the other partitions never saw a sample
            k = self._stamp_n.get((topic, partition), 0)
            stamp = k % max(1, self.stamp_every) == 0
            self._stamp_n[(topic, partition)] = k + 1
        if not (self.idempotent or stamp):
            return self._produce_send(topic, partition, record_set, acks)
        # at most one copy: the send-time header splice, else a bytearray from the encoders is
        # stamped in place (anything immutable is copied once); sequence stamps; one seal
        if stamp:
            b = with_produce_time(record_set, time.time_ns())
        elif isinstance(record_set, bytearray):
            b = record_set
        else:
            b = bytearray(record_set)
        if not self.idempotent:
            seal_batches(b)
            return self._produce_send(topic, partition, b, acks)
        key = (topic, partition)
        with self._seq_guard:
            lk = self._seq_locks.setdefault(key, threading.Lock())
        with lk:                         # sequence order == send order on a partition
            n = self._stamp_sequence(topic, partition, b)
            seal_batches(b)
            if self.max_in_flight > 1:   # the sequence advances at send: answers come in order
                self._seq[key] = (self._seq.get(key, 0) + n) & SEQ_MASK
                return self._produce_send(topic, partition, b, acks)
            base = self._produce_raw(topic, partition, b, acks)   # retries resend the same seq
            self._seq[key] = (self._seq.get(key, 0) + n) & SEQ_MASK
            return base

    # ---------------------------------------------------------------- pipelined produce
    def _produce_send(self, topic: str, partition: int, record_set, acks: int) -> int:
        if self.max_in_flight <= 1:
            return self._produce_raw(topic, partition, record_set, acks)
        # at most one request in flight PER PARTITION (answers of the previous one first): a
        # refused batch can then never be overtaken by a later one of the same partition that a
        # broker without the producer's state would accept out of order
        while any(e[3] == topic and e[4] == partition for e in self._inflight):
            self._complete_one()
        head = (Writer().string(None).i16(acks).i32(int(self.timeout * 1000)).i32(1).string(topic)
                .i32(1).i32(partition).i32(len(record_set)).build())
        node = self.leader_of(topic, partition)
        try:
            if node < 0:
                raise BrokerError(f"{topic}[{partition}] has no leader")
            c = self._pconns.get(node)
            if c is None:
                c = self._pconns[node] = Connection(*self._nodes[node], self.client_id, self.timeout)
            corr = c.send(PRODUCE, 3, [head, record_set])
        except (OSError, ConnectionError, BrokerError, KeyError):
            self._drop_pipe(node)
            c, corr = None, -1
        self._inflight.append((node, c, corr, topic, partition, record_set, acks))
        while len(self._inflight) >= self.max_in_flight:
            self._complete_one()
        return -1

    def _drop_pipe(self, node: int) -> None:
        c = self._pconns.pop(node, None)
        if c is not None:
            c.close()

    def _complete_one(self) -> None:
        node, c, corr, topic, partition, rs, acks = self._inflight.popleft()
        err = ERR_LEADER_NOT_AVAILABLE
        if c is not None and self._pconns.get(node) is c:
            try:
                r = c.recv(corr)
                resp = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i16(), y.i64(), y.i64()))))
                err = resp[0][1][0][1]
            except (OSError, ConnectionError, BrokerError):
                self._drop_pipe(node)
        if err == ERR_NONE:
            return
        if err not in RETRIABLE + (ERR_OUT_OF_ORDER_SEQUENCE,):
            raise BrokerError(f"{topic}[{partition}] produce error {err}")
        # the leader moved or died: this batch and every later one in flight to it failed (or
        # were refused as out of order); they are re-sent, in order, on the synchronous path --
        # the same sequence numbers, so whatever the old leader did store is not stored twice
        self._leaders.pop((topic, partition), None)
        self._produce_raw(topic, partition, rs, acks)

    def flush(self) -> None:
        """Wait for every pipelined produce's answer (re-sending what failed)."""
        while self._inflight:
            self._complete_one()

    def _produce_raw(self, topic: str, partition: int, record_set: bytes, acks: Optional[int] = None) -> int:
        acks = self.default_acks if acks is None else acks
        # [acks, timeout, 1 topic, 1 partition, record set size] + the record set itself, sent
        # without copying it into the request (Connection.request scatter-gather)
        head = (Writer().string(None).i16(acks).i32(int(self.timeout * 1000)).i32(1).string(topic)
                .i32(1).i32(partition).i32(len(record_set)).build())
        body = [head, record_set]

        def parse(r):
            resp = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i16(), y.i64(), y.i64()))))
            _p, err, base, _ts = resp[0][1][0]
            return err, base
        return self._on_leader(topic, partition, PRODUCE, 3, body, parse)

    def produce(self, topic: str, value: bytes, key: Optional[bytes] = None, partition: Optional[int] = None,
                headers: Tuple = ()) -> Tuple[int, int]:
        n = self.partitions(topic)
        if partition is None:
            partition = (zlib.crc32(key) % n) if key is not None else next(self._rr) % n
        return partition, self.produce_batch(topic, partition, [value], [key])

    def produce_many(self, topic: str, values: Iterable[bytes], partition: Optional[int] = None) -> int:
        vals = list(values)
        if partition is None:
            n = self.partitions(topic)
            by: Dict[int, List[bytes]] = {}
            for v in vals:
                by.setdefault(next(self._rr) % n, []).append(v)
            for p, vs in by.items():
                self.produce_batch(topic, p, vs)
        else:
            self.produce_batch(topic, partition, vals)
        return len(vals)

    # ---------------------------------------------------------------- fetch / offsets
    def fetch_raw(self, topic: str, partition: int, offset: int, max_bytes: int = 64 << 20,
                  max_wait_ms: int = 0) -> Tuple[int, int, bytes]:
        """(error, high watermark, record set bytes) from the leader; retriable errors are
        retried, OFFSET_OUT_OF_RANGE is returned to the caller."""
        body = (Writer().i32(-1).i32(max_wait_ms).i32(1 if max_wait_ms else 0).i32(max_bytes).i8(0)
                .array([topic], lambda w, t: w.string(t).array([partition], lambda w2, p: w2.i32(p).i64(offset).i32(max_bytes)))
                .build())

        def parse(r):
            r.i32()                                         # throttle

            def part(x):
                idx, err, hw, _lso = x.i32(), x.i16(), x.i64(), x.i64()
                x.array(lambda y: (y.i64(), y.i64()))
                return idx, err, hw, x.bytes_()
            _t, parts = r.array(lambda x: (x.string(), x.array(part)))[0]
            _idx, err, hw, recs = parts[0]
            if err == ERR_OFFSET_OUT_OF_RANGE:
                return ERR_NONE, (err, hw, b"")
            return err, (err, hw, recs or b"")
        return self._on_leader(topic, partition, FETCH, 4, body, parse)

    def fetch(self, topic: str, partition: int, offset: int, max_records: int = 1000,
              max_bytes: int = 64 << 20, max_wait_ms: int = 0) -> List[Record]:
        err, _hw, recs = self.fetch_raw(topic, partition, offset, max_bytes, max_wait_ms)
        if err == ERR_OFFSET_OUT_OF_RANGE:
            return self.fetch(topic, partition, self.begin_offset(topic, partition), max_records, max_bytes)
        out = [r_ for r_ in decode_record_batches(recs, topic, partition) if r_.offset >= offset] if recs else []
        return out[:max_records]

    def _list_offset(self, topic: str, partition: int, ts: int) -> int:
        body = Writer().i32(-1).array([topic], lambda w, t: w.string(t).array([partition], lambda w2, p: w2.i32(p).i64(ts))).build()

        def parse(r):
            resp = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i16(), y.i64(), y.i64()))))
            _p, err, _ts, off = resp[0][1][0]
            return err, off
        return self._on_leader(topic, partition, LIST_OFFSETS, 1, body, parse)

    def end_offset(self, topic: str, partition: int) -> int:
        return self._list_offset(topic, partition, -1)

    def begin_offset(self, topic: str, partition: int) -> int:
        return self._list_offset(topic, partition, -2)

    def _coordinator(self, group: str) -> Connection:
        if group not in self._coord:
            r = self._boot_request(FIND_COORDINATOR, 0, Writer().string(group).build())
            err, node, host, port = r.i16(), r.i32(), r.string(), r.i32()
            if err:
                raise BrokerError(f"FindCoordinator {group}: error {err}")
            self._nodes.setdefault(node, (host, port))
            self._coord[group] = node
        return self._conn(self._coord[group])

    def _on_coordinator(self, group: str, api: int, ver: int, body: bytes) -> Reader:
        for attempt in range(self.RETRIES):
            try:
                return self._coordinator(group).request(api, ver, body)
            except (OSError, ConnectionError) as e:
                node = self._coord.pop(group, None)
                if node is not None:
                    self._drop(node)
                self.retries_done += 1
                time.sleep(min(0.5, 0.01 * (2 ** attempt)))
                last = e
        raise BrokerError(f"group {group}: coordinator not reachable ({last})")

    def commit(self, group: str, topic: str, partition: int, offset: int) -> None:
        body = (Writer().string(group).i32(-1).string("").i64(-1)
                .array([topic], lambda w, t: w.string(t).array([partition], lambda w2, p: w2.i32(p).i64(offset).string(None)))
                .build())
        r = self._on_coordinator(group, OFFSET_COMMIT, 2, body)
        for _t, parts in r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i16())))):
            for p, err in parts:
                if err:
                    self._coord.pop(group, None)
                    raise BrokerError(f"offset commit {topic}[{p}] error {err}")

    def committed(self, group: str, topic: str, partition: int) -> Optional[int]:
        body = Writer().string(group).array([topic], lambda w, t: w.string(t).array([partition], lambda w2, p: w2.i32(p))).build()
        r = self._on_coordinator(group, OFFSET_FETCH, 1, body)
        resp = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i64(), y.string(), y.i16()))))
        _p, off, _meta, err = resp[0][1][0]
        return None if off < 0 else off

    def lag(self, group: str, topic: str) -> int:
        tot = 0
        for p in range(self.partitions(topic)):
            c = self.committed(group, topic, p)
            tot += self.end_offset(topic, p) - (c if c is not None else self.begin_offset(topic, p))
        return tot

    def consumer(self, group: str, topics: Sequence[str], partitions: Optional[Sequence[Tuple[str, int]]] = None,
                 member_id: Optional[str] = None, auto_commit: bool = False) -> "WireConsumer":
        return WireConsumer(self, group, list(topics), partitions, auto_commit)

    def group_consumer(self, group: str, topics: Sequence[str], **kw):
        """Consumer-group member (JoinGroup/SyncGroup/Heartbeat, range assignor): partitions are
        assigned by the group coordinator and move on member failure (ingest/kafka_group.py)."""
        from .kafka_group import GroupConsumer
        return GroupConsumer(self, group, topics, client_id=self.client_id, **kw)

    def wait_for_data(self, predicate, timeout: float) -> bool:
        end = time.monotonic() + timeout
        while time.monotonic() < end:
            if predicate():
                return True
            time.sleep(0.005)
        return predicate()

    def close(self):
        try:
            self.flush()                         # pipelined produces still waiting for answers
        except BrokerError:
            pass
        self._boot.close()
        for c in list(self._conns.values()) + list(self._pconns.values()):
            c.close()


class WireConsumer:
    """Statically assigned consumer (``partitions`` or every partition of ``topics``)."""

    def __init__(self, broker: KafkaBroker, group: str, topics: List[str],
                 partitions: Optional[Sequence[Tuple[str, int]]], auto_commit: bool):
        self.broker = broker
        self.group = group
        self.topics = topics
        self.auto_commit = auto_commit
        if partitions is None:
            partitions = [(t, p) for t in topics for p in range(broker.partitions(t))]
        self._assignment = list(partitions)
        self._positions = {}
        for t, p in self._assignment:
            c = broker.committed(group, t, p)
            self._positions[(t, p)] = c if c is not None else broker.begin_offset(t, p)
        self.closed = False

    @property
    def assignment(self):
        return list(self._assignment)

    def poll(self, timeout: float = 0.0, max_records: int = 500) -> List[Record]:
        out: List[Record] = []
        end = time.monotonic() + timeout
        # idle back-off 1 -> 8 ms: an idle consumer (the notifier, the response consumer) sent
        # one Fetch per partition every 2 ms -- thousands of empty requests a second through
        # the broker's event loop; data resets it (the next poll() starts at 1 ms again)
        nap = 0.001
        while True:
            for tp in self._assignment:
                if len(out) >= max_records:
                    break
                recs = self.broker.fetch(tp[0], tp[1], self._positions[tp], max_records - len(out))
                if recs:
                    self._positions[tp] = recs[-1].offset + 1
                    out.extend(recs)
            now = time.monotonic()
            if out or now >= end:
                break
            time.sleep(min(nap, max(0.0, end - now)))
            nap = min(0.008, nap * 2)
        if self.auto_commit and out:
            self.commit()
        return out

    def commit(self, offsets=None) -> None:
        for (t, p), o in (offsets or self._positions).items():
            self.broker.commit(self.group, t, p, o)

    def position(self, topic: str, partition: int) -> int:
        return self._positions[(topic, partition)]

    def seek(self, topic: str, partition: int, offset: int) -> None:
        self._positions[(topic, partition)] = offset

    def close(self) -> None:
        self.closed = True
