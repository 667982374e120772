"""Partition logs that keep producer RecordBatches VERBATIM (kafka-lite's storage).

A Kafka broker does not re-encode records: it validates a produced RecordBatch (magic 2,
CRC-32C over attributes..records), stamps its base offset (the 8 bytes in front of the
CRC-covered region, so the CRC stays valid), appends the bytes to the partition log and
serves Fetch by handing out whole stored batches starting at the one that contains the
requested offset (the client skips records below its fetch offset).  This module does the
same, so kafka-lite's per-record cost is zero on both produce and fetch (VERDICT r1 #3:
the round-1 broker decoded and re-encoded every record in Python).

Offsets, begin/end, retention by batch count, committed group offsets.  Thread-safe (one
lock per store); the in-process consumers that want ``Record`` objects use ``fetch``,
which decodes -- the wire path uses ``fetch_raw``.
"""
from __future__ import annotations

import bisect
import struct
import threading
import time
import zlib
from typing import Dict, List, Optional, Tuple

from .broker import BrokerError, Record

_HDR = struct.Struct(">qiibIhi")      # base, batch_len, leader epoch, magic, crc, attrs, last delta
_COUNT_OFF = 57                       # records count (i32) within a batch


_SEQ_MASK = 0x7FFFFFFF            # producer sequences are int32 and wrap to 0


class InvalidBatch(BrokerError):
    pass


class OutOfOrderSequence(BrokerError):
    """An idempotent producer's batch skipped a sequence number (Kafka error 45)."""


_PID = struct.Struct(">qhi")          # producerId, producerEpoch, baseSequence (bytes 43..57)
_PRODUCER_CACHE = 5                   # batches remembered per producer and partition (Kafka: 5)


def split_batches(data: bytes, verify_crc: bool = True) -> List[Tuple[int, int, int, memoryview]]:
    """Validate a produced record set: [(lastOffsetDelta, count, attrs, batch bytes)].
    Raises InvalidBatch on a truncated batch, a magic other than 2 or a CRC mismatch."""
    from .kafka_wire import crc32c
    mv = memoryview(data)
    out = []
    o = 0
    n = len(data)
    while o < n:
        if n - o < 61:
            raise InvalidBatch("truncated record batch header")
        _base, blen, _ep, magic, crc, attrs, last = _HDR.unpack_from(mv, o)
        end = o + 12 + blen
        if blen < 49 or end > n:
            raise InvalidBatch("truncated record batch")
        if magic != 2:
            raise InvalidBatch(f"unsupported magic {magic}")
        if verify_crc and crc32c(mv[o + 21:end]) != crc:
            raise InvalidBatch("record batch CRC mismatch")
        count = struct.unpack_from(">i", mv, o + _COUNT_OFF)[0]
        if count < 0 or last < 0 or (count and last != count - 1):
            raise InvalidBatch("inconsistent record count / last offset delta")
        out.append((last, count, attrs, mv[o:end]))
        o = end
    return out


class _Log:
    __slots__ = ("bases", "batches", "begin", "end", "nbytes", "ts", "visible")

    def __init__(self):
        self.bases: List[int] = []
        self.batches: List[bytes] = []
        self.begin = 0
        self.end = 0                  # next offset to assign
        self.visible = 0              # high watermark: fetches see offsets below it (durable
                                      # stores: what is written; memory: == end)
        self.nbytes = 0
        self.ts: List[float] = []


class BatchStore:
    def __init__(self, default_partitions: int = 1, retention_batches: Optional[int] = None,
                 verify_crc: bool = True):
        self.default_partitions = default_partitions
        self.retention_batches = retention_batches
        self.verify_crc = verify_crc
        self._topics: Dict[str, List[_Log]] = {}
        self._committed: Dict[Tuple[str, str, int], int] = {}
        self._lock = threading.Lock()
        # idempotent producers: (topic, partition) -> producer id -> [epoch, [(first seq, last
        # seq, base offset), ...]] of its last batches; InitProducerId hands out _next_pid
        self._producers: Dict[Tuple[str, int], Dict[int, list]] = {}
        self._next_pid = 0
        self.duplicates_dropped = 0

    # ------------------------------------------------------------------ durability hooks
    # (no-ops here; ingest/durable_store.py writes segments / offsets / producer ids)
    def _persist_appended(self, topic: str, partition: int, L: "_Log", first: int) -> None:
        pass

    def _apply_retention(self, topic: str, partition: int, L: "_Log") -> None:
        pass

    def _persist_commit(self, group: str, topic: str, partition: int, offset: int) -> None:
        pass

    def _persist_producer_ids(self) -> None:
        pass

    def _appended(self, L: "_Log") -> Optional[int]:
        """After an append (under the lock): a memory store shows the data at once; a durable
        one (durable_store.py) returns the write ticket to wait for and shows it once written."""
        L.visible = L.end
        return None

    # ------------------------------------------------------------------ idempotent producers
    def init_producer_id(self, node: int = 0, stride: int = 1) -> Tuple[int, int]:
        """InitProducerId (non-transactional): a fresh producer id, epoch 0.  A replicated
        cluster's brokers hand out disjoint ids: ``node + stride * k``."""
        with self._lock:
            pid = self._next_pid
            if stride > 1:
                pid += (node - pid) % stride
            self._next_pid = pid + 1
            self._persist_producer_ids()
            return pid, 0

    def _track_producer(self, topic: str, partition: int, b, base: int) -> None:
        pid, epoch, seq = _PID.unpack_from(b, 43)
        if pid < 0:
            return
        last = struct.unpack_from(">i", b, 23)[0]
        st = self._producers.setdefault((topic, partition), {}).setdefault(pid, [epoch, []])
        if epoch != st[0]:
            st[0], st[1] = epoch, []
        st[1].append((seq, (seq + last) & _SEQ_MASK, base))     # wraps at 2^31 (Kafka)
        del st[1][:-_PRODUCER_CACHE]
        self._next_pid = max(self._next_pid, pid + 1)

    def _check_sequence(self, topic: str, partition: int, b) -> Optional[int]:
        """None: append; an int: the base offset of the already appended copy (duplicate)."""
        pid, epoch, seq = _PID.unpack_from(b, 43)
        if pid < 0:
            return None
        st = self._producers.get((topic, partition), {}).get(pid)
        if st is None or epoch != st[0] or not st[1]:
            return None                     # a new producer (or epoch): accept
        for first, _last, base in st[1]:
            if first == seq:
                return base
        expect = (st[1][-1][1] + 1) & _SEQ_MASK
        if seq != expect:
            raise OutOfOrderSequence(f"{topic}[{partition}] producer {pid}: sequence {seq}, "
                                     f"expected {expect}")
        return None

    # ------------------------------------------------------------------ topics
    def create_topic(self, name: str, partitions: Optional[int] = None) -> None:
        with self._lock:
            if name not in self._topics:
                self._topics[name] = [_Log() for _ in range(max(1, partitions or self.default_partitions))]

    def topics(self) -> Dict[str, int]:
        with self._lock:
            return {t: len(p) for t, p in self._topics.items()}

    def stored_bytes(self) -> int:
        """Bytes of record batches the log holds (the broker's working set)."""
        with self._lock:
            return sum(L.nbytes for parts in self._topics.values() for L in parts)

    def partitions(self, topic: str) -> int:
        self.create_topic(topic)
        return len(self._topics[topic])

    def _log(self, topic: str, partition: int) -> _Log:
        parts = self._topics.get(topic)
        if parts is None or not 0 <= partition < len(parts):
            raise BrokerError(f"{topic}: no partition {partition}")
        return parts[partition]

    # ------------------------------------------------------------------ produce
    def append_raw(self, topic: str, partition: int, data: bytes) -> Tuple[int, int]:
        """Append a produced record set verbatim; returns (base offset, records) once it is
        stored (and fetchable)."""
        base, n, _ticket = self.append_raw_nowait(topic, partition, data)
        return base, n

    def append_raw_nowait(self, topic: str, partition: int, data: bytes) -> Tuple[int, int, Optional[int]]:
        """``append_raw`` that does not wait for a durable store's write: (base offset, records,
        write ticket or None).  kafka-lite answers the produce once the ticket is written."""
        batches = split_batches(data, self.verify_crc)
        with self._lock:
            L = self._log(topic, partition)
            base0 = L.end
            first_new = len(L.batches)
            nrec = 0
            now = time.time()
            for k, (last, count, _attrs, mv) in enumerate(batches):
                dup = self._check_sequence(topic, partition, mv)
                if dup is not None:         # a retried batch that is already in the log
                    self.duplicates_dropped += 1
                    if k == 0:
                        base0 = dup
                    continue
                # a writable view is memory the broker owns (kafka-lite receives each produce
                # request into its own buffer): kept as is, no copy; anything else is copied once
                b = mv if not mv.readonly else bytearray(mv)
                struct.pack_into(">q", b, 0, L.end)          # broker-assigned base offset
                self._track_producer(topic, partition, b, L.end)
                L.bases.append(L.end)
                L.batches.append(b)
                L.ts.append(now)
                L.end += last + 1
                L.nbytes += len(b)
                nrec += count
            if len(L.batches) > first_new:
                self._persist_appended(topic, partition, L, first_new)
            if self.retention_batches is not None and len(L.batches) > self.retention_batches:
                drop = len(L.batches) - self.retention_batches
                L.nbytes -= sum(len(x) for x in L.batches[:drop])
                del L.bases[:drop], L.batches[:drop], L.ts[:drop]
                L.begin = L.bases[0]
                self._apply_retention(topic, partition, L)
            return base0, nrec, self._appended(L)

    def append_replica(self, topic: str, partition: int, data) -> Tuple[int, Optional[int]]:
        """A follower's append (replicated kafka-lite, ingest/kafka_replica.py): batches fetched
        from the partition leader, base offsets already stamped by it, appended at exactly
        those offsets (a batch this log already holds is skipped; a gap is an error).  The
        idempotent-producer state is tracked as on the leader, so a follower that becomes leader
        deduplicates retried batches.  Returns (batches appended, write ticket or None)."""
        batches = split_batches(data, False)            # the leader verified them
        with self._lock:
            L = self._log(topic, partition)
            first_new = len(L.batches)
            now = time.time()
            for last, _count, _attrs, mv in batches:
                base = struct.unpack_from(">q", mv, 0)[0]
                if base + last + 1 <= L.end:
                    continue                            # already replicated (a re-fetch)
                if base != L.end:
                    raise BrokerError(f"{topic}[{partition}]: replica gap (log end {L.end}, batch {base})")
                b = mv if not mv.readonly else bytearray(mv)
                self._track_producer(topic, partition, b, base)
                L.bases.append(base)
                L.batches.append(b)
                L.ts.append(now)
                L.end = base + last + 1
                L.nbytes += len(b)
            n_new = len(L.batches) - first_new
            if n_new:
                self._persist_appended(topic, partition, L, first_new)
            if self.retention_batches is not None and len(L.batches) > self.retention_batches:
                drop = len(L.batches) - self.retention_batches
                L.nbytes -= sum(len(x) for x in L.batches[:drop])
                del L.bases[:drop], L.batches[:drop], L.ts[:drop]
                L.begin = L.bases[0]
                self._apply_retention(topic, partition, L)
            return n_new, self._appended(L) if n_new else None

    def truncate(self, topic: str, partition: int, offset: int) -> int:
        """Drop every batch at or above ``offset`` (a replica whose leader changed cuts its
        un-acknowledged tail to the high watermark before it follows the new leader, so its
        log is a prefix of the leader's -- ingest/kafka_replica.py).  The idempotent-producer
        state of the partition is rebuilt from the batches that remain.  Returns the batches
        dropped."""
        with self._lock:
            L = self._log(topic, partition)
            if offset >= L.end:
                return 0
            i = bisect.bisect_left(L.bases, offset)
            inside = (0 < i < len(L.bases) and L.bases[i] != offset) or \
                (i == len(L.bases) and L.bases and L.bases[-1] < offset)      # inside the last batch
            if inside:
                raise BrokerError(f"{topic}[{partition}]: truncation point {offset} inside a batch")
            dropped = len(L.batches) - i
            L.nbytes -= sum(len(x) for x in L.batches[i:])
            del L.bases[i:], L.batches[i:], L.ts[i:]
            L.end = max(offset, L.begin)
            L.visible = min(L.visible, L.end)
            self._producers.pop((topic, partition), None)
            for base, b in zip(L.bases, L.batches):
                self._track_producer(topic, partition, b, base)
            self._persist_truncate(topic, partition, L.end)
            return dropped

    def _persist_truncate(self, topic: str, partition: int, offset: int) -> None:
        pass

    def reset_to(self, topic: str, partition: int, offset: int) -> int:
        """Drop the whole partition log and continue at ``offset`` (a replica that was away
        longer than its leader's retention: its log end is below the leader's log start, so it
        restarts from there, as Kafka's follower does).  Returns the batches dropped."""
        with self._lock:
            L = self._log(topic, partition)
            dropped = len(L.batches)
            L.nbytes = 0
            del L.bases[:], L.batches[:], L.ts[:]
            L.begin = L.end = L.visible = int(offset)
            self._producers.pop((topic, partition), None)
            self._persist_reset(topic, partition, int(offset))
            return dropped

    def _persist_reset(self, topic: str, partition: int, offset: int) -> None:
        pass

    def log_end(self, topic: str, partition: int) -> int:
        """The next offset this log assigns (LEO), written or not."""
        with self._lock:
            return self._log(topic, partition).end

    def produce(self, topic: str, value: bytes, key: Optional[bytes] = None,
                partition: Optional[int] = None, headers: Tuple = ()) -> Tuple[int, int]:
        from .kafka_wire import encode_record_batch
        n = self.partitions(topic)
        if partition is None:
            partition = zlib.crc32(key) % n if key is not None else 0
        base, _ = self.append_raw(topic, partition, encode_record_batch([value], [key]))
        return partition, base

    # ------------------------------------------------------------------ fetch
    def fetch_raw(self, topic: str, partition: int, offset: int, max_bytes: int) -> bytes:
        """Whole stored batches from the one containing ``offset``, up to ``max_bytes`` (at
        least one batch, like Kafka, so an oversized batch is never stuck)."""
        return b"".join(self.fetch_parts(topic, partition, offset, max_bytes))

    def fetch_parts(self, topic: str, partition: int, offset: int, max_bytes: int,
                    upto: Optional[int] = None, unwritten: bool = False) -> list:
        """``fetch_raw`` as the list of stored batches themselves (no copy; a fetch response
        is written to the socket from them).  ``upto``: serve only batches below this offset
        (a replicated leader's consumers see up to the high watermark).  ``unwritten``: up to
        the log end, written or not (a follower's replica fetch, and a replicated leader's
        consumers below the high watermark: the copies on the other in-sync brokers are what
        protect a batch the leader has not written yet)."""
        with self._lock:
            L = self._log(topic, partition)
            lim = L.end if unwritten else L.visible
            if upto is not None:
                lim = min(lim, upto)
            if offset >= lim or not L.batches:
                return []
            i = max(0, bisect.bisect_right(L.bases, offset) - 1)
            out, size = [], 0
            while i < len(L.batches):
                b = L.batches[i]
                if L.bases[i] >= lim or (out and size + len(b) > max_bytes):
                    break
                out.append(b)
                size += len(b)
                i += 1
            return out

    def fetch(self, topic: str, partition: int, offset: int, max_records: int = 1000) -> List[Record]:
        from .kafka_wire import decode_record_batches
        offset = max(offset, self.begin_offset(topic, partition))
        recs = decode_record_batches(self.fetch_raw(topic, partition, offset, 64 << 20), topic, partition,
                                     verify_crc=False)
        return [r for r in recs if r.offset >= offset][:max_records]

    def end_offset(self, topic: str, partition: int) -> int:
        """The high watermark: the end of what fetches can see."""
        with self._lock:
            return self._log(topic, partition).visible

    def begin_offset(self, topic: str, partition: int) -> int:
        with self._lock:
            return self._log(topic, partition).begin

    def bytes_stored(self, topic: str, partition: int) -> int:
        with self._lock:
            return self._log(topic, partition).nbytes

    # ------------------------------------------------------------------ offsets
    def commit(self, group: str, topic: str, partition: int, offset: int) -> None:
        with self._lock:
            k = (group, topic, partition)
            v = max(offset, self._committed.get(k, 0))
            if v != self._committed.get(k):
                self._committed[k] = v
                self._persist_commit(group, topic, partition, v)

    def committed(self, group: str, topic: str, partition: int) -> Optional[int]:
        with self._lock:
            return self._committed.get((group, topic, partition))

    def lag(self, group: str, topic: str) -> int:
        """Records not yet committed by ``group`` (consumer lag, summed over partitions)."""
        with self._lock:
            return sum(L.end - self._committed.get((group, topic, p), L.begin)
                       for p, L in enumerate(self._topics.get(topic, [])))
