"""Durable partition logs for kafka-lite: segment files of the verbatim RecordBatches, an
offset index, persisted group offsets and idempotent-producer state, recovered on start.

The reference runs a 3-broker replicated Strimzi cluster (deploy/frauddetection_cr.yaml:
75-77) and its Kafka dashboard watches under-replicated / offline partitions
(deploy/grafana/Kafka.json:271,347): a broker pod that restarts (``restartPolicy: Always``,
deploy/router.yaml:75) must come back with every acknowledged transaction and every
committed consumer offset.  ``DurableBatchStore`` is ``BatchStore`` (batch_store.py) plus:

* per partition a directory ``<topic>-<p>/`` of segments ``<base offset>.log`` -- the
  produced batches byte for byte, base offset stamped (what Fetch serves) -- and
  ``<base offset>.idx``, 16 bytes per batch (base offset, file position).  A segment rolls
  at ``segment_bytes``; retention deletes whole segments below the log start;
* ``offsets.log``: one JSON line per OffsetCommit (last one per group/topic/partition wins),
  compacted on start;
* ``topics.json`` and ``producers.json`` (the next producer id InitProducerId hands out);
* idempotent produce (Kafka's producer id + epoch + base sequence in the batch header): a
  retried batch the broker already appended -- e.g. acknowledged just before a crash, or the
  ack lost -- is answered with its original base offset instead of being appended twice
  (``BatchStore.append_raw`` keeps the last 5 batches per producer and partition); the state
  is rebuilt from the segments on recovery;
* fsync policy: ``always`` (segment + index + offsets fsync'd before the request is
  answered), ``interval`` (a background thread fsyncs dirty files every ``fsync_interval_s``,
  default 1 s -- Kafka's ``log.flush.interval.ms`` model; a killed broker PROCESS loses
  nothing, the writes are in the page cache), ``never``;
* write-behind: the segment / index writes run on ONE writer thread in append order, off the
  broker's event loop.  A produce is answered, and its records become fetchable (the
  partition's high watermark, ``_Log.visible``), only once they are written, so a killed
  broker never loses an acknowledged or consumed record.  Writing on the event loop capped
  the deployed TXB1 topology at 1.0 x 10^7 tx/s against 1.5 x 10^7 with the in-memory store,
  and put the broker's writes in every fetch's p99 (profiles/r4/broker_ab/).

Recovery maps every segment read-only (``mmap``) and the stored batches are memoryviews of
those maps, so Fetch stays zero-copy for recovered data too.  A torn tail (a crash in the
middle of a write) is detected by the batch header / CRC check and truncated; an index
shorter than its segment is rebuilt by scanning the unindexed batches.
"""
from __future__ import annotations

import collections
import json
import mmap
import os
import struct
import threading
import time
from typing import Dict, List, Optional, Tuple

from .batch_store import _HDR, BatchStore, _Log, split_batches
from .broker import BrokerError

_IDX = struct.Struct("<qq")                 # base offset, file position
FSYNC_POLICIES = ("always", "interval", "never")


def _seg_name(base: int) -> str:
    return f"{base:020d}"


class _Segment:
    __slots__ = ("base", "path", "fd", "idx_fd", "size", "nbatches", "last_end", "closed")

    def __init__(self, base: int, path: str):
        self.base = base
        self.path = path                    # without extension
        self.fd = -1
        self.idx_fd = -1
        self.size = 0
        self.nbatches = 0
        self.last_end = base               # next offset after this segment's last batch
        self.closed = False


class DurableBatchStore(BatchStore):
    def __init__(self, data_dir: str, default_partitions: int = 1, retention_batches: Optional[int] = None,
                 verify_crc: bool = True, fsync: str = "interval", fsync_interval_s: float = 1.0,
                 segment_bytes: int = 256 << 20, truncate_to: Optional[Dict[Tuple[str, int], int]] = None):
        """``truncate_to``: (topic, partition) -> offset: recovery drops every batch at or above
        it (a replicated broker restarting truncates to its checkpointed high watermark, so its
        log is a prefix of the current leader's -- ingest/kafka_replica.py)."""
        if fsync not in FSYNC_POLICIES:
            raise ValueError(f"fsync policy {fsync!r}: one of {FSYNC_POLICIES}")
        super().__init__(default_partitions=default_partitions, retention_batches=retention_batches,
                         verify_crc=verify_crc)
        self.data_dir = os.path.abspath(data_dir)
        self.fsync = fsync
        self.fsync_interval_s = float(fsync_interval_s)
        self.segment_bytes = int(segment_bytes)
        os.makedirs(self.data_dir, exist_ok=True)
        self._segs: Dict[Tuple[str, int], List[_Segment]] = {}
        self._dirty: set = set()            # fds written since the last fsync
        # fds of rolled / retired segments: fsync'd and closed by flush() (the flusher thread
        # in "interval" mode), never on the produce path -- a 256 MB segment's fsync under the
        # store lock stalled every produce and fetch of the broker behind it
        self._closing: List[int] = []
        self._off_fd = -1
        self.recovered: Dict[str, object] = {}
        self._limits = dict(truncate_to or {})
        self.truncated_batches = 0
        self.bytes_written = 0
        self.fsyncs = 0
        # write-behind: appends land in memory under the store lock and are queued; ONE writer
        # thread writes segments / index entries in queue order (os.write releases the GIL, so
        # kafka-lite's event loop keeps serving while it runs) and then advances the partition's
        # high watermark -- fetches only see written data, a produce is answered only once its
        # ticket is written (append_raw waits; kafka-lite awaits on_written), so a killed broker
        # never loses an acknowledged or consumed record
        self._wq: collections.deque = collections.deque()
        self._wcv = threading.Condition()
        self._ticket = 0                    # last ticket queued (under the store lock)
        self._written = 0                   # last ticket written (under _wcv)
        self._wstop = False
        self._werr: Optional[BaseException] = None
        self.on_written = None              # callback(ticket, [(topic, partition), ...]), writer thread
        self._writer_on = False
        self._recover()
        for parts in self._topics.values():
            for L in parts:
                L.visible = L.end           # recovered data is on disk
        self._writer = threading.Thread(target=self._write_loop, daemon=True, name="kafka-lite-writer")
        self._writer_on = True
        self._writer.start()
        self._stop = threading.Event()
        self._flusher = None
        if self.fsync == "interval":
            self._flusher = threading.Thread(target=self._flush_loop, daemon=True, name="kafka-lite-fsync")
            self._flusher.start()

    # ------------------------------------------------------------------ files
    def _pdir(self, topic: str, p: int) -> str:
        return os.path.join(self.data_dir, f"{topic}-{p}")

    def _write_all(self, fd: int, data) -> None:
        mv = memoryview(data)
        while len(mv):
            k = os.write(fd, mv)
            mv = mv[k:]
        self._dirty.add(fd)

    def _sync(self, fds) -> None:
        for fd in list(fds):
            try:
                os.fsync(fd)
                self.fsyncs += 1
            except OSError:
                pass

    def _flush_loop(self) -> None:
        while not self._stop.wait(self.fsync_interval_s):
            self.flush()

    def flush(self) -> None:
        """fsync every file written since the last flush; close retired segment files."""
        with self._lock:
            fds, self._dirty = self._dirty, set()
            closing, self._closing = self._closing, []
        self._sync(fds - set(closing))
        for fd in closing:                  # not reachable from the store any more
            if self.fsync != "never":
                try:
                    os.fsync(fd)
                    self.fsyncs += 1
                except OSError:
                    pass
            os.close(fd)

    def _atomic_json(self, name: str, obj) -> None:
        path = os.path.join(self.data_dir, name)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(obj, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)

    def _open_segment(self, topic: str, p: int, base: int) -> _Segment:
        d = self._pdir(topic, p)
        os.makedirs(d, exist_ok=True)
        seg = _Segment(base, os.path.join(d, _seg_name(base)))
        seg.fd = os.open(seg.path + ".log", os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        seg.idx_fd = os.open(seg.path + ".idx", os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        seg.size = os.fstat(seg.fd).st_size
        self._segs.setdefault((topic, p), []).append(seg)
        return seg

    def _close_segment(self, seg: _Segment, now: bool = False) -> None:
        """Retire a segment's files (under the store lock).  ``now``: fsync + close here (shutdown,
        fsync="always"); "interval" hands them to the flusher thread's next flush(), so the produce
        path never waits on a big fsync; "never" closes them at once."""
        if seg.closed:
            return
        for fd in (seg.fd, seg.idx_fd):
            if fd >= 0:
                self._dirty.discard(fd)
                if self.fsync == "interval" and not now:
                    self._closing.append(fd)
                    continue
                if now or self.fsync == "always":
                    try:
                        os.fsync(fd)
                    except OSError:
                        pass
                os.close(fd)                # "never": closed at once, no fsync
        seg.fd = seg.idx_fd = -1
        seg.closed = True

    # ------------------------------------------------------------------ recovery
    def _recover(self) -> None:
        t0 = time.time()
        topics = {}
        tp = os.path.join(self.data_dir, "topics.json")
        if os.path.exists(tp):
            with open(tp) as f:
                topics = json.load(f)
        prod = os.path.join(self.data_dir, "producers.json")
        if os.path.exists(prod):
            with open(prod) as f:
                self._next_pid = int(json.load(f).get("next_producer_id", 0))
        n_batches = n_records = truncated = 0
        for name, nparts in topics.items():
            BatchStore.create_topic(self, name, int(nparts))
            for p in range(int(nparts)):
                b, r, t = self._recover_partition(name, p)
                n_batches += b
                n_records += r
                truncated += t
        # group offsets: last commit per key wins; compacted into a fresh file
        op = os.path.join(self.data_dir, "offsets.log")
        if os.path.exists(op):
            with open(op) as f:
                for line in f:
                    try:
                        d = json.loads(line)
                    except json.JSONDecodeError:
                        continue                    # torn last line
                    k = (d["g"], d["t"], int(d["p"]))
                    self._committed[k] = max(int(d["o"]), self._committed.get(k, 0))
            tmp = op + ".tmp"
            with open(tmp, "w") as f:
                for (g, t, p), o in self._committed.items():
                    f.write(json.dumps({"g": g, "t": t, "p": p, "o": o}) + "\n")
                f.flush()
                os.fsync(f.fileno())
            os.replace(tmp, op)
        self._off_fd = os.open(op, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        self.recovered = {"topics": len(topics), "batches": n_batches, "records": n_records,
                          "committed_offsets": len(self._committed), "torn_tails_truncated": truncated,
                          "producers": sum(len(v) for v in self._producers.values()),
                          "seconds": round(time.time() - t0, 3)}

    def _recover_partition(self, topic: str, p: int) -> Tuple[int, int, int]:
        d = self._pdir(topic, p)
        if not os.path.isdir(d):
            return 0, 0, 0
        bases = sorted(int(f[:-4]) for f in os.listdir(d) if f.endswith(".log"))
        L = self._log(topic, p)
        nb = nr = torn = 0
        lim = self._limits.get((topic, p))
        if lim is not None:
            # segments that start at or past the limit go entirely (the first one is kept, cut
            # to empty, so the partition's offsets continue from the limit)
            keep = [b for b in bases if b < lim] or bases[:1]
            for b in bases:
                if b not in keep:
                    for ext in (".log", ".idx"):
                        try:
                            os.unlink(os.path.join(d, _seg_name(b)) + ext)
                        except OSError:
                            pass
            bases = keep
        for k, base in enumerate(bases):
            path = os.path.join(d, _seg_name(base))
            size = os.path.getsize(path + ".log")
            entries: List[Tuple[int, int]] = []
            if os.path.exists(path + ".idx"):
                with open(path + ".idx", "rb") as f:
                    raw = f.read()
                entries = [_IDX.unpack_from(raw, i) for i in range(0, len(raw) - len(raw) % 16, 16)]
            mm = None
            good_end = 0
            batches: List[Tuple[int, int, int]] = []      # (base offset, position, length)
            if size:
                with open(path + ".log", "rb") as f:
                    mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
                mv = memoryview(mm)
                pos = 0
                # indexed batches first (cheap header check), then scan what the index misses
                for bo, ps in entries:
                    if ps != pos or pos + 12 > size:
                        break
                    hb, blen = struct.unpack_from(">qi", mv, pos)
                    if hb != bo or pos + 12 + blen > size:
                        break
                    batches.append((bo, pos, 12 + blen))
                    pos += 12 + blen
                while pos < size:
                    if size - pos < 61:
                        break
                    blen = struct.unpack_from(">i", mv, pos + 8)[0]
                    if blen < 49 or pos + 12 + blen > size:
                        break
                    try:
                        split_batches(mv[pos:pos + 12 + blen], verify_crc=True)
                    except BrokerError:
                        break
                    batches.append((struct.unpack_from(">q", mv, pos)[0], pos, 12 + blen))
                    pos += 12 + blen
                good_end = pos
                was_cut = False
                if lim is not None:             # replicated: cut at the checkpointed HW
                    cut = [i for i, (bo, _ps, _ln) in enumerate(batches) if bo >= lim]
                    if cut:
                        self.truncated_batches += len(batches) - cut[0]
                        good_end = batches[cut[0]][1]
                        del batches[cut[0]:]
                        was_cut = True
                del mv
            else:
                was_cut = False
            if good_end < size:                 # torn tail (a crash mid-write), or the HW cut
                torn += 0 if was_cut else 1
                if mm is not None:
                    mm.close()
                    mm = None
                with open(path + ".log", "r+b") as f:
                    f.truncate(good_end)
                if good_end:
                    with open(path + ".log", "rb") as f:
                        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
            if len(entries) != len(batches):    # rebuild the index to match
                with open(path + ".idx", "wb") as f:
                    f.write(b"".join(_IDX.pack(bo, ps) for bo, ps, _ln in batches))
            seg = _Segment(base, path)
            seg.size = good_end
            seg.nbatches = len(batches)
            seg.closed = True
            mv = memoryview(mm) if mm is not None else None
            for bo, ps, ln in batches:
                b = mv[ps:ps + ln]
                _b, _blen, _ep, _magic, _crc, _attrs, last = _HDR.unpack_from(b, 0)
                count = struct.unpack_from(">i", b, 57)[0]
                if not L.batches:
                    L.begin = bo
                L.bases.append(bo)
                L.batches.append(b)
                L.ts.append(time.time())
                L.nbytes += ln
                L.end = bo + last + 1
                seg.last_end = L.end
                nr += count
                self._track_producer(topic, p, b, bo)
            nb += len(batches)
            self._segs.setdefault((topic, p), []).append(seg)
            if k == len(bases) - 1 and good_end < self.segment_bytes:
                # the last segment stays the active one: reopen it for appends
                self._segs[(topic, p)].pop()
                act = self._open_segment(topic, p, base)
                act.nbatches, act.last_end = seg.nbatches, seg.last_end
        if lim is not None and not L.batches and lim > 0:
            L.begin = L.end = lim               # everything was past the cut: continue at it
        if self.retention_batches is not None and len(L.batches) > self.retention_batches:
            drop = len(L.batches) - self.retention_batches
            L.nbytes -= sum(len(x) for x in L.batches[:drop])
            del L.bases[:drop], L.batches[:drop], L.ts[:drop]
            L.begin = L.bases[0]
        self._apply_retention(topic, p, L)
        return nb, nr, torn

    # ------------------------------------------------------------------ BatchStore hooks
    def create_topic(self, name: str, partitions: Optional[int] = None) -> None:
        with self._lock:
            if name in self._topics:
                return
        BatchStore.create_topic(self, name, partitions)
        with self._lock:
            self._atomic_json("topics.json", {t: len(v) for t, v in self._topics.items()})

    def _persist_appended(self, topic: str, partition: int, L: _Log, first: int) -> None:
        """Called under the store lock after batches [first:] of L were appended: queued for
        the writer (the batch objects are referenced, so retention cannot drop them unwritten)."""
        items = []
        for i in range(first, len(L.batches)):
            nxt = L.bases[i + 1] if i + 1 < len(L.bases) else L.end
            items.append((L.bases[i], L.batches[i], nxt))
        self._enqueue(("A", topic, partition, items, L.end))

    def _appended(self, L: _Log) -> Optional[int]:
        return self._ticket                 # visible once the writer has written it

    def _enqueue(self, op) -> None:
        with self._wcv:
            self._ticket += 1
            self._wq.append((self._ticket, op))
            self._wcv.notify()

    def append_raw_nowait(self, topic: str, partition: int, data: bytes) -> Tuple[int, int, Optional[int]]:
        """Refused with a BrokerError once the writer has failed: a ticket handed out now
        would never be written, and its produce would wait forever."""
        if self._werr is not None:
            raise BrokerError(f"kafka-lite log write failed: {self._werr!r}")
        return super().append_raw_nowait(topic, partition, data)

    def append_raw(self, topic: str, partition: int, data: bytes) -> Tuple[int, int]:
        base, n, ticket = self.append_raw_nowait(topic, partition, data)
        self.wait_written(ticket)
        return base, n

    def wait_written(self, ticket: Optional[int], timeout: Optional[float] = None) -> bool:
        """Block until ``ticket`` is written (its records on disk in the page cache, fsync'd
        first with fsync="always") and fetchable."""
        if not ticket:
            return True
        with self._wcv:
            ok = self._wcv.wait_for(lambda: self._written >= ticket or self._werr is not None, timeout)
            if self._werr is not None:
                raise BrokerError(f"kafka-lite log write failed: {self._werr!r}")
            return ok

    def written(self) -> int:
        with self._wcv:
            return self._written

    def _write_loop(self) -> None:
        while True:
            with self._wcv:
                while not self._wq and not self._wstop:
                    self._wcv.wait()
                if not self._wq:
                    return
                ops = list(self._wq)
                self._wq.clear()
            ends: Dict[Tuple[str, int], int] = {}
            touched: set = set()
            try:
                for _t, op in ops:
                    kind, topic, p = op[0], op[1], op[2]
                    if kind == "A":
                        touched |= self._write_batches(topic, p, op[3])
                        ends[(topic, p)] = op[4]
                    elif kind == "T":
                        self._truncate_segments(topic, p, op[3])
                        ends.pop((topic, p), None)
                    elif kind == "X":
                        self._reset_segments(topic, p)
                        ends.pop((topic, p), None)
                    else:
                        self._retire_segments(topic, p, op[3])
                if self.fsync == "always" and touched:
                    self._sync(touched)
            except BaseException as e:           # disk full, ...: fail every waiter loudly
                with self._wcv:
                    self._werr = e
                    self._wcv.notify_all()
                if self.on_written is not None:
                    try:
                        self.on_written(-1, [])
                    except RuntimeError:
                        pass
                return
            with self._lock:
                for (topic, p), end in ends.items():
                    L = self._log(topic, p)
                    if end > L.visible:         # (never past a truncation since queued)
                        L.visible = min(end, L.end)
                if self.fsync != "always":
                    self._dirty |= touched
            with self._wcv:
                self._written = ops[-1][0]
                self._wcv.notify_all()
            cb = self.on_written
            if cb is not None and ends:
                try:
                    cb(ops[-1][0], list(ends))
                except RuntimeError:             # the broker's event loop is gone (shutdown):
                    pass                         # keep writing -- close() drains the queue

    def _write_batches(self, topic: str, partition: int, items) -> set:
        """Writer thread: append (base, batch, next base) items to the partition's segments."""
        segs = self._segs.get((topic, partition))
        seg = segs[-1] if segs and not segs[-1].closed else None
        touched = set()
        for base, b, nxt in items:
            if seg is None or seg.size >= self.segment_bytes:
                if seg is not None:
                    # the fds before _close_segment resets them to -1: a closed fd left in
                    # `touched` would be fsync'd later under a number that may be reused
                    old = (seg.fd, seg.idx_fd)
                    with self._lock:            # (fsync="always": fsync'd as it closes)
                        self._close_segment(seg)
                    touched.difference_update(old)
                seg = self._open_segment(topic, partition, base)
            self._write_raw(seg.fd, b)
            self._write_raw(seg.idx_fd, _IDX.pack(base, seg.size))
            touched.update((seg.fd, seg.idx_fd))
            seg.size += len(b)
            seg.nbatches += 1
            seg.last_end = nxt
            self.bytes_written += len(b)
        return touched

    @staticmethod
    def _write_raw(fd: int, data) -> None:
        mv = memoryview(data)
        while len(mv):
            k = os.write(fd, mv)
            mv = mv[k:]

    def _persist_truncate(self, topic: str, partition: int, offset: int) -> None:
        """Under the store lock: the segments follow the in-memory cut, in write order."""
        self._enqueue(("T", topic, partition, offset))

    def _persist_reset(self, topic: str, partition: int, offset: int) -> None:
        """Under the store lock: every segment of the partition goes, in write order; the next
        write opens a segment based at the new start."""
        self._enqueue(("X", topic, partition, offset))

    def _reset_segments(self, topic: str, partition: int) -> None:
        """Writer thread: delete every segment file of the partition."""
        segs = self._segs.get((topic, partition), [])
        while segs:
            seg = segs.pop()
            with self._lock:
                self._close_segment(seg, now=True)
            for ext in (".log", ".idx"):
                try:
                    os.unlink(seg.path + ext)
                except OSError:
                    pass

    def _truncate_segments(self, topic: str, partition: int, offset: int) -> None:
        """Writer thread: cut the partition's files at ``offset`` (a batch boundary)."""
        segs = self._segs.get((topic, partition), [])
        while len(segs) > 1 and segs[-1].base >= offset:
            seg = segs.pop()
            with self._lock:
                self._close_segment(seg, now=True)
            for ext in (".log", ".idx"):
                try:
                    os.unlink(seg.path + ext)
                except OSError:
                    pass
        if not segs:
            return
        seg = segs[-1]
        with open(seg.path + ".idx", "rb") as f:
            raw = f.read()
        entries = [_IDX.unpack_from(raw, i) for i in range(0, len(raw) - len(raw) % 16, 16)]
        k = next((j for j, (bo, _ps) in enumerate(entries) if bo >= offset), None)
        if k is None:
            return                              # nothing of this segment is past the cut
        pos = entries[k][1]
        if seg.closed or seg.fd < 0:            # a rolled / recovered segment: append to it again
            seg.fd = os.open(seg.path + ".log", os.O_WRONLY | os.O_APPEND)
            seg.idx_fd = os.open(seg.path + ".idx", os.O_WRONLY | os.O_APPEND)
            seg.closed = False
        os.ftruncate(seg.fd, pos)
        os.ftruncate(seg.idx_fd, k * _IDX.size)
        seg.size, seg.nbatches, seg.last_end = pos, k, offset

    def _apply_retention(self, topic: str, partition: int, L: _Log) -> None:
        """Delete whole closed segments below the log start (in write order once serving)."""
        if self._writer_on:
            self._enqueue(("R", topic, partition, L.begin))
        else:
            self._retire_segments(topic, partition, L.begin)

    def _retire_segments(self, topic: str, partition: int, begin: int) -> None:
        segs = self._segs.get((topic, partition), [])
        while len(segs) > 1 and segs[0].last_end <= begin:
            seg = segs.pop(0)
            with self._lock:
                self._close_segment(seg)
            for ext in (".log", ".idx"):
                try:
                    os.unlink(seg.path + ext)
                except OSError:
                    pass

    def _persist_commit(self, group: str, topic: str, partition: int, offset: int) -> None:
        self._write_all(self._off_fd, (json.dumps({"g": group, "t": topic, "p": partition, "o": offset}) + "\n").encode())
        if self.fsync == "always":
            self._sync((self._off_fd,))
            self._dirty.discard(self._off_fd)

    def _persist_producer_ids(self) -> None:
        self._atomic_json("producers.json", {"next_producer_id": self._next_pid})

    def close(self) -> None:
        with self._wcv:                     # everything queued is written first
            self._wstop = True
            self._wcv.notify_all()
        self._writer.join(30)
        self._stop.set()
        if self._flusher is not None:
            self._flusher.join(5)
        self.flush()                        # retired segments' deferred fsync + close
        with self._lock:
            for segs in self._segs.values():
                for seg in segs:
                    self._close_segment(seg, now=True)
            if self._off_fd >= 0:
                os.fsync(self._off_fd)
                os.close(self._off_fd)
                self._off_fd = -1
            self._dirty.clear()

    def stats(self) -> Dict[str, object]:
        with self._lock:
            return {"data_dir": self.data_dir, "fsync": self.fsync, "bytes_written": self.bytes_written,
                    "fsyncs": self.fsyncs, "segments": sum(len(v) for v in self._segs.values()),
                    "recovered": self.recovered}
