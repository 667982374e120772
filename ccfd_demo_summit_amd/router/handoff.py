"""Non-blocking, failure-tolerant router -> KIE hand-off (README.md:552 "start a process
instance", :569/:605 "signal the process"; SURVEY.md §7.1 item 8 "pooled, async").

The reference router calls KIE synchronously per transaction; a GPU engine that scores
~1e9 tx/s hands off ~0.2 % of them (the fraud-routed rows) and must never stall scoring,
offset commits or the X2 collective schedule on a slow or absent KIE server.  Here:

* ``submit_starts(items)`` / ``submit_signal(...)`` enqueue and return at once with a
  sequence number; nothing on the caller's thread does network I/O;
* ``workers`` threads drain the queue in batches of up to ``max_batch`` starts, one
  ``POST .../instances/batch`` each, over a pooled HTTP client (the KIE analogue of
  ``SELDON_POOL_SIZE`` / ``SELDON_TIMEOUT``, README.md:386-393);
* a failed request (connection refused, timeout, 5xx) is retried with exponential back-off
  (capped) until it succeeds -- never dropped.  A retry of a request the server did process
  is harmless: fraud starts are idempotent per ``transaction_id`` (process/engine.py), so
  every fraud-routed transaction is started exactly once;
* ``acked_seq`` is the largest sequence number whose every item (and every earlier one) has
  been acknowledged.  The engine commits a Kafka offset only when the hand-off batch that
  carries its fraud rows is acknowledged (launch/engine_service.py), so a crash with a KIE
  outage in flight re-delivers instead of losing fraud starts (at-least-once + idempotent
  start = exactly-once);
* ``full()``: the queue holds ``capacity`` items; the engine stops scoring (its rings fill,
  its Kafka consumers stop fetching) until the queue drains -- back-pressure, never an
  exception out of the scoring step.

* standard-routed rows (``Router(standard_mode="process")``, the reference's "standard
  transaction process", README.md:552) go through the same queue as column batches
  (``submit_standard``) and gate the same offset commits;
* a NON-retryable answer (a 4xx other than 408/429, or a client-side error such as a
  malformed response) is never acknowledged silently: the request is first appended to the
  durable dead-letter journal (``DeadLetterQueue``: JSONL, fsync'd) and only then acked, so
  the Kafka offset that covers it is committed only after the DLQ holds it; with no DLQ
  configured the request is retried (held) like a transient failure and the operator sees
  ``refused`` grow -- scoring back-pressures instead of losing fraud cases.
  ``python -m ccfd_demo_summit_amd.launch dlq-replay`` re-delivers the journal, each entry
  exactly once;
* customer-response signals are coalesced into one ``signal/batch`` request; if the KIE
  server does not have that extension (404 / 405) the hand-off falls back, for good, to the
  standard per-instance ``/instances/{id}/signal/{name}`` route.

``sink`` is anything with the ProcessEngine hand-off interface (``start_fraud_many`` /
``start_fraud`` / ``start_standard_many`` / ``signal``): a ``KieClient`` (HTTP) or an
in-process ``ProcessEngine``.
"""
from __future__ import annotations

import collections
import json
import os
import threading
import time
from typing import Any, Deque, Dict, List, Optional, Tuple

from ..utils.lathist import LatHist

TRANSIENT_HTTP = (500, 502, 503, 504, 429, 408)
MISSING_ROUTE_HTTP = (404, 405, 501)


def _ncols(cols: Dict[str, Any]) -> int:
    return len(next(iter(cols.values()))) if cols else 0


def _concat_columns(parts: List[Dict[str, Any]]) -> Dict[str, Any]:
    import numpy as np
    return {k: np.concatenate([np.asarray(p[k]) for p in parts]) for k in parts[0]}


class HandoffError(RuntimeError):
    """A non-retryable KIE answer (4xx other than 408/429)."""


def _status(e: BaseException) -> Optional[int]:
    resp = getattr(e, "response", None)
    return getattr(resp, "status_code", None)


def _transient(e: BaseException) -> bool:
    """Worth retrying: the server could not be reached or answered 5xx / 408 / 429.  Every
    other error -- a 4xx, a non-JSON 200 body, an invalid URL, a ValueError -- is a definite
    refusal that no retry can fix (requests' exceptions all derive from IOError, so an
    ``OSError`` catch-all would retry those forever).  An in-process sink's back-pressure
    (e.g. process.dedupe.DedupeFull) says so with a ``transient`` attribute."""
    if getattr(e, "transient", False):
        return True
    try:
        import requests
        if isinstance(e, requests.HTTPError):
            st = _status(e)
            return st is None or st in TRANSIENT_HTTP
        if isinstance(e, (requests.ConnectionError, requests.Timeout)):
            return not isinstance(e, (requests.exceptions.InvalidURL, requests.exceptions.InvalidSchema,
                                      requests.exceptions.MissingSchema))
        if isinstance(e, requests.RequestException):
            return False
    except ImportError:                    # pragma: no cover
        pass
    if isinstance(e, ValueError):          # json.JSONDecodeError and friends
        return False
    return isinstance(e, (ConnectionError, TimeoutError))


def _jsonable(kind: str, payload: Any) -> Any:
    if kind == "standard":
        return {k: (v.tolist() if hasattr(v, "tolist") else list(v)) for k, v in payload.items()}
    if kind == "signal":
        iid, name, body = payload
        return [iid, name, body]
    if kind == "signals":
        return [list(x) for x in payload]
    return payload


def _from_json(kind: str, payload: Any) -> Any:
    if kind == "signal":
        return tuple(payload)
    if kind == "signals":
        return [tuple(x) for x in payload]
    return payload


class DeadLetterQueue:
    """Durable journal of hand-off requests KIE refused (README.md:552,558 hops that cannot
    complete).  One JSON line per refused request: ``{"dlq": id, "kind", "payload", "error",
    "ts"}``, fsync'd before ``put`` returns (the caller acks -- and the engine commits the Kafka
    offsets covering it -- only after that).  ``replay(sink)`` re-delivers the entries not yet
    replayed and appends ``{"replayed": id}`` after each success, so running it twice starts
    nothing twice (and fraud / standard starts are idempotent per transaction id at KIE)."""

    def __init__(self, path: str, fsync: bool = True):
        self.path = str(path)
        self.fsync = bool(fsync)
        d = os.path.dirname(os.path.abspath(self.path))
        os.makedirs(d, exist_ok=True)
        self._lock = threading.Lock()
        self._next = 0
        self.total = 0
        for rec in self._records():
            if "dlq" in rec:
                self._next = max(self._next, int(rec["dlq"]) + 1)
                self.total += 1
        self._f = open(self.path, "a", buffering=1)

    def _records(self):
        if not os.path.exists(self.path):
            return
        with open(self.path) as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                try:
                    yield json.loads(line)
                except json.JSONDecodeError:
                    continue                   # a torn last line (killed mid-write)

    def _append(self, rec: Dict[str, Any]) -> None:
        self._f.write(json.dumps(rec, default=float) + "\n")
        self._f.flush()
        if self.fsync:
            os.fsync(self._f.fileno())

    def put(self, kind: str, payload: Any, error: str) -> int:
        with self._lock:
            i = self._next
            self._next += 1
            self._append({"dlq": i, "kind": kind, "payload": _jsonable(kind, payload), "error": error[:500],
                          "ts": time.time()})
            self.total += 1
            return i

    def pending(self) -> List[Dict[str, Any]]:
        """Entries not yet replayed, oldest first."""
        done = set()
        ents = []
        for rec in self._records():
            if "replayed" in rec:
                done.add(int(rec["replayed"]))
            elif "dlq" in rec:
                ents.append(rec)
        return [e for e in ents if int(e["dlq"]) not in done]

    def replay(self, sink, stop_on_error: bool = True) -> Dict[str, int]:
        """Re-deliver every pending entry to ``sink`` (KieClient / ProcessEngine)."""
        ok = failed = 0
        for e in self.pending():
            try:
                deliver(sink, e["kind"], _from_json(e["kind"], e["payload"]))
            except BaseException:              # noqa: BLE001 -- reported, entry stays pending
                failed += 1
                if stop_on_error:
                    break
                continue
            with self._lock:
                self._append({"replayed": int(e["dlq"]), "ts": time.time()})
            ok += 1
        return {"replayed": ok, "failed": failed, "pending": len(self.pending())}

    def close(self) -> None:
        with self._lock:
            if not self._f.closed:
                self._f.close()


def deliver(sink, kind: str, payload: Any, batch_signals: bool = True) -> Tuple[int, int]:
    """One hand-off request to ``sink``; returns (signals ok, signals stale)."""
    if kind == "signals":
        if batch_signals and hasattr(sink, "signal_many"):
            res = sink.signal_many(payload)
        else:
            res = [sink.signal(iid, name, body) for iid, name, body in payload]
        ok = sum(1 for x in res if x)
        return ok, len(res) - ok
    if kind == "start":
        many = getattr(sink, "start_fraud_many", None)
        if many is not None and len(payload) > 1:
            many(payload)
        else:
            for v in payload:
                sink.start_fraud(v)
        return 0, 0
    if kind == "committed":
        note = getattr(sink, "note_committed", None)
        if note is not None:
            note(payload)
        return 0, 0
    if kind == "standard":
        many = getattr(sink, "start_standard_many", None)
        if many is not None:
            many(payload)
        else:
            from ..process.engine import rows_of
            for v in rows_of(payload):
                sink.start_standard(v)
        return 0, 0
    iid, name, body = payload
    ok = sink.signal(iid, name, body)
    return (1, 0) if ok else (0, 1)


class KieHandoff:
    def __init__(self, sink, capacity: int = 1 << 21, max_batch: int = 4096, workers: int = 2,
                 backoff_s: float = 0.05, max_backoff_s: float = 2.0, metrics=None,
                 dlq: Optional[DeadLetterQueue] = None, batch_signals: bool = True,
                 max_standard_batch: int = 16384):
        """``dlq``: where refused requests go before they are acked (None: a refused request
        is held and retried at ``max_backoff_s`` -- never acked unsent).  ``batch_signals``:
        coalesce response signals into the ``signal/batch`` extension (falls back to the
        per-instance route by itself when the server lacks it)."""
        self.sink = sink
        self.dlq = dlq
        self.batch_signals = bool(batch_signals) and hasattr(sink, "signal_many")
        self.commit_notices = True         # False once the server lacks instances/committed
        self.refused = 0                   # refusals seen (held or dead-lettered)
        self.dead_lettered = 0
        self.capacity = int(capacity)
        self.max_batch = int(max_batch)
        # standard starts (one a transaction in process mode, ~1e6/s): queued column batches are
        # coalesced into requests of up to this many rows -- per-request cost, not per-row
        # cost, is what the engine's side of the hand-off pays (HTTP + GIL)
        self.max_standard_batch = max(1, int(max_standard_batch))
        self.backoff_s = float(backoff_s)
        self.max_backoff_s = float(max_backoff_s)
        self.metrics = metrics
        self._cv = threading.Condition()
        # queue entries: (seq, kind, payload, pushed monotonic ns) -- kind "start" (list of
        # variable dicts), "standard" (columns) or "signal" ((instance_id, name, payload))
        self._q: Deque[Tuple[int, str, Any, int]] = collections.deque()
        # where a hand-off's time goes on this side: queued behind other requests, then the
        # request itself (HTTP round trip + the server's handler, retries included)
        self.queue_wait = LatHist()
        self.request_time = LatHist()
        self._queued_items = 0
        self._next_seq = 0
        self._done: set = set()            # acked seqs above the contiguous prefix
        self.acked_seq = -1                # every seq <= this is acknowledged
        self.submitted_items = 0
        self.acked_items = 0
        self.signals_ok = 0
        self.signals_stale = 0
        self.retries = 0
        self.errors: Deque[str] = collections.deque(maxlen=20)
        # non-retryable answers: the most recent are kept for the operator, all are counted
        self.failed: Deque[Tuple[str, Any, str]] = collections.deque(maxlen=1000)
        self.failed_total = 0
        self.outage_s = 0.0
        self._stop = False
        self._inflight = 0
        self._threads = [threading.Thread(target=self._run, daemon=True, name=f"kie-handoff-{i}")
                         for i in range(max(1, int(workers)))]
        for t in self._threads:
            t.start()

    # ------------------------------------------------------------------ producer side
    def _push(self, kind: str, payload: Any, n_items: int) -> int:
        with self._cv:
            seq = self._next_seq
            self._next_seq += 1
            self._q.append((seq, kind, payload, time.monotonic_ns()))
            self._queued_items += n_items
            self.submitted_items += n_items
            self._cv.notify()
            return seq

    def submit_starts(self, items: List[Dict[str, Any]]) -> int:
        """Enqueue fraud-process starts; returns the hand-off sequence number (-1: nothing)."""
        if not items:
            return self.last_seq()
        # split so one request never exceeds max_batch items (keeps server latency bounded)
        seq = -1
        for i in range(0, len(items), self.max_batch):
            chunk = items[i:i + self.max_batch]
            seq = self._push("start", chunk, len(chunk))
        return seq

    def submit_standard(self, cols: Dict[str, list]) -> int:
        """Enqueue standard-process starts (columns of equal length: transaction_id,
        customer_id, amount, proba); returns the hand-off sequence number."""
        n = len(next(iter(cols.values()))) if cols else 0
        if n == 0:
            return self.last_seq()
        seq = -1
        step = self.max_standard_batch
        for i in range(0, n, step):
            chunk = {k: v[i:i + step] for k, v in cols.items()}
            seq = self._push("standard", chunk, min(step, n - i))
        return seq

    def submit_signal(self, instance_id: int, name: str, payload: Any) -> int:
        return self._push("signal", (int(instance_id), name, payload), 1)

    def submit_committed(self, offsets: Dict[int, int]) -> int:
        """Queue a committed-offsets notice behind every start queued so far (it carries no
        items: it frees the shard's commit-gated dedupe keys, process/engine.py)."""
        return self._push("committed", {int(p): int(o) for p, o in offsets.items()}, 0)

    def last_seq(self) -> int:
        with self._cv:
            return self._next_seq - 1

    def depth(self) -> int:
        """Items queued or in flight (not yet acknowledged)."""
        with self._cv:
            return self._queued_items

    def full(self) -> bool:
        return self.depth() >= self.capacity

    def has_room(self, low_water: float = 0.5) -> bool:
        return self.depth() < self.capacity * low_water

    def acked(self, seq: int) -> bool:
        return seq <= self.acked_seq

    def drain(self, timeout_s: float = 30.0) -> bool:
        """Block until everything submitted so far is acknowledged (tests, shutdown)."""
        target = self.last_seq()
        t0 = time.monotonic()
        with self._cv:
            while self.acked_seq < target:
                if time.monotonic() - t0 > timeout_s:
                    return False
                self._cv.wait(0.05)
        return True

    def close(self, drain_s: float = 5.0) -> None:
        self.drain(drain_s)
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        for t in self._threads:
            t.join(2.0)

    # ------------------------------------------------------------------ worker side
    def _ack_many(self, seqs: List[int], n_items: int) -> None:
        with self._cv:
            self._done.update(seqs)
            while self.acked_seq + 1 in self._done:
                self._done.discard(self.acked_seq + 1)
                self.acked_seq += 1
            self._queued_items -= n_items
            self.acked_items += n_items
            self._cv.notify_all()

    def _deliver(self, kind: str, payload: Any) -> None:
        if kind == "committed":
            if not self.commit_notices:
                return
            try:
                deliver(self.sink, kind, payload)
            except BaseException as e:             # noqa: BLE001
                if _status(e) not in MISSING_ROUTE_HTTP:
                    raise
                # a KIE server without the extension keeps a count-window dedupe: stop telling it
                self.commit_notices = False
                with self._cv:
                    self.errors.append(f"instances/committed unsupported ({_status(e)})")
            return
        if kind == "signals" and self.batch_signals:
            try:
                ok, stale = deliver(self.sink, kind, payload, batch_signals=True)
            except BaseException as e:             # noqa: BLE001
                if _status(e) not in MISSING_ROUTE_HTTP:
                    raise
                # the KIE server has no signal/batch extension: use the standard
                # per-instance signal route from now on
                self.batch_signals = False
                with self._cv:
                    self.errors.append(f"signal/batch unsupported ({_status(e)}): per-instance signals")
                ok, stale = deliver(self.sink, kind, payload, batch_signals=False)
        else:
            ok, stale = deliver(self.sink, kind, payload, batch_signals=False)
        if ok or stale:
            with self._cv:
                self.signals_ok += ok
                self.signals_stale += stale

    def _run(self) -> None:
        while True:
            with self._cv:
                while not self._q and not self._stop:
                    self._cv.wait(0.1)
                if self._stop and not self._q:
                    return
                seq, kind, payload, t_push = self._q.popleft()
                seqs = [seq]
                if kind == "signal":
                    # coalesce the run of signals queued behind this one (customer responses
                    # arrive one per message; one HTTP request per signal would cap them)
                    batch = [payload]
                    while self._q and self._q[0][1] == "signal" and len(batch) < self.max_batch:
                        s2, _k, p2, _t = self._q.popleft()
                        seqs.append(s2)
                        batch.append(p2)
                    kind, payload = "signals", batch
                elif kind == "standard":
                    # coalesce the standard batches queued behind this one (same columns)
                    parts, rows = [payload], _ncols(payload)
                    while (self._q and self._q[0][1] == "standard" and set(self._q[0][2]) == set(payload)
                           and rows + _ncols(self._q[0][2]) <= self.max_standard_batch):
                        s2, _k, p2, _t = self._q.popleft()
                        seqs.append(s2)
                        parts.append(p2)
                        rows += _ncols(p2)
                    if len(parts) > 1:
                        payload = _concat_columns(parts)
                elif kind == "committed":
                    # a run of notices is one notice: offsets only grow, keep the max
                    payload = dict(payload)
                    while self._q and self._q[0][1] == "committed":
                        s2, _k, p2, _t = self._q.popleft()
                        seqs.append(s2)
                        for p, o in p2.items():
                            payload[p] = max(payload.get(p, o), o)
            n_items = len(payload) if kind in ("start", "signals") else \
                (len(next(iter(payload.values()))) if kind == "standard" and payload else
                 0 if kind == "committed" else 1)
            t_pop = time.monotonic_ns()
            self.queue_wait.add(t_pop - t_push)
            delay = self.backoff_s
            t_fail = None
            refused_once = False
            while True:
                try:
                    self._deliver(kind, payload)
                    break
                except BaseException as e:          # noqa: BLE001 -- classified below
                    err = repr(e)[:300]
                    if not _transient(e):
                        # a definite refusal (e.g. 404 unknown container): retrying cannot
                        # help.  Durable first, ack after: the offsets covering it are then
                        # committed with the request safe in the dead-letter journal
                        if not refused_once:
                            refused_once = True
                            with self._cv:
                                self.refused += 1
                                self.failed.append((kind, payload, err))
                                self.errors.append(err)
                        if self.dlq is not None:
                            try:
                                self.dlq.put(kind, payload, err)
                            except OSError as de:   # DLQ unwritable: hold, like an outage
                                with self._cv:
                                    self.errors.append(f"DLQ write failed: {de!r}"[:300])
                            else:
                                with self._cv:
                                    self.dead_lettered += n_items
                                    self.failed_total += 1
                                if self.metrics is not None and hasattr(self.metrics, "dead_letter"):
                                    self.metrics.dead_letter.inc(n_items)
                                break
                        delay = self.max_backoff_s  # no DLQ: hold (never ack an unsent request)
                    else:
                        with self._cv:
                            self.retries += 1
                            self.errors.append(err)
                        if self.metrics is not None:
                            self.metrics.retries.inc()
                    if t_fail is None:
                        t_fail = time.monotonic()
                    with self._cv:
                        if self._stop:
                            return
                    time.sleep(delay)
                    delay = min(self.max_backoff_s, delay * 2)
            if t_fail is not None:
                with self._cv:
                    self.outage_s += time.monotonic() - t_fail
            self.request_time.add(time.monotonic_ns() - t_pop)
            self._ack_many(seqs, n_items)

    def stats(self) -> Dict[str, Any]:
        with self._cv:
            return {"submitted": self.submitted_items, "acked": self.acked_items, "depth": self._queued_items,
                    "acked_seq": self.acked_seq, "last_seq": self._next_seq - 1, "retries": self.retries,
                    "signals_ok": self.signals_ok, "signals_stale": self.signals_stale,
                    "failed": self.failed_total, "refused": self.refused,
                    "dead_lettered": self.dead_lettered, "batch_signals": self.batch_signals,
                    "outage_s": round(self.outage_s, 3),
                    "queue_wait_us": self.queue_wait.summary_us(),
                    "request_us": self.request_time.summary_us()}


class ShardedHandoff:
    """The hand-off to a K-shard KIE tier (process/sharding.py): one ``KieHandoff`` per shard
    -- its own queue, workers, retries and dead-letter journal -- so a slow or restarting shard
    holds back only its own requests.  Starts are split by transaction-id shard, signals go to
    the shard that owns the instance id.

    Sequence numbers are global: ``submit_*`` returns ``g`` and records the vector of the
    shards' last sequence numbers at that moment; ``acked(g)`` holds once every shard has
    acknowledged up to its entry of that vector, i.e. everything submitted up to ``g`` -- the
    engine commits a Kafka offset only then, exactly as with one KIE server."""

    def __init__(self, sinks, dlqs: Optional[List[Optional[DeadLetterQueue]]] = None, **kw):
        if not sinks:
            raise ValueError("no KIE shards")
        dlqs = dlqs or [None] * len(sinks)
        self.shards = len(sinks)
        self.parts = [KieHandoff(s, dlq=d, **kw) for s, d in zip(sinks, dlqs)]
        self.capacity = self.parts[0].capacity
        self._lock = threading.Lock()
        self._g = -1
        self._marks: Deque[Tuple[int, Tuple[int, ...]]] = collections.deque()
        self._acked_g = -1

    # ------------------------------------------------------------------ producer side
    def _mark(self) -> int:
        self._g += 1
        self._marks.append((self._g, tuple(p.last_seq() for p in self.parts)))
        return self._g

    def submit_starts(self, items: List[Dict[str, Any]]) -> int:
        from ..process.sharding import shard_of_tx
        with self._lock:
            if not items:
                return self._g
            groups: Dict[int, List[Dict[str, Any]]] = {}
            for v in items:
                tx = v.get("transaction_id", v.get("tx_id"))
                groups.setdefault(0 if tx is None else shard_of_tx(int(tx), self.shards), []).append(v)
            for k, sub in groups.items():
                self.parts[k].submit_starts(sub)
            return self._mark()

    def submit_standard(self, cols: Dict[str, Any]) -> int:
        import numpy as np

        from ..process.sharding import shard_of_tx, split_columns, tx_column
        with self._lock:
            tx = tx_column(cols)
            if tx is None or not len(tx):
                return self._g
            sh = shard_of_tx(np.asarray(tx), self.shards)
            for k, sub in enumerate(split_columns(cols, sh, self.shards)):
                if sub is not None:
                    self.parts[k].submit_standard(sub)
            return self._mark()

    def submit_signal(self, instance_id: int, name: str, payload: Any) -> int:
        with self._lock:
            self.parts[int(instance_id) % self.shards].submit_signal(instance_id, name, payload)
            return self._mark()

    def submit_committed(self, offsets: Dict[int, int]) -> None:
        """Every shard admits standard starts of every partition: broadcast the notice."""
        with self._lock:
            for p in self.parts:
                p.submit_committed(offsets)

    def last_seq(self) -> int:
        with self._lock:
            return self._g

    def depth(self) -> int:
        return sum(p.depth() for p in self.parts)

    def full(self) -> bool:
        return any(p.full() for p in self.parts)

    def has_room(self, low_water: float = 0.5) -> bool:
        return all(p.has_room(low_water) for p in self.parts)

    def acked(self, seq: int) -> bool:
        with self._lock:
            if seq <= self._acked_g:
                return True
            acked = [p.acked_seq for p in self.parts]
            while self._marks and all(a >= v for a, v in zip(acked, self._marks[0][1])):
                self._acked_g = self._marks.popleft()[0]
            return seq <= self._acked_g

    @property
    def acked_seq(self) -> int:
        self.acked(self._acked_g + 1)
        return self._acked_g

    def drain(self, timeout_s: float = 30.0) -> bool:
        t_end = time.monotonic() + timeout_s
        return all(p.drain(max(0.0, t_end - time.monotonic())) for p in self.parts)

    def close(self, drain_s: float = 5.0) -> None:
        self.drain(drain_s)
        for p in self.parts:
            p.close(0.0)

    @property
    def queue_wait(self):
        from ..utils.lathist import merged
        return merged(p.queue_wait for p in self.parts)

    @property
    def request_time(self):
        from ..utils.lathist import merged
        return merged(p.request_time for p in self.parts)

    @property
    def refused(self) -> int:
        return sum(p.refused for p in self.parts)

    @property
    def dead_lettered(self) -> int:
        return sum(p.dead_lettered for p in self.parts)

    def stats(self) -> Dict[str, Any]:
        per = [p.stats() for p in self.parts]
        out: Dict[str, Any] = {"shards": self.shards}
        for k in ("submitted", "acked", "depth", "retries", "signals_ok", "signals_stale", "failed", "refused",
                  "dead_lettered"):
            out[k] = sum(int(s.get(k, 0)) for s in per)
        out["outage_s"] = round(sum(float(s.get("outage_s", 0.0)) for s in per), 3)
        out["acked_seq"] = self.acked_seq
        out["last_seq"] = self.last_seq()
        out["batch_signals"] = all(s.get("batch_signals") for s in per)
        out["queue_wait_us"] = self.queue_wait.summary_us()
        out["request_us"] = self.request_time.summary_us()
        out["per_shard"] = [{k: s[k] for k in ("submitted", "acked", "depth", "retries", "dead_lettered")}
                            for s in per]
        return out
