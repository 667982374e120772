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

``sink`` is anything with the ProcessEngine hand-off interface (``start_fraud_many`` /
``start_fraud`` / ``signal``): a ``KieClient`` (HTTP) or an in-process ``ProcessEngine``.
"""
from __future__ import annotations

import collections
import threading
import time
from typing import Any, Deque, Dict, List, Optional, Tuple

TRANSIENT_HTTP = (500, 502, 503, 504, 429, 408)


class HandoffError(RuntimeError):
    """A non-retryable KIE answer (4xx other than 408/429)."""


def _transient(e: BaseException) -> bool:
    try:
        import requests
        if isinstance(e, (requests.ConnectionError, requests.Timeout)):
            return True
        if isinstance(e, requests.HTTPError) and e.response is not None:
            return e.response.status_code in TRANSIENT_HTTP
    except ImportError:                    # pragma: no cover
        pass
    return isinstance(e, (ConnectionError, TimeoutError, OSError))


class KieHandoff:
    def __init__(self, sink, capacity: int = 1 << 21, max_batch: int = 4096, workers: int = 2,
                 backoff_s: float = 0.05, max_backoff_s: float = 2.0, metrics=None):
        self.sink = sink
        self.capacity = int(capacity)
        self.max_batch = int(max_batch)
        self.backoff_s = float(backoff_s)
        self.max_backoff_s = float(max_backoff_s)
        self.metrics = metrics
        self._cv = threading.Condition()
        # queue entries: (seq, kind, payload) -- kind "start" (list of variable dicts) or
        # "signal" ((instance_id, name, payload))
        self._q: Deque[Tuple[int, str, Any]] = collections.deque()
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
            self._q.append((seq, kind, payload))
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

    def submit_signal(self, instance_id: int, name: str, payload: Any) -> int:
        return self._push("signal", (int(instance_id), name, payload), 1)

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
        if kind == "signals":                       # consecutive signals, one request
            res = self.sink.signal_many(payload)
            ok = sum(1 for x in res if x)
            with self._cv:
                self.signals_ok += ok
                self.signals_stale += len(res) - ok
            return
        if kind == "start":
            many = getattr(self.sink, "start_fraud_many", None)
            if many is not None and len(payload) > 1:
                many(payload)
            else:
                for v in payload:
                    self.sink.start_fraud(v)
            return
        iid, name, body = payload
        ok = self.sink.signal(iid, name, body)
        with self._cv:
            if ok:
                self.signals_ok += 1
            else:
                self.signals_stale += 1

    def _run(self) -> None:
        while True:
            with self._cv:
                while not self._q and not self._stop:
                    self._cv.wait(0.1)
                if self._stop and not self._q:
                    return
                seq, kind, payload = self._q.popleft()
                seqs = [seq]
                if kind == "signal" and hasattr(self.sink, "signal_many"):
                    # coalesce the run of signals queued behind this one (customer responses
                    # arrive one per message; one HTTP request per signal would cap them)
                    batch = [payload]
                    while self._q and self._q[0][1] == "signal" and len(batch) < self.max_batch:
                        s2, _k, p2 = self._q.popleft()
                        seqs.append(s2)
                        batch.append(p2)
                    kind, payload = "signals", batch
            n_items = len(payload) if kind in ("start", "signals") else 1
            delay = self.backoff_s
            t_fail = None
            while True:
                try:
                    self._deliver(kind, payload)
                    break
                except BaseException as e:          # noqa: BLE001 -- classified below
                    if not _transient(e):
                        # a definite refusal (e.g. 404 unknown container): retrying cannot
                        # help; keep it for the operator instead of wedging the queue
                        with self._cv:
                            self.failed.append((kind, payload, repr(e)[:300]))
                            self.failed_total += 1
                            self.errors.append(repr(e)[:300])
                        break
                    with self._cv:
                        self.retries += 1
                        self.errors.append(repr(e)[:300])
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
            self._ack_many(seqs, n_items)

    def stats(self) -> Dict[str, Any]:
        with self._cv:
            return {"submitted": self.submitted_items, "acked": self.acked_items, "depth": self._queued_items,
                    "acked_seq": self.acked_seq, "last_seq": self._next_seq - 1, "retries": self.retries,
                    "signals_ok": self.signals_ok, "signals_stale": self.signals_stale,
                    "failed": self.failed_total, "outage_s": round(self.outage_s, 3)}
