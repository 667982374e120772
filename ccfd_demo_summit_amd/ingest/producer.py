"""Transaction producer (replaces the reference's ``kafka-producer-dc``:
deploy/kafka/ProducerDeployment.yaml; README.md:461-485, 547-548).

Replays ``creditcard.csv`` (local path or S3 object ``s3bucket``/``filename``) or the
synthetic generator onto topic ``topic`` (default ``odh-demo``), either as one JSON
message per transaction (reference-compatible) or as packed TXB1 batches (hot path),
at a fixed rate or as fast as possible.  Env keys of the reference template are honoured
(``topic``, ``bootstrap``, ``s3endpoint``, ``s3bucket``, ``filename``).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Iterator, Optional

import numpy as np

from ..contracts.transaction import TxBatch, Transaction, encode_tx_json
from ..data.synthetic import SyntheticTxSource


@dataclass
class ProducerConfig:
    topic: str = "odh-demo"
    fmt: str = "json"              # json | txb1
    batch: int = 4096              # rows per TXB1 message / per produce loop
    rate_tx_s: float = 0.0         # 0 = max rate
    source: str = "synthetic"      # synthetic | csv | s3
    csv_path: Optional[str] = None
    seed: int = 0
    id_base: int = 0               # first transaction id (distinct per producer process)
    pool_rows: int = 65536         # synthetic JSON: distinct rows whose rendered bodies are cycled

    @classmethod
    def from_env(cls, environ=None) -> "ProducerConfig":
        e = os.environ if environ is None else environ
        c = cls(topic=e.get("topic", e.get("KAFKA_TOPIC", "odh-demo")))
        if e.get("filename") and os.path.exists(e["filename"]):
            c.source, c.csv_path = "csv", e["filename"]
        elif e.get("s3endpoint"):
            c.source = "s3"
        return c


def _batches(cfg: ProducerConfig) -> Iterator[TxBatch]:
    if cfg.source == "synthetic":
        yield from SyntheticTxSource(batch=cfg.batch, seed=cfg.seed)
        return
    if cfg.source == "csv":
        from ..data.csv_source import read_creditcard_csv
        X, y = read_creditcard_csv(cfg.csv_path)
    elif cfg.source == "s3":
        from .s3 import fetch_creditcard_from_env
        X, y = fetch_creditcard_from_env()
    else:
        raise ValueError(f"unknown source {cfg.source}")
    n = X.shape[0]
    base = 0
    while True:                           # replay the file forever, like the demo producer
        for s in range(0, n, cfg.batch):
            e = min(n, s + cfg.batch)
            m = e - s
            yield TxBatch(ids=np.arange(base, base + m, dtype=np.uint64),
                          customer=(np.arange(base, base + m) % 100_000).astype(np.uint32),
                          features=X[s:e], labels=None if y is None else y[s:e], base_offset=base)
            base += m


def json_tail(customer_id: int, features) -> bytes:
    """The part of a transaction's JSON message after its id (contracts/transaction.py
    field names): ``,"customer_id":..,"Time":..,"V1":..,...,"Amount":..}``."""
    from ..contracts import FEATURE_NAMES
    return ((',"customer_id":%d,' % int(customer_id)) + ",".join(
        f'"{n}":{float(v):.7g}' for n, v in zip(FEATURE_NAMES, features)) + "}").encode()


class TransactionProducer:
    """``fmt="json"``: one JSON transaction per Kafka message -- the reference's wire format
    (README.md:547-548) -- produced a batch of messages per partition request
    (``produce_many``: one RecordBatch of ``batch`` records), round-robin over the topic's
    partitions.  Synthetic rows: the bodies of ``pool_rows`` distinct generated transactions
    are rendered once and cycled with fresh ids (rendering 30 floats per message in Python
    would cap one producer at ~1e5 msg/s; the engine still parses every message in full);
    CSV / S3 rows are rendered as read."""

    def __init__(self, broker, cfg: ProducerConfig):
        self.broker = broker
        self.cfg = cfg
        self.sent = 0
        self._it = _batches(cfg)
        self._seq = 0
        self._tails = None
        self._n_parts = None

    def _partitions(self) -> int:
        if self._n_parts is None:
            try:
                self._n_parts = max(1, int(self.broker.partitions(self.cfg.topic)))
            except Exception:
                self._n_parts = 1
        return self._n_parts

    def _ensure_pool(self) -> None:
        if self._tails is None:
            from ..data.synthetic import generate
            n = max(self.cfg.batch, self.cfg.pool_rows)
            X, _ = generate(n, seed=self.cfg.seed + 31)
            self._tails = [json_tail(i % 100_000, X[i]) for i in range(n)]

    def _txb1_pooled(self) -> TxBatch:
        """Synthetic TXB1: the features / customers of ``pool_rows`` generated transactions
        are cycled a batch at a time with fresh ids (like the JSON pool).  Generating 4096 new
        rows per batch was ~30 % of a producer process's time and capped it at ~1.7 x 10^6
        tx/s in the deployed topology (profiles/r4/kie_handoff/)."""
        c = self.cfg
        if getattr(self, "_txb1_pool", None) is None:
            from ..data.synthetic import generate
            nb = max(1, c.pool_rows // c.batch)
            X, y = generate(nb * c.batch, seed=c.seed + 31)
            rng = np.random.default_rng(c.seed + 7919)
            cust = rng.integers(0, 1_000_000, nb * c.batch, dtype=np.uint32)
            self._txb1_pool = (nb, X, y, cust)
        nb, X, y, cust = self._txb1_pool
        k = (self._seq % nb) * c.batch
        base = c.id_base + self.sent
        return TxBatch(ids=np.arange(base, base + c.batch, dtype=np.uint64), customer=cust[k:k + c.batch],
                       features=X[k:k + c.batch], labels=y[k:k + c.batch], base_offset=base)

    def _native_json_record_set(self) -> Optional[bytearray]:
        """One RecordBatch of ``batch`` JSON messages built natively (ids formatted in C++,
        csrc/engine/kafka_codec.cpp ccfd_kafka_encode_json_batch); None without the library."""
        if getattr(self, "_nat", None) is None:
            try:
                import ctypes as C
                from ..ingest.kafka_wire import _native_encoder
                L = _native_encoder()
                if not L:
                    raise RuntimeError("no native encoder")
                L.ccfd_kafka_encode_json_batch.argtypes = [C.c_char_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64,
                                                           C.c_uint64, C.c_int64, C.c_void_p, C.c_int64]
                L.ccfd_kafka_encode_json_batch.restype = C.c_int64
                self._ensure_pool()
                pool = b"".join(self._tails)
                off = np.zeros(len(self._tails) + 1, np.int64)
                np.cumsum([len(t) for t in self._tails], out=off[1:])
                cap = int(L.ccfd_kafka_batch_bound(self.cfg.batch, int(off[1:].max() if len(off) > 1 else 0)
                                                   * self.cfg.batch + 32 * self.cfg.batch))
                self._nat = (L, pool, off, np.zeros(cap, np.uint8))
            except Exception:
                self._nat = False
        if not self._nat:
            return None
        L, pool, off, out = self._nat
        c = self.cfg
        start = (self._seq * c.batch) % (len(off) - 1)
        k = L.ccfd_kafka_encode_json_batch(pool, off.ctypes.data, len(off) - 1, start, c.batch,
                                           c.id_base + self.sent, int(time.time() * 1000), out.ctypes.data, out.size)
        if k <= 0:
            raise RuntimeError("ccfd_kafka_encode_json_batch failed")
        return bytearray(out[:k])           # mutable: an idempotent producer stamps it in place

    def _json_batch(self) -> list:
        c = self.cfg
        base = c.id_base + self.sent
        if c.source == "synthetic" and hasattr(self.broker, "produce_many"):
            self._ensure_pool()
            k0 = (self._seq * c.batch) % len(self._tails)
            tails = self._tails[k0:k0 + c.batch]
            if len(tails) < c.batch:
                tails = tails + self._tails[:c.batch - len(tails)]
            return [b'{"id":%d' % (base + i) + t for i, t in enumerate(tails)]
        b = next(self._it)
        return [b'{"id":%d' % (base + i) + json_tail(b.customer[i], b.features[i]) for i in range(len(b))]

    def produce(self, n_tx: int, until: Optional[float] = None) -> int:
        """Produce at least ``n_tx`` transactions (rate-limited if configured); with ``until``
        (time.perf_counter deadline) stop there instead."""
        t0 = time.perf_counter()
        done = 0
        many = hasattr(self.broker, "produce_many")
        while done < n_tx and (until is None or time.perf_counter() < until):
            if self.cfg.fmt == "txb1":
                if self.cfg.source == "synthetic":
                    b = self._txb1_pooled()
                else:
                    b = next(self._it)
                    if self.cfg.id_base:
                        b.ids[:] = b.ids + np.uint64(self.cfg.id_base)
                self.broker.produce(self.cfg.topic, b.encode(), key=str(int(b.ids[0])).encode())
                k = len(b)
            elif many and self.cfg.source == "synthetic" and hasattr(self.broker, "produce_raw") and \
                    (rs := self._native_json_record_set()) is not None:
                self.broker.produce_raw(self.cfg.topic, self._seq % self._partitions(), rs)
                k = self.cfg.batch
            elif many:
                msgs = self._json_batch()
                self.broker.produce_many(self.cfg.topic, msgs, partition=self._seq % self._partitions())
                k = len(msgs)
            else:
                b = next(self._it)
                for tx in b.transactions():
                    self.broker.produce(self.cfg.topic, encode_tx_json(tx), key=str(tx.customer_id).encode())
                k = len(b)
            self._seq += 1
            done += k
            self.sent += k
            if self.cfg.rate_tx_s > 0:
                ahead = done / self.cfg.rate_tx_s - (time.perf_counter() - t0)
                if ahead > 0:
                    time.sleep(ahead)
        return done


class BatchingPublisher:
    """Fire-and-forget publisher for low-rate side topics (the KIE's CustomerNotification
    messages, README.md:560): ``publish`` enqueues; a daemon thread sends what accumulated as
    one ``produce_many`` RecordBatch every ``linger_s`` (Kafka's linger.ms) instead of one
    produce request per message on the caller's thread -- at 1e6 tx/s the fraud process
    publishes ~2e3 notifications/s.

    ``publish(value, token)``: ``on_sent(tokens)`` is called (publisher thread) with the tokens
    of every batch once the broker acknowledged it -- the KIE outbox clears a notification
    only then, the notifier commits a consumed offset only then (at-least-once hand-over,
    made exactly-once by idempotent produce + consumer-side dedupe)."""

    def __init__(self, broker, topic: str, linger_s: float = 0.002, max_batch: int = 4096, on_sent=None):
        import collections
        import threading
        self.broker = broker
        self.topic = topic
        self.linger_s = linger_s
        self.max_batch = max_batch
        self._q = collections.deque()
        self._cv = threading.Condition()
        self._stop = False
        self.sent = 0
        self.errors = 0
        self._n_parts = None
        self._rr = 0
        self.on_sent = on_sent
        self._th = threading.Thread(target=self._run, daemon=True, name=f"publish-{topic}")
        self._th.start()

    def publish(self, value: bytes, token=None) -> None:
        with self._cv:
            self._q.append((value, token))
            if len(self._q) >= self.max_batch:
                self._cv.notify()

    def _run(self):
        retry = None                          # a batch whose send failed: re-sent AS IS first
        while True:
            if retry is not None:
                batch, retry = retry, None
            else:
                with self._cv:
                    if not self._q and not self._stop:
                        self._cv.wait(self.linger_s)
                    if self._stop and not self._q:
                        return
                    batch = [self._q.popleft() for _ in range(min(len(self._q), self.max_batch))]
            if not batch:
                continue
            try:
                values = [v for v, _t in batch]
                if hasattr(self.broker, "produce_many"):
                    if self._n_parts is None:
                        self._n_parts = max(1, int(self.broker.partitions(self.topic)))
                    self.broker.produce_many(self.topic, values, partition=self._rr % self._n_parts)
                    self._rr += 1
                else:
                    for v in values:
                        self.broker.produce(self.topic, v)
                self.sent += len(batch)
                if self.on_sent is not None:
                    toks = [t for _v, t in batch if t is not None]
                    if toks:
                        self.on_sent(toks)
            except Exception:                 # broker unavailable: retry the SAME batch later
                # (an idempotent producer re-sends it under the same sequence number, so a batch
                # the broker stored before the failure is not stored twice -- and no message
                # joins it, which would be dropped with the duplicate)
                self.errors += 1
                retry = batch
                if self._stop:
                    with self._cv:
                        self._q.extendleft(reversed(batch))
                    return
                time.sleep(0.05)

    def pending(self) -> int:
        with self._cv:
            return len(self._q)

    def close(self, timeout_s: float = 5.0) -> None:
        t0 = time.time()
        while self._q and time.time() - t0 < timeout_s:
            time.sleep(0.01)
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._th.join(timeout_s)

