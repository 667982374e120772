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


class TransactionProducer:
    def __init__(self, broker, cfg: ProducerConfig):
        self.broker = broker
        self.cfg = cfg
        self.sent = 0
        self._it = _batches(cfg)

    def produce(self, n_tx: int) -> int:
        """Produce at least ``n_tx`` transactions (rate-limited if configured)."""
        t0 = time.perf_counter()
        done = 0
        while done < n_tx:
            b = next(self._it)
            if self.cfg.fmt == "txb1":
                self.broker.produce(self.cfg.topic, b.encode(), key=str(int(b.ids[0])).encode())
            else:
                for tx in b.transactions():
                    self.broker.produce(self.cfg.topic, encode_tx_json(tx), key=str(tx.customer_id).encode())
            done += len(b)
            self.sent += len(b)
            if self.cfg.rate_tx_s > 0:
                ahead = done / self.cfg.rate_tx_s - (time.perf_counter() - t0)
                if ahead > 0:
                    time.sleep(ahead)
        return done
