"""Synthetic credit-card transaction generator shaped like the Kaggle dataset.

The reference producer replays ``creditcard.csv`` from S3 onto ``odh-demo``
(README.md:461-485, 547-548; deploy/kafka/ProducerDeployment.yaml:88-97).  There is no
network here, so we generate rows with the same schema and roughly the same marginal
statistics [EXT: public dataset description]: ``Time`` in seconds over two days,
``V1..V28`` PCA components with decreasing spread, a heavy-tailed ``Amount`` and a
0.172 % positive class whose mean is shifted on the known fraud-indicative components.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterator, Optional

import numpy as np

from ..contracts.transaction import N_FEATURES, TxBatch

FRAUD_RATE = 0.00172
TIME_SPAN_S = 172792.0
# per-component standard deviations of V1..V28 (approximate dataset values, [EXT])
V_STD = np.array([1.96, 1.65, 1.52, 1.42, 1.38, 1.33, 1.24, 1.19, 1.10, 1.09, 1.02, 1.00,
                  1.00, 0.96, 0.92, 0.88, 0.85, 0.84, 0.81, 0.77, 0.73, 0.73, 0.62, 0.61,
                  0.52, 0.48, 0.40, 0.33], dtype=np.float32)
# class-conditional mean shift for fraud rows on V1..V28 ([EXT], rounded)
V_FRAUD_SHIFT = np.zeros(28, np.float32)
for _i, _s in {1: -4.8, 2: 3.6, 3: -7.0, 4: 4.5, 5: -3.2, 6: -1.4, 7: -5.6, 9: -2.6,
               10: -5.7, 11: 3.8, 12: -6.3, 14: -7.0, 16: -4.1, 17: -6.7, 18: -2.2}.items():
    V_FRAUD_SHIFT[_i - 1] = _s
AMOUNT_LOG_MU, AMOUNT_LOG_SIGMA, AMOUNT_MAX = 3.0, 1.6, 25691.16


def generate(n: int, seed: int = 0, fraud_rate: float = FRAUD_RATE, start_time: float = 0.0,
             out: Optional[np.ndarray] = None, with_labels: bool = True):
    """Return (features float32 [n,30], labels uint8 [n]).  ``out`` may be a preallocated
    (e.g. pinned) [n,30] float32 buffer, filled in place in chunks."""
    rng = np.random.default_rng(seed)
    X = out if out is not None else np.empty((n, N_FEATURES), np.float32)
    assert X.shape == (n, N_FEATURES) and X.dtype == np.float32
    y = np.empty(n, np.uint8)
    chunk = 1 << 20
    t0 = start_time
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        lab = (rng.random(m) < fraud_rate)
        v = rng.standard_normal((m, 28), dtype=np.float32) * V_STD
        v[lab] += V_FRAUD_SHIFT * rng.uniform(0.15, 1.2, (int(lab.sum()), 1)).astype(np.float32)
        amt = np.exp(rng.normal(AMOUNT_LOG_MU, AMOUNT_LOG_SIGMA, m)).astype(np.float32)
        amt[lab] *= rng.uniform(0.3, 3.0, int(lab.sum())).astype(np.float32)
        np.minimum(amt, AMOUNT_MAX, out=amt)
        amt = np.round(amt, 2)
        dt = TIME_SPAN_S / max(n, 1)
        t = (t0 + dt * np.arange(m, dtype=np.float64)).astype(np.float32)
        t0 += dt * m
        X[s:s + m, 0] = t
        X[s:s + m, 1:29] = v
        X[s:s + m, 29] = amt
        y[s:s + m] = lab
    return X, y


@dataclass
class SyntheticTxSource:
    """Endless stream of TXB1 micro-batches (the producer side of topic ``odh-demo``)."""
    batch: int = 4096
    seed: int = 0
    fraud_rate: float = FRAUD_RATE
    n_customers: int = 1_000_000
    first_id: int = 0

    def __iter__(self) -> Iterator[TxBatch]:
        k = 0
        nid = self.first_id
        rng = np.random.default_rng(self.seed + 7919)
        while True:
            X, y = generate(self.batch, seed=self.seed * 1_000_003 + k, fraud_rate=self.fraud_rate)
            ids = np.arange(nid, nid + self.batch, dtype=np.uint64)
            cust = rng.integers(0, self.n_customers, self.batch, dtype=np.uint32)
            yield TxBatch(ids=ids, customer=cust, features=X, labels=y, base_offset=nid)
            nid += self.batch
            k += 1
