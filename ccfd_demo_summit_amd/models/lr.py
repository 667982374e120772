"""Logistic-regression scorer (BASELINE.json config 1; the reference-topology model).

``p = sigmoid(w . normalize(x) + b)``.  Blob for csrc/kernels/score_lr.hip:
  [0,64) header 'LR01', flags, b (f32) | [64,192) mu[32] | [192,320) isg[32] | [320,448) w[32]
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from ..contracts.transaction import N_FEATURES
from .common import KPAD, Normalizer, header, sigmoid

BLOB_BYTES = 64 + 3 * KPAD * 4


@dataclass
class LogisticModel:
    w: np.ndarray      # [30]
    b: float
    norm: Normalizer
    kind: str = "lr"

    @classmethod
    def random_init(cls, seed: int = 0, norm: Optional[Normalizer] = None) -> "LogisticModel":
        rng = np.random.default_rng(seed)
        bound = 1.0 / np.sqrt(N_FEATURES)
        return cls(rng.uniform(-bound, bound, N_FEATURES).astype(np.float32),
                   float(rng.uniform(-bound, bound)), norm or Normalizer.identity())

    def logits(self, X: np.ndarray) -> np.ndarray:
        Xn = self.norm(X).astype(np.float64)
        return (Xn @ self.w.astype(np.float64) + self.b).astype(np.float32)

    def predict_proba(self, X: np.ndarray) -> np.ndarray:
        return sigmoid(self.logits(X))

    def predict_one(self, x) -> float:
        """batch=1 scalar path used by the CPU Seldon baseline (config 1)."""
        return float(self.predict_proba(np.asarray(x, np.float32).reshape(1, -1))[0])

    def calibrate_bias(self, X: np.ndarray, target_rate: float, threshold: float = 0.5) -> None:
        z = self.logits(X)
        self.b += float(np.log(threshold / (1 - threshold)) - np.quantile(z, 1.0 - target_rate))

    def pack(self, wire: bool = False) -> bytes:
        """``wire=True``: weights/normaliser in W64 row order (see models/mlp.py pack)."""
        from ..contracts.transaction import WIRE_PERM
        from .common import FLAG_WIRE
        w = np.zeros(KPAD, np.float32)
        w[:N_FEATURES] = self.w[WIRE_PERM] if wire else self.w
        blob = (header(b"LR01", self.norm.flags | (FLAG_WIRE if wire else 0), float(self.b))
                + self.norm.packed(wire) + w.tobytes())
        assert len(blob) == BLOB_BYTES
        return blob

    def state_dict(self) -> dict:
        st = {"lr.w": self.w, "lr.b": np.array([self.b], np.float32)}
        st.update(self.norm.state())
        return st

    @classmethod
    def from_state_dict(cls, st: dict) -> "LogisticModel":
        return cls(np.asarray(st["lr.w"], np.float32), float(np.asarray(st["lr.b"]).reshape(-1)[0]),
                   Normalizer.from_state(st))
