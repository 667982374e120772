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
        """``wire=True``: weights in W64 row order with the WHOLE normaliser folded in
        (w' = w * isg, b' = b - sum w * isg * mu; the packed mu/isg become 0/1), so the wire
        kernel's dot product runs on the raw row values (bf16 V-columns, f32 Time, log1p'd
        Amount).  Generic kernels reading the same blob compute (x - 0) * 1 * w' -- the
        same function."""
        from ..contracts.transaction import WIRE_PERM
        from .common import FLAG_WIRE
        w = np.zeros(KPAD, np.float32)
        if wire:
            wd = self.w[WIRE_PERM].astype(np.float64) * self.norm.inv_sigma[WIRE_PERM].astype(np.float64)
            b = float(self.b) - float(wd @ self.norm.mu[WIRE_PERM].astype(np.float64))
            w[:N_FEATURES] = wd
            ident = Normalizer(np.zeros(N_FEATURES, np.float32), np.ones(N_FEATURES, np.float32),
                               self.norm.log_amount)
            blob = header(b"LR01", self.norm.flags | FLAG_WIRE, b) + ident.packed(True) + w.tobytes()
        else:
            w[:N_FEATURES] = self.w
            blob = header(b"LR01", self.norm.flags, float(self.b)) + self.norm.packed(False) + w.tobytes()
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
