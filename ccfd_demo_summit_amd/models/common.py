"""Shared model utilities: normalisation stats, bf16 rounding, blob helpers."""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

from ..contracts.transaction import AMOUNT_COL, N_FEATURES

KPAD = 32            # feature dim padded to one MFMA K-step (16x16x32)
HEADER_BYTES = 64

FLAG_LOG_AMOUNT = 1  # x[AMOUNT_COL] <- log1p(max(x, 0)) before normalisation
FLAG_WIRE = 2        # blob feature order is the W64 wire order (contracts.transaction.WIRE_PERM)


def bf16_round(x: np.ndarray) -> np.ndarray:
    """Round float32 -> bfloat16 (RNE) and back, like v_cvt_pk_bf16_f32."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32).reshape(x.shape)


def bf16_bits(x: np.ndarray) -> np.ndarray:
    """float32 -> uint16 bf16 bit patterns (RNE)."""
    return (bf16_round(x).view(np.uint32) >> 16).astype(np.uint16)


def sigmoid(z):
    z = np.asarray(z, dtype=np.float64)
    return (1.0 / (1.0 + np.exp(-z))).astype(np.float32)


@dataclass
class Normalizer:
    mu: np.ndarray          # float32 [30]
    inv_sigma: np.ndarray   # float32 [30]
    log_amount: bool = True

    @classmethod
    def fit(cls, X: np.ndarray, log_amount: bool = True) -> "Normalizer":
        Xt = cls._transform_raw(X, log_amount).astype(np.float64)
        mu = Xt.mean(0)
        sd = Xt.std(0)
        sd[sd < 1e-6] = 1.0
        return cls(mu.astype(np.float32), (1.0 / sd).astype(np.float32), log_amount)

    @classmethod
    def identity(cls) -> "Normalizer":
        return cls(np.zeros(N_FEATURES, np.float32), np.ones(N_FEATURES, np.float32), False)

    @staticmethod
    def _transform_raw(X: np.ndarray, log_amount: bool) -> np.ndarray:
        X = np.asarray(X, dtype=np.float32)
        if log_amount:
            X = X.copy()
            X[:, AMOUNT_COL] = np.log1p(np.maximum(X[:, AMOUNT_COL], 0.0))
        return X

    def __call__(self, X: np.ndarray) -> np.ndarray:
        Xt = self._transform_raw(X, self.log_amount)
        return ((Xt - self.mu) * self.inv_sigma).astype(np.float32)

    @property
    def flags(self) -> int:
        return FLAG_LOG_AMOUNT if self.log_amount else 0

    def packed(self, wire: bool = False) -> bytes:
        """mu[32] then inv_sigma[32] (lane group g reads entries 8g..8g+7); ``wire``
        permutes them to the W64 row order (contracts.transaction.WIRE_PERM)."""
        from ..contracts.transaction import WIRE_PERM
        mu = np.zeros(KPAD, np.float32)
        isg = np.zeros(KPAD, np.float32)
        perm = WIRE_PERM if wire else np.arange(N_FEATURES)
        mu[:N_FEATURES] = self.mu[perm]
        isg[:N_FEATURES] = self.inv_sigma[perm]
        return mu.tobytes() + isg.tobytes()

    def state(self) -> dict:
        return {"norm.mu": self.mu, "norm.inv_sigma": self.inv_sigma,
                "norm.log_amount": np.array([1 if self.log_amount else 0], np.int32)}

    @classmethod
    def from_state(cls, st: dict) -> "Normalizer":
        return cls(np.asarray(st["norm.mu"], np.float32), np.asarray(st["norm.inv_sigma"], np.float32),
                   bool(int(np.asarray(st["norm.log_amount"]).reshape(-1)[0])))


def header(magic: bytes, flags: int, *vals) -> bytes:
    """64-byte blob header: magic[4], flags u32, then up to 14 float32/int32 words."""
    assert len(magic) == 4
    words = b""
    for v in vals:
        words += struct.pack("<f", v) if isinstance(v, float) else struct.pack("<i", int(v))
    h = magic + struct.pack("<I", flags) + words
    assert len(h) <= HEADER_BYTES
    return h + b"\0" * (HEADER_BYTES - len(h))


def pad16(b: bytes) -> bytes:
    return b + b"\0" * ((-len(b)) % 16)
