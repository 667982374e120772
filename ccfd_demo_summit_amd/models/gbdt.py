"""Oblivious gradient-boosted decision trees (BASELINE.json config 4: 100 trees x depth 6).

In an oblivious (symmetric) tree every node of one level tests the same
``x[feat] > thr``, so the leaf index of a row is ``sum_d bit_d << d`` -- six compares and
shifts, no pointer chasing, and the split of a level is the same for every row of a
wavefront (scalar/SGPR operands in csrc/kernels/score_gbdt.hip).

``proba = sigmoid(base + sum_t leaves[t][idx_t(x)])`` on RAW features (trees are scale
invariant, no normalisation).

Blob for the kernel (16-B aligned sections):
  [0,64)  header 'GBT1', flags, T (i32), D (i32), base (f32)
  feat    i32  [T][D]
  thr     f32  [T][D]
  leaves  f32  [T][2^D]
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ..contracts.transaction import N_FEATURES
from .common import HEADER_BYTES, header, pad16, sigmoid

MAX_DEPTH = 8


@dataclass
class ObliviousGBDT:
    feat: np.ndarray     # int32 [T, D]
    thr: np.ndarray      # float32 [T, D]
    leaves: np.ndarray   # float32 [T, 2^D]
    base: float = 0.0
    kind: str = "gbdt"

    def __post_init__(self):
        self.feat = np.ascontiguousarray(self.feat, np.int32)
        self.thr = np.ascontiguousarray(self.thr, np.float32)
        self.leaves = np.ascontiguousarray(self.leaves, np.float32)
        T, D = self.feat.shape
        if not 1 <= D <= MAX_DEPTH:
            raise ValueError(f"depth must be in [1,{MAX_DEPTH}]")
        if self.thr.shape != (T, D) or self.leaves.shape != (T, 1 << D):
            raise ValueError("inconsistent tree arrays")
        if self.feat.min(initial=0) < 0 or self.feat.max(initial=0) >= N_FEATURES:
            raise ValueError("feature index out of range")

    @property
    def n_trees(self) -> int:
        return int(self.feat.shape[0])

    @property
    def depth(self) -> int:
        return int(self.feat.shape[1])

    @classmethod
    def random_init(cls, n_trees: int = 100, depth: int = 6, seed: int = 0,
                    X_ref: Optional[np.ndarray] = None) -> "ObliviousGBDT":
        """Random oblivious ensemble; split thresholds drawn from feature quantiles of
        ``X_ref`` (or N(0,1)) so that every split actually partitions the data."""
        rng = np.random.default_rng(seed)
        feat = rng.integers(0, N_FEATURES, (n_trees, depth), dtype=np.int32)
        if X_ref is not None:
            q = rng.uniform(0.05, 0.95, (n_trees, depth))
            thr = np.empty((n_trees, depth), np.float32)
            for t in range(n_trees):
                for d in range(depth):
                    thr[t, d] = np.quantile(X_ref[:, feat[t, d]], q[t, d])
        else:
            thr = rng.standard_normal((n_trees, depth)).astype(np.float32)
        leaves = (rng.standard_normal((n_trees, 1 << depth)) * 0.1).astype(np.float32)
        return cls(feat, thr, leaves, 0.0)

    def leaf_index(self, X: np.ndarray) -> np.ndarray:
        X = np.asarray(X, np.float32)
        bits = X[:, self.feat] > self.thr[None]             # [n, T, D]
        return (bits.astype(np.int64) << np.arange(self.depth)).sum(-1)   # [n, T]

    def raw_score(self, X: np.ndarray) -> np.ndarray:
        idx = self.leaf_index(X)
        vals = self.leaves[np.arange(self.n_trees)[None, :], idx]
        return (self.base + vals.astype(np.float64).sum(1)).astype(np.float32)

    def predict_proba(self, X: np.ndarray) -> np.ndarray:
        return sigmoid(self.raw_score(X))

    def calibrate_bias(self, X: np.ndarray, target_rate: float, threshold: float = 0.5) -> None:
        z = self.raw_score(X)
        self.base += float(np.log(threshold / (1 - threshold)) - np.quantile(z, 1.0 - target_rate))

    def pack(self) -> bytes:
        T, D = self.feat.shape
        blob = header(b"GBT1", 0, T, D, float(self.base))
        blob += pad16(self.feat.tobytes()) + pad16(self.thr.tobytes()) + pad16(self.leaves.tobytes())
        return blob

    @staticmethod
    def blob_offsets(T: int, D: int):
        def a16(x):
            return (x + 15) & ~15
        off_feat = HEADER_BYTES
        off_thr = off_feat + a16(4 * T * D)
        off_leaf = off_thr + a16(4 * T * D)
        end = off_leaf + a16(4 * T * (1 << D))
        return off_feat, off_thr, off_leaf, end

    @classmethod
    def unpack(cls, blob: bytes) -> "ObliviousGBDT":
        magic = blob[:4]
        if magic != b"GBT1":
            raise ValueError("not a GBT1 blob")
        T, D = struct.unpack_from("<ii", blob, 8)
        base = struct.unpack_from("<f", blob, 16)[0]
        of, ot, ol, _ = cls.blob_offsets(T, D)
        feat = np.frombuffer(blob, np.int32, T * D, of).reshape(T, D)
        thr = np.frombuffer(blob, np.float32, T * D, ot).reshape(T, D)
        leaves = np.frombuffer(blob, np.float32, T << D, ol).reshape(T, 1 << D)
        return cls(feat.copy(), thr.copy(), leaves.copy(), float(base))

    def state_dict(self) -> dict:
        return {"gbdt.feat": self.feat, "gbdt.thr": self.thr, "gbdt.leaves": self.leaves,
                "gbdt.base": np.array([self.base], np.float32)}

    @classmethod
    def from_state_dict(cls, st: dict) -> "ObliviousGBDT":
        return cls(st["gbdt.feat"], st["gbdt.thr"], st["gbdt.leaves"],
                   float(np.asarray(st["gbdt.base"]).reshape(-1)[0]))
