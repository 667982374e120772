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

G32 rows (contracts/transaction.py, csrc/kernels/score_gbdt_g32.hip) carry one byte per
feature: its bin against a ``BinSpec`` (the ensemble's sorted split thresholds per
feature).  The 'GBB1' blob replaces ``thr`` by the split's bin index ``k`` (i32), so the
kernel's ``bin > k`` is exactly the f32 ``x > thr``; header word 5 is the spec's stamp.
"""
from __future__ import annotations

import struct
import zlib
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from ..contracts.transaction import N_FEATURES
from .common import HEADER_BYTES, header, pad16, sigmoid

MAX_DEPTH = 8
MAX_BINS = 255          # split thresholds per feature a G32 byte can index
G20_MAX_EDGES = 31      # ... and a G20 five-bit field (contracts/transaction.py encode_g20)


@dataclass
class BinSpec:
    """Per-feature bin edges of the G32 row format: ascending, distinct float32 thresholds
    (<= 255 per feature).  ``stamp`` (1..255) is written into every encoded row and into
    the GBB1 blob; the kernel refuses rows whose stamp differs (CCFD_CNT_WIRE_STALE).

    A model can be packed against any spec whose edges CONTAIN its thresholds -- e.g. a
    retrained ensemble against the spec the live partition logs were encoded with, so a hot
    swap needs no re-encoding while the split set stays inside it."""
    edges: List[np.ndarray]
    bits: int = 8            # 8: G32 rows (u8 bins); 5: G20 rows (<= 31 edges per feature)

    def __post_init__(self):
        if len(self.edges) != N_FEATURES:
            raise ValueError(f"need bin edges for all {N_FEATURES} features")
        if self.bits not in (8, 5):
            raise ValueError("bin width is 8 (G32 rows) or 5 (G20 rows)")
        cap = MAX_BINS if self.bits == 8 else G20_MAX_EDGES
        out = []
        for j, e in enumerate(self.edges):
            e = np.ascontiguousarray(e, np.float32).reshape(-1)
            if e.size > cap:
                raise ValueError(f"feature {j}: {e.size} split thresholds > {cap} "
                                 f"({'G32 bins are u8' if self.bits == 8 else 'G20 bins are 5 bits'})")
            if np.isnan(e).any() or (e.size > 1 and not (np.diff(e) > 0).all()):
                raise ValueError(f"feature {j}: bin edges must be ascending, distinct and not NaN")
            out.append(e)
        self.edges = out

    @classmethod
    def from_thresholds(cls, feat: np.ndarray, thr: np.ndarray) -> "BinSpec":
        feat = np.asarray(feat).reshape(-1)
        thr = np.asarray(thr, np.float32).reshape(-1)
        t = [thr[feat == j] for j in range(N_FEATURES)]
        return cls([np.unique(e[~np.isnan(e)]) for e in t])     # NaN splits never fire: k = 255

    @property
    def row_format(self) -> str:
        return "g32" if self.bits == 8 else "g20"

    @property
    def fits_g20(self) -> bool:
        return all(e.size <= G20_MAX_EDGES for e in self.edges)

    def with_bits(self, bits: int) -> "BinSpec":
        """The same edges for the other row format (ValueError if they do not fit)."""
        return BinSpec([e.copy() for e in self.edges], bits=bits)

    @property
    def offsets(self) -> np.ndarray:
        off = np.zeros(N_FEATURES + 1, np.int32)
        np.cumsum([e.size for e in self.edges], out=off[1:])
        return off

    @property
    def flat(self) -> np.ndarray:
        return np.concatenate(self.edges).astype(np.float32) if any(e.size for e in self.edges) \
            else np.zeros(1, np.float32)

    @property
    def stamp(self) -> int:
        """1..255 digest of the edge table (1..63 for G20 rows, whose stamp field is 6 bits;
        0 is never valid: zeroed memory is stale)."""
        h = zlib.crc32(self.offsets.tobytes() + self.flat.tobytes())
        return 1 + h % (255 if self.bits == 8 else 63)

    def bin_index(self, feat: np.ndarray, thr: np.ndarray) -> np.ndarray:
        """k with edges[feat][k] == thr for every split (ValueError if a threshold is missing)."""
        feat = np.asarray(feat)
        thr = np.asarray(thr, np.float32)
        k = np.empty(feat.shape, np.int32)
        for idx in np.ndindex(feat.shape):
            if np.isnan(thr[idx]):            # `x > NaN` is always false: no u8 bin exceeds 255
                k[idx] = MAX_BINS
                continue
            e = self.edges[int(feat[idx])]
            i = int(np.searchsorted(e, thr[idx]))
            if i >= e.size or e[i] != thr[idx]:
                raise ValueError(f"split threshold {float(thr[idx])!r} of feature {int(feat[idx])} "
                                 "is not a bin edge of this spec")
            k[idx] = i
        return k

    def encode(self, X: np.ndarray) -> np.ndarray:
        """numpy oracle of the native encoder: f32 [n,30] -> u8 [n,32] G32 rows (or u8 [n,20]
        G20 rows for a 5-bit spec)."""
        from ..contracts.transaction import encode_g20, encode_g32
        return (encode_g32 if self.bits == 8 else encode_g20)(X, self.edges, self.stamp)

    def to_bytes(self) -> bytes:
        """offsets i32[31] + edges f32[...] (the X1 broadcast payload next to the blob)."""
        return self.offsets.tobytes() + np.concatenate(self.edges + [np.zeros(0, np.float32)]).tobytes()

    @classmethod
    def from_bytes(cls, b: bytes, bits: int = 8) -> "BinSpec":
        off = np.frombuffer(b, np.int32, N_FEATURES + 1)
        e = np.frombuffer(b, np.float32, int(off[-1]), 4 * (N_FEATURES + 1))
        return cls([e[off[j]:off[j + 1]].copy() for j in range(N_FEATURES)], bits=bits)

    def contains(self, other: "BinSpec") -> bool:
        return all(np.isin(o, e).all() for o, e in zip(other.edges, self.edges))


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

    def leaf_index_g32(self, rows: np.ndarray, bins: Optional["BinSpec"] = None) -> np.ndarray:
        """Leaf indices from G32 rows (u8 [n,32], ``BinSpec.encode``) -- the device kernel's
        form of every level, ``bin[f] > k`` with k the threshold's edge index -- [n, T]."""
        spec = bins if bins is not None else self.bin_spec()
        k = spec.bin_index(self.feat, self.thr)              # [T, D]; NaN thresholds: 255
        if spec.bits == 5:
            from ..contracts.transaction import decode_g20_bins
            b = decode_g20_bins(rows).astype(np.int32)
        else:
            b = np.asarray(rows, np.uint8)[:, :N_FEATURES].astype(np.int32)
        bits = b[:, self.feat] > k[None]
        return (bits.astype(np.int64) << np.arange(self.depth)).sum(-1)

    def raw_score(self, X: np.ndarray) -> np.ndarray:
        idx = self.leaf_index(X)
        vals = self.leaves[np.arange(self.n_trees)[None, :], idx]
        return (self.base + vals.astype(np.float64).sum(1)).astype(np.float32)

    def predict_proba(self, X: np.ndarray) -> np.ndarray:
        return sigmoid(self.raw_score(X))

    def calibrate_bias(self, X: np.ndarray, target_rate: float, threshold: float = 0.5) -> None:
        z = self.raw_score(X)
        self.base += float(np.log(threshold / (1 - threshold)) - np.quantile(z, 1.0 - target_rate))

    def bin_spec(self, bits: int = 8) -> BinSpec:
        """The smallest bin table of this ensemble -- its distinct thresholds per feature --
        for G32 rows (``bits=8``) or G20 rows (``bits=5``; ValueError past 31 a feature)."""
        spec = BinSpec.from_thresholds(self.feat, self.thr)
        return spec if bits == 8 else spec.with_bits(bits)

    def pack(self, wire: bool = False, bins: Optional[BinSpec] = None) -> bytes:
        """GBT1 blob for f32 rows, or (``bins``) the GBB1 blob for G32 rows of that spec."""
        if wire:
            raise ValueError("W64 wire rows are for the MLP / LR kernels; GBDT uses G32 (bins=)")
        T, D = self.feat.shape
        if bins is None:
            blob = header(b"GBT1", 0, T, D, float(self.base))
            return blob + pad16(self.feat.tobytes()) + pad16(self.thr.tobytes()) + pad16(self.leaves.tobytes())
        k = bins.bin_index(self.feat, self.thr)
        blob = header(b"GBB1", 0, T, D, float(self.base), int(bins.stamp))
        return blob + pad16(self.feat.tobytes()) + pad16(k.tobytes()) + pad16(self.leaves.tobytes())

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
