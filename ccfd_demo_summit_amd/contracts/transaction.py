"""Transaction schema and wire codecs.

The reference replays the Kaggle ``creditcard.csv`` dataset onto topic ``odh-demo``
(README.md:547-548, ProducerDeployment.yaml:94-95): columns ``Time, V1..V28, Amount``
(+ ``Class`` label).  The dashboards chart ``Amount``, ``V10``, ``V17`` per request
(deploy/grafana/ModelPrediction.json:104,211,322).  The exact JSON field names the
reference producer put on the wire are not in the reference, so we
accept the natural superset:

* JSON per message (compat path): ``{"id":..,"customer_id":..,"Time":..,"V1":..,...,
  "Amount":..}``; also accepts ``{"features":[30 floats]}`` and the Seldon-style
  ``{"data":{"ndarray":[[...]]}}`` wrapper.
* Packed binary batch (``TXB1``, hot path): a columnar micro-batch designed to be
  consumed zero-copy by the GPU engine (features are one contiguous ``[n,30] f32`` block,
  16-byte aligned).

Binary layout (little endian)::

    off  size  field
    0    4     magic  b"TXB1"
    4    2     version (1)
    6    2     flags   (bit0: has labels)
    8    4     n       rows
    12   4     n_features (30)
    16   8     base_offset (stream offset of row 0)
    24   8     reserved
    32   8n    ids        u64[n]
    ..   4n    customer   u32[n]   (padded to 16 B)
    ..   120n  features   f32[n][30] (16-B aligned)
    ..   n     labels     u8[n]    (if flags & 1)
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass, field
from typing import Iterable, Optional, Sequence

import numpy as np

FEATURE_NAMES: tuple = ("Time",) + tuple(f"V{i}" for i in range(1, 29)) + ("Amount",)
N_FEATURES = len(FEATURE_NAMES)          # 30
TIME_COL = 0
AMOUNT_COL = N_FEATURES - 1              # 29
V10_COL = FEATURE_NAMES.index("V10")
V17_COL = FEATURE_NAMES.index("V17")

# ---------------------------------------------------------------------------------------
# W64: the engine's packed 64-byte row (partition logs and rings on the zero-copy path).
# The scoring hot path is bound by host->GPU bytes (PCIe, ~55 GB/s per MI355X), so the log
# row is sized for it: the 28 PCA components V1..V28 -- zero-centred by construction and fed
# to bf16 MFMAs anyway -- travel as bf16 (RNE); Time and Amount, whose magnitude needs more
# than 8 mantissa bits, stay f32.  64 B instead of 120 B per transaction, one float4 per lane
# (a 16-row tile is one fully coalesced 1 KB wave request).
#   bytes [0,56)  V1..V28 bf16     [56,60) Time f32     [60,64) Amount f32
# Wire position p holds canonical feature WIRE_PERM[p]; packed models (pack(wire=True)) are
# permuted to this order so lane group g of the kernel reads exactly bytes [16g, 16g+16).
WIRE_ROW_BYTES = 64
WIRE_PERM = np.array(list(range(1, 29)) + [0, N_FEATURES - 1], np.int64)
WIRE_AMOUNT_F32 = 15                      # Amount as the 16th f32 word of a W64 row


def _bf16_bits(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, np.float32).view(np.uint32)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = (u & 0x7FFFFFFF) > 0x7F800000                      # keep NaN a (quiet) NaN
    if nan.any():
        r[nan] = ((u[nan] >> 16) | 0x0040).astype(np.uint16)
    return r


def encode_wire(X: np.ndarray, out: Optional[np.ndarray] = None) -> np.ndarray:
    """float32 [n, 30] canonical rows -> uint8 [n, 64] W64 rows."""
    X = np.asarray(X, np.float32)
    n = X.shape[0]
    if out is None:
        out = np.empty((n, WIRE_ROW_BYTES), np.uint8)
    w16 = out.view(np.uint16).reshape(n, 32)
    w32 = out.view(np.float32).reshape(n, 16)
    w16[:, :28] = _bf16_bits(X[:, 1:29])
    w32[:, 14] = X[:, TIME_COL]
    w32[:, 15] = X[:, AMOUNT_COL]
    return out


def decode_wire(W: np.ndarray) -> np.ndarray:
    """uint8 [n, 64] W64 rows -> float32 [n, 30] canonical rows (V-columns bf16-exact)."""
    W = np.ascontiguousarray(W).view(np.uint8).reshape(-1, WIRE_ROW_BYTES)
    n = W.shape[0]
    X = np.empty((n, N_FEATURES), np.float32)
    v = (W.view(np.uint16).reshape(n, 32)[:, :28].astype(np.uint32) << 16).view(np.float32)
    X[:, 1:29] = v
    f = W.view(np.float32).reshape(n, 16)
    X[:, TIME_COL] = f[:, 14]
    X[:, AMOUNT_COL] = f[:, 15]
    return X


# ---------------------------------------------------------------------------------------
# G32: the 32-byte row of the tree-ensemble (GBDT) path.  A tree only tests ``x_j > thr``;
# with feature j's sorted split thresholds as bin edges, bin_j(x) = #{edges_j < x} and
# ``x_j > edges_j[k]`` <=> ``bin_j(x) > k`` for every float x (NaN -> 0, every test false),
# so one byte per feature carries exactly what the ensemble can see.  The bin table belongs
# to the model (models/gbdt.py BinSpec); rows carry its stamp so a row encoded for another
# table is detected (counted, never silently mis-scored).
#   bytes [0,30)  bin of Time, V1..V28, Amount (u8)   [30] amount bucket (K6 histogram)
#   [31]          bin-table stamp 1..255
# Amount itself stays host-side (the flagged-record column of the partition log).
G32_ROW_BYTES = 32


def amount_bucket(amount: np.ndarray) -> np.ndarray:
    """K6 histogram bucket (metric_names.AMOUNT_BUCKETS, csrc/kernels/common.h amount_bucket)."""
    from .metric_names import AMOUNT_BUCKETS
    a = np.asarray(amount, np.float32)
    b = np.zeros(a.shape, np.uint8)
    for bound in AMOUNT_BUCKETS:
        b += (a > np.float32(bound)).astype(np.uint8)
    return b


def encode_g32(X: np.ndarray, edges: Sequence[np.ndarray], stamp: int,
               out: Optional[np.ndarray] = None) -> np.ndarray:
    """float32 [n, 30] canonical rows -> uint8 [n, 32] G32 rows (numpy oracle of the native
    ccfd_encode_g32).  ``edges[j]``: ascending float32 bin edges of feature j (<= 255)."""
    X = np.asarray(X, np.float32)
    n = X.shape[0]
    if out is None:
        out = np.empty((n, G32_ROW_BYTES), np.uint8)
    for j in range(N_FEATURES):
        e = np.asarray(edges[j], np.float32)
        b = np.searchsorted(e, X[:, j], side="left")          # #edges < x (ascending edges)
        b[np.isnan(X[:, j])] = 0
        out[:, j] = b.astype(np.uint8)
    out[:, 30] = amount_bucket(X[:, AMOUNT_COL])
    out[:, 31] = np.uint8(stamp)
    return out


# G20: the same bins packed 5 bits each for bin tables of <= 31 edges per feature (every
# BASELINE-size 100 x 6 ensemble: ~20 distinct thresholds a feature), little-endian over
# the row's 160 bits -- bits [5j, 5j+5) bin of feature j, [150, 154) amount bucket,
# [154, 160) bin-table stamp 1..63.  20 B a row: 1.6x the rows of G32 per PCIe byte.
G20_ROW_BYTES = 20


def encode_g20(X: np.ndarray, edges: Sequence[np.ndarray], stamp: int,
               out: Optional[np.ndarray] = None) -> np.ndarray:
    """float32 [n, 30] canonical rows -> uint8 [n, 20] G20 rows (numpy oracle of the native
    ccfd_encode_g20).  ``edges[j]``: ascending float32 bin edges of feature j (<= 31)."""
    g = encode_g32(X, edges, stamp)
    if (g[:, :N_FEATURES] > 31).any() or not 1 <= stamp <= 63:
        raise ValueError("G20 rows need <= 31 bin edges per feature and a stamp in 1..63")
    n = g.shape[0]
    acc = np.zeros((n, 3), np.uint64)                        # 3 x 64 bits >= 160
    fields = [(5 * j, g[:, j]) for j in range(N_FEATURES)] + [(150, g[:, 30]), (154, g[:, 31])]
    for bit, v in fields:
        v = v.astype(np.uint64)
        w, sh = bit >> 6, bit & 63
        acc[:, w] |= v << np.uint64(sh)
        if sh + 6 > 64:
            acc[:, w + 1] |= v >> np.uint64(64 - sh)
    if out is None:
        out = np.empty((n, G20_ROW_BYTES), np.uint8)
    out[:] = acc.view(np.uint8).reshape(n, 24)[:, :G20_ROW_BYTES]
    return out


def decode_g20_bins(rows: np.ndarray) -> np.ndarray:
    """uint8 [n, 20] G20 rows -> uint8 [n, 32] in the G32 byte layout (bins, bucket, stamp)."""
    r = np.ascontiguousarray(rows, np.uint8).reshape(-1, G20_ROW_BYTES)
    n = r.shape[0]
    pad = np.zeros((n, 24), np.uint8)
    pad[:, :G20_ROW_BYTES] = r
    acc = pad.view(np.uint64).reshape(n, 3)
    out = np.empty((n, G32_ROW_BYTES), np.uint8)
    fields = [(5 * j, 5) for j in range(N_FEATURES)] + [(150, 4), (154, 6)]
    for i, (bit, width) in enumerate(fields):
        w, sh = bit >> 6, bit & 63
        v = acc[:, w] >> np.uint64(sh)
        if sh + width > 64:
            v = v | (acc[:, w + 1] << np.uint64(64 - sh))
        out[:, i] = (v & np.uint64((1 << width) - 1)).astype(np.uint8)
    return out


TXB_MAGIC = b"TXB1"
TXB_HEADER = struct.Struct("<4sHHIIQQ")  # 32 bytes
assert TXB_HEADER.size == 32


def _align16(x: int) -> int:
    return (x + 15) & ~15


@dataclass
class Transaction:
    id: int
    customer_id: int
    features: np.ndarray                  # float32[30]
    label: Optional[int] = None

    @property
    def amount(self) -> float:
        return float(self.features[AMOUNT_COL])

    def to_dict(self) -> dict:
        d = {"id": int(self.id), "customer_id": int(self.customer_id)}
        for name, v in zip(FEATURE_NAMES, self.features.tolist()):
            d[name] = v
        if self.label is not None:
            d["Class"] = int(self.label)
        return d


def encode_tx_json(tx: Transaction) -> bytes:
    return json.dumps(tx.to_dict(), separators=(",", ":")).encode()


def decode_tx_json(payload) -> Transaction:
    """Decode one JSON transaction message (all accepted shapes, see module doc)."""
    obj = json.loads(payload) if isinstance(payload, (bytes, bytearray, str)) else payload
    feats = None
    if "features" in obj:
        feats = np.asarray(obj["features"], dtype=np.float32)
    elif "data" in obj:
        data = obj["data"]
        if "ndarray" in data:
            feats = np.asarray(data["ndarray"], dtype=np.float32).reshape(-1)
        elif "tensor" in data:
            feats = np.asarray(data["tensor"]["values"], dtype=np.float32)
    else:
        feats = np.array([float(obj.get(n, 0.0)) for n in FEATURE_NAMES], dtype=np.float32)
    if feats is None or feats.shape[0] != N_FEATURES:
        raise ValueError(f"transaction must carry {N_FEATURES} features")
    label = obj.get("Class")
    return Transaction(
        id=int(obj.get("id", obj.get("tx_id", 0))),
        customer_id=int(obj.get("customer_id", obj.get("customer", 0))),
        features=feats,
        label=None if label is None else int(label),
    )


@dataclass
class TxBatch:
    """Columnar micro-batch (host side).  ``features`` is C-contiguous float32 [n,30]."""
    ids: np.ndarray
    customer: np.ndarray
    features: np.ndarray
    labels: Optional[np.ndarray] = None
    base_offset: int = 0

    def __post_init__(self):
        self.ids = np.ascontiguousarray(self.ids, dtype=np.uint64)
        self.customer = np.ascontiguousarray(self.customer, dtype=np.uint32)
        self.features = np.ascontiguousarray(self.features, dtype=np.float32)
        if self.features.ndim != 2 or self.features.shape[1] != N_FEATURES:
            raise ValueError("features must be [n, 30]")
        n = self.features.shape[0]
        if self.ids.shape != (n,) or self.customer.shape != (n,):
            raise ValueError("ids/customer must be [n]")
        if self.labels is not None:
            self.labels = np.ascontiguousarray(self.labels, dtype=np.uint8)

    def __len__(self) -> int:
        return int(self.features.shape[0])

    @staticmethod
    def layout(n: int, has_labels: bool):
        off_ids = 32
        off_cust = off_ids + 8 * n
        off_feat = _align16(off_cust + 4 * n)
        off_lab = off_feat + 4 * N_FEATURES * n
        end = off_lab + (n if has_labels else 0)
        return off_ids, off_cust, off_feat, off_lab, _align16(end)

    def encode(self) -> bytes:
        n = len(self)
        has_l = self.labels is not None
        oi, oc, of, ol, end = self.layout(n, has_l)
        buf = bytearray(end)
        TXB_HEADER.pack_into(buf, 0, TXB_MAGIC, 1, 1 if has_l else 0, n, N_FEATURES,
                             int(self.base_offset), 0)
        buf[oi:oi + 8 * n] = self.ids.tobytes()
        buf[oc:oc + 4 * n] = self.customer.tobytes()
        buf[of:of + 4 * N_FEATURES * n] = self.features.tobytes()
        if has_l:
            buf[ol:ol + n] = self.labels.tobytes()
        return bytes(buf)

    @classmethod
    def decode(cls, payload) -> "TxBatch":
        mv = memoryview(payload)
        magic, ver, flags, n, nf, base, _ = TXB_HEADER.unpack_from(mv, 0)
        if magic != TXB_MAGIC or ver != 1:
            raise ValueError("not a TXB1 batch")
        if nf != N_FEATURES:
            raise ValueError(f"expected {N_FEATURES} features, got {nf}")
        has_l = bool(flags & 1)
        oi, oc, of, ol, end = cls.layout(n, has_l)
        if len(mv) < end:
            raise ValueError("truncated TXB1 batch")
        ids = np.frombuffer(mv, np.uint64, n, oi)
        cust = np.frombuffer(mv, np.uint32, n, oc)
        feats = np.frombuffer(mv, np.float32, n * N_FEATURES, of).reshape(n, N_FEATURES)
        labels = np.frombuffer(mv, np.uint8, n, ol) if has_l else None
        return cls(ids=ids, customer=cust, features=feats, labels=labels, base_offset=base)

    def transactions(self) -> Iterable[Transaction]:
        for i in range(len(self)):
            yield Transaction(int(self.ids[i]), int(self.customer[i]), self.features[i],
                              None if self.labels is None else int(self.labels[i]))

    @classmethod
    def from_transactions(cls, txs: Sequence[Transaction]) -> "TxBatch":
        n = len(txs)
        feats = np.stack([t.features for t in txs]) if n else np.zeros((0, N_FEATURES), np.float32)
        labels = None
        if n and all(t.label is not None for t in txs):
            labels = np.array([t.label for t in txs], np.uint8)
        return cls(ids=np.array([t.id for t in txs], np.uint64),
                   customer=np.array([t.customer_id for t in txs], np.uint32),
                   features=feats, labels=labels)
