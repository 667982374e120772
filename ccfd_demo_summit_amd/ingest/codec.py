"""Batch decoding of ``odh-demo`` messages into a feature matrix.

JSON messages go through the native C++ parser (csrc/engine/ingest.cpp) in one call per
fetch; TXB1 binary batches are decoded zero-copy.  The pure-Python decoder is the
reference oracle used when the native library is unavailable (CPU-only installs).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

from ..contracts.transaction import TXB_MAGIC, N_FEATURES, TxBatch, decode_tx_json


def parse_json_batch(values: Sequence[bytes], native: bool = True) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    n = len(values)
    feats = np.zeros((n, N_FEATURES), np.float32)
    ids = np.zeros(n, np.uint64)
    cust = np.zeros(n, np.uint32)
    if n == 0:
        return feats, ids, cust
    if native:
        try:
            from .kafka_wire import _codec_lib      # host-only library: no GPU runtime
            L = _codec_lib()
        except Exception:
            L = None
        if L is not None:
            buf = b"".join(values)
            off = np.zeros(n + 1, np.int64)
            np.cumsum([len(v) for v in values], out=off[1:])
            rc = L.ccfd_parse_json_batch(buf, off.ctypes.data, n, feats.ctypes.data, ids.ctypes.data,
                                         cust.ctypes.data)
            if rc == n:
                return feats, ids, cust
            raise ValueError(f"malformed transaction message #{-rc - 1}")
    for i, v in enumerate(values):
        tx = decode_tx_json(v)
        feats[i] = tx.features
        ids[i] = tx.id
        cust[i] = tx.customer_id
    return feats, ids, cust


def decode_records(values: Sequence[bytes], native: bool = True) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Decode a mixed list of JSON and TXB1 messages (in order) into (X, ids, customer)."""
    if not values:
        return parse_json_batch([])
    if all(v[:4] != TXB_MAGIC for v in values):
        return parse_json_batch(values, native)
    Xs: List[np.ndarray] = []
    Is: List[np.ndarray] = []
    Cs: List[np.ndarray] = []
    pend: List[bytes] = []

    def flush():
        if pend:
            x, i, c = parse_json_batch(pend, native)
            Xs.append(x); Is.append(i); Cs.append(c)
            pend.clear()
    for v in values:
        if v[:4] == TXB_MAGIC:
            flush()
            b = TxBatch.decode(v)
            Xs.append(b.features); Is.append(b.ids); Cs.append(b.customer)
        else:
            pend.append(v)
    flush()
    return np.concatenate(Xs), np.concatenate(Is), np.concatenate(Cs)
