"""Windowed idempotency index of the KIE tier: transaction id -> process instance id over the
last ``window`` admitted transactions (native: csrc/engine/dedupe.cpp in libccfd_host.so).

A hand-off batch is admitted in ONE call: a transaction already present (a re-delivered
batch, a transaction twice in one batch) answers its stored instance id, a new one gets the
next id of ``first_id + k * stride`` (shard-encoded ids, process/sharding.py).  ~30 ns a row
against ~1 us for the Python set/dict it replaces -- the difference between one KIE process
absorbing ~2e5 and >1e6 standard starts a second."""
from __future__ import annotations

import ctypes as C
from typing import Tuple

import numpy as np

from ..ops._hostlib import hostlib

_bound = False


def _lib():
    global _bound
    L = hostlib()
    if not _bound:
        L.ccfd_dedupe_new.argtypes = [C.c_int64]
        L.ccfd_dedupe_new.restype = C.c_void_p
        L.ccfd_dedupe_new_gated.argtypes = [C.c_int64]
        L.ccfd_dedupe_new_gated.restype = C.c_void_p
        L.ccfd_dedupe_evict.argtypes = [C.c_void_p, C.c_int64]
        L.ccfd_dedupe_evict.restype = C.c_int64
        L.ccfd_dedupe_erase.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.ccfd_dedupe_erase.restype = C.c_int64
        L.ccfd_dedupe_free.argtypes = [C.c_void_p]
        L.ccfd_dedupe_free.restype = None
        L.ccfd_dedupe_size.argtypes = [C.c_void_p]
        L.ccfd_dedupe_size.restype = C.c_int64
        L.ccfd_dedupe_assign.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64,
                                         C.c_void_p, C.c_void_p]
        L.ccfd_dedupe_assign.restype = C.c_int64
        L.ccfd_dedupe_insert.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
        L.ccfd_dedupe_insert.restype = C.c_int64
        L.ccfd_dedupe_lookup.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
        L.ccfd_dedupe_lookup.restype = C.c_int64
        _bound = True
    return L


def _i64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a).astype(np.int64, copy=False))


class DedupeFull(RuntimeError):
    """A gated index has no room for the batch: nothing was admitted.  Transient -- the KIE
    server answers 503 and the router's hand-off retries once committed offsets free room."""
    transient = True


class DedupeIndex:
    def __init__(self, window: int = 1 << 20, gated: bool = False):
        """``gated=False``: a count window (the oldest key leaves when ``window`` are held).
        ``gated=True``: ``window`` is a hard capacity; keys leave only through ``erase`` and an
        admission that could overflow raises DedupeFull."""
        self.window = int(window)
        self.gated = bool(gated)
        self._L = _lib()
        self._h = (self._L.ccfd_dedupe_new_gated if gated else self._L.ccfd_dedupe_new)(self.window)
        if not self._h:
            raise MemoryError(f"dedupe index of {window} entries")

    def __len__(self) -> int:
        return int(self._L.ccfd_dedupe_size(self._h))

    def assign(self, tx, first_id: int, stride: int = 1) -> Tuple[np.ndarray, np.ndarray]:
        """(instance id per row, newly admitted transaction ids in admission order)."""
        t = _i64(tx)
        n = len(t)
        out = np.empty(n, np.int64)
        new = np.empty(n, np.int64)
        k = self._L.ccfd_dedupe_assign(self._h, t.ctypes.data, n, int(first_id), int(stride),
                                       out.ctypes.data, new.ctypes.data)
        if k == -2:
            raise DedupeFull(f"dedupe index full ({len(self)} of {self.window} keys uncommitted)")
        if k < 0:
            raise ValueError("transaction ids must be non-negative integers")
        return out, new[:k]

    def evict(self, k: int) -> int:
        """Count-window mode: drop the ``k`` oldest admitted keys; returns how many left."""
        return int(self._L.ccfd_dedupe_evict(self._h, int(k)))

    def erase(self, keys) -> int:
        """Gated mode: drop these keys; returns how many were present."""
        t = _i64(keys)
        return int(self._L.ccfd_dedupe_erase(self._h, t.ctypes.data, len(t)))

    def insert(self, tx, ids) -> int:
        t, i = _i64(tx), _i64(ids)
        if len(t) != len(i):
            raise ValueError("keys and ids of different lengths")
        k = self._L.ccfd_dedupe_insert(self._h, t.ctypes.data, i.ctypes.data, len(t))
        if k == -2:
            raise DedupeFull(f"dedupe index full ({len(self)} of {self.window} keys)")
        if k < 0:
            raise ValueError("transaction ids must be non-negative integers")
        return int(k)

    def lookup(self, tx) -> np.ndarray:
        t = _i64(tx)
        out = np.empty(len(t), np.int64)
        self._L.ccfd_dedupe_lookup(self._h, t.ctypes.data, len(t), out.ctypes.data)
        return out

    def __contains__(self, tx) -> bool:
        return bool(self.lookup([tx])[0] >= 0)

    def get(self, tx, default=None):
        v = int(self.lookup([tx])[0])
        return default if v < 0 else v

    def close(self) -> None:
        if self._h:
            self._L.ccfd_dedupe_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:                  # interpreter shutdown
            pass
