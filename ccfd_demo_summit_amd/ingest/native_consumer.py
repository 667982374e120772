"""Python handle of the native Kafka consumer (csrc/engine/kafka_consumer.cpp).

A C++ thread looks up partition leaders (Metadata v1), keeps one connection per leader
broker, fetches (Fetch v4) from all leaders in parallel, validates RecordBatch v2 CRC-32C
(uncompressed or gzip), and writes TXB1 batches / JSON transactions straight into the
engine's pinned partition rings (f32, W64 or G32 rows) -- no Python per message (SURVEY.md §2.4
H1, §7.3 hard part 1: JSON-per-transaction at 1M/s is out of reach for a Python consumer
loop).  Leader moves / broker failures refresh metadata and continue from the same offset;
OFFSET_OUT_OF_RANGE follows ``offset_reset`` (earliest / latest / none).

    kc = NativeKafkaConsumer.for_engine(engine, "127.0.0.1:9092", "odh-demo", {p: committed_offset})
    kc.start()
    ...
    for p, off in kc.committable().items(): consumer_group.commit(p, off)   # scored data only
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List

import numpy as np

from ..ops._lib import check, lib


class KcPartition(C.Structure):
    _fields_ = [("kafka_partition", C.c_int32), ("engine_partition", C.c_int32), ("start_offset", C.c_int64),
                ("feats", C.c_void_p), ("ids", C.c_void_p), ("customer", C.c_void_p), ("capacity", C.c_int64),
                ("amount", C.c_void_p)]


class KcStats(C.Structure):
    _fields_ = [("records", C.c_uint64), ("rows", C.c_uint64), ("bytes", C.c_uint64),
                ("errors", C.c_uint64), ("fetches", C.c_uint64), ("metadata_refreshes", C.c_uint64),
                ("offset_resets", C.c_uint64), ("leaders", C.c_uint64), ("io_ns", C.c_uint64),
                ("handle_ns", C.c_uint64), ("encode_ns", C.c_uint64), ("ring_wait_ns", C.c_uint64)]


RESET_POLICIES = {"earliest": 0, "latest": 1, "none": 2}
ROW_CODES = {"f32": 0, "w64": 1, "g32": 2, "g20": 3}
ROW_WIDTH = {"f32": 30, "w64": 16, "g32": 8, "g20": 5}   # f32 words per row


def _bind(L):
    if getattr(L, "_kc_bound", False):
        return L
    L.ccfd_kc_create_engine.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_char_p, C.c_void_p, C.c_int, C.c_int]
    L.ccfd_kc_create_engine.restype = C.c_void_p
    L.ccfd_kc_create_array.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_void_p, C.c_int, C.c_int]
    L.ccfd_kc_create_array.restype = C.c_void_p
    for f in ("ccfd_kc_start",):
        getattr(L, f).argtypes = [C.c_void_p]
        getattr(L, f).restype = C.c_int
    for f in ("ccfd_kc_stop", "ccfd_kc_destroy"):
        getattr(L, f).argtypes = [C.c_void_p]
        getattr(L, f).restype = None
    L.ccfd_kc_committable.argtypes = [C.c_void_p, C.c_int]
    L.ccfd_kc_committable.restype = C.c_int64
    L.ccfd_kc_get_stats.argtypes = [C.c_void_p, C.POINTER(KcStats)]
    L.ccfd_kc_get_stats.restype = None
    L.ccfd_kc_last_error.argtypes = [C.c_void_p]
    L.ccfd_kc_last_error.restype = C.c_char_p
    L.ccfd_kc_feed_record_set.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
    L.ccfd_kc_feed_record_set.restype = C.c_int64
    L.ccfd_kc_last_origin.argtypes = [C.c_void_p]
    L.ccfd_kc_last_origin.restype = C.c_int64
    L.ccfd_kc_fetch_age_hist.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    L.ccfd_kc_fetch_age_hist.restype = None
    L.ccfd_kc_set_offset_reset.argtypes = [C.c_void_p, C.c_int]
    L.ccfd_kc_set_offset_reset.restype = C.c_int
    L.ccfd_kc_position.argtypes = [C.c_void_p, C.c_int]
    L.ccfd_kc_position.restype = C.c_int64
    L.ccfd_kc_set_bins.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]
    L.ccfd_kc_set_bins.restype = C.c_int
    L._kc_bound = True
    return L


def _split(bootstrap: str):
    """The native side takes the whole bootstrap list ("h1:p1,h2:p2"); ``port`` is the
    default for entries without one."""
    return bootstrap.strip(), 9092


class NativeKafkaConsumer:
    def __init__(self, handle: int, partitions: List[int], keep=None):
        self.h = handle
        self.partitions = list(partitions)
        self._keep = keep            # buffers the C++ side writes into

    @classmethod
    def for_engine(cls, engine, bootstrap: str, topic: str, start_offsets: Dict[int, int]) -> "NativeKafkaConsumer":
        """Consume partitions ``start_offsets`` (kafka partition -> first offset) into the
        engine rings registered with ``engine.set_ring(p, ...)`` under the same index."""
        L = _bind(lib())
        ps = sorted(start_offsets)
        arr = (KcPartition * len(ps))()
        for i, p in enumerate(ps):
            log = engine.logs[p]
            arr[i] = KcPartition(p, p, int(start_offsets[p]), log.feats.ptr, log.ids.ptr, log.customer.ptr, log.n,
                                 log.amount.ptr if log.amount is not None else None)
        host, port = _split(bootstrap)
        h = L.ccfd_kc_create_engine(C.c_void_p(engine.h), host.encode(), port, topic.encode(), arr, len(ps),
                                    ROW_CODES[engine.row_format])
        check(0 if h else -1, "ccfd_kc_create_engine")
        kc = cls(h, ps, keep=arr)
        if engine.row_format in ("g32", "g20"):
            kc._set_bins(engine.bins)
        return kc

    def _set_bins(self, bins) -> None:
        """G32 sink: rows are binned at ingest against ``bins`` (models.gbdt.BinSpec)."""
        flat, off = bins.flat, bins.offsets
        self._bins_keep = (flat, off)
        check(lib().ccfd_kc_set_bins(C.c_void_p(self.h), flat.ctypes.data, off.ctypes.data, int(bins.stamp)),
              "ccfd_kc_set_bins")

    @classmethod
    def for_arrays(cls, bootstrap: str, topic: str, start_offsets: Dict[int, int], capacity: int,
                   wire: bool = False, bins=None) -> "NativeKafkaConsumer":
        """Test sink: flat numpy arrays per partition (no engine, no GPU): ``arrays[p]`` =
        (rows, ids, customer), ``amounts[p]`` = the Amount column of G32 rows (``bins``)."""
        L = _bind(lib())
        ps = sorted(start_offsets)
        fmt = bins.row_format if bins is not None else "w64" if wire else "f32"
        bufs = {p: (np.zeros((capacity, ROW_WIDTH[fmt]), np.float32), np.zeros(capacity, np.uint64),
                    np.zeros(capacity, np.uint32)) for p in ps}
        amounts = {p: np.zeros(capacity, np.float32) for p in ps}
        arr = (KcPartition * len(ps))()
        for i, p in enumerate(ps):
            f, ids, cu = bufs[p]
            arr[i] = KcPartition(p, i, int(start_offsets[p]), f.ctypes.data, ids.ctypes.data, cu.ctypes.data, capacity,
                                 amounts[p].ctypes.data)
        host, port = _split(bootstrap)
        h = L.ccfd_kc_create_array(host.encode(), port, topic.encode(), arr, len(ps), ROW_CODES[fmt])
        check(0 if h else -1, "ccfd_kc_create_array")
        kc = cls(h, ps, keep=(arr, bufs, amounts))
        kc.arrays = bufs
        kc.amounts = amounts
        if bins is not None:
            kc._set_bins(bins)
        return kc

    def set_offset_reset(self, policy: str) -> "NativeKafkaConsumer":
        """auto.offset.reset on OFFSET_OUT_OF_RANGE: earliest / latest / none (before start)."""
        check(lib().ccfd_kc_set_offset_reset(C.c_void_p(self.h), RESET_POLICIES[policy]), "ccfd_kc_set_offset_reset")
        return self

    def position(self) -> Dict[int, int]:
        """partition -> next offset the consumer will fetch."""
        return {p: int(lib().ccfd_kc_position(C.c_void_p(self.h), i)) for i, p in enumerate(self.partitions)}

    def start(self) -> "NativeKafkaConsumer":
        check(lib().ccfd_kc_start(C.c_void_p(self.h)), "ccfd_kc_start")
        return self

    def stop(self) -> None:
        if self.h:
            lib().ccfd_kc_stop(C.c_void_p(self.h))

    def close(self) -> None:
        if self.h:
            lib().ccfd_kc_destroy(C.c_void_p(self.h))
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self) -> Dict[str, int]:
        st = KcStats()
        lib().ccfd_kc_get_stats(C.c_void_p(self.h), C.byref(st))
        return {k: int(getattr(st, k)) for k, _ in KcStats._fields_}

    def last_error(self) -> str:
        return (lib().ccfd_kc_last_error(C.c_void_p(self.h)) or b"").decode(errors="replace")

    def last_origin_ns(self) -> int:
        """Producer send time of the last ingested batch (``ccfd-ts`` header) on the steady
        clock (time.monotonic_ns), 0 = the batch carried none."""
        return int(lib().ccfd_kc_last_origin(C.c_void_p(self.h)))

    def fetch_age_hist(self):
        """Record batches that carried a ``ccfd-ts`` send time, by their age when this
        consumer had fetched them (ns, 256 buckets, 4 per octave: parallel.dp.hist_quantile)."""
        import numpy as np
        out = np.zeros(256, np.uint64)
        lib().ccfd_kc_fetch_age_hist(C.c_void_p(self.h), out.ctypes.data_as(C.POINTER(C.c_uint64)))
        return out

    def feed(self, record_set: bytes) -> int:
        """Parse ``record_set`` as partition 0's fetched bytes (array sink, no socket)."""
        if not isinstance(record_set, bytes):
            record_set = bytes(record_set)
        return int(lib().ccfd_kc_feed_record_set(C.c_void_p(self.h), record_set, len(record_set)))

    def committable(self) -> Dict[int, int]:
        """partition -> next offset to commit (only partitions that advanced)."""
        out = {}
        for i, p in enumerate(self.partitions):
            off = lib().ccfd_kc_committable(C.c_void_p(self.h), i)
            if off >= 0:
                out[p] = int(off)
        return out
