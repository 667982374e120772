"""Python façade of the native streaming engine (csrc/engine/engine.cpp).

The per-micro-batch loop runs in C++ (host launch cost ~ a few µs per batch would make
a Python loop the bottleneck); Python drives it in *steps* (``pump(n_batches)``), owns
device buffers through torch (model blob, epoch counter buffers) and runs the RCCL
collectives on a side stream between steps (parallel/dp.py).
"""
from __future__ import annotations

import ctypes as C
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops._lib import (BATCH_TRACE_DTYPE, BIN_FORMATS, ENGINE_FLAG_FULL, FLAGGED_DTYPE, SCORED_DTYPE, MODEL_IDS,
                        N_COUNTER_SLOTS, ROW_FORMATS, EngineConfig, EngineStats, Flagged, check, last_error, lib)
from ..ops.kernels import ROW_BYTES, DeviceModel

N_FEATURES = 30
WIRE_ROW_F32 = 16            # W64 wire row = 64 B = 16 f32 words (contracts.transaction)
G32_ROW_F32 = 8              # G32 row = 32 B (contracts.transaction)
G20_ROW_F32 = 5              # G20 row = 20 B (contracts.transaction)
INPUT_MODES = {"dma": 0, "zerocopy": 1}
OUTPUT_MODES = {"zerocopy": 0, "dma": 1}


def same_bins(a, b) -> bool:
    """Two bin tables (models.gbdt.BinSpec) are the same table: same width and identical edge
    arrays.  The 6-bit (G20) / 8-bit (G32) in-row stamp is only a last-resort device check --
    two different tables share a G20 stamp with probability ~1/63 -- so the host
    compares the full table wherever it can."""
    if a is None or b is None:
        return a is b
    if a.bits != b.bits or len(a.edges) != len(b.edges):
        return False
    return all(x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))
               for x, y in zip(a.edges, b.edges))


class PinnedArray:
    """numpy view over ``hipHostMalloc`` memory (mapped, portable): the partition log the
    GPU reads by DMA or directly over PCIe."""

    def __init__(self, shape, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        self.shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
        nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        self.nbytes = max(nbytes, 16)
        self.ptr = lib().ccfd_host_alloc(self.nbytes)
        if not self.ptr:
            raise MemoryError(f"ccfd_host_alloc({self.nbytes}) failed: {last_error()}")
        buf = (C.c_uint8 * self.nbytes).from_address(self.ptr)
        self.array = np.frombuffer(buf, dtype=self.dtype, count=int(np.prod(self.shape))).reshape(self.shape)

    def free(self):
        if self.ptr:
            self.array = None
            lib().ccfd_host_free(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def encode_w64(X: np.ndarray, out_ptr: int) -> None:
    """f32 rows [n, 30] -> W64 wire rows at ``out_ptr`` (native encoder, ingest/encode.cpp)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    if X.ndim != 2 or X.shape[1] != N_FEATURES:
        raise ValueError("expected [n, 30] float32 rows")
    if lib().ccfd_encode_w64(X.ctypes.data, X.shape[0], N_FEATURES, C.c_void_p(out_ptr)) != X.shape[0]:
        raise RuntimeError("ccfd_encode_w64 failed")


def encode_g32(X: np.ndarray, bins, out_ptr: int, amount_ptr: Optional[int] = None) -> None:
    """f32 rows [n, 30] -> G32 rows (G20 rows for a 5-bit ``bins``) at ``out_ptr`` against
    ``bins`` (models.gbdt.BinSpec), Amount column to ``amount_ptr`` (native encoders,
    csrc/engine/ingest.cpp)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    if X.ndim != 2 or X.shape[1] != N_FEATURES:
        raise ValueError("expected [n, 30] float32 rows")
    flat, off = bins.flat, bins.offsets
    fn = lib().ccfd_encode_g20 if bins.bits == 5 else lib().ccfd_encode_g32
    if fn(X.ctypes.data, X.shape[0], N_FEATURES, flat.ctypes.data, off.ctypes.data,
          int(bins.stamp), C.c_void_p(out_ptr), C.c_void_p(amount_ptr)) != X.shape[0]:
        raise RuntimeError(f"ccfd_encode_{bins.row_format} failed")


encode_bins = encode_g32


class PartitionLog:
    """One Kafka-partition-like append log of transactions in pinned host memory.

    ``wire=True`` stores W64 rows (64 B, contracts/transaction.py) instead of 30 x f32;
    ``bins=BinSpec`` stores G32 rows (32 B, GBDT) -- G20 rows (20 B) for a 5-bit spec --
    plus a host-side Amount column."""

    def __init__(self, n_rows: int, wire: bool = False, bins=None):
        self.n = int(n_rows)
        self.wire = bool(wire)
        self.bins = bins
        if bins is not None and wire:
            raise ValueError("a log holds one row format: W64 (wire) or G32 (bins)")
        self.row_format = bins.row_format if bins is not None else "w64" if self.wire else "f32"
        self.row_bytes = ROW_BYTES[self.row_format]
        self.feats = PinnedArray((self.n, self.row_bytes // 4), np.float32)
        self.ids = PinnedArray(self.n, np.uint64)
        self.customer = PinnedArray(self.n, np.uint32)
        self.amount = PinnedArray(self.n, np.float32) if bins is not None else None

    def write_rows(self, r: int, X: np.ndarray) -> None:
        """Store canonical f32 rows X at log rows [r, r + len(X))."""
        if self.row_format in BIN_FORMATS:
            encode_g32(X, self.bins, self.feats.ptr + r * self.row_bytes, self.amount.ptr + 4 * r)
        elif self.wire:
            encode_w64(X, self.feats.ptr + r * self.row_bytes)
        else:
            self.feats.array[r:r + X.shape[0]] = X

    @classmethod
    def from_arrays(cls, X: np.ndarray, ids=None, customer=None, wire: bool = False, bins=None) -> "PartitionLog":
        log = cls(X.shape[0], wire=wire, bins=bins)
        log.write_rows(0, X)
        log.ids.array[:] = np.arange(log.n, dtype=np.uint64) if ids is None else ids
        log.customer.array[:] = 0 if customer is None else customer
        return log

    def free(self):
        for a in (self.feats, self.ids, self.customer, self.amount):
            if a is not None:
                a.free()


@dataclass
class LastScored:
    """The last transaction the engine scored (the reference model's "last request":
    deploy/grafana/ModelPrediction.json:96-322 plots proba_1, Amount, V17, V10 of it).
    ``row`` holds its raw log row in the engine's row format."""
    tx_id: int
    proba: float
    amount: float
    partition: int
    row: bytes
    row_format: str

    def features(self, bins=None) -> np.ndarray:
        """float32 [30] canonical row: exact for f32 rows, bf16-exact V-columns for W64 rows;
        for G32 / G20 rows (bins against the ensemble's split table) each feature is the
        midpoint of its bin interval (the end edge for the two open bins, NaN without
        ``bins``) and Amount is exact (the host-side column)."""
        from ..contracts.transaction import AMOUNT_COL, decode_g20_bins, decode_wire
        if self.row_format == "f32":
            return np.frombuffer(self.row[:120], np.float32).copy()
        if self.row_format == "w64":
            return decode_wire(np.frombuffer(self.row[:64], np.uint8))[0]
        g = np.frombuffer(self.row[:32], np.uint8) if self.row_format == "g32" else \
            decode_g20_bins(np.frombuffer(self.row[:20], np.uint8))[0]
        x = np.full(N_FEATURES, np.nan, np.float32)
        if bins is not None:
            for j, e in enumerate(bins.edges):
                b = int(g[j])
                if e.size == 0:
                    continue
                if b == 0:
                    x[j] = e[0]
                elif b >= e.size:
                    x[j] = e[-1]
                else:
                    x[j] = 0.5 * (float(e[b - 1]) + float(e[b]))
        x[AMOUNT_COL] = self.amount
        return x


@dataclass
class StepStats:
    batches: int = 0
    rows: int = 0
    fraud_rows: int = 0
    dropped: int = 0
    wall_s: float = 0.0
    p50_us: float = 0.0
    p99_us: float = 0.0
    max_us: float = 0.0
    mean_us: float = 0.0
    lat_hist: np.ndarray = field(default_factory=lambda: np.zeros(256, np.uint64))
    host_submit_s: float = 0.0
    host_wait_s: float = 0.0
    host_complete_s: float = 0.0
    dev_batches: int = 0                 # K7: device-clock execution time per micro-batch
    dev_exec_mean_us: float = 0.0
    dev_hist: np.ndarray = field(default_factory=lambda: np.zeros(256, np.uint64))
    # row-weighted twins (Seldon request histograms: one transaction = one request)
    lat_hist_rows: np.ndarray = field(default_factory=lambda: np.zeros(256, np.uint64))
    dev_hist_rows: np.ndarray = field(default_factory=lambda: np.zeros(256, np.uint64))
    last_seq: int = 0                    # batches that produced a "last scored" record
    last: Optional[LastScored] = None
    # producer send -> scored (ring batches whose rows carried a send time, ccfd-ts header)
    origin_batches: int = 0
    origin_hist: np.ndarray = field(default_factory=lambda: np.zeros(256, np.uint64))
    origin_hist_rows: np.ndarray = field(default_factory=lambda: np.zeros(256, np.uint64))
    submitted: int = 0                   # micro-batches submitted by the call
    flag_full_events: int = 0            # completions deferred on a full flagged ring (cumulative)


class HandoffLost(RuntimeError):
    """The engine reports fraud-routed records it could not hand off.  The ring reserves room
    for a whole batch before retiring it, so this is a broken invariant, never back-pressure:
    a caller that commits offsets must stop instead of committing past lost fraud cases."""


def check_lossless(st: "StepStats") -> None:
    if st.dropped:
        raise HandoffLost(f"{st.dropped} fraud-routed records were dropped by the engine's flagged ring")


class FlaggedDrainer:
    """The router's collector beside a pumping engine: a thread that moves fraud-routed
    records from the engine's flagged ring into ``sink(records)`` while the caller's thread
    keeps submitting micro-batches (the pump is a native call that releases the GIL).

    The streaming service works this way (native serving thread + Python collector); a
    replay that drained inline instead -- pump a step, then drain -- left the GPU with no new
    work for the length of every drain: ~1e6 fraud records a 0.25 s config-4 step cost it
    4-10 % of its rate (profiles/r6/pass_h/).  ``stop()`` joins the thread and drains what is
    left, so every record reaches ``sink`` exactly once, in completion order; an exception in
    ``sink`` is raised again there."""

    def __init__(self, engine: "StreamEngine", sink, idle_s: float = 2e-4):
        self.engine = engine
        self.sink = sink
        self.idle_s = float(idle_s)
        self.records = 0
        self.drains = 0
        self._stop = threading.Event()
        self._err: Optional[BaseException] = None
        self._th: Optional[threading.Thread] = None

    def start(self) -> "FlaggedDrainer":
        self._stop.clear()
        self._th = threading.Thread(target=self._run, name="flagged-drainer", daemon=True)
        self._th.start()
        return self

    def _hand(self, recs: np.ndarray) -> None:
        if len(recs):
            self.sink(recs)
            self.records += len(recs)
            self.drains += 1

    def _run(self) -> None:
        try:
            while not self._stop.is_set():
                recs = self.engine.drain_flagged()
                if len(recs):
                    self._hand(recs)
                else:
                    time.sleep(self.idle_s)
        except BaseException as e:       # noqa: BLE001 -- re-raised on the caller's thread
            self._err = e

    def stop(self) -> int:
        """Join the thread, hand off what is left in the ring; returns the records handed."""
        if self._th is not None:
            self._stop.set()
            self._th.join()
            self._th = None
        if self._err is not None:
            e, self._err = self._err, None
            raise e
        self._hand(self.engine.drain_flagged())
        return self.records

    def __enter__(self) -> "FlaggedDrainer":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()


_FMT_BY_ROW_BYTES = {120: "f32", 64: "w64", 32: "g32", 20: "g20"}


def _stats(st: EngineStats) -> StepStats:
    last = None
    if st.last_seq:
        nb = int(st.last_row_bytes)
        last = LastScored(int(st.last_tx_id), float(st.last_proba), float(st.last_amount),
                          int(st.last_partition), bytes(st.last_row[:nb]), _FMT_BY_ROW_BYTES.get(nb, "f32"))
    return StepStats(st.batches, st.rows, st.fraud_rows, st.flagged_dropped, st.wall_s,
                     st.lat_p50_us, st.lat_p99_us, st.lat_max_us, st.lat_mean_us,
                     np.ctypeslib.as_array(st.lat_hist).copy(), st.host_submit_ns * 1e-9,
                     st.host_wait_ns * 1e-9, st.host_complete_ns * 1e-9, int(st.dev_batches),
                     (st.dev_exec_ns / st.dev_batches * 1e-3) if st.dev_batches else 0.0,
                     np.ctypeslib.as_array(st.dev_hist).copy(),
                     np.ctypeslib.as_array(st.lat_hist_rows).copy(),
                     np.ctypeslib.as_array(st.dev_hist_rows).copy(), int(st.last_seq), last,
                     int(st.origin_batches), np.ctypeslib.as_array(st.origin_hist).copy(),
                     np.ctypeslib.as_array(st.origin_hist_rows).copy(), int(st.submitted),
                     int(st.flag_full_events))


class StreamEngine:
    def __init__(self, dm: DeviceModel, batch: int = 4096, depth: int = 8, streams: int = 2,
                 input_mode: str = "dma", output_mode: str = "zerocopy", threshold: float = 0.5,
                 device: Optional[int] = None, flag_capacity: int = 1 << 20, exec_mode: str = "launch",
                 persist_grid: int = 0, coalesce: int = 1, rules=None, persist_items: str = "auto"):
        """exec_mode: "launch" = one fused kernel launch per micro-batch; "persistent" = one
        long-running kernel fed through a descriptor ring (MLP/LR, zero-copy outputs).
        persist_items (persistent MLP on W64 rows): "claimed" = 512-row items claimed by 64
        workgroups (the throughput point: 8.7e8 tx/s at 12 batches in flight); "pipelined" =
        static 128-row items over 128 workgroups with the next item's rows fetched while the
        current one is scored (the latency point: 19 us vs 29 us unloaded, better up to ~4
        batches in flight; profiles/r3/latency/); "auto" = claimed unless CCFD_PERSIST_PIPE=1.
        coalesce: launch mode -- up to this many ready, log-contiguous micro-batches go out as
        one launch (MLP, zero-copy in/out); completion stays per micro-batch.
        rules: a compiled routing rule set (ops.kernels.DeviceRules) evaluated per row in the
        kernels' epilogue instead of ``proba >= threshold`` (kept alive by the engine)."""
        self.dm = dm
        self.device = torch.device("cuda", device if device is not None else torch.cuda.current_device())
        self.batch = int(batch)
        self.threshold = float(threshold)
        # two epoch counter buffers (X2: one is all-reduced while the other accumulates)
        self.counters = [torch.zeros(N_COUNTER_SLOTS, dtype=torch.int64, device=self.device) for _ in range(2)]
        cfg = EngineConfig()
        cfg.device = self.device.index
        cfg.model = MODEL_IDS[dm.kind]
        cfg.blob = dm.blob.data_ptr()
        cfg.gbdt_trees, cfg.gbdt_depth = dm.trees, dm.depth
        cfg.threshold = self.threshold
        cfg.max_batch = self.batch
        cfg.depth = int(depth)
        cfg.n_streams = int(streams)
        cfg.input_mode = INPUT_MODES[input_mode]
        cfg.output_mode = OUTPUT_MODES[output_mode]
        cfg.flag_capacity = int(flag_capacity)
        cfg.exec_mode = {"launch": 0, "persistent": 1}[exec_mode]
        cfg.persist_grid = int(persist_grid)
        cfg.coalesce = max(1, min(8, int(coalesce)))
        cfg.persist_items = {"auto": 0, "claimed": 1, "pipelined": 2}[persist_items]
        self.persist_items = persist_items
        self.wire = bool(getattr(dm, "wire", False))
        self.row_format = dm.row_format
        self.bins = getattr(dm, "bins", None)
        if self.bins is not None and rules is not None and rules.ruleset.feature_vars():
            raise ValueError("G32 rows carry bins, not feature values: routing rules may only use proba_1 "
                             "(use f32 rows for rules over transaction columns)")
        cfg.wire = ROW_FORMATS[self.row_format]
        self.exec_mode = exec_mode
        self.flips = 0
        self.rules = rules
        cfg.rules = rules.ptr if rules is not None else None
        cfg.counters[0] = self.counters[0].data_ptr()
        cfg.counters[1] = self.counters[1].data_ptr()
        # counters zeroed before the engine's streams use them (stream sync, never a device
        # sync: another engine's persistent kernel may be resident)
        torch.cuda.current_stream(self.device).synchronize()
        self.h = lib().ccfd_engine_create(C.byref(cfg))
        if not self.h:
            raise RuntimeError(f"ccfd_engine_create failed: {last_error()}")
        self.logs: Dict[int, PartitionLog] = {}
        self._flag_buf = (Flagged * 65536)()
        self._flag_cap = max(1024, int(flag_capacity), self.batch)
        # records taken out of a full flagged ring by a blocking call (drain paths) so it could
        # finish; drain_flagged / serve_collect return them first, in completion order
        self._stash: List[np.ndarray] = []
        # the flagged drains may run on a collector thread beside the pump (FlaggedDrainer):
        # the ring's native drain is lock-protected, the stash and the copy-out are guarded here
        self._drain_lock = threading.Lock()

    def close(self):
        if getattr(self, "h", None):
            self._serving = False                # destroy stops the serving thread first
            lib().ccfd_engine_destroy(C.c_void_p(self.h))
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check_log(self, log: PartitionLog) -> None:
        if log.row_format != self.row_format:
            raise ValueError(f"log rows are {log.row_format}, the engine's model blob expects {self.row_format}")
        if self.row_format in BIN_FORMATS and not same_bins(log.bins, self.bins):
            raise ValueError("log was G32 / G20-encoded against another bin table than the model's")

    def add_log(self, partition: int, log: PartitionLog, cursor: int = 0) -> None:
        self._check_log(log)
        self._call(lambda: lib().ccfd_engine_set_log(C.c_void_p(self.h), int(partition), C.c_void_p(log.feats.ptr),
                                                     C.c_void_p(log.ids.ptr), C.c_void_p(log.customer.ptr),
                                                     log.n, int(cursor)), "ccfd_engine_set_log")
        if log.amount is not None:
            self._call(lambda: lib().ccfd_engine_set_amount(C.c_void_p(self.h), int(partition),
                                                            C.c_void_p(log.amount.ptr)), "ccfd_engine_set_amount")
        self.logs[partition] = log

    def _call(self, fn, what: str) -> None:
        """Run a blocking native call that may need to retire in-flight batches; on a full
        flagged ring it drains the ring into the stash and calls again (nothing is dropped)."""
        while True:
            rc = fn()
            if rc != ENGINE_FLAG_FULL:
                check(rc, what)
                return
            self._stash_ring()

    def _stash_ring(self) -> int:
        with self._drain_lock:
            got = self._drain_ring(1 << 62)
            if len(got):
                self._stash.append(got)
            return len(got)

    def pump(self, n_batches: int, batch_rows: Optional[int] = None, drain: bool = True,
             on_flagged=None) -> StepStats:
        """Score ``n_batches`` micro-batches.  ``drain=False`` keeps up to ``depth`` batches in
        flight across calls (steady-state streaming); the last call of a run must drain.

        Lossless hand-off: when the flagged ring cannot take a finished batch's fraud records,
        the native pump stops (nothing retired, nothing lost); the ring is drained -- into
        ``on_flagged(records)`` when given (the caller's hand-off), else into the stash the
        next ``drain_flagged`` returns -- and pumping resumes with the remaining batches."""
        st = EngineStats()
        left = int(n_batches)
        rows_b = int(batch_rows or self.batch)
        while True:
            before = int(st.submitted)
            rc = lib().ccfd_engine_pump(C.c_void_p(self.h), left, rows_b, 1 if drain else 0, C.byref(st))
            left -= int(st.submitted) - before
            if rc != ENGINE_FLAG_FULL:
                check(rc, "ccfd_engine_pump")
                break
            if on_flagged is not None:
                on_flagged(self.drain_flagged())
            else:
                self._stash_ring()
        out = _stats(st)
        check_lossless(out)
        return out

    def score(self, X: np.ndarray):
        """Synchronous score of a host matrix [n,30] -> (proba [n] f32, route [n] u8)."""
        X = np.ascontiguousarray(X, dtype=np.float32)
        n = X.shape[0]
        if self.row_format in BIN_FORMATS:
            rows = np.empty((n, ROW_BYTES[self.row_format] // 4), np.float32)
            encode_g32(X, self.bins, rows.ctypes.data)
            X = rows
        elif self.wire:
            rows = np.empty((n, WIRE_ROW_F32), np.float32)
            encode_w64(X, rows.ctypes.data)
            X = rows
        proba = np.empty(n, np.float32)
        route = np.empty(n, np.uint8)
        self._call(lambda: lib().ccfd_engine_score_sync(C.c_void_p(self.h), X.ctypes.data, n, proba.ctypes.data,
                                                        route.ctypes.data), "ccfd_engine_score_sync")
        return proba, route

    def flip_epoch(self, side_stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
        """Close the current counter epoch; returns its buffer.  ``side_stream`` is made to
        wait for every batch submitted in that epoch."""
        hs = C.c_void_p(side_stream.cuda_stream) if side_stream is not None else None
        idx = lib().ccfd_engine_flip_epoch(C.c_void_p(self.h), hs)
        if idx < 0:
            raise RuntimeError(f"flip_epoch failed: {last_error()}")
        self.flips += 1
        return self.counters[idx]

    def swap_model(self, dm: DeviceModel) -> None:
        """Hot swap (runtime X1): in-flight micro-batches finish on the old weights, later ones
        use ``dm``.  The new model must have the same kernel kind, row format and GBDT shape."""
        if dm.kind != self.dm.kind or dm.row_format != self.row_format or \
                (dm.trees, dm.depth) != (self.dm.trees, self.dm.depth):
            raise ValueError("hot swap needs a model of the same kind / wire format / tree shape")
        if self.row_format in BIN_FORMATS and not same_bins(dm.bins, self.bins):
            raise ValueError("G32 hot swap: pack the new ensemble against the live bin table "
                             "(DeviceModel(model, bins=engine.bins)); its thresholds must be bin edges")
        self._call(lambda: lib().ccfd_engine_set_blob(C.c_void_p(self.h), C.c_void_p(dm.blob.data_ptr())),
                   "ccfd_engine_set_blob")
        self.dm = dm                     # keeps the new blob alive; the old one may be freed now
        self.model_version = getattr(self, "model_version", 0) + 1

    def epoch_complete(self, flip_count: int) -> bool:
        """True once every micro-batch submitted before flip number ``flip_count`` completed."""
        return lib().ccfd_engine_epoch_complete(C.c_void_p(self.h), int(flip_count)) == 1

    def drain_flagged(self, max_records: int = 1 << 30) -> np.ndarray:
        """Fraud-routed records of completed batches, oldest first (stash, then the ring).
        Safe beside a pump on another thread (the native drain holds only the ring's lock)."""
        with self._drain_lock:
            return self._drain_flagged_locked(max_records)

    def _drain_flagged_locked(self, max_records: int) -> np.ndarray:
        out: List[np.ndarray] = []
        total = 0
        while self._stash and total < max_records:
            a = self._stash[0]
            take = min(len(a), max_records - total)
            out.append(a[:take])
            total += take
            if take == len(a):
                self._stash.pop(0)
            else:
                self._stash[0] = a[take:]
        if total < max_records:
            out.append(self._drain_ring(max_records - total))
        out = [a for a in out if len(a)]
        return np.concatenate(out) if len(out) > 1 else out[0] if out else \
            np.zeros(0, dtype=np.dtype(FLAGGED_DTYPE))

    def _drain_ring(self, max_records: int, chunk: int = 16384) -> np.ndarray:
        # straight into the returned arrays (one copy out of the ring); bounded chunks keep the
        # ring lock -- which the pump's completions also take -- held for tens of microseconds
        out: List[np.ndarray] = []
        total = 0
        while total < max_records:
            want = min(chunk, max_records - total)
            arr = np.empty(want, dtype=np.dtype(FLAGGED_DTYPE))
            k = lib().ccfd_engine_drain_flagged(C.c_void_p(self.h), arr.ctypes.data, want)
            if k <= 0:
                break
            out.append(arr[:k])
            total += k
            if k < want:
                break
        if not out:
            return np.zeros(0, dtype=np.dtype(FLAGGED_DTYPE))
        return out[0] if len(out) == 1 else np.concatenate(out)

    def enable_scored(self, capacity: int = 1 << 20) -> None:
        """Opt in to a per-row scored-record ring of ``capacity`` rows (0 = off): every
        completed row -- fraud- and standard-routed -- with the kernel's proba_1 and route
        (``drain_scored``).  Streaming ``run()`` holds completed batches while it is full."""
        self._call(lambda: lib().ccfd_engine_scored_enable(C.c_void_p(self.h), int(capacity)),
                   "ccfd_engine_scored_enable")
        self._scored_cap = int(capacity)

    def drain_scored(self, max_records: int = 1 << 30) -> np.ndarray:
        """Scored records (SCORED_DTYPE) in completion order, oldest first."""
        cap = getattr(self, "_scored_cap", 0)
        if cap <= 0:
            return np.zeros(0, dtype=np.dtype(SCORED_DTYPE))
        out = np.empty(min(cap, max_records), dtype=np.dtype(SCORED_DTYPE))
        k = lib().ccfd_engine_drain_scored(C.c_void_p(self.h), out.ctypes.data, out.size)
        if k < 0:
            raise RuntimeError(f"ccfd_engine_drain_scored failed: {last_error()}")
        return out[:k]

    def scored_dropped(self) -> int:
        """Rows that completed while the scored ring was full (pump() / drain paths only)."""
        return int(lib().ccfd_engine_scored_dropped(C.c_void_p(self.h)))

    # ------------------------------------------------------------------ native serving thread
    def serve_start(self, budget_us: int = 200, flush_us: int = 500) -> None:
        """Score the rings from a C++ thread (``run(budget_us, flush_us)`` back to back) until
        ``serve_stop``; collect progress with ``serve_collect`` (engine.cpp serving thread)."""
        check(lib().ccfd_engine_serve_start(C.c_void_p(self.h), int(budget_us), int(flush_us)),
              "ccfd_engine_serve_start")
        self._serving = True

    def serve_stop(self) -> None:
        if getattr(self, "_serving", False) and getattr(self, "h", None):
            rc = lib().ccfd_engine_serve_stop(C.c_void_p(self.h))
            self._serving = False
            if rc < 0:
                raise RuntimeError(f"engine serving thread failed: {last_error()}")

    def serve_hold(self, hold: bool) -> None:
        lib().ccfd_engine_serve_hold(C.c_void_p(self.h), 1 if hold else 0)

    def serve_collect(self, want_scored: bool = False):
        """(stats, flagged records, scored records or None) -- one consistent cut: the flagged
        (and scored) records are exactly those of every batch the cumulative stats count that
        an earlier collect did not return.  Raises if the serving thread failed."""
        st = EngineStats()
        if getattr(self, "_collect_flag", None) is None:
            self._collect_flag = np.empty(max(1024, self._flag_cap), dtype=np.dtype(FLAGGED_DTYPE))
        sc = None
        if want_scored:
            cap = getattr(self, "_scored_cap", 0)
            if getattr(self, "_collect_scored", None) is None or len(self._collect_scored) != cap:
                self._collect_scored = np.empty(cap, dtype=np.dtype(SCORED_DTYPE))
            sc = self._collect_scored
        nf, ns = C.c_int64(0), C.c_int64(0)
        rc = lib().ccfd_engine_serve_collect(C.c_void_p(self.h), C.byref(st), self._collect_flag.ctypes.data,
                                             len(self._collect_flag), C.byref(nf),
                                             sc.ctypes.data if sc is not None else None,
                                             len(sc) if sc is not None else 0, C.byref(ns))
        if rc < 0:
            raise RuntimeError(f"engine serving thread failed: {last_error()}")
        fl = self._collect_flag[:nf.value].copy()
        with self._drain_lock:
            if self._stash:                  # stashed by a blocking call: older than the ring's
                fl = np.concatenate(self._stash + [fl])
                self._stash = []
        rec = sc[:ns.value].copy() if sc is not None else None
        out = _stats(st)
        check_lossless(out)
        return out, fl, rec

    # ------------------------------------------------------------------ ring (streaming) mode
    def set_ring(self, partition: int, capacity: int) -> PartitionLog:
        """Register partition ``partition`` as a live SPSC ring of ``capacity`` rows."""
        log = PartitionLog(capacity, wire=self.wire, bins=self.bins)
        self._call(lambda: lib().ccfd_engine_set_ring(C.c_void_p(self.h), int(partition), C.c_void_p(log.feats.ptr),
                                                      C.c_void_p(log.ids.ptr), C.c_void_p(log.customer.ptr), log.n),
                   "ccfd_engine_set_ring")
        if log.amount is not None:
            self._call(lambda: lib().ccfd_engine_set_amount(C.c_void_p(self.h), int(partition),
                                                            C.c_void_p(log.amount.ptr)), "ccfd_engine_set_amount")
        self.logs[partition] = log
        return log

    def ring_write(self, partition: int, X: np.ndarray, ids: Optional[np.ndarray] = None,
                   customer: Optional[np.ndarray] = None, block: bool = True) -> int:
        """Producer side: append rows (copied into the pinned ring, wrapping as needed).
        Returns rows written (< len(X) only when ``block`` is False and the ring is full)."""
        log = self.logs[partition]
        n = X.shape[0]
        done = 0
        row = C.c_int64(0)
        while done < n:
            k = lib().ccfd_engine_ring_acquire(C.c_void_p(self.h), int(partition), n - done, C.byref(row))
            if k < 0:
                raise RuntimeError("partition is not a ring")
            if k == 0:
                if not block:
                    break
                import time as _t
                _t.sleep(50e-6)
                continue
            r = row.value
            log.write_rows(r, X[done:done + k])
            if ids is not None:
                log.ids.array[r:r + k] = ids[done:done + k]
            if customer is not None:
                log.customer.array[r:r + k] = customer[done:done + k]
            lib().ccfd_engine_ring_commit(C.c_void_p(self.h), int(partition), k)
            done += k
        return done

    def ring_write_json(self, partition: int, values) -> int:
        """Parse JSON transaction messages with the native parser straight into the ring."""
        log = self.logs[partition]
        n = len(values)
        done = 0
        row = C.c_int64(0)
        L = lib()
        while done < n:
            k = L.ccfd_engine_ring_acquire(C.c_void_p(self.h), int(partition), n - done, C.byref(row))
            if k <= 0:
                import time as _t
                _t.sleep(50e-6)
                continue
            r = row.value
            chunk = values[done:done + k]
            buf = b"".join(chunk)
            off = np.zeros(k + 1, np.int64)
            np.cumsum([len(v) for v in chunk], out=off[1:])
            if log.row_format in BIN_FORMATS:         # parse to f32, then bin
                tmp = np.empty((k, N_FEATURES), np.float32)
                got = L.ccfd_parse_json_batch(buf, off.ctypes.data, k, tmp.ctypes.data,
                                              log.ids.ptr + r * 8, log.customer.ptr + r * 4)
                if got == k:
                    log.write_rows(r, tmp)
            else:
                parse = L.ccfd_parse_json_batch_w64 if log.wire else L.ccfd_parse_json_batch
                got = parse(buf, off.ctypes.data, k, log.feats.ptr + r * log.row_bytes,
                            log.ids.ptr + r * 8, log.customer.ptr + r * 4)
            if got != k:
                raise ValueError(f"malformed transaction message #{done - got - 1}")
            L.ccfd_engine_ring_commit(C.c_void_p(self.h), int(partition), k)
            done += k
        return done

    def run(self, budget_us: int = 1000, flush_us: int = 500) -> StepStats:
        """Consumer side: score whatever the rings hold for ``budget_us``."""
        st = EngineStats()
        rc = lib().ccfd_engine_run(C.c_void_p(self.h), int(budget_us), int(flush_us), C.byref(st))
        if rc < 0:
            raise RuntimeError(f"ccfd_engine_run failed: {last_error()}")
        out = _stats(st)
        check_lossless(out)
        return out

    def reset_stats(self) -> None:
        lib().ccfd_engine_reset_stats(C.c_void_p(self.h))

    def enable_trace(self, capacity: int = 65536) -> None:
        """Keep the stage timestamps of the last ``capacity`` completed micro-batches
        (0 = off); ``read_trace()`` returns them, ``utils.tracing.batch_trace_events`` turns
        them into a Chrome / Perfetto timeline."""
        check(lib().ccfd_engine_trace_enable(C.c_void_p(self.h), int(capacity)), "ccfd_engine_trace_enable")
        self._trace_cap = int(capacity)

    def read_trace(self) -> np.ndarray:
        """Structured array (BATCH_TRACE_DTYPE), oldest batch first."""
        out = np.zeros(getattr(self, "_trace_cap", 0), BATCH_TRACE_DTYPE)
        if out.size == 0:
            return out
        n = lib().ccfd_engine_trace_read(C.c_void_p(self.h), out.ctypes.data, out.size)
        if n < 0:
            raise RuntimeError(f"ccfd_engine_trace_read failed: {last_error()}")
        return out[:n]

    def progress(self) -> Dict[str, int]:
        """Non-blocking counters for watchdog diagnostics (racy snapshot)."""
        v = np.zeros(5, np.int64)
        if getattr(self, "h", None):
            lib().ccfd_engine_progress(C.c_void_p(self.h), v.ctypes.data)
        return {"submitted": int(v[0]), "completed": int(v[1]), "persist_posted": int(v[2]),
                "persist_resident": int(v[3]), "in_flight": int(v[4])}

    def emergency_stop(self, timeout_ms: int = 5000) -> int:
        """Watchdog exit path: make a resident persistent kernel leave before the process
        ends (0 = nothing resident / drained, -6 = still resident after ``timeout_ms``)."""
        if not getattr(self, "h", None):
            return 0
        return int(lib().ccfd_engine_emergency_stop(C.c_void_p(self.h), int(timeout_ms)))

    def cursor(self, partition: int) -> int:
        return int(lib().ccfd_engine_cursor(C.c_void_p(self.h), int(partition)))
