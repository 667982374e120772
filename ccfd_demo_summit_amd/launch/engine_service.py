"""Per-GPU streaming engine service -- the hot path of a deployment:

    Kafka (odh-demo, partitions p % W == rank)
      -> ingest thread: fetch -> TXB1 memcpy / native JSON parse straight into the pinned
         SPSC ring of the partition (csrc/engine/engine.cpp ring mode)
      -> engine.run(): fused HIP scoring of full micro-batches, deadline flush of partial ones
      -> flagged (fraud-routed) transactions -> Router -> KIE hand-off: a bounded async queue
         drained by pooled HTTP workers with retry/back-off (router/handoff.py), or an
         in-process ProcessEngine; a KIE outage never raises out of step()
      -> Kafka offsets committed only when every row of a message has been scored and the
         hand-off batch carrying its fraud rows is acknowledged (at-least-once; fraud starts
         are idempotent per transaction id, so every fraud-routed row starts exactly once);
         a full hand-off queue pauses scoring (rings fill, consumers stop fetching)
      -> every ``reduce_period_ms``: epoch flip + RCCL all-reduce of device counters and
         latency histograms on a side stream (X2/X3), exported on /prometheus

One process per GPU (torchrun); rank 0 also consumes ``ccd-customer-response`` and signals
the processes (README.md:569,605).
"""
from __future__ import annotations

import collections
import os
import queue
import threading
import time
from dataclasses import dataclass
from typing import Deque, Dict, List, Optional, Tuple

import numpy as np

from ..contracts.transaction import TXB_MAGIC, TxBatch
from ..ops._lib import FLAGGED_DTYPE

FLAGGED_NP = np.dtype(FLAGGED_DTYPE)


@dataclass
class EngineServiceConfig:
    topic: str = "odh-demo"
    response_topic: str = "ccd-customer-response"
    group_id: str = "ccfd-engine"
    batch: int = 4096
    depth: int = 8
    streams: int = 4
    ring_rows: int = 1 << 20
    flush_us: int = 500
    run_budget_us: int = 2000
    reduce_period_ms: float = 10.0
    threshold: float = 0.5
    input_mode: str = "zerocopy"
    output_mode: str = "zerocopy"    # zerocopy (kernel writes pinned host slots) | dma
    exec_mode: str = "auto"          # "persistent": one resident kernel fed by a descriptor ring;
                                     # "launch": a fused launch per (coalesced) micro-batch;
                                     # auto = persistent for zero-copy in/out (MLP / LR, GBDT on
                                     # G20 / G32 rows) -- bench.py's measured mode, else launch
    max_fetch: int = 2000
    persist_items: str = "auto"      # persistent MLP on W64 rows: claimed (throughput) | pipelined
                                     # (a lone full batch 29 -> 19 us; no e2e change in the deployed
                                     # topology, profiles/r3/latency/) | auto = claimed
    coalesce: int = 4                # ready micro-batches per launch (launch mode, MLP)
    native_ingest: bool = True       # Kafka-protocol brokers: C++ consumer thread fetches and writes
                                     # rows straight into the rings (ingest/native_consumer.py)
    ingest_threads: int = 0          # native consumers per rank, partitions split between them
                                     # (0 = auto: one per partition for G20 / G32 rows, whose
                                     # binning is per-row ingest work, else 1)
                                     # (one JSON message per transaction is parse-bound per thread)
    score_thread: bool = True        # drive engine.run() from a dedicated thread (GIL released in
                                     # native code) so scoring latency does not wait on the Python
                                     # router / process loop
    native_serve: bool = True        # ...or from the engine's own C++ serving thread (engine.cpp
                                     # ccfd_engine_serve_start): no Python on the scoring path at
                                     # all -- the round-3 deployed tail was the Python thread waiting
                                     # for the GIL between run() calls (profiles/r4/tail/)
    serve_budget_us: int = 200       # native serving thread: run() budget per iteration
    model_watch: Optional[str] = None   # rank 0: hot-swap when this safetensors file changes
    handoff_hold_low: float = 0.5    # a held (full) hand-off queue resumes scoring below this fill
    standard_mode: str = "count"     # "process": every standard-routed row is handed to the router
                                     # (scored-record ring) to start a standard process
    scored_capacity: int = 1 << 20   # scored-record ring rows (standard_mode="process")


def rule_safe_row_format(model_kind: str, fmt: str, rules) -> Tuple[str, str]:
    """(row format, reason or "") so device routing rules see what the reference's Drools
    rules see -- the raw transaction values:

    * W64 rows store V1..V28 as bf16 (Time / Amount stay f32): a rule over a V-column, e.g.
      ``V17 < -2.5``, could flip for values within ~0.008 of its cutoff, so rules reading any
      V-column score f32 rows;
    * G20 / G32 rows carry bins, not values: rules over any transaction column need f32 rows.
    Rules over ``proba`` only keep the compact format."""
    used = rules.feature_vars() if rules is not None else set()
    if fmt == "w64" and used - {"Time", "Amount"}:
        return "f32", (f"routing rules read {sorted(used)}: scoring f32 rows instead of W64 "
                       "(bf16 V-columns would move rule cutoffs)")
    if fmt in ("g32", "g20") and used:
        return "f32", f"routing rules read {sorted(used)}: GBDT on f32 rows instead of {fmt.upper()}"
    return fmt, ""


def resolve_exec_mode(exec_mode: str, model_kind: str, row_format: str, input_mode: str,
                      output_mode: str) -> str:
    """``auto`` -> the mode bench.py measures: the persistent kernel whenever inputs and
    outputs are zero-copy and the model has a persistent kernel (MLP / LR on any rows, GBDT
    on G20 / G32 rows); coalesced launches otherwise (DMA paths, GBDT on f32 rows)."""
    if exec_mode != "auto":
        return exec_mode
    zc = input_mode == "zerocopy" and output_mode == "zerocopy"
    ok = model_kind in ("mlp", "lr") or row_format in ("g32", "g20")
    return "persistent" if zc and ok else "launch"


class EngineService:
    def __init__(self, ctx, dm, broker, router, cfg: EngineServiceConfig, reducer=None, partitions=None):
        from ..engine import StreamEngine
        from ..parallel.dp import CounterReducer, EpochPipeline, assign_partitions, x_group
        self.ctx = ctx
        self.cfg = cfg
        self.broker = broker
        self.router = router
        # routing rules: the reference threshold rule runs as the kernels' `proba >= T` test;
        # any other rule set (config router.rules / ROUTER_RULES) is compiled to a device
        # program interpreted in the same epilogue (router/rules.py, csrc/kernels/rules.h), so
        # the flagged rows the router receives are already rule-routed
        self.device_rules = None
        rules = getattr(router, "rules", None)
        threshold = cfg.threshold
        if rules is not None:
            if rules.threshold_only is not None:
                threshold = rules.threshold_only
            else:
                from ..ops.kernels import DeviceRules
                self.device_rules = DeviceRules(rules, ctx.device)
        self.exec_mode = resolve_exec_mode(cfg.exec_mode, dm.kind, dm.row_format, cfg.input_mode, cfg.output_mode)
        self.engine = StreamEngine(dm, batch=cfg.batch, depth=cfg.depth, streams=cfg.streams,
                                   input_mode=cfg.input_mode, output_mode=cfg.output_mode, threshold=threshold,
                                   device=ctx.device.index, exec_mode=self.exec_mode, coalesce=cfg.coalesce,
                                   rules=self.device_rules, persist_items=cfg.persist_items)
        if cfg.standard_mode not in ("count", "process"):
            raise ValueError("standard_mode must be 'count' or 'process'")
        self.standard_mode = cfg.standard_mode
        if cfg.standard_mode == "process":
            # every completed row comes back with the kernel's proba / route; run() holds a
            # batch while the ring is full (back-pressure, never loss)
            self.engine.enable_scored(max(cfg.scored_capacity, 4 * cfg.batch))
        n_parts = broker.partitions(cfg.topic)
        self.partitions = partitions if partitions is not None else assign_partitions(n_parts, ctx.rank, ctx.world)
        for p in self.partitions:
            self.engine.set_ring(p, cfg.ring_rows)
        self.native = None
        self.natives = []
        if cfg.native_ingest and hasattr(broker, "_bootstrap"):
            from ..ingest.native_consumer import NativeKafkaConsumer
            starts = {}
            for p in self.partitions:
                c = broker.committed(cfg.group_id, cfg.topic, p)
                starts[p] = c if c is not None else broker.begin_offset(cfg.topic, p)
            seeds = ",".join(f"{h}:{pt}" for h, pt in getattr(broker, "_seeds", [broker._bootstrap]))
            want = int(cfg.ingest_threads) or (len(self.partitions) if self.engine.row_format in ("g20", "g32") else 1)
            nt = max(1, min(want, len(self.partitions)))
            for i in range(nt):
                mine = {p: starts[p] for j, p in enumerate(self.partitions) if j % nt == i}
                self.natives.append(NativeKafkaConsumer.for_engine(self.engine, seeds, cfg.topic, mine))
            self.native = self.natives[0]
            self.consumer = None
        else:
            self.consumer = broker.consumer(cfg.group_id, [cfg.topic], partitions=[(cfg.topic, p) for p in self.partitions]) \
                if hasattr(broker, "_boot") else _StaticInProcConsumer(broker, cfg.group_id, cfg.topic, self.partitions)
        # the scoring thread's collectives (X2 epochs + hot-swap header, blob broadcast) use
        # their own group; the flush agreement uses a third one (see flush_epochs)
        self.group = x_group(ctx)
        self.ctl_group = x_group(ctx)
        self.reducer = reducer or CounterReducer(ctx, ctx.device, group=self.group)
        from ..parallel.hotswap import HotSwap
        self.hotswap = HotSwap(ctx, self.engine, cfg.model_watch, group=self.group)
        self.epochs = EpochPipeline(self.engine, self.reducer, ctrl=self.hotswap)
        # per partition: (ring row end, next kafka offset) of ingested messages, oldest first
        self._pending: Dict[int, Deque[Tuple[int, int]]] = {p: collections.deque() for p in self.partitions}
        self._rows_in: Dict[int, int] = {p: 0 for p in self.partitions}
        # per partition: one past the highest offset ever ingested (set before the rows reach
        # the ring) -- an upper bound on the offset of every row scored so far (_commit_marks)
        self._ingest_hi: Dict[int, int] = {}
        self._notice: Dict[int, int] = {}              # committed offsets not yet told to KIE
        self._notice_t = 0.0
        self.commit_notice_period_s = 0.2
        self._stop = threading.Event()
        self._ingest_err: Optional[BaseException] = None
        self.rows_scored = 0
        self.kernel_exec_mean_us = 0.0
        self.last_reduce = time.monotonic()
        self._lat_prev = np.zeros(256, np.int64)
        # scoring-thread hand-off: rows completed since the last step(), cumulative latency
        # histogram, and engine-touching tasks (epoch flip + all-reduce, hot swap) that must
        # run between two run() calls on the scoring thread
        self._stat_lock = threading.Lock()
        self._rows_new = 0
        self._flagged_new: List[np.ndarray] = []
        self._standard_new: List[np.ndarray] = []
        self._lat_cum = np.zeros(256, np.int64)
        self._tasks: "queue.SimpleQueue" = queue.SimpleQueue()
        self._score_err: Optional[BaseException] = None
        self._reduce_pending = False
        # injected delay / crash of this rank (utils/faults.py; CCFD_FAULTS).  ``drop`` is not
        # applied here: this consumer's position advances on poll, so a drop would be real loss
        from ..utils.faults import FaultPlan
        self.faults = FaultPlan.from_env(ctx.rank)
        if self.faults is not None:
            self.faults.before_exit = lambda: (self.engine.serve_stop(), self.engine.emergency_stop(5000))
        self._fetch = self.cfg.max_fetch
        # commit gating on the KIE hand-off: offsets released by scoring (snapshotted on the
        # scoring thread right after the flagged rows of the same batches were drained) wait
        # here with the hand-off sequence number that carries those fraud rows
        self.handoff = getattr(router, "handoff", None)
        self._commit_snap: Dict[int, int] = {}
        self._commit_wait: Deque[Tuple[int, Dict[int, int]]] = collections.deque()
        self._commit_retry: Dict[int, int] = {}     # acked snapshot a broker outage refused
        self.commit_failures = 0
        self.held = False                  # hand-off queue full: scoring paused (back-pressure)
        self.hold_events = 0
        # "last request" of the reference model's gauges (proba_1 / Amount / V17 / V10) and the
        # row-weighted latency histograms behind the Seldon engine series (metrics/exporter.py)
        self.last_scored = None
        self._lat_rows_cum = np.zeros(256, np.int64)
        self._dev_rows_cum = np.zeros(256, np.int64)
        self._origin_rows_cum = np.zeros(256, np.int64)   # producer send -> scored, per transaction
        # CCFD_SERVICE_TRACE=<dir>: tail attribution (bench/tail_attribution.py) -- the engine's
        # per-batch stage trace plus this process's scoring-loop timeline (every run() call, every
        # task, every GC pause, hand-off holds), dumped to <dir>/rank<r>.npz at stop()
        self._native = bool(cfg.native_serve)
        self._rows_seen = 0
        self._trace_dir = os.environ.get("CCFD_SERVICE_TRACE") or None
        if self._trace_dir:
            import gc
            self.engine.enable_trace(1 << 18)
            self._tr_runs = np.zeros((1 << 21, 3), np.int64)    # t_call, t_return, rows
            self._tr_n = 0
            self._tr_tasks: List[Tuple[int, int, str]] = []
            self._tr_gc: List[Tuple[int, int, int]] = []        # t, phase (0 start / 1 stop), generation
            self._tr_held: List[Tuple[int, int]] = []           # t, held

            def _gc_cb(phase, info, _l=self._tr_gc):
                _l.append((time.monotonic_ns(), 0 if phase == "start" else 1, int(info.get("generation", -1))))
            self._gc_cb = _gc_cb
            gc.callbacks.append(_gc_cb)

    # ------------------------------------------------------------------ ingest (producer side)
    def _ingest_once(self) -> int:
        # max_fetch counts messages: a TXB1 message carries a whole micro-batch, a JSON one a
        # single transaction, so a JSON feed is polled a micro-batch of messages at a time
        recs = self.consumer.poll(timeout=0.001, max_records=self._fetch)
        n = 0
        by_part: Dict[int, List] = collections.defaultdict(list)
        for r in recs:
            by_part[r.partition].append(r)
        for p, rs in by_part.items():         # before any row is written: see _commit_marks
            self._ingest_hi[p] = max(self._ingest_hi.get(p, 0), rs[-1].offset + 1)
        saw_json = False
        for p, rs in by_part.items():
            json_run: List[bytes] = []
            last_off = -1
            for r in rs:
                if r.value[:4] == TXB_MAGIC:
                    if json_run:
                        n += self._write_json(p, json_run)
                        self._pending[p].append((self._rows_in[p], last_off + 1))
                        json_run = []
                    b = TxBatch.decode(r.value)
                    k = self.engine.ring_write(p, b.features, b.ids, b.customer)
                    self._rows_in[p] += k
                    n += k
                    self._pending[p].append((self._rows_in[p], r.offset + 1))
                else:
                    json_run.append(r.value)
                    last_off = r.offset
            if json_run:                     # one commit point per run of JSON messages
                saw_json = True
                n += self._write_json(p, json_run)
                self._pending[p].append((self._rows_in[p], last_off + 1))
        if recs:
            self._fetch = max(self.cfg.max_fetch, self.cfg.batch) if saw_json else self.cfg.max_fetch
        return n

    def _write_json(self, p: int, values: List[bytes]) -> int:
        k = self.engine.ring_write_json(p, values)
        self._rows_in[p] += k
        return k

    def _ingest_loop(self):
        try:
            while not self._stop.is_set():
                if self._ingest_once() == 0:
                    time.sleep(0.0005)
        except BaseException as e:           # surfaced by step()
            self._ingest_err = e

    # ------------------------------------------------------------------ consumer side
    def _snapshot_commits(self) -> Dict[int, int]:
        """Scoring thread, right after drain_flagged: what the completed batches released --
        native consumers: partition -> next offset to commit; Python consumer: partition ->
        released ring rows (mapped to offsets through ``_pending`` at commit time)."""
        if self.native is not None:
            out: Dict[int, int] = {}
            for kc in self.natives:
                out.update(kc.committable())
            return out
        return {p: self.engine.cursor(p) for p in self.partitions}

    def _last_committed_offsets(self, snap: Dict[int, int]) -> Dict[int, int]:
        out = dict(getattr(self, "_committed_now", {}))
        self._committed_now = {}
        return out

    def _commit(self, snap: Dict[int, int]) -> None:
        self._committed_now = {}
        if not snap:
            return
        if self.native is not None:                     # offsets whose rows are all scored
            for p, off in snap.items():
                self.broker.commit(self.cfg.group_id, self.cfg.topic, p, off)
            self._committed_now = dict(snap)
            return
        offs = {}
        for p, released in snap.items():
            dq = self._pending[p]
            last = None
            while dq and dq[0][0] <= released:
                last = dq.popleft()[1]
            if last is not None:
                offs[(self.cfg.topic, p)] = last
        if offs:
            self.consumer.commit(offs)
            self._committed_now = {p: o for (_t, p), o in offs.items()}

    def _commit_done(self) -> None:
        """Commit every snapshot whose fraud rows the hand-off has acknowledged (all of them
        when the hand-off is synchronous).  A commit that fails because the broker is down
        (restart, leader election) is kept and retried on a later step -- scoring goes on."""
        merged: Dict[int, int] = dict(self._commit_retry)
        while self._commit_wait:
            seq, snap = self._commit_wait[0]
            if self.handoff is not None and not self.handoff.acked(seq):
                break
            self._commit_wait.popleft()
            for p, v in snap.items():
                merged[p] = max(merged.get(p, v), v)
        if not merged:
            return
        from ..ingest.broker import BrokerError
        try:
            self._commit(merged)
            self._commit_retry = {}
        except (BrokerError, OSError, ConnectionError):
            self._commit_retry = merged
            self.commit_failures += 1
            return
        self._notify_committed(self._last_committed_offsets(merged))

    def _commit_marks(self) -> Dict[int, int]:
        """partition -> an offset above every row of it scored so far: the native consumers'
        fetch positions, else the highest ingested offset + 1 (both recorded before the rows
        reach a ring).  A standard hand-off batch carries it per row (commit_mark): KIE keeps
        the batch's dedupe keys until the engine's commits pass it (process/engine.py)."""
        if self.natives:
            out: Dict[int, int] = {}
            for kc in self.natives:
                for p, pos in kc.position().items():
                    out[p] = max(pos, self._ingest_hi.get(p, 0))
                    self._ingest_hi[p] = out[p]           # a reset position never lowers a mark
            return out
        return dict(self._ingest_hi)

    def _notify_committed(self, offs: Dict[int, int], force: bool = False) -> None:
        """Tell the KIE shards what this rank committed (throttled): their commit-gated dedupe
        keys below it can never be re-delivered.  Only standard starts are gated."""
        if self.standard_mode != "process":
            return
        for p, o in offs.items():
            self._notice[p] = max(self._notice.get(p, o), o)
        now = time.monotonic()
        if not self._notice or (not force and now - self._notice_t < self.commit_notice_period_s):
            return
        self._notice_t = now
        note, self._notice = self._notice, {}
        if self.handoff is not None and hasattr(self.handoff, "submit_committed"):
            self.handoff.submit_committed(note)
        elif hasattr(getattr(self.router, "processes", None), "note_committed"):
            self.router.processes.note_committed(note)

    def commits_pending(self) -> int:
        return len(self._commit_wait) + (1 if self._commit_retry else 0)

    def _run_once(self, budget_us: Optional[int] = None) -> int:
        t_call = time.monotonic_ns() if self._trace_dir else 0
        st = self.engine.run(self.cfg.run_budget_us if budget_us is None else budget_us, self.cfg.flush_us)
        if self._trace_dir and self._tr_n < len(self._tr_runs):
            self._tr_runs[self._tr_n] = (t_call, time.monotonic_ns(), int(st.rows))
            self._tr_n += 1
        # drain on the same thread, right after the rows were counted: the router must see
        # every completed micro-batch's rows together with its flagged records; the commit
        # snapshot follows the drain, so it never covers a row whose fraud record is not yet
        # in _flagged_new (only this thread completes batches).  Drained on every call, rows or
        # not: a full flagged ring holds completed batches back (lossless hand-off), and only
        # this drain can make room for them.  run() / serve_collect raise HandoffLost rather
        # than return stats that count a dropped fraud record, so no commit ever covers one.
        flagged = self.engine.drain_flagged()
        standard = None
        if self.standard_mode == "process" and st.rows:
            rec = self.engine.drain_scored()
            standard = rec[rec["route"] == 0]
        snap = self._snapshot_commits() if st.rows else None
        with self._stat_lock:
            self._rows_new += int(st.rows)
            if flagged is not None and len(flagged):
                self._flagged_new.append(flagged)
            if standard is not None and len(standard):
                self._standard_new.append(standard)
            if snap:
                for p, v in snap.items():
                    self._commit_snap[p] = max(self._commit_snap.get(p, v), v)
            self._lat_cum = st.lat_hist.astype(np.int64)
            self._lat_rows_cum = st.lat_hist_rows.astype(np.int64)
            self._dev_rows_cum = st.dev_hist_rows.astype(np.int64)
            if st.last_seq:
                self.last_scored = st.last
            if st.dev_batches:
                self.kernel_exec_mean_us = st.dev_exec_mean_us     # K7, cumulative mean
            self._origin_rows_cum = st.origin_hist_rows.astype(np.int64)
        return int(st.rows)

    def _collect_native(self) -> int:
        """Native serving thread: progress since the last call.  The commit snapshot is taken
        BEFORE the collect, and the collect returns the stats together with every flagged /
        scored record of the batches they count (one cut under the engine's lock), so a
        committed offset never covers a row whose records the router has not received."""
        snap = self._snapshot_commits()
        st, flagged, rec = self.engine.serve_collect(want_scored=self.standard_mode == "process")
        rows = int(st.rows) - self._rows_seen
        self._rows_seen = int(st.rows)
        standard = rec[rec["route"] == 0] if rec is not None and len(rec) else None
        with self._stat_lock:
            self._rows_new += rows
            if len(flagged):
                self._flagged_new.append(flagged)
            if standard is not None and len(standard):
                self._standard_new.append(standard)
            for p, v in (snap or {}).items():
                self._commit_snap[p] = max(self._commit_snap.get(p, v), v)
            self._lat_cum = st.lat_hist.astype(np.int64)
            self._lat_rows_cum = st.lat_hist_rows.astype(np.int64)
            self._dev_rows_cum = st.dev_hist_rows.astype(np.int64)
            if st.last_seq:
                self.last_scored = st.last
            if st.dev_batches:
                self.kernel_exec_mean_us = st.dev_exec_mean_us
            self._origin_rows_cum = st.origin_hist_rows.astype(np.int64)
        return rows

    def _progress(self) -> None:
        """Wait helper for X2 ticks: the serving thread retires batches by itself."""
        if self._native:
            time.sleep(20e-6)
        else:
            self._run_once(0)

    def _reduce(self, lat_cum: np.ndarray, block: bool = False) -> bool:
        delta = lat_cum - self._lat_prev                # cumulative since reset -> send the delta
        if (delta < 0).any():                           # stats were reset in between
            delta = lat_cum
        # at most one collective per tick, never waiting for a slower rank (block=False: the
        # tick is skipped while the previous reduction is still in flight); waiting for the
        # closed epoch keeps retiring micro-batches on this (the scoring) thread
        ok = self.epochs.tick(delta, progress=self._progress, block=block)
        if ok:
            self._lat_prev = lat_cum
        self.hotswap.poll()                             # runtime X1: swap once the blob landed
        self._reduce_pending = False
        return ok

    def _score_loop(self) -> None:
        try:
            import torch
            torch.cuda.set_device(self.ctx.device)      # torch's current device is per thread
            while not self._stop.is_set():
                while True:
                    try:
                        task = self._tasks.get_nowait()
                    except queue.Empty:
                        break
                    if self._trace_dir:
                        t0 = time.monotonic_ns()
                        task()
                        self._tr_tasks.append((t0, time.monotonic_ns(), getattr(task, "__name__", "task")))
                    else:
                        task()
                if self.held:                           # hand-off back-pressure: rings fill,
                    time.sleep(200e-6)                  # the Kafka consumers stop fetching
                    continue
                self._run_once()
        except BaseException as e:                      # surfaced by step()
            self._score_err = e

    def step(self) -> int:
        if self.faults is not None:
            self.faults.step()
        if self._ingest_err is not None:
            raise RuntimeError("ingest thread failed") from self._ingest_err
        if self._score_err is not None:
            raise RuntimeError("scoring thread failed") from self._score_err
        threaded = getattr(self, "_score_thread", None) is not None
        if self.handoff is not None:
            if not self.held and self.handoff.full():
                self.held = True
                self.hold_events += 1
                if self._native:
                    self.engine.serve_hold(True)
                if self._trace_dir:
                    self._tr_held.append((time.monotonic_ns(), 1))
            elif self.held and self.handoff.has_room(self.cfg.handoff_hold_low):
                self.held = False
                if self._native:
                    self.engine.serve_hold(False)
                if self._trace_dir:
                    self._tr_held.append((time.monotonic_ns(), 0))
        if self._native:
            self._collect_native()
        elif not threaded and not self.held:
            self._run_once()
        with self._stat_lock:
            rows, self._rows_new = self._rows_new, 0
            fl, self._flagged_new = self._flagged_new, []
            sd, self._standard_new = self._standard_new, []
            snap, self._commit_snap = self._commit_snap, {}
            lat_cum = self._lat_cum
        self.router.scored_ns = time.time_ns()          # hand-off items carry it: scored -> started at KIE
        flagged = np.concatenate(fl) if len(fl) > 1 else (fl[0] if fl else np.zeros(0, FLAGGED_NP))
        standard = (np.concatenate(sd) if len(sd) > 1 else sd[0]) if sd else None
        seq = -1
        if rows or len(flagged):
            if standard is not None:                   # standard_mode="process"
                self.router.on_flagged(flagged, rows, standard=standard, marks=self._commit_marks())
            else:
                self.router.on_flagged(flagged, rows)  # enqueues; never blocks on KIE
            seq = getattr(self.router, "last_handoff_seq", -1)
        if snap:
            if self.handoff is not None and seq < 0:
                seq = self.handoff.last_seq()          # no new fraud rows: wait for the earlier ones
            self._commit_wait.append((seq, snap))
        self.rows_scored += rows
        self._commit_done()
        now = time.monotonic()
        if (now - self.last_reduce) * 1e3 >= self.cfg.reduce_period_ms and not self._reduce_pending:
            self.last_reduce = now
            if threaded:
                self._reduce_pending = True
                self._tasks.put(lambda lat=lat_cum: self._reduce(lat))
            else:
                self._reduce(lat_cum)
        if (threaded or self._native) and rows == 0:
            time.sleep(50e-6)                            # nothing new: do not spin the GIL
        return rows

    def reset_stats(self) -> None:
        """Zero the engine's latency statistics (on the scoring thread when there is one)."""
        def _do():
            self.engine.reset_stats()
            with self._stat_lock:
                self._lat_cum = np.zeros(256, np.int64)
        self._on_engine_thread(_do)

    def _on_engine_thread(self, fn) -> None:
        if getattr(self, "_score_thread", None) is not None and self._score_thread.is_alive():
            done = threading.Event()
            box = []

            def task():
                try:
                    fn()
                except BaseException as e:        # re-raised on the caller's thread
                    box.append(e)
                finally:
                    done.set()
            self._tasks.put(task)
            if not done.wait(60):
                raise TimeoutError("scoring thread did not run the task")
            if box:
                raise box[0]
        else:
            fn()

    def flush_epochs(self) -> None:
        """Reduce the pending and the open counter epoch (X2) -- e.g. before reading final counts
        or stopping.  Collective: every rank calls it.  Ranks first agree on the largest number
        of epoch ticks any of them has done and catch up, so every collective stays paired
        even though ticks are scheduled by each rank's own clock."""
        def _do():
            if self.ctx.initialized:
                import torch
                import torch.distributed as dist
                # the tick count is agreed on the control group: the X-group may still carry
                # this rank's last (async) reduction, which a MAX there would pair against
                t = torch.tensor([self.epochs.ticks], dtype=torch.int64, device=self.ctx.device)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ctl_group)
                target = int(t.item())
                while self.epochs.ticks < target:       # every rank is here: blocking is safe
                    with self._stat_lock:
                        lat = self._lat_cum
                    self._reduce(lat, block=True)
            self.epochs.finish(progress=self._progress)
            self.hotswap.poll(block=True)
        self._on_engine_thread(_do)

    def latency_hist(self) -> np.ndarray:
        """Cumulative ring-arrival -> scored latency histogram (ns, 4 buckets per octave)."""
        with self._stat_lock:
            return self._lat_cum.copy()

    def request_swap(self, model) -> None:
        """Publish new weights to every rank at the next epoch tick (call on rank 0)."""
        self.hotswap.offer(model)

    def start(self) -> "EngineService":
        if self.native is not None:
            self._thread = None
            for kc in self.natives:
                kc.start()
        else:
            self._thread = threading.Thread(target=self._ingest_loop, daemon=True, name="ccfd-ingest")
            self._thread.start()
        self._score_thread = None
        if self._native:
            self.engine.serve_start(self.cfg.serve_budget_us, self.cfg.flush_us)
        elif self.cfg.score_thread:
            self._score_thread = threading.Thread(target=self._score_loop, daemon=True, name="ccfd-score")
            self._score_thread.start()
        return self

    def dump_trace(self) -> Optional[str]:
        """CCFD_SERVICE_TRACE: write <dir>/rank<r>.npz (see __init__)."""
        if not self._trace_dir:
            return None
        import gc
        if self._gc_cb in gc.callbacks:
            gc.callbacks.remove(self._gc_cb)
        os.makedirs(self._trace_dir, exist_ok=True)
        path = os.path.join(self._trace_dir, f"rank{self.ctx.rank}.npz")
        tasks = np.array([(a, b) for a, b, _ in self._tr_tasks], np.int64).reshape(-1, 2)
        np.savez(path, batches=self.engine.read_trace(), runs=self._tr_runs[:self._tr_n], tasks=tasks,
                 task_names=np.array([n for _, _, n in self._tr_tasks], dtype="U32"),
                 gc=np.array(self._tr_gc, np.int64).reshape(-1, 3), held=np.array(self._tr_held, np.int64).reshape(-1, 2),
                 t_dump=np.int64(time.monotonic_ns()), native=np.int64(1 if self._native else 0))
        return path

    def stop(self) -> None:
        self._stop.set()
        if self._native:
            self.engine.serve_stop()
        for kc in self.natives:
            kc.stop()
        for th in (getattr(self, "_score_thread", None), getattr(self, "_thread", None)):
            if th is not None:
                th.join(5)
        for kc in self.natives:
            kc.close()
        if self._trace_dir:
            try:
                print(f"[engine] service trace: {self.dump_trace()}", flush=True)
            except Exception as e:                       # diagnostics must not block shutdown
                print(f"[engine] service trace failed: {e!r}", flush=True)
        self.engine.close()

    def metrics_source(self):
        c, lat = self.reducer.snapshot()
        extra = {"rows_scored_local": self.rows_scored,
                 "kernel_exec_mean_us": self.kernel_exec_mean_us,
                 "model_version": self.hotswap.version,
                 "commits_pending": len(self._commit_wait), "handoff_held": int(self.held),
                 "commit_failures": self.commit_failures}
        if self.natives:
            # where the native consumer threads spend their time (cumulative seconds):
            # broker I/O, response parsing, row writing / encoding, waiting on full rings
            tot: Dict[str, int] = {}
            for kc in self.natives:
                for k, v in kc.stats().items():
                    tot[k] = tot.get(k, 0) + v
            extra.update(ingest_threads=len(self.natives), ingest_rows=tot.get("rows", 0),
                         ingest_errors=tot.get("errors", 0),
                         ingest_io_seconds=tot.get("io_ns", 0) * 1e-9,
                         ingest_parse_seconds=(tot.get("handle_ns", 0) - tot.get("encode_ns", 0)
                                               - tot.get("ring_wait_ns", 0)) * 1e-9,
                         ingest_encode_seconds=tot.get("encode_ns", 0) * 1e-9,
                         ingest_ring_wait_seconds=tot.get("ring_wait_ns", 0) * 1e-9)
            fa = sum(kc.fetch_age_hist().astype(np.int64) for kc in self.natives)
            if int(fa.sum()) > 0:                       # produce -> scored, the broker's share
                from ..parallel.dp import hist_quantile
                extra.update(ingest_fetch_age_p50_seconds=hist_quantile(fa, 0.5) * 1e-9,
                             ingest_fetch_age_p99_seconds=hist_quantile(fa, 0.99) * 1e-9)
        if self.handoff is not None:
            hs = self.handoff.stats()
            extra.update(handoff_queue_depth=hs["depth"], handoff_retries=hs["retries"],
                         handoff_acked=hs["acked"], handoff_failed=hs["failed"],
                         handoff_refused=hs.get("refused", 0),
                         handoff_dead_letter_total=hs.get("dead_lettered", 0))
            for key, h in (("queue_wait", self.handoff.queue_wait), ("request", self.handoff.request_time)):
                if h.count():                           # scored -> started, the engine's share
                    extra[f"handoff_{key}_p50_seconds"] = h.quantile_ns(0.5) * 1e-9
                    extra[f"handoff_{key}_p99_seconds"] = h.quantile_ns(0.99) * 1e-9
        if self.standard_mode == "process":
            extra.update(standard_started=getattr(self.router, "standard_started", 0))
        with self._stat_lock:
            oh = self._origin_rows_cum.copy()
        if oh.sum() > 0:                        # rows that carried their producer's send time
            from ..parallel.dp import hist_quantile
            extra.update(produce_to_scored_p50_seconds=hist_quantile(oh, 0.5) * 1e-9,
                         produce_to_scored_p99_seconds=hist_quantile(oh, 0.99) * 1e-9,
                         produce_to_scored_rows=int(oh.sum()))
        return c, lat, extra

    def model_source(self) -> dict:
        """The model / Seldon series' inputs (metrics/exporter.py EngineModelCollector): last
        scored transaction, row-weighted arrival->scored and device-exec histograms, malformed
        messages (status 400) and rows the kernel refused (status 500); local to this rank,
        like each Seldon replica's own series."""
        malformed = sum(kc.stats()["errors"] for kc in self.natives) if self.natives else 0
        refused = int(self.reducer.local_snapshot()[0][4])        # CNT_WIRE_STALE, this rank
        with self._stat_lock:
            return {"last": self.last_scored, "lat_rows": self._lat_rows_cum.copy(),
                    "dev_rows": self._dev_rows_cum.copy(), "malformed": malformed, "refused": refused}


class _StaticInProcConsumer:
    """Static-assignment consumer over an InProcBroker (same API as WireConsumer)."""

    def __init__(self, broker, group, topic, partitions):
        self.broker, self.group, self.topic = broker, group, topic
        self._positions = {}
        for p in partitions:
            c = broker.committed(group, topic, p)
            self._positions[(topic, p)] = c if c is not None else broker.begin_offset(topic, p)

    def poll(self, timeout: float = 0.0, max_records: int = 500):
        out = []
        for tp, pos in list(self._positions.items()):
            recs = self.broker.fetch(tp[0], tp[1], pos, max_records - len(out))
            if recs:
                self._positions[tp] = recs[-1].offset + 1
                out.extend(recs)
        if not out and timeout:
            time.sleep(timeout)
        return out

    def commit(self, offsets=None):
        for (t, p), o in (offsets or self._positions).items():
            self.broker.commit(self.group, t, p, o)
