"""Business-process engine: the standard and fraud processes of the reference's KIE server
(deploy/ccd-service.yaml; docs/process-fraud.png; README.md:554-605).

Fraud process (explicit state machine of the BPMN):

    start(tx, proba) -> CustomerNotification: publish {customer_id, transaction_id,
        process_id, ...} to CUSTOMER_NOTIFICATION_TOPIC                (README.md:560,590)
    event-based gateway, first of:
      timer expires  -> DMN "Start investigation"                      (README.md:592-596)
                          approve     -> APPROVED_LOW_AMOUNT  (fraud_approved_low_amount)
                          investigate -> User Task "Assign case" (fraud_investigation_amount)
                                         -> prediction service        (README.md:571-581)
      signal(response) -> true  -> APPROVED_BY_CUSTOMER (fraud_approved_amount)
                          false -> CANCELLED            (fraud_rejected_amount)  (README.md:597-599)

Standard process: completes immediately as STANDARD (README.md:552).

Time is injected (``clock``) and timers fire from ``tick()``, so the engine is exact and
deterministic in tests and driven by a periodic task in the service.  Every state change
is appended to an optional JSONL journal; ``recover()`` rebuilds the in-flight instances
after a crash (SURVEY.md §5 checkpoint/resume: "in-flight BP instances: an optional
append-only journal").
"""
from __future__ import annotations

import collections
import hashlib
import enum
import heapq
import itertools
import json
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from ..contracts.outcomes import CustomerResponse, Outcome
from .dmn import Decision, investigation_decision
from .prediction_service import PredictionService


class State(str, enum.Enum):
    WAITING_CUSTOMER = "waiting_customer"
    USER_TASK = "user_task"
    COMPLETED = "completed"


@dataclass
class UserTask:
    id: int
    instance_id: int
    name: str = "Assign case"
    status: str = "Ready"                       # Ready | Completed
    inputs: Dict[str, Any] = field(default_factory=dict)
    suggested_outcome: Optional[str] = None
    confidence: float = 0.0
    outcome: Optional[str] = None
    completed_by: Optional[str] = None


@dataclass
class ProcessInstance:
    id: int
    process_id: str
    variables: Dict[str, Any]
    state: State = State.WAITING_CUSTOMER
    outcome: Optional[str] = None
    started: float = 0.0
    completed: Optional[float] = None
    timer_due: Optional[float] = None
    task_id: Optional[int] = None
    history: List[str] = field(default_factory=list)
    notified: bool = False          # its CustomerNotification was acknowledged by the broker

    @property
    def amount(self) -> float:
        return float(self.variables.get("amount", 0.0))

    @property
    def proba(self) -> float:
        return float(self.variables.get("proba", 0.0))


class ProcessEngine:
    FRAUD = "fraud"
    STANDARD = "standard"

    def __init__(self, notification_timeout_s: float = 30.0, dmn_probability_threshold: float = 0.75,
                 dmn_amount_threshold: float = 100.0,
                 publish_notification: Optional[Callable[[Dict[str, Any]], None]] = None,
                 kie_metrics=None, prediction: Optional[PredictionService] = None,
                 clock: Callable[[], float] = time.monotonic, journal_path: Optional[str] = None,
                 keep_completed: int = 100_000, shard: int = 0, shards: int = 1,
                 standard_dedupe_window: int = 1 << 20, standard_dedupe_capacity: Optional[int] = None,
                 standard_audit_rows: int = 1 << 22):
        """``shard`` / ``shards``: this engine is shard ``shard`` of a K-way KIE tier
        (process/sharding.py) -- its instance and task ids are ``shard + K * n``, so a signal
        or task completion that carries only the id reaches the owner.

        Standard-start idempotency is gated by the engine's committed Kafka offsets: a hand-off
        batch's columns ``kafka_partition`` / ``commit_mark`` say below which offset of each
        partition its rows were consumed, and its transaction ids stay in the dedupe index until
        the engine reports (``note_committed``) that every one of those partitions is committed
        past the mark -- only then can no replay re-deliver them.  ``standard_dedupe_window`` is
        the number of keys kept at least (and the plain count window of ungated starts);
        ``standard_dedupe_capacity`` (default 4x) is a hard bound: a batch that would exceed it is
        refused (DedupeFull -> 503 -> the router's hand-off retries: back-pressure, never an
        unsafe eviction).  ``standard_audit_rows``: standard instances answerable from memory by
        transaction id (``find_transaction``); older ones from the journal."""
        self.timeout = float(notification_timeout_s)
        self.p_thr = float(dmn_probability_threshold)
        self.a_thr = float(dmn_amount_threshold)
        self.publish_notification = publish_notification
        self.metrics = kie_metrics
        self.prediction = prediction or PredictionService()
        self.clock = clock
        self.shard, self.shards = int(shard), max(1, int(shards))
        if not 0 <= self.shard < self.shards:
            raise ValueError(f"shard {shard} of {shards}")
        self.instances: Dict[int, ProcessInstance] = {}
        self.tasks: Dict[int, UserTask] = {}
        self._timers: List = []
        self._next_n = 1                    # next instance sequence number: iid = shard + K * n
        self._task_ids = itertools.count(1)
        self._lock = threading.RLock()
        self.outcome_counts: Dict[str, int] = {o.value: 0 for o in Outcome}
        # order-independent digest of every fraud process's (transaction id, outcome): two runs
        # over the same transactions -- one of them with crashes -- compare outcome for outcome
        self.outcome_digest = 0
        self.standard_count = 0
        self.keep_completed = keep_completed
        self._completed_order: collections.deque = collections.deque()   # O(1) eviction
        self._journal = open(journal_path, "a", buffering=1) if journal_path else None
        if self._journal is not None and self._journal.tell() == 0:
            # ids encode (shard, K): recovery must decode them with the K they were written with
            self._journal.write(json.dumps({"header": {"shard": self.shard, "shards": self.shards, "v": 1}}) + "\n")
        self.dedupe_window = 1_000_000
        self._by_tx: Dict[Any, int] = {}
        self._tx_order = collections.deque()
        self.duplicates = 0
        self.fraud_count = 0                # fraud processes started (all time, recovered)
        # CustomerNotification outbox: a fraud start's journal record (written before the start
        # is acknowledged) holds its notification as pending; ``mark_notified`` clears it once
        # the broker acknowledged the produce; ``recover()`` re-publishes what is still pending
        self.notified_count = 0
        self._pending_notes: List[Dict[str, Any]] = []
        # standard starts are idempotent per transaction id too (a re-delivered hand-off batch
        # must not start a second standard process): tx id -> instance id over a bounded window,
        # native for integer ids (process/dedupe.py); other ids (e.g. strings) use a dict
        self.standard_dedupe_window = int(standard_dedupe_window)
        self.standard_dedupe_capacity = int(standard_dedupe_capacity or 4 * self.standard_dedupe_window)
        if self.standard_dedupe_capacity < self.standard_dedupe_window:
            raise ValueError("standard_dedupe_capacity must be >= standard_dedupe_window")
        from .dedupe import DedupeIndex
        self._std_index = DedupeIndex(self.standard_dedupe_capacity, gated=True)
        # admission batches of the index, oldest first: [new keys, gate] -- gate {partition: mark}
        # (erasable once committed past every mark, in any order) or None (ungated: count window)
        self._std_fifo: List[list] = []
        self.standard_forced_evictions = 0            # recovery only: journal beyond capacity
        self._committed: Dict[int, int] = {}          # partition -> engine's committed offset
        self.standard_evicted = 0
        self.standard_dedupe_full = 0                 # batches refused for lack of room
        self._std_by_tx: Dict[Any, int] = {}
        self._std_order: collections.deque = collections.deque()
        self.standard_duplicates = 0
        # audit of standard instances (never retained as objects): per admitted batch the first
        # id, the id stride, the new transaction ids and their proba / amount, newest last
        self.standard_audit_rows = int(standard_audit_rows)
        self._audit: collections.deque = collections.deque()
        self._audit_rows = 0
        # scored -> process started (the engine's hand-off items carry ``scored_ns``, the wall
        # clock their results were collected): 4 buckets per octave of ns, like the engine's
        self.handoff_hist = [0] * 256
        # journal appends (a write() that dirty-page throttling can stall): attribution
        from ..utils.lathist import LatHist
        self.journal_time = LatHist()

    @classmethod
    def from_config(cls, kie_cfg, **kw) -> "ProcessEngine":
        pred = kw.pop("prediction", None) or PredictionService(kie_cfg.confidence_threshold)
        return cls(kie_cfg.notification_timeout_s, kie_cfg.dmn_probability_threshold,
                   kie_cfg.dmn_amount_threshold, prediction=pred, **kw)

    # ------------------------------------------------------------------ ids
    def _iid(self, n: int) -> int:
        return self.shard + self.shards * int(n)

    def _n_of(self, iid: int) -> int:
        return (int(iid) - self.shard) // self.shards

    def _next_iid(self) -> int:
        iid = self._iid(self._next_n)
        self._next_n += 1
        return iid

    def _next_tid(self) -> int:
        return self.shard + self.shards * next(self._task_ids)

    def owns(self, iid: int) -> bool:
        """Whether instance / task id ``iid`` belongs to this shard."""
        return int(iid) % self.shards == self.shard

    # ------------------------------------------------------------------ journal
    def _record(self, inst: ProcessInstance) -> str:
        # a shallow copy of the fields: dataclasses.asdict deep-copies recursively and was 87 %
        # of a fraud start / signal (76 / 58 us -> the KIE event loop ran ~80 % busy at 7 K
        # fraud starts/s and queued starts for up to 0.6 s, profiles/r4/kie_handoff/)
        d = dict(vars(inst))
        d["state"] = inst.state.value
        rec = {"instance": d}
        if inst.task_id is not None and inst.task_id in self.tasks:
            rec["task"] = vars(self.tasks[inst.task_id])
        return json.dumps(rec, default=float) + "\n"

    def _write_journal(self, text: str) -> None:
        t0 = time.monotonic_ns()
        self._journal.write(text)
        self.journal_time.add(time.monotonic_ns() - t0)

    def _log(self, inst: ProcessInstance) -> None:
        if self._journal is None:
            return
        self._write_journal(self._record(inst))

    @classmethod
    def recover(cls, journal_path: str, **kw) -> "ProcessEngine":
        """Rebuild from the journal (last record per instance wins), then keep appending."""
        last: Dict[int, dict] = {}
        std_events: List[tuple] = []            # ("std", batch) / ("committed", offsets), in order
        notified = set()                        # outbox entries the broker acknowledged
        if os.path.exists(journal_path):
            with open(journal_path) as f:
                for line in f:
                    line = line.strip()
                    if line:
                        try:
                            rec = json.loads(line)
                        except json.JSONDecodeError:
                            continue        # the torn last line of a killed process
                        if "header" in rec:
                            h = rec["header"]
                            want = (int(kw.get("shard", 0)), max(1, int(kw.get("shards", 1))))
                            if (int(h["shard"]), int(h["shards"])) != want:
                                raise ValueError(
                                    f"journal {journal_path} was written by shard {h['shard']} of {h['shards']}, "
                                    f"this process is shard {want[0]} of {want[1]}: its instance ids would be "
                                    "decoded wrongly (start this shard with its own journal and kie.shards)")
                        elif "standard" in rec:
                            std_events.append(("std", rec["standard"]))
                        elif "committed" in rec:
                            std_events.append(("committed", rec["committed"]))
                        elif "notified" in rec:
                            notified.update(rec["notified"])
                        elif "instance" in rec:
                            last[rec["instance"]["id"]] = rec
        if os.path.exists(journal_path) and os.path.getsize(journal_path) > 0:
            with open(journal_path, "rb+") as f:            # end a torn last line, so the
                f.seek(-1, os.SEEK_END)                      # next record starts on its own
                if f.read(1) != b"\n":
                    f.write(b"\n")
        eng = cls(journal_path=journal_path, **kw)
        max_n, max_task = 0, 0
        for iid, rec in last.items():
            d = dict(rec["instance"])
            d["state"] = State(d["state"])
            inst = ProcessInstance(**d)
            eng.instances[iid] = inst
            max_n = max(max_n, eng._n_of(iid))
            txid = inst.variables.get("transaction_id")
            if inst.process_id == cls.FRAUD:
                eng.fraud_count += 1
                if txid is not None:
                    eng._by_tx[txid] = iid
                    eng._tx_order.append(txid)
                # the reference's outcome counters (README.md:593-599) come back too
                if inst.task_id is not None:
                    eng.outcome_counts[Outcome.INVESTIGATION.value] += 1
                if inst.outcome is not None:
                    eng.outcome_counts[inst.outcome] = eng.outcome_counts.get(inst.outcome, 0) + 1
                    eng._digest(inst)
                if inst.notified or iid in notified:
                    inst.notified = True
                    eng.notified_count += 1
                else:                           # in the outbox: published again on restart
                    eng._pending_notes.append(eng._notification(inst))
            if "task" in rec:
                t = UserTask(**rec["task"])
                eng.tasks[t.id] = t
                max_task = max(max_task, (t.id - eng.shard) // eng.shards)
            if inst.state == State.WAITING_CUSTOMER and inst.timer_due is not None:
                heapq.heappush(eng._timers, (inst.timer_due, iid))
        import numpy as np
        for kind, b in std_events:              # batched standard starts + commit watermarks
            if kind == "committed":
                eng._apply_committed(b)
                continue
            if "tx_i64" in b:                   # base64 of the new transaction ids (int64 LE)
                import base64
                tx = np.frombuffer(base64.b64decode(b["tx_i64"]), "<i8")
                ids = int(b["id0"]) + int(b.get("st", 1)) * np.arange(len(tx), dtype=np.int64)
                pr = np.frombuffer(base64.b64decode(b["p_f32"]), "<f4") if "p_f32" in b else None
                am = np.frombuffer(base64.b64decode(b["a_f32"]), "<f4") if "a_f32" in b else None
                eng._audit_add(int(b["id0"]), int(b.get("st", 1)), tx, pr, am)
            else:                               # round-3 form: JSON lists
                tx = b["transaction_id"]
                ids = b["id"] if "id" in b else list(range(int(b["id0"]), int(b["id0"]) + len(tx)))
            if len(ids):
                max_n = max(max_n, eng._n_of(int(np.max(ids))))
            eng.standard_count += len(tx)
            eng.outcome_counts[Outcome.STANDARD.value] += len(tx)
            gate = {int(k): int(v) for k, v in b["g"].items()} if b.get("g") else None
            eng._std_restore(tx, ids, gate=gate)
        for iid, rec in last.items():
            if rec["instance"]["process_id"] == cls.STANDARD:
                eng.standard_count += 1
                eng.outcome_counts[Outcome.STANDARD.value] += 1
                tx = rec["instance"]["variables"].get("transaction_id")
                if tx is not None:
                    eng._std_restore([tx], [iid])
        eng._std_evict()
        eng._next_n = max_n + 1
        eng._task_ids = itertools.count(max_task + 1)
        return eng

    # ------------------------------------------------------------------ notification outbox
    @staticmethod
    def _notification(inst: "ProcessInstance") -> Dict[str, Any]:
        v = inst.variables
        return {"customer_id": v.get("customer_id"), "transaction_id": v.get("transaction_id", v.get("tx_id")),
                "process_id": inst.id, "amount": v.get("amount"), "proba": v.get("proba")}

    def pending_notifications(self) -> List[Dict[str, Any]]:
        """The recovered outbox: notifications of fraud instances whose produce was never
        acknowledged (the caller publishes them again; the notifier dedupes by process id)."""
        with self._lock:
            out, self._pending_notes = self._pending_notes, []
        return out

    def mark_notified(self, iids) -> None:
        """The broker acknowledged these instances' CustomerNotifications: clear them from the
        outbox (one journal line per acknowledged batch)."""
        iids = [int(i) for i in iids]
        if not iids:
            return
        with self._lock:
            for i in iids:
                inst = self.instances.get(i)
                if inst is not None:
                    inst.notified = True
            self.notified_count += len(iids)
            if self._journal is not None:
                self._write_journal('{"notified": %s}\n' % json.dumps(iids))

    # ------------------------------------------------------------------ start
    def start(self, process_id: str, variables: Dict[str, Any]) -> int:
        if process_id.endswith(self.STANDARD) or process_id == self.STANDARD:
            return self.start_standard(variables)
        return self.start_fraud(variables)

    @staticmethod
    def _native_key(tx) -> bool:
        return isinstance(tx, (int,)) and not isinstance(tx, bool) and tx >= 0

    def _std_restore(self, txs, ids, gate=None) -> None:
        """Recovery: put admitted (transaction, instance) pairs back in the dedupe index."""
        import numpy as np
        txs = list(txs) if not hasattr(txs, "dtype") else txs
        if hasattr(txs, "dtype") or all(self._native_key(t) for t in txs):
            t64, i64 = np.asarray(txs, np.int64), np.asarray(ids, np.int64)
            self._restore_insert(t64, i64)
            self._fifo_add(t64, gate)
            self._std_evict()
            return
        for t, i in zip(txs, ids):
            if self._native_key(t):
                self._restore_insert(np.asarray([t], np.int64), np.asarray([i], np.int64))
                self._fifo_add([t], None)
            else:
                self._std_remember(t, int(i))

    def _restore_insert(self, t64, i64) -> None:
        from .dedupe import DedupeFull
        try:
            self._std_index.insert(t64, i64)
            return
        except DedupeFull:
            self._std_evict()
        while len(self._std_index) + len(t64) > self.standard_dedupe_capacity and self._std_fifo:
            keys, _gate = self._std_fifo.pop(0)       # journal older than the capacity: forced
            self.standard_forced_evictions += self._std_index.erase(keys)
        self._std_index.insert(t64, i64)

    # ------------------------------------------------------------------ commit-gated dedupe
    def _fifo_add(self, keys, gate) -> None:
        if not len(keys):
            return
        f = self._std_fifo
        if gate is None and f and f[-1][1] is None and isinstance(f[-1][0], list):
            f[-1][0].extend(int(k) for k in keys)   # runs of ungated starts share one entry
        else:
            f.append([list(keys) if gate is None else keys, gate])

    def _gate_open(self, gate) -> bool:
        c = self._committed
        return gate is None or all(c.get(p, -1) >= m for p, m in gate.items())

    def _std_evict(self) -> None:
        """While the index holds more than the window, erase the oldest batches that can no
        longer be re-delivered (every partition committed past their marks; ungated batches
        always).  A batch still exposed to a replay is skipped, never erased: the index grows
        instead, up to its capacity, then refuses admissions."""
        ix, f = self._std_index, self._std_fifo
        excess = len(ix) - self.standard_dedupe_window
        i = 0
        while excess > 0 and i < len(f):
            keys, gate = f[i]
            if not self._gate_open(gate):
                i += 1
                continue
            k = min(len(keys), excess)
            self.standard_evicted += ix.erase(keys[:k])
            excess -= k
            if k == len(keys):
                del f[i]
            else:
                f[i][0] = keys[k:]
                i += 1

    def _apply_committed(self, offsets) -> bool:
        changed = False
        for p, o in offsets.items():
            p, o = int(p), int(o)
            if o > self._committed.get(p, -1):
                self._committed[p] = o
                changed = True
        return changed

    def note_committed(self, offsets: Dict[int, int]) -> None:
        """The engine committed these Kafka offsets (partition -> next offset to consume): no
        replay will re-deliver a row below them, so dedupe keys gated under them may leave.
        Journaled (when it moves), so recovery rebuilds the same watermark."""
        with self._lock:
            if not self._apply_committed(offsets):
                return
            if self._journal is not None:
                self._write_journal('{"committed": %s}\n' % json.dumps(
                    {str(p): int(o) for p, o in offsets.items()}))
            self._std_evict()

    def dedupe_stats(self) -> Dict[str, int]:
        with self._lock:
            return {"keys": len(self._std_index), "window": self.standard_dedupe_window,
                    "capacity": self.standard_dedupe_capacity, "evicted": self.standard_evicted,
                    "refused_batches": self.standard_dedupe_full, "batches": len(self._std_fifo),
                    "recovery_forced_evictions": self.standard_forced_evictions,
                    "committed_partitions": len(self._committed)}

    # ------------------------------------------------------------------ standard audit
    def _audit_add(self, id0: int, st: int, tx, proba=None, amount=None) -> None:
        import numpy as np
        if self.standard_audit_rows <= 0 or not len(tx):
            return
        self._audit.append((int(id0), int(st), np.asarray(tx, np.int64),
                            None if proba is None else np.asarray(proba, np.float32),
                            None if amount is None else np.asarray(amount, np.float32)))
        self._audit_rows += len(tx)
        while self._audit and self._audit_rows - len(self._audit[0][2]) >= self.standard_audit_rows:
            self._audit_rows -= len(self._audit.popleft()[2])

    def _audit_find(self, iid: int):
        """(tx, proba, amount) of standard instance ``iid`` from the in-memory audit."""
        import bisect
        a = self._audit
        if not a:
            return None
        keys = [b[0] for b in a] if len(a) < 64 else None
        if keys is not None:
            i = bisect.bisect_right(keys, iid) - 1
        else:                                   # ids grow with admission: binary search
            lo, hi = 0, len(a) - 1
            i = -1
            while lo <= hi:
                mid = (lo + hi) // 2
                if a[mid][0] <= iid:
                    i, lo = mid, mid + 1
                else:
                    hi = mid - 1
        if i < 0:
            return None
        id0, st, tx, pr, am = a[i]
        k, r = divmod(iid - id0, st)
        if r or k >= len(tx):
            return None
        return (int(tx[k]), None if pr is None else float(pr[k]), None if am is None else float(am[k]))

    def find_transaction(self, tx_id, deep: bool = False) -> Optional[Dict[str, Any]]:
        """The process a transaction started on this shard (README.md:552: every transaction
        starts a standard or a fraud process): instance id, process, route, state / outcome and
        proba.  Fraud instances come from the live instance table; standard instances (counted,
        never retained as objects) from the in-memory audit of the last ``standard_audit_rows``
        admissions -- or, with ``deep``, from a scan of the journal (older history, slow).
        None: this shard never started a process for it (within the retention)."""
        if isinstance(tx_id, float) and tx_id.is_integer():
            tx_id = int(tx_id)
        with self._lock:
            iid = self._by_tx.get(tx_id)
            if iid is not None:
                inst = self.instances.get(iid)
                out = {"transaction_id": tx_id, "process-instance-id": iid, "process-id": self.FRAUD,
                       "route": "fraud", "source": "memory"}
                if inst is not None:
                    out.update(state=inst.state.value, outcome=inst.outcome, proba=inst.proba,
                               amount=inst.amount)
                return out
            iid = self._std_index.get(tx_id) if self._native_key(tx_id) else self._std_by_tx.get(tx_id)
            if iid is not None:
                out = {"transaction_id": tx_id, "process-instance-id": int(iid), "process-id": self.STANDARD,
                       "route": "standard", "state": State.COMPLETED.value, "outcome": Outcome.STANDARD.value,
                       "source": "memory"}
                hit = self._audit_find(int(iid))
                if hit is not None and hit[0] == tx_id:
                    out.update(proba=hit[1], amount=hit[2])
                return out
            journal = self._journal.name if self._journal is not None else None
        if deep and journal:
            return self._journal_find(journal, tx_id)
        return None

    def _journal_find(self, path: str, tx_id) -> Optional[Dict[str, Any]]:
        import base64

        import numpy as np
        found = None
        with open(path) as f:
            for line in f:
                if '"standard"' not in line[:16]:
                    continue
                try:
                    b = json.loads(line)["standard"]
                except (json.JSONDecodeError, KeyError):
                    continue
                if "tx_i64" not in b:
                    continue
                tx = np.frombuffer(base64.b64decode(b["tx_i64"]), "<i8")
                hit = np.nonzero(tx == int(tx_id))[0]
                if not len(hit):
                    continue
                k = int(hit[0])
                found = {"transaction_id": int(tx_id), "process-instance-id": int(b["id0"]) + int(b.get("st", 1)) * k,
                         "process-id": self.STANDARD, "route": "standard", "state": State.COMPLETED.value,
                         "outcome": Outcome.STANDARD.value, "source": "journal"}
                if "p_f32" in b:
                    found["proba"] = float(np.frombuffer(base64.b64decode(b["p_f32"]), "<f4")[k])
                if "a_f32" in b:
                    found["amount"] = float(np.frombuffer(base64.b64decode(b["a_f32"]), "<f4")[k])
                break                            # a transaction is admitted once
        return found

    def _std_remember(self, tx, iid: int) -> None:
        self._std_by_tx[tx] = iid
        self._std_order.append(tx)
        if len(self._std_order) > self.standard_dedupe_window:
            self._std_by_tx.pop(self._std_order.popleft(), None)

    def start_standard(self, variables: Dict[str, Any]) -> int:
        """Standard process (README.md:552): completes at once as STANDARD.  Idempotent per
        transaction id, like fraud starts."""
        txid = variables.get("transaction_id", variables.get("tx_id"))
        if isinstance(txid, float) and txid.is_integer():
            txid = int(txid)
        with self._lock:
            if self._native_key(txid):
                ids, new = self._assign_std([txid], self._iid(self._next_n))
                iid = int(ids[0])
                if not len(new):
                    self.standard_duplicates += 1
                    return iid
                self._next_n += 1
                self._fifo_add([txid], None)
                self._std_evict()
            else:
                if txid is not None and txid in self._std_by_tx:
                    self.standard_duplicates += 1
                    return self._std_by_tx[txid]
                iid = self._next_iid()
                if txid is not None:
                    self._std_remember(txid, iid)
            now = self.clock()
            inst = ProcessInstance(iid, self.STANDARD, dict(variables), State.COMPLETED,
                                   Outcome.STANDARD.value, now, now, history=["start", "approve"])
            self.standard_count += 1
            self.outcome_counts[Outcome.STANDARD.value] += 1
            self._remember_completed(inst)
            self._log(inst)
            return iid

    def start_standard_many(self, items) -> List[int]:
        """``start_standard_array`` with the ids as a list."""
        ids = self.start_standard_array(items)
        return ids.tolist() if hasattr(ids, "tolist") else ids

    def start_standard_array(self, items):
        """Standard processes for a whole hand-off batch (the engine's standard-routed rows of a
        scoring step).  ``items``: a list of variable dicts, or columns ``{"transaction_id":
        [...], "customer_id": [...], "amount": [...], "proba": [...]}`` (lists or numpy arrays --
        the compact form the router sends at ~1e5..1e6 standard rows a second).  Idempotent per
        transaction id (a re-delivered batch, or a transaction twice in one batch, starts once),
        through the native dedupe window (process/dedupe.py).  New instances get the shard's
        next ids in admission order; the batch is journaled as ONE compact record (first id,
        id stride, the new transaction ids), which ``recover()`` replays.  Returns the instance
        ids in order (an int64 array for numeric columns)."""
        import numpy as np
        gate = None
        if isinstance(items, dict):
            if "kafka_partition" in items or "commit_mark" in items:
                items = dict(items)
                kp, cm = items.pop("kafka_partition", None), items.pop("commit_mark", None)
                gate = _gate_of(kp, cm)
            tx = items.get("transaction_id", items.get("tx_id"))
            sc = items.get("scored_ns")
        else:
            tx = [it.get("transaction_id", it.get("tx_id")) for it in items]
            sc = [it.get("scored_ns") for it in items] if items and "scored_ns" in items[0] else None
        n = 0 if tx is None else len(tx)
        if sc is not None and len(sc) and sc[0]:
            self._note_handoff(int(sc[0]), n)
        if tx is None:
            return [self.start_standard(v) for v in rows_of(items)]
        if hasattr(tx, "dtype") and tx.dtype.kind in "iu":
            tx = np.ascontiguousarray(tx, np.int64)
        else:
            tl = list(tx)
            if not tl or not all(self._native_key(t) for t in tl):
                rows = rows_of(items) if isinstance(items, dict) else list(items)
                return [self.start_standard(v) for v in rows]
            tx = np.asarray(tl, np.int64)
        if n and int(tx.min()) < 0:
            rows = rows_of(items) if isinstance(items, dict) else list(items)
            return [self.start_standard(v) for v in rows]
        with self._lock:
            first = self._iid(self._next_n)
            ids, new = self._assign_std(tx, first)
            n_new = len(new)
            self._next_n += n_new
            self.standard_duplicates += n - n_new
            self.standard_count += n_new
            self.outcome_counts[Outcome.STANDARD.value] += n_new
            self._fifo_add(new, gate)
            if n_new:
                pr, am = _new_rows_column(items, "proba", ids, first, self.shards, n_new), \
                    _new_rows_column(items, "amount", ids, first, self.shards, n_new)
                self._audit_add(first, self.shards, new, pr, am)
            if self._journal is not None and n_new:
                import base64
                tx64 = base64.b64encode(new.astype("<i8").tobytes()).decode()
                extra = ""
                if pr is not None:
                    extra += ', "p_f32": "%s"' % base64.b64encode(pr.astype("<f4").tobytes()).decode()
                if am is not None:
                    extra += ', "a_f32": "%s"' % base64.b64encode(am.astype("<f4").tobytes()).decode()
                if gate:
                    extra += ', "g": %s' % json.dumps({str(p): m for p, m in gate.items()})
                t0 = time.monotonic_ns()
                self._journal.write('{"standard": {"id0": %d, "st": %d, "tx_i64": "%s"%s}}\n'
                                    % (first, self.shards, tx64, extra))
                self.journal_time.add(time.monotonic_ns() - t0)
            self._std_evict()
        return ids

    def _assign_std(self, tx, first: int):
        """Admit into the gated index; a full index first evicts what commits allow."""
        from .dedupe import DedupeFull
        if len(tx) > self.standard_dedupe_capacity:
            raise ValueError(f"a standard batch of {len(tx)} rows exceeds the dedupe capacity "
                             f"({self.standard_dedupe_capacity}): it could never be admitted")
        try:
            return self._std_index.assign(tx, first, self.shards)
        except DedupeFull:
            self._std_evict()
            try:
                return self._std_index.assign(tx, first, self.shards)
            except DedupeFull:
                self.standard_dedupe_full += 1
                raise

    def _note_handoff(self, scored_ns, n: int = 1) -> None:
        if not scored_ns or n <= 0:
            return
        dt = time.time_ns() - int(scored_ns)
        if dt > 0:
            import math
            self.handoff_hist[min(255, int(4.0 * math.log2(dt)))] += n

    def handoff_latency_us(self) -> Dict[str, Any]:
        """p50 / p99 of scored -> started over every start that carried ``scored_ns``."""
        h = self.handoff_hist
        tot = sum(h)
        if not tot:
            return {"n": 0}
        out = {"n": tot}
        for q, name in ((0.5, "p50"), (0.99, "p99")):
            k, c = q * (tot - 1), 0
            for i, v in enumerate(h):
                c += v
                if c > k:
                    out[name] = round(2.0 ** ((i + 0.5) / 4.0) / 1e3, 1)   # bucket mid, us
                    break
        return out

    def start_fraud(self, variables: Dict[str, Any]) -> int:
        """Idempotent per transaction id: at-least-once delivery (a re-scored transaction
        after a rank fail-over) returns the existing instance instead of starting another."""
        self._note_handoff(variables.get("scored_ns"))
        txid = variables.get("transaction_id", variables.get("tx_id"))
        with self._lock:
            if txid is not None and txid in self._by_tx:
                self.duplicates += 1
                return self._by_tx[txid]
            iid = self._next_iid()
            self.fraud_count += 1
            if txid is not None:
                self._by_tx[txid] = iid
                self._tx_order.append(txid)
                if len(self._tx_order) > self.dedupe_window:
                    self._by_tx.pop(self._tx_order.popleft(), None)
            now = self.clock()
            inst = ProcessInstance(iid, self.FRAUD, dict(variables), State.WAITING_CUSTOMER, None, now,
                                   timer_due=now + self.timeout, history=["start", "CustomerNotification"])
            self.instances[iid] = inst
            heapq.heappush(self._timers, (inst.timer_due, iid))
            self._log(inst)
        if self.publish_notification is not None:
            self.publish_notification({
                "customer_id": variables.get("customer_id"),
                "transaction_id": variables.get("transaction_id", variables.get("tx_id")),
                "process_id": iid,
                "amount": variables.get("amount"),
                "proba": variables.get("proba"),
            })
        return iid

    def start_fraud_many(self, items) -> List[int]:
        """Fraud processes for a whole hand-off batch (a list of variable dicts, or columns):
        the same per-transaction semantics as ``start_fraud`` -- idempotent per transaction id,
        one journal record and one CustomerNotification per new instance -- under one lock
        acquisition, with the batch's journal records in one write.  Returns the instance ids
        in order (the existing one for a duplicate)."""
        rows = rows_of(items) if isinstance(items, dict) else items
        out: List[int] = []
        notes: List[Dict[str, Any]] = []
        lines: List[str] = []
        for v in rows:
            self._note_handoff(v.get("scored_ns"))
        with self._lock:
            now = self.clock()
            due = now + self.timeout
            by_tx, order = self._by_tx, self._tx_order
            for v in rows:
                txid = v.get("transaction_id", v.get("tx_id"))
                if txid is not None and txid in by_tx:
                    self.duplicates += 1
                    out.append(by_tx[txid])
                    continue
                iid = self._next_iid()
                self.fraud_count += 1
                if txid is not None:
                    by_tx[txid] = iid
                    order.append(txid)
                inst = ProcessInstance(iid, self.FRAUD, dict(v), State.WAITING_CUSTOMER, None, now,
                                       timer_due=due, history=["start", "CustomerNotification"])
                self.instances[iid] = inst
                heapq.heappush(self._timers, (due, iid))
                if self._journal is not None:
                    lines.append(self._record(inst))
                if self.publish_notification is not None:
                    notes.append({"customer_id": v.get("customer_id"), "transaction_id": txid, "process_id": iid,
                                  "amount": v.get("amount"), "proba": v.get("proba")})
                out.append(iid)
            while len(order) > self.dedupe_window:
                by_tx.pop(order.popleft(), None)
            if lines:
                self._write_journal("".join(lines))
        for m in notes:
            self.publish_notification(m)
        return out

    # ------------------------------------------------------------------ signal
    def signal(self, instance_id: int, name: str, payload: Any) -> bool:
        """Customer response signal.  Returns False if the instance is not waiting (timer
        already fired, unknown id, or duplicate delivery -- at-least-once safe)."""
        with self._lock:
            inst = self.instances.get(int(instance_id))
            if inst is None or inst.state != State.WAITING_CUSTOMER:
                return False
            approved = _truthy(payload)
            inst.history.append(f"signal:{name}:{approved}")
            if approved:
                self._complete(inst, Outcome.APPROVED_BY_CUSTOMER)
                if self.metrics:
                    self.metrics.approved.observe(inst.amount)
            else:
                self._complete(inst, Outcome.CANCELLED)
                if self.metrics:
                    self.metrics.rejected.observe(inst.amount)
            return True

    # ------------------------------------------------------------------ timers
    def tick(self, now: Optional[float] = None) -> int:
        """Fire every due timer; returns how many fired."""
        now = self.clock() if now is None else now
        fired = 0
        while True:
            with self._lock:
                if not self._timers or self._timers[0][0] > now:
                    break
                due, iid = heapq.heappop(self._timers)
                inst = self.instances.get(iid)
                if inst is None or inst.state != State.WAITING_CUSTOMER or inst.timer_due != due:
                    continue
                inst.history.append("timer:Customer notification expired")
                decision = investigation_decision(inst.proba, inst.amount, self.p_thr, self.a_thr)
                if decision == Decision.APPROVE:
                    self._complete(inst, Outcome.APPROVED_LOW_AMOUNT)
                    if self.metrics:
                        self.metrics.approved_low.observe(inst.amount)
                    fired += 1
                    continue
                if self.metrics:
                    self.metrics.investigation.observe(inst.amount)
                self.outcome_counts[Outcome.INVESTIGATION.value] += 1
                tid = self._next_tid()
                task = UserTask(tid, iid, inputs={"amount": inst.amount, "proba": inst.proba,
                                                  "transaction_id": inst.variables.get("transaction_id"),
                                                  "customer_id": inst.variables.get("customer_id")})
                self.tasks[tid] = task
                inst.state = State.USER_TASK
                inst.task_id = tid
                inst.history.append("UserTask:Assign case")
                fired += 1
            # prediction service outside the lock (may be a remote call)
            pred = self.prediction.predict(task.inputs)
            with self._lock:
                task.suggested_outcome, task.confidence = pred.outcome, pred.confidence
                if self.prediction.should_auto_complete(pred):
                    self._complete_task_locked(task, pred.outcome, by="prediction-service")
                else:
                    self._log(inst)
        return fired

    def next_timer_due(self) -> Optional[float]:
        with self._lock:
            return self._timers[0][0] if self._timers else None

    # ------------------------------------------------------------------ tasks
    def list_tasks(self, status: Optional[str] = "Ready") -> List[UserTask]:
        with self._lock:
            return [t for t in self.tasks.values() if status is None or t.status == status]

    def complete_task(self, task_id: int, outcome: str, by: str = "investigator") -> bool:
        with self._lock:
            task = self.tasks.get(int(task_id))
            if task is None or task.status == "Completed":
                return False
            self._complete_task_locked(task, outcome, by)
        self.prediction.train(task.inputs, {"outcome": outcome})
        return True

    def _complete_task_locked(self, task: UserTask, outcome: str, by: str) -> None:
        task.status, task.outcome, task.completed_by = "Completed", outcome, by
        inst = self.instances[task.instance_id]
        res = Outcome.INVESTIGATION_CLOSED_FRAUD if outcome in ("rejected", "fraud", False, "false") \
            else Outcome.INVESTIGATION_CLOSED_LEGIT
        inst.history.append(f"task-complete:{outcome}:{by}")
        self._complete(inst, res)

    # ------------------------------------------------------------------ helpers
    def _complete(self, inst: ProcessInstance, outcome: Outcome) -> None:
        inst.state = State.COMPLETED
        inst.outcome = outcome.value
        inst.completed = self.clock()
        inst.timer_due = None
        self.outcome_counts[outcome.value] += 1
        if inst.process_id == self.FRAUD:
            self._digest(inst)
        self._log(inst)
        self._remember_completed(inst)

    def _digest(self, inst: ProcessInstance) -> None:
        h = hashlib.blake2b(f"{inst.variables.get('transaction_id')}:{inst.outcome}".encode(), digest_size=8)
        self.outcome_digest = (self.outcome_digest + int.from_bytes(h.digest(), "little")) & 0xFFFFFFFFFFFFFFFF

    def _remember_completed(self, inst: ProcessInstance) -> None:
        if inst.process_id == self.STANDARD:
            return          # standard instances are counted, not retained (hot path volume)
        self._completed_order.append(inst.id)
        while len(self._completed_order) > self.keep_completed:
            old = self._completed_order.popleft()
            gone = self.instances.pop(old, None)
            if gone is not None and gone.task_id is not None:
                self.tasks.pop(gone.task_id, None)

    def get(self, instance_id: int) -> Optional[ProcessInstance]:
        with self._lock:
            return self.instances.get(int(instance_id))

    def active_count(self) -> int:
        with self._lock:
            return sum(1 for i in self.instances.values() if i.state != State.COMPLETED)

    def close(self) -> None:
        if self._journal:
            self._journal.close()
            self._journal = None


def columns_of(items) -> Dict[str, list]:
    """Variables of many process starts as columns: accepts a list of dicts or a dict of
    equally long lists (``tx_id`` is accepted for ``transaction_id``)."""
    if isinstance(items, dict):
        cols = {k: (v.tolist() if hasattr(v, "tolist") else list(v)) for k, v in items.items()}
    else:
        keys: List[str] = []
        for it in items:
            for k in it:
                if k not in keys:
                    keys.append(k)
        cols = {k: [it.get(k) for it in items] for k in keys}
    if "transaction_id" not in cols and "tx_id" in cols:
        cols["transaction_id"] = cols.pop("tx_id")
    lens = {len(v) for v in cols.values()}
    if len(lens) > 1:
        raise ValueError("columns of different lengths")
    return cols


def _gate_of(kp, cm) -> Optional[Dict[int, int]]:
    """{partition: max commit mark} of a hand-off batch's gate columns (None if absent)."""
    import numpy as np
    if kp is None or cm is None or not len(kp):
        return None
    kp = np.asarray(kp, np.int64)
    cm = np.asarray(cm, np.int64)
    if kp.shape != cm.shape:
        raise ValueError("kafka_partition / commit_mark columns of different lengths")
    out: Dict[int, int] = {}
    for p in np.unique(kp):
        out[int(p)] = int(cm[kp == p].max())
    return out


def _new_rows_column(items, name: str, ids, first: int, stride: int, n_new: int):
    """Column ``name`` of the newly admitted rows of a standard batch (their ids are
    first + stride * k, k < n_new, each row's position its first occurrence), or None."""
    import numpy as np
    col = items.get(name) if isinstance(items, dict) else None
    if col is None:
        return None
    col = np.asarray(col, np.float32)
    ids = np.asarray(ids, np.int64)
    k = (ids - first) // stride
    fresh = (k >= 0) & ((ids - first) % stride == 0)
    out = np.zeros(n_new, np.float32)
    pos = np.nonzero(fresh)[0]
    # duplicates of a new key inside one batch share its id: keep the first occurrence's value
    out[k[pos][::-1]] = col[pos][::-1]
    return out


def _ncols(cols: Dict[str, list]) -> int:
    return len(next(iter(cols.values()))) if cols else 0


def rows_of(items) -> List[Dict[str, Any]]:
    """The inverse of columns_of: a list of variable dicts."""
    if not isinstance(items, dict):
        return list(items)
    cols = columns_of(items)
    keys = list(cols)
    return [{k: cols[k][i] for k in keys} for i in range(_ncols(cols))]


def _truthy(payload: Any) -> bool:
    if isinstance(payload, dict):
        for k in ("response", "approved", "value", "made_transaction"):
            if k in payload:
                return _truthy(payload[k])
        return False
    if isinstance(payload, str):
        return payload.strip().lower() in ("true", "1", "yes", "approved", CustomerResponse.APPROVED.value)
    return bool(payload)
