"""Transaction router: the replacement for the Camel router ``ccd-fuse`` (deploy/router.yaml;
README.md:424-459, 543-552, 565-569).

Reference hot loop (per transaction): consume ``odh-demo`` -> POST to Seldon -> Drools ->
start a KIE process.  Here the router receives WHOLE SCORED MICRO-BATCHES from the GPU
engine (or from the predict() path) and:

* counts ``transaction.incoming`` and ``transaction.outgoing{type}`` (README.md:524-526);
* starts a *fraud* process per fraud-routed transaction (KIE hand-off, README.md:552);
* standard-routed transactions are counted (``standard_mode="count"``, default: at
  hundreds of millions of tx/s a process instance per legit transaction is not a sane
  design), or start a standard process each (``"process"``, reference-compatible mode);
* consumes ``ccd-customer-response`` and signals the waiting fraud process, counting
  ``notifications.incoming{response}`` (README.md:528-530, 569, 605);
* counts ``notifications.outgoing`` when a fraud process publishes its notification.
"""
from __future__ import annotations

import json
import threading
from typing import Any, Dict, Optional

import numpy as np

from ..contracts.outcomes import CustomerResponse, Route
from ..metrics.exporter import RouterMetrics
from .rules import RuleSet


def standard_columns(rec: np.ndarray, marks: Optional[Dict[int, int]] = None) -> Dict[str, np.ndarray]:
    """Scored records -> the column batch a standard-process hand-off carries (numpy columns:
    KieClient sends them as a binary CCOL body, process/kie_server.py encode_columns).

    ``marks`` (partition -> an offset above every scored row of it, the engine service's
    commit marks) adds the commit-gate columns ``kafka_partition`` / ``commit_mark``: the KIE
    shard keeps these transactions in its dedupe index until the engine's committed offsets
    pass the mark (process/engine.py note_committed)."""
    cols = {"transaction_id": rec["tx_id"].astype(np.int64), "customer_id": rec["customer"].astype(np.int64),
            "amount": rec["amount"].astype(np.float32), "proba": rec["proba"].astype(np.float32)}
    if marks:
        part = rec["partition"].astype(np.int64)
        lut = np.zeros(int(max(int(part.max()) if len(part) else 0, max(marks))) + 1, np.int64)
        for p, m in marks.items():
            lut[int(p)] = int(m)
        mark = lut[part]
        if len(mark) and int(mark.min()) <= 0:
            raise ValueError("standard rows of a partition without a commit mark")
        cols["kafka_partition"] = part
        cols["commit_mark"] = mark
    return cols


class Router:
    def __init__(self, rules: RuleSet, processes, metrics: Optional[RouterMetrics] = None,
                 standard_mode: str = "count", handoff=None):
        """``handoff``: a router.handoff.KieHandoff -- fraud starts and customer-response
        signals are then enqueued (pooled, retried, never blocking the caller) instead of
        sent synchronously; ``last_handoff_seq`` is the sequence number of the latest one."""
        if standard_mode not in ("count", "process"):
            raise ValueError("standard_mode must be 'count' or 'process'")
        self.rules = rules
        self.processes = processes            # ProcessEngine or KieClient (start_fraud/start_standard/signal)
        self.metrics = metrics or RouterMetrics()
        self.standard_mode = standard_mode
        self._lock = threading.Lock()
        self.fraud_started = 0
        self.signals_ok = 0
        self.signals_stale = 0
        self.handoff = handoff
        self.last_handoff_seq = -1
        self.standard_started = 0
        # wall-clock ns the current batch of results was collected from the engine (set by the
        # engine service): hand-off items carry it, KIE measures scored -> process started
        self.scored_ns: Optional[int] = None

    # ------------------------------------------------------------------ scoring results
    def on_scored(self, ids, customers, proba, X: Optional[np.ndarray] = None,
                  amounts: Optional[np.ndarray] = None, routes: Optional[np.ndarray] = None) -> Dict[str, int]:
        """A scored batch: ``routes`` from the GPU epilogue are used as-is when the rule set is
        threshold-only; otherwise the rule set is evaluated vectorised on the batch."""
        proba = np.asarray(proba).reshape(-1)
        n = proba.shape[0]
        if amounts is None and X is not None:
            amounts = np.asarray(X)[:, -1]
        if routes is None or self.rules.threshold_only is None:
            routes = self.rules.evaluate(proba, X=X, amount=amounts)
        routes = np.asarray(routes).reshape(-1)
        fraud_idx = np.nonzero(routes == Route.FRAUD)[0]
        self.metrics.tx_incoming.inc(n)
        self.metrics.tx_outgoing.labels(type="fraud").inc(len(fraud_idx))
        self.metrics.tx_outgoing.labels(type="standard").inc(n - len(fraud_idx))
        for i in fraud_idx:
            self._start_fraud(int(ids[i]), int(customers[i]) if customers is not None else 0,
                              float(amounts[i]) if amounts is not None else 0.0, float(proba[i]))
        if self.standard_mode == "process":
            si = np.nonzero(routes != Route.FRAUD)[0]
            if len(si):
                cols = {"transaction_id": [int(ids[i]) for i in si],
                        "customer_id": [int(customers[i]) if customers is not None else 0 for i in si],
                        "amount": [float(amounts[i]) if amounts is not None else 0.0 for i in si],
                        "proba": [float(proba[i]) for i in si]}
                if self.handoff is not None:
                    self.last_handoff_seq = self.handoff.submit_standard(cols)
                elif hasattr(self.processes, "start_standard_many"):
                    self.processes.start_standard_many(cols)
                else:
                    for i in si:
                        self.processes.start_standard({"transaction_id": int(ids[i]), "proba": float(proba[i]),
                                                       "amount": float(amounts[i]) if amounts is not None else 0.0})
                with self._lock:
                    self.standard_started += len(si)
        return {"incoming": n, "fraud": int(len(fraud_idx)), "standard": int(n - len(fraud_idx))}

    def on_flagged(self, flagged: np.ndarray, total_rows: int,
                   standard: Optional[np.ndarray] = None, marks: Optional[Dict[int, int]] = None) -> Dict[str, int]:
        """Engine hot path: ``flagged`` = the fraud-routed rows (the engine's flagged-record
        array; the GPU epilogue counted the rest).  ``standard``: with ``standard_mode="process"``
        the engine's standard-routed scored records (SCORED_DTYPE: tx_id, customer, proba,
        amount) -- each starts a standard process, like the reference router does for every
        low-probability transaction (README.md:552)."""
        nf = int(len(flagged))
        self.metrics.tx_incoming.inc(total_rows)
        self.metrics.tx_outgoing.labels(type="fraud").inc(nf)
        self.metrics.tx_outgoing.labels(type="standard").inc(total_rows - nf)
        std_cols = None
        if self.standard_mode == "process" and standard is not None and len(standard):
            std_cols = standard_columns(standard, marks)
            if self.scored_ns:
                std_cols["scored_ns"] = np.full(len(standard), self.scored_ns, np.int64)
        if self.handoff is not None:                        # async, retried, acked later
            seq = -1
            if nf:
                ts = self.scored_ns
                seq = self.handoff.submit_starts(
                    [{"transaction_id": int(r["tx_id"]), "customer_id": int(r["customer"]),
                      "amount": float(r["amount"]), "proba": float(r["proba"]), "scored_ns": ts}
                     for r in flagged] if ts else
                    [{"transaction_id": int(r["tx_id"]), "customer_id": int(r["customer"]),
                      "amount": float(r["amount"]), "proba": float(r["proba"])} for r in flagged])
                with self._lock:
                    self.fraud_started += nf
            if std_cols is not None:
                seq = self.handoff.submit_standard(std_cols)
                with self._lock:
                    self.standard_started += len(standard)
            self.last_handoff_seq = seq
            return {"incoming": total_rows, "fraud": nf, "standard": total_rows - nf}
        many = getattr(self.processes, "start_fraud_many", None)
        if many is not None and nf > 1:                     # one hand-off for the whole step
            many([{"transaction_id": int(r["tx_id"]), "customer_id": int(r["customer"]),
                   "amount": float(r["amount"]), "proba": float(r["proba"])} for r in flagged])
            with self._lock:
                self.fraud_started += nf
        else:
            for r in flagged:
                self._start_fraud(int(r["tx_id"]), int(r["customer"]), float(r["amount"]), float(r["proba"]))
        if std_cols is not None:
            smany = getattr(self.processes, "start_standard_many", None)
            if smany is not None:
                smany(std_cols)
            else:
                from ..process.engine import rows_of
                for v in rows_of(std_cols):
                    self.processes.start_standard(v)
            with self._lock:
                self.standard_started += len(standard)
        return {"incoming": total_rows, "fraud": nf, "standard": total_rows - nf}

    def _start_fraud(self, tx_id: int, customer: int, amount: float, proba: float) -> None:
        self.processes.start_fraud({"transaction_id": tx_id, "customer_id": customer,
                                    "amount": amount, "proba": proba})
        with self._lock:
            self.fraud_started += 1

    # ------------------------------------------------------------------ notification loop
    def on_notification_sent(self, _msg: Any = None) -> None:
        self.metrics.notif_outgoing.inc()

    def on_response(self, raw) -> bool:
        msg = json.loads(raw) if isinstance(raw, (bytes, bytearray, str)) else raw
        approved = bool(msg.get("response"))
        self.metrics.notif_incoming.labels(
            response=CustomerResponse.from_bool(approved).value).inc()
        if self.handoff is not None:                        # outcome counted by the hand-off
            self.last_handoff_seq = self.handoff.submit_signal(int(msg["process_id"]), "customerResponse", approved)
            return True
        ok = self.processes.signal(int(msg["process_id"]), "customerResponse", approved)
        with self._lock:
            if ok:
                self.signals_ok += 1
            else:
                self.signals_stale += 1
        return ok
