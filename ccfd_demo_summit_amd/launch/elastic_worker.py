"""Lease-driven stream worker: the failure-tolerant consumer loop used by every rank
(SURVEY.md §5 failure detection; §4.1 "kill a rank mid-stream, its partitions are
re-assigned, final counts correct with no double count").

Per tick: renew/claim partition leases (parallel/elastic.py); for every owned partition
fetch from the committed offset, score (any scorer: GPU engine or CPU), route, then commit
the offset together with the partition's cumulative counts in ONE store write.  A rank that
dies between scoring and committing loses nothing: the next owner re-scores from the
committed offset, the process engine de-duplicates by transaction id, and the committed
counts -- not the scorer's -- are the exactly-once global counters.
"""
from __future__ import annotations

from typing import Dict, Optional

from ..ingest.codec import decode_records
from ..parallel.elastic import PartitionLeases
from ..utils.faults import FaultPlan


class ElasticWorker:
    def __init__(self, rank: int, leases: PartitionLeases, broker, topic: str, scorer, router,
                 group: str = "ccfd-engine", max_records: int = 4096, faults: Optional[FaultPlan] = None):
        self.rank = rank
        self.leases = leases
        self.broker = broker
        self.topic = topic
        self.scorer = scorer
        self.router = router
        self.group = group
        self.max_records = max_records
        self.pos: Dict[int, int] = {}
        self.counts: Dict[int, list] = {}
        self.alive = True
        self.scored_rows = 0
        self.routed = [0, 0]             # rows routed, fraud-routed (incl. re-scored rows): X2 feed
        # injected faults (utils/faults.py; CCFD_FAULTS): drop / delay / crash this rank
        self.faults = faults if faults is not None else FaultPlan.from_env(rank)

    def _adopt(self, p: int) -> None:
        off, rows, fraud = self.leases.committed(p)
        if off == 0:
            c = self.broker.committed(self.group, self.topic, p)
            off = c or self.broker.begin_offset(self.topic, p)
        self.pos[p] = off
        self.counts[p] = [rows, fraud]

    def tick(self, crash_before_commit: bool = False) -> int:
        """One loop iteration; returns rows scored.  ``crash_before_commit`` is the fault
        injection hook: score a batch, then die without committing it."""
        if not self.alive:
            return 0
        if self.faults is not None:
            self.faults.step()
        gained, lost = self.leases.tick()
        for p in gained:
            self._adopt(p)
        for p in lost:
            self.pos.pop(p, None)
            self.counts.pop(p, None)
        n = 0
        for p in self.leases.owned():
            if p not in self.pos:
                self._adopt(p)
            recs = self.broker.fetch(self.topic, p, self.pos[p], self.max_records)
            if not recs:
                continue
            if self.faults is not None and self.faults.drop():
                continue                           # lost in flight: re-fetched from the committed offset
            X, ids, cust = decode_records([r.value for r in recs])
            proba, route = self.scorer.score(X)
            res = self.router.on_scored(ids, cust, proba, X=X, routes=route)
            n += len(X)
            self.scored_rows += len(X)
            self.routed[0] += res["incoming"]
            self.routed[1] += res["fraud"]
            if crash_before_commit:
                self.alive = False                 # dies: no commit, no lease renewal
                return n
            nxt = recs[-1].offset + 1
            self.counts[p][0] += res["incoming"]
            self.counts[p][1] += res["fraud"]
            if self.leases.commit(p, nxt, *self.counts[p]):
                self.broker.commit(self.group, self.topic, p, nxt)
                self.pos[p] = nxt
        return n
