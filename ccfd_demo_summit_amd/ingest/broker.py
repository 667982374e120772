"""In-process message broker with Kafka semantics (topics, partitions, offsets, consumer
groups, committed offsets).

The reference runs a 3-broker Strimzi Kafka cluster (deploy/frauddetection_cr.yaml:73-77)
carrying three topics.  This broker is the "fake broker" of SURVEY.md
§1.1/§4.1: the same produce/fetch/commit contract, used by tests, benchmarks and
single-node deployments; ``kafka_wire.KafkaBroker`` implements the same interface over
the Kafka wire protocol for a real cluster.

Delivery is at-least-once: a consumer's position only becomes durable when committed
(the router commits after scoring -- SURVEY.md §5 "Failure detection").  Rebalancing
assigns partitions round-robin over the live members of a group (partition p goes to the
member at index p % n_members, members sorted by id), like Kafka's RoundRobinAssignor.
"""
from __future__ import annotations

import itertools
import threading
import time
import zlib
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple


@dataclass
class Record:
    topic: str
    partition: int
    offset: int
    key: Optional[bytes]
    value: bytes
    timestamp: float
    headers: Tuple = ()


class _Partition:
    __slots__ = ("records", "base")

    def __init__(self):
        self.records: List[Record] = []
        self.base = 0          # offset of records[0] (after retention trimming)

    @property
    def end(self) -> int:
        return self.base + len(self.records)


class BrokerError(RuntimeError):
    pass


class InProcBroker:
    def __init__(self, default_partitions: int = 1, retention: Optional[int] = None):
        self.default_partitions = default_partitions
        self.retention = retention
        self._topics: Dict[str, List[_Partition]] = {}
        self._committed: Dict[Tuple[str, str, int], int] = {}
        self._groups: Dict[str, Dict[str, "Consumer"]] = {}
        self._generation: Dict[str, int] = {}
        self._rr = itertools.count()
        self._cv = threading.Condition()

    # ------------------------------------------------------------------ topics
    def create_topic(self, name: str, partitions: Optional[int] = None) -> None:
        with self._cv:
            if name not in self._topics:
                self._topics[name] = [_Partition() for _ in range(partitions or self.default_partitions)]

    def topics(self) -> Dict[str, int]:
        with self._cv:
            return {t: len(p) for t, p in self._topics.items()}

    def partitions(self, topic: str) -> int:
        self.create_topic(topic)
        return len(self._topics[topic])

    # ------------------------------------------------------------------ produce / fetch
    def produce(self, topic: str, value: bytes, key: Optional[bytes] = None,
                partition: Optional[int] = None, headers: Tuple = ()) -> Tuple[int, int]:
        self.create_topic(topic)
        with self._cv:
            parts = self._topics[topic]
            if partition is None:
                if key is not None:
                    partition = zlib.crc32(key) % len(parts)
                else:
                    partition = next(self._rr) % len(parts)
            if not 0 <= partition < len(parts):
                raise BrokerError(f"{topic}: no partition {partition}")
            P = parts[partition]
            off = P.end
            P.records.append(Record(topic, partition, off, key, bytes(value), time.time(), headers))
            if self.retention is not None and len(P.records) > self.retention:
                drop = len(P.records) - self.retention
                del P.records[:drop]
                P.base += drop
            self._cv.notify_all()
            return partition, off

    def produce_many(self, topic: str, values: Iterable[bytes], partition: Optional[int] = None) -> int:
        """Append many records; with an explicit partition this takes the lock and wakes the
        consumers once for the whole batch (the one-transaction-per-message producer path)."""
        if partition is None:
            n = 0
            for v in values:
                self.produce(topic, v)
                n += 1
            return n
        self.create_topic(topic)
        now = time.time()
        with self._cv:
            parts = self._topics[topic]
            if not 0 <= partition < len(parts):
                raise BrokerError(f"{topic}: no partition {partition}")
            P = parts[partition]
            off = P.end
            recs = [Record(topic, partition, off + i, None, bytes(v), now) for i, v in enumerate(values)]
            P.records.extend(recs)
            if self.retention is not None and len(P.records) > self.retention:
                drop = len(P.records) - self.retention
                del P.records[:drop]
                P.base += drop
            self._cv.notify_all()
            return len(recs)

    def fetch(self, topic: str, partition: int, offset: int, max_records: int = 1000) -> List[Record]:
        with self._cv:
            P = self._topics[topic][partition]
            if offset < P.base:
                offset = P.base          # auto.offset.reset=earliest for trimmed offsets
            i = offset - P.base
            return P.records[i:i + max_records]

    def end_offset(self, topic: str, partition: int) -> int:
        with self._cv:
            return self._topics[topic][partition].end

    def begin_offset(self, topic: str, partition: int) -> int:
        with self._cv:
            return self._topics[topic][partition].base

    def wait_for_data(self, predicate, timeout: float) -> bool:
        with self._cv:
            return self._cv.wait_for(predicate, timeout)

    # ------------------------------------------------------------------ offsets
    def commit(self, group: str, topic: str, partition: int, offset: int) -> None:
        with self._cv:
            k = (group, topic, partition)
            self._committed[k] = max(offset, self._committed.get(k, 0))

    def committed(self, group: str, topic: str, partition: int) -> Optional[int]:
        with self._cv:
            return self._committed.get((group, topic, partition))

    def lag(self, group: str, topic: str) -> int:
        with self._cv:
            return sum(P.end - self._committed.get((group, topic, p), P.base)
                       for p, P in enumerate(self._topics.get(topic, [])))

    # ------------------------------------------------------------------ groups
    def consumer(self, group: str, topics: Sequence[str], member_id: Optional[str] = None,
                 auto_commit: bool = False) -> "Consumer":
        for t in topics:
            self.create_topic(t)
        c = Consumer(self, group, list(topics), member_id or f"{group}-{next(self._rr)}", auto_commit)
        with self._cv:
            self._groups.setdefault(group, {})[c.member_id] = c
            self._rebalance(group)
        return c

    def _leave(self, c: "Consumer") -> None:
        with self._cv:
            members = self._groups.get(c.group, {})
            members.pop(c.member_id, None)
            self._rebalance(c.group)

    def _rebalance(self, group: str) -> None:
        members = sorted(self._groups.get(group, {}).values(), key=lambda m: m.member_id)
        self._generation[group] = self._generation.get(group, 0) + 1
        for m in members:
            m._assignment = []
        if not members:
            return
        for t in sorted({t for m in members for t in m.topics}):
            subs = [m for m in members if t in m.topics]
            for p in range(len(self._topics[t])):
                subs[p % len(subs)]._assignment.append((t, p))
        for m in members:
            m._positions = {tp: m._positions.get(tp, self._committed.get((group,) + tp, self._topics[tp[0]][tp[1]].base))
                            for tp in m._assignment}
            m.generation = self._generation[group]
        self._cv.notify_all()


class Consumer:
    def __init__(self, broker: InProcBroker, group: str, topics: List[str], member_id: str, auto_commit: bool):
        self.broker = broker
        self.group = group
        self.topics = topics
        self.member_id = member_id
        self.auto_commit = auto_commit
        self._assignment: List[Tuple[str, int]] = []
        self._positions: Dict[Tuple[str, int], int] = {}
        self.generation = 0
        self.closed = False

    @property
    def assignment(self) -> List[Tuple[str, int]]:
        return list(self._assignment)

    def _has_data(self) -> bool:
        return any(self.broker._topics[t][p].end > self._positions.get((t, p), 0) for t, p in self._assignment)

    def poll(self, timeout: float = 0.0, max_records: int = 500) -> List[Record]:
        if self.closed:
            raise BrokerError("consumer closed")
        if timeout > 0:
            self.broker.wait_for_data(lambda: self.closed or self._has_data(), timeout)
        out: List[Record] = []
        with self.broker._cv:
            for tp in list(self._assignment):
                if len(out) >= max_records:
                    break
                pos = self._positions.get(tp, 0)
                recs = self.broker.fetch(tp[0], tp[1], pos, max_records - len(out))
                if recs:
                    self._positions[tp] = recs[-1].offset + 1
                    out.extend(recs)
        if self.auto_commit and out:
            self.commit()
        return out

    def position(self, topic: str, partition: int) -> int:
        return self._positions.get((topic, partition), 0)

    def seek(self, topic: str, partition: int, offset: int) -> None:
        self._positions[(topic, partition)] = offset

    def commit(self, offsets: Optional[Dict[Tuple[str, int], int]] = None) -> None:
        offs = offsets if offsets is not None else dict(self._positions)
        for (t, p), o in offs.items():
            self.broker.commit(self.group, t, p, o)

    def close(self) -> None:
        if not self.closed:
            self.closed = True
            self.broker._leave(self)
