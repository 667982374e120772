"""Kafka consumer-group membership over the wire protocol (JoinGroup v1, SyncGroup v0,
Heartbeat v0, LeaveGroup v0, "consumer" protocol with the range assignor).

SURVEY.md §5 plans "Kafka consumer-group rebalance reassigns partitions" for failure
recovery: in the reference every service (router ``ccd-fuse``, KIE, notifier) is a Kafka
consumer in a group (deploy/router.yaml:55-62, deploy/notification-service.yaml:50-52), and
Kafka moves a dead pod's partitions to the survivors.  ``GroupConsumer`` is that client
side against any Kafka broker -- the production Strimzi cluster or ``kafka-lite``, whose
coordinator lives in ``KafkaLiteServer`` (ingest/kafka_lite.py).  It keeps the
``WireConsumer`` interface (poll / commit / assignment), heartbeats from ``poll``, and on a
rebalance commits what it has consumed, rejoins and resumes every newly assigned partition
from its committed offset (at-least-once, like the reference's Camel consumers).
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence, Tuple

from .broker import BrokerError, Record
from .kafka_wire import Connection, KafkaBroker, Reader, Writer

JOIN_GROUP, HEARTBEAT, LEAVE_GROUP, SYNC_GROUP = 11, 12, 13, 14
GROUP_APIS = {JOIN_GROUP: 1, HEARTBEAT: 0, LEAVE_GROUP: 0, SYNC_GROUP: 0}
ERR_ILLEGAL_GENERATION, ERR_UNKNOWN_MEMBER, ERR_REBALANCE_IN_PROGRESS = 22, 25, 27
ERR_COORDINATOR_NOT_AVAILABLE, ERR_NOT_COORDINATOR = 15, 16
PROTOCOL_TYPE, ASSIGNOR = "consumer", "range"


# --------------------------------------------------------------------------- consumer protocol
def encode_subscription(topics: Sequence[str], user_data: bytes = b"") -> bytes:
    return Writer().i16(0).array(list(topics), lambda w, t: w.string(t)).bytes_(user_data).build()


def decode_subscription(b: bytes) -> List[str]:
    r = Reader(b)
    r.i16()
    return r.array(lambda x: x.string()) or []


def encode_assignment(parts: Dict[str, List[int]]) -> bytes:
    return (Writer().i16(0).array(sorted(parts.items()),
                                  lambda w, kv: w.string(kv[0]).array(kv[1], lambda w2, p: w2.i32(p)))
            .bytes_(b"").build())


def decode_assignment(b: Optional[bytes]) -> List[Tuple[str, int]]:
    if not b:
        return []
    r = Reader(b)
    r.i16()
    out = []
    for t, ps in r.array(lambda x: (x.string(), x.array(lambda y: y.i32()))) or []:
        out += [(t, p) for p in ps]
    return out


def range_assign(members: Dict[str, List[str]], partitions: Dict[str, int]) -> Dict[str, Dict[str, List[int]]]:
    """Kafka's RangeAssignor: per topic, the sorted subscribers get contiguous ranges, the
    first ``n % k`` one partition more."""
    out: Dict[str, Dict[str, List[int]]] = {m: {} for m in members}
    for topic in sorted({t for ts in members.values() for t in ts}):
        subs = sorted(m for m, ts in members.items() if topic in ts)
        n, k = partitions.get(topic, 0), len(subs)
        start = 0
        for i, m in enumerate(subs):
            cnt = n // k + (1 if i < n % k else 0)
            if cnt:
                out[m][topic] = list(range(start, start + cnt))
            start += cnt
    return out


class GroupConsumer:
    """A member of consumer group ``group`` subscribed to ``topics``."""

    def __init__(self, broker: KafkaBroker, group: str, topics: Sequence[str], session_timeout_s: float = 10.0,
                 rebalance_timeout_s: float = 30.0, heartbeat_s: Optional[float] = None,
                 auto_commit: bool = False, client_id: str = "ccfd-mi355x"):
        self.broker = broker
        self.group = group
        self.topics = list(topics)
        self.session_ms = int(session_timeout_s * 1000)
        self.rebalance_ms = int(rebalance_timeout_s * 1000)
        self.heartbeat_s = heartbeat_s if heartbeat_s is not None else session_timeout_s / 3
        self.auto_commit = auto_commit
        host, port = self._coordinator()
        # JoinGroup is a long poll (the coordinator answers once every member has rejoined)
        self.conn = Connection(host, port, client_id, timeout=rebalance_timeout_s + 10.0)
        self.member_id = ""
        self.generation = -1
        self.leader = False
        self._assignment: List[Tuple[str, int]] = []
        self._positions: Dict[Tuple[str, int], int] = {}
        self._last_hb = 0.0
        self.rebalances = 0
        self.closed = False
        self.join()

    def _coordinator(self) -> Tuple[str, int]:
        r = self.broker._boot_request(10, 0, Writer().string(self.group).build())     # FindCoordinator v0
        err = r.i16()
        if err:
            raise BrokerError(f"FindCoordinator error {err}")
        r.i32()
        return r.string(), r.i32()

    # ------------------------------------------------------------------ membership
    def join(self) -> None:
        """JoinGroup -> (leader computes the range assignment) -> SyncGroup -> resume offsets."""
        while True:
            body = (Writer().string(self.group).i32(self.session_ms).i32(self.rebalance_ms).string(self.member_id)
                    .string(PROTOCOL_TYPE)
                    .array([(ASSIGNOR, encode_subscription(self.topics))], lambda w, p: w.string(p[0]).bytes_(p[1]))
                    .build())
            r = self.conn.request(JOIN_GROUP, 1, body)
            err = r.i16()
            gen, _proto, leader, me = r.i32(), r.string(), r.string(), r.string()
            members = r.array(lambda x: (x.string(), x.bytes_())) or []
            if err == ERR_UNKNOWN_MEMBER:
                self.member_id = ""
                continue
            if err:
                raise BrokerError(f"JoinGroup error {err}")
            self.member_id, self.generation, self.leader = me, gen, (leader == me)
            assignments: List[Tuple[str, bytes]] = []
            if self.leader:
                subs = {m: decode_subscription(meta) for m, meta in members}
                parts = {t: self.broker.partitions(t) for ts in subs.values() for t in ts}
                assignments = [(m, encode_assignment(a)) for m, a in range_assign(subs, parts).items()]
            body = (Writer().string(self.group).i32(gen).string(me)
                    .array(assignments, lambda w, a: w.string(a[0]).bytes_(a[1])).build())
            r = self.conn.request(SYNC_GROUP, 0, body)
            err = r.i16()
            if err in (ERR_REBALANCE_IN_PROGRESS, ERR_ILLEGAL_GENERATION):
                continue                                     # membership moved again: rejoin
            if err:
                raise BrokerError(f"SyncGroup error {err}")
            self._assignment = decode_assignment(r.bytes_())
            self._positions = {}
            for t, p in self._assignment:
                c = self.broker.committed(self.group, t, p)
                self._positions[(t, p)] = c if c is not None else self.broker.begin_offset(t, p)
            self._last_hb = time.monotonic()
            self.rebalances += 1
            return

    def heartbeat(self) -> bool:
        """True while the generation is stable; False after a rebalance (assignment may change)."""
        body = Writer().string(self.group).i32(self.generation).string(self.member_id).build()
        err = self.conn.request(HEARTBEAT, 0, body).i16()
        self._last_hb = time.monotonic()
        if err == 0:
            return True
        if err in (ERR_REBALANCE_IN_PROGRESS, ERR_ILLEGAL_GENERATION, ERR_UNKNOWN_MEMBER):
            if err == ERR_UNKNOWN_MEMBER:
                self.member_id = ""
            self.commit()                                     # hand over what we consumed
            self.join()
            return False
        raise BrokerError(f"Heartbeat error {err}")

    # ------------------------------------------------------------------ WireConsumer interface
    @property
    def assignment(self):
        return list(self._assignment)

    def poll(self, timeout: float = 0.0, max_records: int = 500) -> List[Record]:
        if time.monotonic() - self._last_hb >= self.heartbeat_s:
            self.heartbeat()
        out: List[Record] = []
        end = time.monotonic() + timeout
        while True:
            for tp in self._assignment:
                if len(out) >= max_records:
                    break
                recs = self.broker.fetch(tp[0], tp[1], self._positions[tp], max_records - len(out))
                if recs:
                    self._positions[tp] = recs[-1].offset + 1
                    out.extend(recs)
            if out or time.monotonic() >= end:
                break
            time.sleep(0.002)
            if time.monotonic() - self._last_hb >= self.heartbeat_s:
                self.heartbeat()
        if self.auto_commit and out:
            self.commit()
        return out

    def commit(self, offsets=None) -> None:
        for (t, p), o in (offsets or self._positions).items():
            self.broker.commit(self.group, t, p, o)

    def position(self, topic: str, partition: int) -> int:
        return self._positions[(topic, partition)]

    def seek(self, topic: str, partition: int, offset: int) -> None:
        self._positions[(topic, partition)] = offset

    def close(self, commit: bool = True) -> None:
        if self.closed:
            return
        if commit:
            self.commit()
        try:
            self.conn.request(LEAVE_GROUP, 0, Writer().string(self.group).string(self.member_id).build())
        except (OSError, BrokerError):
            pass
        self.conn.close()
        self.closed = True
