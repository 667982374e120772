"""Kafka consumer-group membership over the wire protocol against kafka-lite's coordinator:
range assignment, rebalance on join / leave / session expiry, at-least-once hand-over of a
dead member's partitions from the committed offsets."""
import time

from ccfd_demo_summit_amd.ingest.kafka_group import range_assign
from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteServer
from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker


def test_range_assignor_matches_kafka():
    a = range_assign({"m1": ["t"], "m2": ["t"], "m3": ["t"]}, {"t": 7})
    assert a == {"m1": {"t": [0, 1, 2]}, "m2": {"t": [3, 4]}, "m3": {"t": [5, 6]}}
    b = range_assign({"a": ["x", "y"], "b": ["y"]}, {"x": 2, "y": 3})
    assert b == {"a": {"x": [0, 1], "y": [0, 1]}, "b": {"y": [2]}}


def _drain(c, seen, rounds=40):
    for _ in range(rounds):
        for r in c.poll(timeout=0.01, max_records=1000):
            seen.append((r.partition, r.offset))
        c.commit()


def test_group_rebalance_join_leave_and_session_expiry():
    lite = KafkaLiteServer("127.0.0.1", 0, default_partitions=4).start_in_thread()
    kb = KafkaBroker(lite.bootstrap)
    kb.create_topic("odh-demo", 4)
    for p in range(4):
        kb.produce_batch("odh-demo", p, [b"x%d" % i for i in range(50)])
    try:
        a = kb.group_consumer("ccd-fuse", ["odh-demo"], session_timeout_s=1.0, rebalance_timeout_s=5.0)
        assert sorted(a.assignment) == [("odh-demo", p) for p in range(4)] and a.leader
        # a second member joins: the coordinator rebalances, A learns it on its next heartbeat
        import threading
        box = {}
        t = threading.Thread(target=lambda: box.setdefault(
            "b", KafkaBroker(lite.bootstrap).group_consumer("ccd-fuse", ["odh-demo"], session_timeout_s=1.0,
                                                           rebalance_timeout_s=5.0)))
        t.start()
        seen_a, seen_b = [], []
        t0 = time.time()
        while t.is_alive() and time.time() - t0 < 20:
            seen_a += [(r.partition, r.offset) for r in a.poll(timeout=0.05, max_records=1000)]
        t.join(1)
        b = box["b"]
        assert sorted(a.assignment + b.assignment) == [("odh-demo", p) for p in range(4)]
        assert len(a.assignment) == 2 and len(b.assignment) == 2 and a.generation == b.generation
        for p in range(4):
            kb.produce_batch("odh-demo", p, [b"y%d" % i for i in range(50)])
        # B consumes part of its partitions and commits
        for r in b.poll(timeout=0.1, max_records=30):
            seen_b.append((r.partition, r.offset))
        b.commit()
        # B dies silently (no LeaveGroup): after the session timeout A owns all 4 partitions and
        # resumes B's partitions from B's committed offsets -> every record consumed, none skipped
        b.conn.close()
        t0 = time.time()
        while len(a.assignment) != 4 and time.time() - t0 < 20:
            for r in a.poll(timeout=0.05, max_records=1000):
                seen_a.append((r.partition, r.offset))
            a.commit()
        assert len(a.assignment) == 4 and a.rebalances >= 3
        _drain(a, seen_a)
        got = set(seen_a) | set(seen_b)
        assert len(seen_b) == 30
        assert got == {(p, o) for p in range(4) for o in range(100)}
        assert not (set(seen_a) & set(seen_b))          # B committed what it read: no re-delivery
        # graceful leave: the coordinator empties the group
        a.close()
        assert lite.groups["ccd-fuse"].state == "Empty"
    finally:
        kb.close()
        lite.stop()
