"""kafka-lite as a 3-broker cluster (VERDICT r1 missing #1/#5): leadership spread over the
nodes, NOT_LEADER from a non-leader, the Python client routing by leader and recovering
from a leader move and from a broker failure, gzip batches, verbatim batch storage, and
the under-replicated / offline-partition series."""
import struct

import pytest

from ccfd_demo_summit_amd.ingest.batch_store import BatchStore, InvalidBatch
from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteCluster
from ccfd_demo_summit_amd.ingest.kafka_wire import (CODEC_GZIP, ERR_NOT_LEADER, FETCH, Connection, KafkaBroker,
                                                    Writer, decode_record_batches, encode_record_batch)


@pytest.fixture()
def cluster():
    cl = KafkaLiteCluster(3, default_partitions=6).start_in_thread()
    yield cl
    cl.stop()


def test_batches_are_stored_verbatim_and_offsets_stamped():
    st = BatchStore(default_partitions=1)
    st.create_topic("t")
    b1 = encode_record_batch([b"a", b"b", b"c"], base_offset=999)
    b2 = encode_record_batch([b"d"], compression=CODEC_GZIP)
    assert st.append_raw("t", 0, b1) == (0, 3)
    assert st.append_raw("t", 0, b2) == (3, 1)
    raw = st.fetch_raw("t", 0, 1, 1 << 20)
    # only the base offsets changed
    assert raw == struct.pack(">q", 0) + b1[8:] + struct.pack(">q", 3) + b2[8:]
    recs = decode_record_batches(raw)
    assert [(r.offset, r.value) for r in recs] == [(0, b"a"), (1, b"b"), (2, b"c"), (3, b"d")]
    assert [r.value for r in st.fetch("t", 0, 2)] == [b"c", b"d"]
    bad = bytearray(b1)
    bad[-1] ^= 0xFF
    with pytest.raises(InvalidBatch):
        st.append_raw("t", 0, bytes(bad))
    with pytest.raises(InvalidBatch):
        st.append_raw("t", 0, b1[:40])


def test_non_leader_answers_not_leader(cluster):
    kb = KafkaBroker(cluster.bootstrap)
    kb.create_topic("odh-demo", 6)
    leaders = {p: cluster.leader("odh-demo", p) for p in range(6)}
    assert sorted(set(leaders.values())) == [1, 2, 3]
    p = next(p for p, n in leaders.items() if n != 1)
    c = Connection(cluster.nodes[0].host, cluster.nodes[0].port)          # node 1
    body = (Writer().i32(-1).i32(0).i32(0).i32(1 << 20).i8(0)
            .array(["odh-demo"], lambda w, t: w.string(t).array([p], lambda w2, q: w2.i32(q).i64(0).i32(1 << 20)))
            .build())
    r = c.request(FETCH, 4, body)
    r.i32(); r.i32(); r.string(); r.i32(); r.i32()
    assert r.i16() == ERR_NOT_LEADER
    c.close()
    kb.close()


def test_client_routes_and_survives_leader_move_and_node_failure(cluster):
    kb = KafkaBroker(cluster.bootstrap_all)
    kb.create_topic("odh-demo", 6)
    sent = {p: [] for p in range(6)}
    for i in range(600):
        p = i % 6
        v = b"tx-%d" % i
        kb.produce_batch("odh-demo", p, [v])
        sent[p].append(v)
        if i == 200:
            cluster.move_leader("odh-demo", 0, 3 if cluster.leader("odh-demo", 0) != 3 else 2)
        if i == 400:
            cluster.fail_node(2)                 # node 2 dies; its partitions fail over
    assert kb.retries_done > 0
    gz = KafkaBroker(cluster.bootstrap_all, compression=CODEC_GZIP)
    gz.produce_batch("odh-demo", 5, [b"zipped-1", b"zipped-2"])
    sent[5] += [b"zipped-1", b"zipped-2"]
    got = {p: [r.value for r in kb.fetch("odh-demo", p, 0, 10_000)] for p in range(6)}
    assert got == sent
    text = cluster.metrics.expose().decode()
    assert 'kafka_server_replicamanager_underreplicatedpartitions{strimzi_io_kind="Kafka"} 6.0' in text
    assert 'kafka_controller_kafkacontroller_offlinepartitionscount{strimzi_io_kind="Kafka"} 0.0' in text
    assert 'kafka_controller_kafkacontroller_activebrokercount{strimzi_io_kind="Kafka"} 2.0' in text
    kb.commit("g", "odh-demo", 3, 42)
    assert kb.committed("g", "odh-demo", 3) == 42
    kb.close()
    gz.close()


def test_fetch_long_polls_until_data_or_max_wait(cluster):
    """Fetch with max_wait / min_bytes (what the native consumer sends): an empty partition
    holds the request until a produce lands on it (answered at once, with the data) or max_wait
    passes (answered empty); a fetch with data, or with min_bytes 0, answers at once."""
    import threading
    import time
    kb = KafkaBroker(cluster.bootstrap)
    kb.create_topic("lp", 6)
    node = cluster.leader("lp", 0)
    srv = cluster.nodes[node - 1]
    c = Connection(srv.host, srv.port)

    def fetch(offset, max_wait_ms, min_bytes=1):
        body = (Writer().i32(-1).i32(max_wait_ms).i32(min_bytes).i32(1 << 20).i8(0)
                .array(["lp"], lambda w, t: w.string(t).array([0], lambda w2, q: w2.i32(q).i64(offset).i32(1 << 20)))
                .build())
        t0 = time.perf_counter()
        r = c.request(FETCH, 4, body)
        dt = time.perf_counter() - t0
        r.i32(); r.i32(); r.string(); r.i32(); r.i32()
        err, _hw, _lso = r.i16(), r.i64(), r.i64()
        r.array(lambda x: (x.i64(), x.i64()))
        n = r.i32()
        return err, n, dt

    err, n, dt = fetch(0, 300)                           # nothing there: waits max_wait
    assert err == 0 and n == 0 and 0.25 < dt < 2.0, dt
    err, n, dt = fetch(0, 0, 0)                          # no long poll asked: at once
    assert n == 0 and dt < 0.2
    threading.Timer(0.15, lambda: kb.produce("lp", b"x", partition=0)).start()
    err, n, dt = fetch(0, 5000)                          # woken by the produce, with the data
    assert err == 0 and n > 0 and 0.1 < dt < 1.5, dt
    err, n, dt = fetch(0, 5000)                          # data already there: at once
    assert n > 0 and dt < 0.2
    assert srv.cluster.long_polls >= 2 and not srv.cluster.fetch_waiters
    c.close()
    kb.close()
