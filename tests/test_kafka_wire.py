"""Kafka wire protocol: RecordBatch v2 codec (CRC-32C), client <-> kafka-lite server,
and the end-to-end pipeline running over real Kafka protocol sockets on 127.0.0.1."""
import numpy as np
import pytest

from ccfd_demo_summit_amd.config import load_config
from ccfd_demo_summit_amd.contracts import TxBatch
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.ingest import ProducerConfig, TransactionProducer
from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteServer
from ccfd_demo_summit_amd.ingest.kafka_wire import (KafkaBroker, _crc32c_py, crc32c, decode_record_batches,
                                                    encode_record_batch)
from ccfd_demo_summit_amd.models import build_model
from ccfd_demo_summit_amd.pipeline import FraudPipeline
from ccfd_demo_summit_amd.serving import CpuScorer


def test_crc32c_known_vectors():
    # RFC 3720 test vector: 32 bytes of zeros -> 0x8A9136AA ; "123456789" -> 0xE3069283
    assert crc32c(b"\x00" * 32) == 0x8A9136AA
    assert crc32c(b"123456789") == 0xE3069283
    assert _crc32c_py(b"123456789") == 0xE3069283
    blob = np.random.default_rng(0).bytes(100_003)
    assert crc32c(blob) == _crc32c_py(blob)


def test_record_batch_roundtrip():
    vals = [b"a", b"", b"x" * 1000, None]
    keys = [None, b"k", b"kk", b"z"]
    rb = encode_record_batch(vals, keys, base_offset=42, timestamp_ms=1_700_000_000_000)
    recs = decode_record_batches(rb + rb[:10], "t", 3)    # trailing partial batch is ignored
    assert [r.offset for r in recs] == [42, 43, 44, 45]
    assert [r.value for r in recs] == vals and [r.key for r in recs] == keys
    bad = bytearray(rb)
    bad[-1] ^= 1
    with pytest.raises(Exception):
        decode_record_batches(bytes(bad))


@pytest.fixture()
def lite():
    srv = KafkaLiteServer("127.0.0.1", 0, default_partitions=3).start_in_thread()
    yield srv
    srv.stop()


def test_client_against_kafka_lite(lite):
    kb = KafkaBroker(lite.bootstrap)
    assert kb.api_versions[0][1] >= 3
    kb.create_topic("odh-demo", 3)
    assert kb.partitions("odh-demo") == 3
    for i in range(30):
        kb.produce("odh-demo", f"m{i}".encode(), key=str(i).encode())
    tot = sum(kb.end_offset("odh-demo", p) for p in range(3))
    assert tot == 30
    c = kb.consumer("g", ["odh-demo"])
    got = c.poll(max_records=100)
    assert sorted(r.value for r in got) == sorted(f"m{i}".encode() for i in range(30))
    assert kb.lag("g", "odh-demo") == 30
    c.commit()
    assert kb.lag("g", "odh-demo") == 0
    assert kb.committed("g", "odh-demo", 0) == kb.end_offset("odh-demo", 0)
    # a new consumer in the same group resumes from the committed offsets
    kb.produce("odh-demo", b"late", partition=1)
    c2 = kb.consumer("g", ["odh-demo"], partitions=[("odh-demo", 1)])
    assert [r.value for r in c2.poll()] == [b"late"]
    # TXB1 binary batches survive the wire unchanged
    X, _ = generate(512, seed=1)
    b = TxBatch(ids=np.arange(512, dtype=np.uint64), customer=np.zeros(512, np.uint32), features=X)
    kb.produce("bin", b.encode(), partition=0)
    back = TxBatch.decode(kb.fetch("bin", 0, 0)[0].value)
    np.testing.assert_array_equal(back.features, X)
    kb.close()
    # broker series of the reference's Kafka dashboard (deploy/grafana/Kafka.json)
    text = lite.metrics.expose().decode()
    assert 'kafka_server_brokertopicmetrics_messagesin_total{strimzi_io_kind="Kafka",topic="odh-demo"} 31.0' in text
    assert "kafka_server_brokertopicmetrics_bytesout_total" in text
    assert 'kafka_server_replicamanager_partitioncount{strimzi_io_kind="Kafka"}' in text


def test_pipeline_over_kafka_protocol(lite):
    cfg = load_config(environ={}, overrides={"kafka.partitions": 3, "notifier.mean_delay_s": 0.0})
    kb = KafkaBroker(lite.bootstrap)
    X, _ = generate(2000, seed=3)
    model = build_model("lr", seed=1, X_ref=X, calibrate_rate=0.02)
    pipe = FraudPipeline(cfg, CpuScorer(model), broker=kb)
    TransactionProducer(kb, ProducerConfig(fmt="txb1", batch=500, seed=2)).produce(2000)
    for _ in range(20):
        pipe.step()
    assert pipe.metrics.router.tx_incoming._value.get() == 2000
    assert kb.lag(cfg.kafka.group_id, "odh-demo") == 0
    assert pipe.router.fraud_started == pipe.metrics.router.tx_outgoing.labels(type="fraud")._value.get() > 0
    kb.close()
