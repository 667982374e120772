"""Native Kafka consumer (csrc/engine/kafka_consumer.cpp) against kafka-lite on 127.0.0.1:
TXB1 batches and JSON transactions land in the sink rows bit-exactly (f32, W64, G32 and G20),
offsets become committable once rows are consumed, CRC-corrupted batches are rejected."""
import json
import time

import numpy as np
import pytest

from ccfd_demo_summit_amd.contracts import FEATURE_NAMES, TxBatch, encode_wire
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteServer
from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
from ccfd_demo_summit_amd.ingest.native_consumer import NativeKafkaConsumer
from ccfd_demo_summit_amd.models import build_model


@pytest.fixture()
def lite():
    srv = KafkaLiteServer("127.0.0.1", 0, default_partitions=2).start_in_thread()
    yield srv
    srv.stop()


def _wait(kc, rows, timeout=20):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if kc.stats()["rows"] >= rows:
            return True
        time.sleep(0.01)
    return False


@pytest.mark.parametrize("fmt", ["f32", "w64", "g32", "g20"])
def test_txb1_and_json_into_rows(lite, fmt):
    kb = KafkaBroker(lite.bootstrap)
    kb.create_topic("odh-demo", 2)
    X, _ = generate(3000, seed=4)
    ids = np.arange(3000, dtype=np.uint64) + 10
    cu = (np.arange(3000) % 977).astype(np.uint32)
    # partition 0: three TXB1 batches; partition 1: 200 JSON messages
    for s in (0, 1000, 2000):
        kb.produce("odh-demo", TxBatch(ids=ids[s:s + 1000], customer=cu[s:s + 1000], features=X[s:s + 1000]).encode(),
                   partition=0)
    msgs = [json.dumps({"id": int(ids[i]), "customer_id": int(cu[i]),
                        **{n: float(v) for n, v in zip(FEATURE_NAMES, X[i])}}).encode() for i in range(200)]
    kb.produce_many("odh-demo", msgs, partition=1)
    bins = build_model("gbdt", seed=2, X_ref=X).bin_spec(bits=8 if fmt == "g32" else 5) if fmt[0] == "g" else None
    kc = NativeKafkaConsumer.for_arrays(lite.bootstrap, "odh-demo", {0: 0, 1: 0}, capacity=4000, wire=fmt == "w64",
                                        bins=bins).start()
    try:
        assert _wait(kc, 3200), (kc.stats(), kc.last_error())
        st = kc.stats()
        assert st["records"] == 203 and st["errors"] == 0
        f0, i0, c0 = kc.arrays[0]
        f1, i1, c1 = kc.arrays[1]
        want = {"f32": lambda: X, "w64": lambda: encode_wire(X).view(np.float32).reshape(-1, 16),
                "g32": lambda: bins.encode(X).view(np.float32).reshape(-1, 8),
                "g20": lambda: bins.encode(X).view(np.float32).reshape(-1, 5)}[fmt]()
        if fmt[0] == "g":            # G32 / G20 rows keep Amount host-side (flagged-record column)
            np.testing.assert_array_equal(kc.amounts[0][:3000], X[:, 29])
            np.testing.assert_array_equal(kc.amounts[1][:200], X[:200, 29])
        np.testing.assert_array_equal(f0[:3000], want)
        np.testing.assert_array_equal(i0[:3000], ids)
        np.testing.assert_array_equal(c0[:3000], cu)
        np.testing.assert_array_equal(f1[:200], want[:200])
        np.testing.assert_array_equal(i1[:200], ids[:200])
        assert kc.committable() == {0: 3, 1: 200}
        assert kc.committable() == {}                       # nothing new
    finally:
        kc.stop()
        kc.close()
        kb.close()


def test_large_json_batch_parsed_in_chunks_keeps_order(lite):
    """One produce request of 2500 JSON messages: the parse pool takes it 1024 records at a
    time (kafka_consumer.cpp kParChunk), each chunk written before the next is parsed -- every
    row lands once, in offset order, with its own values."""
    kb = KafkaBroker(lite.bootstrap)
    kb.create_topic("big", 1)
    n = 2500
    X, _ = generate(n, seed=9)
    ids = np.arange(n, dtype=np.uint64) + 1000
    cu = (np.arange(n) % 331).astype(np.uint32)
    msgs = [json.dumps({"id": int(ids[i]), "customer_id": int(cu[i]),
                        **{nm: float(v) for nm, v in zip(FEATURE_NAMES, X[i])}}).encode() for i in range(n)]
    kb.produce_many("big", msgs, partition=0)
    kc = NativeKafkaConsumer.for_arrays(lite.bootstrap, "big", {0: 0}, capacity=4096).start()
    try:
        assert _wait(kc, n), (kc.stats(), kc.last_error())
        st = kc.stats()
        assert st["records"] == n and st["errors"] == 0
        f0, i0, c0 = kc.arrays[0]
        np.testing.assert_array_equal(i0[:n], ids)
        np.testing.assert_array_equal(c0[:n], cu)
        np.testing.assert_array_equal(f0[:n], X)
        assert kc.committable() == {0: n}
    finally:
        kc.stop()
        kc.close()
        kb.close()


def test_resume_from_offset_and_late_data(lite):
    kb = KafkaBroker(lite.bootstrap)
    kb.create_topic("t", 1)
    X, _ = generate(50, seed=1)
    for i in range(50):
        kb.produce("t", json.dumps({"id": i, "features": X[i].tolist()}).encode(), partition=0)
    kc = NativeKafkaConsumer.for_arrays(lite.bootstrap, "t", {0: 20}, capacity=100).start()
    try:
        assert _wait(kc, 30)
        kb.produce("t", json.dumps({"id": 99, "features": X[0].tolist()}).encode(), partition=0)
        assert _wait(kc, 31)
        f, ids, _ = kc.arrays[0]
        assert ids[:31].tolist() == list(range(20, 50)) + [99]
        np.testing.assert_allclose(f[:30], X[20:50], rtol=1e-6)
    finally:
        kc.stop()
        kc.close()
        kb.close()
