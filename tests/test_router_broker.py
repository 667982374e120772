"""Broker semantics, routing rules and the end-to-end pipeline on CPU (SURVEY.md §4.1
"Integration (single process)": counters equal the CPU-computed truth)."""
import json

import numpy as np
import pytest

from ccfd_demo_summit_amd.config import load_config
from ccfd_demo_summit_amd.contracts import Route, TxBatch
from ccfd_demo_summit_amd.contracts.outcomes import Outcome
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.ingest import InProcBroker, ProducerConfig, TransactionProducer, decode_records
from ccfd_demo_summit_amd.models import build_model
from ccfd_demo_summit_amd.pipeline import FraudPipeline
from ccfd_demo_summit_amd.router import RuleError, RuleSet
from ccfd_demo_summit_amd.serving import CpuScorer


def test_broker_offsets_groups_rebalance():
    b = InProcBroker(default_partitions=4)
    for i in range(40):
        b.produce("t", str(i).encode(), key=str(i % 7).encode())
    c1 = b.consumer("g", ["t"], member_id="a")
    c2 = b.consumer("g", ["t"], member_id="b")
    assert sorted(c1.assignment + c2.assignment) == [("t", p) for p in range(4)]
    got = c1.poll(max_records=1000)
    c1.commit()
    c1.close()                                    # c2 takes over c1's partitions
    assert len(c2.assignment) == 4
    rest = c2.poll(max_records=1000)
    assert sorted(int(r.value) for r in got + rest) == list(range(40))
    assert b.lag("g", "t") == 40 - len(got)
    c2.commit()
    assert b.lag("g", "t") == 0
    # keyed records keep per-key order within a partition
    p0 = b.fetch("t", 0, 0, 100)
    assert [r.offset for r in p0] == list(range(len(p0)))


def test_broker_uncommitted_records_are_redelivered():
    b = InProcBroker(default_partitions=1)
    for i in range(5):
        b.produce("t", str(i).encode())
    c = b.consumer("g", ["t"])
    assert len(c.poll()) == 5                      # consumed but NOT committed (crash)
    c.close()
    c2 = b.consumer("g", ["t"])
    assert [int(r.value) for r in c2.poll()] == [0, 1, 2, 3, 4]


def test_rules_threshold_and_dsl():
    rs = RuleSet.threshold(0.5)
    assert rs.threshold_only == 0.5
    np.testing.assert_array_equal(rs.evaluate([0.1, 0.5, 0.9]), [0, 1, 1])
    rs2 = RuleSet.parse("""
        rule "big" when amount > 1000 and proba >= 0.2 then fraud
        when proba >= FRAUD_THRESHOLD then fraud   # default reference rule
        when 0.4 <= proba < 0.5 and not (V17 > -2) then fraud
        otherwise standard
    """, {"FRAUD_THRESHOLD": 0.5})
    assert rs2.threshold_only is None
    X = np.zeros((4, 30), np.float32)
    X[:, 29] = [5000, 10, 10, 10]
    X[:, 17] = [0, 0, -5, 0]
    np.testing.assert_array_equal(rs2.evaluate([0.3, 0.3, 0.45, 0.45], X=X), [1, 0, 1, 0])
    with pytest.raises(RuleError):
        RuleSet.parse("when __import__('os') then fraud")
    with pytest.raises(RuleError):
        RuleSet.parse("when unknown > 1 then fraud")
    with pytest.raises(RuleError):
        RuleSet.parse("this is not a rule")


def test_producer_and_codec_roundtrip():
    b = InProcBroker(default_partitions=2)
    p = TransactionProducer(b, ProducerConfig(fmt="json", batch=64))
    p.produce(128)
    p2 = TransactionProducer(b, ProducerConfig(fmt="txb1", batch=64, seed=1))
    p2.produce(128)
    recs = b.fetch("odh-demo", 0, 0, 10_000) + b.fetch("odh-demo", 1, 0, 10_000)
    X, ids, cust = decode_records([r.value for r in recs])
    assert X.shape == (256, 30)
    Xp, _, _ = decode_records([r.value for r in recs], native=False)
    np.testing.assert_allclose(X, Xp)


@pytest.mark.parametrize("fmt", ["json", "txb1"])
def test_end_to_end_pipeline_counters_match_cpu_truth(fmt):
    cfg = load_config(environ={}, overrides={"kafka.partitions": 3, "notifier.mean_delay_s": 0.0,
                                             "notifier.p_reply": 0.5, "kie.notification_timeout_s": 5.0})
    clock = [0.0]
    X, _ = generate(3000, seed=8)
    model = build_model("mlp", seed=1, X_ref=X, calibrate_rate=0.03)
    pipe = FraudPipeline(cfg, CpuScorer(model, 0.5), clock=lambda: clock[0], max_poll=500)
    prod = TransactionProducer(pipe.broker, ProducerConfig(fmt=fmt, batch=250, seed=4))
    prod.produce(3000)
    pipe.run_until_idle()
    # ground truth from the CPU model over exactly the produced rows
    recs = [r for p in range(3) for r in pipe.broker.fetch("odh-demo", p, 0, 100_000)]
    Xall, ids, _ = decode_records([r.value for r in recs])
    truth = int((model.predict_proba(Xall) >= 0.5).sum())
    rm = pipe.metrics.router
    assert rm.tx_incoming._value.get() == 3000
    assert rm.tx_outgoing.labels(type="fraud")._value.get() == truth
    assert rm.tx_outgoing.labels(type="standard")._value.get() == 3000 - truth
    assert rm.notif_outgoing._value.get() == truth
    replies = rm.notif_incoming.labels(response="approved")._value.get() + \
        rm.notif_incoming.labels(response="non_approved")._value.get()
    assert replies == pipe.notifier.replied
    # the rest of the fraud processes time out into DMN outcomes
    clock[0] = 100.0
    pipe.step()
    oc = pipe.processes.outcome_counts
    assert oc[Outcome.APPROVED_BY_CUSTOMER.value] + oc[Outcome.CANCELLED.value] == pipe.notifier.replied
    assert oc[Outcome.APPROVED_LOW_AMOUNT.value] + oc[Outcome.INVESTIGATION.value] == truth - pipe.notifier.replied
    assert pipe.processes.active_count() == oc[Outcome.INVESTIGATION.value]
    text = pipe.metrics.expose_all().decode()
    for name in ("transaction_incoming_total", "transaction_outgoing_total", "notifications_outgoing_total",
                 "notifications_incoming_total", "fraud_investigation_amount_bucket",
                 "fraud_approved_low_amount_sum", "fraud_approved_amount_count",
                 "fraud_rejected_amount_bucket", "proba_1", "V17", "V10", "Amount"):
        assert name in text, name
    pipe.close()


def test_router_batches_fraud_hand_off_when_supported():
    """Engine path: all fraud-routed rows of a step go to KIE in ONE call when the process
    sink offers start_fraud_many (KieClient's /instances/batch)."""
    import numpy as np
    from ccfd_demo_summit_amd.metrics import RouterMetrics
    from ccfd_demo_summit_amd.ops._lib import FLAGGED_DTYPE
    from ccfd_demo_summit_amd.router import Router, RuleSet

    class Sink:
        def __init__(self):
            self.calls = []

        def start_fraud_many(self, items):
            self.calls.append(items)
            return list(range(len(items)))

        def start_fraud(self, v):
            raise AssertionError("per-row start must not be used")

    sink = Sink()
    r = Router(RuleSet.threshold(0.5), sink, RouterMetrics())
    fl = np.zeros(3, dtype=np.dtype(FLAGGED_DTYPE))
    fl["tx_id"] = [7, 8, 9]
    fl["proba"] = 0.9
    res = r.on_flagged(fl, 1000)
    assert res == {"incoming": 1000, "fraud": 3, "standard": 997}
    assert len(sink.calls) == 1 and [c["transaction_id"] for c in sink.calls[0]] == [7, 8, 9]
    assert r.fraud_started == 3


def test_batching_publisher_delivers_everything_in_few_requests():
    """KIE notifications / notifier replies leave in batches (ingest/producer.py
    BatchingPublisher): everything published arrives, in far fewer produce calls."""
    from ccfd_demo_summit_amd.ingest import InProcBroker
    from ccfd_demo_summit_amd.ingest.producer import BatchingPublisher

    class Counting(InProcBroker):
        calls = 0

        def produce_many(self, topic, values, partition=None):
            Counting.calls += 1
            return super().produce_many(topic, values, partition=partition)
    b = Counting(default_partitions=3)
    b.create_topic("ccd-customer-outgoing", 3)
    pub = BatchingPublisher(b, "ccd-customer-outgoing", linger_s=0.005)
    for i in range(5000):
        pub.publish(b'{"n": %d}' % i)
    pub.close()
    got = sorted(int(r.value[6:-1]) for p in range(3) for r in b.fetch("ccd-customer-outgoing", p, 0, 10_000))
    assert got == list(range(5000)) and Counting.calls < 100
