"""Fault injection: kill a rank mid-stream; its partitions are re-assigned
after the lease ttl, and the final counts are correct with no double count."""
import numpy as np

from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.ingest import InProcBroker, ProducerConfig, TransactionProducer, decode_records
from ccfd_demo_summit_amd.launch.elastic_worker import ElasticWorker
from ccfd_demo_summit_amd.metrics import RouterMetrics
from ccfd_demo_summit_amd.models import build_model
from ccfd_demo_summit_amd.parallel.elastic import MemoryStore, PartitionLeases
from ccfd_demo_summit_amd.process import ProcessEngine
from ccfd_demo_summit_amd.router import Router, RuleSet
from ccfd_demo_summit_amd.serving import CpuScorer


class Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def test_leases_home_then_failover():
    store, clock = MemoryStore(), Clock()
    a = PartitionLeases(store, 0, 2, 4, ttl_s=1.0, clock=clock)
    b = PartitionLeases(store, 1, 2, 4, ttl_s=1.0, clock=clock)
    assert a.tick()[0] == [0, 2] and b.tick()[0] == [1, 3]
    clock.t += 0.5
    a.tick(); b.tick()
    assert a.owned() == [0, 2] and b.owned() == [1, 3]
    # b dies (stops renewing); a adopts only after expiry + ttl
    clock.t += 1.2
    a.tick()
    assert a.owned() == [0, 2]
    clock.t += 1.0
    gained, _ = a.tick()
    assert gained == [1, 3] and a.owned() == [0, 1, 2, 3]
    # b comes back: its renewals fail, it has lost the partitions
    _, lost = b.tick()
    assert lost == [1, 3] and b.owned() == []
    assert a.commit(1, 10, 5, 1) and not b.commit(1, 11, 6, 1)
    assert a.committed(1) == (10, 5, 1)


def test_kill_rank_mid_stream_exact_counts():
    X, _ = generate(8000, seed=2)
    model = build_model("mlp", seed=1, X_ref=X, calibrate_rate=0.02)
    broker = InProcBroker(default_partitions=6)
    broker.create_topic("odh-demo", 6)
    TransactionProducer(broker, ProducerConfig(fmt="json", batch=500, seed=3)).produce(6000)
    store, clock = MemoryStore(), Clock()
    procs = ProcessEngine(notification_timeout_s=1e9, clock=clock)     # shared KIE
    workers = []
    for r in range(3):
        router = Router(RuleSet.threshold(0.5), procs, RouterMetrics())
        workers.append(ElasticWorker(r, PartitionLeases(store, r, 3, 6, ttl_s=1.0, clock=clock), broker,
                                     "odh-demo", CpuScorer(model), router, max_records=300))
    for w in workers:
        w.tick()
    # rank 1 scores a batch and dies before committing it
    workers[1].tick(crash_before_commit=True)
    for _ in range(200):
        clock.t += 0.25
        for w in workers:
            w.tick()
    recs = [r for p in range(6) for r in broker.fetch("odh-demo", p, 0, 100_000)]
    Xall, ids, _ = decode_records([r.value for r in recs])
    truth_fraud = int((model.predict_proba(Xall) >= 0.5).sum())
    rows, fraud = workers[0].leases.global_counts()
    assert rows == 6000                                     # exactly once, despite the re-score
    assert fraud == truth_fraud
    assert sum(w.scored_rows for w in workers) > 6000       # the dead rank's batch was re-scored
    # no double-started fraud process: one instance per fraud-routed transaction
    assert len(procs._by_tx) == truth_fraud
    assert broker.lag("ccfd-engine", "odh-demo") == 0
    owned = sorted(p for w in workers if w.alive for p in w.leases.owned())
    assert owned == list(range(6))
