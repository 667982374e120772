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


def _elastic_proc(rank, world, store_port, bootstrap, model_seed):
    import datetime
    import time as _t
    import torch.distributed as dist
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    store = dist.TCPStore("127.0.0.1", store_port, world + 1, False, timeout=datetime.timedelta(seconds=60))
    X, _ = generate(8000, seed=2)
    model = build_model("mlp", seed=model_seed, X_ref=X, calibrate_rate=0.02)
    broker = KafkaBroker(bootstrap)
    router = Router(RuleSet.threshold(0.5), ProcessEngine(notification_timeout_s=1e9), RouterMetrics())
    w = ElasticWorker(rank, PartitionLeases(store, rank, world, 6, ttl_s=1.0), broker, "odh-demo",
                      CpuScorer(model), router, max_records=100)
    while not store.check(["stop"]):
        w.tick()
        store.set(f"alive/{rank}", str(w.scored_rows))
        _t.sleep(0.01)
    broker.close()


def test_sigkill_rank_over_tcpstore_and_kafka_protocol():
    """Real processes: 3 workers share a TCPStore (leases + committed counts) and a kafka-lite
    broker (Kafka wire protocol); rank 1 is SIGKILLed mid-stream.  Survivors adopt its
    partitions after the lease TTL and the committed global counts are exact."""
    import datetime
    import os
    import signal
    import socket
    import time as _t
    import torch.distributed as dist
    import torch.multiprocessing as mp
    from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteServer
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    store = dist.TCPStore("127.0.0.1", port, 4, True, timeout=datetime.timedelta(seconds=60), wait_for_workers=False)
    lite = KafkaLiteServer("127.0.0.1", 0, default_partitions=6).start_in_thread()
    kb = KafkaBroker(lite.bootstrap)
    kb.create_topic("odh-demo", 6)
    TransactionProducer(kb, ProducerConfig(fmt="json", batch=500, seed=3)).produce(6000)
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_elastic_proc, args=(r, 3, port, lite.bootstrap, 1)) for r in range(3)]
    for p in ps:
        p.start()
    try:
        reader = PartitionLeases(store, 99, 3, 6, ttl_s=1.0)
        t0 = _t.time()
        while _t.time() - t0 < 120:                      # wait until rank 1 is scoring
            if store.check(["alive/1"]) and int(store.get("alive/1")) > 0:
                break
            _t.sleep(0.05)
        os.kill(ps[1].pid, signal.SIGKILL)              # exact PID of our own child
        ps[1].join(10)
        rows = fraud = 0
        while _t.time() - t0 < 180:
            rows, fraud = reader.global_counts()
            if rows >= 6000:
                break
            _t.sleep(0.1)
        store.set("stop", "1")
        for p in (ps[0], ps[2]):
            p.join(30)
        recs = [r for p in range(6) for r in kb.fetch("odh-demo", p, 0, 100_000)]
        Xall, _, _ = decode_records([r.value for r in recs])
        X, _ = generate(8000, seed=2)
        model = build_model("mlp", seed=1, X_ref=X, calibrate_rate=0.02)
        assert rows == 6000
        assert fraud == int((model.predict_proba(Xall) >= 0.5).sum())
    finally:
        for p in ps:
            if p.is_alive():
                p.kill()
        kb.close()
        lite.stop()


def test_fault_plan_parse_and_determinism():
    import pytest
    from ccfd_demo_summit_amd.utils.faults import FaultPlan, InjectedCrash
    p = FaultPlan.parse("drop:p=0.5;delay:ms=0.1,p=1,rank=1;crash:after_steps=3,rank=0", rank=0, seed=4)
    assert [c.kind for c in p.clauses] == ["drop", "delay", "crash"]
    q = FaultPlan.parse("drop:p=0.5", rank=0, seed=4)
    assert [p.drop() for _ in range(50)] == [q.drop() for _ in range(50)]      # seeded
    p.step(); p.step()
    assert p.injected["delay"] == 0                                           # delay is rank 1's
    with pytest.raises(InjectedCrash):
        p.step()
    with pytest.raises(ValueError):
        FaultPlan.parse("explode:p=1")
    with pytest.raises(ValueError):
        FaultPlan.parse("drop:q=1")


def _elastic_cluster(n_workers, faults):
    X, _ = generate(8000, seed=2)
    model = build_model("mlp", seed=1, X_ref=X, calibrate_rate=0.02)
    broker = InProcBroker(default_partitions=6)
    broker.create_topic("odh-demo", 6)
    TransactionProducer(broker, ProducerConfig(fmt="json", batch=500, seed=3)).produce(6000)
    store, clock = MemoryStore(), Clock()
    procs = ProcessEngine(notification_timeout_s=1e9, clock=clock)
    workers = []
    for r in range(n_workers):
        router = Router(RuleSet.threshold(0.5), procs, RouterMetrics())
        workers.append(ElasticWorker(r, PartitionLeases(store, r, n_workers, 6, ttl_s=1.0, clock=clock), broker,
                                     "odh-demo", CpuScorer(model), router, max_records=300,
                                     faults=faults(r) if faults else None))
    return model, broker, procs, clock, workers


def _truth(model, broker):
    recs = [r for p in range(6) for r in broker.fetch("odh-demo", p, 0, 100_000)]
    Xall, _, _ = decode_records([r.value for r in recs])
    return int((model.predict_proba(Xall) >= 0.5).sum())


def test_injected_drops_are_redelivered_exactly_once():
    """drop faults on every rank: lost batches are re-fetched from the committed offset."""
    from ccfd_demo_summit_amd.utils.faults import FaultPlan
    model, broker, procs, clock, workers = _elastic_cluster(
        3, lambda r: FaultPlan.parse("drop:p=0.3", rank=r, seed=11))
    for _ in range(200):
        clock.t += 0.25
        for w in workers:
            w.tick()
    rows, fraud = workers[0].leases.global_counts()
    assert rows == 6000 and fraud == _truth(model, broker)
    assert sum(w.faults.injected["drop"] for w in workers) > 0
    assert len(procs._by_tx) == fraud and broker.lag("ccfd-engine", "odh-demo") == 0


def test_injected_crash_partitions_fail_over():
    """crash fault (mode=raise) on rank 1 after 3 steps: the survivors adopt its partitions."""
    from ccfd_demo_summit_amd.utils.faults import FaultPlan, InjectedCrash
    model, broker, procs, clock, workers = _elastic_cluster(
        3, lambda r: FaultPlan.parse("crash:after_steps=3,rank=1", rank=r))
    crashed = []
    for _ in range(200):
        clock.t += 0.25
        for w in workers:
            try:
                w.tick()
            except InjectedCrash:
                w.alive = False
                crashed.append(w.rank)
    assert crashed == [1]
    rows, fraud = workers[0].leases.global_counts()
    assert rows == 6000 and fraud == _truth(model, broker)
    owned = sorted(p for w in workers if w.alive for p in w.leases.owned())
    assert owned == list(range(6))
