"""Config-5 path on one GPU: broker -> ingest thread -> pinned rings -> fused kernels ->
router -> fraud processes, offsets committed after scoring, counters all-reduced."""
import time

import numpy as np
import pytest
import torch

from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import build_model

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("loop", ["native", "python-thread", "python-inline"])
def test_engine_service_end_to_end(gpu, loop):
    from ccfd_demo_summit_amd.ingest import InProcBroker, ProducerConfig, TransactionProducer
    from ccfd_demo_summit_amd.launch.engine_service import EngineService, EngineServiceConfig
    from ccfd_demo_summit_amd.metrics import MetricsHub
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    from ccfd_demo_summit_amd.parallel import DistContext
    from ccfd_demo_summit_amd.process import ProcessEngine
    from ccfd_demo_summit_amd.router import Router, RuleSet

    X, _ = generate(50_000, seed=1)
    m = build_model("mlp", seed=3, X_ref=X, calibrate_rate=0.01)
    broker = InProcBroker(default_partitions=2)
    broker.create_topic("odh-demo", 2)
    TransactionProducer(broker, ProducerConfig(fmt="txb1", batch=3000, seed=5)).produce(30_000)
    TransactionProducer(broker, ProducerConfig(fmt="json", batch=500, seed=6)).produce(2_000)
    hub = MetricsHub()
    procs = ProcessEngine(notification_timeout_s=60)
    router = Router(RuleSet.threshold(0.5), procs, hub.router)
    ctx = DistContext(0, 1, 0, gpu, "none")
    svc = EngineService(ctx, DeviceModel(m, gpu), broker, router,
                        EngineServiceConfig(batch=4096, depth=4, streams=2, ring_rows=16384, flush_us=200,
                                            reduce_period_ms=1.0, score_thread=loop == "python-thread",
                                            native_serve=loop == "native")).start()
    total = 32_000
    t0 = time.time()
    while svc.rows_scored < total and time.time() - t0 < 60:
        svc.step()
    for _ in range(5):
        svc.step()
    svc.reducer.wait()
    assert svc.rows_scored == total
    assert broker.lag("ccfd-engine", "odh-demo") == 0
    assert hub.router.tx_incoming._value.get() == total
    nf = hub.router.tx_outgoing.labels(type="fraud")._value.get()
    assert router.fraud_started == nf == procs.active_count()
    svc.flush_epochs()           # reduce the pending and the open epoch (on the scoring thread)
    c, lat = svc.reducer.snapshot()
    assert c[0] == total and c[1] == nf
    assert lat.sum() > 0
    svc.stop()


def test_engine_service_native_kafka_ingest_and_hot_swap(gpu, tmp_path):
    """kafka-lite (Kafka wire protocol) -> native C++ consumer -> W64 rings -> GPU, and a
    runtime hot swap triggered by rewriting the watched safetensors file mid-stream."""
    from ccfd_demo_summit_amd.ingest import ProducerConfig, TransactionProducer
    from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteServer
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    from ccfd_demo_summit_amd.launch.engine_service import EngineService, EngineServiceConfig
    from ccfd_demo_summit_amd.metrics import MetricsHub
    from ccfd_demo_summit_amd.models import save_model
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    from ccfd_demo_summit_amd.parallel import DistContext
    from ccfd_demo_summit_amd.process import ProcessEngine
    from ccfd_demo_summit_amd.router import Router, RuleSet

    X, _ = generate(50_000, seed=1)
    m1 = build_model("mlp", seed=3, X_ref=X, calibrate_rate=0.01)
    m2 = build_model("mlp", seed=4, X_ref=X, calibrate_rate=0.05)
    path = str(tmp_path / "model.safetensors")
    save_model(m1, path)
    lite = KafkaLiteServer("127.0.0.1", 0, default_partitions=2).start_in_thread()
    kb = KafkaBroker(lite.bootstrap)
    kb.create_topic("odh-demo", 2)
    TransactionProducer(kb, ProducerConfig(fmt="txb1", batch=4000, seed=5)).produce(24_000)
    hub = MetricsHub()
    procs = ProcessEngine(notification_timeout_s=60)
    router = Router(RuleSet.threshold(0.5), procs, hub.router)
    ctx = DistContext(0, 1, 0, gpu, "none")
    svc = EngineService(ctx, DeviceModel(m1, gpu, wire=True), kb, router,
                        EngineServiceConfig(batch=4096, depth=8, streams=2, ring_rows=1 << 16, flush_us=200,
                                            reduce_period_ms=1.0, model_watch=path)).start()
    try:
        assert svc.native is not None
        t0 = time.time()
        while svc.rows_scored < 24_000 and time.time() - t0 < 60:
            svc.step()
        assert svc.rows_scored == 24_000
        import os
        save_model(m2, path)
        os.utime(path, (time.time() + 10, time.time() + 10))
        t0 = time.time()
        while svc.hotswap.version < 1 and time.time() - t0 < 30:
            svc.step()
        assert svc.hotswap.version == 1 and svc.engine.model_version == 1
        TransactionProducer(kb, ProducerConfig(fmt="txb1", batch=4000, seed=9)).produce(8_000)
        t0 = time.time()
        while svc.rows_scored < 32_000 and time.time() - t0 < 60:
            svc.step()
        assert svc.rows_scored == 32_000
        for _ in range(20):
            svc.step()
        assert kb.lag("ccfd-engine", "odh-demo") == 0          # offsets committed after scoring
        svc.flush_epochs()
        c, _ = svc.reducer.snapshot()
        assert c[0] == 32_000
        assert svc.native.stats()["errors"] == 0
    finally:
        svc.stop()
        kb.close()
        lite.stop()


def test_persistent_engine_service_kafka_kie_outage_exactly_once(gpu):
    """The deployed path: EngineService in exec_mode persistent (the
    bench's mode, now the default for zero-copy) fed by the native Kafka consumer from
    kafka-lite (TXB1 batches + one JSON transaction per message), fraud rows handed to a KIE
    server over HTTP through the async hand-off -- and KIE goes away for 5 s mid-stream
    (2.5 s connection refused, 2.5 s of 503s).  No exception leaves step(); offsets are held
    while hand-offs are unacknowledged; afterwards every row is scored once, the committed
    lag is 0, and every fraud-routed transaction is started exactly once.  The model's
    last-request gauges and Seldon histograms come from the same streamed traffic."""
    from ccfd_demo_summit_amd.contracts import TxBatch
    from ccfd_demo_summit_amd.contracts.transaction import Transaction, encode_tx_json
    from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteServer
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    from ccfd_demo_summit_amd.launch.engine_service import EngineService, EngineServiceConfig
    from ccfd_demo_summit_amd.metrics import MetricsHub
    from ccfd_demo_summit_amd.metrics.exporter import EngineModelCollector
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    from ccfd_demo_summit_amd.parallel import DistContext
    from ccfd_demo_summit_amd.process import ProcessEngine
    from ccfd_demo_summit_amd.process.kie_server import KieClient
    from ccfd_demo_summit_amd.router import Router, RuleSet
    from ccfd_demo_summit_amd.router.handoff import KieHandoff
    from prometheus_client import CollectorRegistry, generate_latest
    from tests.helpers.faulty_proxy import FaultyProxy
    from tests.helpers.kie_thread import KieThread

    n_txb, n_json = 24_000, 12_000
    X, _ = generate(n_txb + n_json, seed=11)
    ids = np.arange(1, n_txb + n_json + 1, dtype=np.uint64) + np.uint64(7 << 32)
    m = build_model("mlp", seed=3, X_ref=X, calibrate_rate=0.02)
    lite = KafkaLiteServer("127.0.0.1", 0, default_partitions=2).start_in_thread()
    kb = KafkaBroker(lite.bootstrap)
    kb.create_topic("odh-demo", 2)
    procs = ProcessEngine(notification_timeout_s=1e9)
    kie = KieThread(procs)
    px = FaultyProxy(kie.port)
    client = KieClient(px.url, timeout_s=1.0, pool_size=4)
    ho = KieHandoff(client, workers=2, backoff_s=0.02, max_backoff_s=0.3)
    hub = MetricsHub()
    router = Router(RuleSet.threshold(0.5), client, hub.router, handoff=ho)
    ctx = DistContext(0, 1, 0, gpu, "none")
    dm = DeviceModel(m, gpu, wire=True)
    svc = EngineService(ctx, dm, kb, router,
                        EngineServiceConfig(batch=4096, depth=8, streams=2, ring_rows=1 << 16, flush_us=200,
                                            reduce_period_ms=1.0)).start()
    try:
        assert svc.exec_mode == "persistent" and svc.native is not None
        for k in range(0, n_txb, 2000):                      # TXB1 micro-batches, both partitions
            kb.produce("odh-demo", TxBatch(ids=ids[k:k + 2000], customer=(ids[k:k + 2000] % 999).astype(np.uint32),
                                           features=X[k:k + 2000]).encode(), partition=(k // 2000) % 2)
        t0 = time.time()
        while svc.rows_scored < n_txb and time.time() - t0 < 60:
            svc.step()
        assert svc.rows_scored == n_txb
        # KIE outage, while JSON transactions (the reference's wire format) keep arriving
        px.set_mode("refuse")
        msgs = [encode_tx_json(Transaction(int(ids[i]), int(ids[i] % 999), X[i])) for i in range(n_txb, n_txb + n_json)]
        for p in range(2):
            kb.produce_many("odh-demo", msgs[p::2], partition=p)
        t_out = time.time()
        held_seen = False
        while time.time() - t_out < 5.0:
            if time.time() - t_out > 2.5 and px.mode != "503":
                px.set_mode("503")
            svc.step()                                        # must never raise
            held_seen |= svc.commits_pending() > 0 and kb.lag("ccfd-engine", "odh-demo") > 0
        assert svc.rows_scored == n_txb + n_json
        assert held_seen, "offsets were committed past unacknowledged fraud hand-offs"
        assert ho.stats()["retries"] > 0
        px.set_mode("pass")
        t0 = time.time()
        while (ho.depth() or svc.commits_pending() or kb.lag("ccfd-engine", "odh-demo")) and time.time() - t0 < 60:
            svc.step()
        assert kb.lag("ccfd-engine", "odh-demo") == 0 and ho.depth() == 0
        nf = int(hub.router.tx_outgoing.labels(type="fraud")._value.get())
        started = sorted(int(i.variables["transaction_id"]) for i in procs.instances.values())
        assert len(started) == len(set(started)) == nf == router.fraud_started > 0
        # routes: the device's fraud set vs the fp32 oracle -- any difference only inside the
        # bf16 rounding band around the threshold
        p32 = m.predict_proba(X)
        want = set(ids[p32 >= 0.5].tolist())
        diff = want.symmetric_difference(started)
        band = {int(ids[i]) for i in np.nonzero(np.abs(p32 - 0.5) < 0.01)[0]}
        assert diff <= band, sorted(diff - band)[:5]
        # the model / Seldon series of the streamed traffic (ModelPrediction / SeldonCore boards)
        ms = svc.model_source()
        assert ms["last"] is not None and int(ms["lat_rows"].sum()) == n_txb + n_json
        assert ms["malformed"] == 0 and ms["refused"] == 0
        assert int(ms["last"].tx_id) in set(ids.tolist())
        reg = CollectorRegistry()
        reg.register(EngineModelCollector(svc.model_source))
        text = generate_latest(reg).decode()
        for name in ("proba_1 ", "Amount ", "V17 ", "V10 ",
                     'seldon_api_engine_server_requests_seconds_count{status="200"} %d.0' % (n_txb + n_json),
                     "seldon_api_engine_client_requests_seconds_bucket{"):
            assert name in text, name
    finally:
        svc.stop()
        ho.close(drain_s=1.0)
        px.close()
        kie.close()
        kb.close()
        lite.stop()


def test_engine_service_standard_mode_process_starts_every_row_once(gpu):
    """standard_mode="process" (README.md:549-552 "instantiate a standard or
    fraudulent transaction business process, depending on the value returned by Seldon"): the
    persistent W64 engine surfaces every scored row through the scored-record ring, the router
    hands standard rows to KIE as column batches next to the fraud starts, and afterwards
    standard + fraud starts == rows, 0 duplicates, each row's proba_1 (as KIE received it) is
    the fp32 oracle's within 1e-2, and the committed lag is 0."""
    from ccfd_demo_summit_amd.contracts import TxBatch
    from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteServer
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    from ccfd_demo_summit_amd.launch.engine_service import EngineService, EngineServiceConfig
    from ccfd_demo_summit_amd.metrics import MetricsHub
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    from ccfd_demo_summit_amd.parallel import DistContext
    from ccfd_demo_summit_amd.process import ProcessEngine
    from ccfd_demo_summit_amd.process.kie_server import KieClient
    from ccfd_demo_summit_amd.router import Router, RuleSet
    from ccfd_demo_summit_amd.router.handoff import KieHandoff
    from tests.helpers.kie_thread import KieThread

    seen = {}

    class Recording(ProcessEngine):
        def start_standard_array(self, items):     # KIE instances/batch, column bodies (round 5)
            for tx, p in zip(items["transaction_id"], items["proba"]):
                seen.setdefault(int(tx), []).append(("standard", float(p)))
            return super().start_standard_array(items)

        def start_fraud(self, v):
            seen.setdefault(int(v["transaction_id"]), []).append(("fraud", float(v["proba"])))
            return super().start_fraud(v)

        def start_fraud_many(self, items):          # KIE instances/batch (round 4)
            for v in (items if isinstance(items, list) else []):
                seen.setdefault(int(v["transaction_id"]), []).append(("fraud", float(v["proba"])))
            return super().start_fraud_many(items)

    n = 40_000
    X, _ = generate(n, seed=12)
    ids = np.arange(1, n + 1, dtype=np.uint64) + np.uint64(9 << 32)
    m = build_model("mlp", seed=5, X_ref=X, calibrate_rate=0.02)
    lite = KafkaLiteServer("127.0.0.1", 0, default_partitions=2).start_in_thread()
    kb = KafkaBroker(lite.bootstrap)
    kb.create_topic("odh-demo", 2)
    procs = Recording(notification_timeout_s=1e9)
    kie = KieThread(procs)
    client = KieClient(f"http://127.0.0.1:{kie.port}", timeout_s=5.0, pool_size=4)
    ho = KieHandoff(client, workers=2, max_batch=4096)
    hub = MetricsHub()
    router = Router(RuleSet.threshold(0.5), client, hub.router, standard_mode="process", handoff=ho)
    svc = EngineService(DistContext(0, 1, 0, gpu, "none"), DeviceModel(m, gpu, wire=True), kb, router,
                        EngineServiceConfig(batch=4096, depth=8, streams=2, ring_rows=1 << 16, flush_us=200,
                                            reduce_period_ms=2.0, standard_mode="process",
                                            scored_capacity=1 << 15)).start()
    try:
        assert svc.exec_mode == "persistent" and svc.native is not None
        for k in range(0, n, 2000):
            kb.produce("odh-demo", TxBatch(ids=ids[k:k + 2000], customer=(ids[k:k + 2000] % 999).astype(np.uint32),
                                           features=X[k:k + 2000]).encode(), partition=(k // 2000) % 2)
        t0 = time.time()
        while (svc.rows_scored < n or ho.depth() or svc.commits_pending()
               or kb.lag("ccfd-engine", "odh-demo")) and time.time() - t0 < 90:
            svc.step()
        assert svc.rows_scored == n and kb.lag("ccfd-engine", "odh-demo") == 0 and ho.depth() == 0
        nf = int(hub.router.tx_outgoing.labels(type="fraud")._value.get())
        assert procs.standard_count + len(procs._by_tx) == n
        assert procs.standard_count == n - nf and router.standard_started == n - nf
        assert procs.duplicates == 0 and procs.standard_duplicates == 0
        assert sorted(seen) == ids.astype(np.int64).tolist() and all(len(v) == 1 for v in seen.values())
        p32 = m.predict_proba(X)
        got = np.array([seen[int(t)][0][1] for t in ids])
        assert np.abs(got - p32).max() < 1e-2
        kinds = np.array([seen[int(t)][0][0] == "fraud" for t in ids])
        far = np.abs(p32 - 0.5) > 1e-2
        np.testing.assert_array_equal(kinds[far], (p32 >= 0.5)[far])
    finally:
        svc.stop()
        ho.close()
        kie.close()
        kb.close()
        lite.stop()


def test_process_mode_sharded_kie_back_pressure_holds_and_resumes(gpu):
    """Round 5: process mode over a 2-shard KIE tier whose shard 1 refuses
    connections for 3 s, with a hand-off capacity small enough that the engine HOLDS (the
    native serving thread pauses, the scored ring and the ingest rings back up) and resumes
    several times.  Afterwards every row started exactly one process on the shard its id hashes
    to, the committed lag is 0, and nothing was lost or repeated."""
    from ccfd_demo_summit_amd.contracts import TxBatch
    from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteServer
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    from ccfd_demo_summit_amd.launch.engine_service import EngineService, EngineServiceConfig
    from ccfd_demo_summit_amd.metrics import MetricsHub
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    from ccfd_demo_summit_amd.parallel import DistContext
    from ccfd_demo_summit_amd.process import ProcessEngine
    from ccfd_demo_summit_amd.process.kie_server import KieClient
    from ccfd_demo_summit_amd.process.sharding import ShardedKieClient, shard_of_tx
    from ccfd_demo_summit_amd.router import Router, RuleSet
    from ccfd_demo_summit_amd.router.handoff import ShardedHandoff
    from tests.helpers.faulty_proxy import FaultyProxy
    from tests.helpers.kie_thread import KieThread

    n = 80_000
    X, _ = generate(n, seed=21)
    ids = np.arange(1, n + 1, dtype=np.uint64) + np.uint64(11 << 36)
    m = build_model("mlp", seed=4, X_ref=X, calibrate_rate=0.01)
    lite = KafkaLiteServer("127.0.0.1", 0, default_partitions=2).start_in_thread()
    kb = KafkaBroker(lite.bootstrap)
    kb.create_topic("odh-demo", 2)
    engines = [ProcessEngine(notification_timeout_s=1e9, shard=k, shards=2) for k in range(2)]
    kies = [KieThread(e) for e in engines]
    px = FaultyProxy(kies[1].port)
    clients = [KieClient(f"http://127.0.0.1:{kies[0].port}", timeout_s=2.0), KieClient(px.url, timeout_s=1.0)]
    ho = ShardedHandoff(clients, capacity=6000, workers=2, backoff_s=0.02, max_backoff_s=0.2)
    hub = MetricsHub()
    router = Router(RuleSet.threshold(0.5), ShardedKieClient(clients), hub.router, standard_mode="process",
                    handoff=ho)
    svc = EngineService(DistContext(0, 1, 0, gpu, "none"), DeviceModel(m, gpu, wire=True), kb, router,
                        EngineServiceConfig(batch=4096, depth=8, streams=2, ring_rows=1 << 15, flush_us=200,
                                            reduce_period_ms=2.0, standard_mode="process",
                                            scored_capacity=1 << 14)).start()
    try:
        assert svc.exec_mode == "persistent" and svc.native is not None
        px.set_mode("refuse")
        held_rows = []
        for k in range(0, n, 2000):                           # arriving in waves while shard 1 is away
            kb.produce("odh-demo", TxBatch(ids=ids[k:k + 2000], customer=(ids[k:k + 2000] % 999).astype(np.uint32),
                                           features=X[k:k + 2000]).encode(), partition=(k // 2000) % 2)
            t0 = time.time()
            while time.time() - t0 < 0.075:
                svc.step()                                    # never raises
                if svc.held:
                    held_rows.append(svc.rows_scored)
        assert svc.hold_events >= 1 and held_rows
        assert held_rows[-1] < n                              # scoring paused while held
        px.set_mode("pass")
        t0 = time.time()
        while (svc.rows_scored < n or ho.depth() or svc.commits_pending()
               or kb.lag("ccfd-engine", "odh-demo")) and time.time() - t0 < 90:
            svc.step()
        assert svc.rows_scored == n and kb.lag("ccfd-engine", "odh-demo") == 0 and ho.depth() == 0
        tx = ids.astype(np.int64)
        for k, e in enumerate(engines):
            assert e.standard_count + e.fraud_count == int((shard_of_tx(tx, 2) == k).sum())
            assert e.duplicates == 0 and e.standard_duplicates == 0
        nf = int(hub.router.tx_outgoing.labels(type="fraud")._value.get())
        assert sum(e.fraud_count for e in engines) == nf
    finally:
        svc.stop()
        ho.close(drain_s=1.0)
        px.close()
        for k_ in kies:
            k_.close()
        kb.close()
        lite.stop()
