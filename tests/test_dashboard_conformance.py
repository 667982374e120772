"""The reference's six Grafana dashboards work unchanged against this stack (SURVEY.md §5;
VERDICT r2 next #3): every vector selector of every ``expr`` in the reference's
deploy/grafana/*.json (tests/fixtures/reference_dashboard_exprs.json, or the reference
checkout itself when present) matches at least one series scraped over HTTP from running
exporters -- kafka-lite, KIE, the router, the engine's model endpoint and the trainer --
with the target labels Prometheus adds (instance, job; operator/render.py scrape jobs)."""
import json
import os
import time
from pathlib import Path

import numpy as np
import pytest

from ccfd_demo_summit_amd.metrics import promql
from tests.helpers.expose_http import serve

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference/deploy/grafana")


def reference_exprs():
    if REF.is_dir() and list(REF.glob("*.json")):
        return {p.name: promql.dashboard_exprs(json.loads(p.read_text())) for p in sorted(REF.glob("*.json"))}
    doc = json.loads((ROOT / "tests/fixtures/reference_dashboard_exprs.json").read_text())
    return {k: [e["expr"] for e in v] for k, v in doc["dashboards"].items()}


def test_fixture_matches_reference_when_present():
    if not REF.is_dir():
        pytest.skip("reference checkout not present")
    doc = json.loads((ROOT / "tests/fixtures/reference_dashboard_exprs.json").read_text())
    assert {k: [e["expr"] for e in v] for k, v in doc["dashboards"].items()} == reference_exprs()
    assert sum(len(v) for v in doc["dashboards"].values()) == 45


def test_selector_parser():
    s = promql.selectors('sum without(instance)(rate(kafka_server_brokertopicmetrics_bytesin_total'
                         '{strimzi_io_kind="Kafka",topic!="",topic!="__consumer_offsets"}[5m]))')
    assert [str(x) for x in s] == ['kafka_server_brokertopicmetrics_bytesin_total{strimzi_io_kind="Kafka",'
                                   'topic!="",topic!="__consumer_offsets"}']
    s = promql.selectors('histogram_quantile(0.5, sum(rate(seldon_api_engine_client_requests_seconds_bucket'
                         '{status="200"}[2m])) by (deployment_name,status,le))')
    assert [x.name for x in s] == ["seldon_api_engine_client_requests_seconds_bucket"]
    s = promql.selectors('sum(rate(x_count{model_name=~"$model_name"}[2m])) by (model_name)')
    assert s[0].matchers == [("model_name", "=~", ".*")]
    series = [("x_count", {"model_name": "m"}), ("y", {"a": "1"})]
    assert promql.matches(s[0], series) == 1
    assert promql.matches(promql.selectors('y{a!~"1"}')[0], series) == 0


def _engine_model_source():
    """The engine's model endpoint inputs (launch/engine_service.py model_source) for a
    scored W64 row; the GPU tests drive the real engine (test_engine_service_gpu.py)."""
    from ccfd_demo_summit_amd.contracts.transaction import encode_wire
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.engine.stream_engine import LastScored
    X, _ = generate(4, seed=1)
    row = encode_wire(X[-1:])[0].tobytes()
    lat = np.zeros(256, np.int64)
    lat[int(4 * np.log2(50_000))] = 4096          # 4096 rows at ~50 us
    dev = np.zeros(256, np.int64)
    dev[int(4 * np.log2(36_000))] = 4096
    return lambda: {"last": LastScored(7, 0.12, float(X[-1, 29]), 0, row, "w64"), "lat_rows": lat,
                    "dev_rows": dev, "malformed": 0, "refused": 0}


def test_reference_dashboards_match_scraped_series():
    from prometheus_client import CollectorRegistry, generate_latest

    from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteServer
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    from ccfd_demo_summit_amd.metrics import KieMetrics
    from ccfd_demo_summit_amd.metrics.exporter import EngineModelCollector, RouterMetrics, TrainMetrics
    from ccfd_demo_summit_amd.process import PredictionService, ProcessEngine
    from ccfd_demo_summit_amd.process.kie_server import KieClient
    from ccfd_demo_summit_amd.router import Router, RuleSet
    from tests.helpers.kie_thread import KieThread

    servers = []
    series = []
    # Kafka: kafka-lite with traffic on the transaction topic (Strimzi pod labels in-series)
    lite = KafkaLiteServer("127.0.0.1", 0, default_partitions=2).start_in_thread()
    kb = KafkaBroker(lite.bootstrap)
    kb.create_topic("odh-demo", 2)
    kb.produce_many("odh-demo", [b'{"id": %d}' % i for i in range(50)], partition=0)
    kb.fetch("odh-demo", 0, 0, 10)
    srv, url = serve(lite.metrics.expose)
    servers.append(srv)
    series += promql.scrape(url, "kafka")
    # KIE: the fraud process over HTTP, timers and signals driving every amount histogram
    procs = ProcessEngine(notification_timeout_s=0.05, kie_metrics=KieMetrics(), prediction=PredictionService(1.0))
    kie = KieThread(procs)
    kc = KieClient(f"http://127.0.0.1:{kie.port}")
    router_metrics = RouterMetrics()
    router = Router(RuleSet.threshold(0.5), kc, router_metrics)
    ids = [kc.start_fraud({"transaction_id": i, "customer_id": i, "amount": a, "proba": p})
           for i, (a, p) in enumerate([(10.0, 0.6), (5000.0, 0.9), (20.0, 0.6), (30.0, 0.7)])]
    router.on_notification_sent({})
    router.on_response(json.dumps({"process_id": ids[2], "response": True}))
    router.on_response(json.dumps({"process_id": ids[3], "response": False}))
    time.sleep(0.4)                                  # timers: low-amount approve + investigation
    series += promql.scrape(f"http://127.0.0.1:{kie.port}/rest/metrics", "kie")
    # router (:8091/prometheus in a deployment)
    srv, url = serve(router_metrics.expose)
    servers.append(srv)
    series += promql.scrape(url, "router")
    # the engine's model endpoint; Prometheus' ccfd-model job addresses it as <pod>:8000
    reg = CollectorRegistry()
    reg.register(EngineModelCollector(_engine_model_source()))
    srv, url = serve(lambda: generate_latest(reg))
    servers.append(srv)
    series += promql.scrape(url, "ccfd-model", instance="10.0.0.7:8000")
    # trainer (the "Spark Metrics" scrape job), after a few CPU training steps
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.train.trainer import TrainConfig, train_logistic
    tm = TrainMetrics()
    tm.workers.set(2)
    X, y = generate(20_000, seed=3, fraud_rate=0.02)
    train_logistic(X, y, TrainConfig(epochs=1, batch=4096, device="cpu", metrics=tm))
    srv, url = serve(tm.expose)
    servers.append(srv)
    series += promql.scrape(url, "Spark Metrics")
    try:
        rep = promql.check(reference_exprs(), series)
        assert rep["unmatched"] == [], json.dumps(rep["unmatched"], indent=1)
        assert rep["selectors"] >= 45 and set(rep["by_source"]) == {
            "KIE.json", "Kafka.json", "ModelPrediction.json", "Router.json", "SeldonCore.json", "SparkMetrics.json"}
    finally:
        for s in servers:
            s.shutdown()
        kie.close()
        kb.close()
        lite.stop()


def test_rendered_prometheus_config_has_the_reference_jobs():
    """ModelPrediction.json selects instance=~".*:8000", SparkMetrics.json job="Spark Metrics":
    the rendered Prometheus config scrapes the engine ranks' model ports and the trainer
    under those names (operator/render.py)."""
    import yaml
    from ccfd_demo_summit_amd.operator import load, render
    ms = render(load(str(ROOT / "deploy/cr/frauddetection-mi355x.yaml")))
    cm = [m for m in ms if m["kind"] == "ConfigMap" and m["metadata"]["name"] == "ccfd-prometheus"][0]
    jobs = {j["job_name"]: j for j in yaml.safe_load(cm["data"]["prometheus.yml"])["scrape_configs"]}
    assert {"ccfd-pods", "ccfd-model", "Spark Metrics"} <= set(jobs)
    eng = [m for m in ms if m["kind"] == "StatefulSet" and m["metadata"]["name"] == "ccfd-engine"][0]
    ports = {p["name"]: p["containerPort"] for p in eng["spec"]["template"]["spec"]["containers"][0]["ports"]}
    assert ports["model-0"] == 8000
