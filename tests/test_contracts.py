"""Contract tests: topic names, env defaults, metric names, codecs."""
import json

import numpy as np
import pytest

from ccfd_demo_summit_amd.config import load_config
from ccfd_demo_summit_amd.contracts import (DEFAULT_TOPICS, FEATURE_NAMES, N_FEATURES, Topics, TxBatch,
                                            Transaction, decode_tx_json, encode_tx_json, metric_names, seldon)
from ccfd_demo_summit_amd.contracts.env import REFERENCE_ENV


def test_topic_names_match_reference():
    assert DEFAULT_TOPICS.transactions == "odh-demo"                 # router.yaml:61-62
    assert DEFAULT_TOPICS.customer_outgoing == "ccd-customer-outgoing"  # router.yaml:57-58
    assert DEFAULT_TOPICS.customer_response == "ccd-customer-response"  # router.yaml:59-60
    t = Topics.from_env({"KAFKA_TOPIC": "x", "CUSTOMER_RESPONSE_TOPIC": "y"})
    assert t.transactions == "x" and t.customer_response == "y"
    assert t.customer_outgoing == "ccd-customer-outgoing"


def test_env_defaults_match_reference():
    c = load_config(environ={})
    assert c.kafka.broker_url == "odh-message-bus-kafka-brokers:9092"
    assert c.kie.url == "http://ccd-service:8090"
    assert c.seldon.url == "http://modelfull-modelfull:8000"
    assert c.seldon.endpoint == "api/v0.1/predictions"
    assert c.router.fraud_threshold == 0.5
    assert c.kie.confidence_threshold == 1.0
    assert c.kie.seldon_endpoint == "predict"
    assert REFERENCE_ENV["FRAUD_THRESHOLD"][0] == 0.5


def test_env_and_yaml_override(tmp_path):
    y = tmp_path / "c.yaml"
    y.write_text("router:\n  fraud_threshold: 0.7\nengine:\n  batch: 1024\n")
    c = load_config(str(y), environ={"FRAUD_THRESHOLD": "0.9", "SELDON_TIMEOUT": "250"},
                    overrides={"engine.depth": 3})
    assert c.router.fraud_threshold == 0.9      # env beats YAML
    assert c.engine.batch == 1024
    assert c.seldon.timeout_ms == 250
    assert c.engine.depth == 3
    with pytest.raises(KeyError):
        load_config(environ={}, overrides={"engine.nope": 1})


def test_metric_names():
    assert metric_names.TRANSACTION_INCOMING == "transaction_incoming"
    assert metric_names.NOTIFICATIONS_INCOMING == "notifications_incoming"
    assert set(metric_names.KIE_METRICS) == {"fraud_investigation_amount", "fraud_approved_low_amount",
                                             "fraud_approved_amount", "fraud_rejected_amount"}
    assert metric_names.MODEL_GAUGES == ("proba_1", "Amount", "V17", "V10")
    assert metric_names.N_AMOUNT_BUCKETS == 14


def test_feature_schema():
    assert N_FEATURES == 30
    assert FEATURE_NAMES[0] == "Time" and FEATURE_NAMES[-1] == "Amount"
    assert FEATURE_NAMES[10] == "V10" and FEATURE_NAMES[17] == "V17"


def test_tx_json_roundtrip():
    f = np.arange(30, dtype=np.float32) * 0.5
    tx = Transaction(id=42, customer_id=7, features=f, label=1)
    back = decode_tx_json(encode_tx_json(tx))
    assert back.id == 42 and back.customer_id == 7 and back.label == 1
    np.testing.assert_array_equal(back.features, f)
    alt = decode_tx_json(json.dumps({"features": f.tolist(), "id": 3}))
    np.testing.assert_array_equal(alt.features, f)
    sel = decode_tx_json(json.dumps({"data": {"ndarray": [f.tolist()]}}))
    np.testing.assert_array_equal(sel.features, f)
    with pytest.raises(ValueError):
        decode_tx_json(json.dumps({"features": [1, 2]}))


def test_txb1_roundtrip():
    rng = np.random.default_rng(0)
    n = 1001
    b = TxBatch(ids=np.arange(n, dtype=np.uint64) + 5, customer=rng.integers(0, 100, n, dtype=np.uint32),
                features=rng.standard_normal((n, 30)).astype(np.float32),
                labels=(rng.random(n) < 0.1).astype(np.uint8), base_offset=77)
    raw = b.encode()
    d = TxBatch.decode(raw)
    assert d.base_offset == 77 and len(d) == n
    np.testing.assert_array_equal(d.features, b.features)
    np.testing.assert_array_equal(d.ids, b.ids)
    np.testing.assert_array_equal(d.labels, b.labels)
    # features block is 16-byte aligned inside the message (zero-copy GPU consumption)
    _, _, off_feat, _, _ = TxBatch.layout(n, True)
    assert off_feat % 16 == 0
    with pytest.raises(ValueError):
        TxBatch.decode(raw[:100])
    txs = list(d.transactions())
    assert TxBatch.from_transactions(txs).features.shape == (n, 30)


def test_seldon_codec():
    X = np.random.default_rng(1).standard_normal((3, 30)).astype(np.float32)
    req = seldon.build_request(X)
    X2, names = seldon.parse_request(json.dumps(req))
    np.testing.assert_allclose(X2, X)
    assert names == list(FEATURE_NAMES)
    req_t = seldon.build_request(X, tensor=True)
    np.testing.assert_allclose(seldon.parse_request(req_t)[0], X)
    # named columns in a different order are re-ordered
    perm = list(reversed(FEATURE_NAMES))
    Xp, _ = seldon.parse_request({"data": {"names": perm, "ndarray": X[:, ::-1].tolist()}})
    np.testing.assert_allclose(Xp, X)
    resp = seldon.build_response([0.1, 0.9, 0.5])
    assert resp["data"]["names"] == ["proba_0", "proba_1"]
    np.testing.assert_allclose(seldon.proba1_from_response(resp), [0.1, 0.9, 0.5])
    with pytest.raises(seldon.SeldonError):
        seldon.parse_request({"nodata": 1})
    with pytest.raises(seldon.SeldonError):
        seldon.parse_request(b"{not json")


def test_dashboards_reference_metric_names():
    from ccfd_demo_summit_amd.metrics.dashboards import all_dashboards
    text = json.dumps(all_dashboards())
    for name in ("transaction_incoming_total", "transaction_outgoing_total", "notifications_incoming_total",
                 "fraud_investigation_amount", "fraud_approved_low_amount", "fraud_approved_amount",
                 "fraud_rejected_amount", "proba_1", "V17", "V10", "Amount",
                 "seldon_api_engine_server_requests_seconds_count",
                 "seldon_api_engine_client_requests_seconds_bucket", "ccfd_gpu_rows_total",
                 "kafka_server_brokertopicmetrics_messagesin_total", "kafka_server_replicamanager_partitioncount",
                 "kafka_controller_kafkacontroller_offlinepartitionscount", "ccfd_train_workers"):
        assert name in text, name
    # one generated dashboard per reference dashboard (Spark -> Training) plus the GPU one
    assert set(all_dashboards()) == {"Router.json", "KIE.json", "ModelPrediction.json", "SeldonCore.json",
                                     "Kafka.json", "Training.json", "GpuEngine.json"}


def test_trainer_exports_training_metrics():
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.metrics.exporter import TrainMetrics
    from ccfd_demo_summit_amd.train import TrainConfig, train_logistic
    X, y = generate(5000, seed=1, fraud_rate=0.05)
    tm = TrainMetrics()
    train_logistic(X, y, TrainConfig(epochs=1, batch=1000, device="cpu", metrics=tm))
    text = tm.expose().decode()
    assert 'ccfd_train_steps_total{model="lr"} 5.0' in text and "ccfd_train_workers 1.0" in text


def test_deploy_manifests_use_real_services_and_reference_names():
    """deploy/k8s/*.yaml: every container runs a launcher service that exists, and the
    reference's service names / ports (deploy/model/modelfull.json, deploy/ccd-service.yaml,
    deploy/router.yaml) are kept."""
    import glob
    import re

    import yaml

    from ccfd_demo_summit_amd.launch.__main__ import parse_args
    services = {}
    for f in glob.glob("deploy/k8s/*.yaml"):
        for d in yaml.safe_load_all(open(f)):
            if not d:
                continue
            if d["kind"] == "Service":
                services[d["metadata"]["name"]] = [p["port"] for p in d["spec"]["ports"]]
            spec = d.get("spec", {}).get("template", {}).get("spec", {})
            for c in spec.get("containers", []):
                cmd = " ".join(c.get("command", []))
                for svc in re.findall(r"ccfd_demo_summit_amd\.launch (\S+)", cmd):
                    if svc in ("supervise", "--"):
                        continue
                    parse_args([svc])                      # exits on an unknown service
    assert services["modelfull-modelfull"] == [8000]
    assert services["ccd-service"] == [8090]
    assert services["ccd-fuse"] == [8091]
    assert services["ccfd-seldon-model"] == [5000]
