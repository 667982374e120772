"""FraudDetection CR -> Kubernetes manifests (what an operator's reconcile writes to the API
server).  Service names, ports and env keys are the reference's (deploy/router.yaml,
deploy/ccd-service.yaml, deploy/notification-service.yaml, deploy/model/modelfull.json,
deploy/kafka/ProducerDeployment.yaml), so clients and the Grafana dashboards keep working;
deploy/k8s/ccfd-mi355x.yaml is this module's output for deploy/cr/frauddetection-mi355x.yaml.

``validate(manifests)`` is the structural check the tests run on every rendering: object
identity, selector <-> template label agreement, Service -> workload selection, ports,
ConfigMap references, env keys against the reference's contract, GPU requests only where
a GPU is used.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any, Dict, List

import yaml

from .spec import FraudDetectionSpec

LAUNCH = ["python", "-m", "ccfd_demo_summit_amd.launch"]
GRAFANA_DIR = Path(__file__).resolve().parents[2] / "deploy" / "grafana"


def _probes(path: str, port: int, start_s: int = 30) -> Dict[str, Any]:
    """readiness + liveness on a service's health route (tcp when ``path`` is None)."""
    act = {"httpGet": {"path": path, "port": port}} if path else {"tcpSocket": {"port": port}}
    return {"readinessProbe": dict(act, periodSeconds=5, failureThreshold=3),
            "livenessProbe": dict(act, initialDelaySeconds=start_s, periodSeconds=10, failureThreshold=6)}


def _container(spec: FraudDetectionSpec, name: str, command: List[str], ports=(), gpus: int = 0,
               env=None, envfrom: bool = True, probe=None) -> Dict[str, Any]:
    c: Dict[str, Any] = {"name": name, "image": spec.image, "workingDir": "/app", "command": command}
    if envfrom:
        c["envFrom"] = [{"configMapRef": {"name": "ccfd-env"}}]
    if env:
        c["env"] = [{"name": k, "value": str(v)} for k, v in env.items()]
    if ports:
        c["ports"] = [dict(p) for p in ports]
    if gpus:
        c["resources"] = {"limits": {"amd.com/gpu": gpus}}
    if probe:
        c.update(_probes(*probe))
    return c


RDZV_PORT = 29400        # multi-node engine: torchrun c10d rendezvous on pod ccfd-engine-0
TRAIN_METRICS_PORT = 8095   # trainer /metrics (+ local rank): the SparkMetrics dashboard's series


def _workload(kind: str, name: str, app: str, replicas: int, containers, annotations=None, grace: int = 30,
              extra_spec=None, volumes=None) -> Dict[str, Any]:
    tmpl_meta: Dict[str, Any] = {"labels": {"app": app}}
    if annotations:
        tmpl_meta["annotations"] = annotations
    pod: Dict[str, Any] = {"terminationGracePeriodSeconds": grace, "containers": containers}
    if volumes:
        pod["volumes"] = volumes
    spec: Dict[str, Any] = {"replicas": replicas, "selector": {"matchLabels": {"app": app}},
                            "template": {"metadata": tmpl_meta, "spec": pod}}
    if kind == "StatefulSet":
        spec["serviceName"] = name
    spec.update(extra_spec or {})
    return {"apiVersion": "apps/v1", "kind": kind, "metadata": {"name": name, "labels": {"app": app}}, "spec": spec}


def _service(name: str, app: str, ports) -> Dict[str, Any]:
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name},
            "spec": {"selector": {"app": app}, "ports": [dict(p) for p in ports]}}


def _scrape(path: str, port: int) -> Dict[str, str]:
    return {"prometheus.io/scrape": "true", "prometheus.io/path": path, "prometheus.io/port": str(port)}


def render(spec: FraudDetectionSpec) -> List[Dict[str, Any]]:
    from ..parallel.dp import resolve_row_format
    spec.validate()
    out: List[Dict[str, Any]] = []
    env = {"BROKER_URL": spec.broker_url, "KAFKA_TOPIC": "odh-demo",
           "CUSTOMER_NOTIFICATION_TOPIC": "ccd-customer-outgoing", "CUSTOMER_RESPONSE_TOPIC": "ccd-customer-response",
           "KIE_SERVER_URL": "http://ccd-service:8090", "SELDON_URL": "http://modelfull-modelfull:8000",
           "SELDON_ENDPOINT": "api/v0.1/predictions", "FRAUD_THRESHOLD": "0.5", "CONFIDENCE_THRESHOLD": "1.0",
           "CCFD_MODEL": spec.engine.model, "CCFD_WIRE": resolve_row_format(spec.engine.model, spec.engine.row_format),
           "CCFD_EXEC_MODE": spec.engine.exec_mode, "CCFD_OUTPUT_MODE": spec.engine.output_mode, "CCFD_PERSIST_ITEMS": spec.engine.persist_items}
    if spec.engine.rules:
        env["ROUTER_RULES"] = spec.engine.rules
    env["ROUTER_STANDARD_MODE"] = spec.engine.standard_mode
    if spec.engine.handoff_dlq:
        env["CCFD_HANDOFF_DLQ"] = spec.engine.handoff_dlq
    if spec.kie.shards > 1:            # one URL per shard pod (process/sharding.py kie_urls)
        env["KIE_SERVER_URL"] = "http://ccd-service-{shard}.ccd-service-shards:8090"
        env["CCFD_KIE_SHARDS"] = str(spec.kie.shards)
    env.update(spec.env)
    data = dict(env)
    data["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"          # dmabuf IPC for RCCL / cross-process tensors
    out.append({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "ccfd-env"}, "data": data})
    weights = ["--weights", spec.engine.weights] if spec.engine.weights else []

    if spec.kafka.deploy and spec.kafka.replicated:
        # replicated kafka-lite (ingest/kafka_replica.py): `brokers` broker pods, each its own
        # durable log on its own claim, replication factor min(3, brokers); pod k is node k + 1
        # (--node-id auto), advertised under the headless service; the controller keeps
        # membership, leaders / ISR and the committed offsets (ingest/kafka_controller.py) --
        # `controllers` member pods of a replicated quorum (ingest/controller_quorum.py, the
        # reference's three ZooKeeper nodes), pod k = member k + 1 (--member-id auto)
        name = f"{spec.kafka.cluster_name}-kafka"
        ctl = f"{name}-controller"
        nctl = max(1, spec.kafka.controllers)
        members = [f"http://{ctl}-{k}.{ctl}-members:9093" for k in range(nctl)]
        quorum = ["--member-id", "auto", "--peers", ",".join(f"{k + 1}={u}" for k, u in enumerate(members))] \
            if nctl > 1 else []
        cc = _container(spec, "controller", LAUNCH + ["kafka-controller", "--port", "9093", "--nodes",
                                                      str(spec.kafka.brokers), "--replication-factor",
                                                      str(spec.kafka.replication_factor),
                                                      "--data-dir", "/var/lib/kafka-controller"] + quorum,
                        ports=[{"containerPort": 9093, "name": "http"}], envfrom=False,
                        probe=("/health/ping", 9093, 20))
        cc["volumeMounts"] = [{"name": "controller-data", "mountPath": "/var/lib/kafka-controller"}]
        ctl_extra = {"serviceName": f"{ctl}-members", "podManagementPolicy": "Parallel",
                     "volumeClaimTemplates": [{"metadata": {"name": "controller-data"}, "spec": {
                         "accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}}}}]}
        out.append(_workload("StatefulSet", ctl, ctl, nctl, [cc], annotations=_scrape("/metrics", 9093),
                             extra_spec=ctl_extra))
        out.append(_service(ctl, ctl, [{"name": "http", "port": 9093, "targetPort": 9093}]))
        out.append({"apiVersion": "v1", "kind": "Service", "metadata": {"name": f"{ctl}-members"},
                    "spec": {"clusterIP": "None", "selector": {"app": ctl}, "publishNotReadyAddresses": True,
                             "ports": [{"name": "http", "port": 9093, "targetPort": 9093}]}})
        ctl_urls = ",".join(members) if nctl > 1 else f"http://{ctl}:9093"
        kc = _container(
            spec, "kafka", LAUNCH + ["kafka-lite", "--node-id", "auto", "--controller", ctl_urls,
                                     "--port", "9092", "--advertise", f"$(POD_NAME).{name}-brokers",
                                     "--data-dir", "/var/lib/kafka-lite", "--fsync", spec.kafka.fsync],
            ports=[{"containerPort": 9092, "name": "broker"}, {"containerPort": 9404, "name": "metrics"}],
            env={"CCFD_KAFKA_PARTITIONS": spec.kafka.partitions}, envfrom=False, probe=(None, 9092, 20))
        kc["env"].append({"name": "POD_NAME", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}})
        kc["volumeMounts"] = [{"name": "kafka-data", "mountPath": "/var/lib/kafka-lite"}]
        extra = {"serviceName": f"{name}-brokers", "podManagementPolicy": "Parallel"}
        vols = None
        if spec.kafka.storage:
            extra["volumeClaimTemplates"] = [{"metadata": {"name": "kafka-data"}, "spec": {
                "accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": spec.kafka.storage}}}}]
        else:
            vols = [{"name": "kafka-data", "emptyDir": {}}]
        out.append(_workload("StatefulSet", name, name, spec.kafka.brokers, [kc], annotations=_scrape("/metrics", 9404),
                             extra_spec=extra, volumes=vols))
        out.append({"apiVersion": "v1", "kind": "Service", "metadata": {"name": f"{name}-brokers"},
                    "spec": {"clusterIP": "None", "selector": {"app": name},
                             "ports": [{"name": "broker", "port": 9092, "targetPort": 9092}]}})
        out.append(_service(f"{name}-bootstrap", name, [{"name": "broker", "port": 9092, "targetPort": 9092}]))
    elif spec.kafka.deploy:
        # kafka-lite: one process, `brokers` listeners over a shared controller/store (the
        # Strimzi cluster of frauddetection_cr.yaml:71-77 in miniature)
        name = f"{spec.kafka.cluster_name}-kafka"
        ports = [{"containerPort": 9092 + i, "name": f"broker-{i}"} for i in range(spec.kafka.brokers)]
        ports.append({"containerPort": 9404, "name": "metrics"})
        # durable logs (ingest/durable_store.py): a restarted broker pod recovers every
        # acknowledged record and committed offset from its volume
        kc = _container(
            spec, "kafka", LAUNCH + ["kafka-lite", "--nodes", str(spec.kafka.brokers), "--port", "9092",
                                     "--advertise", f"{name}-brokers", "--data-dir", "/var/lib/kafka-lite",
                                     "--fsync", spec.kafka.fsync],
            ports=ports, env={"CCFD_KAFKA_PARTITIONS": spec.kafka.partitions}, envfrom=False,
            probe=(None, 9092, 20))
        kc["volumeMounts"] = [{"name": "kafka-data", "mountPath": "/var/lib/kafka-lite"}]
        if spec.kafka.storage:
            extra = {"volumeClaimTemplates": [{"metadata": {"name": "kafka-data"}, "spec": {
                "accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": spec.kafka.storage}}}}]}
            out.append(_workload("StatefulSet", name, name, 1, [kc], annotations=_scrape("/metrics", 9404),
                                 extra_spec=extra))
        else:
            out.append(_workload("StatefulSet", name, name, 1, [kc], annotations=_scrape("/metrics", 9404),
                                 volumes=[{"name": "kafka-data", "emptyDir": {}}]))
        for svc in (f"{name}-brokers", f"{name}-bootstrap"):
            out.append(_service(svc, name, [{"name": f"broker-{i}", "port": 9092 + i, "targetPort": 9092 + i}
                                            for i in range(spec.kafka.brokers)]))

    if spec.engine.deploy:
        g, nodes = spec.engine.gpus_per_node, spec.engine.nodes
        # one data-parallel job over every engine pod: ranks own partitions p = rank (mod
        # nodes x GPUs), so the pods must share ONE world -- torchrun's c10d rendezvous hosted
        # by pod 0 (stable name through the headless service) assigns the ranks
        dist_args = (["--standalone"] if nodes == 1 else
                     ["--nnodes", str(nodes), "--rdzv-backend", "c10d", "--rdzv-id", "ccfd-engine",
                      "--rdzv-endpoint", f"ccfd-engine-0.ccfd-engine:{RDZV_PORT}"])
        cmd = LAUNCH + ["supervise", "--", "python", "-m", "torch.distributed.run"] + dist_args + [
            "--nproc-per-node", str(g)] + LAUNCH[1:] + ["engine"] + weights
        # rank r also serves the model's own /prometheus on 8000 + r (launch engine
        # --model-metrics-port): proba_1 / Amount / V17 / V10 + seldon_api_engine_* of its traffic,
        # scraped by the "ccfd-model" job below (one target per declared port)
        ports = [{"containerPort": 8091, "name": "metrics"}] + \
            [{"containerPort": 8000 + r, "name": f"model-{r}"} for r in range(g)]
        if nodes > 1:
            ports.append({"containerPort": RDZV_PORT, "name": "rendezvous"})
            out.append({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "ccfd-engine"},
                        "spec": {"clusterIP": "None", "selector": {"app": "ccfd-engine"},
                                 "ports": [{"name": "rendezvous", "port": RDZV_PORT, "targetPort": RDZV_PORT}]}})
        eng_c = _container(spec, "engine", cmd, ports=ports, gpus=g, probe=("/health/ping", 8091, 120))
        vols = None
        eng_extra = None
        if spec.engine.handoff_dlq:            # the hand-off dead-letter journal's directory
            import posixpath
            eng_c["volumeMounts"] = [{"name": "handoff-dlq", "mountPath": posixpath.dirname(spec.engine.handoff_dlq)}]
            if spec.engine.dlq_storage:        # its offsets are committed: it must outlive the pod
                eng_extra = {"volumeClaimTemplates": [{"metadata": {"name": "handoff-dlq"}, "spec": {
                    "accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": spec.engine.dlq_storage}}}}]}
            else:                              # emptyDir: survives container restarts, not pod deletion
                vols = [{"name": "handoff-dlq", "emptyDir": {}}]
        out.append(_workload("StatefulSet", "ccfd-engine", "ccfd-engine", nodes, [eng_c],
                             annotations=_scrape("/prometheus", 8091), volumes=vols, extra_spec=eng_extra))

    if spec.seldon.deploy:
        cmd = LAUNCH + ["seldon", "--device", "auto"] + weights
        if spec.seldon.native:
            cmd += ["--native", "--workers", str(spec.seldon.workers)]
        out.append(_workload("Deployment", "modelfull-modelfull", "modelfull", spec.seldon.replicas, [_container(
            spec, "modelfull", cmd, ports=[{"containerPort": 8000, "name": "http"}], gpus=spec.seldon.gpus,
            probe=("/health/ping", 8000, 60))],
            annotations=_scrape("/prometheus", 8000), grace=20))
        out.append(_service("modelfull-modelfull", "modelfull", [{"name": "http", "port": 8000, "targetPort": 8000}]))

    if spec.usertask.deploy:
        out.append(_workload("Deployment", "ccfd-seldon-model", "ccfd-seldon-model", spec.usertask.replicas,
                             [_container(spec, "usertask", LAUNCH + ["usertask", "--port", "5000"],
                                         ports=[{"containerPort": 5000, "name": "http"}], envfrom=False,
                                         probe=("/health/ping", 5000, 30))]))
        out.append(_service("ccfd-seldon-model", "ccfd-seldon-model", [{"name": "http", "port": 5000, "targetPort": 5000}]))

    if spec.kie.deploy:
        # the KIE tier: kie.shards pods of one StatefulSet; pod ccd-service-k is shard k (the
        # launcher reads the ordinal from its host name) with its own journal volume, reached
        # through the headless service as ccd-service-k.ccd-service-shards (process/sharding.py)
        kie_extra: Dict[str, Any] = {"serviceName": "ccd-service-shards", "podManagementPolicy": "Parallel",
                                     "updateStrategy": {"type": "RollingUpdate"}}
        kie_vols = None
        if spec.kie.storage:
            kie_extra["volumeClaimTemplates"] = [{"metadata": {"name": "journal"}, "spec": {
                "accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": spec.kie.storage}}}}]
        else:
            kie_vols = [{"name": "journal", "emptyDir": {}}]
        out.append(_workload(
            "StatefulSet", "ccd-service", "ccd-service", spec.kie.shards,
            [dict(_container(spec, "kie", LAUNCH + ["kie", "--journal", "/data/bp-journal.jsonl", "--remote-prediction"],
                             ports=[{"containerPort": 8090, "name": "http"}],
                             env={"SELDON_URL": "ccfd-seldon-model:5000", "SELDON_ENDPOINT": "predict"},
                             probe=("/services/rest/server", 8090, 30)),
                  volumeMounts=[{"name": "journal", "mountPath": "/data"}])],
            annotations=_scrape("/rest/metrics", 8090), extra_spec=kie_extra, volumes=kie_vols))
        out.append(_service("ccd-service", "ccd-service", [{"name": "http", "port": 8090, "targetPort": 8090}]))
        out.append({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "ccd-service-shards"},
                    "spec": {"clusterIP": "None", "selector": {"app": "ccd-service"},
                             "ports": [{"name": "http", "port": 8090, "targetPort": 8090}]}})

    if spec.notifier.deploy:
        out.append(_workload("Deployment", "ccfd-notification-service", "ccfd-notification-service",
                             spec.notifier.replicas, [_container(spec, "notifier", LAUNCH + ["notifier"],
                                                                 ports=[{"containerPort": 8080, "name": "health"}],
                                                                 probe=("/health/ping", 8080, 30))]))

    if spec.router.deploy:
        out.append(_workload("Deployment", "ccd-fuse", "ccd-fuse", spec.router.replicas, [_container(
            spec, "router", LAUNCH + ["supervise", "--"] + LAUNCH + ["router", "--group-membership"],
            ports=[{"containerPort": 8091, "name": "metrics"}], probe=("/health/ping", 8091, 30))],
            annotations=_scrape("/prometheus", 8091),
            extra_spec={"strategy": {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": "25%", "maxSurge": "25%"}}}))
        out.append(_service("ccd-fuse", "ccd-fuse", [{"name": "metrics", "port": 8091, "targetPort": 8091}]))

    if spec.producer.deploy:
        p = spec.producer
        out.append({"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "kafka-producer"},
                    "spec": {"template": {"metadata": {"labels": {"app": "kafka-producer"}}, "spec": {
                        "restartPolicy": "OnFailure",
                        "containers": [_container(spec, "producer", LAUNCH + ["producer", "--fmt", p.format,
                                                                              "--count", str(p.count)],
                                                  env={"topic": "odh-demo", "bootstrap": spec.broker_url,
                                                       "filename": p.csv})]}}}})

    if spec.training.deploy:
        t = spec.training
        cmd = ["python", "-m", "torch.distributed.run", "--standalone", "--nproc-per-node", str(t.workers),
               "-m", "ccfd_demo_summit_amd.train", "--model", t.model, "--out", "/models/model.safetensors",
               "--metrics-port", str(TRAIN_METRICS_PORT)]
        out.append({"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "ccfd-training"},
                    "spec": {"template": {"metadata": {"labels": {"app": "ccfd-training"}}, "spec": {
                        "restartPolicy": "OnFailure",
                        "containers": [dict(_container(spec, "train", cmd, gpus=t.gpus * t.workers,
                                                       ports=[{"containerPort": TRAIN_METRICS_PORT + r,
                                                               "name": f"spark-metrics-{r}"}
                                                              for r in range(t.workers)]),
                                            volumeMounts=[{"name": "models", "mountPath": "/models"}])],
                        "volumes": [{"name": "models", "emptyDir": {}}]}}}})

    if spec.monitoring.deploy:
        jobs = [{"job_name": "ccfd-pods", "kubernetes_sd_configs": [{"role": "pod"}],
                 "relabel_configs": [
                     {"source_labels": ["__meta_kubernetes_pod_annotation_prometheus_io_scrape"], "action": "keep",
                      "regex": "true"},
                     {"source_labels": ["__meta_kubernetes_pod_annotation_prometheus_io_path"],
                      "target_label": "__metrics_path__", "regex": "(.+)"},
                     {"source_labels": ["__address__", "__meta_kubernetes_pod_annotation_prometheus_io_port"],
                      "target_label": "__address__", "regex": "([^:]+)(?::\\d+)?;(\\d+)", "replacement": "$1:$2"}]},
                # the engine ranks' model endpoints (8000 + r): ModelPrediction.json selects
                # instance=~".*:8000", SeldonCore.json sums every rank
                {"job_name": "ccfd-model", "metrics_path": "/prometheus", "kubernetes_sd_configs": [{"role": "pod"}],
                 "relabel_configs": [
                     {"source_labels": ["__meta_kubernetes_pod_container_port_name"], "action": "keep",
                      "regex": "model-\\d+"}]},
                # the trainer: SparkMetrics.json selects job="Spark Metrics" (its series are the
                # Spark analogues of metrics/exporter.py TrainMetrics)
                {"job_name": "Spark Metrics", "metrics_path": "/metrics", "kubernetes_sd_configs": [{"role": "pod"}],
                 "relabel_configs": [
                     {"source_labels": ["__meta_kubernetes_pod_container_port_name"], "action": "keep",
                      "regex": "spark-metrics-\\d+"}]}]
        out.append({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "ccfd-prometheus"},
                    "data": {"prometheus.yml": yaml.safe_dump({"global": {"scrape_interval": "5s"},
                                                               "scrape_configs": jobs}, sort_keys=False)}})
        boards = sorted(p.name for p in GRAFANA_DIR.glob("*.json")) if GRAFANA_DIR.is_dir() else []
        out.append({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "ccfd-grafana-dashboards",
                                                                          "annotations": {"ccfd/source": "deploy/grafana"}},
                    "data": {b: f"deploy/grafana/{b}" for b in boards}})
    return out


def dump(manifests: List[Dict[str, Any]], header: str = "") -> str:
    return header + yaml.safe_dump_all(manifests, sort_keys=False, width=120)


# --------------------------------------------------------------------------- validation
def validate(manifests: List[Dict[str, Any]]) -> List[str]:
    """Structural problems of a rendering (empty list = valid)."""
    from ..config import ENV_MAP
    from ..contracts.env import REFERENCE_ENV
    probs: List[str] = []
    seen = set()
    workloads = []
    configmaps = {m["metadata"]["name"] for m in manifests if m.get("kind") == "ConfigMap"}
    allowed_env = set(REFERENCE_ENV) | set(ENV_MAP) | {"HSA_ENABLE_IPC_MODE_LEGACY", "CCFD_KAFKA_PARTITIONS",
                                                     "POD_NAME"}   # (downward API: a broker pod's own name)
    for m in manifests:
        for k in ("apiVersion", "kind", "metadata"):
            if k not in m:
                probs.append(f"object without {k}: {m}")
        key = (m.get("kind"), m.get("metadata", {}).get("name"))
        if key in seen:
            probs.append(f"duplicate {key}")
        seen.add(key)
        kind = m.get("kind")
        if kind == "ConfigMap":
            for k in m.get("data", {}):
                if m["metadata"]["name"] == "ccfd-env" and k not in allowed_env:
                    probs.append(f"ccfd-env: unknown env key {k}")
        if kind in ("Deployment", "StatefulSet", "Job"):
            tmpl = m["spec"]["template"]
            labels = tmpl.get("metadata", {}).get("labels", {})
            if kind != "Job":
                sel = m["spec"]["selector"]["matchLabels"]
                if any(labels.get(k) != v for k, v in sel.items()):
                    probs.append(f"{key}: selector {sel} does not match template labels {labels}")
                if m["spec"].get("replicas", 1) < 0:
                    probs.append(f"{key}: negative replicas")
                workloads.append(labels)
            ports = set()
            for c in tmpl["spec"]["containers"]:
                if not c.get("image") or not c.get("command"):
                    probs.append(f"{key}/{c.get('name')}: image and command required")
                for p in c.get("ports", []):
                    if p["containerPort"] in ports:
                        probs.append(f"{key}: duplicate container port {p['containerPort']}")
                    ports.add(p["containerPort"])
                for ef in c.get("envFrom", []):
                    if ef["configMapRef"]["name"] not in configmaps:
                        probs.append(f"{key}: envFrom unknown ConfigMap {ef['configMapRef']['name']}")
                for e in c.get("env", []):
                    if e["name"] not in allowed_env:
                        probs.append(f"{key}: unknown env key {e['name']}")
                for pk in ("readinessProbe", "livenessProbe"):
                    pr = c.get(pk)
                    if pr:
                        port = (pr.get("httpGet") or pr.get("tcpSocket") or {}).get("port")
                        if port not in {p["containerPort"] for p in c.get("ports", [])}:
                            probs.append(f"{key}/{c['name']}: {pk} on undeclared port {port}")
                gpu = c.get("resources", {}).get("limits", {}).get("amd.com/gpu", 0)
                if gpu and c["name"] not in ("engine", "modelfull", "train"):
                    probs.append(f"{key}: GPU requested by {c['name']}")
                if c["name"] == "engine":
                    cmd = c["command"]
                    nproc = int(cmd[cmd.index("--nproc-per-node") + 1])
                    if nproc != gpu:
                        probs.append(f"{key}: {nproc} ranks for {gpu} GPUs (one rank per GPU)")
                    nodes = m["spec"].get("replicas", 1)
                    if nodes > 1:
                        # every pod must join ONE world, or each would score the same partitions
                        nn = int(cmd[cmd.index("--nnodes") + 1]) if "--nnodes" in cmd else 1
                        if nn != nodes or "--rdzv-endpoint" not in cmd:
                            probs.append(f"{key}: {nodes} engine pods without a shared rendezvous "
                                         f"(--nnodes {nn}): each pod would score the same partitions")
                        headless = [x for x in manifests if x.get("kind") == "Service"
                                    and x["metadata"]["name"] == m["spec"].get("serviceName")
                                    and x["spec"].get("clusterIP") == "None"]
                        if not headless:
                            probs.append(f"{key}: no headless Service {m['spec'].get('serviceName')} for the pods' "
                                         "stable names")
            m["_ports"] = ports
    for m in manifests:
        if m.get("kind") == "Service":
            sel = m["spec"]["selector"]
            targets = [w for w in manifests if w.get("kind") in ("Deployment", "StatefulSet")
                       and all(w["spec"]["template"]["metadata"]["labels"].get(k) == v for k, v in sel.items())]
            if not targets:
                probs.append(f"Service {m['metadata']['name']}: selects no workload")
            for p in m["spec"]["ports"]:
                if targets and all(p["targetPort"] not in t.get("_ports", ()) for t in targets):
                    probs.append(f"Service {m['metadata']['name']}: targetPort {p['targetPort']} not exposed")
    for m in manifests:
        m.pop("_ports", None)
    return probs
