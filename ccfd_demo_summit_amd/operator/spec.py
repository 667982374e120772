"""The FraudDetection custom resource: one declarative document for the whole stack -- the
analogue of the reference's OpenDataHub CR (deploy/frauddetection_cr.yaml:1-89), which an
operator reconciles into Kafka / Seldon / Spark / monitoring deployments (SURVEY.md §2.1
C18, §1 L0).

Two document kinds are accepted:

* ``kind: FraudDetection`` (apiVersion ``ccfd.amd.com/v1alpha1``) -- this framework's CR,
  see deploy/cr/frauddetection-mi355x.yaml;
* ``kind: OpenDataHub`` -- the reference's CR.  The components that have an equivalent
  here are mapped (``kafka.kafka_cluster_name`` / ``kafka_broker_replicas``,
  ``seldon.odh_deploy``, ``monitoring.odh_deploy``, the Spark cluster's
  ``spark_worker_nodes`` -> data-parallel training ranks); the notebook / BeakerX /
  AI-library components have none and are listed in ``notes``.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Any, Dict, List

import yaml

API_VERSION = "ccfd.amd.com/v1alpha1"
KIND = "FraudDetection"


class SpecError(ValueError):
    pass


@dataclass
class KafkaSpec:
    deploy: bool = True              # False: use the external cluster at ``bootstrap``
    cluster_name: str = "odh-message-bus"
    brokers: int = 3                 # kafka-lite listeners (reference: kafka_broker_replicas 3)
    partitions: int = 16
    bootstrap: str = ""              # external bootstrap list when deploy is False
    storage: str = "50Gi"            # kafka-lite's durable logs (--data-dir): a PersistentVolumeClaim of
                                     # this size per broker pod; "" = emptyDir (survives container, not pod, restarts)
    fsync: str = "interval"          # kafka-lite flush policy: always | interval | never
    replicated: bool = True          # brokers = separate pods, each its own log, a controller for
                                     # fail-over (ingest/kafka_controller.py) -- the reference's Strimzi
                                     # cluster of 3 brokers; False = one pod, N listeners
    replication_factor: int = 3      # copies of every partition (1 = scale-out only, Kafka's default for
                                     # auto-created topics; 3 = a broker loss loses nothing acknowledged)
    controllers: int = 3             # replicated controller members (ingest/controller_quorum.py) -- the
                                     # reference's kafka_zookeeper_replicas; 1 = a single controller


@dataclass
class EngineSpec:
    deploy: bool = True
    nodes: int = 1                   # engine pods, one per 8-GPU node
    gpus_per_node: int = 8           # ranks per pod (torchrun), one per GPU
    model: str = "mlp"
    weights: str = ""                # safetensors file (models.save_model); "" = random init
    row_format: str = "auto"         # f32 | w64 | g32 | g20 | auto
    exec_mode: str = "auto"          # persistent | launch | auto (persistent for zero-copy in/out)
    output_mode: str = "zerocopy"    # zerocopy | dma
    persist_items: str = "auto"      # persistent MLP on W64 rows: claimed (throughput, = auto) | pipelined
    rules: str = ""                  # routing rule text or file (ROUTER_RULES)
    standard_mode: str = "count"     # count | process: a standard process per standard-routed
                                     # transaction, as the reference router does (README.md:552)
    handoff_dlq: str = ""            # dead-letter journal of KIE-refused hand-offs ("" = hold + retry)
    dlq_storage: str = "1Gi"         # the DLQ's volume: a PersistentVolumeClaim of this size per engine pod
                                     # (its entries' offsets are already committed); "" = emptyDir


@dataclass
class ServiceSpec:
    deploy: bool = True
    replicas: int = 1


@dataclass
class KieSpec(ServiceSpec):
    shards: int = 1                  # KIE shard pods (process/sharding.py): starts routed by transaction
                                     # hash, signals / tasks by shard-encoded id; replicas stays 1 (a KIE
                                     # replica with its own state IS a shard)
    storage: str = "10Gi"            # each shard's journal volume (PVC); "" = emptyDir


@dataclass
class SeldonSpec(ServiceSpec):
    gpus: int = 1
    native: bool = False             # C++ epoll REST front end
    workers: int = 1


@dataclass
class ProducerSpec:
    deploy: bool = True
    format: str = "txb1"             # txb1 | json (the reference's one transaction per message)
    count: int = 100_000_000
    csv: str = "OPEN/uploaded/creditcard.csv"


@dataclass
class TrainingSpec:
    deploy: bool = False
    workers: int = 2                 # data-parallel ranks (reference: 2 Spark executors)
    model: str = "mlp"
    gpus: int = 1                    # GPUs per worker (0 = CPU / gloo)


@dataclass
class FraudDetectionSpec:
    name: str = "ccfd"
    image: str = "ccfd-mi355x:latest"
    kafka: KafkaSpec = field(default_factory=KafkaSpec)
    engine: EngineSpec = field(default_factory=EngineSpec)
    seldon: SeldonSpec = field(default_factory=SeldonSpec)
    usertask: ServiceSpec = field(default_factory=ServiceSpec)
    kie: KieSpec = field(default_factory=KieSpec)
    notifier: ServiceSpec = field(default_factory=ServiceSpec)
    router: ServiceSpec = field(default_factory=lambda: ServiceSpec(deploy=False))   # compat REST router
    producer: ProducerSpec = field(default_factory=ProducerSpec)
    training: TrainingSpec = field(default_factory=TrainingSpec)
    monitoring: ServiceSpec = field(default_factory=ServiceSpec)
    env: Dict[str, str] = field(default_factory=dict)      # reference env keys (contracts/env.py)
    notes: List[str] = field(default_factory=list)         # mapping remarks (OpenDataHub input)

    @property
    def broker_url(self) -> str:
        """BROKER_URL of every client (reference: ``<cluster>-kafka-brokers:9092``)."""
        if not self.kafka.deploy:
            if not self.kafka.bootstrap:
                raise SpecError("kafka.deploy is false but kafka.bootstrap is empty")
            return self.kafka.bootstrap
        host = f"{self.kafka.cluster_name}-kafka-brokers"
        if self.kafka.replicated:           # one broker pod each: <sts>-<k>.<headless svc>:9092
            sts = f"{self.kafka.cluster_name}-kafka"
            return ",".join(f"{sts}-{i}.{host}:9092" for i in range(self.kafka.brokers))
        return ",".join(f"{host}:{9092 + i}" for i in range(self.kafka.brokers))

    def validate(self) -> "FraudDetectionSpec":
        from ..config import ENV_MAP
        from ..contracts.env import REFERENCE_ENV
        if self.kafka.brokers < 1 or self.kafka.partitions < 1:
            raise SpecError("kafka.brokers and kafka.partitions must be >= 1")
        if self.engine.deploy and (self.engine.nodes < 1 or not 1 <= self.engine.gpus_per_node <= 8):
            raise SpecError("engine.nodes >= 1 and 1 <= engine.gpus_per_node <= 8 (one rank per GPU of a node)")
        ranks = self.engine.nodes * self.engine.gpus_per_node
        if self.engine.deploy and self.kafka.deploy and self.kafka.partitions < ranks:
            # ranks own partitions p = rank (mod world): a rank without one would sit idle
            raise SpecError(f"kafka.partitions {self.kafka.partitions} < {ranks} engine ranks "
                            f"(nodes x gpusPerNode): every rank needs at least one partition")
        if self.engine.exec_mode not in ("auto", "persistent", "launch"):
            raise SpecError(f"engine.exec_mode {self.engine.exec_mode!r}: auto | persistent | launch")
        if self.engine.persist_items not in ("pipelined", "claimed", "auto"):
            raise SpecError(f"engine.persist_items {self.engine.persist_items!r}: pipelined | claimed | auto")
        if self.kafka.fsync not in ("always", "interval", "never"):
            raise SpecError(f"kafka.fsync {self.kafka.fsync!r}: always | interval | never")
        if self.engine.standard_mode not in ("count", "process"):
            raise SpecError(f"engine.standard_mode {self.engine.standard_mode!r}: count | process")
        if self.engine.output_mode not in ("zerocopy", "dma"):
            raise SpecError(f"engine.output_mode {self.engine.output_mode!r}: zerocopy | dma")
        if self.engine.exec_mode == "persistent" and self.engine.output_mode != "zerocopy":
            raise SpecError("engine.exec_mode persistent needs engine.output_mode zerocopy")
        if self.engine.model not in ("mlp", "lr", "gbdt"):
            raise SpecError(f"engine.model {self.engine.model!r}: mlp | lr | gbdt")
        from ..parallel.dp import resolve_row_format
        try:
            resolve_row_format(self.engine.model, self.engine.row_format)
        except ValueError as e:
            raise SpecError(f"engine.row_format: {e}") from None
        for n, s in (("seldon", self.seldon), ("usertask", self.usertask), ("kie", self.kie),
                     ("notifier", self.notifier), ("router", self.router)):
            if s.replicas < 0:
                raise SpecError(f"{n}.replicas must be >= 0")
        if self.kie.shards < 1:
            raise SpecError("kie.shards must be >= 1")
        if self.kie.deploy and self.kie.replicas != 1:
            raise SpecError("kie.replicas must be 1: KIE instances keep their own state, so scale the tier "
                            "with kie.shards (each shard owns a hash range of transactions)")
        if self.producer.format not in ("txb1", "json"):
            raise SpecError("producer.format: txb1 | json")
        if self.training.workers < 1:
            raise SpecError("training.workers must be >= 1")
        unknown = [k for k in self.env if k not in REFERENCE_ENV and k not in ENV_MAP]
        if unknown:
            raise SpecError(f"env: unknown keys {unknown} (reference keys: contracts/env.py, CCFD_*: config.py)")
        self.broker_url   # kafka bootstrap consistency
        return self

    def to_dict(self) -> Dict[str, Any]:
        d = dataclasses.asdict(self)
        d.pop("notes")
        name = d.pop("name")
        return {"apiVersion": API_VERSION, "kind": KIND, "metadata": {"name": name}, "spec": _camel(d)}


# --------------------------------------------------------------------------- parsing
def _snake(k: str) -> str:
    return "".join("_" + c.lower() if c.isupper() else c for c in k).replace("-", "_")


def _camel(d):
    if isinstance(d, dict):
        out = {}
        for k, v in d.items():
            parts = k.split("_")
            key = parts[0] + "".join(p.title() for p in parts[1:]) if k != "env" else k
            out[key] = v if k == "env" else _camel(v)
        return out
    return d


def _fill(obj, doc: Dict[str, Any], path: str):
    if not isinstance(doc, dict):
        raise SpecError(f"{path}: expected a mapping")
    names = {f.name: f for f in dataclasses.fields(obj)}
    for k, v in doc.items():
        sk = _snake(k)
        if sk not in names or sk in ("notes", "name"):
            raise SpecError(f"{path}.{k}: unknown field")
        cur = getattr(obj, sk)
        if dataclasses.is_dataclass(cur):
            _fill(cur, v or {}, f"{path}.{k}")
        elif isinstance(cur, dict):
            setattr(obj, sk, {str(a): str(b) for a, b in (v or {}).items()})
        elif isinstance(cur, bool):
            if not isinstance(v, bool):
                raise SpecError(f"{path}.{k}: expected true/false")
            setattr(obj, sk, v)
        elif isinstance(cur, int):
            if isinstance(v, bool) or not isinstance(v, int):
                raise SpecError(f"{path}.{k}: expected an integer")
            setattr(obj, sk, v)
        else:
            setattr(obj, sk, "" if v is None else str(v))


def from_odh(doc: Dict[str, Any]) -> FraudDetectionSpec:
    """The reference's OpenDataHub CR -> the equivalent FraudDetection spec."""
    spec = FraudDetectionSpec(name=(doc.get("metadata") or {}).get("name", "ccfd"))
    s = doc.get("spec") or {}
    on = lambda comp: bool((s.get(comp) or {}).get("odh_deploy", False))
    k = s.get("kafka") or {}
    spec.kafka.deploy = on("kafka")
    spec.kafka.cluster_name = str(k.get("kafka_cluster_name", spec.kafka.cluster_name))
    spec.kafka.brokers = int(k.get("kafka_broker_replicas", spec.kafka.brokers))
    if "kafka_zookeeper_replicas" in k:
        spec.kafka.controllers = max(1, int(k["kafka_zookeeper_replicas"]))
        spec.notes.append(f"kafka.kafka_zookeeper_replicas {spec.kafka.controllers} -> a {spec.kafka.controllers}-member "
                          "replicated kafka-lite controller (ingest/controller_quorum.py) in ZooKeeper's role")
    spec.seldon.deploy = on("seldon")
    spec.monitoring.deploy = on("monitoring")
    jh = s.get("aicoe-jupyterhub") or {}
    if on("spark-operator") or on("aicoe-jupyterhub"):
        spec.training.deploy = True
        spec.training.workers = max(1, int(jh.get("spark_worker_nodes", 2)))
        spec.notes.append(f"spark cluster ({spec.training.workers} workers) -> data-parallel training job "
                          f"with {spec.training.workers} ranks (train/trainer.py)")
    for comp in ("aicoe-jupyterhub", "jupyter-on-openshift", "beakerx", "ai-library"):
        if on(comp):
            spec.notes.append(f"{comp}: notebooks have no equivalent here (training is a job, not a notebook)")
    if not spec.kafka.deploy and not spec.kafka.bootstrap:
        spec.kafka.deploy = True
        spec.notes.append("kafka.odh_deploy false without an external bootstrap: deploying kafka-lite")
    return spec


def parse(doc: Dict[str, Any]) -> FraudDetectionSpec:
    if not isinstance(doc, dict):
        raise SpecError("CR document must be a mapping")
    kind = doc.get("kind")
    if kind == "OpenDataHub":
        return from_odh(doc).validate()
    if kind != KIND:
        raise SpecError(f"kind {kind!r}: expected {KIND} or OpenDataHub")
    if doc.get("apiVersion") != API_VERSION:
        raise SpecError(f"apiVersion {doc.get('apiVersion')!r}: expected {API_VERSION}")
    spec = FraudDetectionSpec(name=str((doc.get("metadata") or {}).get("name", "ccfd")))
    _fill(spec, doc.get("spec") or {}, "spec")
    return spec.validate()


def load(path: str) -> FraudDetectionSpec:
    with open(path) as f:
        return parse(yaml.safe_load(f))
