"""Single typed configuration for every component.

Precedence (SURVEY.md §5 "Config / flag system"): dataclass defaults (= the reference
values from deploy/*.yaml) -> optional YAML file -> the same env var names the
reference uses -> explicit overrides (CLI flags).
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Mapping, Optional

import yaml

from .contracts.env import KIE_SELDON_ENDPOINT_DEFAULT, KIE_SELDON_URL_DEFAULT


@dataclass
class KafkaConfig:
    broker_url: str = "odh-message-bus-kafka-brokers:9092"   # BROKER_URL
    transactions_topic: str = "odh-demo"                      # KAFKA_TOPIC
    notification_topic: str = "ccd-customer-outgoing"         # CUSTOMER_NOTIFICATION_TOPIC
    response_topic: str = "ccd-customer-response"             # CUSTOMER_RESPONSE_TOPIC
    partitions: int = 8
    group_id: str = "ccfd-engine"
    backend: str = "inproc"          # "inproc" (fake broker) | "kafka" (wire protocol client)


@dataclass
class SeldonConfig:
    url: str = "http://modelfull-modelfull:8000"              # SELDON_URL (router)
    endpoint: str = "api/v0.1/predictions"                    # SELDON_ENDPOINT (router)
    token: Optional[str] = None                               # SELDON_TOKEN
    timeout_ms: int = 5000                                    # SELDON_TIMEOUT
    pool_size: int = 5                                        # SELDON_POOL_SIZE
    host: str = "0.0.0.0"
    port: int = 8000                                          # modelfull.json / router.yaml:68
    model_name: str = "modelfull"
    max_batch: int = 4096
    max_delay_us: int = 200          # dynamic batching deadline for predict()


@dataclass
class KieConfig:
    url: str = "http://ccd-service:8090"                      # KIE_SERVER_URL
    port: int = 8090
    seldon_url: str = KIE_SELDON_URL_DEFAULT                  # ccd-service.yaml:61-62
    seldon_endpoint: str = KIE_SELDON_ENDPOINT_DEFAULT        # README.md:379
    confidence_threshold: float = 1.0                         # CONFIDENCE_THRESHOLD
    notification_timeout_s: float = 30.0                      # BP timer (value not in reference)
    dmn_probability_threshold: float = 0.75                   # DMN (README.md:592-596), value not in reference
    dmn_amount_threshold: float = 100.0                       # "sufficiently small" amount
    container_id: str = "ccd-fraud-kjar"
    fraud_process_id: str = "ccd-fraud-kjar.CCDProcess"
    standard_process_id: str = "ccd-fraud-kjar.StandardProcess"
    signal_name: str = "customerResponse"
    shards: int = 1                  # KIE shard processes (process/sharding.py): starts routed by
                                     # transaction-id hash, signals / tasks by shard-encoded id;
                                     # KIE_SERVER_URL then lists one URL per shard or a {shard} template
    standard_dedupe_window: int = 1 << 20    # standard-start dedupe keys kept at least (per shard)
    standard_dedupe_capacity: int = 0        # hard bound of uncommitted + kept keys (0 = 4 x window):
                                             # beyond it a start batch is refused (503, retried) --
                                             # keys leave only once the engine committed past them
    standard_audit_rows: int = 1 << 22       # standard instances answerable by transaction id from
                                             # memory (per shard); older ones from the journal


@dataclass
class RouterConfig:
    fraud_threshold: float = 0.5                              # FRAUD_THRESHOLD (router.yaml:69-70)
    port: int = 8091                                          # README.md:503-506
    rules: str = ""                  # ROUTER_RULES: routing rule file or inline rules ("when ... then
                                     # fraud; otherwise standard"); "" = the reference threshold rule
    standard_mode: str = "count"     # standard-routed transactions: "count" (counters only -- the
                                     # default at 1e9 tx/s) | "process": start a standard process per
                                     # transaction, like the reference router (README.md:552)


@dataclass
class NotifierConfig:
    p_reply: float = 0.8             # "randomly generate a reply (or no reply)" README.md:414,565
    p_approve: float = 0.5
    mean_delay_s: float = 0.5
    seed: int = 0
    port: int = 8080                 # notification-service.yaml:47-49


@dataclass
class EngineConfig:
    model: str = "mlp"               # lr | mlp | gbdt
    batch: int = 4096                # micro-batch rows (BASELINE config 2)
    depth: int = 12                  # micro-batches in flight per GPU (p50 53 us at the PCIe rate)
    streams: int = 4                 # HIP streams per engine
    input_mode: str = "zerocopy"     # dma (H2D into HBM) | zerocopy (kernel reads pinned host)
    wire: str = "auto"               # ring row format: f32 | w64 | g32 | g20 | auto (w64 for mlp/lr, g20 for gbdt)
    coalesce: int = 4                # ready micro-batches per kernel launch (MLP, launch mode)
    ingest_threads: int = 0          # native Kafka consumer threads per rank (partitions split; 0 = auto:
                                     # one per partition for GBDT's binned rows, else 1)
    model_watch: str = ""            # hot-swap when this safetensors file changes (rank 0)
    output_mode: str = "zerocopy"    # zerocopy (kernel writes pinned host) | dma
    exec_mode: str = "auto"          # persistent | launch | auto (persistent for zero-copy in/out:
                                     # the mode bench.py measures; launch_/engine_service.py)
    persist_items: str = "auto"      # persistent MLP on W64 rows: claimed (throughput, = auto) | pipelined
    handoff_capacity: int = 1 << 21  # fraud starts queued for KIE before scoring pauses (back-pressure)
    handoff_workers: int = 2         # pooled HTTP workers of the KIE hand-off (router/handoff.py)
    handoff_dlq: str = ""            # dead-letter journal of requests KIE refused (4xx); "" = no DLQ:
                                     # a refused request is held and retried, never acked unsent
    scored_capacity: int = 1 << 20   # standard_mode=process: per-row scored-record ring (rows)
    native_serve: bool = True        # score the rings from the engine's C++ serving thread (no Python
                                     # on the scoring path); False = the Python scoring thread
    max_delay_us: int = 500          # deadline flush for partially filled micro-batches
    reduce_period_ms: float = 10.0   # X2 counter all-reduce period
    gbdt_trees: int = 100
    gbdt_depth: int = 6


@dataclass
class Config:
    kafka: KafkaConfig = field(default_factory=KafkaConfig)
    seldon: SeldonConfig = field(default_factory=SeldonConfig)
    kie: KieConfig = field(default_factory=KieConfig)
    router: RouterConfig = field(default_factory=RouterConfig)
    notifier: NotifierConfig = field(default_factory=NotifierConfig)
    engine: EngineConfig = field(default_factory=EngineConfig)
    seed: int = 0

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


# env key -> (section, field, type)
ENV_MAP = {
    "BROKER_URL": ("kafka", "broker_url", str),
    "KAFKA_TOPIC": ("kafka", "transactions_topic", str),
    "CUSTOMER_NOTIFICATION_TOPIC": ("kafka", "notification_topic", str),
    "CUSTOMER_RESPONSE_TOPIC": ("kafka", "response_topic", str),
    "KIE_SERVER_URL": ("kie", "url", str),
    "SELDON_URL": ("seldon", "url", str),
    "SELDON_ENDPOINT": ("seldon", "endpoint", str),
    "SELDON_TOKEN": ("seldon", "token", str),
    "SELDON_TIMEOUT": ("seldon", "timeout_ms", int),
    "SELDON_POOL_SIZE": ("seldon", "pool_size", int),
    "CONFIDENCE_THRESHOLD": ("kie", "confidence_threshold", float),
    "FRAUD_THRESHOLD": ("router", "fraud_threshold", float),
    "ROUTER_RULES": ("router", "rules", str),
    "ROUTER_STANDARD_MODE": ("router", "standard_mode", str),
    # framework-specific keys
    "CCFD_MODEL": ("engine", "model", str),
    "CCFD_BATCH": ("engine", "batch", int),
    "CCFD_DEPTH": ("engine", "depth", int),
    "CCFD_WIRE": ("engine", "wire", str),
    "CCFD_COALESCE": ("engine", "coalesce", int),
    "CCFD_MODEL_WATCH": ("engine", "model_watch", str),
    "CCFD_INPUT_MODE": ("engine", "input_mode", str),
    "CCFD_OUTPUT_MODE": ("engine", "output_mode", str),
    "CCFD_EXEC_MODE": ("engine", "exec_mode", str),
    "CCFD_PERSIST_ITEMS": ("engine", "persist_items", str),
    "CCFD_HANDOFF_CAPACITY": ("engine", "handoff_capacity", int),
    "CCFD_HANDOFF_DLQ": ("engine", "handoff_dlq", str),
    "CCFD_NATIVE_SERVE": ("engine", "native_serve", str),
    "CCFD_KAFKA_BACKEND": ("kafka", "backend", str),
    "CCFD_KAFKA_PARTITIONS": ("kafka", "partitions", int),
    "CCFD_INGEST_THREADS": ("engine", "ingest_threads", int),
    "CCFD_KIE_NOTIFICATION_TIMEOUT_S": ("kie", "notification_timeout_s", float),
    "CCFD_KIE_SHARDS": ("kie", "shards", int),
    "CCFD_KIE_DEDUPE_WINDOW": ("kie", "standard_dedupe_window", int),
    "CCFD_KIE_DEDUPE_CAPACITY": ("kie", "standard_dedupe_capacity", int),
    "CCFD_KIE_AUDIT_ROWS": ("kie", "standard_audit_rows", int),
    "CCFD_NOTIFIER_SEED": ("notifier", "seed", int),
}


def _apply(cfg: Config, section: str, key: str, value: Any) -> None:
    sec = getattr(cfg, section)
    if not hasattr(sec, key):
        raise KeyError(f"unknown config key {section}.{key}")
    cur = getattr(sec, key)
    if value is not None and cur is not None and not isinstance(value, type(cur)):
        if isinstance(cur, bool):
            value = str(value).lower() in ("1", "true", "yes")
        else:
            value = type(cur)(value)
    setattr(sec, key, value)


def load_config(path: Optional[str] = None, environ: Optional[Mapping[str, str]] = None,
                overrides: Optional[Mapping[str, Any]] = None) -> Config:
    cfg = Config()
    if path:
        with open(path) as f:
            doc = yaml.safe_load(f) or {}
        for section, vals in doc.items():
            if section == "seed":
                cfg.seed = int(vals)
                continue
            for k, v in (vals or {}).items():
                _apply(cfg, section, k, v)
    env = os.environ if environ is None else environ
    for key, (section, fld, typ) in ENV_MAP.items():
        if key in env and env[key] != "":
            _apply(cfg, section, fld, typ(env[key]))
    for dotted, v in (overrides or {}).items():
        section, k = dotted.split(".", 1)
        _apply(cfg, section, k, v)
    return cfg
