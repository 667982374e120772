"""Grafana dashboard generator.

The reference ships six hand-made dashboards (deploy/grafana/*.json) that query the
metric names kept by this framework.  Rather than vendoring them, this module GENERATES
equivalent dashboards from the metric registry -- the same PromQL the reference panels use
(e.g. ``round(sum(irate(seldon_api_engine_server_requests_seconds_count[2m])),0.001)``,
SeldonCore.json:119; ``histogram_quantile`` over ``seldon_api_engine_client_requests_seconds_bucket``,
SeldonCore.json:499-531) -- plus a GPU engine dashboard for the ``ccfd_gpu_*`` series.

    python -m ccfd_demo_summit_amd.metrics.dashboards deploy/grafana
"""
from __future__ import annotations

import itertools
import json
import os
import sys
from typing import Dict, List

from ..contracts import metric_names as M

_ids = itertools.count(1)


def _panel(title: str, exprs: List[str], kind: str = "graph", unit: str = "short", w: int = 12, h: int = 8,
           legend: List[str] = None) -> Dict:
    targets = [{"expr": e, "refId": chr(65 + i), "legendFormat": (legend or [""] * len(exprs))[i]}
               for i, e in enumerate(exprs)]
    p = {"id": next(_ids), "title": title, "type": kind, "datasource": "Prometheus", "targets": targets,
         "gridPos": {"w": w, "h": h, "x": 0, "y": 0}}
    if kind == "graph":
        p["yaxes"] = [{"format": unit, "show": True}, {"format": "short", "show": False}]
        p["lines"] = True
    elif kind == "singlestat":
        p["format"] = unit
        p["valueName"] = "current"
    elif kind == "heatmap":
        p["dataFormat"] = "tsbuckets"
    return p


def _layout(panels: List[Dict]) -> List[Dict]:
    x = y = 0
    for p in panels:
        w, h = p["gridPos"]["w"], p["gridPos"]["h"]
        if x + w > 24:
            x, y = 0, y + h
        p["gridPos"].update(x=x, y=y)
        x += w
    return panels


def _dashboard(title: str, uid: str, panels: List[Dict], refresh: str = "10s") -> Dict:
    return {"title": title, "uid": uid, "schemaVersion": 16, "version": 1, "editable": True,
            "refresh": refresh, "time": {"from": "now-30m", "to": "now"}, "timezone": "browser",
            "tags": ["ccfd", "mi355x"], "panels": _layout(panels)}


def router_dashboard() -> Dict:
    return _dashboard("Router", "ccfd-router", [
        _panel("Incoming transactions /s", [f"sum(rate({M.TRANSACTION_INCOMING}_total[1m]))"], unit="ops"),
        _panel("Outgoing transactions /s by process", [f"sum by (type) (rate({M.TRANSACTION_OUTGOING}_total[1m]))"],
               unit="ops", legend=["{{type}}"]),
        _panel("Customers notified", [f"{M.NOTIFICATIONS_OUTGOING}_total"]),
        _panel("Customer responses", [f"sum by (response) ({M.NOTIFICATIONS_INCOMING}_total)"], legend=["{{response}}"]),
    ])


def kie_dashboard() -> Dict:
    panels = []
    for name, title in ((M.FRAUD_REJECTED_AMOUNT, "Rejected by customer"),
                        (M.FRAUD_APPROVED_AMOUNT, "Approved by customer"),
                        (M.FRAUD_APPROVED_LOW_AMOUNT, "Approved (low amount, no reply)"),
                        (M.FRAUD_INVESTIGATION_AMOUNT, "Sent to investigation")):
        panels.append(_panel(f"{title}: count", [f"sum({name}_count)"], kind="singlestat", w=6, h=4))
        panels.append(_panel(f"{title}: amount distribution", [f"sum by (le) (increase({name}_bucket[5m]))"],
                             kind="heatmap", w=12))
        panels.append(_panel(f"{title}: total amount", [f"sum({name}_sum)"], kind="singlestat", unit="currencyUSD", w=6, h=4))
    return _dashboard("KIE fraud process", "ccfd-kie", panels)


def model_dashboard() -> Dict:
    return _dashboard("Model prediction", "ccfd-model", [
        _panel("proba_1 (last request)", ['proba_1{instance=~".*:8000"}'], unit="percentunit"),
        _panel("Amount (last request)", ['Amount{instance=~".*:8000"}'], unit="currencyUSD"),
        _panel("V17", ['V17{instance=~".*:8000"}']),
        _panel("V10", ['V10{instance=~".*:8000"}']),
    ])


def seldon_dashboard() -> Dict:
    s, c = M.SELDON_SERVER_REQUESTS, M.SELDON_CLIENT_REQUESTS
    qs = [f'histogram_quantile({q}, sum(rate({c}_bucket{{status="200"}}[1m])) by (le))' for q in
          (0.5, 0.75, 0.9, 0.95, 0.99)]
    return _dashboard("Seldon core", "ccfd-seldon", [
        _panel("Global request rate", [f"round(sum(irate({s}_count[2m])),0.001)"], kind="singlestat", unit="ops", w=6, h=4),
        _panel("Success ratio", [f'sum(rate({s}_count{{status!~"5.*"}}[1m])) / sum(rate({s}_count[1m]))'],
               kind="singlestat", unit="percentunit", w=6, h=4),
        _panel("Latency quantiles", qs, unit="s", w=24, legend=["p50", "p75", "p90", "p95", "p99"]),
        _panel("Requests by status", [f"sum by (status) (rate({s}_count[1m]))"], unit="ops", legend=["{{status}}"]),
    ])


def kafka_dashboard() -> Dict:
    """The broker series of deploy/grafana/Kafka.json:119-1093, served by kafka-lite's
    /metrics (ingest/kafka_lite.py BrokerMetrics) or a Strimzi JMX exporter."""
    k = 'strimzi_io_kind="Kafka"'
    return _dashboard("Kafka", "ccfd-kafka", [
        _panel("Brokers online", [f"count(kafka_server_replicamanager_leadercount)"], kind="singlestat", w=6, h=4),
        _panel("Partitions", ["sum(kafka_server_replicamanager_partitioncount)"], kind="singlestat", w=6, h=4),
        _panel("Under-replicated partitions", ["sum(kafka_server_replicamanager_underreplicatedpartitions)"],
               kind="singlestat", w=6, h=4),
        _panel("Offline partitions", ["sum(kafka_controller_kafkacontroller_offlinepartitionscount)"],
               kind="singlestat", w=6, h=4),
        _panel("Incoming messages /s", [f"sum without(instance)(rate(kafka_server_brokertopicmetrics_messagesin_total{{{k}}}[5m]))"],
               unit="ops", legend=["{{topic}}"]),
        _panel("Incoming bytes /s", [f"sum without(instance)(rate(kafka_server_brokertopicmetrics_bytesin_total{{{k}}}[5m]))"],
               unit="Bps", legend=["{{topic}}"]),
        _panel("Outgoing bytes /s", [f"sum without(instance)(rate(kafka_server_brokertopicmetrics_bytesout_total{{{k}}}[5m]))"],
               unit="Bps", legend=["{{topic}}"]),
        _panel("Failed produce / fetch", ['sum(kafka_server_brokertopicmetrics_failedproducerequests_total{topic!=""})',
                                          'sum(kafka_server_brokertopicmetrics_failedfetchrequests_total{topic!=""})'],
               legend=["produce", "fetch"]),
        # broker process resources (Kafka.json:416,499,582; ingest/kafka_lite.py ProcessResourceCollector)
        _panel("Broker CPU", [f"rate(process_cpu_seconds_total{{{k}}}[2m])"], unit="percentunit", w=8),
        _panel("Broker memory", [f"sum without(area)(jvm_memory_bytes_used{{{k}}})"], unit="bytes", w=8),
        _panel("Time in GC", [f"sum without(gc)(rate(jvm_gc_collection_seconds_sum{{{k}}}[5m]))"],
               unit="percentunit", w=8),
    ])


def training_dashboard() -> Dict:
    """Replaces deploy/grafana/SparkMetrics.json (Spark workbench) with the trainer's series."""
    return _dashboard("Training", "ccfd-train", [
        _panel("Alive training workers (DDP ranks)", ["ccfd_train_workers"], kind="singlestat", w=6, h=4),
        _panel("Device memory", ["ccfd_train_device_memory_bytes"], unit="bytes", w=18, h=4),
        _panel("Loss", ["ccfd_train_loss"], legend=["{{model}}"]),
        _panel("Samples /s", ["ccfd_train_samples_per_second"], unit="ops", legend=["{{model}}"]),
        # the reference workbench board's series (SparkMetrics.json:119-352; exporter.TrainMetrics)
        _panel("Alive workers (Spark name)", ["metrics_master_aliveworkers_value"], kind="singlestat", w=6, h=4),
        _panel("Memory used / max", ["sum(jvm_memory_bytes_used) / sum(jvm_memory_bytes_max) * 100"],
               kind="singlestat", w=6, h=4),
        _panel("Host memory (heap analogue)", ['jvm_memory_bytes_used{area="heap", job="Spark Metrics"}'],
               unit="bytes", w=6, h=4),
        _panel("Live device tensors (eden analogue)", ["metrics_jvm_pools_ps_eden_space_used_value"], unit="bytes",
               w=6, h=4),
    ])


def gpu_dashboard() -> Dict:
    return _dashboard("MI355X scoring engine", "ccfd-gpu", [
        _panel("Rows scored /s (whole node)", [f"sum(rate({M.GPU_ROWS}_total[30s]))"], unit="ops"),
        _panel("Rows scored /s per rank", [f"sum by (rank) (rate({M.GPU_ROWS}_total[30s]))"], unit="ops",
               legend=["rank {{rank}}"]),
        _panel("Micro-batch latency", [f'ccfd_gpu_batch_latency_quantile_seconds{{quantile="{q}"}}'
                                       for q in ("0.5", "0.9", "0.99")], unit="s", legend=["p50", "p90", "p99"]),
        _panel("Global fraud-route rate (RCCL all-reduced)", [M.GPU_GLOBAL_FRAUD_RATE], unit="percentunit"),
        _panel("Amount distribution by route (device histogram)",
               [f"sum by (le, type) (rate({M.GPU_AMOUNT}_bucket[1m]))"], kind="heatmap", w=24),
        _panel("Kernel execution per micro-batch (device clock, K7)", [M.GPU_PREFIX + "kernel_exec_mean_us"],
               unit="µs"),
        _panel("Model version (hot swaps)", [M.GPU_PREFIX + "model_version"], kind="singlestat"),
    ])


def all_dashboards() -> Dict[str, Dict]:
    return {"Router.json": router_dashboard(), "KIE.json": kie_dashboard(),
            "ModelPrediction.json": model_dashboard(), "SeldonCore.json": seldon_dashboard(),
            "GpuEngine.json": gpu_dashboard(), "Kafka.json": kafka_dashboard(),
            "Training.json": training_dashboard()}


def write_all(out_dir: str) -> List[str]:
    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for name, d in all_dashboards().items():
        p = os.path.join(out_dir, name)
        with open(p, "w") as f:
            json.dump(d, f, indent=2)
        paths.append(p)
    return paths


if __name__ == "__main__":
    for p in write_all(sys.argv[1] if len(sys.argv) > 1 else "deploy/grafana"):
        print(p)
