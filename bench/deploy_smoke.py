"""Whole-stack deployment smoke on one node, driven by the operator (SURVEY.md §3.4 deployment
order, §1 L0): a FraudDetection CR -> LocalOperator -> kafka-lite (3 listeners), user-task
model, KIE server, notifier, the GPU engine (torchrun, 1 rank per GPU) and the producer as
supervised processes.  After ``--seconds`` it scrapes the engine's and KIE's Prometheus
endpoints and prints one JSON line: rows scored on the GPU, fraud / standard processes
started, notifications and replies, service restarts.  Exit 1 if a service crash-looped or
nothing flowed end to end.

    python bench/deploy_smoke.py --seconds 40 [--gpus 1] [--model mlp] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import random
import sys
import time
import urllib.request
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _scrape(url: str) -> dict:
    try:
        text = urllib.request.urlopen(url, timeout=2).read().decode()
    except Exception:
        return {}
    out = {}
    for line in text.splitlines():
        if line.startswith("#") or not line.strip():
            continue
        name, _, val = line.rpartition(" ")
        try:
            out[name] = out.get(name, 0.0) + float(val)
        except ValueError:
            pass
    return out


def _sum(metrics: dict, prefix: str) -> float:
    return sum(v for k, v in metrics.items() if k.split("{")[0] == prefix)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=40.0)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--model", default="mlp", choices=["mlp", "lr", "gbdt"])
    ap.add_argument("--count", type=int, default=2_000_000, help="transactions the producer job publishes")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    from ccfd_demo_summit_amd.operator import LocalOperator, parse
    cr = {"apiVersion": "ccfd.amd.com/v1alpha1", "kind": "FraudDetection", "metadata": {"name": "smoke"},
          "spec": {"kafka": {"brokers": 3, "partitions": 4},
                   "engine": {"nodes": 1, "gpusPerNode": a.gpus, "model": a.model},
                   "seldon": {"deploy": False}, "usertask": {"replicas": 1}, "kie": {"replicas": 1},
                   "notifier": {"replicas": 1}, "producer": {"format": "txb1", "count": a.count},
                   "monitoring": {"deploy": False}}}
    spec = parse(cr)
    off = random.randint(1000, 20000)
    op = LocalOperator(spec, workdir=str(ROOT), grace_s=10, log=lambda m: print(m, flush=True), port_offset=off)
    t0 = time.time()
    status = {}
    try:
        while time.time() - t0 < a.seconds:
            status = op.reconcile()
            time.sleep(1.0)
        eng = _scrape(f"http://127.0.0.1:{8091 + off}/prometheus")
        kie = _scrape(f"http://127.0.0.1:{8090 + off}/rest/metrics")
    finally:
        op.shutdown()
    rows = _sum(eng, "ccfd_gpu_rows_total") or _sum(eng, "ccfd_gpu_rows")
    # KIE outcome histograms (README.md:532-537): how many fraud processes ended which way
    outcomes = {k.split("{")[0][:-len("_count")]: v for k, v in kie.items()
                if k.split("{")[0].endswith("_count") and k.startswith("fraud_")}
    out = {"seconds": round(time.time() - t0, 1), "model": a.model, "gpus": a.gpus,
           "gpu_rows_scored": rows, "engine_metrics": len(eng), "kie_metrics": len(kie),
           "kie_fraud_outcomes": outcomes,
           "transaction_incoming": _sum(eng, "transaction_incoming_total"),
           "transaction_outgoing": {k: v for k, v in eng.items() if k.startswith("transaction_outgoing_total")},
           "notifications": _sum(eng, "notifications_outgoing_total"),
           "responses": _sum(eng, "notifications_incoming_total"),
           "restarts": {k: v["restarts"] for k, v in status.items()},
           "services": {k: v["ready"] for k, v in status.items()},
           "healthy": {k: v["healthy"] for k, v in status.items() if "healthy" in v}}
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        Path(a.out).write_text(line + "\n")
    crash_loop = any(v["restarts"] > 1 and k != "producer" for k, v in status.items())
    return 1 if crash_loop or rows <= 0 else 0


if __name__ == "__main__":
    sys.exit(main())
