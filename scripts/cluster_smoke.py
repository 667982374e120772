"""Multi-process deployment smoke test: every service as its own process, talking Kafka
protocol and HTTP on 127.0.0.1, like the reference's pods:

  kafka-lite  <-  producer (TXB1)           KIE server (REST, fraud BP, notifications)
      |                                          ^            |
      v                                          | batch start|  ccd-customer-outgoing
  engine (GPU: native Kafka consumer -> rings -> kernels -> router)    v
      ^                                                  notifier -> ccd-customer-response
      +-------------- responses -> KIE signal ------------------------+

Checks after ``--seconds``: the engine's ``transaction_incoming_total`` equals what the
producer sent, fraud instances were started in KIE, notifications went out and responses
were signalled.  Every child runs under its own process group and is killed by PID.

    python scripts/cluster_smoke.py --seconds 20
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time
from pathlib import Path

import requests

ROOT = Path(__file__).resolve().parents[1]


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def scrape(url: str) -> dict:
    out = {}
    for line in requests.get(url, timeout=5).text.splitlines():
        if line and not line.startswith("#"):
            k, _, v = line.rpartition(" ")
            try:
                out[k] = float(v)
            except ValueError:
                pass
    return out


def wait_http(url: str, timeout: float = 120.0) -> None:
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            if requests.get(url, timeout=1).status_code < 500:
                return
        except requests.RequestException:
            time.sleep(0.2)
    raise TimeoutError(url)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=15.0)
    ap.add_argument("--count", type=int, default=2_000_000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)

    kport, kie_port, notif_port, eng_port = free_port(), free_port(), free_port(), free_port()
    env = dict(os.environ, BROKER_URL=f"127.0.0.1:{kport}", KIE_SERVER_URL=f"http://127.0.0.1:{kie_port}",
               PYTHONPATH=str(ROOT), CCFD_MODEL="mlp", CCFD_INPUT_MODE="zerocopy")
    logs = ROOT / "gpurun_out" / "cluster"
    logs.mkdir(parents=True, exist_ok=True)
    procs = {}

    def start(name, *args):
        f = open(logs / f"{name}.log", "w")
        procs[name] = subprocess.Popen([sys.executable, "-m", "ccfd_demo_summit_amd.launch", *args], env=env,
                                       stdout=f, stderr=subprocess.STDOUT, start_new_session=True)

    result = {"ok": False}
    try:
        start("kafka", "kafka-lite", "--host", "127.0.0.1", "--port", str(kport))
        t0 = time.time()
        while True:                                       # broker accepting connections
            try:
                socket.create_connection(("127.0.0.1", kport), timeout=1).close()
                break
            except OSError:
                if time.time() - t0 > 180:
                    raise
                time.sleep(0.2)
        start("kie", "kie", "--host", "127.0.0.1", "--port", str(kie_port))
        start("notifier", "notifier", "--host", "127.0.0.1", "--port", str(notif_port))
        wait_http(f"http://127.0.0.1:{kie_port}/rest/metrics")
        start("engine", "engine", "--host", "127.0.0.1", "--port", str(eng_port))
        wait_http(f"http://127.0.0.1:{eng_port}/prometheus", timeout=300)
        start("producer", "producer", "--fmt", "txb1", "--batch", "4096", "--count", str(a.count))
        t0 = time.time()
        sent = None                                       # producer rounds up to whole batches
        got = 0.0
        while time.time() - t0 < a.seconds + 60:
            if sent is None and procs["producer"].poll() is not None:
                for line in (logs / "producer.log").read_text().splitlines():
                    if line.startswith("{") and '"produced"' in line:
                        sent = int(json.loads(line)["produced"])
                if sent is None:
                    raise RuntimeError("producer exited without a report")
            m = scrape(f"http://127.0.0.1:{eng_port}/prometheus")
            got = m.get("transaction_incoming_total", 0.0)
            if sent is not None and got >= sent:
                break
            if procs["engine"].poll() is not None:
                raise RuntimeError("engine exited")
            time.sleep(0.5)
        dt = time.time() - t0
        time.sleep(3.0)                                   # notification/response loop
        em = scrape(f"http://127.0.0.1:{eng_port}/prometheus")
        km = scrape(f"http://127.0.0.1:{kie_port}/rest/metrics")
        result = {
            "ok": (sent is not None and em.get("transaction_incoming_total", 0.0) == sent
                   and em.get('transaction_outgoing_total{type="fraud"}', 0.0) > 0
                   and em.get("notifications_outgoing_total", 0.0) > 0
                   and km.get("fraud_approved_amount_count", 0.0) + km.get("fraud_rejected_amount_count", 0.0) > 0),
            "sent": sent, "scored": em.get("transaction_incoming_total"), "seconds": round(dt, 2),
            "fraud_routed": em.get('transaction_outgoing_total{type="fraud"}'),
            "notifications_outgoing": em.get("notifications_outgoing_total"),
            "kie_investigations": km.get("fraud_investigation_amount_count"),
            "kie_approved": km.get("fraud_approved_amount_count"),
            "kie_rejected": km.get("fraud_rejected_amount_count"),
        }
    finally:
        for name, p in procs.items():
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)      # the child's own process group
                except ProcessLookupError:
                    pass
        for p in procs.values():
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
    print(json.dumps(result), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(result) + "\n")
    return 0 if result.get("ok") else 1


if __name__ == "__main__":
    sys.exit(main())
