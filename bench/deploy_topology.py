#!/usr/bin/env python3
"""Config 5 in the DEPLOYED topology: every service its own OS process, talking over the
network the way the reference's pods do (README.md:543-569; deploy/router.yaml:55-70;
deploy/frauddetection_cr.yaml:73-77):

    producer x P  --(Kafka wire: one JSON transaction per message, or TXB1)-->
    kafka-lite (3 broker listeners, one process)  -->
    engine ranks under torchrun (partitions p % W == rank; native consumers; persistent
    kernel; RCCL X1/X2/X3)  --(HTTP, async hand-off)-->  KIE (fraud BP, one process)
    KIE --(ccd-customer-outgoing)--> notifier process --(ccd-customer-response)--> engine
    rank 0 --(HTTP signal)--> KIE

Throughput and latency are read from the services' own Prometheus endpoints (router
``transaction_incoming_total`` on 8091 + r, the engine's X3-merged latency quantiles, the
model endpoint's ``seldon_api_engine_*`` histograms), sampled every ``--sample-s`` over the
``--seconds`` window; after the producers stop the harness waits for the consumer-group lag
to reach 0 and the hand-off to drain, then checks:

* ``transaction_incoming_total`` (all ranks) == transactions produced (all producers);
* every partition of the topic consumed by exactly one rank (the ranks' partition lists);
* KIE started one fraud process per fraud-routed transaction (router counters, all ranks)
  and saw no duplicate start it had to drop (exactly once);
* every selector of the reference's six Grafana dashboards matches a scraped series
  (metrics/promql.py; tests/fixtures/reference_dashboard_exprs.json).

The JSON line states ``topology: "shared"`` (vs bench/e2e.py's per-rank stacks).

    python bench/deploy_topology.py --seconds 60 --producers 3 --fmt json         # 1 GPU
    python bench/deploy_topology.py --ranks 4 --rehearsal --seconds 20             # 4 ranks, 1 GPU, gloo
    python bench/deploy_topology.py --standard-mode process --kie-shards 4 --rate 1.2e6 \
        --kie-outage-at 25 --kie-kill-shard 1                                      # reference semantics
    python bench/deploy_topology.py --standard-mode process --kie-shards 4 --rate 1.0e6 \
        --kie-outage-at 15 --kie-outage-s 12 --engine-kill-at 20 --engine-down-s 3   # idempotency drill
    python bench/deploy_topology.py --kafka-replicated --kafka-controllers 3 --rate 1.2e6 \
        --controller-kill-at 25                                                    # controller fail-over

``--engine-kill-at`` SIGKILLs the engine (torchrun and every rank) and restarts it: it resumes
from the committed offsets, so rows scored since the last commit are scored again.  Its
counters restart at 0, so the harness adds the killed incarnation's last scrape; the exact
check is then at KIE: standard + fraud processes == transactions produced (every replayed
start recognised as a duplicate, none started twice).  ``--kafka-controllers 3`` runs the
replicated controller quorum (ingest/controller_quorum.py); ``--controller-kill-at`` SIGKILLs
its ACTIVE member and reports when a standby took over and when the engine's offset commits
resumed.

KIE runs as ``--kie-shards`` processes (process/sharding.py): the hand-off routes starts by
transaction-id hash and signals by shard-encoded instance id; every shard keeps its own
journal and the engine one hand-off queue + DLQ per shard.  The KIE checks sum the shards'
``/rest/stats``.  ``--count`` runs a fixed input (each producer a fixed number of
transactions) so two runs with the same seed can be compared outcome for outcome
(``--settle``: wait until no fraud process waits for its customer before reading them).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import signal
import socket
import subprocess
import sys
import time
import urllib.request
from pathlib import Path
from typing import Dict, List, Optional

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
PY = sys.executable


def _port_base() -> int:
    """Service ports come from below the kernel's ephemeral range: a port handed out here and
    bound later (a restarted broker re-binds its own) must not meanwhile become the local port
    of some outgoing connection (a restarted broker's metrics port was, once: EADDRINUSE)."""
    try:
        lo, _hi = (int(x) for x in Path("/proc/sys/net/ipv4/ip_local_port_range").read_text().split())
    except (OSError, ValueError):
        lo = 32768
    top = max(2048, min(lo, 65535) - 1024)             # leave room below the ephemeral range
    bottom = max(1024, top - 12000)
    return bottom + (os.getpid() * 37) % max(1, top - bottom - 2000)


_PORT_CURSOR = [_port_base()]


def free_ports(n: int, contiguous: int = 1) -> List[int]:
    """n base ports, each followed by contiguous-1 free ports; never hands out a port twice
    in this process (the services bind them later)."""
    out = []
    p = _PORT_CURSOR[0]
    while len(out) < n:
        ok = True
        for k in range(contiguous):
            s = socket.socket()
            try:
                s.bind(("127.0.0.1", p + k))
            except OSError:
                ok = False
            finally:
                s.close()
            if not ok:
                break
        if ok:
            out.append(p)
            p += contiguous + 1
        else:
            p += 1
    _PORT_CURSOR[0] = p
    return out


def cgroup_cpu() -> Dict:
    """This cgroup's CPU quota and throttling counters (cgroup v2): a deployment sharing a CPU
    quota stalls in whole scheduler periods once the quota is spent."""
    out: Dict = {}
    v1 = Path("/sys/fs/cgroup/cpu")
    for f in ("cpu.max", "cpu.stat"):
        try:
            txt = Path("/sys/fs/cgroup", f).read_text()
        except OSError:
            continue
        if f == "cpu.max":
            out["cpu.max"] = txt.strip()
        else:
            for ln in txt.splitlines():
                k, _, v = ln.partition(" ")
                if k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                    out[k] = int(v)
    if not out and v1.is_dir():                    # cgroup v1: the same counters, other names
        try:
            out["cpu.max"] = (f"{(v1 / 'cpu.cfs_quota_us').read_text().strip()} "
                              f"{(v1 / 'cpu.cfs_period_us').read_text().strip()}")
            for ln in (v1 / "cpu.stat").read_text().splitlines():
                k, _, v = ln.partition(" ")
                if k in ("nr_periods", "nr_throttled"):
                    out[k] = int(v)
                elif k == "throttled_time":
                    out["throttled_usec"] = int(v) // 1000
        except OSError:
            pass
    return out


def wait_port(port: int, timeout: float = 120.0) -> None:
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
            return
        except OSError:
            time.sleep(0.2)
    raise TimeoutError(f"port {port} did not open")


def active_controller(ports: List[int], timeout: float = 60.0) -> int:
    """The port of the controller member that is active (a single controller is always)."""
    t_end = time.time() + timeout
    while time.time() < t_end:
        for p in ports:
            try:
                q = json.loads(http_text(f"http://127.0.0.1:{p}/quorum", timeout=0.5))
            except Exception:                           # noqa: BLE001 -- that member is down
                continue
            if q.get("active"):
                return p
        time.sleep(0.05)
    raise TimeoutError(f"no active controller among {ports}")


def http_text(url: str, timeout: float = 5.0) -> str:
    with urllib.request.urlopen(url, timeout=timeout) as r:
        return r.read().decode()


def metric_sum(text: str, name: str, labels: Optional[Dict[str, str]] = None) -> float:
    from prometheus_client.parser import text_string_to_metric_families
    tot = 0.0
    for fam in text_string_to_metric_families(text):
        for s in fam.samples:
            if s.name == name and all(s.labels.get(k) == v for k, v in (labels or {}).items()):
                tot += s.value
    return tot


def hist_quantile_le(text: str, name: str, q: float, labels: Optional[Dict[str, str]] = None) -> Optional[float]:
    """histogram_quantile over Prometheus ``le`` buckets (linear inside a bucket)."""
    from prometheus_client.parser import text_string_to_metric_families
    b: Dict[float, float] = {}
    for fam in text_string_to_metric_families(text):
        for s in fam.samples:
            if s.name == name + "_bucket" and all(s.labels.get(k) == v for k, v in (labels or {}).items()):
                le = float("inf") if s.labels["le"] == "+Inf" else float(s.labels["le"])
                b[le] = b.get(le, 0.0) + s.value
    if not b:
        return None
    les = sorted(b)
    tot = b[les[-1]]
    if tot <= 0:
        return None
    target = q * tot
    prev_le, prev_c = 0.0, 0.0
    for le in les:
        c = b[le]
        if c >= target:
            if le == float("inf"):
                return prev_le
            return prev_le + (le - prev_le) * (target - prev_c) / max(c - prev_c, 1e-12)
        prev_le, prev_c = le, c
    return les[-2] if len(les) > 1 else None


class Proc:
    def __init__(self, name: str, cmd: List[str], env: Dict[str, str], log_dir: Path):
        self.name = name
        self.log = open(log_dir / f"{name}.log", "w")
        self.p = subprocess.Popen(cmd, env=env, stdout=self.log, stderr=subprocess.STDOUT, cwd=str(ROOT),
                                  start_new_session=True)
        self.path = log_dir / f"{name}.log"

    def alive(self) -> bool:
        return self.p.poll() is None

    def stop(self, sig=signal.SIGTERM, wait: float = 10.0) -> Optional[int]:
        if self.p.poll() is None:
            try:
                os.killpg(self.p.pid, sig)            # the process group this harness started
            except ProcessLookupError:
                pass
            try:
                self.p.wait(wait)
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(self.p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                self.p.wait(5)
        self.log.close()
        return self.p.returncode

    def cpu_s(self) -> Optional[float]:
        """CPU seconds of the process and its children so far (torchrun's ranks are children)."""
        try:
            import psutil
            root = psutil.Process(self.p.pid)
            tot = 0.0
            for q in [root] + root.children(recursive=True):
                try:
                    t = q.cpu_times()
                    tot += t.user + t.system
                except psutil.Error:
                    pass
            return round(tot, 1)
        except Exception:                              # noqa: BLE001 -- diagnostics only
            return None

    def text(self) -> str:
        try:
            return self.path.read_text()
        except OSError:
            return ""


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--seconds", type=float, default=60.0, help="producer window (sustained rate)")
    ap.add_argument("--ranks", type=int, default=1, help="engine ranks (torchrun --nproc-per-node)")
    ap.add_argument("--rehearsal", action="store_true",
                    help="several ranks on one GPU: gloo collectives + CCFD_DEVICE_MODULO (functional check)")
    ap.add_argument("--rehearsal-hw-queues", type=int, default=2,
                    help="--rehearsal with several ranks on one GPU: GPU_MAX_HW_QUEUES per rank (0 = inherit)")
    ap.add_argument("--producers", type=int, default=3)
    ap.add_argument("--rate", type=float, default=0.0, help="total produce rate tx/s (0 = open loop, max)")
    ap.add_argument("--fmt", default="json", choices=["json", "txb1"])
    ap.add_argument("--batch", type=int, default=None,
                    help="messages (json, default 1024) / rows (txb1, default 4096) per produce request")
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--kafka-nodes", type=int, default=3)
    ap.add_argument("--retention-batches", type=int, default=500,
                    help="kafka-lite batches kept per partition (~2 MB each): a consumer that falls this "
                         "far behind loses data and the incoming == produced check fails")
    ap.add_argument("--model", default="mlp", choices=["mlp", "lr", "gbdt"])
    ap.add_argument("--ingest-threads", type=int, default=0, help="native consumers per rank (0 = partitions / ranks)")
    ap.add_argument("--notification-timeout-s", type=float, default=30.0)
    ap.add_argument("--kie-shards", type=int, default=1, help="KIE shard processes (kie.shards)")
    ap.add_argument("--kie-outage-at", type=float, default=0.0,
                    help="SIGKILL a KIE shard process this many seconds into the window (0 = never) ...")
    ap.add_argument("--kie-outage-s", type=float, default=5.0,
                    help="... and restart it from its journal this long after")
    ap.add_argument("--kie-kill-shard", type=int, default=0, help="which KIE shard --kie-outage-at kills")
    ap.add_argument("--notifier-kill-at", type=float, default=0.0,
                    help="SIGKILL the notifier this many seconds into the window (0 = never) ...")
    ap.add_argument("--notifier-down-s", type=float, default=3.0, help="... and restart it this long after")
    ap.add_argument("--count", type=int, default=0,
                    help="transactions per producer (fixed input; 0 = open loop for --seconds)")
    ap.add_argument("--settle", action="store_true",
                    help="after the drain, wait until no fraud process waits for its customer (outcomes final)")
    ap.add_argument("--notifier-seed", type=int, default=0, help="the simulated customers' seed")
    ap.add_argument("--compare-to", default=None,
                    help="a previous run's --out JSON over the same transactions: outcomes must be equal")
    ap.add_argument("--kafka-kill-at", type=float, default=0.0,
                    help="SIGKILL kafka-lite this many seconds into the window (0 = never) ...")
    ap.add_argument("--kafka-down-s", type=float, default=2.0,
                    help="... and restart it from its data directory this long after")
    ap.add_argument("--fsync", default="interval", choices=["always", "interval", "never"],
                    help="kafka-lite durability flush policy (its logs are always on disk here)")
    ap.add_argument("--kafka-replicated", action="store_true",
                    help="replicated kafka-lite: --kafka-nodes broker PROCESSES (each its own durable log, "
                         "replication factor 3) + the controller (ingest/kafka_controller.py); producers "
                         "use acks=all; --kafka-kill-at then SIGKILLs broker --kafka-kill-node")
    ap.add_argument("--kafka-kill-node", type=int, default=2, help="replicated: the broker node id to kill")
    ap.add_argument("--kafka-controllers", type=int, default=1,
                    help="replicated: controller quorum members (ingest/controller_quorum.py; 1 = one controller)")
    ap.add_argument("--controller-kill-at", type=float, default=0.0,
                    help="replicated: SIGKILL the ACTIVE controller member this many s into the window")
    ap.add_argument("--controller-down-s", type=float, default=5.0, help="... and restart it this long after")
    ap.add_argument("--engine-kill-at", type=float, default=0.0,
                    help="SIGKILL the engine (torchrun + ranks) this many s into the window; it restarts from "
                         "the committed offsets --engine-down-s later")
    ap.add_argument("--engine-down-s", type=float, default=3.0)
    ap.add_argument("--kafka-rf", type=int, default=3,
                    help="replicated: replication factor (1 = scale-out over the brokers, no copies)")
    ap.add_argument("--producer-acks", type=int, default=None, choices=[1, -1],
                    help="producers' acks (default: -1 with --kafka-replicated, else 1)")
    ap.add_argument("--producer-max-in-flight", type=int, default=None,
                    help="producers' pipelined requests (default: 5 with --kafka-replicated, else 1)")
    ap.add_argument("--kafka-memory", action="store_true",
                    help="kafka-lite without --data-dir (round 3's in-memory broker): the A/B of durability")
    ap.add_argument("--standard-mode", default="count", choices=["count", "process"],
                    help="process: a standard process per standard-routed transaction (README.md:552)")
    ap.add_argument("--serving", default="native", choices=["native", "python"],
                    help="engine scoring loop: the C++ serving thread, or the round-3 Python thread")
    ap.add_argument("--trace", action="store_true",
                    help="engine ranks record their stage trace + scoring-loop timeline "
                         "(CCFD_SERVICE_TRACE) and the tail is attributed (bench/tail_attribution.py)")
    ap.add_argument("--journal-dir", default=None,
                    help="parent directory of the KIE journal / hand-off DLQ (default: $TMPDIR, the same "
                         "disk as kafka-lite's data; /dev/shm separates it from the broker's writeback)")
    ap.add_argument("--sample-s", type=float, default=5.0)
    ap.add_argument("--drain-timeout-s", type=float, default=120.0)
    ap.add_argument("--log-dir", default="gpurun_out/deploy_topology")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    if a.batch is None:
        a.batch = 1024 if a.fmt == "json" else 4096
    log_dir = ROOT / a.log_dir
    log_dir.mkdir(parents=True, exist_ok=True)

    kafka_port, = free_ports(1, a.kafka_nodes)
    metrics_port, notif_port, master_port, master_port2 = free_ports(4)
    NC = max(1, a.kafka_controllers)
    ctl_ports = free_ports(NC)
    ctl_port = ctl_ports[0]
    kmetrics = [metrics_port] + (free_ports(a.kafka_nodes - 1) if a.kafka_replicated else [])
    acks = a.producer_acks if a.producer_acks is not None else (-1 if a.kafka_replicated else 1)
    inflight = a.producer_max_in_flight if a.producer_max_in_flight is not None else (5 if a.kafka_replicated else 1)
    kie_port, = free_ports(1, max(1, a.kie_shards))
    K = max(1, a.kie_shards)
    kie_ports = [kie_port + k for k in range(K)]
    router_base, = free_ports(1, a.ranks)
    model_base, = free_ports(1, a.ranks)
    brokers = ",".join(f"127.0.0.1:{kafka_port + i}" for i in range(a.kafka_nodes))
    env = dict(os.environ, PYTHONPATH=str(ROOT), BROKER_URL=brokers,
               KIE_SERVER_URL=",".join(f"http://127.0.0.1:{p}" for p in kie_ports), CCFD_KIE_SHARDS=str(K),
               CCFD_KAFKA_BACKEND="kafka", CCFD_KAFKA_PARTITIONS=str(a.partitions), CCFD_MODEL=a.model,
               HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1",
               PYTHONFAULTHANDLER="1")          # a native crash prints every thread's Python stack
    if a.model == "gbdt":
        env.setdefault("CCFD_WIRE", "auto")
    procs: List[Proc] = []
    out: Dict = {"metric": "end-to-end tx/s, deployed topology (separate processes)", "topology": "shared",
                 "n_gpus": 1 if a.rehearsal else a.ranks, "ranks": a.ranks, "rehearsal": a.rehearsal,
                 "fmt": a.fmt, "producers": a.producers, "producer_batch": a.batch, "partitions": a.partitions, "kafka_nodes": a.kafka_nodes,
                 "model": a.model, "kie_shards": K, "kafka_replicated": a.kafka_replicated,
                 "producer_acks": acks, "producer_max_in_flight": inflight,
                 "kafka_rf": a.kafka_rf if a.kafka_replicated else None}
    import tempfile
    kdir = tempfile.mkdtemp(prefix="ccfd-kafka-lite-")          # durable logs + committed offsets
    out["kafka_durable"] = {"fsync": a.fsync} if not a.kafka_memory else False
    try:
        L = "ccfd_demo_summit_amd.launch"
        kafka_cmd = [PY, "-m", "ccfd_demo_summit_amd.ingest.kafka_lite", "--host", "127.0.0.1",
                     "--port", str(kafka_port), "--nodes", str(a.kafka_nodes),
                     "--partitions", str(a.partitions), "--metrics-port", str(metrics_port),
                     "--retention-batches", str(a.retention_batches)] + \
            ([] if a.kafka_memory else ["--data-dir", kdir, "--fsync", a.fsync])
        broker_cmds = {}
        if a.kafka_replicated:
            # the controller + one broker process per node, each with its own durable log
            peers = ",".join(f"{k + 1}=http://127.0.0.1:{ctl_ports[k]}" for k in range(NC))
            ctl_cmds = [[PY, "-m", "ccfd_demo_summit_amd.ingest.kafka_controller", "--host", "127.0.0.1",
                         "--port", str(ctl_ports[k]), "--brokers", str(a.kafka_nodes), "--rf", str(a.kafka_rf),
                         "--data-dir", str(Path(kdir) / f"controller{k + 1}")]
                        + (["--member-id", str(k + 1), "--peers", peers] if NC > 1 else []) for k in range(NC)]
            for k in range(NC):
                procs.append(Proc(f"kafka-controller{k + 1}", ctl_cmds[k], env, log_dir))
            for k in range(NC):
                wait_port(ctl_ports[k], 60)
            ctl_port = active_controller(ctl_ports)
            out["kafka_controllers"] = NC
            for i in range(a.kafka_nodes):
                broker_cmds[i + 1] = [PY, "-m", "ccfd_demo_summit_amd.ingest.kafka_lite", "--host", "127.0.0.1",
                                      "--port", str(kafka_port + i), "--node-id", str(i + 1),
                                      "--controller", ",".join(f"http://127.0.0.1:{p_}" for p_ in ctl_ports),
                                      "--metrics-port", str(kmetrics[i]),
                                      "--retention-batches", str(a.retention_batches),
                                      "--data-dir", str(Path(kdir) / f"broker{i + 1}"), "--fsync", a.fsync]
                procs.append(Proc(f"kafka-broker{i + 1}", broker_cmds[i + 1], env, log_dir))
            for i in range(a.kafka_nodes):
                wait_port(kafka_port + i, 60)
            t_md = time.time()
            while time.time() - t_md < 30:
                md = json.loads(http_text(f"http://127.0.0.1:{ctl_port}/metadata"))
                if len(md["nodes"]) == a.kafka_nodes:
                    break
                time.sleep(0.2)
        else:
            procs.append(Proc("kafka-lite", kafka_cmd, env, log_dir))
            wait_port(kafka_port, 60)
        from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
        kb = KafkaBroker(brokers, connect_wait_s=30)
        for t, n in (("odh-demo", a.partitions), ("ccd-customer-outgoing", 4), ("ccd-customer-response", 4)):
            kb.create_topic(t, n)
        kie_env = dict(env)
        kie_env["CCFD_KIE_NOTIFICATION_TIMEOUT_S"] = str(a.notification_timeout_s)
        # the journal grows ~1 KB per fraud process: keep it out of the log directory
        import tempfile
        jdir = tempfile.mkdtemp(prefix="ccfd-kie-journal-", dir=a.journal_dir)
        journals = [Path(jdir) / f"kie-journal.shard{k}.jsonl" for k in range(K)]
        kie_cmds = [[PY, "-m", L, "kie", "--host", "127.0.0.1", "--port", str(kie_ports[k]), "--shard", str(k),
                     "--journal", str(journals[k])] for k in range(K)]
        for k in range(K):
            procs.append(Proc(f"kie{k}", kie_cmds[k], kie_env, log_dir))
        notif_env = dict(env, CCFD_NOTIFIER_SEED=str(a.notifier_seed))
        notif_cmd = [PY, "-m", L, "notifier", "--host", "127.0.0.1", "--port", str(notif_port)]
        procs.append(Proc("notifier", notif_cmd, notif_env, log_dir))
        for p_ in kie_ports:
            wait_port(p_, 60)
        eng_env = dict(env)
        eng_env["CCFD_INGEST_THREADS"] = str(a.ingest_threads or max(1, a.partitions // a.ranks))
        eng_env["ROUTER_STANDARD_MODE"] = a.standard_mode
        eng_env["CCFD_NATIVE_SERVE"] = "1" if a.serving == "native" else "0"
        if a.rehearsal and a.ranks > 1 and a.rehearsal_hw_queues > 0:
            # several ranks on ONE GPU: 2 hardware queues each (the persistent kernel's and one
            # for everything else).  With HIP's default 4, 4 ranks' 16 queues oversubscribe the
            # GPU's queue slots and the scheduler time-slices them -- ~10 ms stalls every ~85 ms,
            # arrival -> scored p99 8 ms; with 2, p99 45-49 us (profiles/r5/final/)
            eng_env["GPU_MAX_HW_QUEUES"] = str(a.rehearsal_hw_queues)
        out["serving"] = a.serving
        if a.trace:
            eng_env["CCFD_SERVICE_TRACE"] = str(log_dir / "service_trace")
        eng_env["CCFD_HANDOFF_DLQ"] = str(Path(jdir) / "handoff-dlq.jsonl")
        if a.rehearsal:
            eng_env.update(CCFD_DIST_BACKEND="gloo", CCFD_DEVICE_MODULO="1")
        def eng_cmd(mport):
            return [PY, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(a.ranks),
                    "--master-addr", "127.0.0.1", "--master-port", str(mport),
                    "-m", L, "engine", "--host", "127.0.0.1", "--port", str(router_base),
                    "--model-metrics-port", str(model_base)]
        procs.append(Proc("engine", eng_cmd(master_port), eng_env, log_dir))
        eng = procs[-1]

        def wait_engine(e):
            t0 = time.time()
            while time.time() - t0 < 300:
                found = re.findall(r"\[engine\] rank (\d+)/(\d+) partitions \[([0-9, ]*)\]", e.text())
                if len(found) >= a.ranks:
                    return found
                if not e.alive():
                    raise RuntimeError("engine exited during start-up:\n" + e.text()[-3000:])
                time.sleep(0.5)
            raise TimeoutError("engine ranks did not come up:\n" + e.text()[-3000:])
        parts = wait_engine(eng)
        owners: Dict[int, List[int]] = {}
        for r, _w, plist in parts:
            for p in (int(x) for x in plist.replace(" ", "").split(",") if x):
                owners.setdefault(p, []).append(int(r))
        out["partition_owners"] = {str(p): owners.get(p, []) for p in range(a.partitions)}
        out["every_partition_exactly_one_rank"] = all(len(owners.get(p, [])) == 1 for p in range(a.partitions))
        for r in range(a.ranks):
            wait_port(router_base + r, 60)

        # an engine restart (--engine-kill-at) zeroes its counters: the killed incarnation's last
        # scrape is carried as a base, so the totals count every row scored, replays included
        eng_base = {"rows": 0.0, "fraud": 0.0}
        eng_last = {"rows": 0.0, "fraud": 0.0, "texts": {}}

        def scrape_all():
            rows = fraud = 0.0
            texts = {}
            try:
                for r in range(a.ranks):
                    t = http_text(f"http://127.0.0.1:{router_base + r}/prometheus")
                    texts[f"router{r}"] = t
                    rows += metric_sum(t, "transaction_incoming_total")
                    fraud += metric_sum(t, "transaction_outgoing_total", {"type": "fraud"})
            except OSError:
                if not eng_restarts["n"]:
                    raise
                return (eng_base["rows"] + eng_last["rows"], eng_base["fraud"] + eng_last["fraud"],
                        eng_last["texts"])                  # the engine is down right now
            eng_last.update(rows=rows, fraud=fraud, texts=texts)
            return eng_base["rows"] + rows, eng_base["fraud"] + fraud, texts
        eng_restarts = {"n": 0}

        # ---- producers: open loop (or --rate split), time-bounded; distinct id ranges
        prods = []
        per_rate = a.rate / a.producers if a.rate > 0 else 0.0
        for i in range(a.producers):
            prods.append(Proc(f"producer{i}", [PY, "-m", L, "producer", "--fmt", a.fmt, "--batch", str(a.batch),
                                               "--count", str(a.count), "--seconds", str(a.seconds),
                                               "--rate", str(per_rate), "--acks", str(acks),
                                               "--max-in-flight", str(inflight),
                                               "--id-base", str((i + 1) << 40), "--seed-offset", str(i * 101)],
                              env, log_dir))
        procs.extend(prods)
        # wait until all producers rendered their pools and started (first tx seen)
        rows_prev, _, _ = scrape_all()
        t_start = time.time()
        while time.time() - t_start < 120:
            rows_now, _, _ = scrape_all()
            if rows_now > rows_prev:
                break
            time.sleep(0.2)
        samples = []
        cg0 = cgroup_cpu()
        cpu0 = {q.name: q.cpu_s() for q in procs}
        t_w0 = time.time()
        r_w0, f_w0, _ = scrape_all()
        last_t, last_r = t_w0, r_w0
        outage = {}
        koutage = {}
        noutage = {}
        coutage = {}
        eoutage = {}
        kill_name = f"kie{a.kie_kill_shard}"
        import threading

        def watch_commits(t_kill, box):
            # when the engine's offset commits resume after the controller kill: the group's
            # committed offsets (read through the brokers, i.e. from the new active controller)
            # move past their values at the kill
            from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker as _KB
            kc = _KB(brokers, connect_wait_s=30)
            kc.RETRIES = 40
            try:
                base = box.get("committed_at_kill") or {}
                while time.time() - t_kill < 60:
                    try:
                        cur = {p: kc.committed("ccfd-engine", "odh-demo", p) for p in range(a.partitions)}
                    except Exception:                        # no active controller yet
                        time.sleep(0.05)
                        continue
                    if any((cur[p] or -1) > (base.get(p) or -1) for p in cur):
                        box["commits_resumed_after_s"] = round(time.time() - t_kill, 3)
                        return
                    time.sleep(0.05)
            finally:
                kc.close()
        while any(p.alive() for p in prods):
            if a.controller_kill_at > 0 and a.kafka_replicated and not coutage \
                    and time.time() - t_w0 >= a.controller_kill_at:
                ia = ctl_ports.index(active_controller(ctl_ports))
                try:
                    before = {p: kb.committed("ccfd-engine", "odh-demo", p) for p in range(a.partitions)}
                except Exception:
                    before = {}
                [p for p in procs if p.name.startswith(f"kafka-controller{ia + 1}")][-1].stop(sig=signal.SIGKILL, wait=5)
                t_kill = time.time()
                coutage = {"member": ia + 1, "killed_at_s": round(t_kill - t_w0, 1), "committed_at_kill": before}
                threading.Thread(target=watch_commits, args=(t_kill, coutage), daemon=True).start()
                try:
                    nxt = active_controller([p_ for k, p_ in enumerate(ctl_ports) if k != ia], timeout=30)
                    coutage["new_active_member"] = ctl_ports.index(nxt) + 1
                    coutage["new_active_after_s"] = round(time.time() - t_kill, 3)
                    ctl_port = nxt
                except TimeoutError:
                    coutage["new_active_after_s"] = None
            if coutage and "restarted_at_s" not in coutage and \
                    time.time() - t_w0 >= a.controller_kill_at + a.controller_down_s:
                m = coutage["member"]
                procs.append(Proc(f"kafka-controller{m}-restarted", ctl_cmds[m - 1], env, log_dir))
                coutage["restarted_at_s"] = round(time.time() - t_w0, 1)
            if a.engine_kill_at > 0 and not eoutage and time.time() - t_w0 >= a.engine_kill_at:
                e = [p for p in procs if p.name.startswith("engine")][-1]
                scrape_all()                                  # the incarnation's last counters
                # every rank crashes at once (SIGUSR1: no drain, no commit, no hand-off flush --
                # a SIGKILL's aftermath -- but its persistent kernel is stopped first: a process
                # must never end with one resident), then torchrun and anything left are killed
                import psutil
                try:
                    ranks = [c for c in psutil.Process(e.p.pid).children(recursive=True)
                             if "ccfd_demo_summit_amd.launch" in " ".join(c.cmdline())]
                except psutil.Error:
                    ranks = []
                for c in ranks:
                    try:
                        c.send_signal(signal.SIGUSR1)
                    except psutil.Error:
                        pass
                psutil.wait_procs(ranks, timeout=15)
                e.stop(sig=signal.SIGKILL, wait=10)          # torchrun (its group)
                eng_restarts["n"] += 1
                eng_base["rows"] += eng_last["rows"]
                eng_base["fraud"] += eng_last["fraud"]
                eng_last.update(rows=0.0, fraud=0.0)
                eoutage = {"killed_at_s": round(time.time() - t_w0, 1),
                           "rows_scored_before_kill": eng_base["rows"]}
            if eoutage and "restarted_at_s" not in eoutage and \
                    time.time() - t_w0 >= a.engine_kill_at + a.engine_down_s:
                procs.append(Proc("engine-restarted", eng_cmd(master_port2), eng_env, log_dir))
                eoutage["restarted_at_s"] = round(time.time() - t_w0, 1)
                wait_engine(procs[-1])
                for r in range(a.ranks):
                    wait_port(router_base + r, 60)
                eoutage["serving_at_s"] = round(time.time() - t_w0, 1)
            if a.notifier_kill_at > 0 and not noutage and time.time() - t_w0 >= a.notifier_kill_at:
                [p for p in procs if p.name.startswith("notifier")][-1].stop(sig=signal.SIGKILL, wait=5)
                noutage = {"killed_at_s": round(time.time() - t_w0, 1)}
            if noutage and "restarted_at_s" not in noutage and \
                    time.time() - t_w0 >= a.notifier_kill_at + a.notifier_down_s:
                procs.append(Proc("notifier-restarted", notif_cmd, notif_env, log_dir))
                noutage["restarted_at_s"] = round(time.time() - t_w0, 1)
            kname = f"kafka-broker{a.kafka_kill_node}" if a.kafka_replicated else "kafka-lite"
            if a.kafka_kill_at > 0 and not koutage and time.time() - t_w0 >= a.kafka_kill_at:
                kl = [p for p in procs if p.name.startswith(kname)][-1]
                kl.stop(sig=signal.SIGKILL, wait=5)            # a crashed broker pod
                koutage = {"killed_at_s": round(time.time() - t_w0, 1)}
                if a.kafka_replicated:
                    koutage["node"] = a.kafka_kill_node
            if koutage and "restarted_at_s" not in koutage and \
                    time.time() - t_w0 >= a.kafka_kill_at + a.kafka_down_s:
                cmd = broker_cmds[a.kafka_kill_node] if a.kafka_replicated else kafka_cmd
                procs.append(Proc(f"{kname}-restarted", cmd, env, log_dir))   # recovers from disk
                koutage["restarted_at_s"] = round(time.time() - t_w0, 1)
                wait_port(kafka_port + (a.kafka_kill_node - 1 if a.kafka_replicated else 0), 60)
                koutage["serving_at_s"] = round(time.time() - t_w0, 1)
            if a.kie_outage_at > 0 and not outage and time.time() - t_w0 >= a.kie_outage_at:
                kie = [p for p in procs if p.name == kill_name][0]
                kie.stop(sig=signal.SIGKILL, wait=5)           # a crashed KIE shard pod
                outage = {"shard": a.kie_kill_shard, "killed_at_s": round(time.time() - t_w0, 1)}
            if outage and "restarted_at_s" not in outage and \
                    time.time() - t_w0 >= a.kie_outage_at + a.kie_outage_s:
                procs.append(Proc(f"{kill_name}-restarted", kie_cmds[a.kie_kill_shard], kie_env,
                                  log_dir))                    # recovers its journal (+ outbox)
                outage["restarted_at_s"] = round(time.time() - t_w0, 1)
            crashes = a.kie_outage_at > 0 or a.kafka_kill_at > 0 or a.notifier_kill_at > 0 or \
                a.controller_kill_at > 0 or a.engine_kill_at > 0
            time.sleep(min(a.sample_s, 0.5) if crashes else a.sample_s)
            if time.time() - last_t < a.sample_s:
                continue
            now = time.time()
            r_now, _, _ = scrape_all()
            try:
                lag = kb.lag("ccfd-engine", "odh-demo")
            except Exception:                               # the broker is down right now
                lag = None
            samples.append({"t_s": round(now - t_w0, 1), "tx_s": round((r_now - last_r) / (now - last_t), 1),
                            "lag_msgs": lag, "loadavg_1m": round(os.getloadavg()[0], 1)})
            if a.kafka_replicated:                          # the reference dashboard's panel
                under = 0
                for mp in kmetrics:
                    try:
                        under += int(metric_sum(http_text(f"http://127.0.0.1:{mp}/metrics", timeout=2.0),
                                                "kafka_server_replicamanager_underreplicatedpartitions"))
                    except Exception:                       # that broker is down right now
                        pass
                samples[-1]["under_replicated"] = under
            print(f"[deploy] {time.strftime('%H:%M:%S')} sample {samples[-1]} kie_outage {outage} "
                  f"kafka_outage {koutage} notifier_outage {noutage}", file=sys.stderr, flush=True)
            last_t, last_r = now, r_now
        t_w1 = time.time()
        r_w1, _, _ = scrape_all()
        produced_lines = []
        for p in prods:
            m = re.findall(r'(\{"produced".*\})', p.text())
            if m:
                produced_lines.append(json.loads(m[-1]))
        produced = sum(d["produced"] for d in produced_lines)
        # ---- drain: consumer lag 0 and the engine counters settled
        t_d = time.time()
        while time.time() - t_d < a.drain_timeout_s:
            rows_all, fraud_all, texts = scrape_all()
            if kb.lag("ccfd-engine", "odh-demo") == 0 and rows_all >= produced:
                break
            time.sleep(0.5)
        time.sleep(2.0)                                  # last hand-offs / X2 ticks
        rows_all, fraud_all, texts = scrape_all()
        steady = [s["tx_s"] for s in samples[1:-1]] or [s["tx_s"] for s in samples]
        if eoutage:
            out["engine_outage"] = dict(eoutage, rows_scored_incl_replays=rows_all,
                                        replayed_rows=int(rows_all) - int(produced))
        if coutage:
            coutage.pop("committed_at_kill", None)
            out["controller_outage"] = dict(coutage)
        out.update({
            "value": round((r_w1 - r_w0) / max(t_w1 - t_w0, 1e-9), 1), "unit": "tx/s",
            # wall clock of the measured window and of the end of the drain (the services'
            # attribution maxima carry "max_at" on the same clock)
            "window_wall": [round(t_w0, 3), round(t_w1, 3)],
            "window_s": round(t_w1 - t_w0, 1), "samples": samples,
            "min_sample_tx_s": min(steady) if steady else None,
            "producers_tx_s": [d["tx_s"] for d in produced_lines],
            "produced_total": produced,
            "transaction_incoming_total": rows_all,
            # an engine restart re-scores what it had not committed: incoming counts the replays
            "incoming_equals_produced": int(rows_all) == int(produced) if not eoutage else int(rows_all) >= int(produced),
            "drain_s": round(time.time() - t_d, 1),
            "drained_wall": round(time.time(), 3),
            "final_lag_msgs": kb.lag("ccfd-engine", "odh-demo"),
        })
        # ---- ingest attribution: the engine's native consumer threads (ccfd_gpu_ingest_*)
        att = {}
        for key in ("ingest_threads", "ingest_io_seconds", "ingest_parse_seconds", "ingest_encode_seconds",
                    "ingest_ring_wait_seconds", "ingest_rows"):
            att[key] = sum(metric_sum(texts[f"router{r}"], "ccfd_gpu_" + key) for r in range(a.ranks))
        if att.get("ingest_threads"):
            ts = att["ingest_threads"] * max(1e-9, t_w1 - t_start)    # thread-seconds since producers began
            out["ingest_attribution"] = {
                "threads": int(att["ingest_threads"]),
                "broker_io_frac": round(att["ingest_io_seconds"] / ts, 3),
                "parse_frac": round(att["ingest_parse_seconds"] / ts, 3),
                "encode_frac": round(att["ingest_encode_seconds"] / ts, 3),
                "ring_full_wait_frac": round(att["ingest_ring_wait_seconds"] / ts, 3),
                "parse_ns_per_msg": round(att["ingest_parse_seconds"] * 1e9 / max(1.0, att["ingest_rows"]), 1),
                "note": "fractions of the consumer threads' wall time since the producers started "
                        "(includes start-up idle); cumulative counters of the whole run"}
        # ---- latency: the engine's X3-merged arrival -> scored quantiles (micro-batch
        # weighted, exported by rank 0 .. W-1 identically) and the Seldon histogram (row-weighted,
        # coarse buckets) summed over the ranks' model endpoints
        t0_text = texts["router0"]
        q = {}
        from prometheus_client.parser import text_string_to_metric_families
        for fam in text_string_to_metric_families(t0_text):
            for s in fam.samples:
                if s.name == "ccfd_gpu_batch_latency_quantile_seconds":
                    q[s.labels["quantile"]] = s.value
        out["arrival_to_scored_p50_us"] = round(q.get("0.5", float("nan")) * 1e6, 1)
        out["arrival_to_scored_p99_us"] = round(q.get("0.99", float("nan")) * 1e6, 1)
        # producer send (ccfd-ts record header) -> scored, per transaction, per rank
        out["produce_to_scored_us"] = [
            {"rank": r, "p50": round(metric_sum(texts[f"router{r}"], "ccfd_gpu_produce_to_scored_p50_seconds") * 1e6, 1),
             "p99": round(metric_sum(texts[f"router{r}"], "ccfd_gpu_produce_to_scored_p99_seconds") * 1e6, 1),
             "rows": int(metric_sum(texts[f"router{r}"], "ccfd_gpu_produce_to_scored_rows")),
             # the broker's share: send -> the consumer thread has the record batch
             "fetched_p50": round(metric_sum(texts[f"router{r}"], "ccfd_gpu_ingest_fetch_age_p50_seconds") * 1e6, 1),
             "fetched_p99": round(metric_sum(texts[f"router{r}"], "ccfd_gpu_ingest_fetch_age_p99_seconds") * 1e6, 1)}
            for r in range(a.ranks)]
        # scored -> started, the engine's share: hand-off queue wait and request time per rank
        out["handoff_engine_us"] = [
            {"rank": r, **{f"{k}_{q}": round(metric_sum(texts[f"router{r}"], f"ccfd_gpu_handoff_{k}_{q}_seconds") * 1e6, 1)
                           for k in ("queue_wait", "request") for q in ("p50", "p99")}}
            for r in range(a.ranks)]
        model_texts = [http_text(f"http://127.0.0.1:{model_base + r}/prometheus") for r in range(a.ranks)]
        mt = "\n".join(model_texts)
        for qq in (0.5, 0.99):
            v = hist_quantile_le(mt, "seldon_api_engine_server_requests_seconds", qq, {"status": "200"})
            out[f"seldon_server_p{int(qq * 100)}_us_bucketed"] = None if v is None else round(v * 1e6, 1)
        # ---- KIE: exactly one fraud process per fraud-routed transaction, summed over the
        # shards (the async hand-off may still be delivering the last batches)
        def kie_stats():
            per = [json.loads(http_text(f"http://127.0.0.1:{p_}/rest/stats")) for p_ in kie_ports]
            tot = {k: sum(int(d.get(k) or 0) for d in per)
                   for k in ("fraud_started", "duplicates", "standard_started", "standard_duplicates", "active",
                             "notified", "waiting_customer", "fraud_instances_retained")}
            tot["outcomes"] = {k: sum(int(d["outcomes"].get(k, 0)) for d in per) for k in per[0]["outcomes"]}
            tot["outcome_digest"] = f"{sum(int(d.get('outcome_digest') or '0', 16) for d in per) & (2**64 - 1):016x}"
            tot["per_shard"] = [{k: d.get(k) for k in ("shard", "fraud_started", "standard_started", "duplicates",
                                                      "standard_duplicates", "notified", "scored_to_started_us")}
                                for d in per]
            tot["scored_to_started_us"] = {
                "n": sum(int((d.get("scored_to_started_us") or {}).get("n", 0)) for d in per),
                "p50_max_over_shards": max(((d.get("scored_to_started_us") or {}).get("p50") or 0) for d in per),
                "p99_max_over_shards": max(((d.get("scored_to_started_us") or {}).get("p99") or 0) for d in per)}
            tot["handoff_attribution"] = [d.get("handoff_attribution") for d in per]
            return tot
        t_k = time.time()
        while True:
            stats = kie_stats()
            if int(stats["fraud_started"]) >= int(fraud_all) or time.time() - t_k > 30:
                break
            time.sleep(0.5)
        out["fraud_routed_total"] = fraud_all
        if outage:
            out["kie_outage"] = dict(outage, recovered=re.findall(r"\[kie\] (?:recovered|outbox).*", "".join(
                p.text() for p in procs if p.name == f"{kill_name}-restarted")))
        out["kie_fraud_started_equals_routed"] = (int(stats["fraud_started"]) == int(fraud_all)) if not eoutage \
            else int(stats["fraud_started"]) <= int(fraud_all)   # routed counts the replayed rows too
        out["kie_duplicates"] = stats["duplicates"]
        out["standard_mode"] = a.standard_mode
        # the host this topology shares: every service and engine rank runs on these CPUs
        out["host_cpus"] = {"affinity": len(os.sched_getaffinity(0)), "machine": os.cpu_count(),
                            "loadavg_1m_max": max((sm.get("loadavg_1m", 0) for sm in samples), default=None)}
        # where the CPU went during the measured window (and whether the cgroup's quota throttled it)
        cg1 = cgroup_cpu()
        out["cgroup_cpu"] = {"cpu.max": cg1.get("cpu.max"),
                             **{k: cg1[k] - cg0.get(k, 0) for k in ("usage_usec", "nr_periods", "nr_throttled",
                                                                   "throttled_usec") if k in cg1}}
        out["cpu_s_by_service"] = {q.name: (round(q.cpu_s() - cpu0[q.name], 1)
                                            if q.cpu_s() is not None and cpu0.get(q.name) is not None else None)
                                   for q in procs if q.name in cpu0}
        out["window_s"] = round(time.time() - t_w0, 1)
        if a.standard_mode == "process":
            # every transaction started exactly one process: standard + fraud == incoming
            t_k = time.time()
            while int(stats["standard_started"]) + int(stats["fraud_started"]) < int(rows_all) \
                    and time.time() - t_k < 60:
                time.sleep(0.5)
                stats = kie_stats()
            out["kie_standard_plus_fraud_equals_incoming"] = \
                int(stats["standard_started"]) + int(stats["fraud_started"]) == int(rows_all)
            out["kie_standard_duplicates"] = stats.get("standard_duplicates")
            # every transaction produced started exactly one process, replays included: the
            # duplicates are what the shards recognised (a start counted twice would break it)
            out["kie_standard_plus_fraud_equals_produced"] = \
                int(stats["standard_started"]) + int(stats["fraud_started"]) == int(produced)
            if eoutage:
                t_k = time.time()
                while int(stats["standard_started"]) + int(stats["fraud_started"]) < int(produced) \
                        and time.time() - t_k < 60:
                    time.sleep(0.5)
                    stats = kie_stats()
                out["kie_standard_plus_fraud_equals_produced"] = \
                    int(stats["standard_started"]) + int(stats["fraud_started"]) == int(produced)
                out["kie_standard_plus_fraud_equals_incoming"] = out["kie_standard_plus_fraud_equals_produced"]
                out["kie_standard_duplicates"] = stats.get("standard_duplicates")
                out["duplicates_recognised"] = int(stats.get("standard_duplicates") or 0) + int(stats["duplicates"])
        if a.settle:
            # outcomes are final once no fraud process waits for its customer (timer or reply)
            t_k = time.time()
            while int(stats["waiting_customer"]) > 0 and time.time() - t_k < a.notification_timeout_s + 60:
                time.sleep(1.0)
                stats = kie_stats()
            out["settled"] = int(stats["waiting_customer"]) == 0
            out["settle_s"] = round(time.time() - t_k, 1)
        out["kie"] = stats
        out["scored_to_process_started_us"] = stats["scored_to_started_us"]
        out["kie_handoff_attribution"] = stats["handoff_attribution"]
        if koutage:
            rec = re.findall(r"\[kafka-lite\] (?:node \d+ )?recovered from .*", "".join(
                p.text() for p in procs if p.name.endswith("-restarted") and p.name.startswith("kafka")))
            out["kafka_outage"] = dict(koutage, recovered=rec)
            if a.kafka_replicated:
                # the under-replicated series rose while the broker was away and is back to 0
                under = [sm.get("under_replicated", 0) for sm in samples]
                out["under_replicated_max"] = max(under) if under else None
                fin = 0
                for mp in kmetrics:
                    try:
                        fin += int(metric_sum(http_text(f"http://127.0.0.1:{mp}/metrics", timeout=2.0),
                                              "kafka_server_replicamanager_underreplicatedpartitions"))
                    except Exception:
                        fin = -1
                out["under_replicated_final"] = fin
                out["min_sample_ratio"] = (round(min(sm["tx_s"] for sm in samples[1:-1]) /
                                                 max(sm["tx_s"] for sm in samples[1:-1]), 3)
                                           if len(samples) > 2 else None)
        if noutage:
            out["notifier_outage"] = noutage
        out["handoff_dead_lettered"] = sum(sum(1 for _ in open(f)) for f in Path(jdir).glob("handoff-dlq*.jsonl"))
        try:
            out["notifier"] = json.loads(http_text(f"http://127.0.0.1:{notif_port}/health/ping"))
        except Exception as e:
            out["notifier"] = {"error": repr(e)}
        # the notification loop: every fraud process notified (the KIE outbox drained) and, once
        # settled, every reply the customers sent applied exactly once (the rest were stale)
        out["kie_notified_equals_fraud_started"] = int(stats["notified"]) >= int(stats["fraud_started"])
        oc = stats["outcomes"]
        out["customer_replies_applied"] = int(oc.get("approved_by_customer", 0)) + int(oc.get("cancelled", 0))
        if a.compare_to:
            # the same transactions (--count, same seeds) through a run with crashes: every fraud
            # process must end with the outcome it had in the reference run
            ref = json.loads(Path(a.compare_to).read_text())
            out["same_outcomes_as"] = {
                "run": a.compare_to, "outcomes_equal": ref["kie"]["outcomes"] == oc,
                "digest_equal": ref["kie"].get("outcome_digest") == stats["outcome_digest"],
                "reference_outcomes": ref["kie"]["outcomes"]}
        # ---- the reference dashboards against everything this deployment serves
        from ccfd_demo_summit_amd.metrics import promql
        series = []
        scrape_errors = []

        def scrape(url, job, **kw):
            try:
                return promql.scrape(url, job, **kw)
            except OSError as e:                    # a service that is down: recorded, not fatal
                scrape_errors.append(f"{url}: {e}")
                return []
        for r in range(a.ranks):
            series += scrape(f"http://127.0.0.1:{router_base + r}/prometheus", "ccfd-pods")
            series += scrape(f"http://127.0.0.1:{model_base + r}/prometheus", "ccfd-model",
                             instance=f"engine-{r}:8000")   # k8s: <pod ip>:8000 (operator/render.py)
        for p_ in kie_ports:
            series += scrape(f"http://127.0.0.1:{p_}/rest/metrics", "ccfd-pods")
        for mp in kmetrics:
            series += scrape(f"http://127.0.0.1:{mp}/metrics", "ccfd-pods")
        if a.kafka_replicated:
            series += scrape(f"http://127.0.0.1:{ctl_port}/metrics", "ccfd-pods")
        out["scrape_errors"] = scrape_errors
        fx = json.loads((ROOT / "tests/fixtures/reference_dashboard_exprs.json").read_text())
        exprs = {k: [e["expr"] for e in v] for k, v in fx["dashboards"].items() if k != "SparkMetrics.json"}
        rep = promql.check(exprs, series)
        out["reference_dashboards"] = {"selectors": rep["selectors"], "matched": rep["matched"],
                                       "unmatched": [u["selector"] for u in rep["unmatched"]],
                                       "note": "SparkMetrics.json: the trainer is not part of this topology "
                                               "(tests/test_dashboard_conformance.py scrapes it)"}
        ok = (out["incoming_equals_produced"] and out["every_partition_exactly_one_rank"]
              and out["kie_fraud_started_equals_routed"] and not rep["unmatched"]
              and (out["kie_duplicates"] == 0 or bool(eoutage))
              and out.get("kie_standard_plus_fraud_equals_produced", True)
              and out.get("kie_standard_plus_fraud_equals_incoming", True)
              and out["kie_notified_equals_fraud_started"] and out.get("settled", True)
              and not scrape_errors and out.get("under_replicated_final", 0) == 0
              and all(out.get("same_outcomes_as", {"x": True}).get(k, True) for k in ("outcomes_equal", "digest_equal")))
        out["checks_passed"] = bool(ok)
    finally:
        for p in reversed(procs):
            p.stop(wait=40.0 if p.name.startswith("engine") else 10.0)   # the engine drains on SIGTERM
        if "jdir" in locals():
            import shutil
            out["kie_journal_bytes"] = sum(j.stat().st_size for j in journals if j.exists())
            shutil.rmtree(jdir, ignore_errors=True)
        import shutil
        try:
            out["kafka_data_bytes"] = sum(f.stat().st_size for f in Path(kdir).rglob("*") if f.is_file())
        except OSError:
            pass
        shutil.rmtree(kdir, ignore_errors=True)
    # the engine ranks' hand-off totals (printed as they stop): signals applied vs stale
    eng_logs = "".join(p.text() for p in procs if p.name.startswith("engine"))
    hs = []
    dec = json.JSONDecoder()
    for m in re.finditer(r"hand-off \{", eng_logs):      # ranks stopping together may share a line
        try:
            hs.append(dec.raw_decode(eng_logs, m.end() - 1)[0])
        except ValueError:
            pass
    if hs:
        out["handoff_signals"] = {"ok": sum(h.get("signals_ok", 0) for h in hs),
                                  "stale": sum(h.get("signals_stale", 0) for h in hs),
                                  "dead_lettered": sum(h.get("dead_lettered", 0) for h in hs)}
        if "customer_replies_applied" in out:
            out["every_reply_signalled_once"] = out["handoff_signals"]["ok"] == out["customer_replies_applied"]
    if a.trace:
        sys.path.insert(0, str(ROOT / "bench"))
        import tail_attribution
        out["tail_attribution"] = [tail_attribution.attribute(str(t))
                                   for t in sorted((log_dir / "service_trace").glob("rank*.npz"))]
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        Path(a.out).write_text(line + "\n")
    return 0 if out.get("checks_passed") else 1


if __name__ == "__main__":
    sys.exit(main())
