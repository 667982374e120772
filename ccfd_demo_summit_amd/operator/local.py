"""Local operator: reconciles a FraudDetection CR into supervised processes on this host --
what the ODH operator does with the reference's CR on a cluster (deploy/frauddetection_cr.yaml;
SURVEY.md §2.1 C18/C20, §1 L0), for a single MI355X node without Kubernetes.

``reconcile()`` compares the desired replicas of every service (from the CR) with the live
processes: it starts missing replicas, restarts exited ones (crash-loop back-off like the
reference's ``restartPolicy: Always`` DeploymentConfigs), stops surplus replicas when the CR
scales down, health-checks every replica on the route its Kubernetes probes use (a replica
that keeps failing after its start window is killed and restarted, like a liveness probe),
replaces replicas whose command or environment changed with the CR a few at a time
(rolling update), and writes a status document (per service: desired / ready (running) / healthy / restarts,
the CR generation it reflects).  ``run()`` re-reads the CR file when it changes, so editing the
CR is how the local deployment is scaled -- the same declarative loop as on a cluster.

Every replica is its own process group (never exec'd from a GPU-initialised parent); stop
sends SIGTERM, waits ``grace_s`` (the reference's terminationGracePeriodSeconds 30), then
SIGKILLs the group.  Local ports: replica r of a service listens on its base port + r.
"""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Callable, Dict, Optional

from .spec import FraudDetectionSpec, load

PY = [sys.executable, "-m", "ccfd_demo_summit_amd.launch"]


@dataclass
class Replica:
    proc: subprocess.Popen
    started: float
    restarts: int = 0
    last_exit: Optional[int] = None
    healthy: bool = False
    probe_fails: int = 0
    template: str = ""                      # argv + env it was started with (rolling updates)


@dataclass
class ServiceState:
    desired: int = 0
    replicas: Dict[int, Replica] = field(default_factory=dict)
    restarts: int = 0
    backoff_until: Dict[int, float] = field(default_factory=dict)
    job: bool = False                       # run-to-completion (Job): restart only on failure
    succeeded: set = field(default_factory=set)
    rollouts: int = 0                       # replicas replaced because their template changed

JOBS = ("producer", "training")             # Kubernetes Jobs in the rendering (restartPolicy OnFailure)


def probe_ok(target: tuple, timeout_s: float = 0.5) -> bool:
    """One health check: ("http", url) -> 2xx, ("tcp", host, port) -> connect succeeds."""
    try:
        if target[0] == "tcp":
            with socket.create_connection((target[1], target[2]), timeout=timeout_s):
                return True
        import urllib.request
        with urllib.request.urlopen(target[1], timeout=timeout_s) as r:
            return 200 <= r.status < 300
    except Exception:
        return False


def local_commands(spec: FraudDetectionSpec, host: str = "127.0.0.1", port_offset: int = 0,
                   state_dir: str = ".ccfd-state") -> Dict[str, tuple]:
    """service -> (desired replicas, argv factory(replica index), env (a dict, or a factory of
    the replica index), probe) for a one-node run; every port is the service's reference
    port + ``port_offset`` (+ replica index).
    ``probe`` is (target factory(replica index), start seconds) -- the same health routes the
    rendered readiness / liveness probes use (render.py) -- or None.  ``state_dir`` holds what
    must survive a restart: kafka-lite's logs, the KIE journal, the hand-off DLQ."""
    state = os.path.abspath(state_dir)
    o = port_offset
    kafka_port = 9092 + o
    ctl_port = 9290 + o                     # replicated kafka-lite's controller
    broker = (spec.kafka.bootstrap if not spec.kafka.deploy
              else ",".join(f"{host}:{kafka_port + i}" for i in range(spec.kafka.brokers)))
    K = max(1, spec.kie.shards)
    kie_url = ",".join(f"http://{host}:{8090 + o + k}" for k in range(K))     # one per shard
    env = {"BROKER_URL": broker, "KIE_SERVER_URL": kie_url, "CCFD_KIE_SHARDS": str(K),
           "SELDON_URL": f"http://{host}:{8000 + o}",
           "CCFD_KAFKA_BACKEND": "kafka", "CCFD_KAFKA_PARTITIONS": str(spec.kafka.partitions),
           "CCFD_MODEL": spec.engine.model, "CCFD_EXEC_MODE": spec.engine.exec_mode,
           "CCFD_OUTPUT_MODE": spec.engine.output_mode, "CCFD_PERSIST_ITEMS": spec.engine.persist_items, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    if spec.engine.rules:
        env["ROUTER_RULES"] = spec.engine.rules
    env["ROUTER_STANDARD_MODE"] = spec.engine.standard_mode
    if spec.engine.handoff_dlq:
        # the CR names the pod path; locally the DLQ lives in the state directory
        env["CCFD_HANDOFF_DLQ"] = os.path.join(state, os.path.basename(spec.engine.handoff_dlq))
    env.update(spec.env)
    w = ["--weights", spec.engine.weights] if spec.engine.weights else []
    svc: Dict[str, tuple] = {}
    if spec.kafka.deploy and spec.kafka.replicated:
        # replica r is broker node r + 1 (its own port, log and metrics port); controller replica
        # r is quorum member r + 1 (ingest/controller_quorum.py) on ctl_port + r
        nctl = max(1, spec.kafka.controllers)
        peers = ",".join(f"{k + 1}=http://{host}:{ctl_port + k}" for k in range(nctl))
        ctl_urls = ",".join(f"http://{host}:{ctl_port + k}" for k in range(nctl))
        svc["kafka-controller"] = (nctl, lambda r: [sys.executable, "-m", "ccfd_demo_summit_amd.ingest.kafka_controller",
                                                    "--host", host, "--port", str(ctl_port + r),
                                                    "--brokers", str(spec.kafka.brokers),
                                                    "--rf", str(spec.kafka.replication_factor),
                                                    "--data-dir", os.path.join(state, "kafka-controller"
                                                                               + (f"-{r + 1}" if nctl > 1 else ""))]
                                   + (["--member-id", str(r + 1), "--peers", peers] if nctl > 1 else []))
        svc["kafka"] = (spec.kafka.brokers, lambda r: [
            sys.executable, "-m", "ccfd_demo_summit_amd.ingest.kafka_lite", "--host", host,
            "--port", str(kafka_port + r), "--node-id", str(r + 1), "--controller", ctl_urls,
            "--metrics-port", str(9404 + o + r), "--data-dir", os.path.join(state, f"kafka-lite-{r + 1}"),
            "--fsync", spec.kafka.fsync])
    elif spec.kafka.deploy:
        svc["kafka"] = (1, lambda r: [sys.executable, "-m", "ccfd_demo_summit_amd.ingest.kafka_lite",
                                      "--nodes", str(spec.kafka.brokers), "--port", str(kafka_port), "--host", host,
                                      "--partitions", str(spec.kafka.partitions), "--metrics-port", str(9404 + o),
                                      "--data-dir", os.path.join(state, "kafka-lite"), "--fsync", spec.kafka.fsync])
    if spec.usertask.deploy:
        svc["usertask"] = (spec.usertask.replicas, lambda r: PY + ["usertask", "--host", host, "--port", str(5000 + o + r)])
    if spec.seldon.deploy:
        svc["seldon"] = (spec.seldon.replicas, lambda r: PY + ["seldon", "--host", host, "--port", str(8000 + o + r)] + w
                         + (["--native", "--workers", str(spec.seldon.workers)] if spec.seldon.native else []))
    if spec.kie.deploy:
        # replica r is KIE shard r (its own port and journal)
        svc["kie"] = (K, lambda r: PY + ["kie", "--host", host, "--port", str(8090 + o + r), "--shard", str(r),
                                         "--remote-prediction",
                                         "--journal", os.path.join(state, f"kie-journal-{r}.jsonl")])
    if spec.notifier.deploy:
        svc["notifier"] = (spec.notifier.replicas, lambda r: PY + ["notifier", "--host", host,
                                                                   "--port", str(8080 + o + r)])
    if spec.engine.deploy:
        g, nodes = spec.engine.gpus_per_node, spec.engine.nodes
        # engine.nodes > 1 on one host: replica r plays node r of ONE job (c10d rendezvous on
        # 127.0.0.1) and sees GPUs [r*g, (r+1)*g) -- the same world the cluster rendering builds
        dist_args = (["--nnodes", "1", "--master-addr", "127.0.0.1", "--master-port", str(29500 + o)]
                     if nodes == 1 else
                     ["--nnodes", str(nodes), "--rdzv-backend", "c10d", "--rdzv-id", f"ccfd-engine-{o}",
                      "--rdzv-endpoint", f"127.0.0.1:{29500 + o}"])
        svc["engine"] = (nodes, lambda r: [sys.executable, "-m", "torch.distributed.run"] + dist_args
                         + ["--nproc-per-node", str(g), "-m", "ccfd_demo_summit_amd.launch", "engine", "--host", host,
                            "--port", str(8091 + o + 16 * r),
                            # the model's /prometheus (+ local rank): its own range, never Seldon's
                            # 8000 + o + r nor another replica's
                            "--model-metrics-port", str(8300 + o + 16 * r)] + w)
    if spec.router.deploy:
        svc["router"] = (spec.router.replicas, lambda r: PY + ["router", "--group-membership", "--host", host,
                                                               "--port", str(8191 + o + r)])
    if spec.producer.deploy:
        svc["producer"] = (1, lambda r: PY + ["producer", "--fmt", spec.producer.format,
                                              "--count", str(spec.producer.count)])
    own = {k: dict(env) for k in svc}
    if "kie" in own:               # the KIE pod's prediction service targets the user-task model
        own["kie"].update(SELDON_URL=f"http://{host}:{5000 + o}", SELDON_ENDPOINT="predict")
    if "engine" in own and spec.engine.nodes > 1:
        base, g = own["engine"], spec.engine.gpus_per_node
        own["engine"] = lambda r: dict(base, HIP_VISIBLE_DEVICES=",".join(str(r * g + i) for i in range(g)))

    def http(port, path, stride=1):
        return lambda r: ("http", f"http://{host}:{port + o + stride * r}{path}")
    probes = {"kafka": (lambda r: ("tcp", host, kafka_port + (r if spec.kafka.replicated else 0)), 20),
              "kafka-controller": (lambda r: ("http", f"http://{host}:{ctl_port}/health/ping"), 20),
              "usertask": (http(5000, "/health/ping"), 30), "seldon": (http(8000, "/health/ping"), 60),
              "kie": (http(8090, "/services/rest/server"), 30), "notifier": (http(8080, "/health/ping"), 30),
              "engine": (http(8091, "/health/ping", 16), 120), "router": (http(8191, "/health/ping"), 30)}
    return {k: (n, f, own[k], probes.get(k)) for k, (n, f) in svc.items()}


class LocalOperator:
    def __init__(self, spec: FraudDetectionSpec, workdir: str = ".", status_path: Optional[str] = None,
                 commands: Optional[Dict[str, tuple]] = None, grace_s: float = 30.0, backoff_s: float = 1.0,
                 max_backoff_s: float = 30.0, log: Callable[[str], None] = print, port_offset: int = 0,
                 liveness_failures: int = 6, state_dir: Optional[str] = None):
        self.spec = spec
        self.workdir = workdir
        self.state_dir = state_dir or os.path.join(workdir, ".ccfd-state")
        self.status_path = status_path
        self.grace_s = grace_s
        self.backoff_s = backoff_s
        self.max_backoff_s = max_backoff_s
        self.log = log
        self.generation = 1
        self._commands_override = commands
        self.port_offset = port_offset
        self.liveness_failures = liveness_failures
        self.services: Dict[str, ServiceState] = {}
        self._commands = commands if commands is not None else local_commands(spec, port_offset=port_offset,
                                                                              state_dir=self.state_dir)

    # ------------------------------------------------------------------ spec changes
    def update(self, spec: FraudDetectionSpec) -> None:
        """A new CR generation: the next reconcile converges to it."""
        self.spec = spec
        self.generation += 1
        if self._commands_override is None:
            self._commands = local_commands(spec, port_offset=self.port_offset, state_dir=self.state_dir)

    def _env(self, name: str, r: int) -> Dict[str, str]:
        env = self._commands[name][2]
        return env(r) if callable(env) else env           # per-replica env (e.g. its GPUs)

    def _template(self, name: str, r: int) -> str:
        argv_of = self._commands[name][1]
        return json.dumps([list(argv_of(r)), sorted((str(k), str(v)) for k, v in self._env(name, r).items())])

    def _start(self, name: str, r: int) -> Replica:
        argv_of, env = self._commands[name][1], self._env(name, r)
        e = dict(os.environ)
        e.update({str(k): str(v) for k, v in env.items()})
        root = str(Path(__file__).resolve().parents[2])             # the package, from any cwd
        e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
        p = subprocess.Popen(argv_of(r), cwd=self.workdir, env=e, start_new_session=True,
                             stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        return Replica(p, time.time(), template=self._template(name, r))

    def _stop(self, rep: Replica) -> None:
        if rep.proc.poll() is None:
            try:
                os.killpg(rep.proc.pid, signal.SIGTERM)
            except ProcessLookupError:
                return
            try:
                rep.proc.wait(timeout=self.grace_s)
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(rep.proc.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                rep.proc.wait()

    def reconcile(self) -> Dict[str, Dict[str, int]]:
        now = time.time()
        for name in list(self.services):
            if name not in self._commands:                  # service removed from the CR
                st = self.services.pop(name)
                for rep in st.replicas.values():
                    self._stop(rep)
        for name, cmd in self._commands.items():
            desired, probe = cmd[0], (cmd[3] if len(cmd) > 3 else None)
            st = self.services.setdefault(name, ServiceState(job=name in JOBS))
            st.desired = desired
            for r in sorted((k for k in st.replicas if k >= desired), reverse=True):   # scale down: highest first
                self._stop(st.replicas.pop(r))
                st.backoff_until.pop(r, None)
            for r in range(desired):
                rep = st.replicas.get(r)
                if rep is not None and rep.proc.poll() is None:
                    if probe is None:
                        continue
                    # readiness / liveness: failures before the start window are not counted;
                    # ``liveness_failures`` in a row after it kill the (hung) replica -> restart
                    target_of, start_s = probe
                    rep.healthy = probe_ok(target_of(r))
                    rep.probe_fails = 0 if rep.healthy else rep.probe_fails + (now - rep.started >= start_s)
                    if rep.probe_fails < self.liveness_failures:
                        continue
                    self.log(f"[operator] {name}[{r}] failed {rep.probe_fails} liveness probes: killing it")
                    self._stop(rep)
                if r in st.succeeded:
                    continue
                if rep is not None and st.job and rep.proc.returncode == 0:   # a Job that completed
                    st.succeeded.add(r)
                    continue
                if rep is not None:                                    # exited: restart with back-off
                    if now < st.backoff_until.get(r, 0.0):
                        continue
                    rc = rep.proc.returncode
                    nxt = self._start(name, r)
                    nxt.restarts, nxt.last_exit = rep.restarts + 1, rc
                    st.replicas[r] = nxt
                    st.restarts += 1
                    delay = min(self.max_backoff_s, self.backoff_s * (2 ** min(nxt.restarts, 10)))
                    st.backoff_until[r] = now + delay
                    self.log(f"[operator] {name}[{r}] exited rc={rc}: restarted (#{nxt.restarts})")
                else:
                    st.replicas[r] = self._start(name, r)
            if not st.job:
                self._roll(name, st, desired, probe)
        status = self.status()
        if self.status_path:
            tmp = self.status_path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(status, f, indent=1)
            os.replace(tmp, self.status_path)
        return status["services"]

    def _roll(self, name: str, st: ServiceState, desired: int, probe) -> None:
        """Rolling update (the reference DeploymentConfigs' Rolling strategy, maxUnavailable
        25 %): replicas whose argv / env changed with the CR are replaced -- stop, then start on
        the same port -- at most max(1, desired // 4) unavailable at a time; with a probe a new
        replica counts as unavailable until its health route answers."""
        outdated = [r for r in sorted(st.replicas) if st.replicas[r].proc.poll() is None
                    and st.replicas[r].template != self._template(name, r)]
        if not outdated:
            return
        unavailable = sum(1 for rep in st.replicas.values()
                          if rep.proc.poll() is not None or (probe is not None and not rep.healthy))
        for r in outdated[:max(0, max(1, desired // 4) - unavailable)]:
            self._stop(st.replicas[r])
            st.replicas[r] = self._start(name, r)
            st.rollouts += 1
            self.log(f"[operator] {name}[{r}] rolled to generation {self.generation}")

    def status(self) -> Dict:
        svc = {}
        for name, st in self.services.items():
            ready = sum(1 for rep in st.replicas.values() if rep.proc.poll() is None)
            svc[name] = {"desired": st.desired, "ready": ready, "restarts": st.restarts,
                         "pids": sorted(rep.proc.pid for rep in st.replicas.values() if rep.proc.poll() is None)}
            if st.rollouts:
                svc[name]["rollouts"] = st.rollouts
            cmd = self._commands.get(name)
            if cmd is not None and len(cmd) > 3 and cmd[3] is not None:
                svc[name]["healthy"] = sum(1 for rep in st.replicas.values()
                                           if rep.healthy and rep.proc.poll() is None)
            if st.job:
                svc[name]["succeeded"] = len(st.succeeded)
        return {"name": self.spec.name, "observedGeneration": self.generation, "services": svc,
                "notes": list(self.spec.notes)}

    def shutdown(self) -> None:
        for st in self.services.values():
            for rep in st.replicas.values():
                self._stop(rep)
            st.replicas.clear()

    def run(self, cr_path: str, interval_s: float = 1.0, until: Optional[Callable[[], bool]] = None) -> None:
        """Reconcile loop; re-reads ``cr_path`` whenever it changes (a scale / config edit)."""
        mtime = os.path.getmtime(cr_path)
        stopping = {"flag": False}

        def on_signal(_s, _f):
            stopping["flag"] = True
        old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
        try:
            while not stopping["flag"] and not (until and until()):
                m = os.path.getmtime(cr_path)
                if m != mtime:
                    mtime = m
                    try:
                        self.update(load(cr_path))
                        self.log(f"[operator] CR generation {self.generation}")
                    except Exception as e:                  # keep the running generation
                        self.log(f"[operator] invalid CR update ignored: {e}")
                self.reconcile()
                time.sleep(interval_s)
        finally:
            self.shutdown()
            for s, h in old.items():
                signal.signal(s, h)
