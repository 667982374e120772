"""Operator analogue: the FraudDetection CR parses and validates,
renders into a structurally valid set of Kubernetes objects (the checked-in
deploy/k8s/ccfd-mi355x.yaml IS that rendering), the reference's OpenDataHub CR maps onto it,
and the local reconcile loop starts / restarts / scales / stops supervised processes -- including
a real 3-listener kafka-lite cluster that a Kafka client then uses."""
import copy
import os
import random
import signal
import sys
import time
from pathlib import Path

import pytest
import yaml

from ccfd_demo_summit_amd.operator import (FraudDetectionSpec, LocalOperator, SpecError, load, parse, render,
                                           validate)

ROOT = Path(__file__).resolve().parents[1]
CR = ROOT / "deploy" / "cr" / "frauddetection-mi355x.yaml"


def _doc():
    return yaml.safe_load(CR.read_text())


def test_default_cr_renders_the_checked_in_manifests():
    spec = load(str(CR))
    ms = render(spec)
    assert validate(ms) == []
    checked_in = [d for d in yaml.safe_load_all((ROOT / "deploy/k8s/ccfd-mi355x.yaml").read_text()) if d]
    assert checked_in == ms, "deploy/k8s/ccfd-mi355x.yaml is stale: re-render it from the CR"
    kinds = {(m["kind"], m["metadata"]["name"]) for m in ms}
    # the reference's service names (router.yaml, ccd-service.yaml, modelfull.json, ...)
    for k in [("Service", "modelfull-modelfull"), ("Service", "ccd-service"), ("Service", "ccfd-seldon-model"),
              ("Deployment", "ccfd-notification-service"), ("Job", "kafka-producer"),
              ("Service", "odh-message-bus-kafka-brokers"), ("StatefulSet", "ccfd-engine")]:
        assert k in kinds, k


def test_cr_fields_drive_the_rendering():
    d = _doc()
    d["spec"]["kafka"]["brokers"] = 5
    d["spec"]["engine"].update(nodes=2, gpusPerNode=4, model="gbdt")
    d["spec"]["kafka"]["partitions"] = 16
    d["spec"]["seldon"]["replicas"] = 3
    d["spec"]["router"] = {"deploy": True, "replicas": 2}
    d["spec"]["training"] = {"deploy": True, "workers": 4, "model": "gbdt", "gpus": 1}
    ms = render(parse(d))
    assert validate(ms) == []
    by = {(m["kind"], m["metadata"]["name"]): m for m in ms}
    env = by[("ConfigMap", "ccfd-env")]["data"]
    assert env["BROKER_URL"].count(",") == 4 and env["CCFD_WIRE"] == "g20" and env["CCFD_MODEL"] == "gbdt"
    eng = by[("StatefulSet", "ccfd-engine")]
    c = eng["spec"]["template"]["spec"]["containers"][0]
    assert eng["spec"]["replicas"] == 2 and c["resources"]["limits"]["amd.com/gpu"] == 4
    assert c["command"][c["command"].index("--nproc-per-node") + 1] == "4"
    assert by[("Deployment", "modelfull-modelfull")]["spec"]["replicas"] == 3
    assert by[("Deployment", "ccd-fuse")]["spec"]["replicas"] == 2
    # replicated kafka-lite: 5 broker pods (one listener each) + the controller
    sts = by[("StatefulSet", "odh-message-bus-kafka")]
    kafka = sts["spec"]["template"]["spec"]["containers"][0]
    assert sts["spec"]["replicas"] == 5 and [p["containerPort"] for p in kafka["ports"]] == [9092, 9404]
    assert "--controller" in kafka["command"] and ("StatefulSet", "odh-message-bus-kafka-controller") in by
    # the controller is a 3-member replicated quorum (ZooKeeper's role); brokers know every member
    ctl = by[("StatefulSet", "odh-message-bus-kafka-controller")]
    cc = ctl["spec"]["template"]["spec"]["containers"][0]["command"]
    assert ctl["spec"]["replicas"] == 3 and ctl["spec"]["serviceName"] == "odh-message-bus-kafka-controller-members"
    assert cc[cc.index("--member-id") + 1] == "auto" and cc[cc.index("--peers") + 1].count("=http://") == 3
    assert kafka["command"][kafka["command"].index("--controller") + 1].count("http://") == 3
    assert by[("Service", "odh-message-bus-kafka-controller-members")]["spec"]["clusterIP"] == "None"
    assert by[("Service", "odh-message-bus-kafka-brokers")]["spec"]["clusterIP"] == "None"
    d["spec"]["kafka"]["replicated"] = False                 # one pod with 5 listeners
    one = {(m["kind"], m["metadata"]["name"]): m for m in render(parse(d))}
    kafka1 = one[("StatefulSet", "odh-message-bus-kafka")]["spec"]["template"]["spec"]["containers"][0]
    assert len([p for p in kafka1["ports"] if p["name"].startswith("broker")]) == 5
    train = by[("Job", "ccfd-training")]["spec"]["template"]["spec"]["containers"][0]["command"]
    assert train[train.index("--nproc-per-node") + 1] == "4" and "gbdt" in train


@pytest.mark.parametrize("patch,msg", [
    (lambda s: s["engine"].update(gpusPerNode=9), "gpus_per_node"),
    (lambda s: s["engine"].update(model="gbdt", rowFormat="w64"), "row_format"),
    (lambda s: s["env"].update(NOT_A_KEY="1"), "unknown keys"),
    (lambda s: s["kafka"].update(replicas=3), "unknown field"),
    (lambda s: s["seldon"].update(replicas="two"), "integer"),
    (lambda s: s["kafka"].update(deploy=False), "bootstrap"),
    (lambda s: s["engine"].update(nodes=3, gpusPerNode=8), "every rank needs at least one partition"),
])
def test_invalid_crs_are_refused(patch, msg):
    d = _doc()
    patch(d["spec"])
    with pytest.raises(SpecError, match=msg):
        parse(d)


def test_reference_opendatahub_cr_maps_onto_the_stack():
    odh = {"apiVersion": "opendatahub.io/v1alpha1", "kind": "OpenDataHub", "metadata": {"name": "example"},
           "spec": {"aicoe-jupyterhub": {"odh_deploy": True, "spark_worker_nodes": 2},
                    "spark-operator": {"odh_deploy": True}, "seldon": {"odh_deploy": True},
                    "kafka": {"odh_deploy": True, "kafka_cluster_name": "odh-message-bus",
                              "kafka_broker_replicas": 3, "kafka_zookeeper_replicas": 3},
                    "monitoring": {"odh_deploy": True}, "beakerx": {"odh_deploy": False}}}
    spec = parse(odh)
    assert spec.kafka.brokers == 3 and spec.kafka.cluster_name == "odh-message-bus"
    assert spec.training.deploy and spec.training.workers == 2 and spec.seldon.deploy and spec.monitoring.deploy
    assert any("zookeeper" in n for n in spec.notes) and any("notebook" in n for n in spec.notes)
    assert spec.broker_url.startswith("odh-message-bus-kafka-0.odh-message-bus-kafka-brokers:9092")
    assert validate(render(spec)) == []


def test_multi_node_engine_is_one_rendezvous_job():
    """engine.nodes > 1: the pods join ONE torchrun world (c10d rendezvous on ccfd-engine-0
    behind a headless Service) so ranks own disjoint partitions; separate per-pod jobs -- each
    scoring the same partitions -- are refused by validate(); the local operator gives every
    replica its own GPUs of the same world."""
    d = _doc()
    d["spec"]["engine"].update(nodes=3, gpusPerNode=8)
    d["spec"]["kafka"]["partitions"] = 24
    ms = render(parse(d))
    assert validate(ms) == []
    by = {(m["kind"], m["metadata"]["name"]): m for m in ms}
    assert by[("Service", "ccfd-engine")]["spec"]["clusterIP"] == "None"
    sts = by[("StatefulSet", "ccfd-engine")]
    cmd = sts["spec"]["template"]["spec"]["containers"][0]["command"]
    assert cmd[cmd.index("--nnodes") + 1] == "3" and "ccfd-engine-0.ccfd-engine:29400" in cmd
    bad = copy.deepcopy(ms)
    c = next(m for m in bad if m["kind"] == "StatefulSet" and m["metadata"]["name"] == "ccfd-engine")
    c["spec"]["template"]["spec"]["containers"][0]["command"] = [x for x in cmd if x not in ("--nnodes", "3")]
    bad = [m for m in bad if not (m["kind"] == "Service" and m["metadata"]["name"] == "ccfd-engine")]
    probs = "\n".join(validate(bad))
    assert "without a shared rendezvous" in probs and "no headless Service" in probs
    from ccfd_demo_summit_amd.operator import local_commands
    d["spec"]["engine"].update(gpusPerNode=2)
    n, argv_of, env_of, _ = local_commands(parse(d), port_offset=50)["engine"]
    assert n == 3 and [env_of(r)["HIP_VISIBLE_DEVICES"] for r in range(3)] == ["0,1", "2,3", "4,5"]
    a0, a2 = argv_of(0), argv_of(2)
    assert a0[a0.index("--rdzv-endpoint") + 1] == a2[a2.index("--rdzv-endpoint") + 1] == "127.0.0.1:29550"


def test_every_long_running_container_has_health_probes():
    """Deployments / StatefulSets carry readiness + liveness probes on the service's own health
    route (engine /health/ping :8091, KIE /services/rest/server :8090, kafka tcp :9092, ...)."""
    ms = render(load(str(CR)))
    seen = {}
    for m in ms:
        if m["kind"] not in ("Deployment", "StatefulSet"):
            continue
        for c in m["spec"]["template"]["spec"]["containers"]:
            assert "readinessProbe" in c and "livenessProbe" in c, (m["metadata"]["name"], c["name"])
            seen[c["name"]] = c["livenessProbe"]
    assert seen["engine"]["httpGet"] == {"path": "/health/ping", "port": 8091}
    assert seen["kie"]["httpGet"]["path"] == "/services/rest/server"
    assert seen["kafka"]["tcpSocket"] == {"port": 9092}
    bad = copy.deepcopy(ms)
    eng = next(m for m in bad if m["metadata"]["name"] == "ccfd-engine")
    eng["spec"]["template"]["spec"]["containers"][0]["livenessProbe"]["httpGet"]["port"] = 9999
    assert any("livenessProbe on undeclared port 9999" in p for p in validate(bad))


def test_validate_reports_broken_manifests():
    ms = render(load(str(CR)))
    bad = copy.deepcopy(ms)
    by = {(m["kind"], m["metadata"]["name"]): m for m in bad}
    by[("StatefulSet", "ccd-service")]["spec"]["selector"]["matchLabels"]["app"] = "nope"
    by[("Service", "modelfull-modelfull")]["spec"]["ports"][0]["targetPort"] = 1234
    eng = by[("StatefulSet", "ccfd-engine")]["spec"]["template"]["spec"]["containers"][0]
    eng["resources"]["limits"]["amd.com/gpu"] = 4
    by[("Deployment", "ccfd-notification-service")]["spec"]["template"]["spec"]["containers"][0]["env"] = \
        [{"name": "WHATEVER", "value": "1"}]
    probs = "\n".join(validate(bad))
    assert "does not match template labels" in probs
    assert "targetPort 1234" in probs
    assert "8 ranks for 4 GPUs" in probs
    assert "unknown env key WHATEVER" in probs


SLEEPER = [sys.executable, "-c", "import time; time.sleep(120)"]


def test_local_operator_reconciles_restarts_scales_and_stops(tmp_path):
    spec = FraudDetectionSpec()
    cmds = {"router": (2, lambda r: SLEEPER, {}), "kie": (1, lambda r: SLEEPER, {})}
    status = tmp_path / "status.json"
    op = LocalOperator(spec, status_path=str(status), commands=cmds, grace_s=5, backoff_s=0.0, log=lambda m: None)
    try:
        st = op.reconcile()
        assert st["router"]["ready"] == 2 and st["kie"]["ready"] == 1
        victim = op.services["router"].replicas[1].proc
        os.killpg(victim.pid, signal.SIGKILL)
        victim.wait()
        st = op.reconcile()
        assert st["router"]["ready"] == 2 and st["router"]["restarts"] == 1
        assert op.services["router"].replicas[1].proc.pid != victim.pid
        # a new CR generation scales the router down to 1 and removes kie
        op._commands = {"router": (1, lambda r: SLEEPER, {})}
        op.generation += 1
        st = op.reconcile()
        assert st == {"router": {"desired": 1, "ready": 1, "restarts": 1,
                                 "pids": [op.services["router"].replicas[0].proc.pid]}}
        import json
        doc = json.loads(status.read_text())
        assert doc["observedGeneration"] == 2 and doc["services"]["router"]["ready"] == 1
    finally:
        procs = [rep.proc for st in op.services.values() for rep in st.replicas.values()]
        op.shutdown()
    assert all(p.poll() is not None for p in procs)


def test_local_operator_jobs_run_to_completion():
    """producer / training are Jobs: a successful exit completes them, a failure restarts."""
    ok = [sys.executable, "-c", "pass"]
    bad_then_ok = [sys.executable, "-c", "import os,sys; p='/tmp/ccfd_op_job_marker_%d' % os.getppid(); "
                   "sys.exit(0) if os.path.exists(p) else (open(p,'w').close(), sys.exit(3))"]
    op = LocalOperator(FraudDetectionSpec(), commands={"producer": (1, lambda r: ok, {}),
                                                       "training": (1, lambda r: bad_then_ok, {})},
                       grace_s=5, backoff_s=0.0, log=lambda m: None)
    try:
        for _ in range(40):
            st = op.reconcile()
            if st["producer"].get("succeeded") == 1 and st["training"].get("succeeded") == 1:
                break
            time.sleep(0.1)
        assert st["producer"]["succeeded"] == 1 and st["producer"]["restarts"] == 0
        assert st["training"]["succeeded"] == 1 and st["training"]["restarts"] == 1
        assert op.reconcile()["producer"]["ready"] == 0          # not restarted after success
    finally:
        op.shutdown()
        try:
            os.remove(f"/tmp/ccfd_op_job_marker_{os.getpid()}")
        except OSError:
            pass


def test_local_operator_rolls_a_changed_template_a_quarter_at_a_time():
    """A CR generation that changes a service's command replaces its replicas with at most
    max(1, n // 4) unavailable at a time, without counting them as crash restarts."""
    version = {"v": "1"}
    cmd = lambda r: [sys.executable, "-c", "import time; time.sleep(120)", version["v"]]
    op = LocalOperator(FraudDetectionSpec(), commands={"kie": (8, cmd, {})}, grace_s=5, backoff_s=0.0,
                       log=lambda m: None)
    try:
        op.reconcile()
        old = set(op.status()["services"]["kie"]["pids"])
        version["v"] = "2"
        op.generation += 1
        rolled = []
        for _ in range(10):
            st = op.reconcile()["kie"]
            rolled.append(st.get("rollouts", 0))
            if rolled[-1] == 8:
                break
        assert rolled[:4] == [2, 4, 6, 8]                       # 8 // 4 = 2 replaced per pass
        assert st["ready"] == 8 and st["restarts"] == 0 and not (set(st["pids"]) & old)
        assert op.reconcile()["kie"]["rollouts"] == 8           # converged: nothing more to roll
    finally:
        op.shutdown()


def test_local_operator_liveness_probe_restarts_a_hung_replica():
    """A replica that is running but never answers its health route is killed after
    ``liveness_failures`` probes and restarted; one that answers is reported healthy."""
    port = random.randint(41000, 49000)
    http = [sys.executable, "-c", "import http.server as h; h.HTTPServer(('127.0.0.1', %d), "
            "h.SimpleHTTPRequestHandler).serve_forever()" % port]
    cmds = {"hung": (1, lambda r: SLEEPER, {}, (lambda r: ("tcp", "127.0.0.1", port + 1), 0)),
            "web": (1, lambda r: http, {}, (lambda r: ("http", f"http://127.0.0.1:{port}/"), 0))}
    op = LocalOperator(FraudDetectionSpec(), workdir="/tmp", commands=cmds, grace_s=5, backoff_s=0.0,
                       log=lambda m: None, liveness_failures=3)
    try:
        first = None
        for _ in range(60):
            st = op.reconcile()
            first = first or op.services["hung"].replicas[0].proc.pid
            if st["hung"]["restarts"] >= 1 and st["web"]["healthy"] == 1:
                break
            time.sleep(0.1)
        assert st["hung"]["restarts"] >= 1 and st["hung"]["healthy"] == 0
        assert op.services["hung"].replicas[0].proc.pid != first
        assert st["web"]["healthy"] == 1 and st["web"]["restarts"] == 0
    finally:
        op.shutdown()


def test_local_commands_probe_the_rendered_health_routes():
    from ccfd_demo_summit_amd.operator import local_commands
    cmds = local_commands(load(str(CR)), port_offset=100)
    assert cmds["engine"][3][0](1) == ("http", "http://127.0.0.1:8207/health/ping")
    assert cmds["kie"][3][0](0) == ("http", "http://127.0.0.1:8190/services/rest/server")
    assert cmds["kafka"][3][0](0)[0] == "tcp" and cmds["producer"][3] is None


def _free_offset(bases, tries=200):
    import socket
    for _ in range(tries):
        off = random.randint(20000, 40000)
        ok = True
        for b in bases:
            sk = socket.socket()
            try:
                sk.bind(("127.0.0.1", b + off))
            except OSError:
                ok = False
            finally:
                sk.close()
            if not ok:
                break
        if ok:
            return off
    raise RuntimeError("no free port offset")


def test_local_operator_brings_up_a_working_kafka_cluster(tmp_path):
    """Only the CR's kafka section deployed: the operator starts the replicated kafka-lite
    cluster (a 3-member controller quorum + 3 broker processes) and a Kafka client produces to /
    fetches from it through the bootstrap list."""
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    d = _doc()
    for k in ("engine", "seldon", "usertask", "kie", "notifier", "producer", "monitoring"):
        d["spec"][k]["deploy"] = False
    d["spec"]["kafka"].update(brokers=3, partitions=6)
    spec = parse(d)
    off = _free_offset([9092, 9093, 9094, 9404, 9405, 9406, 9290, 9291, 9292])   # parallel workers: never a taken port
    op = LocalOperator(spec, workdir=str(ROOT), commands=None, grace_s=5, log=lambda m: None, port_offset=off,
                       state_dir=str(tmp_path / "state"))
    try:
        t0 = time.time()
        while time.time() - t0 < 60:
            st = op.reconcile()
            if st["kafka"]["ready"] == 3 and st["kafka-controller"]["ready"] == 3:
                break
            time.sleep(0.5)
        assert st["kafka"]["ready"] == 3 and st["kafka-controller"]["ready"] == 3
        bootstrap = ",".join(f"127.0.0.1:{9092 + off + i}" for i in range(3))
        kb = KafkaBroker(bootstrap, connect_wait_s=60.0)
        try:
            kb.create_topic("odh-demo", 6)
            for p in range(6):
                kb.produce("odh-demo", f"tx-{p}".encode(), partition=p)
            c = kb.consumer("g", ["odh-demo"])
            got = []
            t0 = time.time()
            while len(got) < 6 and time.time() - t0 < 30:
                got += [r.value for r in c.poll(max_records=100)]
            assert sorted(got) == sorted(f"tx-{p}".encode() for p in range(6))
            kb.metadata(["odh-demo"])
            leaders = {n for (t, _p), n in kb._leaders.items() if t == "odh-demo"}
            assert len(leaders) == 3                                           # leadership spread over 3 nodes
        finally:
            kb.close()
    finally:
        op.shutdown()


def _launch_argvs(cmd):
    """Every `python -m ccfd_demo_summit_amd.launch ...` invocation inside a container command
    (a supervised one nests the child's after `--`)."""
    out = []
    for i in range(len(cmd) - 1):
        if cmd[i] == "-m" and cmd[i + 1] == "ccfd_demo_summit_amd.launch":
            rest = cmd[i + 2:]
            nxt = [j for j in range(len(rest) - 1) if rest[j] == "-m" and rest[j + 1] == "ccfd_demo_summit_amd.launch"]
            out.append(rest[:nxt[0]] if nxt else rest)
    return out


@pytest.mark.parametrize("variant", ["default", "wide"])
def test_every_rendered_launch_command_parses(variant):
    """each rendered container's launcher argv is accepted by the launcher's
    own parser, and kafka-lite keeps its durability options (a pod that crash-loops on
    'unrecognized arguments' never shows up in the local-operator tests)."""
    from ccfd_demo_summit_amd.launch.__main__ import parse_args
    d = _doc()
    if variant == "wide":
        d["spec"]["router"] = {"deploy": True, "replicas": 2}
        d["spec"]["training"] = {"deploy": True, "workers": 2, "model": "mlp", "gpus": 1}
        d["spec"]["engine"].update(nodes=2, gpusPerNode=4)
    seen = set()
    for m in render(parse(d)):
        tmpl = m.get("spec", {}).get("template", {}).get("spec", {})
        if m["kind"] == "CronJob":
            tmpl = m["spec"]["jobTemplate"]["spec"]["template"]["spec"]
        for c in tmpl.get("containers", []) + tmpl.get("initContainers", []):
            for argv in _launch_argvs(c.get("command", []) + c.get("args", [])):
                a = parse_args(argv)          # SystemExit on an unknown option
                seen.add(a.service)
                if a.service == "kafka-lite":
                    assert a.data_dir == "/var/lib/kafka-lite" and a.fsync in ("always", "interval", "never")
    assert {"kafka-lite", "kie", "engine", "notifier", "producer"} <= seen, seen


def test_launcher_forwards_kafka_lite_durability(monkeypatch):
    from ccfd_demo_summit_amd.launch import __main__ as L
    got = {}
    import ccfd_demo_summit_amd.ingest.kafka_lite as K
    monkeypatch.setattr(K, "main", lambda argv: got.setdefault("argv", argv))
    a = L.parse_args(["kafka-lite", "--nodes", "3", "--data-dir", "/x", "--fsync", "always", "--metrics-port", "0"])
    L.cmd_kafka_lite(a, L.load_config(None, environ={}))
    argv = got["argv"]
    assert argv[argv.index("--data-dir") + 1] == "/x" and argv[argv.index("--fsync") + 1] == "always"
    assert argv[argv.index("--metrics-port") + 1] == "0" and argv[argv.index("--nodes") + 1] == "3"


def test_kie_shards_render_a_statefulset_and_shard_urls():
    """kie.shards: a StatefulSet of shard pods (journal PVC each), a headless service for the
    per-pod names, KIE_SERVER_URL as a {shard} template; replicas > 1 is refused (an unsharded
    KIE replica would keep state of its own)."""
    from ccfd_demo_summit_amd.process.sharding import kie_urls
    d = _doc()
    d["spec"]["kie"] = {"deploy": True, "shards": 4}
    ms = render(parse(d))
    assert validate(ms) == []
    by = {(m["kind"], m["metadata"]["name"]): m for m in ms}
    sts = by[("StatefulSet", "ccd-service")]
    assert sts["spec"]["replicas"] == 4 and sts["spec"]["serviceName"] == "ccd-service-shards"
    assert sts["spec"]["volumeClaimTemplates"][0]["metadata"]["name"] == "journal"
    assert by[("Service", "ccd-service-shards")]["spec"]["clusterIP"] == "None"
    env = by[("ConfigMap", "ccfd-env")]["data"]
    assert env["CCFD_KIE_SHARDS"] == "4"
    assert kie_urls(env["KIE_SERVER_URL"], 4)[3] == "http://ccd-service-3.ccd-service-shards:8090"
    d["spec"]["kie"] = {"deploy": True, "replicas": 2}
    with pytest.raises(SpecError, match="kie.shards"):
        parse(d)
    # the engine's hand-off DLQ lives on a claim of its own, not an emptyDir
    eng = by[("StatefulSet", "ccfd-engine")]
    assert eng["spec"]["volumeClaimTemplates"][0]["metadata"]["name"] == "handoff-dlq"
    assert "volumes" not in eng["spec"]["template"]["spec"]
