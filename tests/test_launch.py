"""Launcher + supervisor (restart-on-crash, crash-loop give-up, graceful stop)."""
import os
import subprocess
import sys

from ccfd_demo_summit_amd.launch.supervisor import supervise


def test_supervisor_restarts_until_success(tmp_path):
    marker = tmp_path / "count"
    script = tmp_path / "flaky.py"
    script.write_text(
        "import sys, pathlib\n"
        f"p = pathlib.Path({str(marker)!r})\n"
        "n = int(p.read_text()) if p.exists() else 0\n"
        "p.write_text(str(n + 1))\n"
        "sys.exit(0 if n >= 2 else 3)\n")
    logs = []
    rc = supervise([sys.executable, str(script)], max_restarts=5, backoff_s=0.01, log=logs.append)
    assert rc == 0
    assert marker.read_text() == "3"
    assert len(logs) == 2


def test_supervisor_gives_up_on_crash_loop():
    logs = []
    rc = supervise([sys.executable, "-c", "import sys; sys.exit(7)"], max_restarts=2, backoff_s=0.01,
                   log=logs.append)
    assert rc == 7
    assert "crash loop" in logs[-1]


def test_launch_help_and_demo():
    env = dict(os.environ, CCFD_NO_NUMA_BIND="1")
    out = subprocess.run([sys.executable, "-m", "ccfd_demo_summit_amd.launch", "--help"], capture_output=True,
                         text=True, env=env, timeout=120)
    assert out.returncode == 0 and "kafka-lite" in out.stdout
    out = subprocess.run([sys.executable, "-m", "ccfd_demo_summit_amd.launch", "demo", "--device", "cpu",
                          "--seconds", "1", "--batch", "500", "--port", "0"],
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert '"consumed"' in out.stdout


def test_launch_options_after_service_name_are_parsed():
    from ccfd_demo_summit_amd.launch.__main__ import parse_args
    a = parse_args(["engine", "--port", "18091", "--host", "127.0.0.1", "--watch-model", "m.safetensors"])
    assert (a.service, a.port, a.host, a.watch_model, a.cmd) == ("engine", 18091, "127.0.0.1", "m.safetensors", [])
    a = parse_args(["--port", "1", "kafka-lite"])
    assert a.port == 1 and a.service == "kafka-lite"
    a = parse_args(["supervise", "--max-restarts", "3", "--", "python", "-c", "print(1)", "--port", "9"])
    assert a.max_restarts == 3 and a.cmd == ["python", "-c", "print(1)", "--port", "9"] and a.port is None


def test_elastic_service_ranks_score_topic_exactly_once():
    """`launch elastic` ranks (real processes) share a TCPStore and a kafka-lite broker:
    the topic is scored once (committed counts) and every rank's X2 totals -- reduced over
    the membership generation's process group -- equal the global counts."""
    import datetime
    import os
    import socket
    import time

    import torch.distributed as dist

    from ccfd_demo_summit_amd.ingest import ProducerConfig, TransactionProducer
    from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteServer
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    from ccfd_demo_summit_amd.parallel.elastic import PartitionLeases

    def free_port():
        s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close()
        return p
    sport = free_port()
    store = dist.TCPStore("127.0.0.1", sport, 1, True, timeout=datetime.timedelta(seconds=60), wait_for_workers=False)
    lite = KafkaLiteServer("127.0.0.1", 0, default_partitions=4).start_in_thread()
    kb = KafkaBroker(lite.bootstrap)
    kb.create_topic("odh-demo", 4)
    TransactionProducer(kb, ProducerConfig(fmt="json", batch=500, seed=5)).produce(3000)
    env = dict(os.environ, BROKER_URL=lite.bootstrap, KAFKA_TOPIC="odh-demo")
    mport = free_port()
    procs = [subprocess.Popen([sys.executable, "-m", "ccfd_demo_summit_amd.launch", "elastic", "--store",
                               f"127.0.0.1:{sport}", "--rank", str(r), "--world", "2", "--partitions", "4",
                               "--device", "cpu", "--kie", "local", "--ttl", "1.0", "--host", "127.0.0.1",
                               "--port", str(mport)], env=env)
             for r in range(2)]
    try:
        reader = PartitionLeases(store, 99, 2, 4, ttl_s=1.0)
        t0 = time.time()
        rows = fraud = 0
        while time.time() - t0 < 180:
            rows, fraud = reader.global_counts()
            x2 = [store.get(f"x2/{r}").decode() if store.check([f"x2/{r}"]) else "" for r in range(2)]
            if rows == 3000 and all(x.endswith(f"|{rows},{fraud}") for x in x2):
                break
            assert all(p.poll() is None for p in procs), "an elastic rank exited"
            time.sleep(0.1)
        assert rows == 3000
        assert all(x.split("|")[1] == "0,1" and x.endswith(f"|3000,{fraud}") for x in x2), x2
    finally:
        store.set("stop", "1")
        for p in procs:
            try:
                p.wait(30)
            except subprocess.TimeoutExpired:
                p.kill()
        kb.close()
        lite.stop()


def test_rule_safe_row_format():
    """Device routing rules see what the reference's Drools rules see: rules over
    V-columns move off W64's bf16 V-columns onto f32 rows; Time / Amount rules stay on W64 (those
    columns are f32 there); binned G20 / G32 rows only serve proba-only rules."""
    from ccfd_demo_summit_amd.launch.engine_service import rule_safe_row_format
    from ccfd_demo_summit_amd.router.rules import RuleSet
    v = RuleSet.parse("when proba >= 0.5 or V17 < -2.5 then fraud\notherwise standard")
    amt = RuleSet.parse("when proba >= 0.5 and amount > 100 then fraud\notherwise standard")
    p = RuleSet.parse("when proba >= 0.7 then fraud\notherwise standard")
    assert rule_safe_row_format("mlp", "w64", v)[0] == "f32"
    assert rule_safe_row_format("mlp", "w64", amt) == ("w64", "")
    assert rule_safe_row_format("mlp", "w64", p) == ("w64", "")
    assert rule_safe_row_format("gbdt", "g20", amt)[0] == "f32"
    assert rule_safe_row_format("gbdt", "g20", p) == ("g20", "")
    assert rule_safe_row_format("mlp", "f32", v) == ("f32", "")
