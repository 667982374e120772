"""Produce-only throughput of the replicated kafka-lite: a controller, N broker
processes (durable), P producer processes (TXB1 by default) for T seconds, no engine.  Runs on
a CPU box; prints one JSON line with the producers' total tx/s and each producer's own line.

    python bench/experiments/replicated_produce.py --producers 4 --seconds 10 --acks -1

``--probe-ms M`` adds a visibility probe on its own topic: one small acks=all record every M ms,
and a long-polling consumer that reports produce -> visible-to-consumers (the HW covers it)
and produce -> acked latencies, p50 / p99 / max, under whatever load the producers add.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "bench"))
sys.path.insert(0, str(ROOT))
from deploy_topology import free_ports, wait_port  # noqa: E402

PY = sys.executable


class _Probe:
    """acks=all records on topic ``probe`` every ``period_ms``; a second connection long-polls
    the partition and stamps when each offset becomes visible to consumers."""

    def __init__(self, url: str, period_ms: float, seconds: float):
        import threading
        from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
        self.sent, self.acked, self.seen = {}, {}, {}
        self.prod = KafkaBroker(url, connect_wait_s=30.0)
        self.cons = KafkaBroker(url, connect_wait_s=30.0)
        self.period, self.seconds = period_ms / 1e3, seconds
        self.stop = threading.Event()
        self.tp = threading.Thread(target=self._produce, daemon=True)
        self.tc = threading.Thread(target=self._consume, daemon=True)
        self.tc.start()
        self.tp.start()

    def _produce(self):
        t_end = time.monotonic() + self.seconds
        k = 0
        while time.monotonic() < t_end:
            t0 = time.perf_counter()
            self.sent[k] = t0
            self.prod.produce_batch("probe", 0, [b"%d" % k], acks=-1)
            self.acked[k] = time.perf_counter()
            k += 1
            time.sleep(max(0.0, self.period - (time.perf_counter() - t0)))
        time.sleep(0.5)
        self.stop.set()

    def _consume(self):
        off = 0
        while not self.stop.is_set():
            for r in self.cons.fetch("probe", 0, off, max_wait_ms=200):
                self.seen.setdefault(int(r.value), time.perf_counter())
                off = max(off, r.offset + 1)

    def join(self):
        import numpy as np
        self.tp.join()
        self.tc.join(5)
        self.prod.close()
        self.cons.close()

        def q(d):
            v = np.array([(d[k] - self.sent[k]) * 1e3 for k in d if k in self.sent])
            if not len(v):
                return None
            return {"n": int(len(v)), "p50_ms": round(float(np.percentile(v, 50)), 3),
                    "p99_ms": round(float(np.percentile(v, 99)), 3), "max_ms": round(float(v.max()), 3)}
        t0 = min(self.sent.values()) if self.sent else 0.0
        slow = sorted((round((self.sent[k] - t0) * 1e3, 1), round((self.acked[k] - self.sent[k]) * 1e3, 2))
                      for k in self.acked if self.acked[k] - self.sent[k] > 0.005)
        return {"visible": q(self.seen), "acked": q(self.acked), "sent": len(self.sent),
                "slow_acks_at_ms": slow[:40]}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--brokers", type=int, default=3)
    ap.add_argument("--producers", type=int, default=4)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--acks", type=int, default=-1)
    ap.add_argument("--max-in-flight", type=int, default=5)
    ap.add_argument("--fmt", default="txb1")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--single", action="store_true", help="the single-process durable broker instead")
    ap.add_argument("--rf", type=int, default=3, help="replication factor of the topic (controller --rf)")
    ap.add_argument("--retention-batches", type=int, default=500, help="per partition (the deploy harness's default)")
    ap.add_argument("--probe-ms", type=float, default=0.0, help="visibility probe period (0: off)")
    a = ap.parse_args(argv)
    kdir = tempfile.mkdtemp(prefix="ccfd-repl-produce-")
    ctl, = free_ports(1)
    base, = free_ports(1, a.brokers)
    mbase, = free_ports(1, a.brokers)
    env = dict(os.environ, PYTHONPATH=str(ROOT), CCFD_KAFKA_BACKEND="kafka",
               CCFD_KAFKA_PARTITIONS=str(a.partitions),
               BROKER_URL=",".join(f"127.0.0.1:{base + i}" for i in range(a.brokers)))
    procs = []
    names = []
    logs = []

    def start(name, cmd):
        names.append(name)
        f = open(Path(kdir) / f"{name}.log", "w")
        logs.append(f)
        procs.append(subprocess.Popen(cmd, env=env, stdout=f, stderr=subprocess.STDOUT))
    try:
        K = "ccfd_demo_summit_amd.ingest."
        if a.single:
            start("kafka-lite", [PY, "-m", K + "kafka_lite", "--host", "127.0.0.1", "--port", str(base),
                                 "--nodes", str(a.brokers), "--partitions", str(a.partitions),
                                 "--metrics-port", str(mbase), "--data-dir", kdir + "/single",
                                 "--retention-batches", str(a.retention_batches)])
        else:
            start("controller", [PY, "-m", K + "kafka_controller", "--host", "127.0.0.1", "--port", str(ctl),
                                 "--brokers", str(a.brokers), "--rf", str(a.rf), "--data-dir", kdir + "/ctl"])
            wait_port(ctl, 60)
            for i in range(a.brokers):
                start(f"broker{i + 1}", [PY, "-m", K + "kafka_lite", "--host", "127.0.0.1", "--port", str(base + i),
                                         "--node-id", str(i + 1), "--controller", f"http://127.0.0.1:{ctl}",
                                         "--metrics-port", str(mbase + i), "--data-dir", f"{kdir}/b{i + 1}",
                                         "--retention-batches", str(a.retention_batches)])
        for i in range(a.brokers):
            wait_port(base + i, 60)
        from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
        kb = KafkaBroker(env["BROKER_URL"], connect_wait_s=60.0)
        kb.create_topic("odh-demo", a.partitions)
        if a.probe_ms > 0:
            kb.create_topic("probe", 1)
        kb.close()
        probe = _Probe(env["BROKER_URL"], a.probe_ms, a.seconds) if a.probe_ms > 0 else None
        prods = []
        for i in range(a.producers):
            f = open(Path(kdir) / f"producer{i}.log", "w+")
            logs.append(f)
            prods.append((subprocess.Popen(
                [PY, "-m", "ccfd_demo_summit_amd.launch", "producer", "--fmt", a.fmt, "--batch", str(a.batch), "--count", "0",
                 "--seconds", str(a.seconds), "--acks", str(a.acks), "--max-in-flight", str(a.max_in_flight),
                 "--id-base", str((i + 1) << 40), "--seed-offset", str(i * 101)],
                env=env, stdout=f, stderr=subprocess.STDOUT), f))
        probe_res = probe.join() if probe is not None else None
        res = []
        for p, f in prods:
            p.wait(timeout=a.seconds + 180)
            f.seek(0)
            lines = [ln for ln in f.read().splitlines() if ln.startswith("{")]
            res.append(json.loads(lines[-1]) if lines else {"error": "no result"})
        import psutil
        cpu = {}
        for name, p in zip(names, procs):
            try:
                t = psutil.Process(p.pid).cpu_times()
                cpu[name] = round(t.user + t.system, 1)
            except psutil.Error:
                cpu[name] = None
        tot = sum(r.get("produced", 0) for r in res)
        secs = max([r.get("seconds", a.seconds) for r in res] or [a.seconds])
        print(json.dumps({"tx_s": round(tot / secs, 1), "produced": tot, "producers": a.producers,
                          "acks": a.acks, "max_in_flight": a.max_in_flight, "replicated": not a.single, "rf": a.rf,
                          "cpu_s": cpu, "probe": probe_res, "per_producer": res}))
    except BaseException:
        for f in logs:
            f.flush()
        for lp in sorted(Path(kdir).glob("*.log")):
            print(f"== {lp.name}\n" + lp.read_text()[-2000:], file=sys.stderr)
        raise
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        for f in logs:
            f.close()
        import shutil
        if os.environ.get("CCFD_KEEP_LOGS"):            # broker / producer logs kept for reading
            keep = Path(os.environ["CCFD_KEEP_LOGS"])
            keep.mkdir(parents=True, exist_ok=True)
            for lp in Path(kdir).glob("*.log"):
                shutil.copy(lp, keep / lp.name)
        shutil.rmtree(kdir, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
