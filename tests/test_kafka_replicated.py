"""Replicated, multi-process kafka-lite (the reference's 3-broker Strimzi
cluster, deploy/frauddetection_cr.yaml:75-77, and its under-replicated / offline panels,
deploy/grafana/Kafka.json:271,347): three broker PROCESSES each leading a third of the
partitions, followers replicating by fetch, acks=all against the ISR, leader fail-over by
the controller.  A broker is SIGKILLed mid-stream: no acknowledged record is lost or
duplicated, the under-replicated gauge rises and returns to 0 once the broker is back and
caught up."""
import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
import urllib.request
from pathlib import Path

import pytest

from ccfd_demo_summit_amd.ingest.kafka_controller import ControllerState
from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker, decode_record_batches, encode_record_batch

ROOT = Path(__file__).resolve().parents[1]


def _free_ports(n):
    out = []
    socks = []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        out.append(s.getsockname()[1])
        socks.append(s)
    for s in socks:
        s.close()
    return out


def _wait(port, t=60):
    t0 = time.time()
    while time.time() - t0 < t:
        try:
            socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
            return
        except OSError:
            time.sleep(0.1)
    raise TimeoutError(port)


def _text(url):
    with urllib.request.urlopen(url, timeout=5) as r:
        return r.read().decode()


def _gauge(text, name):
    for line in text.splitlines():
        if line.startswith(name):
            return float(line.rsplit(" ", 1)[1])
    return None


def test_controller_elects_the_highest_leo_isr_member_and_fences_restarts():
    now = [0.0]
    st = ControllerState(None, session_s=1.0, clock=lambda: now[0])
    for n in (1, 2, 3):
        st.heartbeat(n, "h", 9000 + n, f"inc{n}", {}, [])
    st.create_topic("t", 3)
    p0 = st.parts["t/0"]
    assert p0["leader"] == 1 and sorted(p0["isr"]) == [1, 2, 3]
    # node 1 dies; the followers report different LEOs: the longer log wins
    now[0] = 1.2
    st.heartbeat(2, "h", 9002, "inc2", {"t/0": 90}, [])
    st.heartbeat(3, "h", 9003, "inc3", {"t/0": 100}, [])
    now[0] = 1.6
    st.tick()                                           # node 1 silent > session: failed
    assert st.parts["t/0"]["leader"] == -1 and 1 not in st.parts["t/0"]["isr"]
    now[0] = 1.7
    st.heartbeat(2, "h", 9002, "inc2", {"t/0": 90}, [])
    st.heartbeat(3, "h", 9003, "inc3", {"t/0": 100}, [])
    assert st.parts["t/0"]["leader"] == 3 and st.parts["t/0"]["epoch"] == 1
    # a stale ISR proposal (old epoch) is refused; the leader's current one applies
    st.heartbeat(3, "h", 9003, "inc3", {}, [{"tp": "t/0", "epoch": 0, "isr": [3]}])
    assert sorted(st.parts["t/0"]["isr"]) == [2, 3]
    st.heartbeat(3, "h", 9003, "inc3", {}, [{"tp": "t/0", "epoch": 1, "isr": [3]}])
    assert st.parts["t/0"]["isr"] == [3] and st.under_replicated() >= 1
    # node 3 restarts (new incarnation): fenced -- its leadership is failed over first, and
    # as the sole ISR member it is the only one that can take it back
    st.heartbeat(3, "h", 9003, "inc3-b", {"t/0": 100}, [])
    assert st.parts["t/0"]["leader"] == 3 and st.parts["t/0"]["epoch"] == 2
    # committed offsets are monotone and survive in the state
    st.commit("g", [("t", 0, 10), ("t", 0, 5)])
    assert st.fetch_offsets("g", [("t", 0), ("t", 1)]) == [10, -1]


@pytest.fixture()
def cluster(tmp_path):
    yield from _cluster(tmp_path, [])


@pytest.fixture()
def small_retention_cluster(tmp_path):
    yield from _cluster(tmp_path, ["--retention-batches", "20"])


def _cluster(tmp_path, extra):
    ports = _free_ports(7)
    cport, bports, mports = ports[0], ports[1:4], ports[4:7]
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    procs = {}

    def start(name, cmd):
        procs[name] = subprocess.Popen(cmd, cwd=str(ROOT), env=env, stdout=subprocess.DEVNULL,
                                       stderr=subprocess.DEVNULL, start_new_session=True)

    def broker_cmd(k):
        return [sys.executable, "-m", "ccfd_demo_summit_amd.ingest.kafka_lite", "--host", "127.0.0.1",
                "--port", str(bports[k - 1]), "--node-id", str(k), "--controller", f"http://127.0.0.1:{cport}",
                "--metrics-port", str(mports[k - 1]), "--data-dir", str(tmp_path / f"b{k}"), "--fsync", "interval"] + extra
    start("ctl", [sys.executable, "-m", "ccfd_demo_summit_amd.ingest.kafka_controller", "--host", "127.0.0.1",
                  "--port", str(cport), "--data-dir", str(tmp_path / "ctl"), "--session-s", "1.0",
                  "--brokers", "3"])
    _wait(cport)
    for k in (1, 2, 3):
        start(f"b{k}", broker_cmd(k))
    for p in bports:
        _wait(p)
    c = {"cport": cport, "bports": bports, "mports": mports, "procs": procs, "start": start,
         "broker_cmd": broker_cmd}
    yield c
    for p in procs.values():
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait(10)


def test_broker_sigkill_loses_no_acknowledged_record(cluster):
    boot = ",".join(f"127.0.0.1:{p}" for p in cluster["bports"])
    deadline = time.time() + 30
    while True:
        md = json.loads(_text(f"http://127.0.0.1:{cluster['cport']}/metadata"))
        if len(md["nodes"]) == 3 or time.time() > deadline:
            break
        time.sleep(0.1)
    kb = KafkaBroker(boot, idempotent=True, connect_wait_s=10)
    kb.RETRIES = 14                                      # rides out a fail-over (~1 s)
    kb.create_topic("odh-demo", 6)
    acked = {}
    stop = threading.Event()
    errors = []

    def produce():
        k = 0
        while not stop.is_set():
            p = k % 6
            vals = [b"%d-%d" % (k, i) for i in range(50)]
            try:
                kb.produce_raw("odh-demo", p, encode_record_batch(vals), acks=-1)
            except Exception as e:                       # noqa: BLE001
                errors.append(repr(e))
                time.sleep(0.05)
                continue                                 # (not acknowledged: not counted)
            for v in vals:
                acked[v] = p
            k += 1
    th = threading.Thread(target=produce, daemon=True)
    th.start()
    time.sleep(1.5)
    victim = 2
    os.killpg(cluster["procs"][f"b{victim}"].pid, signal.SIGKILL)     # a crashed broker pod
    cluster["procs"][f"b{victim}"].wait(10)
    t_kill = time.time()
    seen_under = 0.0
    while time.time() - t_kill < 3.0:
        for mp in (cluster["mports"][0], cluster["mports"][2]):
            try:
                seen_under = max(seen_under, _gauge(_text(f"http://127.0.0.1:{mp}/metrics"),
                                                    "kafka_server_replicamanager_underreplicatedpartitions") or 0)
            except OSError:
                pass
        time.sleep(0.2)
    n_during = len(acked)
    cluster["start"](f"b{victim}", cluster["broker_cmd"](victim))             # restarted from disk
    _wait(cluster["bports"][victim - 1])
    time.sleep(2.0)
    stop.set()
    th.join(30)
    assert seen_under >= 1, "under-replicated partitions never reported while a broker was down"
    assert len(acked) > n_during > 0
    # caught up: every ISR full again, under-replicated back to 0 on every broker
    deadline = time.time() + 30
    while time.time() < deadline:
        md = json.loads(_text(f"http://127.0.0.1:{cluster['cport']}/metadata"))
        under = [_gauge(_text(f"http://127.0.0.1:{mp}/metrics"), "kafka_server_replicamanager_underreplicatedpartitions")
                 for mp in cluster["mports"]]
        if all(len(v["isr"]) == 3 for v in md["parts"].values() if v) and not any(under):
            break
        time.sleep(0.3)
    assert all(len(v["isr"]) == 3 for v in md["parts"].values()), md["parts"]
    assert not any(under), under
    # every acknowledged record is there exactly once
    got = {}
    for p in range(6):
        off, end = 0, kb.end_offset("odh-demo", p)
        while off < end:
            _err, _hw, raw = kb.fetch_raw("odh-demo", p, off)
            recs = [r for r in decode_record_batches(raw, "odh-demo", p) if r.offset >= off]
            for r in recs:
                got[r.value] = got.get(r.value, 0) + 1
            off = recs[-1].offset + 1 if recs else end
    missing = [v for v in acked if v not in got]
    dups = [v for v, n in got.items() if n > 1]
    assert not missing, (len(missing), missing[:5])
    assert not dups, dups[:5]
    kb.close()


def test_pipelined_idempotent_producer_through_a_leader_failover(cluster):
    """max.in.flight 5 (requests pipelined per leader connection) under acks=all, with the
    leader of half the partitions SIGKILLed mid-stream: after flush() every record is stored
    exactly once, in order per partition (re-sent batches keep their sequence numbers)."""
    boot = ",".join(f"127.0.0.1:{p}" for p in cluster["bports"])
    deadline = time.time() + 30
    while len(json.loads(_text(f"http://127.0.0.1:{cluster['cport']}/metadata"))["nodes"]) < 3:
        assert time.time() < deadline
        time.sleep(0.1)
    kb = KafkaBroker(boot, idempotent=True, connect_wait_s=10)
    kb.RETRIES = 14
    kb.max_in_flight = 5
    kb.default_acks = -1
    kb.create_topic("pipe", 4)
    n_batches = 400
    for k in range(n_batches):
        if k == n_batches // 3:
            victim = kb.leader_of("pipe", 0)
            os.killpg(cluster["procs"][f"b{victim}"].pid, signal.SIGKILL)
        kb.produce_raw("pipe", k % 4, encode_record_batch([b"%d:%d" % (k, i) for i in range(20)]))
    kb.flush()
    assert not kb._inflight
    for p in range(4):
        end = kb.end_offset("pipe", p)
        vals = []
        off = 0
        while off < end:
            _e, _hw, raw = kb.fetch_raw("pipe", p, off)
            recs = [r for r in decode_record_batches(raw, "pipe", p) if r.offset >= off]
            vals += [r.value for r in recs]
            off = recs[-1].offset + 1 if recs else end
        want = [b"%d:%d" % (k, i) for k in range(p, n_batches, 4) for i in range(20)]
        assert vals == want, (p, len(vals), len(want))
    kb.close()


def test_native_consumer_reads_every_row_once_across_a_broker_kill(cluster):
    """The engine's C++ consumer (csrc/engine/kafka_consumer.cpp) on the replicated cluster:
    TXB1 batches produced with acks=all while the leader of two partitions is SIGKILLed; the
    consumer follows the new leaders (metadata refresh) and every row lands exactly once --
    it only ever sees records below the high watermark, so nothing it read can vanish."""
    import numpy as np

    from ccfd_demo_summit_amd.contracts import TxBatch
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.ingest.native_consumer import NativeKafkaConsumer
    boot = ",".join(f"127.0.0.1:{p}" for p in cluster["bports"])
    deadline = time.time() + 30
    while len(json.loads(_text(f"http://127.0.0.1:{cluster['cport']}/metadata"))["nodes"]) < 3:
        assert time.time() < deadline
        time.sleep(0.1)
    P, per, step = 6, 3000, 250
    kb = KafkaBroker(boot, idempotent=True, connect_wait_s=10)
    kb.RETRIES = 14
    kb.default_acks = -1
    kb.create_topic("odh-demo", P)
    X, _ = generate(P * per, seed=3)
    kc = NativeKafkaConsumer.for_arrays(boot, "odh-demo", {p: 0 for p in range(P)}, capacity=per + 100).start()
    try:
        for k in range(per // step):
            if k == (per // step) // 2:
                victim = kb.leader_of("odh-demo", 0)
                os.killpg(cluster["procs"][f"b{victim}"].pid, signal.SIGKILL)
            for p in range(P):
                s = p * per + k * step
                ids = np.arange(s, s + step, dtype=np.uint64)
                kb.produce("odh-demo", TxBatch(ids=ids, customer=(ids % 1000).astype(np.uint32),
                                               features=X[s:s + step]).encode(), partition=p)
        t0 = time.time()
        while kc.stats()["rows"] < P * per and time.time() - t0 < 60:
            time.sleep(0.05)
        time.sleep(0.3)
        st = kc.stats()
        assert st["rows"] == P * per, (st, kc.last_error())
        for p in range(P):
            _f, ids, _c = kc.arrays[p]
            np.testing.assert_array_equal(ids[:per], np.arange(p * per, (p + 1) * per, dtype=np.uint64))
    finally:
        kc.stop()
        kc.close()
        kb.close()


def test_broker_away_past_the_leaders_retention_restarts_at_its_log_start(small_retention_cluster):
    """A follower that was down while its leaders' retention (20 batches here) moved past its
    log end gets OFFSET_OUT_OF_RANGE below the log start: it restarts those partitions at the
    leader's log start (ListOffsets earliest), catches up and rejoins every ISR (round 5: the
    deployed broker-kill run stayed under-replicated until this)."""
    c = small_retention_cluster
    boot = ",".join(f"127.0.0.1:{p}" for p in c["bports"])
    deadline = time.time() + 30
    while len(json.loads(_text(f"http://127.0.0.1:{c['cport']}/metadata"))["nodes"]) < 3 and time.time() < deadline:
        time.sleep(0.1)
    kb = KafkaBroker(boot, idempotent=True, connect_wait_s=10)
    kb.RETRIES = 14
    kb.create_topic("t", 3)
    for k in range(30):
        kb.produce_raw("t", k % 3, encode_record_batch([b"a%d" % k]), acks=-1)
    os.killpg(c["procs"]["b2"].pid, signal.SIGKILL)
    c["procs"]["b2"].wait(10)
    for k in range(300):                                 # 100 batches per partition: > retention
        kb.produce_raw("t", k % 3, encode_record_batch([b"b%d" % k]), acks=-1)
    starts = [kb.begin_offset("t", p) for p in range(3)]
    assert min(starts) > 30, starts                      # the leaders' logs start past the old end
    c["start"]("b2", c["broker_cmd"](2))
    _wait(c["bports"][1])
    deadline = time.time() + 30
    md = {}
    under = [None]
    while time.time() < deadline:
        time.sleep(0.3)
        try:                                             # the restarted broker's metrics come up last
            md = json.loads(_text(f"http://127.0.0.1:{c['cport']}/metadata"))
            under = [_gauge(_text(f"http://127.0.0.1:{mp}/metrics"),
                            "kafka_server_replicamanager_underreplicatedpartitions") for mp in c["mports"]]
        except OSError:
            continue
        if all(len(v["isr"]) == 3 for k_, v in md["parts"].items() if k_.startswith("t/")) and not any(under):
            break
    assert all(len(v["isr"]) == 3 for k_, v in md["parts"].items() if k_.startswith("t/")), md["parts"]
    assert not any(under), under
    kb.close()


def test_sole_isr_leader_sigkill_loses_no_acknowledged_record(cluster):
    """with the ISR shrunk to the leader alone, an acks=all produce must not be
    answered before the leader WROTE it (no other copy exists), and the leader's sole-ISR
    status must be on disk before such an answer -- else a SIGKILL + restart cut the log to an
    older checkpointed HW.  Two brokers die, the third takes acknowledged writes alone, is
    SIGKILLed right after, restarts: every acknowledged record is there."""
    c = cluster
    boot = ",".join(f"127.0.0.1:{p}" for p in c["bports"])
    deadline = time.time() + 30
    while len(json.loads(_text(f"http://127.0.0.1:{c['cport']}/metadata"))["nodes"]) < 3:
        assert time.time() < deadline
        time.sleep(0.1)
    kb = KafkaBroker(boot, idempotent=True, connect_wait_s=10)
    kb.RETRIES = 20
    kb.create_topic("solo", 3)
    for k in range(30):
        kb.produce_raw("solo", k % 3, encode_record_batch([b"pre%d" % k]), acks=-1)
    for victim in (2, 3):
        os.killpg(c["procs"][f"b{victim}"].pid, signal.SIGKILL)
        c["procs"][f"b{victim}"].wait(10)
    deadline = time.time() + 30                          # every partition: leader 1, ISR [1]
    while True:
        md = json.loads(_text(f"http://127.0.0.1:{c['cport']}/metadata"))
        ps = [v for k, v in md["parts"].items() if k.startswith("solo/")]
        if all(v["leader"] == 1 and v["isr"] == [1] for v in ps):
            break
        assert time.time() < deadline, ps
        time.sleep(0.1)
    kb.close()
    kb = KafkaBroker(f"127.0.0.1:{c['bports'][0]}", idempotent=True, connect_wait_s=10)
    kb.RETRIES = 20
    acked = []
    for k in range(300):
        vals = [b"solo-%d-%d" % (k, i) for i in range(20)]
        kb.produce_raw("solo", k % 3, encode_record_batch(vals), acks=-1)
        acked += vals
    os.killpg(c["procs"]["b1"].pid, signal.SIGKILL)       # right after the last acknowledgement
    c["procs"]["b1"].wait(10)
    kb.close()
    for k in (1, 2, 3):
        c["start"](f"b{k}", c["broker_cmd"](k))
    for p in c["bports"]:
        _wait(p)
    kb = KafkaBroker(boot, idempotent=True, connect_wait_s=10)
    kb.RETRIES = 30
    got = set()
    deadline = time.time() + 30
    while time.time() < deadline:
        got = set()
        try:
            for p in range(3):
                off, end = 0, kb.end_offset("solo", p)
                while off < end:
                    _e, _hw, raw = kb.fetch_raw("solo", p, off)
                    recs = [r for r in decode_record_batches(raw, "solo", p) if r.offset >= off]
                    got.update(r.value for r in recs)
                    off = recs[-1].offset + 1 if recs else end
        except Exception:                                 # noqa: BLE001 -- leaders still moving
            time.sleep(0.3)
            continue
        if all(v in got for v in acked):
            break
        time.sleep(0.3)
    missing = [v for v in acked if v not in got]
    assert not missing, (len(missing), missing[:5])
    kb.close()
