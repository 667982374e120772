"""Replicated kafka-lite controller (the reference's three ZooKeeper nodes
next to three brokers, deploy/frauddetection_cr.yaml:75-77, and the Kafka dashboard's
active-controller / offline-partition panels, deploy/grafana/Kafka.json:271,347).

Three controller member PROCESSES (ingest/controller_quorum.py) and three broker processes.
The active controller is SIGKILLed together with a partition leader: a standby takes over,
the dead broker's partitions are re-elected, no acknowledged record and no committed offset
is lost, and the killed members rejoin.
"""
import asyncio
import json
import os
import signal
import subprocess
import sys
import threading
import time
import urllib.request

import pytest

from ccfd_demo_summit_amd.ingest.controller_quorum import QuorumMember
from ccfd_demo_summit_amd.ingest.kafka_controller import ControllerState, make_app
from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker, decode_record_batches, encode_record_batch

from test_kafka_replicated import ROOT, _free_ports, _gauge, _text, _wait


def _json(url, timeout=2):
    with urllib.request.urlopen(url, timeout=timeout) as r:
        return json.loads(r.read().decode())


def _active(cports, exclude=()):
    for i, p in enumerate(cports):
        if i in exclude:
            continue
        try:
            q = _json(f"http://127.0.0.1:{p}/quorum", timeout=0.5)
        except OSError:
            continue
        if q.get("active"):
            return i, q
    return None, None


def _wait_active(cports, exclude=(), t=20):
    deadline = time.time() + t
    while time.time() < deadline:
        i, q = _active(cports, exclude)
        if i is not None:
            return i, q
        time.sleep(0.05)
    raise TimeoutError("no active controller")


def test_in_process_quorum_elects_replicates_and_fails_over(tmp_path):
    """Three members in one event loop: one becomes active, a committed change reaches every
    standby's disk, the active's loss elects a standby that holds the change."""
    from aiohttp import web

    async def go():
        ports = _free_ports(3)
        peers = {k + 1: f"http://127.0.0.1:{ports[k]}" for k in range(3)}
        members, runners = {}, {}
        for k in (1, 2, 3):
            st = ControllerState(None, session_s=1.0)
            q = QuorumMember(k, peers, st, data_dir=str(tmp_path / f"m{k}"))
            app = make_app(st, q)
            runner = web.AppRunner(app)
            await runner.setup()
            await web.TCPSite(runner, "127.0.0.1", ports[k - 1]).start()
            members[k], runners[k] = q, runner
        t0 = time.monotonic()
        while not any(m.is_active() for m in members.values()):
            assert time.monotonic() - t0 < 10
            await asyncio.sleep(0.05)
        lead = next(k for k, m in members.items() if m.is_active())
        st = members[lead].state
        st.commit("g", [("t", 0, 42)])
        assert await members[lead].commit_mutation()
        for k in members:
            if k != lead:
                assert members[k].snapshot["offsets"]["g|t|0"] == 42    # replicated (on disk)
                disk = json.load(open(tmp_path / f"m{k}" / "quorum.json"))
                assert disk["snapshot"]["offsets"]["g|t|0"] == 42
        await runners[lead].cleanup()                # the active member dies
        del members[lead]
        t0 = time.monotonic()
        while not any(m.is_active() for m in members.values()):
            assert time.monotonic() - t0 < 10
            await asyncio.sleep(0.05)
        new = next(k for k, m in members.items() if m.is_active())
        assert new != lead and members[new].state.fetch_offsets("g", [("t", 0)]) == [42]
        assert members[new].term > 1 or members[new].elections_won >= 1
        for k, r in runners.items():
            if k != lead:
                await r.cleanup()
    asyncio.new_event_loop().run_until_complete(go())


@pytest.fixture()
def qcluster(tmp_path):
    ports = _free_ports(9)
    cports, bports, mports = ports[0:3], ports[3:6], ports[6:9]
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    procs = {}
    peers = ",".join(f"{k + 1}=http://127.0.0.1:{cports[k]}" for k in range(3))
    ctl_urls = ",".join(f"http://127.0.0.1:{p}" for p in cports)

    def start(name, cmd):
        procs[name] = subprocess.Popen(cmd, cwd=str(ROOT), env=env, stdout=subprocess.DEVNULL,
                                       stderr=subprocess.DEVNULL, start_new_session=True)

    def ctl_cmd(k):
        return [sys.executable, "-m", "ccfd_demo_summit_amd.ingest.kafka_controller", "--host", "127.0.0.1",
                "--port", str(cports[k]), "--data-dir", str(tmp_path / f"c{k}"), "--session-s", "1.0",
                "--brokers", "3", "--member-id", str(k + 1), "--peers", peers]

    def broker_cmd(k):
        return [sys.executable, "-m", "ccfd_demo_summit_amd.ingest.kafka_lite", "--host", "127.0.0.1",
                "--port", str(bports[k - 1]), "--node-id", str(k), "--controller", ctl_urls,
                "--metrics-port", str(mports[k - 1]), "--data-dir", str(tmp_path / f"b{k}"), "--fsync", "interval"]
    for k in range(3):
        start(f"c{k}", ctl_cmd(k))
    for p in cports:
        _wait(p)
    for k in (1, 2, 3):
        start(f"b{k}", broker_cmd(k))
    for p in bports:
        _wait(p)
    yield {"cports": cports, "bports": bports, "mports": mports, "procs": procs, "start": start,
           "ctl_cmd": ctl_cmd, "broker_cmd": broker_cmd}
    for p in procs.values():
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait(10)


def test_active_controller_sigkill_during_broker_failure(qcluster):
    c = qcluster
    ia, _ = _wait_active(c["cports"], t=30)
    deadline = time.time() + 30
    while len(_json(f"http://127.0.0.1:{c['cports'][ia]}/metadata")["nodes"]) < 3:
        assert time.time() < deadline
        time.sleep(0.1)
    boot = ",".join(f"127.0.0.1:{p}" for p in c["bports"])
    kb = KafkaBroker(boot, idempotent=True, connect_wait_s=10)
    kb.RETRIES = 20
    kb.create_topic("odh-demo", 6)
    for p in range(6):                                   # committed offsets before the failure
        kb.commit("ccfd-engine", "odh-demo", p, 100 + p)
    acked, errors = {}, []
    stop = threading.Event()

    def produce():
        k = 0
        while not stop.is_set():
            p = k % 6
            vals = [b"%d-%d" % (k, i) for i in range(40)]
            try:
                kb.produce_raw("odh-demo", p, encode_record_batch(vals), acks=-1)
            except Exception as e:                       # noqa: BLE001
                errors.append(repr(e))
                time.sleep(0.05)
                continue
            for v in vals:
                acked[v] = p
            k += 1
    th = threading.Thread(target=produce, daemon=True)
    th.start()
    time.sleep(1.5)
    # the broker leading partition 0 and the active controller die together
    victim = kb.leader_of("odh-demo", 0)
    md0 = _json(f"http://127.0.0.1:{c['cports'][ia]}/metadata")
    led = [k for k, v in md0["parts"].items() if v["leader"] == victim and k.startswith("odh-demo/")]
    os.killpg(c["procs"][f"b{victim}"].pid, signal.SIGKILL)
    os.killpg(c["procs"][f"c{ia}"].pid, signal.SIGKILL)
    c["procs"][f"c{ia}"].wait(10)
    t_kill = time.time()
    ib, q = _wait_active(c["cports"], exclude=(ia,), t=20)
    t_active = time.time() - t_kill
    assert ib != ia
    # the dead broker's partitions are re-elected by the new active controller
    deadline = time.time() + 20
    while True:
        md = _json(f"http://127.0.0.1:{c['cports'][ib]}/metadata")
        if all(md["parts"][k]["leader"] not in (-1, victim) for k in led):
            break
        assert time.time() < deadline, {k: md["parts"][k] for k in led}
        time.sleep(0.1)
    t_failover = time.time() - t_kill
    n_during = len(acked)
    time.sleep(1.0)
    assert len(acked) > n_during                          # producing resumed on the new leaders
    # committed offsets survived, and commits work against the new active controller
    assert [kb.committed("ccfd-engine", "odh-demo", p) for p in range(6)] == [100 + p for p in range(6)]
    kb.commit("ccfd-engine", "odh-demo", 0, 200)
    assert kb.committed("ccfd-engine", "odh-demo", 0) == 200
    # both come back: the broker re-syncs, the member rejoins as a standby
    c["start"](f"b{victim}", c["broker_cmd"](victim))
    c["start"](f"c{ia}", c["ctl_cmd"](ia))
    _wait(c["bports"][victim - 1])
    _wait(c["cports"][ia])
    time.sleep(1.5)
    stop.set()
    th.join(30)
    deadline = time.time() + 30
    while time.time() < deadline:
        try:
            md = _json(f"http://127.0.0.1:{c['cports'][ib]}/metadata")
            rq = _json(f"http://127.0.0.1:{c['cports'][ia]}/quorum")
        except OSError:
            time.sleep(0.2)
            continue
        if all(len(v["isr"]) == 3 for k, v in md["parts"].items() if k.startswith("odh-demo/")) and \
                rq["role"] == "follower" and rq["version"][0] >= q["term"]:
            break
        time.sleep(0.2)
    assert all(len(v["isr"]) == 3 for k, v in md["parts"].items() if k.startswith("odh-demo/")), md["parts"]
    assert rq["role"] == "follower" and not rq["active"]
    actives = sum(_gauge(_text(f"http://127.0.0.1:{p}/metrics"), "kafka_controller_kafkacontroller_activecontrollercount")
                  for p in c["cports"])
    assert actives == 1
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
    assert t_active < 5.0 and t_failover < 10.0, (t_active, t_failover)
    print(f"[quorum] new active in {t_active:.2f} s, partitions re-elected in {t_failover:.2f} s, "
          f"{len(acked)} records acked")
    kb.close()
