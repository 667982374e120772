"""Controller of a replicated, multi-process kafka-lite cluster.

The reference runs Strimzi Kafka with ``kafka_broker_replicas: 3`` and three ZooKeeper nodes
(deploy/frauddetection_cr.yaml:75-77), and its Kafka dashboard watches under-replicated and
offline partitions (deploy/grafana/Kafka.json:271,347).  Round 4's kafka-lite was one
process; here each broker is its own process with its own durable log
(ingest/kafka_replica.py), and this small service plays ZooKeeper + the Kafka controller:

* **membership**: every broker heartbeats (``POST /heartbeat``, ~100 ms) with its node id,
  address, an incarnation token (new on every process start) and the log end offset (LEO)
  of every replica it hosts.  A broker silent for ``session_s`` -- or one that comes back with
  a new incarnation, i.e. restarted -- is failed: it leaves every ISR (the last ISR member
  stays, the partition goes offline) and the partitions it led are re-elected;
* **election**: the new leader is the live ISR member with the HIGHEST reported LEO, chosen
  only after every live ISR member has reported since the failure (a follower cannot append
  once its leader is gone, so the reports are final), so no acknowledged record is lost; the
  other replicas cut their un-acknowledged tails to their high watermark before following it
  (ingest/kafka_replica.py).  Unclean election is off: a
  partition whose ISR is all dead stays offline until an ISR member returns;
* **ISR**: leaders propose shrink / expand (a follower that stopped fetching or caught up)
  with their leader epoch; stale proposals are refused;
* **preferred leaders**: a partition whose first replica is alive and in the ISR is handed
  back to it (load spread after a broker returns), every ``rebalance_s``;
* **topics**: created here (``POST /topics``); replicas ``[(p + i) % N]`` over the registered
  brokers, replication factor ``min(rf, N)``;
* **committed offsets** (``POST /offsets/commit``, ``/offsets/fetch``): the group offsets
  (Kafka keeps them in a replicated internal topic; ZooKeeper-era Kafka kept them here);
* everything durable in ``data_dir/controller.json`` (+ an offsets log), so a restarted
  controller resumes with the same metadata.

The controller is off the data path: produces, fetches and replication flow broker to broker.
It runs as one process, or -- ``--member-id/--peers`` -- as a 3-member replicated quorum
(ingest/controller_quorum.py, the ZooKeeper ensemble's role): one active member, hot standbys
with a majority-replicated copy of the state, fail-over in well under a second.
Metrics (``/metrics``): active controller, offline partitions, leader elections, brokers.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import threading
import time
from typing import Any, Dict, List, Optional, Tuple


def tp_key(topic: str, p: int) -> str:
    return f"{topic}/{p}"


def tp_split(k: str) -> Tuple[str, int]:
    t, p = k.rsplit("/", 1)
    return t, int(p)


class ControllerState:
    """The controller's state machine (no I/O except its own persistence; unit-testable with
    an injected clock)."""

    def __init__(self, data_dir: Optional[str] = None, session_s: float = 1.5, rf: int = 3,
                 rebalance_s: float = 5.0, clock=time.monotonic, expected_brokers: int = 0):
        """``expected_brokers``: topics are created only once that many brokers registered
        (a topic created while one of three brokers is up would get replication factor 1)."""
        self.expected_brokers = int(expected_brokers)
        self.data_dir = data_dir
        self.session_s = float(session_s)
        self.rf = int(rf)
        self.rebalance_s = float(rebalance_s)
        self.clock = clock
        self.lock = threading.RLock()
        self.nodes: Dict[int, Dict[str, Any]] = {}          # id -> host, port, incarnation, alive, hb
        self.topics: Dict[str, int] = {}
        self.parts: Dict[str, Dict[str, Any]] = {}           # "t/p" -> replicas, leader, epoch, isr
        self.leo: Dict[int, Dict[str, int]] = {}             # node -> "t/p" -> LEO (last report)
        self.reported_at: Dict[int, float] = {}
        self.electing: Dict[str, float] = {}                 # "t/p" -> failure time (leader -1)
        self.meta_epoch = 0
        self.elections = 0
        self.offsets: Dict[str, int] = {}                    # "g|t|p" -> committed offset
        self.mutations = 0                  # every change (replicated by controller_quorum.py)
        self._last_rebalance = clock()
        self._off_f = None
        self._load()

    # ------------------------------------------------------------------ persistence
    def _path(self, name: str) -> Optional[str]:
        return os.path.join(self.data_dir, name) if self.data_dir else None

    def _load(self) -> None:
        if not self.data_dir:
            return
        os.makedirs(self.data_dir, exist_ok=True)
        p = self._path("controller.json")
        if os.path.exists(p):
            with open(p) as f:
                d = json.load(f)
            self.topics = {k: int(v) for k, v in d.get("topics", {}).items()}
            self.parts = d.get("parts", {})
            self.meta_epoch = int(d.get("meta_epoch", 0)) + 1
            for nid, n in d.get("nodes", {}).items():
                # every broker must heartbeat again before it counts as alive
                self.nodes[int(nid)] = {"host": n["host"], "port": int(n["port"]), "incarnation": n.get("incarnation"),
                                        "alive": False, "hb": self.clock()}
            now = self.clock()
            for k, st in self.parts.items():
                if st["leader"] >= 0:           # its leader must prove alive before serving again
                    self.electing[k] = now
        op = self._path("offsets.log")
        if os.path.exists(op):
            with open(op) as f:
                for line in f:
                    try:
                        d = json.loads(line)
                    except json.JSONDecodeError:
                        continue
                    k = d["k"]
                    self.offsets[k] = max(int(d["o"]), self.offsets.get(k, 0))
        self._off_f = open(op, "a", buffering=1)

    def _save(self) -> None:
        if not self.data_dir:
            return
        p = self._path("controller.json")
        tmp = p + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"topics": self.topics, "parts": self.parts, "meta_epoch": self.meta_epoch,
                       "nodes": {str(k): {"host": v["host"], "port": v["port"], "incarnation": v.get("incarnation")}
                                 for k, v in self.nodes.items()}}, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, p)

    def _changed(self) -> None:
        self.meta_epoch += 1
        self.mutations += 1
        self._save()

    # ------------------------------------------------------------------ replication (quorum)
    def snapshot(self) -> Dict[str, Any]:
        """The replicated part of the state (controller_quorum.py ships it to the standbys):
        everything but broker liveness, heartbeat times and LEO reports, which a new active
        controller collects afresh."""
        with self.lock:
            return {"topics": dict(self.topics), "parts": json.loads(json.dumps(self.parts)),
                    "meta_epoch": self.meta_epoch, "elections": self.elections, "offsets": dict(self.offsets),
                    "nodes": {str(k): {"host": v["host"], "port": v["port"], "incarnation": v.get("incarnation")}
                              for k, v in self.nodes.items()}}

    def restore(self, snap: Optional[Dict[str, Any]], takeover: bool = False) -> None:
        """Adopt a replicated snapshot.  ``takeover``: this process becomes the active
        controller -- every known broker gets a fresh session (alive, heartbeat now: one that
        stays silent is failed after ``session_s`` as usual), partitions without a leader wait
        for new LEO reports before their election."""
        with self.lock:
            now = self.clock()
            if snap is not None:
                self.topics = {k: int(v) for k, v in snap.get("topics", {}).items()}
                self.parts = json.loads(json.dumps(snap.get("parts", {})))
                self.meta_epoch = int(snap.get("meta_epoch", 0))
                self.elections = int(snap.get("elections", 0))
                self.offsets = {k: int(v) for k, v in snap.get("offsets", {}).items()}
                self.nodes = {int(k): {"host": v["host"], "port": int(v["port"]), "incarnation": v.get("incarnation"),
                                       "alive": False, "hb": now} for k, v in snap.get("nodes", {}).items()}
            if takeover:
                for n in self.nodes.values():
                    n["alive"], n["hb"] = True, now
                self.leo, self.reported_at = {}, {}
                self.electing = {k: now for k, st in self.parts.items() if st["leader"] < 0}
                self._last_rebalance = now
            self.meta_epoch += 1                 # brokers re-read the metadata from the new active
            self.mutations += 1

    # ------------------------------------------------------------------ metadata
    def metadata(self) -> Dict[str, Any]:
        with self.lock:
            return {"meta_epoch": self.meta_epoch,
                    "nodes": {str(k): [v["host"], v["port"]] for k, v in self.nodes.items() if v["alive"]},
                    "topics": dict(self.topics),
                    "parts": {k: dict(v) for k, v in self.parts.items()}}

    def can_create(self) -> bool:
        with self.lock:
            return len(self.nodes) >= self.expected_brokers

    def create_topic(self, name: str, partitions: int) -> bool:
        with self.lock:
            if name in self.topics:
                return False
            if not self.can_create():
                raise RuntimeError(f"{len(self.nodes)} of {self.expected_brokers} brokers registered")
            ids = sorted(self.nodes) or [1]
            rf = max(1, min(self.rf, len(ids)))
            for p in range(max(1, int(partitions))):
                reps = [ids[(p + i) % len(ids)] for i in range(rf)]
                live = [r for r in reps if self.nodes.get(r, {}).get("alive")]
                self.parts[tp_key(name, p)] = {"replicas": reps, "leader": (live or [-1])[0], "epoch": 0,
                                               "isr": live or reps[:1]}
            self.topics[name] = max(1, int(partitions))
            self._changed()
            return True

    # ------------------------------------------------------------------ membership
    def heartbeat(self, node: int, host: str, port: int, incarnation: str, leos: Dict[str, int],
                  isr_changes: List[Dict[str, Any]], seen_epoch: int = -1) -> Dict[str, Any]:
        now = self.clock()
        with self.lock:
            n = self.nodes.get(node)
            changed = False
            if n is None:
                self.nodes[node] = n = {"host": host, "port": int(port), "incarnation": incarnation,
                                        "alive": False, "hb": now}
                changed = True
            elif n["incarnation"] != incarnation:
                # the broker restarted: whatever it led or replicated before is failed over
                # first, then it rejoins as a follower (its log was cut to its checkpointed HW)
                if n["alive"]:
                    self._fail(node, now)
                n.update(host=host, port=int(port), incarnation=incarnation)
                changed = True
            n["hb"] = now
            if not n["alive"]:
                n["alive"] = True
                changed = True
            self.leo[node] = {k: int(v) for k, v in leos.items()}
            self.reported_at[node] = now
            for ch in isr_changes or []:
                k = ch["tp"]
                st = self.parts.get(k)
                if st is None or st["leader"] != node or int(ch["epoch"]) != st["epoch"]:
                    continue                    # stale: not the leader of that epoch
                isr = [int(x) for x in ch["isr"] if int(x) in st["replicas"]]
                if node not in isr:
                    continue
                if sorted(isr) != sorted(st["isr"]):
                    st["isr"] = isr
                    changed = True
            changed |= self._elect(now)
            if changed:
                self._changed()
            if seen_epoch == self.meta_epoch:
                return {"meta_epoch": self.meta_epoch}
        return self.metadata()

    def _fail(self, node: int, now: float) -> None:
        """Under the lock: ``node`` is dead (or restarted)."""
        self.nodes[node]["alive"] = False
        for k, st in self.parts.items():
            if node in st["isr"] and len(st["isr"]) > 1:
                st["isr"] = [x for x in st["isr"] if x != node]
            if st["leader"] == node:
                st["leader"] = -1
                self.electing[k] = now

    def _elect(self, now: float) -> bool:
        """Under the lock: leaders for the partitions without one, where possible."""
        changed = False
        for k in list(self.electing):
            st = self.parts[k]
            t0 = self.electing[k]
            cands = [x for x in st["isr"] if self.nodes.get(x, {}).get("alive")]
            if not cands:
                continue                         # offline until an ISR member returns
            if any(self.reported_at.get(x, -1.0) < t0 for x in cands) and now - t0 < 5 * self.session_s:
                continue                         # wait for every live ISR member's final LEO
            best = max(cands, key=lambda x: (self.leo.get(x, {}).get(k, -1), -st["replicas"].index(x)
                                             if x in st["replicas"] else 0))
            st["leader"] = best
            st["epoch"] += 1
            del self.electing[k]
            self.elections += 1
            changed = True
        return changed

    def tick(self) -> bool:
        """Failure detection, pending elections, preferred-leader hand-back."""
        now = self.clock()
        with self.lock:
            changed = False
            for nid, n in self.nodes.items():
                if n["alive"] and now - n["hb"] > self.session_s:
                    self._fail(nid, now)
                    changed = True
            changed |= self._elect(now)
            if now - self._last_rebalance >= self.rebalance_s:
                self._last_rebalance = now
                for k, st in self.parts.items():
                    pref = st["replicas"][0]
                    if (st["leader"] >= 0 and st["leader"] != pref and pref in st["isr"]
                            and self.nodes.get(pref, {}).get("alive")):
                        st["leader"] = pref
                        st["epoch"] += 1
                        self.elections += 1
                        changed = True
            if changed:
                self._changed()
            return changed

    # ------------------------------------------------------------------ offsets
    def commit(self, group: str, entries: List[Tuple[str, int, int]]) -> None:
        with self.lock:
            for t, p, o in entries:
                k = f"{group}|{t}|{int(p)}"
                v = max(int(o), self.offsets.get(k, 0))
                if v != self.offsets.get(k):
                    self.offsets[k] = v
                    self.mutations += 1
                    if self._off_f is not None:
                        self._off_f.write(json.dumps({"k": k, "o": v}) + "\n")
            if self._off_f is not None:
                self._off_f.flush()
                os.fsync(self._off_f.fileno())

    def fetch_offsets(self, group: str, tps: List[Tuple[str, int]]) -> List[int]:
        with self.lock:
            return [self.offsets.get(f"{group}|{t}|{int(p)}", -1) for t, p in tps]

    # ------------------------------------------------------------------ metrics
    def offline(self) -> int:
        with self.lock:
            return sum(1 for st in self.parts.values() if st["leader"] < 0)

    def under_replicated(self) -> int:
        with self.lock:
            return sum(1 for st in self.parts.values() if len(st["isr"]) < len(st["replicas"]))

    def expose(self, active: bool = True, quorum: Optional[Dict[str, Any]] = None) -> bytes:
        with self.lock:
            alive = sum(1 for n in self.nodes.values() if n["alive"])
            lines = [
                "# TYPE kafka_controller_kafkacontroller_activecontrollercount gauge",
                f"kafka_controller_kafkacontroller_activecontrollercount {1 if active else 0}",
                "# TYPE kafka_controller_kafkacontroller_offlinepartitionscount gauge",
                f"kafka_controller_kafkacontroller_offlinepartitionscount {self.offline()}",
                "# TYPE kafka_controller_controllerstats_leaderelectionrateandtimems_count counter",
                f"kafka_controller_controllerstats_leaderelectionrateandtimems_count {self.elections}",
                "# TYPE ccfd_kafka_controller_brokers_alive gauge",
                f"ccfd_kafka_controller_brokers_alive {alive}",
                "# TYPE ccfd_kafka_controller_underreplicated_partitions gauge",
                f"ccfd_kafka_controller_underreplicated_partitions {self.under_replicated()}",
            ]
            if quorum is not None:
                lines += ["# TYPE ccfd_kafka_controller_quorum_term gauge",
                          f"ccfd_kafka_controller_quorum_term {quorum['term']}",
                          "# TYPE ccfd_kafka_controller_quorum_elections_won_total counter",
                          f"ccfd_kafka_controller_quorum_elections_won_total {quorum['elections_won']}",
                          "# TYPE ccfd_kafka_controller_quorum_round_failures_total counter",
                          f"ccfd_kafka_controller_quorum_round_failures_total {quorum['round_failures']}"]
        return ("\n".join(lines) + "\n").encode()


def make_app(state: ControllerState, quorum=None):
    """HTTP front of the controller.  With ``quorum`` (controller_quorum.QuorumMember) this
    process is one member of a replicated controller: only the active member answers the
    broker API (a standby answers 421 with the active's URL), and every answer that depends on
    a change -- new metadata, a created topic, a committed offset -- waits until a majority of
    the members holds that change (503 if the member lost the active role meanwhile)."""
    from aiohttp import web

    def not_active():
        return web.json_response({"error": "not the active controller",
                                  "leader": quorum.leader_url() if quorum is not None else None}, status=421)

    async def durable() -> bool:
        return quorum is None or await quorum.commit_mutation()

    def standby() -> bool:
        return quorum is not None and not quorum.is_active()

    async def hb(request):
        if standby():
            return not_active()
        d = await request.json()
        out = state.heartbeat(int(d["node"]), d["host"], int(d["port"]), str(d["incarnation"]),
                              d.get("leos", {}), d.get("isr_changes", []), int(d.get("seen_epoch", -1)))
        if not await durable():                      # never publish metadata a failover could undo
            return web.json_response({"error": "lost the controller majority"}, status=503)
        return web.json_response(out)

    async def topics(request):
        if standby():
            return not_active()
        d = await request.json()
        try:
            created = state.create_topic(d["name"], int(d["partitions"]))
        except RuntimeError as e:                    # not every broker is up yet: ask again
            return web.json_response({"error": str(e)}, status=503)
        if not await durable():
            return web.json_response({"error": "lost the controller majority"}, status=503)
        return web.json_response({"created": created, **state.metadata()})

    async def metadata(_request):
        if standby():
            return not_active()
        if not await durable():
            return web.json_response({"error": "lost the controller majority"}, status=503)
        return web.json_response(state.metadata())

    async def commit(request):
        if standby():
            return not_active()
        d = await request.json()
        state.commit(d["group"], [(e[0], int(e[1]), int(e[2])) for e in d["offsets"]])
        if not await durable():                      # acknowledged = on a majority of members
            return web.json_response({"error": "lost the controller majority"}, status=503)
        return web.json_response({"ok": True})

    async def fetch(request):
        if standby():
            return not_active()
        d = await request.json()
        if not await durable():                      # never answer an offset a failover could undo
            return web.json_response({"error": "lost the controller majority"}, status=503)
        return web.json_response({"offsets": state.fetch_offsets(d["group"], [(e[0], int(e[1])) for e in d["tps"]])})

    async def metrics(_request):
        body = state.expose(active=quorum is None or quorum.is_active(),
                            quorum=quorum.status() if quorum is not None else None)
        return web.Response(body=body, headers={"Content-Type": "text/plain; version=0.0.4"})

    async def quorum_status(_request):
        return web.json_response(quorum.status() if quorum is not None else {"role": "single", "active": True})

    async def vote(request):
        return web.json_response(quorum.on_vote(await request.json()))

    async def append(request):
        return web.json_response(quorum.on_append(await request.json()))

    async def ticker(app):
        if quorum is not None:
            await quorum.start()

        async def loop():
            while True:
                if quorum is None or quorum.is_active():
                    state.tick()                     # failure detection / elections: the active only
                await asyncio.sleep(min(0.05, state.session_s / 4))
        app["ticker"] = asyncio.get_running_loop().create_task(loop())

    async def stop(app):
        app["ticker"].cancel()
        if quorum is not None:
            await quorum.close()

    app = web.Application()
    app.router.add_get("/quorum", quorum_status)
    if quorum is not None:
        app.router.add_post("/quorum/vote", vote)
        app.router.add_post("/quorum/append", append)
    app.router.add_post("/heartbeat", hb)
    app.router.add_post("/topics", topics)
    app.router.add_get("/metadata", metadata)
    app.router.add_post("/offsets/commit", commit)
    app.router.add_post("/offsets/fetch", fetch)
    app.router.add_get("/metrics", metrics)
    app.router.add_get("/health/ping", lambda _r: web.json_response({"status": "ok"}))
    app.on_startup.append(ticker)
    app.on_cleanup.append(stop)
    return app


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=9093)
    ap.add_argument("--data-dir", default=None)
    ap.add_argument("--session-s", type=float, default=1.5, help="broker heartbeat timeout")
    ap.add_argument("--rf", type=int, default=3, help="replication factor of new topics")
    ap.add_argument("--brokers", type=int, default=0,
                    help="create topics only once this many brokers registered (0 = whatever is up)")
    ap.add_argument("--member-id", type=int, default=0,
                    help="replicated controller: this member's id in --peers (0 = a single controller)")
    ap.add_argument("--peers", default="",
                    help="replicated controller: every member as id=url, comma-separated "
                         "(e.g. 1=http://c0:9093,2=http://c1:9093,3=http://c2:9093)")
    a = ap.parse_args(argv)
    from aiohttp import web
    if a.member_id:
        from .controller_quorum import QuorumMember, parse_peers
        peers = parse_peers(a.peers)
        # the quorum member persists the replicated state itself (quorum.json)
        state = ControllerState(None, session_s=a.session_s, rf=a.rf, expected_brokers=a.brokers)
        quorum = QuorumMember(a.member_id, peers, state, data_dir=a.data_dir)
        print(f"[kafka-controller] member {a.member_id} of {len(peers)} on :{a.port} term {quorum.term} "
              f"state version {list(quorum.version)}", flush=True)
        web.run_app(make_app(state, quorum), host=a.host, port=a.port, print=None, access_log=None)
        return
    state = ControllerState(a.data_dir, session_s=a.session_s, rf=a.rf, expected_brokers=a.brokers)
    print(f"[kafka-controller] :{a.port} topics {len(state.topics)} meta epoch {state.meta_epoch}", flush=True)
    web.run_app(make_app(state), host=a.host, port=a.port, print=None, access_log=None)


if __name__ == "__main__":
    main()
