"""Replicated kafka-lite controller: a 3-member quorum in place of the reference's three
ZooKeeper nodes (deploy/frauddetection_cr.yaml:75-77).

One member is the ACTIVE controller (it alone answers brokers: heartbeats, topic creation,
offset commits); the others are hot standbys holding a replicated copy of its state.  The
protocol is Raft reduced to a single log entry -- the controller's whole state is small
(topics, leaders / ISR, broker incarnations, committed group offsets: a few KB), so each
replication round ships the latest state, not a log of operations:

* **terms and votes** (persisted, fsync'd, before any answer): a member that has not heard
  from an active controller for a randomised election timeout becomes a candidate for the
  next term and asks the others for votes; a vote goes to at most one candidate a term, and
  only to one whose state version ``(term, seq)`` is at least the voter's own -- so a member
  elected by a majority holds every state a majority accepted (the Raft election rule);
* **leader stickiness**: a member that heard from a live active controller within the minimum
  election timeout refuses to vote (a partitioned member cannot depose a healthy active);
* **replication**: every mutation (a broker heartbeat that changed leaders / ISR / membership,
  a topic, an offset commit) bumps the active's state; a replication round sends the newest
  state, versioned ``(term, seq + 1)``, to every standby, which persists it and acknowledges.
  The mutation is answered only when a MAJORITY (the active counts itself after its own fsync)
  holds that version -- an acknowledged offset commit or leader election survives the loss of
  any one member;
* **step-down**: an active that sees a higher term, or cannot reach a majority for the maximum
  election timeout, stops answering (421 + the leader it knows) -- two actives can never both
  complete a mutation, because a mutation needs a majority at the active's own term;
* **takeover**: a new active restores the replicated state and first commits a no-op round of
  its own term.  Broker liveness is soft state: every broker gets a fresh session (it is failed
  normally if it stays silent), LEO reports are collected anew before any election.

Brokers (ingest/kafka_replica.py) and any other client take the member list
(``http://a:9093,http://b:9093,http://c:9093``) and follow the active: a standby answers
``421 {"leader": url}``.
"""
from __future__ import annotations

import asyncio
import json
import os
import random
import time
from typing import Any, Dict, List, Optional, Tuple

Version = Tuple[int, int]
NOT_LEADER = 421


def _write_atomic(path: str, obj: Dict[str, Any]) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def parse_peers(spec: str) -> Dict[int, str]:
    """``"1=http://h1:9093,2=http://h2:9093,3=http://h3:9093"`` -> {1: url, ...}."""
    out: Dict[int, str] = {}
    for part in (spec or "").split(","):
        part = part.strip()
        if not part:
            continue
        k, _, url = part.partition("=")
        out[int(k)] = url.rstrip("/")
    return out


class QuorumMember:
    def __init__(self, node_id: int, peers: Dict[int, str], state, data_dir: Optional[str] = None,
                 election_s: Tuple[float, float] = (0.4, 0.8), hb_s: float = 0.06, rpc_timeout_s: float = 0.3,
                 clock=time.monotonic):
        """``peers``: every member's URL by id, this one included; ``state``: the
        ControllerState this member drives while it is the active one."""
        if node_id not in peers:
            raise ValueError(f"member {node_id} is not in the peer list {sorted(peers)}")
        self.id = int(node_id)
        self.peers = {int(k): v for k, v in peers.items()}
        self.others = [k for k in sorted(self.peers) if k != self.id]
        self.majority = len(self.peers) // 2 + 1
        self.state = state
        self.data_dir = data_dir
        self.election_s = election_s
        self.hb_s = float(hb_s)
        self.rpc_timeout_s = float(rpc_timeout_s)
        self.clock = clock
        # persistent
        self.term = 0
        self.voted_for: Optional[int] = None
        self.version: Version = (0, 0)
        self.snapshot: Optional[Dict[str, Any]] = None
        # volatile
        self.role = "follower"
        self.leader_id: Optional[int] = None
        self.ready = False                      # active and its takeover round committed
        self.last_contact = clock()
        self._deadline = self._new_deadline()
        self._peer_ver: Dict[int, Version] = {}
        self.committed: Version = (0, 0)
        self.committed_mut = -1                 # state mutations a majority holds (this term)
        self._built_mut = -1                    # state mutation counter behind self.version
        self._built: List[Tuple[int, Version]] = []     # (mutations, version) of recent rounds
        self._cv: Optional[asyncio.Condition] = None
        self._kick: Optional[asyncio.Event] = None
        self._session = None
        self._tasks: List[asyncio.Task] = []
        self.elections_won = 0
        self.rounds = 0
        self.round_failures = 0
        self._last_majority = clock()
        self._load()

    # ------------------------------------------------------------------ persistence
    def _path(self) -> Optional[str]:
        return os.path.join(self.data_dir, "quorum.json") if self.data_dir else None

    def _load(self) -> None:
        p = self._path()
        if p is None:
            return
        os.makedirs(self.data_dir, exist_ok=True)
        if not os.path.exists(p):
            return
        with open(p) as f:
            d = json.load(f)
        self.term = int(d.get("term", 0))
        self.voted_for = d.get("voted_for")
        self.version = tuple(d.get("version", (0, 0)))
        self.snapshot = d.get("snapshot")

    def _persist_sync(self) -> None:
        p = self._path()
        if p is not None:
            _write_atomic(p, {"term": self.term, "voted_for": self.voted_for, "version": list(self.version),
                              "snapshot": self.snapshot})

    async def _persist(self) -> None:
        if self._path() is not None:
            await asyncio.get_running_loop().run_in_executor(None, self._persist_sync)

    # ------------------------------------------------------------------ lifecycle
    def _new_deadline(self) -> float:
        return self.clock() + random.uniform(*self.election_s)

    async def start(self) -> None:
        import aiohttp
        self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.rpc_timeout_s))
        self._cv = asyncio.Condition()
        self._kick = asyncio.Event()
        loop = asyncio.get_running_loop()
        self._tasks = [loop.create_task(self._main_loop())]

    async def close(self) -> None:
        for t in self._tasks:
            t.cancel()
        if self._session is not None:
            await self._session.close()

    def leader_url(self) -> Optional[str]:
        return self.peers.get(self.leader_id) if self.leader_id is not None else None

    def is_active(self) -> bool:
        return self.role == "leader" and self.ready

    # ------------------------------------------------------------------ main loop
    async def _main_loop(self) -> None:
        while True:
            if self.role == "leader":
                await self._replicate_round()
                if self.clock() - self._last_majority > self.election_s[1]:
                    self._step_down(None)               # cut off from the majority: stop serving
                    continue
                try:
                    await asyncio.wait_for(self._kick.wait(), self.hb_s)
                except asyncio.TimeoutError:
                    pass
                self._kick.clear()
            else:
                await asyncio.sleep(0.02)
                if self.clock() >= self._deadline:
                    await self._run_election()

    def _step_down(self, leader: Optional[int]) -> None:
        self.role = "follower"
        self.ready = False
        self.leader_id = leader
        self._deadline = self._new_deadline()

    async def _rpc(self, peer: int, path: str, body: Dict[str, Any]) -> Optional[Dict[str, Any]]:
        try:
            async with self._session.post(self.peers[peer] + path, json=body) as r:
                if r.status != 200:
                    return None
                return await r.json()
        except Exception:                           # noqa: BLE001 -- a member away
            return None

    # ------------------------------------------------------------------ election
    async def _run_election(self) -> None:
        self.role = "candidate"
        self.term += 1
        self.voted_for = self.id
        self.leader_id = None
        term = self.term
        await self._persist()
        self._deadline = self._new_deadline()
        votes = 1
        body = {"term": term, "candidate": self.id, "version": list(self.version)}
        res = await asyncio.gather(*[self._rpc(p, "/quorum/vote", body) for p in self.others])
        for r in res:
            if r is None:
                continue
            if int(r["term"]) > self.term:
                self.term = int(r["term"])
                self.voted_for = None
                await self._persist()
                self._step_down(None)
                return
            if r.get("granted"):
                votes += 1
        if self.role != "candidate" or self.term != term:
            return                                  # a leader of this or a later term appeared
        if votes >= self.majority:
            await self._become_leader()

    async def _become_leader(self) -> None:
        self.role = "leader"
        self.leader_id = self.id
        self.ready = False
        self.elections_won += 1
        self._peer_ver = {}
        self.state.restore(self.snapshot, takeover=True)
        self._built_mut = -1                        # force a takeover round of this term
        self._built = []
        self.committed_mut = -1
        self._last_majority = self.clock()
        await self._replicate_round()              # serves once this round is committed

    def on_vote(self, d: Dict[str, Any]) -> Dict[str, Any]:
        term, cand = int(d["term"]), int(d["candidate"])
        ver = tuple(d.get("version", (0, 0)))
        now = self.clock()
        if term < self.term:
            return {"term": self.term, "granted": False}
        # stickiness: a live active (or this member, active) is not deposed by a newcomer
        if term > self.term and ((self.role == "leader" and self.ready) or
                                 (self.role == "follower" and self.leader_id is not None
                                  and now - self.last_contact < self.election_s[0])):
            return {"term": self.term, "granted": False}
        changed = False
        if term > self.term:
            self.term = term
            self.voted_for = None
            changed = True
            if self.role != "follower":
                self._step_down(None)
        granted = self.voted_for in (None, cand) and ver >= self.version
        if granted and self.voted_for != cand:
            self.voted_for = cand
            changed = True
        if granted:
            self._deadline = self._new_deadline()
        if changed:
            self._persist_sync()                    # before the answer leaves
        return {"term": self.term, "granted": granted}

    # ------------------------------------------------------------------ replication
    async def _replicate_round(self) -> bool:
        """Leader: ship the newest state to every standby that lacks it (a heartbeat to the
        others) and advance ``committed`` when a majority holds it."""
        term = self.term
        mut = self.state.mutations
        if mut != self._built_mut:
            self._built_mut = mut
            self.version = (term, self.version[1] + 1 if self.version[0] == term else 1)
            self.snapshot = self.state.snapshot()
            self._built.append((mut, self.version))
            del self._built[:-256]
            await self._persist()
        ver = self.version
        snap = self.snapshot

        async def send(p: int):
            body = {"term": term, "leader": self.id, "version": list(ver)}
            if tuple(self._peer_ver.get(p, (0, 0))) < ver:
                body["snapshot"] = snap
            return p, await self._rpc(p, "/quorum/append", body)
        res = await asyncio.gather(*[send(p) for p in self.others])
        if self.role != "leader" or self.term != term:
            return False
        acks = 1                                    # this member persisted ver above
        for p, r in res:
            if r is None:
                continue
            if int(r["term"]) > term:
                self.term = int(r["term"])
                self.voted_for = None
                await self._persist()
                self._step_down(None)
                return False
            if r.get("ok"):
                self._peer_ver[p] = tuple(r["version"])
                if tuple(r["version"]) >= ver:
                    acks += 1
        self.rounds += 1
        if acks < self.majority:
            self.round_failures += 1
            return False
        self._last_majority = self.clock()
        if not self.ready and ver[0] == term:      # the takeover round of this term is committed
            self.ready = True
            print(f"[kafka-controller] member {self.id}: ACTIVE for term {term} (state version {list(ver)})",
                  flush=True)
        if ver > self.committed:
            self.committed = ver
            for m, v in self._built:
                if v == ver:
                    self.committed_mut = max(self.committed_mut, m)
            async with self._cv:
                self._cv.notify_all()
        return True

    def on_append(self, d: Dict[str, Any]) -> Dict[str, Any]:
        term, leader = int(d["term"]), int(d["leader"])
        if term < self.term:
            return {"term": self.term, "ok": False, "version": list(self.version)}
        changed = False
        if term > self.term:
            self.term = term
            self.voted_for = None
            changed = True
        if self.role != "follower" or self.leader_id != leader:
            self._step_down(leader)
        self.last_contact = self.clock()
        self._deadline = self._new_deadline()
        ver = tuple(d["version"])
        if d.get("snapshot") is not None and ver > self.version:
            self.snapshot = d["snapshot"]
            self.version = ver
            changed = True
        if changed:
            self._persist_sync()                    # the ack promises it is on disk
        return {"term": self.term, "ok": True, "version": list(self.version)}

    async def commit_mutation(self, timeout_s: float = 3.0) -> bool:
        """Active: wait until the state as of now is held by a majority (False: this member
        lost the active role or the majority, the caller answers 503 and the client retries)."""
        if not self.is_active():
            return False
        want_mut = self.state.mutations
        t_end = self.clock() + timeout_s
        while True:
            if not self.is_active():
                return False
            if self.committed_mut >= want_mut:
                return True
            self._kick.set()
            left = t_end - self.clock()
            if left <= 0:
                return False
            async with self._cv:
                try:
                    await asyncio.wait_for(self._cv.wait(), min(left, self.hb_s * 2))
                except asyncio.TimeoutError:
                    pass

    def status(self) -> Dict[str, Any]:
        return {"id": self.id, "role": self.role, "active": self.is_active(), "term": self.term,
                "leader": self.leader_id, "leader_url": self.leader_url(), "version": list(self.version),
                "committed": list(self.committed), "elections_won": self.elections_won, "rounds": self.rounds,
                "round_failures": self.round_failures, "members": len(self.peers)}
