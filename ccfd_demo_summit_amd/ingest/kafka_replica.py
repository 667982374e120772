"""Broker side of replicated, multi-process kafka-lite.

Each broker process owns ONE durable log (ingest/durable_store.py) and leads the partitions
the controller (ingest/kafka_controller.py) gives it; the other replicas of a partition are
followers that replicate by FETCHING from the leader, as Kafka's replica fetchers do:

* **followers** run one fetcher THREAD per leader broker (off the event loop): a Kafka Fetch v4 with ``replica_id`` =
  their node id, from their log end offset (LEO), appended verbatim at the leader's offsets
  (``BatchStore.append_replica``) and written by the store's writer right behind -- the next
  fetch reports the in-memory LEO, which is what the leader counts;
* **the leader** tracks each follower's LEO from its fetches; the partition's high watermark
  (HW) is the minimum LEO over the in-sync replicas (ISR).  Consumers only see offsets below
  the HW; a produce with ``acks=all`` (-1) is answered once the HW covers it, so an
  acknowledged record is on every ISR member.  The LEOs are IN-MEMORY log ends (a follower
  reports its log end at its next fetch, before its background writer has written it), so the
  guarantee assumes no correlated crash of every ISR member within the write-behind window --
  Kafka's page-cache assumption.  With the leader alone in the ISR there is no second copy to
  cover that window: the HW then counts the leader's WRITTEN offset only;
* **ISR**: the leader proposes (in its next heartbeat) to drop a follower that has not caught
  up for ``replica_lag_s`` and to re-admit one that has caught up; the controller applies
  proposals of the current leader epoch only;
* **fail-over**: the controller elects the live ISR member with the highest LEO (it holds
  every acknowledged record).  Every other replica -- a deposed leader included -- cuts its log
  to the HW it knows when it starts following a new leader, and re-fetches from there, so its
  log is a prefix of the leader's.  A broker that restarts cuts its logs to its checkpointed
  HW (``replication.json``, every 200 ms) -- except where it was the sole ISR member (its log is
  then the authority; becoming sole is checkpointed synchronously, before any answer relies
  on it);
* **pipelined producers** (``max.in.flight`` > 1, kafka_wire.py) keep one request in flight
  per partition, so a refused batch is never overtaken by a later one;
* producer ids are per-broker disjoint (``node + 1024 k``) and the idempotent-producer state
  is replicated with the batches, so a batch retried against a new leader is stored once.

The under-replicated gauge (``kafka_server_replicamanager_underreplicatedpartitions``, the
reference Kafka dashboard's panel, deploy/grafana/Kafka.json:271) counts the partitions this
broker leads whose ISR is smaller than their replica set.
"""
from __future__ import annotations

import asyncio
import heapq
import json
import os
import socket
import struct
import threading
import time
import uuid
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from .broker import BrokerError
from .kafka_controller import tp_key, tp_split

TP = Tuple[str, int]
PID_STRIDE = 1024                      # producer ids: node + PID_STRIDE * k (disjoint per broker)
FETCH, FETCH_V, LIST_OFFSETS = 1, 4, 2


def load_checkpoint(data_dir: Optional[str]) -> Dict[TP, int]:
    """The recovery cut of a restarting broker: (topic, partition) -> checkpointed HW, for the
    partitions where it was NOT the sole in-sync replica."""
    if not data_dir:
        return {}
    p = os.path.join(data_dir, "replication.json")
    if not os.path.exists(p):
        return {}
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, json.JSONDecodeError):
        return {}
    sole = set(d.get("sole", []))
    return {tp_split(k): int(v) for k, v in d.get("hw", {}).items() if k not in sole}


def _write_json_atomic(path: str, obj: Dict[str, Any]) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, path)


class ReplicaManager:
    def __init__(self, node_id: int, advertise_host: str, port: int, controller_url: str, store, server=None,
                 hb_s: float = 0.1, replica_lag_s: float = 5.0, data_dir: Optional[str] = None):
        self.node_id = int(node_id)
        self.host = advertise_host
        self.port = int(port)
        # one controller URL, or the members of a replicated controller (comma-separated):
        # requests go to the active member, found by following 421 {"leader": url} answers
        self.controllers = [u.strip().rstrip("/") for u in controller_url.split(",") if u.strip()]
        self.controller = self.controllers[0]
        self.controller_failovers = 0
        self.store = store
        self.server = server                      # KafkaLiteServer: fetch wake-ups
        self.hb_s = float(hb_s)
        self.replica_lag_s = float(replica_lag_s)
        self.data_dir = data_dir
        self.incarnation = uuid.uuid4().hex
        self.meta_epoch = -1
        self.parts: Dict[TP, Dict[str, Any]] = {}
        self.nodes: Dict[int, Tuple[str, int]] = {}
        self.topics: Dict[str, int] = {}
        self.hw: Dict[TP, int] = {}
        self.fol: Dict[TP, Dict[int, List[float]]] = {}     # leader: follower -> [leo, fetched at, caught up at]
        self._acks: Dict[TP, list] = {}                      # leader: heap of (end offset, seq, future)
        self._ack_seq = 0
        self._isr_prop: Dict[TP, Dict[str, Any]] = {}
        self._fetchers: Dict[int, Any] = {}
        self._stopping = False
        # follower fetchers: a thread per leader (default; round-6 pass E2: RF-3 JSON produce ->
        # scored p99 4.3 ms vs 15.5 ms as event-loop tasks at 1024-message produces) or a task
        # on the broker's event loop (=loop)
        self.fetch_mode = os.environ.get("CCFD_REPLICA_FETCH", "thread")
        # a fetcher thread checks a partition's leader epoch and appends under this lock, and
        # new metadata is applied under it: no append from a deposed leader's response can
        # land after the truncation that starts following the new one
        self._follow_lock = threading.RLock()
        self._tasks: List[asyncio.Task] = []
        self._session = None
        self.ready = None                                    # asyncio.Event: first metadata applied
        self.controller_ok = False
        self.replica_fetches = 0
        self.replicated_bytes = 0
        self.fetch_errors: Dict[str, int] = {}       # "leader/topic/p:code" -> count (status line)
        self.isr_changes = 0
        self.resets = 0                               # partitions restarted at the leader's log start
        self.report_s = float(os.environ.get("CCFD_KAFKA_REPL_REPORT_S", "5"))
        self.hb_failures = 0
        self._lead_since: Dict[TP, float] = {}
        self.truncations = 0
        self.truncated_batches = 0
        self._sole_ckpt: set = set()                  # sole-ISR partitions in replication.json

    # ------------------------------------------------------------------ lifecycle
    async def start(self) -> None:
        import aiohttp
        self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=5))
        self.ready = asyncio.Event()
        loop = asyncio.get_running_loop()
        self._tasks = [loop.create_task(self._hb_loop()), loop.create_task(self._isr_loop()),
                       loop.create_task(self._ckpt_loop()), loop.create_task(self._report_loop())]

    async def close(self) -> None:
        self._stopping = True                          # the fetcher threads leave at their next turn
        for t in self._tasks + [f for f in self._fetchers.values() if isinstance(f, asyncio.Task)]:
            t.cancel()
        if self._session is not None:
            await self._session.close()

    # ------------------------------------------------------------------ metadata view
    def leader(self, topic: str, p: int) -> int:
        st = self.parts.get((topic, p))
        return -1 if st is None else int(st["leader"])

    def is_leader(self, topic: str, p: int) -> bool:
        return self.leader(topic, p) == self.node_id

    def isr(self, topic: str, p: int) -> List[int]:
        st = self.parts.get((topic, p))
        return [] if st is None else list(st["isr"])

    def replicas(self, topic: str, p: int) -> List[int]:
        st = self.parts.get((topic, p))
        return [] if st is None else list(st["replicas"])

    def live_nodes(self) -> List[int]:
        return sorted(self.nodes)

    def under_replicated(self) -> int:
        return sum(1 for tp, st in self.parts.items()
                   if st["leader"] == self.node_id and len(st["isr"]) < len(st["replicas"]))

    def led(self) -> int:
        return sum(1 for st in self.parts.values() if st["leader"] == self.node_id)

    def hosted(self) -> List[TP]:
        return [tp for tp, st in self.parts.items() if self.node_id in st["replicas"]]

    def high_watermark(self, topic: str, p: int) -> int:
        return self.hw.get((topic, p), 0)

    def _leo(self, tp: TP) -> int:
        """This replica's log end offset as appended, written or not: the high watermark is
        the minimum of these over the ISR, so a record below it is in the memory of every
        in-sync broker (and on its way to each one's disk) -- one broker's death loses nothing
        acknowledged, and consumer latency does not wait on the leader's own disk writes
        (Kafka counts the page cache the same way)."""
        try:
            return self.store.log_end(*tp)
        except BrokerError:
            return 0

    async def _ctl(self, path: str, body: Dict[str, Any], wait_s: float = 5.0) -> Tuple[int, Dict[str, Any]]:
        """POST to the active controller: a standby's 421 names the active member, an
        unreachable one or a 503 (the active lost its majority mid-request) moves on to the
        next member; gives up after ``wait_s`` (an election takes well under a second)."""
        t_end = time.monotonic() + wait_s
        last = "unreachable"
        while True:
            url = self.controller
            try:
                async with self._session.post(url + path, json=body) as r:
                    d = await r.json(content_type=None)
                    if r.status == 421 or (r.status == 503 and len(self.controllers) > 1
                                           and "majority" in str(d.get("error", ""))):
                        lead = d.get("leader")
                        self._next_controller(lead if lead in self.controllers else None)
                        last = f"HTTP {r.status} from {url}"
                    else:
                        return r.status, d
            except (OSError, asyncio.TimeoutError, ValueError) as e:
                self._next_controller(None)
                last = f"{url}: {e!r}"
            except Exception as e:                           # noqa: BLE001 -- aiohttp client errors
                self._next_controller(None)
                last = f"{url}: {e!r}"
            if time.monotonic() > t_end:
                raise BrokerError(f"no active controller ({last})")
            await asyncio.sleep(0.05)

    def _next_controller(self, url: Optional[str]) -> None:
        if len(self.controllers) <= 1:
            return
        if url is None:
            i = self.controllers.index(self.controller) if self.controller in self.controllers else -1
            url = self.controllers[(i + 1) % len(self.controllers)]
        if url != self.controller:
            self.controller = url
            self.controller_failovers += 1

    async def create_topic(self, name: str, partitions: int, wait_s: float = 30.0) -> None:
        """Through the controller; while it waits for the cluster's brokers to register (503),
        asked again every 200 ms."""
        t_end = time.monotonic() + wait_s
        while True:
            status, d = await self._ctl("/topics", {"name": name, "partitions": int(partitions)})
            if status == 200:
                break
            if time.monotonic() > t_end:
                raise BrokerError(f"controller: {d.get('error')}")
            await asyncio.sleep(0.2)
        self._apply(d)

    async def commit_offsets(self, group: str, entries) -> None:
        status, _d = await self._ctl("/offsets/commit", {"group": group, "offsets": [list(e) for e in entries]})
        if status != 200:
            raise BrokerError(f"controller commit: HTTP {status}")

    async def fetch_offsets(self, group: str, tps) -> List[int]:
        status, d = await self._ctl("/offsets/fetch", {"group": group, "tps": [list(t) for t in tps]})
        if status != 200:
            raise BrokerError(f"controller offset fetch: HTTP {status}")
        return d["offsets"]

    # ------------------------------------------------------------------ heartbeat
    async def _hb_loop(self) -> None:
        while True:
            body = {"node": self.node_id, "host": self.host, "port": self.port, "incarnation": self.incarnation,
                    "seen_epoch": self.meta_epoch,
                    "leos": {tp_key(*tp): self._leo(tp) for tp in self.hosted()},
                    "isr_changes": list(self._isr_prop.values())}
            try:
                status, d = await self._ctl("/heartbeat", body, wait_s=self.hb_s)
                if status != 200:
                    raise BrokerError(f"heartbeat: HTTP {status}")
                self._isr_prop.clear()
                self.controller_ok = True
                if "parts" in d:
                    self._apply(d)
                elif self.ready is not None and not self.ready.is_set() and self.meta_epoch >= 0:
                    self.ready.set()
            except Exception:                               # noqa: BLE001 -- controller away
                self.controller_ok = False
                self.hb_failures += 1
            await asyncio.sleep(self.hb_s)

    def _apply(self, d: Dict[str, Any]) -> None:
        """New metadata from the controller: leadership / ISR / topics / brokers."""
        if "parts" not in d:
            return
        with self._follow_lock:
            self._apply_locked(d)

    def _apply_locked(self, d: Dict[str, Any]) -> None:
        self.meta_epoch = int(d["meta_epoch"])
        self.nodes = {int(k): (v[0], int(v[1])) for k, v in d["nodes"].items()}
        for name, n in d["topics"].items():
            if name not in self.topics:
                self.store.create_topic(name, int(n))
            self.topics[name] = int(n)
        old = self.parts
        self.parts = {tp_split(k): v for k, v in d["parts"].items()}
        for tp, st in self.parts.items():
            was = old.get(tp)
            if st["leader"] == self.node_id and (was is None or was["leader"] != self.node_id
                                                 or was["epoch"] != st["epoch"]):
                # leader from now: followers' LEOs are unknown until they fetch
                self.fol[tp] = {}
                self.hw.setdefault(tp, 0)
                self._lead_since[tp] = time.monotonic()
            elif st["leader"] != self.node_id:
                self.fol.pop(tp, None)
                self._fail_acks(tp)
                # (no leader yet = an election in progress: this replica may be the one elected,
                # with acknowledged records above the HW it has heard of -- keep them)
                if self.node_id in st["replicas"] and st["leader"] >= 0 and (
                        was is None or was["leader"] != st["leader"] or was["epoch"] != st["epoch"]):
                    # a new leader: cut the tail this replica holds past the high watermark it
                    # knows (never acknowledged; a deposed leader's may not be on the new one),
                    # so the log is a prefix of the leader's before following it
                    self._truncate_to_hw(tp)
            if st["leader"] == self.node_id:
                self._advance_hw(tp)
        sole = self._sole()
        if sole - self._sole_ckpt:
            # newly sole ISR member: checkpoint that NOW -- a restart before the periodic write
            # would cut this log to an older HW and delete batches acknowledged meanwhile
            self._write_ckpt_sync()
        self._reconcile_fetchers()
        if self.ready is not None:
            self.ready.set()

    # ------------------------------------------------------------------ leader side
    def on_replica_fetch(self, node: int, topic: str, p: int, offset: int) -> None:
        tp = (topic, p)
        if not self.is_leader(topic, p):
            return
        now = time.monotonic()
        rec = self.fol.setdefault(tp, {}).setdefault(node, [0, now, 0.0, 0])
        # caught up = it now holds everything the leader held when it answered the previous
        # fetch (Kafka's lastCaughtUpTime): under a steady produce stream the leader's log end
        # has always moved on a little by the time the next fetch arrives
        if offset >= rec[3]:
            rec[2] = now
        rec[0], rec[1] = offset, now
        rec[3] = self._leo(tp)
        self._advance_hw(tp)

    def on_written(self, tps) -> None:
        """The leader's own write advanced its LEO."""
        for tp in tps:
            if self.is_leader(*tp):
                self._advance_hw(tp)

    def _written(self, tp: TP) -> int:
        """This replica's written (durable) log end."""
        try:
            return self.store.end_offset(*tp)
        except BrokerError:
            return 0

    def _advance_hw(self, tp: TP) -> None:
        st = self.parts.get(tp)
        if st is None or st["leader"] != self.node_id:
            return
        # alone in the ISR, nothing else holds an unwritten batch: count only what is written
        # (an in-memory LEO here would acknowledge acks=all records a crash could still lose)
        leos = [self._leo(tp) if len(st["isr"]) > 1 else self._written(tp)]
        fol = self.fol.get(tp, {})
        for n in st["isr"]:
            if n != self.node_id:
                leos.append(int(fol[n][0]) if n in fol else 0)
        new = min(leos)
        if new > self.hw.get(tp, 0):
            self.hw[tp] = new
            h = self._acks.get(tp)
            while h and h[0][0] <= new:
                _e, _s, fut = heapq.heappop(h)
                if not fut.done():
                    fut.set_result(True)
            if self.server is not None:
                self.server._wake_fetches(tp)

    def wait_hw(self, topic: str, p: int, end: int) -> "asyncio.Future":
        """Resolves once the HW reaches ``end`` (acks=all); fails if leadership is lost."""
        fut = asyncio.get_running_loop().create_future()
        tp = (topic, p)
        if self.hw.get(tp, 0) >= end:
            fut.set_result(True)
            return fut
        self._ack_seq += 1
        heapq.heappush(self._acks.setdefault(tp, []), (end, self._ack_seq, fut))
        return fut

    def _fail_acks(self, tp: TP) -> None:
        for _e, _s, fut in self._acks.pop(tp, []):
            if not fut.done():
                fut.set_result(False)                    # answered NOT_LEADER: the producer retries

    async def _isr_loop(self) -> None:
        while True:
            await asyncio.sleep(0.2)
            now = time.monotonic()
            for tp, st in list(self.parts.items()):
                if st["leader"] != self.node_id:
                    continue
                isr = list(st["isr"])
                fol = self.fol.get(tp, {})
                leo = self._leo(tp)
                new = list(isr)
                for n in st["replicas"]:
                    if n == self.node_id:
                        continue
                    rec = fol.get(n)
                    if n in isr:
                        lagging = rec is None or (rec[0] < leo and now - max(rec[2], 0.0) > self.replica_lag_s) \
                            or now - rec[1] > self.replica_lag_s
                        if lagging and (rec is not None or now - self._since(tp) > self.replica_lag_s):
                            new.remove(n)
                    elif rec is not None and rec[0] >= self.hw.get(tp, 0) and now - rec[1] < 1.0 \
                            and now - rec[2] < 1.0 and n in self.nodes:
                        new.append(n)
                if sorted(new) != sorted(isr):
                    self._isr_prop[tp] = {"tp": tp_key(*tp), "epoch": st["epoch"], "isr": new}

    async def _report_loop(self) -> None:
        """A status line every report_s (0 = off): what this broker replicates, its errors and
        how far the partitions it follows are behind their leaders' high watermarks."""
        if self.report_s <= 0:
            return
        last = (0, 0)
        while True:
            await asyncio.sleep(self.report_s)
            behind = {}
            for tp, st in self.parts.items():
                if st["leader"] != self.node_id and self.node_id in st["replicas"] and st["leader"] >= 0:
                    behind[tp_key(*tp)] = max(0, self.hw.get(tp, 0) - self.store.log_end(*tp))
            lead_isr = {tp_key(*tp): st["isr"] for tp, st in self.parts.items() if st["leader"] == self.node_id}
            mb = (self.replicated_bytes - last[1]) / 1e6 / self.report_s
            print(f"[kafka-lite] node {self.node_id} replication: {self.replica_fetches - last[0]} fetches, "
                  f"{mb:.1f} MB/s in; following {len(behind)} partitions, behind the HW by "
                  f"{sum(behind.values())} records (max {max(behind.values(), default=0)}); leading "
                  f"{len(lead_isr)}, ISR {json.dumps(lead_isr)}; errors {json.dumps(self.fetch_errors)}",
                  flush=True)
            last = (self.replica_fetches, self.replicated_bytes)

    def _since(self, tp: TP) -> float:
        """When this broker became leader of tp (a follower gets replica_lag_s to show up)."""
        return self._lead_since.setdefault(tp, time.monotonic())

    def _sole(self) -> set:
        return {tp_key(*tp) for tp, st in self.parts.items()
                if st["leader"] == self.node_id and st["isr"] == [self.node_id]}

    def _ckpt_body(self) -> Dict[str, Any]:
        hw = {}
        for tp, st in self.parts.items():
            if self.node_id in st["replicas"]:
                hw[tp_key(*tp)] = min(self.hw.get(tp, 0), self._leo(tp))
        sole = sorted(self._sole())
        return {"hw": hw, "sole": sole}

    def _write_ckpt_sync(self) -> None:
        if not self.data_dir:
            return
        body = self._ckpt_body()
        _write_json_atomic(os.path.join(self.data_dir, "replication.json"), body)
        self._sole_ckpt = set(body["sole"])

    async def _ckpt_loop(self) -> None:
        if not self.data_dir:
            return
        path = os.path.join(self.data_dir, "replication.json")
        while True:
            await asyncio.sleep(0.2)
            body = self._ckpt_body()
            # written off the event loop: the file replace alone took ~4-6 ms on the test boxes'
            # overlay filesystems, every 200 ms, in front of every fetch and produce
            await asyncio.get_running_loop().run_in_executor(None, _write_json_atomic, path, body)
            self._sole_ckpt = set(body["sole"])

    def _truncate_to_hw(self, tp: TP, hw: Optional[int] = None) -> None:
        h = self.hw.get(tp, 0) if hw is None else hw
        try:
            if self.store.log_end(*tp) > h:
                n = self.store.truncate(tp[0], tp[1], h)
                self.truncations += 1
                self.truncated_batches += n
        except BrokerError:
            pass

    # ------------------------------------------------------------------ follower side
    def _followed(self) -> Dict[int, List[TP]]:
        by: Dict[int, List[TP]] = {}
        for tp, st in self.parts.items():
            if self.node_id in st["replicas"] and st["leader"] not in (self.node_id, -1):
                by.setdefault(int(st["leader"]), []).append(tp)
        return by

    def _reconcile_fetchers(self) -> None:
        """One fetcher per leader this broker follows (event-loop thread): a thread
        (CCFD_REPLICA_FETCH=thread) or a task on the event loop (=loop, the default)."""
        want = self._followed()
        for node, th in list(self._fetchers.items()):
            done = th.done() if isinstance(th, asyncio.Task) else not th.is_alive()
            if node not in want and isinstance(th, asyncio.Task):
                th.cancel()
                done = True
            if done:
                del self._fetchers[node]
        for node in want:
            if node not in self._fetchers and node in self.nodes:
                if self.fetch_mode == "thread":
                    th = threading.Thread(target=self._fetch_thread, args=(node,), daemon=True,
                                          name=f"replica-fetch-{node}")
                    self._fetchers[node] = th
                    th.start()
                else:
                    self._fetchers[node] = asyncio.get_running_loop().create_task(self._fetch_loop(node))

    async def _fetch_loop(self, leader: int) -> None:
        from .kafka_wire import Reader, Writer
        corr = 0
        while True:
            tps = self._followed().get(leader, [])
            if not tps or leader not in self.nodes:
                return
            host, port = self.nodes[leader]
            loop = asyncio.get_running_loop()
            sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            sock.setblocking(False)
            try:
                await loop.sock_connect(sock, (host, port))
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                sock.close()
                await asyncio.sleep(0.1)
                continue

            async def recv_exact(n: int):
                # straight into one buffer of the response's size (uninitialised: a zero-filled
                # bytearray cost ~1 ms per large response): the fetched batches are stored as
                # views of it (no stream-buffer copies of replicated bytes)
                buf = np.empty(n, np.uint8)
                mv = memoryview(buf).cast("B")
                got = 0
                while got < n:
                    k = await loop.sock_recv_into(sock, mv[got:])
                    if k == 0:
                        raise ConnectionError("replica fetch: leader closed the connection")
                    got += k
                return buf
            try:
                while True:
                    tps = self._followed().get(leader, [])
                    if not tps:
                        return
                    by_topic: Dict[str, List[Tuple[int, int]]] = {}
                    for t, p in tps:                # fetch from this replica's log end, written or not
                        by_topic.setdefault(t, []).append((p, self.store.log_end(t, p)))
                    # bounded responses (8 MB, 2 MB a partition): a follower catching up from
                    # its leader's log start pulls GBs, and the leader's single event loop must
                    # keep answering produces and consumer fetches between those responses (64 MB
                    # ones stalled the consumers for seconds after a broker restart)
                    body = (Writer().i32(self.node_id).i32(200).i32(1).i32(8 << 20).i8(0)
                            .array(sorted(by_topic.items()), lambda w, kv: w.string(kv[0]).array(
                                kv[1], lambda w2, q: w2.i32(q[0]).i64(q[1]).i32(2 << 20))).build())
                    corr += 1
                    hdr = Writer().i16(FETCH).i16(FETCH_V).i32(corr).string(f"replica-{self.node_id}").build()
                    await loop.sock_sendall(sock, struct.pack(">i", len(hdr) + len(body)) + hdr + body)
                    size = struct.unpack(">i", await recv_exact(4))[0]
                    r = Reader(memoryview(await recv_exact(size)).cast("B"))
                    if r.i32() != corr:
                        raise BrokerError("replica fetch: correlation mismatch")
                    r.i32()                                          # throttle

                    def part(x):
                        idx, err, hw, _lso = x.i32(), x.i16(), x.i64(), x.i64()
                        x.array(lambda y: (y.i64(), y.i64()))
                        return idx, err, hw, x.view_()
                    resp = r.array(lambda x: (x.string(), x.array(part)))
                    moved = False
                    below = []
                    for t, parts in resp:
                        for p, err, hw, recs in parts:
                            if err == 1 and self.store.log_end(t, p) > int(hw):
                                # OFFSET_OUT_OF_RANGE past the leader's log: this replica holds
                                # a tail the leader never had -- cut it to the leader's HW
                                self._truncate_to_hw((t, p), int(hw))
                                continue
                            if err == 1:
                                below.append((t, p))                  # before the leader's log start?
                                continue
                            if err:
                                k = f"{leader}/{t}/{p}:{err}"
                                self.fetch_errors[k] = self.fetch_errors.get(k, 0) + 1
                                moved = True                          # not the leader any more
                                continue
                            if recs is not None and len(recs):
                                try:
                                    self.store.append_replica(t, p, recs)
                                except BrokerError:
                                    k = f"{leader}/{t}/{p}:gap"
                                    self.fetch_errors[k] = self.fetch_errors.get(k, 0) + 1
                                    raise
                                self.replicated_bytes += len(recs)
                            self.hw[(t, p)] = max(self.hw.get((t, p), 0), min(int(hw), self.store.log_end(t, p)))
                    if below:
                        # away longer than the leader's retention: restart these partitions at
                        # the leader's log start (ListOffsets earliest), as a Kafka follower does
                        corr += 1
                        lo_body = Writer().i32(self.node_id).array(
                            sorted({t for t, _ in below}), lambda w, t: w.string(t).array(
                                [q for tt, q in below if tt == t], lambda w2, q: w2.i32(q).i64(-2))).build()
                        lo_hdr = Writer().i16(LIST_OFFSETS).i16(1).i32(corr).string(f"replica-{self.node_id}").build()
                        await loop.sock_sendall(sock, struct.pack(">i", len(lo_hdr) + len(lo_body)) + lo_hdr + lo_body)
                        size = struct.unpack(">i", await recv_exact(4))[0]
                        r2 = Reader(memoryview(await recv_exact(size)).cast("B"))
                        if r2.i32() != corr:
                            raise BrokerError("replica list-offsets: correlation mismatch")
                        lo = r2.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i16(), y.i64(), y.i64()))))
                        for t, parts in lo:
                            for p, err, _ts, start in parts:
                                if err == 0 and self.store.log_end(t, p) < int(start):
                                    n = self.store.reset_to(t, p, int(start))
                                    self.resets += 1
                                    print(f"[kafka-lite] node {self.node_id}: {t}[{p}] was below leader {leader}'s "
                                          f"log start {start}: dropped {n} batches, following from there", flush=True)
                                else:
                                    k = f"{leader}/{t}/{p}:1"
                                    self.fetch_errors[k] = self.fetch_errors.get(k, 0) + 1
                                    moved = True
                    self.replica_fetches += 1
                    # the next fetch reports this log end to the leader at once, without waiting
                    # for the local write: an acknowledged batch is then on every in-sync
                    # replica (in memory, written by each broker's writer right behind) -- a
                    # single broker's death loses nothing acknowledged, as in Kafka, where a
                    # follower's append is its page cache
                    if moved:
                        await asyncio.sleep(0.05)
            except (OSError, BrokerError, ConnectionError):
                await asyncio.sleep(0.05)                            # leader away: metadata will move it
            finally:
                sock.close()

    def _fetch_thread(self, leader: int) -> None:
        """Replicate the partitions ``leader`` leads: Fetch v4 as replica ``node_id`` from this
        log's end, append verbatim, repeat.  A thread of its own, on a blocking socket, not a
        task on the broker's event loop: the response bytes (the whole produce stream of the
        partitions followed -- two thirds of what a broker receives at RF 3) are copied in by
        ``recv_into``, which releases the GIL, so that copy runs beside the loop that answers
        produces and consumer fetches instead of queueing in front of them (round 5: the RF-3
        JSON produce -> scored tail was those three loops' queueing)."""
        from .kafka_wire import Reader, Writer
        corr = 0
        while not self._stopping:
            tps = self._followed().get(leader, [])
            if not tps or leader not in self.nodes:
                self._fetchers.pop(leader, None)
                return
            host, port = self.nodes[leader]
            try:
                sock = socket.create_connection((host, port), timeout=5.0)
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                time.sleep(0.1)
                continue

            def recv_exact(n: int):
                # straight into one buffer of the response's size (uninitialised: a zero-filled
                # bytearray cost ~1 ms per large response): the fetched batches are stored as
                # views of it (no stream-buffer copies of replicated bytes)
                buf = np.empty(n, np.uint8)
                mv = memoryview(buf).cast("B")
                got = 0
                while got < n:
                    k = sock.recv_into(mv[got:])
                    if k == 0:
                        raise ConnectionError("replica fetch: leader closed the connection")
                    got += k
                return buf
            try:
                while not self._stopping:
                    tps = self._followed().get(leader, [])
                    if not tps:
                        return
                    # the leader epoch each partition is fetched under: a response that arrives
                    # after a leadership change is dropped, never appended
                    epochs = {tp: (self.parts[tp]["leader"], self.parts[tp]["epoch"]) for tp in tps}
                    by_topic: Dict[str, List[Tuple[int, int]]] = {}
                    for t, p in tps:                # fetch from this replica's log end, written or not
                        by_topic.setdefault(t, []).append((p, self.store.log_end(t, p)))
                    # bounded responses (8 MB, 2 MB a partition): a follower catching up from
                    # its leader's log start pulls GBs, and the leader's single event loop must
                    # keep answering produces and consumer fetches between those responses (64 MB
                    # ones stalled the consumers for seconds after a broker restart)
                    body = (Writer().i32(self.node_id).i32(200).i32(1).i32(8 << 20).i8(0)
                            .array(sorted(by_topic.items()), lambda w, kv: w.string(kv[0]).array(
                                kv[1], lambda w2, q: w2.i32(q[0]).i64(q[1]).i32(2 << 20))).build())
                    corr += 1
                    hdr = Writer().i16(FETCH).i16(FETCH_V).i32(corr).string(f"replica-{self.node_id}").build()
                    sock.sendall(struct.pack(">i", len(hdr) + len(body)) + hdr + body)
                    size = struct.unpack(">i", recv_exact(4))[0]
                    r = Reader(memoryview(recv_exact(size)).cast("B"))
                    if r.i32() != corr:
                        raise BrokerError("replica fetch: correlation mismatch")
                    r.i32()                                          # throttle

                    def part(x):
                        idx, err, hw, _lso = x.i32(), x.i16(), x.i64(), x.i64()
                        x.array(lambda y: (y.i64(), y.i64()))
                        return idx, err, hw, x.view_()
                    resp = r.array(lambda x: (x.string(), x.array(part)))
                    moved = False
                    below = []
                    for t, parts in resp:
                        for p, err, hw, recs in parts:
                            with self._follow_lock:                   # epoch check + append, atomic
                                cur = self.parts.get((t, p))          # against _apply
                                if cur is None or (cur["leader"], cur["epoch"]) != epochs.get((t, p)):
                                    moved = True                      # leadership moved meanwhile
                                    continue
                                if err == 1 and self.store.log_end(t, p) > int(hw):
                                    # OFFSET_OUT_OF_RANGE past the leader's log: this replica holds
                                    # a tail the leader never had -- cut it to the leader's HW
                                    self._truncate_to_hw((t, p), int(hw))
                                    continue
                                if err == 1:
                                    below.append((t, p))              # before the leader's log start?
                                    continue
                                if err:
                                    k = f"{leader}/{t}/{p}:{err}"
                                    self.fetch_errors[k] = self.fetch_errors.get(k, 0) + 1
                                    moved = True                      # not the leader any more
                                    continue
                                if recs is not None and len(recs):
                                    try:
                                        self.store.append_replica(t, p, recs)
                                    except BrokerError:
                                        k = f"{leader}/{t}/{p}:gap"
                                        self.fetch_errors[k] = self.fetch_errors.get(k, 0) + 1
                                        raise
                                    self.replicated_bytes += len(recs)
                                self.hw[(t, p)] = max(self.hw.get((t, p), 0), min(int(hw), self.store.log_end(t, p)))
                    if below:
                        # away longer than the leader's retention: restart these partitions at
                        # the leader's log start (ListOffsets earliest), as a Kafka follower does
                        corr += 1
                        lo_body = Writer().i32(self.node_id).array(
                            sorted({t for t, _ in below}), lambda w, t: w.string(t).array(
                                [q for tt, q in below if tt == t], lambda w2, q: w2.i32(q).i64(-2))).build()
                        lo_hdr = Writer().i16(LIST_OFFSETS).i16(1).i32(corr).string(f"replica-{self.node_id}").build()
                        sock.sendall(struct.pack(">i", len(lo_hdr) + len(lo_body)) + lo_hdr + lo_body)
                        size = struct.unpack(">i", recv_exact(4))[0]
                        r2 = Reader(memoryview(recv_exact(size)).cast("B"))
                        if r2.i32() != corr:
                            raise BrokerError("replica list-offsets: correlation mismatch")
                        lo = r2.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i16(), y.i64(), y.i64()))))
                        for t, parts in lo:
                            for p, err, _ts, start in parts:
                                with self._follow_lock:
                                    cur = self.parts.get((t, p))
                                    same = cur is not None and (cur["leader"], cur["epoch"]) == epochs.get((t, p))
                                    if same and err == 0 and self.store.log_end(t, p) < int(start):
                                        n = self.store.reset_to(t, p, int(start))
                                        self.resets += 1
                                        print(f"[kafka-lite] node {self.node_id}: {t}[{p}] was below leader {leader}'s "
                                              f"log start {start}: dropped {n} batches, following from there", flush=True)
                                    else:
                                        k = f"{leader}/{t}/{p}:1"
                                        self.fetch_errors[k] = self.fetch_errors.get(k, 0) + 1
                                        moved = True
                    self.replica_fetches += 1
                    # the next fetch reports this log end to the leader at once, without waiting
                    # for the local write: an acknowledged batch is then on every in-sync
                    # replica (in memory, written by each broker's writer right behind) -- a
                    # single broker's death loses nothing acknowledged, as in Kafka, where a
                    # follower's append is its page cache
                    if moved:
                        time.sleep(0.05)
            except (OSError, BrokerError, ConnectionError, ValueError):
                time.sleep(0.05)                                     # leader away: metadata will move it
            finally:
                sock.close()
