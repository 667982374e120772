"""``kafka-lite``: a single-node broker speaking the Kafka wire protocol subset of
``kafka_wire`` on top of the in-process log store.

Stands in for the reference's 3-broker Strimzi cluster (deploy/frauddetection_cr.yaml:
73-77) in development, CI and single-node deployments: every service of the framework
(producer, engine/router, KIE, notifier) can run as a separate process and talk real Kafka
protocol to it, and switching to a production cluster is only a ``BROKER_URL`` change.

    python -m ccfd_demo_summit_amd.ingest.kafka_lite --port 9092 --partitions 8
"""
from __future__ import annotations

import argparse
import asyncio
import itertools
import struct
import threading
import time
from typing import Dict, Optional, Set

from .broker import InProcBroker
from .kafka_wire import (API_VERSIONS, CREATE_TOPICS, ERR_NONE, ERR_OFFSET_OUT_OF_RANGE, ERR_TOPIC_EXISTS,
                         ERR_UNKNOWN_TOPIC, ERR_UNSUPPORTED_VERSION, FETCH, FIND_COORDINATOR, LIST_OFFSETS,
                         METADATA, OFFSET_COMMIT, OFFSET_FETCH, PRODUCE, SUPPORTED, Reader, Writer,
                         decode_record_batches, encode_record_batch)

NODE_ID = 1
ERR_ILLEGAL_GENERATION, ERR_UNKNOWN_MEMBER, ERR_REBALANCE_IN_PROGRESS = 22, 25, 27


class _Member:
    def __init__(self, mid: str, session_ms: int, rebalance_ms: int):
        self.mid = mid
        self.session_s = session_ms / 1000.0
        self.rebalance_s = rebalance_ms / 1000.0
        self.metadata = b""
        self.assignment = b""
        self.last_seen = time.monotonic()
        self.join_fut: Optional[asyncio.Future] = None
        self.sync_fut: Optional[asyncio.Future] = None


class _Group:
    """Classic group coordinator state: Empty -> PreparingRebalance (members rejoin) ->
    CompletingRebalance (leader's SyncGroup) -> Stable."""

    def __init__(self):
        self.state = "Empty"
        self.generation = 0
        self.members: Dict[str, _Member] = {}
        self.joined: Set[str] = set()
        self.leader = ""
        self.deadline_task: Optional[asyncio.Task] = None


class BrokerMetrics:
    """The Strimzi/JMX-exporter series the reference's Kafka dashboard queries
    (deploy/grafana/Kafka.json:119-1093): topic message/byte rates, failed requests,
    partition/leader counts; under-replicated / offline partitions are 0 on one node."""

    def __init__(self, server: "KafkaLiteServer"):
        from prometheus_client import CollectorRegistry, Counter
        from prometheus_client.core import GaugeMetricFamily
        self.registry = CollectorRegistry()
        lab = ["topic", "strimzi_io_kind"]
        mk = lambda n, d: Counter(f"kafka_server_brokertopicmetrics_{n}", d, lab, registry=self.registry)
        self.messages_in = mk("messagesin", "messages produced")
        self.bytes_in = mk("bytesin", "bytes produced")
        self.bytes_out = mk("bytesout", "bytes fetched")
        self.failed_produce = mk("failedproducerequests", "failed produce requests")
        self.failed_fetch = mk("failedfetchrequests", "failed fetch requests")
        srv = server

        class _Gauges:
            def collect(self_):
                parts = sum(srv.store.partitions(t) for t in srv.store.topics())
                for name, v in (("kafka_server_replicamanager_partitioncount", parts),
                                ("kafka_server_replicamanager_leadercount", parts),
                                ("kafka_server_replicamanager_underreplicatedpartitions", 0),
                                ("kafka_controller_kafkacontroller_offlinepartitionscount", 0)):
                    g = GaugeMetricFamily(name, name, labels=["strimzi_io_kind"])
                    g.add_metric(["Kafka"], v)
                    yield g
        self.registry.register(_Gauges())

    def expose(self) -> bytes:
        from prometheus_client import generate_latest
        return generate_latest(self.registry)


class KafkaLiteServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 9092, default_partitions: int = 1,
                 store: Optional[InProcBroker] = None, auto_create: bool = True):
        self.host = host
        self.port = port
        self.store = store or InProcBroker(default_partitions=default_partitions)
        self.auto_create = auto_create
        self._server: Optional[asyncio.base_events.Server] = None
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._thread: Optional[threading.Thread] = None
        self.metrics = BrokerMetrics(self)
        self.groups: Dict[str, _Group] = {}
        self._mid = itertools.count(1)
        self._reaper: Optional[asyncio.Task] = None

    # ------------------------------------------------------------------ lifecycle
    async def start(self):
        self._server = await asyncio.start_server(self._serve, self.host, self.port)
        self.port = self._server.sockets[0].getsockname()[1]
        self._reaper = asyncio.get_running_loop().create_task(self._reap_sessions())

    def start_in_thread(self) -> "KafkaLiteServer":
        ready = threading.Event()

        def run():
            self._loop = asyncio.new_event_loop()
            self._loop.run_until_complete(self.start())
            ready.set()
            self._loop.run_forever()
        self._thread = threading.Thread(target=run, daemon=True, name="kafka-lite")
        self._thread.start()
        ready.wait(10)
        return self

    def stop(self):
        if self._loop is not None:
            async def _shutdown():
                self._server.close()
                me = asyncio.current_task()
                tasks = [t for t in asyncio.all_tasks() if t is not me]
                for t in tasks:                      # open connection handlers
                    t.cancel()
                await asyncio.gather(*tasks, return_exceptions=True)
                self._loop.stop()
            asyncio.run_coroutine_threadsafe(_shutdown(), self._loop)
            self._thread.join(5)

    @property
    def bootstrap(self) -> str:
        return f"{self.host}:{self.port}"

    # ------------------------------------------------------------------ connection loop
    async def _serve(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        try:
            while True:
                hdr = await reader.readexactly(4)
                size = struct.unpack(">i", hdr)[0]
                msg = await reader.readexactly(size)
                r = Reader(msg)
                api, ver, corr = r.i16(), r.i16(), r.i32()
                r.string()                                  # client id
                body = self._dispatch(api, ver, r)
                if not isinstance(body, (bytes, bytearray)):   # group APIs long-poll (JoinGroup, SyncGroup)
                    body = await body
                out = struct.pack(">i", corr) + body
                writer.write(struct.pack(">i", len(out)) + out)
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        finally:
            writer.close()

    def _topic(self, name: str) -> bool:
        if name in self.store.topics():
            return True
        if self.auto_create:
            self.store.create_topic(name)
            return True
        return False

    def _dispatch(self, api: int, ver: int, r: Reader) -> bytes:
        if api not in SUPPORTED or ver > SUPPORTED[api]:
            return Writer().i16(ERR_UNSUPPORTED_VERSION).build()
        return getattr(self, f"_api_{api}")(r)

    # ------------------------------------------------------------------ APIs
    def _api_18(self, r: Reader) -> bytes:                  # ApiVersions v0
        return Writer().i16(ERR_NONE).array(sorted(SUPPORTED.items()), lambda w, kv: w.i16(kv[0]).i16(0).i16(kv[1])).build()

    def _api_3(self, r: Reader) -> bytes:                   # Metadata v1
        topics = r.array(lambda x: x.string())
        names = sorted(self.store.topics()) if topics is None else topics
        w = Writer().array([(NODE_ID, self.host, self.port)], lambda w_, b: w_.i32(b[0]).string(b[1]).i32(b[2]).string(None))
        w.i32(NODE_ID)

        def topic(w_, name):
            if not self._topic(name):
                w_.i16(ERR_UNKNOWN_TOPIC).string(name).i8(0).array([], None)
                return
            n = self.store.partitions(name)
            w_.i16(ERR_NONE).string(name).i8(0).array(range(n), lambda w2, p: w2.i16(0).i32(p).i32(NODE_ID)
                                                   .array([NODE_ID], lambda w3, x: w3.i32(x))
                                                   .array([NODE_ID], lambda w3, x: w3.i32(x)))
        w.array(names, topic)
        return w.build()

    def _api_19(self, r: Reader) -> bytes:                  # CreateTopics v0
        def req(x):
            name, n, _rf = x.string(), x.i32(), x.i16()
            x.array(lambda y: (y.i32(), y.array(lambda z: z.i32())))
            x.array(lambda y: (y.string(), y.string()))
            return name, n
        reqs = r.array(req)
        r.i32()
        res = []
        for name, n in reqs:
            if name in self.store.topics():
                res.append((name, ERR_TOPIC_EXISTS))
            else:
                self.store.create_topic(name, max(1, n))
                res.append((name, ERR_NONE))
        return Writer().array(res, lambda w, t: w.string(t[0]).i16(t[1])).build()

    def _api_0(self, r: Reader) -> bytes:                   # Produce v3
        r.string(); r.i16(); r.i32()
        data = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.bytes_()))))
        resp = []
        for topic, parts in data:
            pr = []
            self._topic(topic)
            for p, rb in parts:
                try:
                    recs = decode_record_batches(rb or b"", topic, p)
                    base = self.store.end_offset(topic, p)
                    for rec in recs:
                        self.store.produce(topic, rec.value, key=rec.key, partition=p)
                    pr.append((p, ERR_NONE, base))
                    self.metrics.messages_in.labels(topic, "Kafka").inc(len(recs))
                    self.metrics.bytes_in.labels(topic, "Kafka").inc(len(rb or b""))
                except Exception:
                    pr.append((p, 2, -1))
                    self.metrics.failed_produce.labels(topic, "Kafka").inc()
            resp.append((topic, pr))
        w = Writer().array(resp, lambda w_, t: w_.string(t[0]).array(t[1], lambda w2, q: w2.i32(q[0]).i16(q[1]).i64(q[2]).i64(-1)))
        return w.i32(0).build()

    def _api_1(self, r: Reader) -> bytes:                   # Fetch v4
        r.i32(); r.i32(); r.i32(); max_bytes = r.i32(); r.i8()
        reqs = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i64(), y.i32()))))
        resp = []
        for topic, parts in reqs:
            pr = []
            for p, off, pmax in parts:
                if topic not in self.store.topics() or p >= self.store.partitions(topic):
                    pr.append((p, ERR_UNKNOWN_TOPIC, -1, None))
                    self.metrics.failed_fetch.labels(topic, "Kafka").inc()
                    continue
                hw = self.store.end_offset(topic, p)
                if off < self.store.begin_offset(topic, p) or off > hw:
                    pr.append((p, ERR_OFFSET_OUT_OF_RANGE, hw, None))
                    self.metrics.failed_fetch.labels(topic, "Kafka").inc()
                    continue
                recs, size = [], 0
                for rec in self.store.fetch(topic, p, off, 100_000):
                    size += len(rec.value or b"") + 32
                    if recs and size > min(pmax, max_bytes):
                        break
                    recs.append(rec)
                rb = encode_record_batch([x.value for x in recs], [x.key for x in recs], base_offset=off) if recs else b""
                pr.append((p, ERR_NONE, hw, rb))
                if rb:
                    self.metrics.bytes_out.labels(topic, "Kafka").inc(len(rb))
            resp.append((topic, pr))
        w = Writer().i32(0)
        w.array(resp, lambda w_, t: w_.string(t[0]).array(
            t[1], lambda w2, q: w2.i32(q[0]).i16(q[1]).i64(q[2]).i64(q[2]).array([], None).bytes_(q[3])))
        return w.build()

    def _api_2(self, r: Reader) -> bytes:                   # ListOffsets v1
        r.i32()
        reqs = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i64()))))
        resp = []
        for topic, parts in reqs:
            pr = []
            for p, ts in parts:
                if not self._topic(topic) or p >= self.store.partitions(topic):
                    pr.append((p, ERR_UNKNOWN_TOPIC, -1))
                    continue
                off = self.store.begin_offset(topic, p) if ts == -2 else self.store.end_offset(topic, p)
                pr.append((p, ERR_NONE, off))
            resp.append((topic, pr))
        return Writer().array(resp, lambda w_, t: w_.string(t[0]).array(
            t[1], lambda w2, q: w2.i32(q[0]).i16(q[1]).i64(-1).i64(q[2]))).build()

    def _api_10(self, r: Reader) -> bytes:                  # FindCoordinator v0
        r.string()
        return Writer().i16(ERR_NONE).i32(NODE_ID).string(self.host).i32(self.port).build()

    def _api_8(self, r: Reader) -> bytes:                   # OffsetCommit v2
        group = r.string(); r.i32(); r.string(); r.i64()
        reqs = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i64(), y.string()))))
        resp = []
        for topic, parts in reqs:
            for p, off, _m in parts:
                self.store.commit(group, topic, p, off)
            resp.append((topic, [(p, ERR_NONE) for p, _o, _m in parts]))
        return Writer().array(resp, lambda w_, t: w_.string(t[0]).array(t[1], lambda w2, q: w2.i32(q[0]).i16(q[1]))).build()

    def _api_9(self, r: Reader) -> bytes:                   # OffsetFetch v1
        group = r.string()
        reqs = r.array(lambda x: (x.string(), x.array(lambda y: y.i32())))
        resp = []
        for topic, parts in reqs:
            pr = []
            for p in parts:
                c = self.store.committed(group, topic, p)
                pr.append((p, -1 if c is None else c))
            resp.append((topic, pr))
        return Writer().array(resp, lambda w_, t: w_.string(t[0]).array(
            t[1], lambda w2, q: w2.i32(q[0]).i64(q[1]).string(None).i16(ERR_NONE))).build()


    # ------------------------------------------------------------------ group coordinator
    # JoinGroup v1 / SyncGroup v0 / Heartbeat v0 / LeaveGroup v0 (client: ingest/kafka_group.py)
    def _prepare_rebalance(self, g: _Group, rebalance_s: float) -> None:
        if g.state == "PreparingRebalance":
            return
        g.state = "PreparingRebalance"
        g.joined = set()
        for m in g.members.values():                 # members parked in SyncGroup must rejoin
            if m.sync_fut is not None and not m.sync_fut.done():
                m.sync_fut.set_result(Writer().i16(ERR_REBALANCE_IN_PROGRESS).bytes_(b"").build())
            m.sync_fut = None
        if g.deadline_task is not None:
            g.deadline_task.cancel()

        async def deadline():
            await asyncio.sleep(rebalance_s)
            if g.state == "PreparingRebalance":     # stragglers are dropped from the group
                for mid in [m for m in g.members if m not in g.joined]:
                    del g.members[mid]
                self._maybe_complete_join(g)
        g.deadline_task = asyncio.get_running_loop().create_task(deadline())

    def _maybe_complete_join(self, g: _Group) -> None:
        if g.state != "PreparingRebalance" or not g.joined >= set(g.members):
            return
        if g.deadline_task is not None:
            g.deadline_task.cancel()
            g.deadline_task = None
        if not g.members:
            g.state = "Empty"
            return
        g.generation += 1
        if g.leader not in g.members:
            g.leader = sorted(g.members)[0]
        g.state = "CompletingRebalance"
        everyone = [(m.mid, m.metadata) for m in g.members.values()]
        for m in g.members.values():
            m.last_seen = time.monotonic()
            body = (Writer().i16(ERR_NONE).i32(g.generation).string("range").string(g.leader).string(m.mid)
                    .array(everyone if m.mid == g.leader else [], lambda w, e: w.string(e[0]).bytes_(e[1])).build())
            if m.join_fut is not None and not m.join_fut.done():
                m.join_fut.set_result(body)
            m.join_fut = None

    def _remove_member(self, g: _Group, mid: str) -> None:
        m = g.members.pop(mid, None)
        if m is None:
            return
        g.joined.discard(mid)
        if g.members:
            self._prepare_rebalance(g, max(x.rebalance_s for x in g.members.values()))
            self._maybe_complete_join(g)
        else:
            g.state = "Empty"

    async def _reap_sessions(self):
        while True:
            await asyncio.sleep(0.1)
            now = time.monotonic()
            for g in self.groups.values():
                for mid, m in list(g.members.items()):
                    parked = m.join_fut is not None and not m.join_fut.done()
                    if not parked and now - m.last_seen > m.session_s:
                        self._remove_member(g, mid)

    def _api_11(self, r: Reader):                           # JoinGroup v1 (long poll)
        group, session_ms, rebalance_ms, mid, _ptype = r.string(), r.i32(), r.i32(), r.string(), r.string()
        protos = dict(r.array(lambda x: (x.string(), x.bytes_())) or [])
        g = self.groups.setdefault(group, _Group())
        if mid and mid not in g.members:
            return Writer().i16(ERR_UNKNOWN_MEMBER).i32(-1).string("").string("").string(mid).array([], None).build()
        if not mid:
            mid = f"member-{next(self._mid)}"
            g.members[mid] = _Member(mid, session_ms, rebalance_ms)
        m = g.members[mid]
        m.metadata = protos.get("range", b"")
        m.last_seen = time.monotonic()
        fut = asyncio.get_running_loop().create_future()
        m.join_fut = fut
        self._prepare_rebalance(g, rebalance_ms / 1000.0)
        g.joined.add(mid)
        self._maybe_complete_join(g)
        return fut

    def _api_14(self, r: Reader):                           # SyncGroup v0
        group, gen, mid = r.string(), r.i32(), r.string()
        assignments = r.array(lambda x: (x.string(), x.bytes_())) or []
        g = self.groups.get(group)
        err = None
        if g is None or mid not in g.members:
            err = ERR_UNKNOWN_MEMBER
        elif g.state == "PreparingRebalance":
            err = ERR_REBALANCE_IN_PROGRESS
        elif gen != g.generation:
            err = ERR_ILLEGAL_GENERATION
        if err is not None:
            return Writer().i16(err).bytes_(b"").build()
        m = g.members[mid]
        m.last_seen = time.monotonic()
        if mid == g.leader and g.state == "CompletingRebalance":
            for member, a in assignments:
                if member in g.members:
                    g.members[member].assignment = a
            g.state = "Stable"
            for o in g.members.values():
                if o.sync_fut is not None and not o.sync_fut.done():
                    o.sync_fut.set_result(Writer().i16(ERR_NONE).bytes_(o.assignment).build())
                o.sync_fut = None
        if g.state == "Stable":
            return Writer().i16(ERR_NONE).bytes_(m.assignment).build()
        fut = asyncio.get_running_loop().create_future()
        m.sync_fut = fut
        return fut

    def _api_12(self, r: Reader) -> bytes:                  # Heartbeat v0
        group, gen, mid = r.string(), r.i32(), r.string()
        g = self.groups.get(group)
        if g is None or mid not in g.members:
            return Writer().i16(ERR_UNKNOWN_MEMBER).build()
        g.members[mid].last_seen = time.monotonic()
        if g.state == "PreparingRebalance":
            return Writer().i16(ERR_REBALANCE_IN_PROGRESS).build()
        if gen != g.generation:
            return Writer().i16(ERR_ILLEGAL_GENERATION).build()
        return Writer().i16(ERR_NONE).build()

    def _api_13(self, r: Reader) -> bytes:                  # LeaveGroup v0
        group, mid = r.string(), r.string()
        g = self.groups.get(group)
        if g is None or mid not in g.members:
            return Writer().i16(ERR_UNKNOWN_MEMBER).build()
        self._remove_member(g, mid)
        return Writer().i16(ERR_NONE).build()

def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=9092)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--metrics-port", type=int, default=9404, help="Prometheus /metrics (0 = off)")
    a = ap.parse_args(argv)
    srv = KafkaLiteServer(a.host, a.port, a.partitions)

    async def run():
        await srv.start()
        if a.metrics_port:
            from aiohttp import web
            app = web.Application()
            app.router.add_get("/metrics", lambda _r: web.Response(
                body=srv.metrics.expose(), headers={"Content-Type": "text/plain; version=0.0.4"}))
            runner = web.AppRunner(app)
            await runner.setup()
            await web.TCPSite(runner, a.host, a.metrics_port).start()
        print(f"[kafka-lite] listening on {a.host}:{srv.port}", flush=True)
        await asyncio.Event().wait()
    asyncio.run(run())


if __name__ == "__main__":
    main()
