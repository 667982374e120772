"""``kafka-lite``: a broker (or a small multi-broker cluster) speaking the Kafka wire
protocol subset of ``kafka_wire``.

Stands in for the reference's 3-broker Strimzi cluster (deploy/frauddetection_cr.yaml:
73-77) in development, CI and single-node deployments: every service of the framework
(producer, engine/router, KIE, notifier) can run as a separate process and talk real Kafka
protocol to it, and switching to a production cluster is only a ``BROKER_URL`` change.

Storage keeps producer RecordBatches verbatim (``batch_store.py``): Produce validates the
CRC and stamps the base offset, Fetch slices stored batches -- no per-record work.  With
``--data-dir`` the logs, committed group offsets and idempotent-producer state are also on
disk (``durable_store.py``: segments + offset index, fsync policy) and a restarted broker
recovers them; InitProducerId + per-partition sequence numbers make a producer's retry after
a broker crash store its batch once.

``KafkaLiteCluster(n)`` runs n broker listeners (node ids 1..n) over one shared log store,
with partition leadership spread over the nodes (p -> node p % n).  Produce / Fetch /
ListOffsets sent to a node that does not lead the partition answer NOT_LEADER_FOR_PARTITION,
Metadata reports per-partition leaders, ``move_leader`` moves one partition and
``fail_node`` closes a broker and fails its partitions over to the next live node (the
controller's job), so clients have to route by leader and recover like against a real
cluster.  Replication is not simulated beyond that (one shared store): replicas = every
node, ISR = the live nodes, so the under-replicated / offline-partition series of the
reference's Kafka dashboard (deploy/grafana/Kafka.json:127-355) move when a node fails.

    python -m ccfd_demo_summit_amd.ingest.kafka_lite --port 9092 --partitions 8 [--nodes 3]
"""
from __future__ import annotations

import argparse
import asyncio
import collections
import itertools
import json
import os
import socket
import struct
import zlib
import sys
import threading
import time
from typing import Dict, List, Optional, Set, Tuple

import numpy as np

from .batch_store import BatchStore, InvalidBatch, OutOfOrderSequence
from .broker import BrokerError
from .kafka_wire import (ERR_CORRUPT, ERR_LEADER_NOT_AVAILABLE, ERR_NONE, ERR_NOT_COORDINATOR, ERR_NOT_LEADER,
                         ERR_OFFSET_OUT_OF_RANGE,
                         ERR_OUT_OF_ORDER_SEQUENCE, ERR_TOPIC_EXISTS, ERR_UNKNOWN_TOPIC, ERR_UNSUPPORTED_VERSION, SUPPORTED, Reader, Writer)

NODE_ID = 1
ERR_ILLEGAL_GENERATION, ERR_UNKNOWN_MEMBER, ERR_REBALANCE_IN_PROGRESS = 22, 25, 27
ERR_KAFKA_STORAGE_ERROR = 56


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


class ClusterState:
    """Node table + partition leadership (the controller's view) shared by the listeners."""

    def __init__(self, store: BatchStore):
        self.store = store
        # called (loop thread) once the durable store's writer failed: the broker process
        # exits non-zero so its supervisor / pod restarts it and it recovers from its segments
        # (a wedged broker would keep passing its TCP liveness probe)
        self.on_store_failure = None
        self.nodes: Dict[int, List] = {}                  # id -> [host, port, alive]
        self.leaders: Dict[Tuple[str, int], int] = {}
        self.groups: Dict[str, _Group] = {}
        self.mid = itertools.count(1)
        self.lock = threading.Lock()
        self.leader_moves = 0
        # long-polling fetches (Fetch max_wait / min_bytes): (topic, partition) -> futures woken
        # by the next append; the listeners share one event loop, so no cross-thread wake-up
        self.fetch_waiters: Dict[Tuple[str, int], set] = {}
        self.replica_waiters: Dict[Tuple[str, int], set] = {}   # followers' long polls: woken on append
        self.long_polls = 0
        # durable store (write-behind): produce answers waiting for their write ticket, in
        # ticket order; the last ticket the store's writer reported written
        self.produce_waiters: collections.deque = collections.deque()
        self.written = 0
        # replicated multi-process mode (ingest/kafka_replica.py): the controller's view
        # replaces the in-process node table and leadership
        self.replica = None

    def live(self) -> List[int]:
        if self.replica is not None:
            return self.replica.live_nodes()
        return sorted(n for n, v in self.nodes.items() if v[2])

    def address(self, node: int) -> Tuple[str, int]:
        if self.replica is not None:
            return self.replica.nodes[node]
        host, port, _ = self.nodes[node]
        return host, port

    def leader(self, topic: str, partition: int) -> int:
        if self.replica is not None:
            return self.replica.leader(topic, partition)
        with self.lock:
            key = (topic, partition)
            if key not in self.leaders:
                ids = sorted(self.nodes)
                cand = ids[partition % len(ids)]
                if not self.nodes[cand][2]:
                    live = self.live()
                    cand = live[partition % len(live)] if live else -1
                self.leaders[key] = cand
            return self.leaders[key]

    def move_leader(self, topic: str, partition: int, node: int) -> None:
        with self.lock:
            if node not in self.nodes or not self.nodes[node][2]:
                raise ValueError(f"node {node} is not a live broker")
            self.leaders[(topic, partition)] = node
            self.leader_moves += 1

    def fail_node(self, node: int) -> None:
        """Broker failure as the controller sees it: the node leaves the ISR and every
        partition it led moves to the next live node."""
        with self.lock:
            self.nodes[node][2] = False
            live = sorted(n for n, v in self.nodes.items() if v[2])
            for key, lead in list(self.leaders.items()):
                if lead == node:
                    self.leaders[key] = live[key[1] % len(live)] if live else -1
                    self.leader_moves += 1

    def under_replicated(self) -> int:
        if self.replica is not None:
            return self.replica.under_replicated()
        dead = len(self.nodes) - len(self.live())
        return self.partition_count() if dead else 0

    def offline(self) -> int:
        if self.replica is not None:
            return 0                            # reported by the controller alone (as in Kafka)
        return sum(1 for t, n in self.store.topics().items() for p in range(n) if self.leader(t, p) < 0)

    def partition_count(self) -> int:
        if self.replica is not None:
            return len(self.replica.hosted())
        return sum(self.store.topics().values())

    def leader_count(self) -> int:
        if self.replica is not None:
            return self.replica.led()
        return self.partition_count() - self.offline()


class _GcTimer:
    """Process-wide garbage-collection time per generation (one ``gc.callbacks`` hook)."""

    def __init__(self):
        import gc
        self.s = [0.0, 0.0, 0.0]
        self.n = [0, 0, 0]
        self._t0 = 0.0
        gc.callbacks.append(self._cb)

    def _cb(self, phase, info):
        if phase == "start":
            self._t0 = time.perf_counter()
        else:
            g = min(2, int(info.get("generation", 0)))
            self.s[g] += time.perf_counter() - self._t0
            self.n[g] += 1


_GC = None


def gc_timer() -> _GcTimer:
    global _GC
    if _GC is None:
        _GC = _GcTimer()
    return _GC


class ProcessResourceCollector:
    """The broker-process series of the reference's Kafka dashboard -- CPU, memory and GC
    (deploy/grafana/Kafka.json:416 ``process_cpu_seconds_total``, :499 ``jvm_memory_bytes_used``,
    :582 ``jvm_gc_collection_seconds_sum``), all labelled ``strimzi_io_kind="Kafka"`` as the
    Strimzi pod labels make them.  kafka-lite is not a JVM; the names are kept so the
    dashboard works unchanged, with these meanings:

    * ``process_cpu_seconds_total`` -- user + system CPU seconds of the broker process;
    * ``jvm_memory_bytes_used{area="heap"}`` -- bytes of record batches the log holds (the
      broker's data working set), ``{area="nonheap"}`` -- the rest of the resident set;
      ``jvm_memory_bytes_max{area="heap"}`` -- physical memory (the ceiling of the log);
    * ``jvm_gc_collection_seconds`` (summary, ``gc`` = Python collector generation) -- time
      the broker process spent in garbage collection, measured with ``gc.callbacks``.
    """

    def __init__(self, store, labels=("strimzi_io_kind",), values=("Kafka",)):
        self.store = store
        self.labels = list(labels)
        self.values = list(values)
        self.gc = gc_timer()

    def collect(self):
        import os
        from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily, SummaryMetricFamily
        t = os.times()
        c = CounterMetricFamily("process_cpu_seconds", "Broker process CPU seconds (user + system)",
                                labels=self.labels)
        c.add_metric(self.values, t.user + t.system)
        yield c
        rss = 0
        try:
            with open("/proc/self/statm") as f:
                rss = int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
        except (OSError, ValueError):
            pass
        heap = self.store.stored_bytes() if self.store is not None else 0
        used = GaugeMetricFamily("jvm_memory_bytes_used", "Broker memory in use (heap = log working set)",
                                 labels=["area"] + self.labels)
        used.add_metric(["heap"] + self.values, float(heap))
        used.add_metric(["nonheap"] + self.values, float(max(0, rss - heap)))
        yield used
        mx = GaugeMetricFamily("jvm_memory_bytes_max", "Broker memory ceiling (physical memory)",
                               labels=["area"] + self.labels)
        try:
            phys = os.sysconf("SC_PHYS_PAGES") * os.sysconf("SC_PAGE_SIZE")
        except (OSError, ValueError):
            phys = 0
        mx.add_metric(["heap"] + self.values, float(phys))
        yield mx
        g = SummaryMetricFamily("jvm_gc_collection_seconds", "Time spent in garbage collection",
                                labels=["gc"] + self.labels)
        for gen in range(3):
            g.add_metric([f"python-gen{gen}"] + self.values, count_value=self.gc.n[gen], sum_value=self.gc.s[gen])
        yield g


class BrokerMetrics:
    """The Strimzi/JMX-exporter series the reference's Kafka dashboard queries
    (deploy/grafana/Kafka.json:119-1093): topic message/byte rates, failed requests,
    partition/leader counts, under-replicated and offline partitions (from the cluster
    state: non-zero while a node is down / a partition has no live leader), and the
    broker-process CPU / memory / GC panels (ProcessResourceCollector)."""

    def __init__(self, cluster: ClusterState):
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
        self._seen: Set[str] = set()
        cl = cluster

        class _Gauges:
            def collect(self_):
                for name, v in (("kafka_server_replicamanager_partitioncount", cl.partition_count()),
                                ("kafka_server_replicamanager_leadercount", cl.leader_count()),
                                ("kafka_server_replicamanager_underreplicatedpartitions", cl.under_replicated()),
                                ("kafka_controller_kafkacontroller_offlinepartitionscount", cl.offline()),
                                ("kafka_controller_kafkacontroller_activebrokercount", len(cl.live()))):
                    g = GaugeMetricFamily(name, name, labels=["strimzi_io_kind"])
                    g.add_metric(["Kafka"], v)
                    yield g
        self.registry.register(_Gauges())
        self.registry.register(ProcessResourceCollector(cl.store))

    def topic(self, name: str) -> None:
        """Create every per-topic series at 0 the first time a topic is used, so the failed
        produce / fetch panels (Kafka.json:1017,1093) read 0 instead of "no data"."""
        if name in self._seen:
            return
        self._seen.add(name)
        for c in (self.messages_in, self.bytes_in, self.bytes_out, self.failed_produce, self.failed_fetch):
            c.labels(name, "Kafka")

    def expose(self) -> bytes:
        from prometheus_client import generate_latest
        return generate_latest(self.registry)


class _KafkaConn(asyncio.BufferedProtocol):
    """One client connection: requests are received straight into memory the broker owns
    (``recv_into``, no stream-reader copies) and handled from a memoryview of it.  A large
    request (>= BIG, e.g. a produce of a 4096-message RecordBatch) is received into its own
    buffer, which the log then keeps as is: produced record batches are never copied
    (batch_store.append_raw stores views); small requests share a compacting ring buffer,
    and a small produce request is copied out of it before handling.  Responses keep request
    order (a long-polling group request holds the ones behind it); reading pauses while the
    client is slow to take responses (write-side back-pressure)."""

    MAX_FRAME = 256 << 20
    BIG = 1 << 16

    def __init__(self, server: "KafkaLiteServer"):
        self.server = server
        self.buf = bytearray(1 << 18)              # ring for headers + small frames
        self.w = 0
        self.frame = None                          # dedicated buffer of the big frame in progress
        self.fw = 0
        self.transport = None
        self.outq = None                           # responses not yet written, in request order
        self.draining = False
        self.wsock = None                          # a dup of the connection's socket: gathered sends

    # asyncio.BufferedProtocol
    def connection_made(self, transport):
        import collections
        self.transport = transport
        self.outq = collections.deque()
        self.server._writers.add(self)
        ts = transport.get_extra_info("socket")
        if ts is not None and ts.family in (socket.AF_INET, socket.AF_INET6):
            try:
                self.wsock = socket.fromfd(ts.fileno(), ts.family, socket.SOCK_STREAM)
                self.wsock.setblocking(False)
            except OSError:
                self.wsock = None

    def connection_lost(self, exc):
        self.server._writers.discard(self)
        if self.wsock is not None:
            self.wsock.close()
            self.wsock = None

    def pause_writing(self):
        self.transport.pause_reading()

    def resume_writing(self):
        self.transport.resume_reading()

    def get_buffer(self, sizehint):
        if self.frame is not None:
            return memoryview(self.frame)[self.fw:]
        if len(self.buf) - self.w < 1 << 15:       # small frames only: bounded growth
            nb = bytearray(2 * len(self.buf))
            nb[:self.w] = self.buf[:self.w]
            self.buf = nb                          # the transport holds no view across calls
        return memoryview(self.buf)[self.w:]

    def buffer_updated(self, nbytes):
        if self.frame is not None:
            self.fw += nbytes
            if self.fw == len(self.frame):
                f, self.frame = self.frame, None
                self._handle(memoryview(f), owned=True)
            return
        self.w += nbytes
        r = 0
        mv = memoryview(self.buf)
        try:
            while self.w - r >= 4:
                size = struct.unpack_from(">i", self.buf, r)[0]
                if size < 0 or size > self.MAX_FRAME:
                    self.transport.close()
                    return
                have = self.w - r - 4
                if have < size:
                    if size >= self.BIG:           # receive the rest into its own buffer
                        # uninitialised (np.empty): bytearray(size) zero-filled every produce
                        # frame before the socket overwrote it
                        self.frame = np.empty(size, np.uint8)
                        self.frame[:have] = mv[r + 4:self.w]   # (a bytearray slice would copy twice)
                        self.fw = have
                        r = self.w
                    break
                msg = mv[r + 4:r + 4 + size]
                if size >= 2 and msg[0] == 0 and msg[1] == 0:     # produce (api 0): own copy
                    self._handle(memoryview(bytearray(msg)), owned=True)
                else:
                    self._handle(msg, owned=False)
                r += 4 + size
        finally:
            mv.release()
        if r:                                      # keep the partial frame at the front
            tail = self.w - r
            self.buf[:tail] = self.buf[r:self.w]
            self.w = tail

    def _handle(self, msg, owned: bool):
        # every request is handled as it arrives -- a produce is appended at once, in request
        # order -- and only its RESPONSE may wait (written to disk, acks=all behind the high
        # watermark, a long poll): a pipelining producer's next batches are in the log while
        # the first one's replicas catch up.  Responses leave in request order (outq).
        try:
            out = self.server._frame(msg)
        except Exception:                          # malformed request: drop the connection
            self.transport.close()
            return
        if isinstance(out, (bytes, bytearray, list)):
            if not self.outq:
                self._write(out)
            else:
                self.outq.append(out)              # behind a response still waited for
            return
        self.outq.append(asyncio.ensure_future(out))
        if not self.draining:
            self.draining = True
            asyncio.ensure_future(self._drain())

    def _write(self, out) -> None:
        if isinstance(out, list):
            # a fetch response: header + stored batches.  Python 3.10's writelines joins them
            # into one new bytes (a copy of every fetched byte -- the leader's largest single
            # cost at replicated TXB1 rates); with nothing queued in the transport, send them
            # gathered (sendmsg) straight from the stored buffers, and hand the transport
            # only what the socket did not take
            if self.wsock is not None and not self.transport.get_write_buffer_size() \
                    and not self.transport.is_closing():
                head = out[:512]                   # well under IOV_MAX
                try:
                    n = self.wsock.sendmsg(head)
                except (BlockingIOError, InterruptedError):
                    n = 0
                except OSError:                    # the transport sees the error on its own write
                    n = 0
                for i, b in enumerate(head):
                    ln = len(b)
                    if n >= ln:
                        n -= ln
                        continue
                    self.transport.write(memoryview(b)[n:] if n else b)
                    for b2 in head[i + 1:]:
                        self.transport.write(b2)
                    break
                for b in out[512:]:
                    self.transport.write(b)
                return
            self.transport.writelines(out)
        else:
            self.transport.write(out)

    async def _drain(self):
        try:
            while self.outq:
                item = self.outq[0]
                if isinstance(item, asyncio.Future):
                    try:
                        item = await item
                    except Exception:
                        self.transport.close()
                        return
                self.outq.popleft()
                if self.transport.is_closing():
                    return
                self._write(item)
        finally:
            self.draining = False

    def close(self):
        if self.transport is not None:
            self.transport.close()


class KafkaLiteServer:
    """One broker listener.  Alone it is a one-node cluster; ``KafkaLiteCluster`` builds
    several over a shared store / cluster state / metrics."""

    def __init__(self, host: str = "127.0.0.1", port: int = 9092, default_partitions: int = 1,
                 store: Optional[BatchStore] = None, auto_create: bool = True, node_id: int = NODE_ID,
                 cluster: Optional[ClusterState] = None, metrics: Optional[BrokerMetrics] = None,
                 advertise: Optional[str] = None):
        self.host = host
        self.port = port
        # host clients are told to connect to (Metadata); a 0.0.0.0 bind needs a real name
        self.advertise = advertise or host
        self.store = store or BatchStore(default_partitions=default_partitions)
        self.auto_create = auto_create
        self.node_id = node_id
        self.cluster = cluster or ClusterState(self.store)
        self.cluster.nodes.setdefault(node_id, [self.advertise, port, True])
        self._server: Optional[asyncio.base_events.Server] = None
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._thread: Optional[threading.Thread] = None
        self.metrics = metrics or BrokerMetrics(self.cluster)
        self.groups = self.cluster.groups
        self._mid = self.cluster.mid
        self._reaper: Optional[asyncio.Task] = None
        self._writers: Set["_KafkaConn"] = set()

    # ------------------------------------------------------------------ lifecycle
    async def start(self):
        loop = asyncio.get_running_loop()
        if hasattr(self.store, "on_written") and self.store.on_written is None:
            # the durable store's writer thread reports written tickets to this loop
            self.store.on_written = lambda t, tps: loop.call_soon_threadsafe(self._on_written, t, tps)
        self._server = await loop.create_server(lambda: _KafkaConn(self), self.host, self.port)
        self.port = self._server.sockets[0].getsockname()[1]
        self.cluster.nodes[self.node_id] = [self.advertise, self.port, True]
        self._reaper = asyncio.get_running_loop().create_task(self._reap_sessions())
        rep = self.cluster.replica
        if rep is not None:                     # replicated: join the controller's cluster
            rep.port, rep.server = self.port, self
            await rep.start()

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

    async def close_listener(self):
        """Stop accepting and drop every open connection (a broker crash, seen from clients)."""
        if self._server is not None:
            self._server.close()
        if self._reaper is not None:
            self._reaper.cancel()
        for w in list(self._writers):
            w.close()                               # _KafkaConn.close: transport close

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
    def _frame(self, msg) -> object:
        """One request frame (memoryview) -> the response frame (bytes), or an awaitable of it
        (the group APIs long-poll: JoinGroup, SyncGroup)."""
        r = Reader(msg)
        api, ver, corr = r.i16(), r.i16(), r.i32()
        r.string()                                  # client id
        body = self._dispatch(api, ver, r)
        if isinstance(body, list):                 # response parts, written without joining
            return [struct.pack(">ii", sum(len(b) for b in body) + 4, corr)] + body
        if isinstance(body, asyncio.Future):
            # a long-polled fetch or an acks=all produce: framed in a done callback, so the
            # response is written one loop iteration after the event that completes it (a
            # coroutine wrapper costs a task step per layer -- each a loop iteration, several
            # on the replication path of every acknowledged batch)
            out = asyncio.get_running_loop().create_future()

            def framed(f):
                if f.cancelled():
                    out.cancel()
                elif f.exception() is not None:
                    out.set_exception(f.exception())
                else:
                    b = f.result()
                    if isinstance(b, list):
                        out.set_result([struct.pack(">ii", sum(len(x) for x in b) + 4, corr)] + b)
                    else:
                        out.set_result(struct.pack(">ii", len(b) + 4, corr) + b)
            body.add_done_callback(framed)
            return out
        if not isinstance(body, (bytes, bytearray)):
            async def later():
                b = await body
                if isinstance(b, list):            # a long-polled fetch: parts, no join
                    return [struct.pack(">ii", sum(len(x) for x in b) + 4, corr)] + b
                out = struct.pack(">i", corr) + b
                return struct.pack(">i", len(out)) + out
            return later()
        return struct.pack(">ii", len(body) + 4, corr) + body

    def _on_written(self, ticket: int, tps) -> None:
        """Loop thread: answer the produces whose records are written (ticket -1: the log
        write failed -- their connections are dropped, the producers retry), and wake the
        long-polling fetches of the partitions whose high watermark moved."""
        cl = self.cluster
        if ticket < 0:
            while cl.produce_waiters:
                _t, f = cl.produce_waiters.popleft()
                if not f.done():
                    f.set_exception(BrokerError("kafka-lite log write failed"))
            if cl.on_store_failure is not None:
                cl.on_store_failure()
            return
        cl.written = max(cl.written, ticket)
        while cl.produce_waiters and cl.produce_waiters[0][0] <= cl.written:
            _t, f = cl.produce_waiters.popleft()
            if not f.done():
                f.set_result(None)
        for tp in tps:
            self._wake_fetches(tp)
        if cl.replica is not None:
            cl.replica.on_written(tps)          # the leader's LEO moved: maybe the HW too

    def _wake_fetches(self, tp, waiters=None) -> None:
        ws = (self.cluster.fetch_waiters if waiters is None else waiters).pop(tp, None)
        if ws:
            for f in ws:
                if not f.done():
                    f.set_result(None)

    def _produce_later(self, body: bytes, ticket: int) -> "asyncio.Future":
        """The produce response, once the durable store's writer has written ``ticket`` (a
        future filled in the done callback of the write, like the long-polled fetches)."""
        loop = asyncio.get_running_loop()
        out = loop.create_future()
        if not ticket or ticket <= self.cluster.written:
            out.set_result(body)
            return out
        fut = loop.create_future()
        self.cluster.produce_waiters.append((ticket, fut))

        def written(f) -> None:
            if f.cancelled():
                out.cancel()
            elif f.exception() is not None:
                out.set_exception(f.exception())
            else:
                out.set_result(body)
        fut.add_done_callback(written)
        return out

    def _topic(self, name: str) -> bool:
        if self.cluster.replica is not None:    # topics exist once the controller created them
            return name in self.cluster.replica.topics
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

    def _partition_error(self, topic: str, p: int) -> int:
        """ERR_NONE when this node leads an existing partition."""
        if topic not in self.store.topics() or not 0 <= p < self.store.partitions(topic):
            return ERR_UNKNOWN_TOPIC
        if self.cluster.leader(topic, p) != self.node_id:
            return ERR_NOT_LEADER
        return ERR_NONE

    # ------------------------------------------------------------------ APIs
    def _api_18(self, r: Reader) -> bytes:                  # ApiVersions v0
        return Writer().i16(ERR_NONE).array(sorted(SUPPORTED.items()), lambda w, kv: w.i16(kv[0]).i16(0).i16(kv[1])).build()

    def _api_3(self, r: Reader) -> bytes:                   # Metadata v1
        topics = r.array(lambda x: x.string())
        cl = self.cluster
        rep = cl.replica
        names = sorted(rep.topics if rep is not None else self.store.topics()) if topics is None else topics
        live = cl.live()
        w = Writer().array([(n,) + tuple(cl.address(n)) for n in live],
                           lambda w_, b: w_.i32(b[0]).string(b[1]).i32(b[2]).string(None))
        w.i32(live[0] if live else -1)                      # controller id
        replicas = sorted(cl.nodes)

        def topic(w_, name):
            if not self._topic(name):
                w_.i16(ERR_UNKNOWN_TOPIC).string(name).i8(0).array([], None)
                return
            n = rep.topics[name] if rep is not None else self.store.partitions(name)

            def part(w2, p):
                lead = cl.leader(name, p)
                reps = rep.replicas(name, p) if rep is not None else replicas
                isr = rep.isr(name, p) if rep is not None else live
                w2.i16(ERR_NONE if lead >= 0 else 5).i32(p).i32(lead)
                w2.array(reps, lambda w3, x: w3.i32(x)).array(isr, lambda w3, x: w3.i32(x))
            w_.i16(ERR_NONE).string(name).i8(0).array(range(n), part)
        w.array(names, topic)
        return w.build()

    def _api_19(self, r: Reader) -> bytes:                  # CreateTopics v0
        def req(x):
            name, n, _rf = x.string(), x.i32(), x.i16()
            x.array(lambda y: (y.i32(), y.array(lambda z: z.i32())))
            x.array(lambda y: (y.string(), y.string()))
            return name, n
        reqs = r.array(req)
        timeout_ms = r.i32()
        build = lambda res: Writer().array(res, lambda w, t: w.string(t[0]).i16(t[1])).build()
        rep = self.cluster.replica
        if rep is not None:                                 # created by the controller
            async def later():
                res = []
                # answered within the request's own timeout (the controller waits for every
                # broker to register): LEADER_NOT_AVAILABLE then, which the client retries
                wait_s = max(0.5, min(30.0, timeout_ms / 1000.0 - 1.0))
                for name, n in reqs:
                    if name in rep.topics:
                        res.append((name, ERR_TOPIC_EXISTS))
                        continue
                    try:
                        await rep.create_topic(name, max(1, n), wait_s=wait_s)
                        res.append((name, ERR_NONE))
                    except Exception:                       # noqa: BLE001 -- controller away / brokers not all up
                        res.append((name, ERR_LEADER_NOT_AVAILABLE))
                return build(res)
            return later()
        res = []
        for name, n in reqs:
            if name in self.store.topics():
                res.append((name, ERR_TOPIC_EXISTS))
            else:
                self.store.create_topic(name, max(1, n))
                res.append((name, ERR_NONE))
        return build(res)

    def _api_0(self, r: Reader) -> bytes:                   # Produce v3: batches stored verbatim
        r.string()
        acks, timeout_ms = r.i16(), r.i32()
        data = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.view_()))))
        resp = []
        ticket = 0
        rep = self.cluster.replica
        waits = []                                          # acks=all: (topic, p, log end, response entry)
        for topic, parts in data:
            pr = []
            self._topic(topic)
            self.metrics.topic(topic)
            for p, rb in parts:
                err = self._partition_error(topic, p)
                if err:
                    pr.append((p, err, -1))
                    self.metrics.failed_produce.labels(topic, "Kafka").inc()
                    continue
                try:
                    base, nrec, t = self.store.append_raw_nowait(topic, p, rb or b"")
                    pr.append([p, ERR_NONE, base])
                    if rep is not None and acks == -1:
                        waits.append((topic, p, self.store.log_end(topic, p), pr[-1]))
                    if t:
                        ticket = max(ticket, t)     # answered (and fetchable) once written
                    else:
                        self._wake_fetches((topic, p))
                    if rep is not None:
                        self._wake_fetches((topic, p), self.cluster.replica_waiters)
                        # the HW counts in-memory log ends: with no other in-sync replica
                        # (RF 1, or a shrunk ISR) it moves right here, not after the disk write
                        rep.on_written([(topic, p)])
                    self.metrics.messages_in.labels(topic, "Kafka").inc(nrec)
                    self.metrics.bytes_in.labels(topic, "Kafka").inc(len(rb or b""))
                except OutOfOrderSequence:
                    pr.append((p, ERR_OUT_OF_ORDER_SEQUENCE, -1))
                    self.metrics.failed_produce.labels(topic, "Kafka").inc()
                except InvalidBatch:
                    pr.append((p, ERR_CORRUPT, -1))
                    self.metrics.failed_produce.labels(topic, "Kafka").inc()
                except BrokerError:             # the durable log can no longer be written
                    pr.append((p, ERR_KAFKA_STORAGE_ERROR, -1))
                    self.metrics.failed_produce.labels(topic, "Kafka").inc()
            resp.append((topic, pr))
        build = lambda: Writer().array(resp, lambda w_, t: w_.string(t[0]).array(
            t[1], lambda w2, q: w2.i32(q[0]).i16(q[1]).i64(q[2]).i64(-1))).i32(0).build()
        if waits:
            return self._produce_replicated(build, ticket, waits, timeout_ms)
        body = build()
        if ticket and ticket > self.cluster.written:
            return self._produce_later(body, ticket)
        return body

    def _produce_replicated(self, build, ticket: int, waits, timeout_ms: int) -> "asyncio.Future":
        """acks=all on a replicated leader: answered once the partition's high watermark covers
        the batch (every in-sync replica has it).  Leadership lost meanwhile, or the timeout:
        NOT_LEADER, so the producer refreshes metadata and retries (its idempotent sequence
        makes a retry of a replicated batch a no-op)."""
        # acks=all: answered once the high watermark covers the batch (in the memory of every
        # in-sync replica, each writing it to disk right behind) -- not after this broker's own
        # write, which would put the leader's disk latency in front of every acknowledgement.
        # Callbacks, not a coroutine: the response is built in the iteration that moves the HW.
        rep = self.cluster.replica
        loop = asyncio.get_running_loop()
        out = loop.create_future()
        hw = [(rep.wait_hw(topic, p, end), topic, entry) for topic, p, end, entry in waits]

        def answer(timed_out: bool) -> None:
            if out.done():
                return
            if not timed_out and not all(f.done() for f, _t, _e in hw):
                return
            th.cancel()
            for f, topic, entry in hw:
                if not (f.done() and f.result()):
                    entry[1] = ERR_NOT_LEADER
                    self.metrics.failed_produce.labels(topic, "Kafka").inc()
            out.set_result(build())
        th = loop.call_later(max(0.1, timeout_ms / 1000.0), answer, True)
        for f, _t, _e in hw:
            if not f.done():
                f.add_done_callback(lambda _f: answer(False))
        answer(False)
        return out

    def _api_22(self, r: Reader) -> bytes:                  # InitProducerId v0 (idempotence only)
        r.string(); r.i32()
        if self.cluster.replica is not None:                # disjoint ids per broker
            from .kafka_replica import PID_STRIDE
            pid, epoch = self.store.init_producer_id(self.node_id, PID_STRIDE)
        else:
            pid, epoch = self.store.init_producer_id()
        return Writer().i32(0).i16(ERR_NONE).i64(pid).i16(epoch).build()

    def _api_1(self, r: Reader):                            # Fetch v4: stored batches, sliced
        replica_id = r.i32()
        max_wait_ms, min_bytes, max_bytes = r.i32(), r.i32(), r.i32()
        r.i8()
        reqs = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i64(), y.i32()))))
        parts, n, ok = self._fetch_parts(reqs, max_bytes, replica_id)
        if n == 0 and ok and max_wait_ms > 0 and min_bytes > 0:
            # Kafka's long poll: hold the request until a requested partition gets data or
            # max_wait passes.  Without it every idle consumer thread re-fetched every few
            # hundred microseconds, thousands of empty fetches a second through this event loop
            return self._fetch_later(reqs, max_bytes, max_wait_ms, replica_id)
        return parts

    def _fetch_later(self, reqs, max_bytes: int, max_wait_ms: int, replica_id: int = -1) -> "asyncio.Future":
        """The long poll: a future of the response parts, filled in the callback of the wake-up
        (data / a high watermark move on a requested partition) or of max_wait."""
        loop = asyncio.get_running_loop()
        wake = loop.create_future()
        out = loop.create_future()
        tps = [(t, p) for t, ps in reqs for p, _o, _m in ps]
        waiters = self.cluster.fetch_waiters if replica_id < 0 else self.cluster.replica_waiters
        for tp in tps:
            waiters.setdefault(tp, set()).add(wake)
        self.cluster.long_polls += 1
        th = loop.call_later(max_wait_ms / 1000.0, lambda: wake.done() or wake.set_result(None))

        def finish(_f) -> None:
            th.cancel()
            for tp in tps:
                ws = waiters.get(tp)
                if ws is not None:
                    ws.discard(wake)
                    if not ws:
                        waiters.pop(tp, None)
            if out.done():
                return
            try:
                out.set_result(self._fetch_parts(reqs, max_bytes, replica_id)[0])
            except Exception as e:                      # noqa: BLE001 -- the connection is closed
                out.set_exception(e)
        wake.add_done_callback(finish)
        return out

    def _fetch_parts(self, reqs, max_bytes: int, replica_id: int = -1):
        """(response parts, record bytes in them, no partition errored).  Replicated mode: a
        follower's fetch (``replica_id`` >= 0) reports its log end to the leader and reads up to
        the leader's written end; a consumer reads up to the high watermark."""
        resp = []
        ok = True
        budget = max_bytes
        rep = self.cluster.replica
        for topic, parts in reqs:
            pr = []
            self.metrics.topic(topic)
            for p, off, pmax in parts:
                err = self._partition_error(topic, p)
                if err:
                    pr.append((p, err, -1, None))
                    self.metrics.failed_fetch.labels(topic, "Kafka").inc()
                    ok = False
                    continue
                hw = self.store.end_offset(topic, p)
                upto = None
                limit = hw
                unwritten = False
                if rep is not None:
                    if replica_id >= 0:
                        rep.on_replica_fetch(replica_id, topic, p, off)
                        # followers copy the log as appended, written or not: replication runs
                        # beside the leader's own write instead of after it
                        unwritten = True
                        limit = self.store.log_end(topic, p)
                    else:
                        # consumers see data below the HW; an offset between the HW and the log
                        # end is valid (a new leader's HW catches up) -- an empty answer, not
                        # OFFSET_OUT_OF_RANGE
                        upto = rep.high_watermark(topic, p)
                        unwritten = True                  # below the HW = on every in-sync replica
                        # a consumer may have read (from the old leader) up to a HW that this new
                        # leader holds in memory but has not written yet: in range, not an error
                        limit = self.store.log_end(topic, p)
                    hw = rep.high_watermark(topic, p)
                if off < self.store.begin_offset(topic, p) or off > limit:
                    pr.append((p, ERR_OFFSET_OUT_OF_RANGE, hw, None))
                    self.metrics.failed_fetch.labels(topic, "Kafka").inc()
                    ok = False
                    continue
                rb = (self.store.fetch_parts(topic, p, off, max(1, min(pmax, budget)), upto, unwritten)
                      if budget > 0 else [])
                n = sum(len(b) for b in rb)
                budget -= n
                pr.append((p, ERR_NONE, hw, rb))
                if n:
                    self.metrics.bytes_out.labels(topic, "Kafka").inc(n)
            resp.append((topic, pr))

        def records(w2, q):
            w2.i32(q[0]).i16(q[1]).i64(q[2]).i64(q[2]).array([], None)
            if q[3] is None:
                w2.i32(-1)
                return
            w2.i32(sum(len(b) for b in q[3]))
            for b in q[3]:                         # the stored batches, by reference
                w2.raw(b)
        w = Writer().i32(0)
        w.array(resp, lambda w_, t: w_.string(t[0]).array(t[1], records))
        return w.parts, max_bytes - budget, ok    # parts: written with one gather (_KafkaConn)

    def _api_2(self, r: Reader) -> bytes:                   # ListOffsets v1
        r.i32()
        reqs = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i64()))))
        resp = []
        for topic, parts in reqs:
            pr = []
            for p, ts in parts:
                self._topic(topic)
                err = self._partition_error(topic, p)
                if err:
                    pr.append((p, err, -1))
                    continue
                if ts == -2:
                    off = self.store.begin_offset(topic, p)
                elif self.cluster.replica is not None:     # consumers see up to the HW
                    off = self.cluster.replica.high_watermark(topic, p)
                else:
                    off = self.store.end_offset(topic, p)
                pr.append((p, ERR_NONE, off))
            resp.append((topic, pr))
        return Writer().array(resp, lambda w_, t: w_.string(t[0]).array(
            t[1], lambda w2, q: w2.i32(q[0]).i16(q[1]).i64(-1).i64(q[2]))).build()

    def _api_10(self, r: Reader) -> bytes:                  # FindCoordinator v0
        group = r.string() or ""
        live = self.cluster.live()
        # one process: group state is shared, any node works; replicated: the group's hash picks
        # a live broker (offsets are kept by the controller, so any broker can coordinate, and a
        # new coordinator has them) -- every group's commits on the lowest broker made it the
        # busiest, and its event loop the produce -> scored tail
        if self.cluster.replica is not None and live:
            node = live[zlib.crc32(group.encode()) % len(live)]
        else:
            node = live[0] if live else self.node_id
        if self.cluster.replica is not None and node not in self.cluster.replica.nodes:
            return Writer().i16(ERR_NOT_COORDINATOR).i32(-1).string("").i32(-1).build()
        host, port = self.cluster.address(node)
        return Writer().i16(ERR_NONE).i32(node).string(host).i32(port).build()

    def _api_8(self, r: Reader) -> bytes:                   # OffsetCommit v2
        group = r.string(); r.i32(); r.string(); r.i64()
        reqs = r.array(lambda x: (x.string(), x.array(lambda y: (y.i32(), y.i64(), y.string()))))
        build = lambda resp: Writer().array(resp, lambda w_, t: w_.string(t[0]).array(
            t[1], lambda w2, q: w2.i32(q[0]).i16(q[1]))).build()
        rep = self.cluster.replica
        if rep is not None:                                 # durable at the controller first
            async def later():
                err = ERR_NONE
                try:
                    await rep.commit_offsets(group, [(t, p, off) for t, parts in reqs for p, off, _m in parts])
                except Exception:                           # noqa: BLE001 -- controller away
                    err = ERR_NOT_COORDINATOR
                for t, parts in reqs:
                    for p, off, _m in parts:
                        if err == ERR_NONE:
                            self.store.commit(group, t, p, off)      # this coordinator's cache
                return build([(t, [(p, err) for p, _o, _m in parts]) for t, parts in reqs])
            return later()
        resp = []
        for topic, parts in reqs:
            for p, off, _m in parts:
                self.store.commit(group, topic, p, off)
            resp.append((topic, [(p, ERR_NONE) for p, _o, _m in parts]))
        return build(resp)

    def _api_9(self, r: Reader) -> bytes:                   # OffsetFetch v1
        group = r.string()
        reqs = r.array(lambda x: (x.string(), x.array(lambda y: y.i32())))
        build = lambda resp, err=ERR_NONE: Writer().array(resp, lambda w_, t: w_.string(t[0]).array(
            t[1], lambda w2, q: w2.i32(q[0]).i64(q[1]).string(None).i16(err))).build()
        rep = self.cluster.replica
        if rep is not None:
            async def later():
                tps = [(t, p) for t, parts in reqs for p in parts]
                try:
                    offs = await rep.fetch_offsets(group, tps)
                except Exception:                           # noqa: BLE001 -- controller away
                    return build([(t, [(p, -1) for p in parts]) for t, parts in reqs], ERR_NOT_COORDINATOR)
                got = dict(zip(tps, offs))
                return build([(t, [(p, int(got[(t, p)])) for p in parts]) for t, parts in reqs])
            return later()
        resp = []
        for topic, parts in reqs:
            pr = []
            for p in parts:
                c = self.store.committed(group, topic, p)
                pr.append((p, -1 if c is None else c))
            resp.append((topic, pr))
        return build(resp)

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


class KafkaLiteCluster:
    """``n`` broker listeners (node ids 1..n, ports ``base_port + i`` or ephemeral) on one
    event loop over a shared store: leadership p -> node (p % n) + 1 until moved."""

    def __init__(self, n: int = 3, host: str = "127.0.0.1", base_port: int = 0, default_partitions: int = 1,
                 auto_create: bool = True, retention_batches: Optional[int] = None,
                 advertise: Optional[str] = None, data_dir: Optional[str] = None, fsync: str = "interval",
                 store: Optional[BatchStore] = None):
        """``data_dir``: keep the logs, committed offsets and producer state on disk
        (ingest/durable_store.py) and recover them on start; None = in memory only."""
        if store is None and data_dir:
            from .durable_store import DurableBatchStore
            store = DurableBatchStore(data_dir, default_partitions=default_partitions,
                                      retention_batches=retention_batches, fsync=fsync)
        self.store = store or BatchStore(default_partitions=default_partitions, retention_batches=retention_batches)
        self.state = ClusterState(self.store)
        self.metrics = BrokerMetrics(self.state)
        self.nodes = [KafkaLiteServer(host, base_port + i if base_port else 0, store=self.store,
                                      auto_create=auto_create, node_id=i + 1, cluster=self.state,
                                      metrics=self.metrics, advertise=advertise) for i in range(n)]
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._thread: Optional[threading.Thread] = None

    async def start(self):
        for s in self.nodes:
            await s.start()

    def start_in_thread(self) -> "KafkaLiteCluster":
        ready = threading.Event()

        def run():
            self._loop = asyncio.new_event_loop()
            for s in self.nodes:
                s._loop = self._loop
            self._loop.run_until_complete(self.start())
            ready.set()
            self._loop.run_forever()
        self._thread = threading.Thread(target=run, daemon=True, name="kafka-lite-cluster")
        self._thread.start()
        ready.wait(10)
        return self

    @property
    def bootstrap(self) -> str:
        return self.nodes[0].bootstrap

    @property
    def bootstrap_all(self) -> str:
        return ",".join(s.bootstrap for s in self.nodes)

    def leader(self, topic: str, partition: int) -> int:
        return self.state.leader(topic, partition)

    def move_leader(self, topic: str, partition: int, node: int) -> None:
        self.state.move_leader(topic, partition, node)

    def fail_node(self, node: int) -> None:
        """Close broker ``node`` (listener + open connections) and fail its partitions over."""
        self.state.fail_node(node)
        srv = self.nodes[node - 1]
        if self._loop is not None:
            asyncio.run_coroutine_threadsafe(srv.close_listener(), self._loop).result(5)

    def stop(self):
        if self._loop is not None:
            async def _shutdown():
                for s in self.nodes:
                    if s._server is not None:
                        s._server.close()
                me = asyncio.current_task()
                tasks = [t for t in asyncio.all_tasks() if t is not me]
                for t in tasks:
                    t.cancel()
                await asyncio.gather(*tasks, return_exceptions=True)
                self._loop.stop()
            asyncio.run_coroutine_threadsafe(_shutdown(), self._loop)
            self._thread.join(5)
        if hasattr(self.store, "close"):
            self.store.close()


class ReplicatedBroker:
    """One broker PROCESS of a replicated kafka-lite cluster (ingest/kafka_replica.py): its own
    durable log (cut to its checkpointed high watermark on start), one listener, a replica
    manager that heartbeats the controller, follows the partitions other brokers lead and
    serves the ones it leads."""

    def __init__(self, node_id: int, controller: str, host: str = "127.0.0.1", port: int = 0,
                 data_dir: Optional[str] = None, fsync: str = "interval", advertise: Optional[str] = None,
                 retention_batches: Optional[int] = None, hb_s: float = 0.1, replica_lag_s: float = 5.0):
        from .kafka_replica import ReplicaManager, load_checkpoint
        if data_dir:
            from .durable_store import DurableBatchStore
            self.store = DurableBatchStore(data_dir, retention_batches=retention_batches, fsync=fsync,
                                           truncate_to=load_checkpoint(data_dir))
        else:
            self.store = BatchStore(retention_batches=retention_batches)
        self.state = ClusterState(self.store)
        self.server = KafkaLiteServer(host, port, store=self.store, auto_create=False, node_id=node_id,
                                      cluster=self.state, advertise=advertise)
        self.state.replica = ReplicaManager(node_id, advertise or host, port, controller, self.store,
                                            server=self.server, hb_s=hb_s, replica_lag_s=replica_lag_s,
                                            data_dir=data_dir)
        self.metrics = self.server.metrics

    @property
    def replica(self):
        return self.state.replica

    @property
    def bootstrap(self) -> str:
        return self.server.bootstrap

    async def start(self):
        await self.server.start()

    def start_in_thread(self) -> "ReplicatedBroker":
        self.server.start_in_thread()
        return self

    def stop(self):
        if self.server._loop is not None:
            asyncio.run_coroutine_threadsafe(self.state.replica.close(), self.server._loop).result(5)
        self.server.stop()
        if hasattr(self.store, "close"):
            self.store.close()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=9092, help="first node's port (node i listens on port + i)")
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--nodes", type=int, default=1, help="broker listeners (leadership spread over them)")
    ap.add_argument("--metrics-port", type=int, default=9404, help="Prometheus /metrics (0 = off)")
    ap.add_argument("--advertise", default=None, help="host name put in Metadata (default: --host)")
    ap.add_argument("--retention-batches", type=int, default=0,
                    help="record batches kept per partition (0 = unbounded)")
    ap.add_argument("--data-dir", default=None,
                    help="durable logs: segments + offset index + committed offsets + producer state, "
                         "recovered on start (ingest/durable_store.py); default: memory only")
    ap.add_argument("--fsync", default="interval", choices=["always", "interval", "never"],
                    help="--data-dir flush policy: before every answer, every second in the background, "
                         "or left to the OS (a killed broker process loses nothing in any mode)")
    ap.add_argument("--node-id", type=int, default=0,
                    help="replicated mode: this broker's node id (one broker per process; needs --controller)")
    ap.add_argument("--controller", default=None,
                    help="replicated mode: the kafka-lite controller's URL (ingest/kafka_controller.py)")
    a = ap.parse_args(argv)
    if a.controller:
        return _main_replicated(a)
    # the durable store's writer thread hands every written ticket back to this event loop,
    # and takes the GIL back after each write: at CPython's 5 ms switch interval a busy loop
    # kept it waiting for the GIL, so acknowledgements and fetch visibility lagged the writes
    # (profiles/r4/broker_ab/write_behind/)
    sys.setswitchinterval(0.0005)
    from .kafka_wire import warm_native
    print(f"[kafka-lite] native codecs loaded in {warm_native():.2f} s", flush=True)
    cl = KafkaLiteCluster(a.nodes, a.host, a.port, a.partitions, advertise=a.advertise,
                          retention_batches=a.retention_batches or None, data_dir=a.data_dir, fsync=a.fsync)
    if a.data_dir:
        print(f"[kafka-lite] recovered from {a.data_dir}: {json.dumps(cl.store.recovered)}", flush=True)

    def store_failed():
        # the durable log writer died (disk full, EIO): answer nothing more, exit non-zero so
        # the supervisor / pod restarts the broker, which recovers from its segments
        print(f"[kafka-lite] FATAL: log write failed ({getattr(cl.store, '_werr', None)!r}); exiting",
              file=sys.stderr, flush=True)
        asyncio.get_running_loop().call_later(0.2, os._exit, 75)
    cl.state.on_store_failure = store_failed

    async def run():
        await cl.start()
        if a.metrics_port:
            from aiohttp import web
            app = web.Application()
            app.router.add_get("/metrics", lambda _r: web.Response(
                body=cl.metrics.expose(), headers={"Content-Type": "text/plain; version=0.0.4"}))
            runner = web.AppRunner(app)
            await runner.setup()
            await web.TCPSite(runner, a.host, a.metrics_port).start()
        from ..utils.gcpolicy import tune_for_service
        print(f"[kafka-lite] {a.nodes} node(s) listening on {cl.bootstrap_all}; gc: {tune_for_service()}",
              flush=True)
        await asyncio.Event().wait()
    asyncio.run(run())


def _main_replicated(a):
    """One broker process of a replicated cluster (--node-id N --controller URL)."""
    if a.node_id <= 0:
        raise SystemExit("kafka-lite: replicated mode needs --node-id >= 1")
    sys.setswitchinterval(0.0005)
    from ..utils.pyprof import install_from_env
    install_from_env(f"kafka-lite-node{a.node_id}")          # CCFD_PYPROF=<dir>: cProfile of this broker
    from .kafka_wire import warm_native
    print(f"[kafka-lite] native codecs loaded in {warm_native():.2f} s", flush=True)
    br = ReplicatedBroker(a.node_id, a.controller, a.host, a.port, data_dir=a.data_dir, fsync=a.fsync,
                          advertise=a.advertise, retention_batches=a.retention_batches or None)
    if a.data_dir:
        print(f"[kafka-lite] node {a.node_id} recovered from {a.data_dir}: {json.dumps(br.store.recovered)} "
              f"(cut to the checkpointed HW: {getattr(br.store, 'truncated_batches', 0)} batches)", flush=True)

    def store_failed():
        print(f"[kafka-lite] FATAL: log write failed ({getattr(br.store, '_werr', None)!r}); exiting",
              file=sys.stderr, flush=True)
        asyncio.get_running_loop().call_later(0.2, os._exit, 75)
    br.state.on_store_failure = store_failed

    async def run():
        await br.start()
        if a.metrics_port:
            from aiohttp import web
            app = web.Application()
            app.router.add_get("/metrics", lambda _r: web.Response(
                body=br.metrics.expose(), headers={"Content-Type": "text/plain; version=0.0.4"}))
            runner = web.AppRunner(app)
            await runner.setup()
            await web.TCPSite(runner, a.host, a.metrics_port).start()
        from ..utils.gcpolicy import tune_for_service
        print(f"[kafka-lite] node {a.node_id} listening on {br.bootstrap} (controller {a.controller}); "
              f"gc: {tune_for_service()}", flush=True)
        await asyncio.Event().wait()
    asyncio.run(run())


if __name__ == "__main__":
    main()
