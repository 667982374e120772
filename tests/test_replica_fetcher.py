"""The follower's fetcher thread (ingest/kafka_replica.py ``_fetch_thread``, the default since
round 6) appends a fetched response only under the leader epoch it fetched with.  Metadata
applied while a fetch is in flight (a new leader epoch) makes it drop that response: no
append from a deposed leader can land after the truncation that starts following the new
one.  A fake leader holds the first fetch until the test has (or has not) moved the epoch."""
import socket
import struct
import threading
import time

from ccfd_demo_summit_amd.ingest.batch_store import BatchStore
from ccfd_demo_summit_amd.ingest.kafka_controller import tp_key
from ccfd_demo_summit_amd.ingest.kafka_replica import ReplicaManager
from ccfd_demo_summit_amd.ingest.kafka_wire import Reader, Writer, encode_record_batch

T = "odh-demo"


class FakeLeader:
    """Answers replica fetches for partition 0 of T: the first with one record batch (after
    ``gate`` is set), every later one with no records."""

    def __init__(self):
        self.srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(4)
        self.srv.settimeout(0.2)
        self.port = self.srv.getsockname()[1]
        self.got_request = threading.Event()
        self.gate = threading.Event()
        self.stop = threading.Event()
        self.batch = encode_record_batch([b"fraud-case-1"], base_offset=0)
        self.answered = 0
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    def _recv(self, c, n):
        b = b""
        while len(b) < n:
            k = c.recv(n - len(b))
            if not k:
                raise ConnectionError
            b += k
        return b

    def _serve(self, c):
        c.settimeout(0.2)
        while not self.stop.is_set():
            try:
                size = struct.unpack(">i", self._recv(c, 4))[0]
            except socket.timeout:
                continue
            r = Reader(self._recv(c, size))
            r.i16(), r.i16()
            corr = r.i32()
            first = self.answered == 0
            if first:
                self.got_request.set()
                self.gate.wait(5)
            recs = self.batch if first else None
            hw = 1
            body = (Writer().i32(corr).i32(0)
                    .array([T], lambda w, t: w.string(t).array([0], lambda w2, p: w2.i32(p).i16(0).i64(hw).i64(hw)
                                                                .array([], None).bytes_(recs))).build())
            c.sendall(struct.pack(">i", len(body)) + body)
            self.answered += 1

    def _run(self):
        while not self.stop.is_set():
            try:
                c, _ = self.srv.accept()
            except socket.timeout:
                continue
            try:
                self._serve(c)
            except (ConnectionError, OSError):
                pass
            finally:
                c.close()

    def close(self):
        self.stop.set()
        self.gate.set()
        self.th.join(5)
        self.srv.close()


def _meta(port, epoch, meta_epoch):
    return {"meta_epoch": meta_epoch, "nodes": {"1": ["127.0.0.1", port]}, "topics": {T: 1},
            "parts": {tp_key(T, 0): {"leader": 1, "epoch": epoch, "replicas": [0, 1], "isr": [0, 1]}}}


def _follower(leader: FakeLeader):
    store = BatchStore()
    rm = ReplicaManager(0, "127.0.0.1", 0, "http://127.0.0.1:1", store)
    rm.report_s = 0
    with rm._follow_lock:                       # the metadata a follower of node 1 starts with
        rm.meta_epoch = 1
        rm.nodes = {1: ("127.0.0.1", leader.port)}
        store.create_topic(T, 1)
        rm.topics = {T: 1}
        rm.parts = {(T, 0): {"leader": 1, "epoch": 5, "replicas": [0, 1], "isr": [0, 1]}}
    th = threading.Thread(target=rm._fetch_thread, args=(1,), daemon=True)
    rm._fetchers[1] = th                        # _apply's reconcile keeps this fetcher
    th.start()
    return store, rm, th


def _wait(pred, timeout=5.0):
    t0 = time.monotonic()
    while not pred():
        assert time.monotonic() - t0 < timeout
        time.sleep(0.005)


def test_fetch_under_the_same_epoch_is_appended():
    leader = FakeLeader()
    store, rm, th = _follower(leader)
    try:
        assert leader.got_request.wait(5)
        leader.gate.set()
        _wait(lambda: rm.replica_fetches >= 1)
        assert store.log_end(T, 0) == 1
        assert rm.hw[(T, 0)] == 1
    finally:
        rm._stopping = True
        leader.close()
        th.join(6)


def test_response_of_a_deposed_epoch_is_dropped():
    leader = FakeLeader()
    store, rm, th = _follower(leader)
    try:
        assert leader.got_request.wait(5)        # the epoch-5 fetch is in flight
        rm._apply(_meta(leader.port, epoch=6, meta_epoch=2))
        leader.gate.set()
        _wait(lambda: rm.replica_fetches >= 1)
        assert store.log_end(T, 0) == 0          # fetched under epoch 5: never appended
        _wait(lambda: leader.answered >= 2)      # the fetcher goes on under epoch 6
        assert store.log_end(T, 0) == 0
    finally:
        rm._stopping = True
        leader.close()
        th.join(6)
