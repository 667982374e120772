"""Durable kafka-lite: segments + offset index + committed offsets +
idempotent-producer state survive a broker crash; torn tails are truncated, a lost index is
rebuilt, retention deletes whole segments; a SIGKILLed kafka-lite process restarted from its
data directory serves every acknowledged record exactly once (producers retry; their
sequence numbers make the retried batches land once)."""
import os
import signal
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np
import pytest

from ccfd_demo_summit_amd.ingest.batch_store import OutOfOrderSequence
from ccfd_demo_summit_amd.ingest.durable_store import DurableBatchStore
from ccfd_demo_summit_amd.ingest.kafka_wire import decode_record_batches, encode_record_batch

ROOT = Path(__file__).resolve().parents[1]


def _batch(vals, pid=-1, seq=0):
    import struct
    from ccfd_demo_summit_amd.ingest.kafka_wire import crc32c
    b = bytearray(encode_record_batch([v if isinstance(v, bytes) else v.encode() for v in vals]))
    if pid >= 0:
        struct.pack_into(">qhi", b, 43, pid, 0, seq)
        struct.pack_into(">I", b, 17, crc32c(memoryview(b)[21:]))
    return bytes(b)


def _values(store, topic, p):
    recs = decode_record_batches(store.fetch_raw(topic, p, 0, 1 << 30), topic, p, verify_crc=True)
    return [(r.offset, r.value) for r in recs]


def test_logs_offsets_and_producers_survive_a_crash(tmp_path):
    d = str(tmp_path / "kl")
    s = DurableBatchStore(d, default_partitions=2, fsync="never")
    s.create_topic("odh-demo", 2)
    for k in range(20):
        s.append_raw("odh-demo", k % 2, _batch([f"tx{k}-{i}" for i in range(5)], pid=7, seq=(k // 2) * 5))
    s.commit("g", "odh-demo", 0, 30)
    s.commit("g", "odh-demo", 1, 25)
    before = {p: _values(s, "odh-demo", p) for p in range(2)}
    # crash: nothing closed or fsync'd -- the writes are in the page cache
    s2 = DurableBatchStore(d, fsync="never")
    assert s2.topics() == {"odh-demo": 2}
    for p in range(2):
        assert _values(s2, "odh-demo", p) == before[p]
        assert s2.end_offset("odh-demo", p) == 50
    assert s2.committed("g", "odh-demo", 0) == 30 and s2.committed("g", "odh-demo", 1) == 25
    assert s2.recovered["batches"] == 20 and s2.recovered["records"] == 100
    # the producer's last sequence was recovered: a retry of its last batch is a duplicate,
    # a gap is refused, the next batch appends
    base, n = s2.append_raw("odh-demo", 0, _batch([f"tx18-{i}" for i in range(5)], pid=7, seq=45))
    assert (base, n) == (45, 0) and s2.end_offset("odh-demo", 0) == 50
    with pytest.raises(OutOfOrderSequence):
        s2.append_raw("odh-demo", 0, _batch(["x"], pid=7, seq=77))
    assert s2.append_raw("odh-demo", 0, _batch(["next"], pid=7, seq=50)) == (50, 1)
    s2.close()
    s3 = DurableBatchStore(d, fsync="never")
    assert s3.end_offset("odh-demo", 0) == 51 and _values(s3, "odh-demo", 0)[-1] == (50, b"next")
    s3.close()


def test_torn_tail_is_truncated_and_index_rebuilt(tmp_path):
    d = str(tmp_path / "kl")
    s = DurableBatchStore(d, default_partitions=1, fsync="always")
    s.create_topic("t", 1)
    for k in range(4):
        s.append_raw("t", 0, _batch([f"v{k}"] * 3))
    s.close()
    seg = sorted((Path(d) / "t-0").glob("*.log"))[-1]
    good = seg.stat().st_size
    with open(seg, "ab") as f:                     # a crash in the middle of the 5th batch
        f.write(_batch(["torn"] * 3)[:40])
    (seg.with_suffix(".idx")).write_bytes(b"")     # and a lost index
    s2 = DurableBatchStore(d, fsync="never")
    assert s2.recovered["torn_tails_truncated"] == 1
    assert seg.stat().st_size == good and s2.end_offset("t", 0) == 12
    assert len(seg.with_suffix(".idx").read_bytes()) == 4 * 16
    assert [v for _o, v in _values(s2, "t", 0)] == [f"v{k}".encode() for k in range(4) for _ in range(3)]
    assert s2.append_raw("t", 0, _batch(["after"])) == (12, 1)
    s2.close()


def test_retention_deletes_whole_segments(tmp_path):
    d = str(tmp_path / "kl")
    s = DurableBatchStore(d, default_partitions=1, retention_batches=10, fsync="never", segment_bytes=2000)
    s.create_topic("t", 1)
    for k in range(60):
        s.append_raw("t", 0, _batch([f"value-{k:04d}" * 4] * 4))
    segs = sorted((Path(d) / "t-0").glob("*.log"))
    first_base = int(segs[0].stem)
    assert s.begin_offset("t", 0) == 50 * 4 and first_base <= 200
    assert len(segs) < 20                           # old segments were deleted
    s2 = DurableBatchStore(d, retention_batches=10, fsync="never", segment_bytes=2000)
    assert s2.begin_offset("t", 0) == 200 and s2.end_offset("t", 0) == 240
    s.close()
    s2.close()


@pytest.mark.parametrize("policy", ["interval", "never", "always"])
def test_rolled_segments_are_closed_without_leaking_fds(tmp_path, policy):
    """Segment rolls never fsync on the produce path in "interval" mode (the flusher closes
    the retired files); no policy leaks file descriptors across many rolls, and every record
    is read back after a restart."""
    d = str(tmp_path / "kl")
    fds0 = len(os.listdir("/proc/self/fd"))
    s = DurableBatchStore(d, default_partitions=1, fsync=policy, fsync_interval_s=0.05, segment_bytes=1500)
    s.create_topic("t", 1)
    for k in range(200):
        s.append_raw("t", 0, _batch([f"v{k:04d}" * 8] * 4))
    if policy == "interval":
        t0 = time.time()                       # (the flusher may hold the swapped-out list)
        while not (s._closing or s.fsyncs) and time.time() - t0 < 2:
            time.sleep(0.01)
        assert s._closing or s.fsyncs          # handed to the flusher, not fsync'd inline
        time.sleep(0.3)
        assert not s._closing                  # ... which fsync'd and closed them
    assert len(os.listdir("/proc/self/fd")) - fds0 < 12     # only the active files stay open
    s.close()
    s2 = DurableBatchStore(d, fsync="never")
    vals = _values(s2, "t", 0)
    assert [o for o, _ in vals] == list(range(800))
    s2.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _start(port, d):
    return subprocess.Popen([sys.executable, "-m", "ccfd_demo_summit_amd.ingest.kafka_lite", "--host", "127.0.0.1",
                             "--port", str(port), "--partitions", "2", "--metrics-port", "0", "--data-dir", d],
                            cwd=str(ROOT), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                            env=dict(os.environ, PYTHONPATH=str(ROOT)))


def _wait(port, t=60):
    t0 = time.time()
    while time.time() - t0 < t:
        try:
            socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
            return
        except OSError:
            time.sleep(0.1)
    raise TimeoutError


def test_sigkilled_broker_restarts_from_disk_exactly_once(tmp_path):
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    port = _free_port()
    d = str(tmp_path / "data")
    proc = _start(port, d)
    try:
        _wait(port)
        prod = KafkaBroker(f"127.0.0.1:{port}", idempotent=True, connect_wait_s=30)
        prod.create_topic("odh-demo", 2)
        sent = 0
        killed = restarted = False
        t0 = time.time()
        import threading

        def chaos():
            nonlocal proc, killed, restarted
            time.sleep(0.4)
            proc.send_signal(signal.SIGKILL)        # a crashed broker pod
            proc.wait(10)
            killed = True
            time.sleep(1.0)
            proc = _start(port, d)                  # restartPolicy: Always
            restarted = True
        th = threading.Thread(target=chaos)
        th.start()
        while sent < 400 * 50:
            k = sent // 50
            prod.produce_batch("odh-demo", k % 2, [f"{sent + i}".encode() for i in range(50)])
            sent += 50
            if killed and not restarted:
                time.sleep(0.01)
        th.join()
        assert killed and restarted and time.time() - t0 < 120
        prod.commit("g", "odh-demo", 0, 100) if hasattr(prod, "commit") else None
        cons = KafkaBroker(f"127.0.0.1:{port}", connect_wait_s=30)
        got = []
        for p in range(2):
            off = 0
            end = cons.end_offset("odh-demo", p)
            while off < end:
                recs = cons.fetch("odh-demo", p, off, 10_000)
                got += [int(r.value) for r in recs]
                off = recs[-1].offset + 1
        assert len(got) == len(set(got)) == sent           # every acked record once
        assert sorted(got) == list(range(sent))
    finally:
        proc.send_signal(signal.SIGKILL)
        proc.wait(10)


def test_write_behind_answers_and_shows_only_written_records(tmp_path):
    """kafka-lite over the durable store writes on a writer thread: a produce is answered only
    once its batch is in the segment file, and fetches / the high watermark only ever show
    written records (a killed broker never loses a record that was acknowledged or consumed)."""
    from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteCluster
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    d = tmp_path / "kl"
    cl = KafkaLiteCluster(1, default_partitions=2, data_dir=str(d), fsync="interval").start_in_thread()
    try:
        kb = KafkaBroker(cl.bootstrap)
        kb.create_topic("t", 2)
        store = cl.nodes[0].store
        seg = None
        for k in range(40):
            kb.produce_many("t", [f"v{k}-{i}".encode() * 20 for i in range(50)], partition=0)
            if seg is None:
                seg = next((d / "t-0").glob("*.log"))
            # acknowledged => written: the file holds every acknowledged batch
            assert store.written() >= 1 and seg.stat().st_size >= (k + 1) * 50 * 40
            assert store.end_offset("t", 0) == (k + 1) * 50
        err, hw, raw = kb.fetch_raw("t", 0, 0)
        assert err == 0 and hw == 2000
        # a ticket is visible only once written: the append is in memory, the fetch waits for it
        base, n, ticket = store.append_raw_nowait("t", 1, _batch(["x"] * 10))
        assert ticket > 0 and store.wait_written(ticket, 5.0)
        assert store.end_offset("t", 1) == 10 and len(_values(store, "t", 1)) == 10
        kb.close()
    finally:
        cl.stop()


def test_write_failure_refuses_new_produces_and_stops_the_broker(tmp_path):
    """once the writer thread failed (disk full / EIO), a produce is
    refused with a BrokerError -- never handed a ticket nobody will write -- and kafka-lite
    answers KAFKA_STORAGE_ERROR and asks to be restarted (on_store_failure)."""
    import errno

    from ccfd_demo_summit_amd.ingest.broker import BrokerError
    store = DurableBatchStore(str(tmp_path / "kl"), default_partitions=1, fsync="never")
    store.create_topic("t", 1)
    base, n, t = store.append_raw_nowait("t", 0, _batch(["a"] * 5))
    assert store.wait_written(t, 5.0)
    calls = []
    store.on_written = lambda ticket, tps: calls.append(ticket)

    def disk_full(fd, data):
        raise OSError(errno.ENOSPC, "No space left on device")
    store._write_raw = disk_full
    _b, _n, t2 = store.append_raw_nowait("t", 0, _batch(["b"] * 5))
    with pytest.raises(BrokerError):
        store.wait_written(t2, 5.0)
    assert calls and calls[-1] == -1
    with pytest.raises(BrokerError):                 # no more tickets after the failure
        store.append_raw_nowait("t", 0, _batch(["c"] * 5))
    store._werr = None                                # (let close() run)
    store.close()

    # kafka-lite over a failing store: the produce is answered with an error, the broker asks
    # to be restarted
    from ccfd_demo_summit_amd.ingest.kafka_lite import ERR_KAFKA_STORAGE_ERROR, KafkaLiteCluster
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    cl = KafkaLiteCluster(1, default_partitions=1, data_dir=str(tmp_path / "kl2"), fsync="never")
    failed = []
    cl.state.on_store_failure = lambda: failed.append(1)
    cl.start_in_thread()
    try:
        kb = KafkaBroker(cl.bootstrap)
        kb.create_topic("t", 1)
        kb.produce_many("t", [b"ok"] * 10, partition=0)
        cl.store._write_raw = disk_full
        with pytest.raises(BrokerError):
            kb.produce_many("t", [b"lost"] * 10, partition=0)
        t0 = time.time()
        while not failed and time.time() - t0 < 5:
            time.sleep(0.05)
        assert failed
        with pytest.raises(BrokerError) as ei:
            kb.produce_many("t", [b"refused"] * 10, partition=0)
        assert str(ERR_KAFKA_STORAGE_ERROR) in str(ei.value) or "storage" in str(ei.value).lower() \
            or "error" in str(ei.value).lower()
        kb.close()
    finally:
        cl.store._werr = None
        cl.stop()


def test_producer_sequences_wrap_at_2_pow_31():
    """idempotent sequences are int32 and wrap to 0 (Kafka semantics) on both
    the client and the broker -- a long-running producer neither dies on struct.pack nor gets
    OutOfOrderSequence after 2^31 records."""
    from ccfd_demo_summit_amd.ingest.batch_store import BatchStore
    from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteCluster
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    st = BatchStore(default_partitions=1)
    st.create_topic("t", 1)
    top = (1 << 31) - 3
    st.append_raw("t", 0, _batch(["a"] * 5, pid=7, seq=top))            # seqs top .. 1 (wrapped)
    st.append_raw("t", 0, _batch(["b"] * 5, pid=7, seq=2))              # the next one after the wrap
    assert st.append_raw("t", 0, _batch(["b"] * 5, pid=7, seq=2)) == (5, 0)   # a retry: stored once
    with pytest.raises(OutOfOrderSequence):
        st.append_raw("t", 0, _batch(["c"] * 5, pid=7, seq=top + 2))
    assert st.end_offset("t", 0) == 10
    cl = KafkaLiteCluster(1, default_partitions=1).start_in_thread()
    try:
        kb = KafkaBroker(cl.bootstrap, idempotent=True)
        kb.create_topic("w", 1)
        kb.produce_many("w", [b"x"] * 4, partition=0)
        kb._seq[("w", 0)] = (1 << 31) - 2            # as if 2^31 records had been sent
        st2 = cl.store
        pid = next(iter(st2._producers[("w", 0)]))
        st2._producers[("w", 0)][pid][1][-1] = ((1 << 31) - 6, (1 << 31) - 3, 0)
        for _ in range(3):
            kb.produce_many("w", [b"y"] * 4, partition=0)
        assert kb._seq[("w", 0)] == 10 and st2.end_offset("w", 0) == 16
        kb.close()
    finally:
        cl.stop()


def test_truncate_refuses_a_cut_inside_the_last_batch():
    """an offset inside the LAST batch (bisect lands past the end) was accepted and
    left the log end pointing into a stored batch."""
    from ccfd_demo_summit_amd.ingest.batch_store import BatchStore
    from ccfd_demo_summit_amd.ingest.broker import BrokerError
    s = BatchStore(default_partitions=1)
    s.create_topic("t", 1)
    s.append_raw("t", 0, _batch(["a", "b", "c"]))
    s.append_raw("t", 0, _batch(["d", "e", "f"]))
    with pytest.raises(BrokerError):
        s.truncate("t", 0, 4)                 # inside the last batch [3, 6)
    with pytest.raises(BrokerError):
        s.truncate("t", 0, 1)                 # inside the first batch [0, 3)
    assert s.end_offset("t", 0) == 6
    assert s.truncate("t", 0, 3) == 1 and s.end_offset("t", 0) == 3
