"""CPU side of the lossless fraud hand-off: the Python pump resumes a
native pump that stopped on a full flagged ring, routes the drained records to the caller's
hand-off (or the stash) in completion order, and any report of a dropped record is refused
-- by the engine wrapper (HandoffLost) and by bench.py (no JSON line, exit 5)."""
import ctypes as C
import threading
import time

import numpy as np
import pytest

from ccfd_demo_summit_amd.engine import stream_engine as se
from ccfd_demo_summit_amd.ops._lib import ENGINE_FLAG_FULL, FLAGGED_DTYPE


class FakeNative:
    """Stands in for libccfd_hip: batches of 4 rows, every row fraud-routed, a flagged ring of
    8 records that pump() refuses to overfill (the contract of engine.cpp complete())."""

    def __init__(self, cap=8, rows=4):
        self.cap, self.rows = cap, rows
        self.ring = []
        self.next_id = 0
        self.dropped = 0
        self.full_events = 0
        self.pump_calls = 0
        self.mu = threading.Lock()                           # engine.cpp ring_mu

    def ccfd_engine_pump(self, h, n, rows, drain, st_ref):
        st = st_ref._obj
        self.pump_calls += 1
        done = 0
        while done < n:
            with self.mu:
                full = len(self.ring) + self.rows > self.cap
                if not full:
                    self.ring.extend(range(self.next_id, self.next_id + self.rows))
                    self.next_id += self.rows
            if full:                                         # no room: stop, lose nothing
                self.full_events += 1
                st.submitted += done
                st.flag_full_events = self.full_events
                return ENGINE_FLAG_FULL
            st.batches += 1
            st.rows += self.rows
            st.fraud_rows += self.rows
            done += 1
        st.submitted += done
        st.flagged_dropped = self.dropped
        st.flag_full_events = self.full_events
        return 0

    def ccfd_engine_drain_flagged(self, h, buf, k):
        with self.mu:
            take = self.ring[:k]
            del self.ring[:k]
        if isinstance(buf, int):                             # an address (numpy array's data)
            buf = (se.Flagged * max(1, k)).from_address(buf)
        arr = np.frombuffer(buf, dtype=np.dtype(FLAGGED_DTYPE), count=len(take))
        arr["tx_id"] = take
        return len(take)


def _engine(fake, monkeypatch):
    monkeypatch.setattr(se, "lib", lambda: fake)
    eng = object.__new__(se.StreamEngine)
    eng.h = 1
    eng.batch = fake.rows
    eng._flag_buf = (se.Flagged * 65536)()
    eng._stash = []
    eng._drain_lock = threading.Lock()
    return eng


def test_pump_resumes_after_flag_full_and_hands_off_everything(monkeypatch):
    fake = FakeNative()
    eng = _engine(fake, monkeypatch)
    got = []
    st = eng.pump(10, on_flagged=lambda r: got.extend(r["tx_id"].tolist()))
    got.extend(eng.drain_flagged()["tx_id"].tolist())
    assert st.batches == 10 and st.submitted == 10
    assert st.flag_full_events > 0 and fake.pump_calls > 1
    assert got == list(range(40))                      # every record once, in completion order
    eng.h = None


def test_pump_without_callback_stashes_in_order(monkeypatch):
    fake = FakeNative()
    eng = _engine(fake, monkeypatch)
    eng.pump(7)
    eng.pump(3)
    out = eng.drain_flagged()["tx_id"].tolist()
    assert out == list(range(40))
    assert len(eng.drain_flagged()) == 0
    # a bounded drain takes from the stash first and keeps the rest
    eng.pump(5)
    a = eng.drain_flagged(6)["tx_id"].tolist()
    b = eng.drain_flagged()["tx_id"].tolist()
    assert a + b == list(range(40, 60)) and len(a) == 6
    eng.h = None


def test_dropped_record_is_refused(monkeypatch):
    fake = FakeNative()
    fake.dropped = 3
    eng = _engine(fake, monkeypatch)
    with pytest.raises(se.HandoffLost):
        eng.pump(1)
    with pytest.raises(se.HandoffLost):
        se.check_lossless(se.StepStats(dropped=1))
    se.check_lossless(se.StepStats(dropped=0))
    eng.h = None


def test_bench_refuses_a_lossy_line():
    """bench.py prints no JSON line (exit 5) unless hand-offs == the kernels' fraud counter."""
    import importlib.util
    from pathlib import Path
    spec = importlib.util.spec_from_file_location("bench_mod", Path(__file__).resolve().parents[1] / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.handoff_refusal(21_772_280, 21_772_280) is None
    msg = bench.handoff_refusal(20_971_520, 21_772_280)     # the round-5 config-4 line
    assert msg and "refusing" in msg


def test_collector_thread_beside_the_pump_hands_off_everything_once(monkeypatch):
    """bench.py's hand-off: a FlaggedDrainer thread drains while this thread pumps (the
    pump's own full-ring path drains into the same sink); every record arrives exactly once,
    in completion order, and stop() leaves the ring empty."""
    fake = FakeNative(cap=64, rows=4)
    eng = _engine(fake, monkeypatch)
    got = []
    mu = threading.Lock()

    def sink(r):
        with mu:
            got.extend(r["tx_id"].tolist())
    dr = se.FlaggedDrainer(eng, sink, idle_s=1e-5).start()
    for _ in range(50):
        eng.pump(40, on_flagged=sink)
    n = dr.stop()
    assert got == list(range(50 * 40 * 4))
    assert n <= len(got) and dr.drains > 0
    assert fake.ring == []
    eng.h = None


def test_collector_thread_reraises_a_sink_failure(monkeypatch):
    fake = FakeNative(cap=64, rows=4)
    eng = _engine(fake, monkeypatch)

    def sink(_r):
        raise RuntimeError("router down")
    dr = se.FlaggedDrainer(eng, sink, idle_s=1e-5).start()
    eng.pump(2, on_flagged=lambda r: None)
    time.sleep(0.05)
    with pytest.raises(RuntimeError, match="router down"):
        dr.stop()
    eng.h = None
