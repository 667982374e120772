"""Lossless fraud hand-off from the kernel epilogue to the router.

The engine's flagged ring holds the fraud-routed records of completed micro-batches until the
router hand-off drains them.  It is deliberately tiny here (``flag_capacity`` 1024 = one
micro-batch) and every row routes to fraud (threshold 0), so every batch fills it: scoring has
to stall on the slow drainer, and every fraud row must still be handed off exactly once
(reference: README.md:552,558 -- a fraud transaction starts a fraud process).
"""
import threading
import time

import numpy as np
import pytest
import torch

from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import build_model

pytestmark = pytest.mark.gpu

B = 1024


@pytest.fixture(scope="module")
def setup(gpu):
    X, _ = generate(B * 40, seed=61)
    m = build_model("mlp", seed=6, X_ref=X[:20000], calibrate_rate=0.01)
    return X, m


def _exactly_once(tx_ids, expect_ids):
    got = np.sort(np.asarray(tx_ids, np.uint64))
    assert len(got) == len(expect_ids), (len(got), len(expect_ids))
    np.testing.assert_array_equal(got, np.sort(expect_ids))


@pytest.mark.parametrize("exec_mode,wire", [("launch", False), ("persistent", False), ("persistent", True)])
def test_pump_slow_drainer_every_fraud_row_once(gpu, setup, exec_mode, wire):
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, m = setup
    eng = StreamEngine(DeviceModel(m, gpu, wire=wire), batch=B, depth=4, streams=2, input_mode="zerocopy",
                       exec_mode=exec_mode, threshold=0.0, flag_capacity=1024)
    n_b = 32
    log = PartitionLog.from_arrays(X[:n_b * B], ids=np.arange(n_b * B, dtype=np.uint64) + 5, wire=wire)
    eng.add_log(0, log)
    handed = []

    def slow_handoff(rec):
        time.sleep(0.002)                       # a router that is slower than the GPU
        handed.append(rec["tx_id"].copy())

    st = eng.pump(n_b, drain=True, on_flagged=slow_handoff)
    handed.append(eng.drain_flagged()["tx_id"])
    assert st.rows == n_b * B and st.batches == n_b
    assert st.dropped == 0
    assert st.flag_full_events > 0               # scoring stalled on the ring instead of dropping
    assert st.fraud_rows == n_b * B
    _exactly_once(np.concatenate(handed), np.arange(n_b * B, dtype=np.uint64) + 5)
    side = torch.cuda.Stream(gpu)
    c = eng.flip_epoch(side)
    side.synchronize()
    assert int(c.cpu()[1]) == n_b * B            # device fraud counter == records handed off
    eng.close()
    log.free()


@pytest.mark.parametrize("wire", [False, True])
def test_collector_thread_beside_pump_every_fraud_row_once(gpu, setup, wire):
    """bench.py's hand-off: a FlaggedDrainer thread drains while the pump keeps submitting,
    steps of drain=False pumps like the bench's, a small ring so the pump also meets a full
    ring and drains into the same sink: every fraud row once, the device counter agrees."""
    from ccfd_demo_summit_amd.engine import FlaggedDrainer, PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, m = setup
    eng = StreamEngine(DeviceModel(m, gpu, wire=wire), batch=B, depth=4, streams=2, input_mode="zerocopy",
                       exec_mode="persistent", threshold=0.0, flag_capacity=4 * B)
    n_b = 40
    log = PartitionLog.from_arrays(X[:n_b * B], ids=np.arange(n_b * B, dtype=np.uint64) + 11, wire=wire)
    eng.add_log(0, log)
    handed = []
    mu = threading.Lock()

    def sink(rec):
        with mu:
            handed.append(rec["tx_id"].copy())
    dr = FlaggedDrainer(eng, sink).start()
    rows = fraud = 0
    for k in range(4):                            # 4 steps of 10 micro-batches, the last drains
        st = eng.pump(10, drain=(k == 3), on_flagged=sink)
        rows += st.rows
        fraud += st.fraud_rows
        assert st.dropped == 0
    dr.stop()
    assert rows == n_b * B and fraud == n_b * B
    _exactly_once(np.concatenate(handed), np.arange(n_b * B, dtype=np.uint64) + 11)
    side = torch.cuda.Stream(gpu)
    c = eng.flip_epoch(side)
    side.synchronize()
    assert int(c.cpu()[1]) == n_b * B
    eng.close()
    log.free()


def test_pump_without_callback_stashes_for_drain(gpu, setup):
    """No hand-off callback: a blocking pump stashes what it had to take out of the ring, and
    drain_flagged returns it first, in completion order (nothing lost, nothing repeated)."""
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, m = setup
    eng = StreamEngine(DeviceModel(m, gpu), batch=B, depth=4, streams=2, input_mode="zerocopy",
                       exec_mode="persistent", threshold=0.0, flag_capacity=1024)
    log = PartitionLog.from_arrays(X[:8 * B], ids=np.arange(8 * B, dtype=np.uint64), wire=False)
    eng.add_log(0, log)
    st = eng.pump(8, drain=True)
    assert st.rows == 8 * B and st.dropped == 0
    fl = eng.drain_flagged()["tx_id"]
    assert len(fl) == 8 * B
    for k in range(8):          # batch completion order (the kernel compacts a batch's rows in any order)
        np.testing.assert_array_equal(np.sort(fl[k * B:(k + 1) * B]), np.arange(k * B, (k + 1) * B, dtype=np.uint64))
    eng.close()
    log.free()


def test_g20_persistent_slow_drainer(gpu):
    """Config-4 path (persistent G20 GBDT kernel): same guarantee with a low threshold."""
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    Bg = 8192
    X, _ = generate(Bg * 12, seed=62)
    m = build_model("gbdt", seed=8, X_ref=X[:20000], gbdt_trees=100, gbdt_depth=6, calibrate_rate=0.3)
    dm = DeviceModel(m, gpu, bins="g20")
    eng = StreamEngine(dm, batch=Bg, depth=4, streams=1, exec_mode="persistent", flag_capacity=1024)
    log = PartitionLog.from_arrays(X, ids=np.arange(X.shape[0], dtype=np.uint64) + 9, bins=dm.bins)
    eng.add_log(0, log)
    handed = []
    st = eng.pump(12, drain=True, on_flagged=lambda r: (time.sleep(0.001), handed.append(r["tx_id"].copy())))
    handed.append(eng.drain_flagged()["tx_id"])
    ref = np.nonzero(m.predict_proba(X) >= 0.5)[0].astype(np.uint64) + 9
    assert len(ref) > 2 * Bg                     # several batches overflow the 8192-record ring
    assert st.dropped == 0 and st.flag_full_events > 0
    _exactly_once(np.concatenate(handed), ref)
    eng.close()
    log.free()


@pytest.mark.parametrize("exec_mode", ["launch", "persistent"])
def test_serving_thread_slow_collector_stalls_not_drops(gpu, setup, exec_mode):
    """Streaming: the native serving thread scores the ring while a slow collector drains;
    completed batches wait for ring room (the ingest ring back-pressures the producer)."""
    from ccfd_demo_summit_amd.engine import StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, m = setup
    n = 30 * B
    eng = StreamEngine(DeviceModel(m, gpu), batch=B, depth=4, streams=2, input_mode="zerocopy",
                       exec_mode=exec_mode, threshold=0.0, flag_capacity=1024)
    eng.set_ring(0, 4 * B)
    eng.serve_start(200, 200)
    ids = np.arange(n, dtype=np.uint64) + 11
    done = threading.Event()

    def produce():
        eng.ring_write(0, X[:n], ids=ids)        # blocks while the ring is full
        done.set()
    th = threading.Thread(target=produce, daemon=True)
    th.start()
    handed, rows, full = [], 0, 0
    t0 = time.time()
    while rows < n and time.time() - t0 < 60:
        time.sleep(0.005)                        # slow hand-off consumer
        st, fl, _ = eng.serve_collect()
        handed.append(fl["tx_id"].copy())
        rows, full = int(st.rows), int(st.flag_full_events)
        assert st.dropped == 0
    th.join(10)
    eng.serve_stop()
    st, fl, _ = eng.serve_collect()
    handed.append(fl["tx_id"].copy())
    assert done.is_set() and int(st.rows) == n
    assert full > 0
    _exactly_once(np.concatenate(handed), ids)
    eng.close()
