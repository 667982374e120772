"""Native streaming engine on the GPU: DMA and zero-copy modes, counters, flagged
hand-off ring, epoch flip (X2 side stream)."""
import numpy as np
import pytest
import torch

from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import build_model

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup(gpu):
    X, y = generate(4096 * 6 + 100, seed=21)
    m = build_model("mlp", seed=4, X_ref=X[:20000], calibrate_rate=0.01)
    return X, m


@pytest.mark.parametrize("input_mode,output_mode,exec_mode", [
    ("dma", "zerocopy", "launch"), ("zerocopy", "zerocopy", "launch"), ("dma", "dma", "launch"),
    ("zerocopy", "dma", "launch"), ("zerocopy", "zerocopy", "persistent"), ("dma", "zerocopy", "persistent"),
    ("zerocopy", "zerocopy", "launch-wire"), ("dma", "zerocopy", "launch-wire"),
    ("zerocopy", "zerocopy", "persistent-wire"), ("zerocopy", "zerocopy", "launch-c4"),
    ("zerocopy", "zerocopy", "launch-wire-c3")])
def test_engine_pump_matches_oracle(gpu, setup, input_mode, output_mode, exec_mode):
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, m = setup
    coalesce = int(exec_mode.split("-c")[1]) if "-c" in exec_mode else 1
    exec_mode = exec_mode.split("-c")[0]
    wire = exec_mode.endswith("-wire")
    exec_mode = exec_mode.replace("-wire", "")
    dm = DeviceModel(m, gpu, wire=wire)
    eng = StreamEngine(dm, batch=4096, depth=4, streams=2, input_mode=input_mode,
                       output_mode=output_mode, exec_mode=exec_mode, coalesce=coalesce)
    log = PartitionLog.from_arrays(X, ids=np.arange(X.shape[0], dtype=np.uint64) + 1000, wire=wire)
    eng.add_log(0, log)
    st = eng.pump(6)
    assert st.batches == 6 and st.rows == 6 * 4096
    if wire:
        from ccfd_demo_summit_amd.contracts import decode_wire, encode_wire
        ref = m.wire_proba(X[:6 * 4096])
    else:
        ref = m.predict_proba(X[:6 * 4096], emulate_bf16=True)
    flagged = eng.drain_flagged()
    got = np.zeros(6 * 4096, bool)
    got[(flagged["tx_id"] - 1000).astype(np.int64)] = True
    # rows clearly away from the threshold must route exactly like the bf16 oracle
    clear = np.abs(ref - 0.5) > 2e-3
    np.testing.assert_array_equal(got[clear], (ref >= 0.5)[clear])
    assert st.fraud_rows == len(flagged)
    side = torch.cuda.Stream(gpu)
    closed = eng.flip_epoch(side)
    side.synchronize()
    c = closed.cpu().numpy()
    assert c[0] == 6 * 4096 and c[1] == st.fraud_rows
    amt = X[(flagged["tx_id"] - 1000).astype(np.int64), 29]
    np.testing.assert_allclose(flagged["amount"], amt)
    assert st.p50_us > 0
    if output_mode == "zerocopy":
        # K7: every micro-batch carries a device-clock execution window (launch + persistent)
        assert st.dev_batches == 6 and 0 < st.dev_exec_mean_us < 10_000
    eng.close()
    log.free()


def test_engine_score_sync_pageable_input(gpu, setup):
    from ccfd_demo_summit_amd.engine import StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, m = setup
    eng = StreamEngine(DeviceModel(m, gpu), batch=1024, depth=2, input_mode="zerocopy")
    p, r = eng.score(X[:3000])          # numpy (pageable) input is staged by DMA
    assert np.abs(p - m.predict_proba(X[:3000])).max() < 1e-2
    eng.close()


@pytest.mark.parametrize("exec_mode", ["launch", "persistent", "launch-wire", "launch-wire-c4", "persistent-wire"])
def test_ring_streaming_mode_deadline_flush(gpu, setup, exec_mode):
    """Live ingest: producer writes into the pinned SPSC ring (rows + JSON), run() scores full
    micro-batches and deadline-flushes the partial tail; ring space is recycled."""
    import json
    import time
    from ccfd_demo_summit_amd.contracts import FEATURE_NAMES
    from ccfd_demo_summit_amd.engine import StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, m = setup
    coalesce = int(exec_mode.split("-c")[1]) if "-c" in exec_mode else 1
    exec_mode = exec_mode.split("-c")[0]
    wire = exec_mode.endswith("-wire")
    eng = StreamEngine(DeviceModel(m, gpu, wire=wire), batch=1024, depth=8, streams=2, input_mode="zerocopy",
                       exec_mode=exec_mode.replace("-wire", ""), coalesce=coalesce)
    eng.set_ring(0, 4096)
    n = 10_000                                   # > capacity: exercises wrap + backpressure
    ids = np.arange(n, dtype=np.uint64) + 7
    written, scored = 0, 0
    t_start = time.time()
    while scored < n and time.time() - t_start < 60:
        if written < n:
            e = min(n, written + 1500)
            written += eng.ring_write(0, X[written:e], ids[written:e], block=False)
        st = eng.run(budget_us=2000, flush_us=200)
        scored += st.rows
    assert scored == n
    flagged = eng.drain_flagged()
    if wire:
        from ccfd_demo_summit_amd.contracts import decode_wire, encode_wire
        ref = m.wire_proba(X[:n])
    else:
        ref = m.predict_proba(X[:n], emulate_bf16=True)
    got = np.zeros(n, bool)
    got[(flagged["tx_id"] - 7).astype(np.int64)] = True
    clear = np.abs(ref - 0.5) > 2e-3
    np.testing.assert_array_equal(got[clear], (ref >= 0.5)[clear])
    # JSON messages parsed natively straight into the ring, partial batch flushed by deadline
    msgs = [json.dumps({"id": 100000 + i, **{k: float(v) for k, v in zip(FEATURE_NAMES, X[i])}}).encode()
            for i in range(300)]
    assert eng.ring_write_json(0, msgs) == 300
    got_rows = 0
    t0 = time.time()
    while got_rows < 300 and time.time() - t0 < 10:
        got_rows += eng.run(budget_us=1000, flush_us=100).rows
    assert got_rows == 300
    assert eng.cursor(0) == n + 300
    eng.close()


def test_persistent_engine_many_steps_counters_exact(gpu, setup):
    """Persistent kernel across repeated halt/relaunch cycles: counters and epochs exact."""
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    from ccfd_demo_summit_amd.parallel import CounterReducer, DistContext, EpochPipeline
    X, m = setup
    eng = StreamEngine(DeviceModel(m, gpu), batch=2048, depth=8, input_mode="zerocopy", exec_mode="persistent")
    log = PartitionLog.from_arrays(X)
    eng.add_log(0, log)
    red = CounterReducer(DistContext(0, 1, 0, gpu, "none"), gpu)
    ep = EpochPipeline(eng, red)
    total = 0
    for k in range(12):
        st = eng.pump(37, batch_rows=2000 if k % 3 else 2048, drain=(k % 4 == 3))
        total += 37 * (2000 if k % 3 else 2048)
        ep.tick()
    eng.pump(0, drain=True)
    ep.finish()
    c, _ = red.snapshot()
    assert c[0] == total
    assert c[1] + c[2] == total
    eng.close()
    log.free()


@pytest.mark.parametrize("exec_mode", ["launch", "persistent"])
def test_hot_swap_between_micro_batches(gpu, setup, exec_mode):
    """Runtime X1: batches before the swap route with model A, batches after with model B."""
    from ccfd_demo_summit_amd.contracts import decode_wire, encode_wire
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, mA = setup
    mB = build_model("mlp", seed=77, X_ref=X[:20000], calibrate_rate=0.05)
    eng = StreamEngine(DeviceModel(mA, gpu, wire=True), batch=4096, depth=4, streams=2, input_mode="zerocopy",
                       exec_mode=exec_mode, coalesce=2)
    log = PartitionLog.from_arrays(X, ids=np.arange(X.shape[0], dtype=np.uint64), wire=True)
    eng.add_log(0, log)
    eng.pump(3)
    eng.swap_model(DeviceModel(mB, gpu, wire=True))
    eng.pump(3)
    flagged = eng.drain_flagged()
    got = np.zeros(6 * 4096, bool)
    got[flagged["tx_id"].astype(np.int64)] = True
    Xd = decode_wire(encode_wire(X[:6 * 4096]))
    ref = np.concatenate([mA.wire_proba(X[:3 * 4096]), mB.wire_proba(X[3 * 4096:6 * 4096])])
    clear = np.abs(ref - 0.5) > 2e-3
    np.testing.assert_array_equal(got[clear], (ref >= 0.5)[clear])
    assert eng.model_version == 1
    with pytest.raises(ValueError):
        eng.swap_model(DeviceModel(mB, gpu, wire=False))
    eng.close()
    log.free()


@pytest.mark.parametrize("wire", [False, True])
def test_lr_coalesced_pump_matches_oracle(gpu, setup, wire):
    from ccfd_demo_summit_amd.contracts import decode_wire, encode_wire
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, _ = setup
    m = build_model("lr", seed=5, X_ref=X[:20000], calibrate_rate=0.02)
    eng = StreamEngine(DeviceModel(m, gpu, wire=wire), batch=4096, depth=8, streams=2, input_mode="zerocopy",
                       coalesce=4)
    log = PartitionLog.from_arrays(X, ids=np.arange(X.shape[0], dtype=np.uint64), wire=wire)
    eng.add_log(0, log)
    st = eng.pump(6)
    assert st.rows == 6 * 4096
    Xs = decode_wire(encode_wire(X[:6 * 4096])) if wire else X[:6 * 4096]
    ref = m.predict_proba(Xs)
    got = np.zeros(6 * 4096, bool)
    got[eng.drain_flagged()["tx_id"].astype(np.int64)] = True
    clear = np.abs(ref - 0.5) > 1e-4
    np.testing.assert_array_equal(got[clear], (ref >= 0.5)[clear])
    side = torch.cuda.Stream(gpu)
    c = eng.flip_epoch(side)
    side.synchronize()
    assert int(c[0]) == 6 * 4096
    eng.close()
    log.free()


def test_persistent_queue_isolation(gpu):
    """While the persistent kernel is resident, fresh torch streams (normal and high
    priority) and the default stream still make progress: the kernel owns a hardware queue
    no other stream is mapped onto (GPU_MAX_HW_QUEUES=4 multiplexes streams onto queues)."""
    import subprocess
    import sys
    from pathlib import Path
    probe = Path(__file__).parent / "helpers" / "queue_probe.py"
    r = subprocess.run([sys.executable, str(probe), "12"], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "ALL_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("exec_mode", ["launch", "persistent"])
@pytest.mark.parametrize("wire", [False, True])
def test_engine_score_sync_every_exec_mode(gpu, setup, exec_mode, wire):
    """StreamEngine.score (synchronous DMA path, used by the native Seldon REST server) scores
    every row in persistent mode too (round-1 bug: the descriptor carried a stale row count
    of 0, so the resident kernel completed the batch without scoring it)."""
    from ccfd_demo_summit_amd.engine import StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, m = setup
    eng = StreamEngine(DeviceModel(m, gpu, wire=wire), batch=4096, depth=4, streams=2, input_mode="zerocopy",
                       exec_mode=exec_mode)
    p, r = eng.score(X[:10_000])
    eng.close()
    ref = m.wire_proba(X[:10_000]) if wire else m.predict_proba(X[:10_000], emulate_bf16=True)
    assert np.abs(p - ref).max() < 2e-3
    np.testing.assert_array_equal(r, (p >= 0.5).astype(np.uint8))


@pytest.mark.parametrize("kind", ["mlp", "lr"])
@pytest.mark.parametrize("item_rows", [64, 128, 256, 512, 1024])
def test_persistent_wire_item_sizes_exact(gpu, setup, monkeypatch, kind, item_rows):
    """Every persistent work-item size on W64 rows -- 256 / 512 take the all-tiles-in-flight
    paired path, the others the one-tile prefetch loop -- scores every row once, full and
    partial micro-batches alike: rows, routes and the proba sum match the wire oracle."""
    from ccfd_demo_summit_amd.contracts import decode_wire, encode_wire
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, m = setup
    if kind == "lr":
        m = build_model("lr", seed=5, X_ref=X[:20000], calibrate_rate=0.01)
    monkeypatch.setenv("CCFD_PERSIST_ITEM_ROWS", str(item_rows))
    eng = StreamEngine(DeviceModel(m, gpu, wire=True), batch=4096, depth=4, streams=1, exec_mode="persistent")
    log = PartitionLog.from_arrays(X, ids=np.arange(X.shape[0], dtype=np.uint64) + 1000, wire=True)
    eng.add_log(0, log)
    a = eng.pump(3)
    b = eng.pump(2, batch_rows=1000)                  # partial items: 1000 = 3 x 256 + 232
    n = 3 * 4096 + 2000
    assert a.rows + b.rows == n
    Xw = X[:n]
    ref = m.wire_proba(Xw) if kind == "mlp" else m.predict_proba(decode_wire(encode_wire(Xw)))
    flagged = eng.drain_flagged()
    got = np.zeros(n, bool)
    got[(flagged["tx_id"] - 1000).astype(np.int64)] = True
    clear = np.abs(ref - 0.5) > 2e-3
    np.testing.assert_array_equal(got[clear], (ref >= 0.5)[clear])
    side = torch.cuda.Stream(gpu)
    c = eng.flip_epoch(side)
    side.synchronize()
    c = c.cpu().numpy()
    assert c[0] == n and c[1] == len(flagged) and c[1] + c[2] == n
    assert abs(int(c[3]) - float(np.round(ref.astype(np.float64) * 1e6).sum())) < 2e-4 * n * 1e6 / 100
    assert int(c[8:22].sum() + c[24:38].sum()) == n          # amount histogram covers every row
    eng.close()
    log.free()


@pytest.mark.parametrize("item_rows,grid", [(64, 0), (128, 0), (64, 3), (128, 200)])
def test_persistent_pipe_items_exact(gpu, setup, monkeypatch, item_rows, grid):
    """Pipelined static work items (CCFD_PERSIST_PIPE, MLP on W64 rows; grid 3 = two workers
    that each own every other item): every row scored once for full and partial micro-batches,
    routes equal the wire oracle, and the counters -- incoming / fraud / standard, the proba
    sum and BOTH amount histograms -- equal the ones recomputed on the host from the device
    routes; the kernel halts and relaunches between pump calls."""
    from ccfd_demo_summit_amd.contracts.metric_names import AMOUNT_BUCKETS
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, m = setup
    monkeypatch.setenv("CCFD_PERSIST_PIPE", "1")
    monkeypatch.setenv("CCFD_PERSIST_ITEM_ROWS", str(item_rows))
    eng = StreamEngine(DeviceModel(m, gpu, wire=True), batch=4096, depth=6, streams=1, exec_mode="persistent",
                       persist_grid=grid)
    log = PartitionLog.from_arrays(X, ids=np.arange(X.shape[0], dtype=np.uint64) + 1000, wire=True)
    eng.add_log(0, log)
    a = eng.pump(5, drain=True)
    b = eng.pump(3, batch_rows=1000, drain=True)      # partial items and a partial last tile
    n = 5 * 4096 + 3000
    assert a.rows + b.rows == n
    ref = m.wire_proba(X[:n])
    flagged = eng.drain_flagged()
    got = np.zeros(n, bool)
    got[(flagged["tx_id"] - 1000).astype(np.int64)] = True
    assert len(flagged) == got.sum()                  # no row flagged twice
    clear = np.abs(ref - 0.5) > 2e-3
    np.testing.assert_array_equal(got[clear], (ref >= 0.5)[clear])
    side = torch.cuda.Stream(gpu)
    c = eng.flip_epoch(side)
    side.synchronize()
    c = c.cpu().numpy()
    assert c[0] == n and c[1] == got.sum() and c[2] == n - got.sum()
    assert abs(int(c[3]) - float(np.round(ref.astype(np.float64) * 1e6).sum())) < 2e-4 * n * 1e6 / 100
    bk = np.searchsorted(np.asarray(AMOUNT_BUCKETS, np.float32), X[:n, 29], side="left")
    np.testing.assert_array_equal(c[8:22], np.bincount(bk[~got], minlength=14))
    np.testing.assert_array_equal(c[24:38], np.bincount(bk[got], minlength=14))
    eng.close()
    log.free()


@pytest.mark.parametrize("wire", [False, True])
def test_score_sync_small_batches_zero_copy_stage(gpu, setup, monkeypatch, wire):
    """score() of small pageable batches goes through the pinned zero-copy stage
    (CCFD_SYNC_ZC_ROWS, the REST front end's path); larger ones through the DMA staging:
    outputs are identical to the all-DMA engine's at every size across the cut-over."""
    from ccfd_demo_summit_amd.engine import StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, m = setup
    out = {}
    for zc in ("0", "512"):
        monkeypatch.setenv("CCFD_SYNC_ZC_ROWS", zc)
        eng = StreamEngine(DeviceModel(m, gpu, wire=wire), batch=1024, depth=2, input_mode="dma")
        out[zc] = [eng.score(X[7:7 + n]) for n in (1, 31, 511, 512, 513, 1024, 3000)]
        eng.close()
    for (p0, r0), (p1, r1) in zip(out["0"], out["512"]):
        np.testing.assert_array_equal(p0, p1)
        np.testing.assert_array_equal(r0, r1)
    ref = m.wire_proba(X[7:3007]) if wire else m.predict_proba(X[7:3007])
    assert np.abs(out["512"][-1][0] - ref).max() < 1e-2



@pytest.mark.parametrize("exec_mode", ["launch", "persistent"])
def test_batch_stage_trace(gpu, setup, exec_mode, tmp_path):
    """Per-batch stage trace ring: one entry per retired micro-batch (the newest `capacity`),
    stages in order (submit <= landed <= retired, device window non-empty), rows and flagged
    counts match the pump, and the Chrome conversion writes a loadable timeline."""
    import json
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    from ccfd_demo_summit_amd.utils.tracing import dump_batch_trace
    X, m = setup
    eng = StreamEngine(DeviceModel(m, gpu, wire=True), batch=2048, depth=4, streams=2, exec_mode=exec_mode)
    log = PartitionLog.from_arrays(X, wire=True)
    eng.add_log(0, log)
    eng.enable_trace(8)
    st = eng.pump(11)
    tr = eng.read_trace()
    assert len(tr) == 8 and list(tr["seq"]) == list(range(3, 11))          # newest 8, oldest first
    assert (tr["rows"] == 2048).all() and int(st.fraud_rows) >= int(tr["flagged"].sum())
    assert (tr["t_submit"] <= tr["t_landed"]).all() and (tr["t_landed"] <= tr["t_complete"]).all()
    assert (tr["dev_end"] > tr["dev_start"]).all() and (tr["dev_start"] > 0).all()
    doc = json.loads(open(dump_batch_trace(tr, str(tmp_path / "t.json"))).read())
    assert len([e for e in doc["traceEvents"] if e["ph"] == "X"]) == 3 * 8   # no ring arrival in pump
    eng.close()
    log.free()
