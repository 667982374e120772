"""G20 rows (GBDT bins packed 5 bits each, csrc/kernels/g32_core.h g20_*): the launch and
persistent binned-row kernels choose exactly the f32 oracle's leaves on 20-byte rows, at any
4-byte-aligned start, counters and histogram exact, stale stamps detected, and broadcast_model
widens G20 -> G32 when an ensemble's table needs more than 31 edges a feature
(BASELINE.json configs[3])."""
import numpy as np
import pytest
import torch

from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import build_model

from test_kernels_gpu import _check_counters

pytestmark = pytest.mark.gpu


def _model(seed, X_ref, trees=100, depth=6, rate=0.01):
    m = build_model("gbdt", seed=seed, X_ref=X_ref, gbdt_trees=trees, gbdt_depth=depth, calibrate_rate=rate)
    assert m.bin_spec().fits_g20, "test ensemble must fit 5-bit bins"
    return m


@pytest.fixture(scope="module")
def data():
    X, _ = generate(65536 + 7, seed=51)
    X[3, 5] = np.nan
    X[4, 2] = np.inf
    X[5, 7] = -np.inf
    return X


@pytest.mark.parametrize("n", [1, 31, 4097, 65543])
@pytest.mark.parametrize("depth", [6, 3, 8])
def test_g20_kernel_exact(gpu, data, n, depth):
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel, new_counters, score
    X = data[:n]
    m = _model(3, generate(5000, seed=2)[0], trees=100 if depth != 8 else 40, depth=depth)
    dm = DeviceModel(m, gpu, bins="g20")
    assert dm.row_format == "g20"
    rows = torch.from_numpy(dm.bins.encode(X)).to(gpu)
    cnt = new_counters(gpu)
    p, r = score(dm, rows, 0.5, counters=cnt)
    torch.cuda.synchronize(gpu)
    p, r = p.cpu().numpy(), r.cpu().numpy()
    ref = m.predict_proba(X)
    assert np.abs(p - ref).max() < 1e-5
    np.testing.assert_array_equal(r, (ref >= 0.5).astype(np.uint8))
    _check_counters(cnt, p, r, X)
    assert int(cnt[4]) == 0


def test_g20_unaligned_start_and_stale_stamp(gpu, data):
    """A batch starting at row 1 of a buffer is only 4-byte aligned (20 B rows): the dword
    loads still read it exactly; rows of another stamp are counted, not scored."""
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel, new_counters, score
    X = data[:4098]
    m = _model(6, X)
    dm = DeviceModel(m, gpu, bins="g20")
    enc = dm.bins.encode(X)
    st = dm.bins.stamp
    bad_stamp = (st % 63) + 1
    enc[101:201, 19] = (enc[101:201, 19] & 0x03) | (bad_stamp << 2)   # stamp = bits 154..159
    enc[301, :] = 0
    full = torch.from_numpy(enc).to(gpu)
    view = full[1:]
    assert view.data_ptr() % 16 == 4
    cnt = new_counters(gpu)
    p, r = score(dm, view, 0.5, counters=cnt)
    torch.cuda.synchronize(gpu)
    p, r = p.cpu().numpy(), r.cpu().numpy()
    assert int(cnt[4]) == 101 and int(cnt[0]) == 4097
    assert np.isnan(p[100:200]).all() and np.isnan(p[300]) and not r[100:200].any()
    ok = np.ones(4097, bool)
    ok[100:200] = False
    ok[300] = False
    assert np.abs(p[ok] - m.predict_proba(X[1:])[ok]).max() < 1e-5


@pytest.mark.parametrize("input_mode,exec_mode", [("zerocopy", "launch"), ("dma", "launch"),
                                                   ("zerocopy", "persistent"), ("dma", "persistent")])
def test_g20_engine_pump_exact(gpu, input_mode, exec_mode):
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    B = 8192
    X, _ = generate(B * 4 + 100, seed=54)
    m = _model(8, X[:20000])
    dm = DeviceModel(m, gpu, bins="g20")
    eng = StreamEngine(dm, batch=B, depth=4, streams=2, input_mode=input_mode, exec_mode=exec_mode)
    log = PartitionLog.from_arrays(X, ids=np.arange(X.shape[0], dtype=np.uint64) + 7, bins=dm.bins)
    assert log.row_format == "g20" and log.row_bytes == 20
    eng.add_log(0, log)
    st = eng.pump(4)
    assert st.rows == 4 * B
    ref = m.predict_proba(X[:4 * B]) >= 0.5
    fl = eng.drain_flagged()
    got = np.zeros(4 * B, bool)
    got[(fl["tx_id"] - 7).astype(np.int64)] = True
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_allclose(fl["amount"], X[(fl["tx_id"] - 7).astype(np.int64), 29])
    side = torch.cuda.Stream(gpu)
    c = eng.flip_epoch(side)
    side.synchronize()
    c = c.cpu().numpy()
    assert c[0] == 4 * B and c[1] == ref.sum() and c[4] == 0
    p, _ = eng.score(X[:1000])
    assert np.abs(p - m.predict_proba(X[:1000])).max() < 1e-5
    eng.close()
    log.free()


@pytest.mark.parametrize("inflight", ["0", "1"])
@pytest.mark.parametrize("item_rows", [256, 1024])
def test_g20_persistent_partial_batches_exact(gpu, monkeypatch, inflight, item_rows):
    """Both persistent item loops, partial micro-batches starting at rows that are not a
    multiple of 4 (4-byte-aligned G20 rows): every row scored once, routes exact."""
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    monkeypatch.setenv("CCFD_G32_INFLIGHT", inflight)
    monkeypatch.setenv("CCFD_PERSIST_ITEM_ROWS", str(item_rows))
    B = 8192
    X, _ = generate(B * 3 + 3000, seed=55)
    m = _model(10, X[:20000], rate=0.05)
    dm = DeviceModel(m, gpu, bins="g20")
    eng = StreamEngine(dm, batch=B, depth=3, streams=1, exec_mode="persistent")
    log = PartitionLog.from_arrays(X, ids=np.arange(X.shape[0], dtype=np.uint64) + 7, bins=dm.bins)
    eng.add_log(0, log)
    n = 1301 + B + 2 * 1303
    assert eng.pump(1, batch_rows=1301).rows + eng.pump(1).rows + eng.pump(2, batch_rows=1303).rows == n
    pr = m.predict_proba(X[:n])
    fl = eng.drain_flagged()
    got = np.zeros(n, bool)
    got[(fl["tx_id"] - 7).astype(np.int64)] = True
    np.testing.assert_array_equal(got, pr >= 0.5)
    side = torch.cuda.Stream(gpu)
    c = eng.flip_epoch(side)
    side.synchronize()
    c = c.cpu().numpy()
    assert c[0] == n and c[1] == (pr >= 0.5).sum() and c[4] == 0
    assert int(c[8:22].sum() + c[24:38].sum()) == n
    eng.close()
    log.free()


def test_broadcast_model_widens_g20_to_g32(gpu):
    """> 31 thresholds on a feature: G20 is impossible, broadcast_model hands out a G32 model."""
    from ccfd_demo_summit_amd.models.gbdt import ObliviousGBDT
    from ccfd_demo_summit_amd.ops.kernels import score
    from ccfd_demo_summit_amd.parallel import broadcast_model, init_distributed
    X, _ = generate(30000, seed=57)
    T = 40
    feat = np.zeros((T, 2), np.int32)                 # 80 thresholds on feature 0
    thr = np.quantile(X[:, 0], np.linspace(0.01, 0.99, 2 * T)).astype(np.float32).reshape(T, 2)
    rng = np.random.default_rng(3)
    m = ObliviousGBDT(feat, thr, (rng.standard_normal((T, 4)) * 0.05).astype(np.float32), -1.0)
    ctx = init_distributed()
    with pytest.warns(UserWarning, match="G20 rows impossible"):
        dm = broadcast_model(ctx, m, "gbdt", "g20")
    assert dm.row_format == "g32"
    p, _ = score(dm, torch.from_numpy(dm.bins.encode(X[:5000])).to(gpu))
    torch.cuda.synchronize(gpu)
    assert np.abs(p.cpu().numpy() - m.predict_proba(X[:5000])).max() < 2e-5


@pytest.mark.parametrize("exec_mode", ["launch", "persistent"])
def test_g20_rules_hot_swap_and_global_leaves(gpu, exec_mode):
    """The kernels' other G20 instantiations: proba-only routing rules (kR), a hot swap inside
    the live bin table, and a 70 x 8 ensemble whose 17920 leaves exceed both LDS stages (kGL)."""
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.models.gbdt import ObliviousGBDT
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel, DeviceRules
    from ccfd_demo_summit_amd.router.rules import RuleSet
    B = 8192
    X, _ = generate(B * 3, seed=58)
    # rules
    m = _model(12, X[:20000], rate=0.05)
    dm = DeviceModel(m, gpu, bins="g20")
    rs = RuleSet.parse("when proba >= 0.8 then fraud\nwhen proba < 0.001 then fraud\notherwise standard")
    eng = StreamEngine(dm, batch=B, depth=3, streams=1, exec_mode=exec_mode, rules=DeviceRules(rs, gpu))
    log = PartitionLog.from_arrays(X, ids=np.arange(X.shape[0], dtype=np.uint64), bins=dm.bins)
    eng.add_log(0, log)
    st = eng.pump(3)
    p = m.predict_proba(X)
    want = rs.evaluate(p).astype(bool)
    got = np.zeros(len(X), bool)
    got[eng.drain_flagged()["tx_id"].astype(np.int64)] = True
    clear = (np.abs(p - 0.8) > 1e-5) & (np.abs(p - 0.001) > 1e-6)
    np.testing.assert_array_equal(got[clear], want[clear])
    assert st.fraud_rows == got.sum() and st.rows == len(X)
    # hot swap: a permuted, rescaled ensemble packed against the live table
    perm = np.random.default_rng(0).permutation(m.n_trees)
    m2 = ObliviousGBDT(m.feat[perm], m.thr[perm], (m.leaves[perm] * 1.5).astype(np.float32), m.base)
    eng.swap_model(DeviceModel(m2, gpu, bins=dm.bins))
    p2, _ = eng.score(X[:2000])
    assert np.abs(p2 - m2.predict_proba(X[:2000])).max() < 1e-5
    eng.close()
    log.free()
    # leaves gathered from global memory
    big = build_model("gbdt", seed=13, X_ref=X[:20000], gbdt_trees=70, gbdt_depth=8, calibrate_rate=0.02)
    assert big.bin_spec().fits_g20 and big.n_trees * (1 << big.depth) > 16384
    dmb = DeviceModel(big, gpu, bins="g20")
    eng = StreamEngine(dmb, batch=B, depth=3, streams=1, exec_mode=exec_mode)
    log = PartitionLog.from_arrays(X, ids=np.arange(X.shape[0], dtype=np.uint64) + 7, bins=dmb.bins)
    eng.add_log(0, log)
    n = 2 * B + 1234
    assert eng.pump(2).rows + eng.pump(1, batch_rows=1234).rows == n
    fl = eng.drain_flagged()
    got = np.zeros(n, bool)
    got[(fl["tx_id"] - 7).astype(np.int64)] = True
    np.testing.assert_array_equal(got, big.predict_proba(X[:n]) >= 0.5)
    eng.close()
    log.free()


@pytest.mark.parametrize("fmt", ["g20", "g32"])
@pytest.mark.parametrize("item_rows", [256, 512])
def test_persistent_item_sizes_exact(gpu, monkeypatch, fmt, item_rows):
    """The persistent G20 / G32 kernel at 256- and 512-row items: full, partial and
    back-to-back micro-batches over several pump calls (the kernel halts and relaunches
    between them), every row once, proba per row exact (scored ring), counters and
    histograms exact.  (Round 4 also measured a two-item prefetch pipeline here: 2.30 vs
    2.51 x 10^9 tx/s, removed -- profiles/r4/g20/item_prefetch/.)"""
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    monkeypatch.setenv("CCFD_PERSIST_ITEM_ROWS", str(item_rows))
    B = 65536
    X, _ = generate(B * 4 + 5000, seed=59)
    m = _model(14, X[:20000], rate=0.05)
    dm = DeviceModel(m, gpu, bins=fmt)
    eng = StreamEngine(dm, batch=B, depth=4, streams=1, exec_mode="persistent")
    eng.enable_scored(X.shape[0])
    log = PartitionLog.from_arrays(X, ids=np.arange(X.shape[0], dtype=np.uint64), bins=dm.bins)
    eng.add_log(0, log)
    n = 1301 + 3 * B + 2 * 1303
    got_rows = eng.pump(1, batch_rows=1301).rows + eng.pump(3).rows + eng.pump(2, batch_rows=1303).rows
    assert got_rows == n
    rec = eng.drain_scored()
    ids = rec["tx_id"].astype(np.int64)
    np.testing.assert_array_equal(np.sort(ids), np.arange(n))
    pr = m.predict_proba(X[ids])
    assert np.abs(rec["proba"] - pr).max() < 2e-5
    np.testing.assert_array_equal(rec["route"] == 1, pr >= 0.5)
    side = torch.cuda.Stream(gpu)
    c = eng.flip_epoch(side)
    side.synchronize()
    c = c.cpu().numpy()
    assert c[0] == n and c[1] == (pr >= 0.5).sum() and c[4] == 0
    assert int(c[8:22].sum() + c[24:38].sum()) == n
    eng.close()
    log.free()
