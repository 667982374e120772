"""Configurable routing rules on the GPU (VERDICT r1 Next #5): a 3-rule set compiled to a
device program routes every row inside the fused kernels' epilogue exactly like
RuleSet.evaluate does on the host (same proba, same features as the kernel saw, float32 on
both sides) -- through the plain kernels (MLP / LR / GBDT, f32 and W64 rows), the streaming
engine (launch and persistent) and EngineService end to end."""
import time

import numpy as np
import pytest
import torch

from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import build_model
from ccfd_demo_summit_amd.router.rules import RuleSet, run_device_program

pytestmark = pytest.mark.gpu

RULES3 = """
when amount > 200 and proba >= 0.2 then fraud
when V17 < -2.5 or abs(V14) > 4 then fraud
otherwise standard
"""
RULES_ARITH = """
when log1p(max(amount, 0)) * proba > 0.9 then fraud
when -1 < V1 < -0.5 and not (V2 > 0) then standard
when (V10 + V12) / 2 < -1.5 then fraud
otherwise standard
"""


def _seen(X, wire):
    from ccfd_demo_summit_amd.contracts import decode_wire, encode_wire
    return decode_wire(encode_wire(X)) if wire else X


@pytest.mark.parametrize("kind,wire", [("mlp", False), ("mlp", True), ("lr", False), ("lr", True),
                                       ("gbdt", False)])
@pytest.mark.parametrize("n", [1, 31, 4097, 65536])
@pytest.mark.parametrize("text", [RULES3, RULES_ARITH])
def test_kernel_routes_equal_host_rules(gpu, kind, wire, n, text):
    from ccfd_demo_summit_amd.contracts import encode_wire
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel, DeviceRules, new_counters, score
    X, _ = generate(n, seed=11)
    m = build_model(kind, seed=2, X_ref=generate(20000, seed=3)[0], calibrate_rate=0.05)
    dm = DeviceModel(m, gpu, wire=wire)
    rs = RuleSet.parse(text)
    dr = DeviceRules(rs, gpu)
    xt = torch.from_numpy(encode_wire(X) if wire else X).to(gpu)
    cnt = new_counters(gpu)
    p, r = score(dm, xt, 0.5, counters=cnt, rules=dr)
    torch.cuda.synchronize(gpu)
    p, r = p.cpu().numpy(), r.cpu().numpy()
    Xs = _seen(X, wire)
    want = rs.evaluate(p, X=Xs)
    if "log1p" in text:            # libm vs device log1pf may differ by an ulp: allow only those rows
        ref = run_device_program(dr.ruleset.device_program(), p, Xs)
        np.testing.assert_array_equal(want, ref)
        assert (r != want).sum() <= max(1, n // 10000)
    else:
        np.testing.assert_array_equal(r, want)
    c = cnt.cpu().numpy()
    assert c[0] == n and c[1] == r.sum() and c[2] == n - r.sum()


@pytest.mark.parametrize("exec_mode,wire", [("launch", False), ("launch", True), ("persistent", True),
                                            ("persistent", False), ("persistent_pipe", True)])
def test_engine_routes_by_rules(gpu, monkeypatch, exec_mode, wire):
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel, DeviceRules
    X, _ = generate(4096 * 6, seed=12)
    m = build_model("mlp", seed=4, X_ref=X[:20000], calibrate_rate=0.05)
    rs = RuleSet.parse(RULES3)
    dm = DeviceModel(m, gpu, wire=wire)
    if exec_mode == "persistent_pipe":            # pipelined static items (score_persist.hip)
        monkeypatch.setenv("CCFD_PERSIST_PIPE", "1")
        exec_mode = "persistent"
    eng = StreamEngine(dm, batch=4096, depth=4, streams=2, input_mode="zerocopy", exec_mode=exec_mode,
                       rules=DeviceRules(rs, gpu))
    p, r = eng.score(X)
    want = rs.evaluate(p, X=_seen(X, wire))
    np.testing.assert_array_equal(r, want)
    log = PartitionLog.from_arrays(X, ids=np.arange(len(X), dtype=np.uint64), wire=wire)
    eng.add_log(0, log)
    st = eng.pump(6)
    fl = eng.drain_flagged()
    assert st.rows == len(X) and st.fraud_rows == len(fl) == want.sum()
    assert set(fl["tx_id"].tolist()) == set(np.nonzero(want)[0].tolist())
    eng.close()
    log.free()


@pytest.mark.parametrize("wire", [False, True])
def test_engine_service_routes_every_row_like_host_rules(gpu, wire):
    from ccfd_demo_summit_amd.contracts import TxBatch, encode_wire
    from ccfd_demo_summit_amd.ingest import InProcBroker
    from ccfd_demo_summit_amd.launch.engine_service import EngineService, EngineServiceConfig
    from ccfd_demo_summit_amd.metrics import MetricsHub
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel, score
    from ccfd_demo_summit_amd.parallel import DistContext
    from ccfd_demo_summit_amd.router import Router

    class Sink:
        def __init__(self):
            self.ids = []

        def start_fraud(self, d):
            self.ids.append(d["transaction_id"])

        def start_fraud_many(self, ds):
            self.ids.extend(d["transaction_id"] for d in ds)

    X, _ = generate(40_000, seed=13)
    ids = np.arange(len(X), dtype=np.uint64) + 10_000
    m = build_model("mlp", seed=5, X_ref=X[:20000], calibrate_rate=0.05)
    dm = DeviceModel(m, gpu, wire=wire)
    rs = RuleSet.parse(RULES3)
    broker = InProcBroker(default_partitions=2)
    broker.create_topic("odh-demo", 2)
    for k, s in enumerate(range(0, len(X), 2500)):
        b = TxBatch(ids=ids[s:s + 2500], customer=(ids[s:s + 2500] % 977).astype(np.uint32), features=X[s:s + 2500])
        broker.produce("odh-demo", b.encode(), partition=k % 2)
    sink = Sink()
    hub = MetricsHub()
    router = Router(rs, sink, hub.router)
    svc = EngineService(DistContext(0, 1, 0, gpu, "none"), dm, broker, router,
                        EngineServiceConfig(batch=4096, depth=4, streams=2, ring_rows=16384, flush_us=200,
                                            reduce_period_ms=1.0)).start()
    assert svc.device_rules is not None
    t0 = time.time()
    while svc.rows_scored < len(X) and time.time() - t0 < 60:
        svc.step()
    for _ in range(5):
        svc.step()
    svc.stop()
    assert svc.rows_scored == len(X)
    xt = torch.from_numpy(encode_wire(X) if wire else X).to(gpu)
    p, _ = score(dm, xt, 0.5)
    want = rs.evaluate(p.cpu().numpy(), X=_seen(X, wire))
    assert sorted(sink.ids) == sorted((ids[want.astype(bool)]).tolist())
    assert hub.router.tx_outgoing.labels(type="fraud")._value.get() == want.sum()
