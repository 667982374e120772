"""REST surfaces: Seldon predict() (all request shapes, batching, auth, metrics) and the
KIE-compatible process API -- exercised over real HTTP on 127.0.0.1."""
import asyncio
import json

import numpy as np
import pytest
from aiohttp.test_utils import TestClient, TestServer

from ccfd_demo_summit_amd.contracts import seldon
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.metrics import KieMetrics
from ccfd_demo_summit_amd.models import build_model
from ccfd_demo_summit_amd.process import PredictionService, ProcessEngine
from ccfd_demo_summit_amd.process.kie_server import BASE, KieServer
from ccfd_demo_summit_amd.serving import CpuScorer
from ccfd_demo_summit_amd.serving.seldon_server import SeldonServer, usertask_server


@pytest.fixture(scope="module")
def model_and_X():
    X, _ = generate(2000, seed=2)
    return build_model("lr", seed=0, X_ref=X), X


def _run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


def test_seldon_predict_shapes_batching_auth(model_and_X):
    model, X = model_and_X

    async def go():
        srv = SeldonServer(CpuScorer(model), token="s3cret", max_batch=64, max_delay_us=2000)
        async with TestClient(TestServer(srv.app)) as cl:
            h = {"Authorization": "Bearer s3cret"}
            r = await cl.post("/api/v0.1/predictions", json=seldon.build_request(X[:3]), headers=h)
            assert r.status == 200
            body = await r.json()
            assert body["data"]["names"] == ["proba_0", "proba_1"]
            np.testing.assert_allclose(seldon.proba1_from_response(body), model.predict_proba(X[:3]), rtol=1e-5)
            # tensor form
            r = await cl.post("/predict", json=seldon.build_request(X[:2], tensor=True), headers=h)
            assert "tensor" in (await r.json())["data"]
            # legacy form-encoded json=
            r = await cl.post("/predict", data={"json": json.dumps(seldon.build_request(X[:1]))}, headers=h)
            assert r.status == 200
            # auth + bad input
            assert (await cl.post("/predict", json=seldon.build_request(X[:1]))).status == 401
            assert (await cl.post("/predict", data=b"{nope", headers=h)).status == 400
            assert (await cl.post("/predict", json={"data": {"ndarray": [[1, 2]]}}, headers=h)).status == 400
            # 32 concurrent batch=1 requests are coalesced into few launches
            before = srv.batcher.launches
            rs = await asyncio.gather(*[cl.post("/api/v0.1/predictions", json=seldon.build_request(X[i:i + 1]),
                                                headers=h) for i in range(32)])
            outs = [seldon.proba1_from_response(await r.json())[0] for r in rs]
            np.testing.assert_allclose(outs, model.predict_proba(X[:32]), rtol=1e-5)
            assert srv.batcher.launches - before < 32
            text = await (await cl.get("/prometheus")).text()
            assert "seldon_api_engine_server_requests_seconds_count" in text
            assert 'status="401"' in text and "proba_1 " in text and "V17 " in text
            assert (await cl.get("/health/ping")).status == 200
    _run(go())


def test_usertask_model_slot():
    async def go():
        srv = usertask_server()
        async with TestClient(TestServer(srv.app)) as cl:
            r = await cl.post("/predict", json={"data": {"names": ["proba_1", "log_amount"],
                                                         "ndarray": [[0.99, 9.9], [0.01, 1.0]]}})
            body = await r.json()
            assert body["data"]["names"] == ["approved", "rejected"]
            mat = np.asarray(body["data"]["ndarray"])
            assert mat.shape == (2, 2) and mat[0, 1] > 0.5 and mat[1, 0] > 0.5
    _run(go())


def test_kie_rest_lifecycle():
    async def go():
        sent = []
        eng = ProcessEngine(notification_timeout_s=0.05, publish_notification=sent.append,
                            kie_metrics=KieMetrics(), prediction=PredictionService(1.0))
        srv = KieServer(eng, tick_s=0.01)
        c = "ccd-fraud-kjar"
        async with TestClient(TestServer(srv.app)) as cl:
            r = await cl.post(f"{BASE}/containers/{c}/processes/ccd-fraud-kjar.CCDProcess/instances",
                              json={"transaction_id": 5, "customer_id": 9, "amount": 5000.0, "proba": 0.9})
            assert r.status == 201
            iid = await r.json()
            assert sent[0]["process_id"] == iid
            r = await cl.post(f"{BASE}/containers/{c}/processes/ccd-fraud-kjar.StandardProcess/instances",
                              json={"transaction_id": 6})
            assert r.status == 201
            assert (await cl.post(f"{BASE}/containers/other/processes/x/instances", json={})).status == 404
            await asyncio.sleep(0.2)                     # timer fires -> DMN -> user task
            tasks = (await (await cl.get(f"{BASE}/queries/tasks/instances/pot-owners")).json())["task-summary"]
            assert len(tasks) == 1 and tasks[0]["task-proc-inst-id"] == iid
            tid = tasks[0]["task-id"]
            assert (await cl.put(f"{BASE}/containers/{c}/tasks/{tid}/states/completed",
                                 json={"outcome": "approved"})).status == 201
            inst = await (await cl.get(f"{BASE}/containers/{c}/processes/instances/{iid}")).json()
            assert inst["outcome"] == "investigation_closed_legit"
            # signal on a completed instance is rejected
            r = await cl.post(f"{BASE}/containers/{c}/processes/instances/{iid}/signal/customerResponse", json=True)
            assert r.status == 404
            text = await (await cl.get("/rest/metrics")).text()
            assert "fraud_investigation_amount_count 1.0" in text
            # batch start (engine router hand-off): one request, idempotent per transaction id
            items = [{"transaction_id": 100 + i, "customer_id": i, "amount": 1.0, "proba": 0.9} for i in range(5)]
            r = await cl.post(f"{BASE}/containers/{c}/processes/ccd-fraud-kjar.CCDProcess/instances/batch", json=items)
            assert r.status == 201
            ids = await r.json()
            assert len(set(ids)) == 5
            r = await cl.post(f"{BASE}/containers/{c}/processes/ccd-fraud-kjar.CCDProcess/instances/batch",
                              json=items[:2])
            assert await r.json() == ids[:2]                 # duplicates return the same instances
    _run(go())
