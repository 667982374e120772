"""GPU scorer behind predict(): the dynamic micro-batcher coalesces concurrent batch=1
requests into single fused-kernel launches on the MI355X."""
import asyncio

import numpy as np
import pytest
from aiohttp.test_utils import TestClient, TestServer

from ccfd_demo_summit_amd.contracts import seldon
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import build_model

pytestmark = pytest.mark.gpu


def test_gpu_scorer_predict_server(gpu):
    from ccfd_demo_summit_amd.serving import GpuScorer
    from ccfd_demo_summit_amd.serving.seldon_server import SeldonServer
    X, _ = generate(5000, seed=6)
    m = build_model("mlp", seed=2, X_ref=X)
    sc = GpuScorer(m, 0.5, max_batch=1024)
    p, r = sc.score(X)                       # > max_batch: split into several launches
    assert np.abs(p - m.predict_proba(X)).max() < 1e-2

    async def go():
        srv = SeldonServer(sc, max_batch=256, max_delay_us=3000)
        async with TestClient(TestServer(srv.app)) as cl:
            rs = await asyncio.gather(*[cl.post("/api/v0.1/predictions", json=seldon.build_request(X[i:i + 1]))
                                        for i in range(64)])
            got = np.array([seldon.proba1_from_response(await q.json())[0] for q in rs])
            assert np.abs(got - m.predict_proba(X[:64])).max() < 1e-2
            assert srv.batcher.launches < 64
    asyncio.new_event_loop().run_until_complete(go())
    sc.close()


def test_native_seldon_server_scores_on_gpu():
    """The C++ REST front end calls the GPU engine directly (no Python on the request path):
    responses equal the fp32 model within bf16 tolerance; concurrent requests are batched."""
    import http.client
    import json

    from ccfd_demo_summit_amd.contracts import seldon
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.serving.native_seldon import NativeSeldonServer, http_load
    from ccfd_demo_summit_amd.serving.scorers import GpuScorer
    X, _ = generate(20_000, seed=9)
    m = build_model("mlp", seed=2, X_ref=X, calibrate_rate=0.02)
    sc = GpuScorer(m, 0.5, max_batch=4096)
    srv = NativeSeldonServer(sc, "127.0.0.1", 0)
    try:
        c = http.client.HTTPConnection("127.0.0.1", srv.port, timeout=30)
        c.request("POST", "/api/v0.1/predictions", body=json.dumps(seldon.build_request(X[:257])),
                  headers={"Content-Type": "application/json"})
        r = c.getresponse()
        assert r.status == 200
        p = seldon.proba1_from_response(json.loads(r.read()))
        assert np.abs(p - m.predict_proba(X[:257])).max() < 1e-2
        c.close()
        res = http_load("127.0.0.1", srv.port, json.dumps(seldon.build_request(X[:1])).encode(), conns=32, seconds=1.0)
        assert res["errors"] == 0 and res["requests"] > 100
        st = srv.stats()
        assert st["rows"] > st["batches"]
    finally:
        srv.stop()
        sc.close()
