"""Seldon gRPC Predict (seldon.protos.Seldon / seldon.protos.Model) on the CPU scorer:
tensor and ndarray payloads, named-column reordering, auth and bad-input status codes."""
import asyncio
import threading

import grpc
import numpy as np
import pytest
from google.protobuf import json_format

from ccfd_demo_summit_amd.contracts import FEATURE_NAMES
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import build_model
from ccfd_demo_summit_amd.serving.scorers import CpuScorer
from ccfd_demo_summit_amd.serving.seldon_grpc import (SeldonGrpcClient, SeldonGrpcServer, SeldonMessage,
                                                      matrix_request, response_proba1)


@pytest.fixture(scope="module")
def served():
    X, _ = generate(2000, seed=4)
    m = build_model("mlp", seed=1, X_ref=X)
    loop = asyncio.new_event_loop()
    srv = SeldonGrpcServer(CpuScorer(m), token="s3cret", max_batch=256, max_delay_us=500)
    port = loop.run_until_complete(srv.start("127.0.0.1", 0))
    th = threading.Thread(target=loop.run_forever, daemon=True)
    th.start()
    yield m, X, port
    asyncio.run_coroutine_threadsafe(srv.stop(), loop).result(10)
    loop.call_soon_threadsafe(loop.stop)


def test_tensor_roundtrip_both_services(served):
    m, X, port = served
    for svc in ("seldon.protos.Seldon", "seldon.protos.Model"):
        c = SeldonGrpcClient(f"127.0.0.1:{port}", token="s3cret", service=svc)
        np.testing.assert_allclose(c.predict(X[:33]), m.predict_proba(X[:33]), atol=1e-6)
        c.close()


def test_ndarray_and_reordered_names(served):
    m, X, port = served
    c = SeldonGrpcClient(f"127.0.0.1:{port}", token="s3cret")
    perm = np.random.default_rng(0).permutation(30)
    body = {"data": {"names": [FEATURE_NAMES[i] for i in perm], "ndarray": X[:5][:, perm].tolist()}}
    msg = json_format.ParseDict(body, SeldonMessage())
    np.testing.assert_allclose(response_proba1(c.predict_message(msg)), m.predict_proba(X[:5]), atol=1e-6)
    c.close()


def test_concurrent_calls_share_batches(served):
    m, X, port = served
    c = SeldonGrpcClient(f"127.0.0.1:{port}", token="s3cret")
    futs = [c._call.future(matrix_request(X[i:i + 1]), metadata=c.md) for i in range(64)]
    got = np.concatenate([response_proba1(f.result()) for f in futs])
    np.testing.assert_allclose(got, m.predict_proba(X[:64]), atol=1e-6)
    c.close()


def test_errors(served):
    _, X, port = served
    bad = SeldonGrpcClient(f"127.0.0.1:{port}", token="wrong")
    with pytest.raises(grpc.RpcError) as ei:
        bad.predict(X[:1])
    assert ei.value.code() == grpc.StatusCode.UNAUTHENTICATED
    bad.close()
    c = SeldonGrpcClient(f"127.0.0.1:{port}", token="s3cret")
    r = c.predict_message(matrix_request(X[:2, :10], names=FEATURE_NAMES[:10]))
    assert r.status.code == 400
    c.close()
