"""Native Seldon REST front end (csrc/engine/seldon_http.cpp): the reference's predict()
contract (ndarray / tensor / named columns, Seldon error JSON, token auth), keep-alive,
dynamic batching, /prometheus with the reference metric names, and the native load
generator.  CPU: scoring goes through the ctypes scorer callback."""
import http.client
import json

import numpy as np
import pytest

from ccfd_demo_summit_amd.contracts import seldon
from ccfd_demo_summit_amd.contracts.transaction import FEATURE_NAMES
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import build_model
from ccfd_demo_summit_amd.serving import CpuScorer
from ccfd_demo_summit_amd.serving.native_seldon import NativeSeldonServer, http_load


@pytest.fixture(scope="module")
def srv():
    X, _ = generate(5000, seed=3)
    m = build_model("lr", seed=1, X_ref=X, calibrate_rate=0.05)
    s = NativeSeldonServer(CpuScorer(m), host="127.0.0.1", port=0)
    yield s, m, X
    s.stop()


def _post(port, body, path="/api/v0.1/predictions", headers=None, conn=None):
    c = conn or http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    c.request("POST", path, body=json.dumps(body) if not isinstance(body, (bytes, str)) else body,
              headers={"Content-Type": "application/json", **(headers or {})})
    r = c.getresponse()
    out = r.status, json.loads(r.read())
    if conn is None:
        c.close()
    return out


def test_predict_ndarray_tensor_and_named_columns(srv):
    s, m, X = srv
    ref = m.predict_proba(X[:5])
    st, body = _post(s.port, seldon.build_request(X[:5]))
    assert st == 200 and body["data"]["names"] == ["proba_0", "proba_1"]
    np.testing.assert_allclose(seldon.proba1_from_response(body), ref, rtol=1e-6, atol=1e-7)
    assert "puid" in body["meta"] and body["meta"]["requestPath"] == {"modelfull": "modelfull"}
    st, body = _post(s.port, seldon.build_request(X[:3], tensor=True), path="/predict")
    assert st == 200 and body["data"]["tensor"]["shape"] == [3, 2]
    np.testing.assert_allclose(seldon.proba1_from_response(body), ref[:3], rtol=1e-6, atol=1e-7)
    # columns sent in another order are re-ordered by name
    perm = np.random.default_rng(0).permutation(30)
    req = {"data": {"names": [FEATURE_NAMES[i] for i in perm], "ndarray": X[:4, perm].tolist()}}
    st, body = _post(s.port, req)
    np.testing.assert_allclose(seldon.proba1_from_response(body), ref[:4], rtol=1e-6, atol=1e-7)
    # a flat single row
    st, body = _post(s.port, {"data": {"ndarray": X[0].tolist()}})
    assert st == 200 and len(body["data"]["ndarray"]) == 1


def test_errors_keepalive_metrics_and_health(srv):
    s, m, X = srv
    before = s.stats()
    st, body = _post(s.port, b"{not json")
    assert st == 400 and body["status"]["status"] == "FAILURE"
    st, body = _post(s.port, {"data": {"ndarray": [[1.0, 2.0]]}})
    assert st == 400 and "30 features" in body["status"]["info"]
    c = http.client.HTTPConnection("127.0.0.1", s.port, timeout=10)
    for i in range(5):                              # one keep-alive connection
        st, body = _post(s.port, seldon.build_request(X[i:i + 1]), conn=c)
        assert st == 200
    c.request("GET", "/prometheus")
    text = c.getresponse().read().decode()
    c.request("GET", "/health/ping")
    assert json.loads(c.getresponse().read())["server"] == "native"
    c.close()
    assert 'seldon_api_engine_server_requests_seconds_count{status="200"}' in text
    assert 'seldon_api_engine_client_requests_seconds_bucket{' in text
    assert "proba_1 " in text and "Amount " in text
    st_ = s.stats()
    assert st_["count"]["400"] - before["count"]["400"] == 2
    assert st_["count"]["200"] - before["count"]["200"] == 5 and st_["rows"] - before["rows"] == 5


def test_token_and_native_load_generator():
    X, _ = generate(2000, seed=4)
    m = build_model("lr", seed=2, X_ref=X)
    s = NativeSeldonServer(CpuScorer(m), host="127.0.0.1", port=0, token="s3cret")
    try:
        assert _post(s.port, seldon.build_request(X[:1]))[0] == 401
        assert _post(s.port, seldon.build_request(X[:1]), headers={"Authorization": "Bearer s3cret"})[0] == 200
    finally:
        s.stop()
    s = NativeSeldonServer(CpuScorer(m), host="127.0.0.1", port=0)
    try:
        r = http_load("127.0.0.1", s.port, json.dumps(seldon.build_request(X[:1])).encode(), conns=8, seconds=0.5)
        assert r["requests"] > 50 and r["errors"] == 0
        assert s.stats()["batches"] < s.stats()["rows"]          # concurrent requests were batched
    finally:
        s.stop()


def test_multi_worker_server_shares_port_and_stats():
    X, _ = generate(2000, seed=5)
    m = build_model("lr", seed=3, X_ref=X)
    s = NativeSeldonServer(CpuScorer(m), host="127.0.0.1", port=0, workers=3)
    try:
        r = http_load("127.0.0.1", s.port, json.dumps(seldon.build_request(X[:2])).encode(), conns=12,
                      seconds=0.5, threads=3)
        assert r["errors"] == 0 and r["requests"] > 30
        assert s.stats()["count"]["200"] >= r["requests"]
        st, body = _post(s.port, seldon.build_request(X[:3]))
        np.testing.assert_allclose(seldon.proba1_from_response(body), m.predict_proba(X[:3]), rtol=1e-6, atol=1e-7)
    finally:
        s.stop()


def test_native_seldon_parser_and_server_under_asan(tmp_path):
    """Host ASan+UBSan build: the Seldon JSON parser on mutated bodies, and the live server on
    garbage, truncated, oversized and pipelined requests over raw sockets."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    from ccfd_demo_summit_amd.ops.build import asan_runtime, build
    try:
        build(sanitize="address,undefined", verbose=False)
        rt = asan_runtime()
    except Exception as e:
        pytest.skip(f"sanitizer build unavailable: {e}")
    if not rt or not os.path.exists(rt):
        pytest.skip("clang ASan runtime not found")
    script = tmp_path / "asan_seldon.py"
    script.write_text(
        "import ctypes as C, json, socket, numpy as np\n"
        "from ccfd_demo_summit_amd.ops._lib import lib\n"
        "from ccfd_demo_summit_amd.contracts import seldon\n"
        "from ccfd_demo_summit_amd.data import generate\n"
        "from ccfd_demo_summit_amd.models import build_model\n"
        "from ccfd_demo_summit_amd.serving import CpuScorer\n"
        "from ccfd_demo_summit_amd.serving.native_seldon import NativeSeldonServer\n"
        "L = lib(); assert 'address' in L._name\n"
        "L.ccfd_seldon_parse_fuzz.restype = C.c_int64\n"
        "L.ccfd_seldon_parse_fuzz.argtypes = [C.c_char_p, C.c_int64, C.c_void_p, C.c_int64]\n"
        "X, _ = generate(64, seed=1)\n"
        "good = [json.dumps(seldon.build_request(X[:3])).encode(), json.dumps(seldon.build_request(X[:2], tensor=True)).encode(),\n"
        "        json.dumps({'data': {'ndarray': X[0].tolist()}}).encode()]\n"
        "out = np.zeros((8, 30), np.float32)\n"
        "assert L.ccfd_seldon_parse_fuzz(good[0], len(good[0]), out.ctypes.data, 8) == 3\n"
        "r = np.random.default_rng(2)\n"
        "for it in range(4000):\n"
        "    b = bytearray(good[it % 3])\n"
        "    for _ in range(int(r.integers(1, 6))): b[int(r.integers(0, len(b)))] = int(r.integers(0, 256))\n"
        "    b = bytes(b[:int(r.integers(0, len(b) + 1))]) if it % 2 else bytes(b)\n"
        "    L.ccfd_seldon_parse_fuzz(b, len(b), out.ctypes.data, 8)\n"
        "    L.ccfd_seldon_parse_fuzz(b'[' * 200 + b'{' * 200, 400, out.ctypes.data, 8)\n"
        "m = build_model('lr', seed=1, X_ref=X)\n"
        "srv = NativeSeldonServer(CpuScorer(m), host='127.0.0.1', port=0, workers=2)\n"
        "def send(raw, read=True):\n"
        "    s = socket.create_connection(('127.0.0.1', srv.port), timeout=5)\n"
        "    s.sendall(raw)\n"
        "    data = b''\n"
        "    if read:\n"
        "        s.shutdown(socket.SHUT_WR)\n"
        "        try:\n"
        "            while True:\n"
        "                d = s.recv(65536)\n"
        "                if not d: break\n"
        "                data += d\n"
        "        except socket.timeout: pass\n"
        "    s.close(); return data\n"
        "req = lambda body: b'POST /api/v0.1/predictions HTTP/1.1\\r\\nContent-Length: %d\\r\\n\\r\\n' % len(body) + body\n"
        "assert b'200 OK' in send(req(good[0]))\n"
        "assert send(req(good[0]) * 5).count(b'200 OK') == 5\n"
        "assert b'413' in send(b'POST /predict HTTP/1.1\\r\\nContent-Length: 999999999999\\r\\n\\r\\n')\n"
        "for it in range(300):\n"
        "    b = bytearray(req(good[it % 3]))\n"
        "    for _ in range(int(r.integers(1, 6))): b[int(r.integers(0, len(b)))] = int(r.integers(0, 256))\n"
        "    send(bytes(b[:int(r.integers(0, len(b) + 1))]), read=(it % 4 == 0))\n"
        "    send(bytes(r.integers(0, 256, int(r.integers(0, 2000)), dtype=np.uint8)), read=False)\n"
        "assert b'200 OK' in send(req(good[1]))\n"
        "z = json.dumps({'data': {'tensor': {'shape': [0, 30], 'values': []}}}).encode()\n"
        "for _ in range(3): assert b'200 OK' in send(req(z))\n"
        "assert send(req(z) + req(good[0]) + req(z)).count(b'200 OK') == 3\n"
        "srv.stop()\n"
        "print('asan seldon ok')\n")
    env = dict(os.environ, CCFD_SANITIZE="address,undefined", LD_PRELOAD=rt, CCFD_NO_AUTOBUILD="1",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               PYTHONPATH=str(Path(__file__).resolve().parents[1]), HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "asan seldon ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def _raw(port, raw):
    import socket
    s = socket.create_connection(("127.0.0.1", port), timeout=10)
    s.sendall(raw)
    s.shutdown(socket.SHUT_WR)
    data = b""
    while True:
        d = s.recv(65536)
        if not d:
            break
        data += d
    s.close()
    return data


def _req(body: bytes, path=b"/api/v0.1/predictions"):
    return b"POST " + path + b" HTTP/1.1\r\nContent-Length: %d\r\n\r\n" % len(body) + body


def test_zero_row_requests(srv):
    """a [0,30] tensor / empty ndarray is answered with an empty result
    instead of reading past the scored rows."""
    s, m, X = srv
    st, body = _post(s.port, {"data": {"tensor": {"shape": [0, 30], "values": []}}})
    assert st == 200 and body["data"]["tensor"]["shape"] == [0, 2] and body["data"]["tensor"]["values"] == []
    # a zero-row request batched together with real ones
    z = json.dumps({"data": {"tensor": {"shape": [0, 30], "values": []}}}).encode()
    g = json.dumps(seldon.build_request(X[:2])).encode()
    out = _raw(s.port, _req(z) + _req(g) + _req(z))
    assert out.count(b"200 OK") == 3
    st, body = _post(s.port, seldon.build_request(X[:1]))
    assert st == 200


def test_pipelined_responses_keep_request_order(srv):
    """POST predict then GET ping on one connection -- the predict's
    response comes first (HTTP/1.1 pipelining pairs responses by order)."""
    s, m, X = srv
    g = json.dumps(seldon.build_request(X[:3])).encode()
    ping = b"GET /health/ping HTTP/1.1\r\n\r\n"
    bad = _req(b"{nope")
    out = _raw(s.port, _req(g) + ping + _req(g) + bad + ping + _req(g))
    heads = [blk.split(b"\r\n", 1)[0] for blk in out.split(b"HTTP/1.1 ")[1:]]
    assert heads == [b"200 OK", b"200 OK", b"200 OK", b"400 Bad Request", b"200 OK", b"200 OK"], heads
    bodies = [blk.split(b"\r\n\r\n", 1)[1] for blk in out.split(b"HTTP/1.1 ")[1:]]
    assert b"proba_1" in bodies[0] and b"native" in bodies[1] and b"proba_1" in bodies[2]
    assert b"FAILURE" in bodies[3] and b"native" in bodies[4] and b"proba_1" in bodies[5]


def test_scoring_failure_is_a_5xx():
    """a scorer failure answers 500 Internal Server Error and is counted in
    the 5xx bucket, not as a client error."""
    class Boom:
        def score(self, X):
            raise RuntimeError("device lost")
    s = NativeSeldonServer(Boom(), host="127.0.0.1", port=0)
    try:
        X, _ = generate(4, seed=1)
        out = _raw(s.port, _req(json.dumps(seldon.build_request(X[:2])).encode()))
        assert out.startswith(b"HTTP/1.1 500 Internal Server Error")
        st = s.stats()
        assert st["count"]["500"] == 1 and st["count"]["400"] == 0
        assert b'status="500"' in s.expose()
    finally:
        s.stop()
