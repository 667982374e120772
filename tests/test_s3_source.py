"""Producer S3 source (reference: Ceph RGW bucket ``ccdata``, key
``OPEN/uploaded/creditcard.csv``, secret ``keysecret``; ProducerDeployment.yaml:78-95)
against a local fake RGW on 127.0.0.1 that checks the SigV4 request shape and recomputes
the signature from the canonical request it actually received."""
import hashlib
import hmac
import http.server
import io
import threading

import numpy as np

from ccfd_demo_summit_amd.contracts import TxBatch
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.data.csv_source import write_creditcard_csv
from ccfd_demo_summit_amd.ingest.broker import InProcBroker
from ccfd_demo_summit_amd.ingest.producer import ProducerConfig, TransactionProducer

ACCESS, SECRET = "AKIDEXAMPLE", "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY"


def _expected_sig(method, path, headers, region="us-east-1"):
    amz_date = headers["x-amz-date"]
    date = amz_date[:8]
    signed = "host;x-amz-content-sha256;x-amz-date"
    canonical = "\n".join([method, path, "", f"host:{headers['host']}",
                           f"x-amz-content-sha256:{headers['x-amz-content-sha256']}", f"x-amz-date:{amz_date}", "",
                           signed, headers["x-amz-content-sha256"]])
    scope = f"{date}/{region}/s3/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canonical.encode()).hexdigest()])
    k = ("AWS4" + SECRET).encode()
    for part in (date, region, "s3", "aws4_request"):
        k = hmac.new(k, part.encode(), hashlib.sha256).digest()
    return hmac.new(k, sts.encode(), hashlib.sha256).hexdigest(), scope


def test_producer_replays_csv_from_s3(tmp_path):
    X, y = generate(700, seed=3, fraud_rate=0.05)
    p = tmp_path / "creditcard.csv"
    write_creditcard_csv(str(p), X, y)
    body = p.read_bytes()
    seen = []

    class RGW(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            h = {k.lower(): v for k, v in self.headers.items()}
            sig, scope = _expected_sig("GET", self.path, h)
            auth = h.get("authorization", "")
            ok = (self.path == "/ccdata/OPEN/uploaded/creditcard.csv"
                  and auth == f"AWS4-HMAC-SHA256 Credential={ACCESS}/{scope}, "
                              f"SignedHeaders=host;x-amz-content-sha256;x-amz-date, Signature={sig}")
            seen.append(ok)
            self.send_response(200 if ok else 403)
            self.end_headers()
            if ok:
                self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = http.server.HTTPServer(("127.0.0.1", 0), RGW)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        env = {"s3endpoint": f"127.0.0.1:{srv.server_port}", "s3bucket": "ccdata",
               "filename": "OPEN/uploaded/creditcard.csv", "ACCESS_KEY_ID": ACCESS, "SECRET_ACCESS_KEY": SECRET}
        import ccfd_demo_summit_amd.ingest.s3 as s3mod
        import os
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            cfg = ProducerConfig.from_env()
            assert cfg.source == "s3"
            cfg.fmt, cfg.batch = "txb1", 256
            broker = InProcBroker(default_partitions=1)
            prod = TransactionProducer(broker, cfg)
            assert prod.produce(700) == 700
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        assert seen == [True]
        recs = broker.fetch("odh-demo", 0, 0, 100)
        got = np.concatenate([TxBatch.decode(r.value).features for r in recs])
        np.testing.assert_allclose(got, X, rtol=1e-6)
    finally:
        srv.shutdown()


def _expected_sig_q(method, path, query, headers, region="us-east-1"):
    """SigV4 over the canonical request the fake RGW received (query string included)."""
    import urllib.parse
    amz_date = headers["x-amz-date"]
    date = amz_date[:8]
    q = urllib.parse.parse_qsl(query, keep_blank_values=True)
    cq = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}" for k, v in sorted(q))
    canonical = "\n".join([method, path, cq, f"host:{headers['host']}",
                           f"x-amz-content-sha256:{headers['x-amz-content-sha256']}", f"x-amz-date:{amz_date}", "",
                           "host;x-amz-content-sha256;x-amz-date", headers["x-amz-content-sha256"]])
    scope = f"{date}/{region}/s3/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canonical.encode()).hexdigest()])
    k = ("AWS4" + SECRET).encode()
    for part in (date, region, "s3", "aws4_request"):
        k = hmac.new(k, part.encode(), hashlib.sha256).digest()
    return (f"AWS4-HMAC-SHA256 Credential={ACCESS}/{scope}, SignedHeaders=host;x-amz-content-sha256;x-amz-date, "
            f"Signature={hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()}")


def test_upload_cli_then_producer_reads_it_back(tmp_path, monkeypatch, capsys):
    """The reference's data-loading step (README.md:319-343, ``aws s3 cp``) with our client:
    bucket create + signed-payload PUT + paginated ListObjectsV2 against a fake RGW that
    verifies every signature and payload hash; the producer then replays the uploaded CSV."""
    import urllib.parse
    from ccfd_demo_summit_amd.ingest import s3 as s3mod
    store, buckets = {}, set()

    class RGW(http.server.BaseHTTPRequestHandler):
        def _auth(self, method, body=b""):
            u = urllib.parse.urlsplit(self.path)
            h = {k.lower(): v for k, v in self.headers.items()}
            ok = (h.get("authorization") == _expected_sig_q(method, u.path, u.query, h)
                  and h["x-amz-content-sha256"] == hashlib.sha256(body).hexdigest())
            if not ok:
                self.send_response(403)
                self.end_headers()
            return ok, urllib.parse.unquote(u.path), dict(urllib.parse.parse_qsl(u.query))

        def do_PUT(self):
            body = self.rfile.read(int(self.headers.get("Content-Length") or 0))
            ok, path, _ = self._auth("PUT", body)
            if not ok:
                return
            parts = path.strip("/").split("/", 1)
            if len(parts) == 1:
                code = 409 if parts[0] in buckets else 200
                buckets.add(parts[0])
            else:
                code = 200 if parts[0] in buckets else 404
                if code == 200:
                    store[(parts[0], parts[1])] = body
            self.send_response(code)
            self.end_headers()

        def do_GET(self):
            ok, path, q = self._auth("GET")
            if not ok:
                return
            parts = path.strip("/").split("/", 1)
            if len(parts) == 2:
                body = store.get((parts[0], parts[1]))
                self.send_response(200 if body is not None else 404)
                self.end_headers()
                self.wfile.write(body or b"")
                return
            keys = sorted(k for b, k in store if b == parts[0] and k.startswith(q.get("prefix", "")))
            start = int(q.get("continuation-token", "0"))
            page = keys[start:start + 2]                       # tiny pages: exercise pagination
            more = start + 2 < len(keys)
            xml = ('<?xml version="1.0"?><ListBucketResult xmlns="http://s3.amazonaws.com/doc/2006-03-01/">'
                   + "".join(f"<Contents><Key>{k}</Key><Size>{len(store[(parts[0], k)])}</Size></Contents>"
                             for k in page)
                   + f"<IsTruncated>{'true' if more else 'false'}</IsTruncated>"
                   + (f"<NextContinuationToken>{start + 2}</NextContinuationToken>" if more else "")
                   + "</ListBucketResult>")
            self.send_response(200)
            self.end_headers()
            self.wfile.write(xml.encode())

        def log_message(self, *a):
            pass

    srv = http.server.HTTPServer(("127.0.0.1", 0), RGW)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        X, y = generate(500, seed=5, fraud_rate=0.05)
        p = tmp_path / "creditcard.csv"
        write_creditcard_csv(str(p), X, y)
        ep = f"127.0.0.1:{srv.server_port}"
        for k, v in {"s3endpoint": ep, "s3bucket": "ccdata", "filename": "OPEN/uploaded/creditcard.csv",
                     "ACCESS_KEY_ID": ACCESS, "SECRET_ACCESS_KEY": SECRET}.items():
            monkeypatch.setenv(k, v)
        assert s3mod.main(["upload", str(p)]) == 0
        assert s3mod.main(["upload", str(p), "--key", "OPEN/uploaded/copy one.csv"]) == 0   # bucket exists: 409 ok
        for i in range(3):
            s3mod.put_object(ep, "ccdata", f"OPEN/extra/{i}.bin", bytes([i]) * (i + 1), ACCESS, SECRET)
        listing = s3mod.list_objects(ep, "ccdata", ACCESS, SECRET, prefix="OPEN/")
        assert [k for k, _ in listing] == sorted(k for _, k in store) and len(listing) == 5
        assert dict(listing)["OPEN/extra/2.bin"] == 3
        assert store[("ccdata", "OPEN/uploaded/creditcard.csv")] == p.read_bytes()
        capsys.readouterr()
        s3mod.main(["ls", "--prefix", "OPEN/uploaded/"])
        assert "copy one.csv" in capsys.readouterr().out
        Xr, yr = s3mod.fetch_creditcard_from_env()
        np.testing.assert_allclose(Xr, X, rtol=1e-6)
        np.testing.assert_array_equal(yr, y)
    finally:
        srv.shutdown()
