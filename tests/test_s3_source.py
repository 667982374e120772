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
