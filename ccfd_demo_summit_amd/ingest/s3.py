"""Minimal S3 GET (AWS SigV4) for the reference's Ceph RGW dataset source
(README.md:136-343; ProducerDeployment.yaml:78-95: ``ACCESS_KEY_ID``, ``SECRET_ACCESS_KEY``,
``s3endpoint``, ``s3bucket``, ``filename``).  Optional: there is no network in CI."""
from __future__ import annotations

import datetime
import hashlib
import hmac
import io
import os
import urllib.request
from typing import Optional, Tuple

import numpy as np


def _sign(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def presign_headers(method: str, host: str, path: str, access_key: str, secret_key: str,
                    region: str = "us-east-1", now: Optional[datetime.datetime] = None) -> dict:
    now = now or datetime.datetime.now(datetime.timezone.utc)
    amz_date = now.strftime("%Y%m%dT%H%M%SZ")
    date = now.strftime("%Y%m%d")
    payload_hash = hashlib.sha256(b"").hexdigest()
    canonical = "\n".join([method, path, "", f"host:{host}", f"x-amz-content-sha256:{payload_hash}",
                           f"x-amz-date:{amz_date}", "", "host;x-amz-content-sha256;x-amz-date", payload_hash])
    scope = f"{date}/{region}/s3/aws4_request"
    to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canonical.encode()).hexdigest()])
    k = _sign(_sign(_sign(_sign(("AWS4" + secret_key).encode(), date), region), "s3"), "aws4_request")
    sig = hmac.new(k, to_sign.encode(), hashlib.sha256).hexdigest()
    return {"x-amz-date": amz_date, "x-amz-content-sha256": payload_hash,
            "Authorization": f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, "
                             f"SignedHeaders=host;x-amz-content-sha256;x-amz-date, Signature={sig}"}


def get_object(endpoint: str, bucket: str, key: str, access_key: str, secret_key: str, timeout: float = 30.0) -> bytes:
    scheme = "https" if endpoint.endswith(":443") or endpoint.startswith("https") else "http"
    host = endpoint.split("://")[-1]
    path = f"/{bucket}/{key}"
    req = urllib.request.Request(f"{scheme}://{host}{path}",
                                 headers=presign_headers("GET", host, path, access_key, secret_key))
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.read()


def fetch_creditcard_from_env(environ=None) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    e = os.environ if environ is None else environ
    raw = get_object(e["s3endpoint"], e.get("s3bucket", "ccdata"), e.get("filename", "OPEN/uploaded/creditcard.csv"),
                     e.get("ACCESS_KEY_ID", ""), e.get("SECRET_ACCESS_KEY", ""))
    import tempfile
    from ..data.csv_source import read_creditcard_csv
    with tempfile.NamedTemporaryFile("wb", suffix=".csv", delete=False) as f:
        f.write(raw)
        p = f.name
    try:
        return read_creditcard_csv(p)
    finally:
        os.unlink(p)
