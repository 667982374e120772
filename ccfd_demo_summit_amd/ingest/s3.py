"""Minimal S3 client (AWS SigV4) for the reference's Ceph RGW dataset source
(README.md:136-343; ProducerDeployment.yaml:78-95: ``ACCESS_KEY_ID``, ``SECRET_ACCESS_KEY``,
``s3endpoint``, ``s3bucket``, ``filename``): GET for the producer, and bucket create / PUT /
list for the data-loading step the reference does with ``aws s3 cp`` (README.md:319-343):

    python -m ccfd_demo_summit_amd.ingest.s3 upload creditcard.csv [--bucket ccdata]
        [--key OPEN/uploaded/creditcard.csv]     # endpoint / keys from the producer's env keys
    python -m ccfd_demo_summit_amd.ingest.s3 ls [--bucket ccdata] [--prefix OPEN/]

Optional: there is no network in CI (tests run it against a signature-checking fake RGW)."""
from __future__ import annotations

import datetime
import hashlib
import hmac
import os
import urllib.error
import urllib.parse
import urllib.request
import xml.etree.ElementTree as ET
from typing import Dict, List, Optional, Tuple

import numpy as np


def _sign(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def _canonical_query(query: Optional[Dict[str, str]]) -> str:
    return "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(str(v), safe='-_.~')}"
                    for k, v in sorted((query or {}).items()))


def presign_headers(method: str, host: str, path: str, access_key: str, secret_key: str,
                    region: str = "us-east-1", now: Optional[datetime.datetime] = None,
                    payload: bytes = b"", query: Optional[Dict[str, str]] = None) -> dict:
    now = now or datetime.datetime.now(datetime.timezone.utc)
    amz_date = now.strftime("%Y%m%dT%H%M%SZ")
    date = now.strftime("%Y%m%d")
    payload_hash = hashlib.sha256(payload).hexdigest()
    canonical = "\n".join([method, path, _canonical_query(query), f"host:{host}",
                           f"x-amz-content-sha256:{payload_hash}", f"x-amz-date:{amz_date}", "",
                           "host;x-amz-content-sha256;x-amz-date", payload_hash])
    scope = f"{date}/{region}/s3/aws4_request"
    to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canonical.encode()).hexdigest()])
    k = _sign(_sign(_sign(_sign(("AWS4" + secret_key).encode(), date), region), "s3"), "aws4_request")
    sig = hmac.new(k, to_sign.encode(), hashlib.sha256).hexdigest()
    return {"x-amz-date": amz_date, "x-amz-content-sha256": payload_hash,
            "Authorization": f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, "
                             f"SignedHeaders=host;x-amz-content-sha256;x-amz-date, Signature={sig}"}


def _request(method: str, endpoint: str, path: str, access_key: str, secret_key: str, body: bytes = b"",
             query: Optional[Dict[str, str]] = None, timeout: float = 30.0) -> bytes:
    scheme = "https" if endpoint.endswith(":443") or endpoint.startswith("https") else "http"
    host = endpoint.split("://")[-1]
    path = urllib.parse.quote(path, safe="/-_.~")
    url = f"{scheme}://{host}{path}" + (f"?{_canonical_query(query)}" if query else "")
    hdr = presign_headers(method, host, path, access_key, secret_key, payload=body, query=query)
    req = urllib.request.Request(url, data=body if method == "PUT" else None, method=method, headers=hdr)
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.read()


def get_object(endpoint: str, bucket: str, key: str, access_key: str, secret_key: str, timeout: float = 30.0) -> bytes:
    return _request("GET", endpoint, f"/{bucket}/{key}", access_key, secret_key, timeout=timeout)


def put_object(endpoint: str, bucket: str, key: str, body: bytes, access_key: str, secret_key: str,
               timeout: float = 300.0) -> None:
    """Single PUT with a signed payload hash (files up to the RGW's 5 GB single-part limit;
    creditcard.csv is 150 MB)."""
    _request("PUT", endpoint, f"/{bucket}/{key}", access_key, secret_key, body=body, timeout=timeout)


def create_bucket(endpoint: str, bucket: str, access_key: str, secret_key: str) -> bool:
    """PUT /bucket; False when it already exists (409 BucketAlreadyOwnedByYou / Exists)."""
    try:
        _request("PUT", endpoint, f"/{bucket}", access_key, secret_key)
        return True
    except urllib.error.HTTPError as e:
        if e.code == 409:
            return False
        raise


def list_objects(endpoint: str, bucket: str, access_key: str, secret_key: str, prefix: str = "") -> List[Tuple[str, int]]:
    """ListObjectsV2 (all pages) -> [(key, size)]."""
    out: List[Tuple[str, int]] = []
    token = None
    while True:
        q = {"list-type": "2", "prefix": prefix}
        if token:
            q["continuation-token"] = token
        root = ET.fromstring(_request("GET", endpoint, f"/{bucket}", access_key, secret_key, query=q))
        ns = root.tag.split("}")[0] + "}" if root.tag.startswith("{") else ""
        for c in root.findall(f"{ns}Contents"):
            out.append((c.findtext(f"{ns}Key"), int(c.findtext(f"{ns}Size") or 0)))
        if (root.findtext(f"{ns}IsTruncated") or "false").lower() != "true":
            return out
        token = root.findtext(f"{ns}NextContinuationToken")


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


def main(argv=None) -> int:
    import argparse
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("cmd", choices=["upload", "ls"])
    ap.add_argument("file", nargs="?")
    ap.add_argument("--endpoint", default=os.environ.get("s3endpoint", ""))
    ap.add_argument("--bucket", default=os.environ.get("s3bucket", "ccdata"))
    ap.add_argument("--key", default=os.environ.get("filename", "OPEN/uploaded/creditcard.csv"))
    ap.add_argument("--prefix", default="")
    a = ap.parse_args(argv)
    ak, sk = os.environ.get("ACCESS_KEY_ID", ""), os.environ.get("SECRET_ACCESS_KEY", "")
    if not a.endpoint:
        raise SystemExit("no S3 endpoint: --endpoint or the s3endpoint env key")
    if a.cmd == "upload":
        if not a.file:
            raise SystemExit("upload needs a file")
        create_bucket(a.endpoint, a.bucket, ak, sk)
        with open(a.file, "rb") as f:
            body = f.read()
        put_object(a.endpoint, a.bucket, a.key, body, ak, sk)
        print(f"uploaded {a.file} ({len(body)} B) -> s3://{a.bucket}/{a.key}")
    else:
        for k, n in list_objects(a.endpoint, a.bucket, ak, sk, a.prefix):
            print(f"{n:>12d}  {k}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
