"""Seldon Core v0.1 prediction protocol codec.

The router POSTs to ``{SELDON_URL}/{SELDON_ENDPOINT}`` with default endpoint
``api/v0.1/predictions`` (deploy/router.yaml:65-68); the KIE prediction service
defaults to ``predict`` (README.md:379).  Protocol shape ([EXT]):

request:  ``{"data": {"names": [...], "ndarray": [[...], ...]}}``
          or ``{"data": {"tensor": {"shape": [n, d], "values": [...]}}}``
          (the legacy Seldon wrapper also accepts form field ``json=<same>``)
response: ``{"meta": {...}, "data": {"names": ["proba_0", "proba_1"], "ndarray": [[p0, p1], ...]}}``

The ``proba_1`` column name is what the model dashboard plots
(deploy/grafana/ModelPrediction.json:96).
"""
from __future__ import annotations

import json
import uuid
from typing import Optional, Sequence, Tuple

import numpy as np

from .transaction import FEATURE_NAMES, N_FEATURES

DEFAULT_ROUTER_ENDPOINT = "api/v0.1/predictions"   # router.yaml:65-66
DEFAULT_KIE_ENDPOINT = "predict"                   # README.md:379
PROBA_NAMES = ["proba_0", "proba_1"]


class SeldonError(ValueError):
    pass


def parse_request(body) -> Tuple[np.ndarray, Optional[list]]:
    """Returns (X float32 [n, d], names or None). Accepts dict/bytes/str."""
    if isinstance(body, (bytes, bytearray, str)):
        try:
            body = json.loads(body)
        except json.JSONDecodeError as e:
            raise SeldonError(f"invalid JSON: {e}") from None
    if not isinstance(body, dict) or "data" not in body:
        raise SeldonError("request must carry a 'data' object")
    data = body["data"]
    names = data.get("names")
    if "ndarray" in data:
        arr = np.asarray(data["ndarray"], dtype=np.float32)
    elif "tensor" in data:
        t = data["tensor"]
        arr = np.asarray(t["values"], dtype=np.float32).reshape(t["shape"])
    else:
        raise SeldonError("data must contain 'ndarray' or 'tensor'")
    if arr.ndim == 1:
        arr = arr.reshape(1, -1)
    if arr.ndim != 2:
        raise SeldonError("expected a 2-D feature matrix")
    if names and arr.shape[1] == len(names) and list(names) != list(FEATURE_NAMES):
        # re-order columns by name when the caller sent named features in another order
        idx = {n: i for i, n in enumerate(names)}
        if all(n in idx for n in FEATURE_NAMES):
            arr = arr[:, [idx[n] for n in FEATURE_NAMES]]
    return np.ascontiguousarray(arr), names


def build_request(X, names: Sequence[str] = FEATURE_NAMES, tensor: bool = False) -> dict:
    X = np.asarray(X, dtype=np.float32)
    if X.ndim == 1:
        X = X.reshape(1, -1)
    if tensor:
        return {"data": {"names": list(names), "tensor": {"shape": list(X.shape),
                                                          "values": X.reshape(-1).tolist()}}}
    return {"data": {"names": list(names), "ndarray": X.tolist()}}


def build_response(proba1, model_name: str = "modelfull", extra_meta: Optional[dict] = None,
                   names: Sequence[str] = PROBA_NAMES, tensor: bool = False) -> dict:
    p = np.asarray(proba1, dtype=np.float64).reshape(-1)
    mat = np.stack([1.0 - p, p], axis=1)
    meta = {"puid": uuid.uuid4().hex, "tags": {}, "routing": {}, "requestPath": {model_name: model_name}}
    if extra_meta:
        meta.update(extra_meta)
    if tensor:
        data = {"names": list(names), "tensor": {"shape": list(mat.shape), "values": mat.reshape(-1).tolist()}}
    else:
        data = {"names": list(names), "ndarray": mat.tolist()}
    return {"meta": meta, "data": data}


def build_matrix_response(mat, names: Sequence[str], model_name: str) -> dict:
    mat = np.asarray(mat)
    meta = {"puid": uuid.uuid4().hex, "tags": {}, "routing": {}, "requestPath": {model_name: model_name}}
    return {"meta": meta, "data": {"names": list(names), "ndarray": mat.tolist()}}


def parse_response(body) -> Tuple[np.ndarray, list]:
    if isinstance(body, (bytes, bytearray, str)):
        body = json.loads(body)
    data = body["data"]
    names = data.get("names", [])
    if "ndarray" in data:
        arr = np.asarray(data["ndarray"])
    else:
        t = data["tensor"]
        arr = np.asarray(t["values"]).reshape(t["shape"])
    return arr, names


def proba1_from_response(body) -> np.ndarray:
    arr, names = parse_response(body)
    arr = np.asarray(arr, dtype=np.float64)
    if "proba_1" in names:
        return arr[:, names.index("proba_1")]
    return arr[:, -1]


def error_response(status: int, reason: str) -> dict:
    return {"status": {"code": status, "info": reason, "reason": "MICROSERVICE_BAD_DATA",
                       "status": "FAILURE"}}


assert N_FEATURES == 30
