"""Seldon gRPC predict endpoint ("Seldon-compatible REST predict() (+ gRPC)").

Seldon Core exposes ``seldon.protos.Seldon/Predict`` (engine) and ``seldon.protos.Model/Predict``
(model wrapper) taking and returning a ``SeldonMessage``.  There is no ``protoc`` in this image,
so the message types are declared here as a ``FileDescriptorProto`` and materialised with the
protobuf runtime -- the wire format is the public Seldon ``prediction.proto`` subset the router
uses: ``data.names``, ``data.tensor{shape, values}``, ``data.ndarray`` (ListValue),
``meta.puid``, ``status``.

Scoring goes through the same dynamic micro-batcher as the REST server
(``seldon_server._Batcher``), so concurrent gRPC calls coalesce into one kernel launch.
"""
from __future__ import annotations

import time
import uuid
from typing import Optional

import grpc
import numpy as np
from google.protobuf import descriptor_pb2, descriptor_pool, json_format, message_factory, struct_pb2

from ..contracts import seldon
from ..contracts.transaction import FEATURE_NAMES

_F = descriptor_pb2.FieldDescriptorProto


def _build_pool():
    pool = descriptor_pool.DescriptorPool()
    pool.AddSerializedFile(struct_pb2.DESCRIPTOR.serialized_pb)
    fd = descriptor_pb2.FileDescriptorProto(name="ccfd_seldon_prediction.proto", package="seldon.protos",
                                            syntax="proto3", dependency=["google/protobuf/struct.proto"])

    def msg(name, fields, oneofs=()):
        m = fd.message_type.add(name=name)
        for o in oneofs:
            m.oneof_decl.add(name=o)
        for f in fields:
            fname, num, ftype, label = f[:4]
            fld = m.field.add(name=fname, number=num, type=ftype, label=label, json_name=fname)
            if len(f) > 4 and f[4]:
                fld.type_name = f[4]
            if len(f) > 5 and f[5] is not None:
                fld.oneof_index = f[5]
            if ftype in (_F.TYPE_INT32, _F.TYPE_DOUBLE) and label == _F.LABEL_REPEATED:
                fld.options.packed = True
        return m

    O, R = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
    msg("Tensor", [("shape", 1, _F.TYPE_INT32, R), ("values", 2, _F.TYPE_DOUBLE, R)])
    msg("DefaultData", [("names", 1, _F.TYPE_STRING, R),
                        ("tensor", 2, _F.TYPE_MESSAGE, O, ".seldon.protos.Tensor", 0),
                        ("ndarray", 3, _F.TYPE_MESSAGE, O, ".google.protobuf.ListValue", 0)],
        oneofs=["data_oneof"])
    msg("Status", [("code", 1, _F.TYPE_INT32, O), ("info", 2, _F.TYPE_STRING, O),
                   ("reason", 3, _F.TYPE_STRING, O), ("status", 4, _F.TYPE_INT32, O)])
    msg("Meta", [("puid", 1, _F.TYPE_STRING, O),
                 ("tags", 2, _F.TYPE_MESSAGE, O, ".google.protobuf.Struct")])
    msg("SeldonMessage", [("status", 1, _F.TYPE_MESSAGE, O, ".seldon.protos.Status"),
                          ("meta", 2, _F.TYPE_MESSAGE, O, ".seldon.protos.Meta"),
                          ("data", 3, _F.TYPE_MESSAGE, O, ".seldon.protos.DefaultData", 0),
                          ("binData", 4, _F.TYPE_BYTES, O, None, 0),
                          ("strData", 5, _F.TYPE_STRING, O, None, 0),
                          ("jsonData", 6, _F.TYPE_MESSAGE, O, ".google.protobuf.Value", 0)],
        oneofs=["data_oneof"])
    pool.Add(fd)
    return pool


_POOL = _build_pool()
SeldonMessage = message_factory.GetMessageClass(_POOL.FindMessageTypeByName("seldon.protos.SeldonMessage"))
SERVICES = ("seldon.protos.Seldon", "seldon.protos.Model")


def message_to_matrix(m) -> np.ndarray:
    """SeldonMessage -> float32 [n, 30] (tensor fast path, ndarray/jsonData via the REST codec)."""
    which = m.WhichOneof("data_oneof")
    if which == "data":
        d = m.data
        kind = d.WhichOneof("data_oneof")
        if kind == "tensor":
            X = np.asarray(d.tensor.values, np.float32).reshape(tuple(d.tensor.shape) or (1, -1))
            if X.ndim == 1:
                X = X.reshape(1, -1)
            names = list(d.names)
            if names and list(names) != list(FEATURE_NAMES) and X.shape[1] == len(names):
                X, _ = seldon.parse_request({"data": {"names": names, "ndarray": X.tolist()}})
            return X
        X, _ = seldon.parse_request({"data": json_format.MessageToDict(d)})
        return X
    if which == "jsonData":
        X, _ = seldon.parse_request(json_format.MessageToDict(m.jsonData))
        return X
    if which == "strData":
        X, _ = seldon.parse_request(m.strData)
        return X
    raise seldon.SeldonError("SeldonMessage carries no data")


def matrix_request(X: np.ndarray, names=FEATURE_NAMES):
    m = SeldonMessage()
    X = np.asarray(X, np.float32)
    m.data.names.extend(list(names))
    m.data.tensor.shape.extend(list(X.shape))
    m.data.tensor.values.extend(X.astype(np.float64).ravel().tolist())
    return m


def proba_response(proba1: np.ndarray, model_name: str):
    p1 = np.asarray(proba1, np.float64)
    m = SeldonMessage()
    m.meta.puid = uuid.uuid4().hex
    m.meta.tags.update({"model": model_name})
    m.data.names.extend(seldon.PROBA_NAMES)
    m.data.tensor.shape.extend([int(p1.size), 2])
    m.data.tensor.values.extend(np.stack([1.0 - p1, p1], 1).ravel().tolist())
    return m


def response_proba1(m) -> np.ndarray:
    if m.status.code not in (0, 200):
        raise seldon.SeldonError(f"seldon status {m.status.code}: {m.status.info}")
    v = np.asarray(m.data.tensor.values, np.float64).reshape(tuple(m.data.tensor.shape))
    return v[:, list(m.data.names).index("proba_1")].astype(np.float32)


def _error(code: int, info: str):
    m = SeldonMessage()
    m.status.code = code
    m.status.info = info
    m.status.reason = "MICROSERVICE_BAD_DATA" if code == 400 else "MICROSERVICE_INTERNAL_ERROR"
    m.status.status = 1   # FAILURE
    return m


class SeldonGrpcServer:
    """Async gRPC server sharing the REST server's scorer and micro-batcher."""

    def __init__(self, scorer, model_name: str = "modelfull", token: Optional[str] = None,
                 max_batch: int = 4096, max_delay_us: int = 200, metrics=None):
        from .seldon_server import _Batcher
        self.scorer = scorer
        self.model_name = model_name
        self.token = token
        self.metrics = metrics
        self.batcher = _Batcher(scorer, max_batch, max_delay_us)
        self.server: Optional[grpc.aio.Server] = None
        self.port: Optional[int] = None

    async def _predict(self, request, context):
        t0 = time.perf_counter()
        if self.token:
            md = dict(context.invocation_metadata() or ())
            if md.get("authorization") not in (f"Bearer {self.token}",) and md.get("access_token") != self.token:
                await context.abort(grpc.StatusCode.UNAUTHENTICATED, "unauthorized")
        try:
            X = message_to_matrix(request)
        except (seldon.SeldonError, ValueError, KeyError) as e:
            return _error(400, str(e))
        if X.shape[1] != 30:
            return _error(400, "expected 30 features")
        proba, model_dt = await self.batcher.submit(X)
        if self.metrics is not None:
            self.metrics.observe_request(time.perf_counter() - t0, 200, model_dt)
            self.metrics.set_last(X[-1], float(proba[-1]))
        return proba_response(proba, self.model_name)

    async def start(self, host: str = "0.0.0.0", port: int = 5001) -> int:
        self.server = grpc.aio.server(options=[("grpc.max_receive_message_length", 64 << 20),
                                               ("grpc.max_send_message_length", 64 << 20)])
        handler = grpc.unary_unary_rpc_method_handler(self._predict, request_deserializer=SeldonMessage.FromString,
                                                      response_serializer=SeldonMessage.SerializeToString)
        self.server.add_generic_rpc_handlers([grpc.method_handlers_generic_handler(svc, {"Predict": handler})
                                              for svc in SERVICES])
        self.port = self.server.add_insecure_port(f"{host}:{port}")
        self.batcher.start()
        await self.server.start()
        return self.port

    async def stop(self, grace: float = 0.5) -> None:
        if self.server is not None:
            await self.server.stop(grace)
        await self.batcher.stop()


class SeldonGrpcClient:
    def __init__(self, target: str, token: Optional[str] = None, timeout_ms: int = 5000,
                 service: str = "seldon.protos.Seldon"):
        self.channel = grpc.insecure_channel(target)
        self.timeout_s = timeout_ms / 1000.0
        self.md = [("authorization", f"Bearer {token}")] if token else None
        self._call = self.channel.unary_unary(f"/{service}/Predict",
                                              request_serializer=SeldonMessage.SerializeToString,
                                              response_deserializer=SeldonMessage.FromString)

    def predict(self, X: np.ndarray) -> np.ndarray:
        return response_proba1(self._call(matrix_request(X), timeout=self.timeout_s, metadata=self.md))

    def predict_message(self, m):
        return self._call(m, timeout=self.timeout_s, metadata=self.md)

    def close(self):
        self.channel.close()
