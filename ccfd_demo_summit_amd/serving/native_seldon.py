"""Native Seldon predict() REST front end (csrc/engine/seldon_http.cpp) -- the
``modelfull-modelfull:8000`` endpoint of the reference (deploy/model/modelfull.json:37-44,
deploy/router.yaml:65-68) served by a C++ epoll loop that batches every request that
arrived during the previous GPU call into one fused-kernel launch.

Same routes and JSON as the aiohttp server (serving/seldon_server.py): POST
``/api/v0.1/predictions``, ``/api/v1.0/predictions``, ``/predict``; GET ``/prometheus``
(reference metric names: Seldon engine histograms and the proba_1 / Amount / V17 / V10
gauges, rendered here from the native counters); health routes.  Scoring is a
``StreamEngine`` over f32 rows (GPU) or any object with ``score(X) -> (proba, route)``
(CPU, through a ctypes callback -- tests and CPU-only hosts).
"""
from __future__ import annotations

import ctypes as C
import struct
from typing import Optional

import numpy as np

from ..contracts import metric_names as M
from ..metrics.exporter import LATENCY_BUCKETS
from ..ops._lib import lib

_SCORE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_float), C.c_int32, C.POINTER(C.c_float), C.c_void_p)
_RENDER_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, C.c_void_p)
_NB = 32                                   # native latency buckets (+Inf)
_STATUS = ("200", "400", "401", "500")


def _bind():
    L = lib()
    if getattr(L, "_seldon_bound", False):
        return L
    L.ccfd_seldon_http_start.restype = C.c_void_p
    L.ccfd_seldon_http_start.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_void_p), C.c_int, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_char_p, C.c_char_p, C.c_int,
                                         C.POINTER(C.c_double), C.c_int]
    L.ccfd_seldon_http_port.argtypes = [C.c_void_p]
    L.ccfd_seldon_http_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    L.ccfd_seldon_http_stop.argtypes = [C.c_void_p]
    L.ccfd_http_load.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_double,
                                 C.POINTER(C.c_double), C.c_int]
    L._seldon_bound = True
    return L


class NativeSeldonServer:
    """``scorer``: one scorer, or a list (one per epoll worker thread -- GPU engines are not
    shared between threads; a CPU scorer is reused by every worker)."""

    def __init__(self, scorer, host: str = "0.0.0.0", port: int = 8000, model_name: str = "modelfull",
                 token: Optional[str] = None, max_batch: int = 65536,
                 deployment: str = "modelfull", model_image: str = "ccfd-mi355x", workers: int = 1):
        L = _bind()
        self.model_name = model_name
        self.labels = dict(deployment_name=deployment, predictor_name=model_name, predictor_version="1",
                           model_name=model_name, model_image=model_image, model_version="1")
        scorers = list(scorer) if isinstance(scorer, (list, tuple)) else [scorer]
        engines = [getattr(sc, "engine", sc) for sc in scorers]         # GpuScorer -> its StreamEngine
        native = all(hasattr(e, "h") and not getattr(e, "wire", False) for e in engines)
        self._score_cb = None
        eng_arr = None
        if native:
            workers = len(engines) if len(engines) > 1 else max(1, workers)
            if len(engines) < workers:
                raise ValueError("one GPU engine per worker thread")
            eng_arr = (C.c_void_p * workers)(*[e.h for e in engines[:workers]])
        else:
            first = scorers[0]

            def _score(rows, n, proba, _ctx):
                try:
                    X = np.ctypeslib.as_array(rows, shape=(n, 30))
                    p, _r = first.score(X)
                    np.ctypeslib.as_array(proba, shape=(n,))[:] = p
                    return 0
                except Exception:                           # scoring failure -> HTTP 500
                    return -1
            self._score_cb = _SCORE_FN(_score)
        self._render_cb = _RENDER_FN(self._render)
        b = (C.c_double * len(LATENCY_BUCKETS))(*LATENCY_BUCKETS)
        self.h = L.ccfd_seldon_http_start(host.encode(), int(port), eng_arr, int(max(1, workers)),
                                          C.cast(self._score_cb, C.c_void_p) if self._score_cb else None, None,
                                          C.cast(self._render_cb, C.c_void_p), None, model_name.encode(),
                                          (token or "").encode(), int(max_batch), b, len(LATENCY_BUCKETS))
        if not self.h:
            raise OSError(f"native Seldon server could not bind {host}:{port}")
        self.port = L.ccfd_seldon_http_port(self.h)
        self.scorer = scorer
        self.workers = max(1, workers)

    # ------------------------------------------------------------------ stats / metrics
    def stats(self) -> dict:
        ns = len(_STATUS)
        out = (C.c_uint64 * (2 * ns + 3 + 4 + ns * (_NB + 1)))()
        _bind().ccfd_seldon_http_stats(self.h, out)
        v = list(out)
        b0 = 2 * ns + 3
        last = [struct.unpack("<f", struct.pack("<I", int(x) & 0xFFFFFFFF))[0] for x in v[b0:b0 + 4]]
        h0 = b0 + 4
        hist = [v[h0 + i * (_NB + 1): h0 + (i + 1) * (_NB + 1)] for i in range(ns)]
        return {"count": dict(zip(_STATUS, v[0:ns])), "sum_s": dict(zip(_STATUS, [x * 1e-9 for x in v[ns:2 * ns]])),
                "rows": v[2 * ns], "batches": v[2 * ns + 1], "model_s": v[2 * ns + 2] * 1e-9,
                "last": dict(zip(M.MODEL_GAUGES, last)), "hist": dict(zip(_STATUS, hist))}

    def expose(self) -> bytes:
        """Prometheus text with the reference names (same series as serving/seldon_server.py;
        the native path has one latency per request, used for the server and client series)."""
        from prometheus_client import CollectorRegistry, generate_latest
        from prometheus_client.core import GaugeMetricFamily, HistogramMetricFamily
        st = self.stats()
        nb = len(LATENCY_BUCKETS)

        class _Coll:
            def collect(self_):
                srv = HistogramMetricFamily(M.SELDON_SERVER_REQUESTS, "Seldon engine server request latency",
                                            labels=["status"])
                cli = HistogramMetricFamily(M.SELDON_CLIENT_REQUESTS, "Seldon engine -> model request latency",
                                            labels=list(M.SELDON_CLIENT_LABELS))
                for s in _STATUS:
                    h = st["hist"][s]
                    cum, buckets = 0, []
                    for i, bound in enumerate(LATENCY_BUCKETS):
                        cum += h[i]
                        buckets.append((str(bound), cum))
                    buckets.append(("+Inf", cum + sum(h[nb:])))
                    srv.add_metric([s], buckets, st["sum_s"][s])
                    cli.add_metric([s] + [self.labels[k] for k in M.SELDON_CLIENT_LABELS[1:]], buckets, st["sum_s"][s])
                yield srv
                yield cli
                for name, val in st["last"].items():
                    g = GaugeMetricFamily(name, f"last request {name}")
                    g.add_metric([], val)
                    yield g
        reg = CollectorRegistry()
        reg.register(_Coll())
        return generate_latest(reg)

    def _render(self, buf, cap, _ctx) -> int:
        try:
            body = self.expose()
        except Exception:
            return 0
        n = min(len(body), int(cap))
        C.memmove(buf, body, n)
        return n

    def stop(self) -> None:
        if self.h:
            _bind().ccfd_seldon_http_stop(self.h)
            self.h = None

    def __del__(self):
        try:
            self.stop()
        except Exception:
            pass


def http_load(host: str, port: int, body: bytes, conns: int = 64, seconds: float = 5.0,
              path: str = "/api/v0.1/predictions", threads: int = 0) -> dict:
    """Native keep-alive load generator (csrc/engine/http_load.cpp); threads 0 = 1 per 64 conns."""
    out = (C.c_double * 5)()
    rc = _bind().ccfd_http_load(host.encode(), int(port), path.encode(), body, len(body), int(conns),
                                float(seconds), out, int(threads))
    if rc != 0:
        raise OSError("load generator could not connect")
    return {"req_per_s": out[0], "p50_us": out[1], "p99_us": out[2], "errors": int(out[3]), "requests": int(out[4])}
