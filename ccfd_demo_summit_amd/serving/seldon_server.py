"""Seldon-compatible prediction server (replaces the SeldonDeployment ``modelfull`` and
the engine in front of it: deploy/model/modelfull.json).

Endpoints (port 8000 like ``SELDON_URL=http://modelfull-modelfull:8000``, router.yaml:67-68):
  POST /api/v0.1/predictions   Seldon engine API (router default SELDON_ENDPOINT)
  POST /api/v1.0/predictions   same, newer path
  POST /predict                model-wrapper API (KIE default endpoint, README.md:379); also
                               accepts form field ``json=``
  GET  /prometheus, /metrics   model gauges + seldon_api_engine_* histograms
  GET  /health/ping, /health/status, /ready, /live

Dynamic micro-batching: concurrent requests are coalesced (up to ``max_batch`` rows or
``max_delay_us``) into ONE fused-kernel launch on the GPU back-end; with the CPU
back-end and ``max_batch=1`` it is exactly the reference topology's batch=1 predict()
(BASELINE.json config 1).  Optional bearer-token auth (``SELDON_TOKEN``).
"""
from __future__ import annotations

import asyncio
import json
import time
from typing import List, Optional, Tuple

import numpy as np
from aiohttp import web

from ..contracts import seldon
from ..metrics.exporter import CONTENT_TYPE, ModelMetrics


class _Batcher:
    def __init__(self, scorer, max_batch: int, max_delay_us: int):
        self.scorer = scorer
        self.max_batch = max(1, int(max_batch))
        self.max_delay = max(0, int(max_delay_us)) * 1e-6
        self.queue: asyncio.Queue = asyncio.Queue()
        self.task: Optional[asyncio.Task] = None
        self.launches = 0
        self.rows = 0

    def start(self):
        self.task = asyncio.get_running_loop().create_task(self._run())

    async def stop(self):
        if self.task:
            self.task.cancel()
            try:
                await self.task
            except asyncio.CancelledError:
                pass

    async def submit(self, X: np.ndarray) -> Tuple[np.ndarray, float]:
        fut = asyncio.get_running_loop().create_future()
        await self.queue.put((X, fut))
        return await fut

    async def _run(self):
        loop = asyncio.get_running_loop()
        while True:
            X, fut = await self.queue.get()
            items = [(X, fut)]
            rows = X.shape[0]
            deadline = loop.time() + self.max_delay
            while rows < self.max_batch:
                timeout = deadline - loop.time()
                try:
                    if timeout <= 0:
                        nxt = self.queue.get_nowait()
                    else:
                        nxt = await asyncio.wait_for(self.queue.get(), timeout)
                except (asyncio.TimeoutError, asyncio.QueueEmpty):
                    break
                items.append(nxt)
                rows += nxt[0].shape[0]
            Xb = np.concatenate([it[0] for it in items]) if len(items) > 1 else items[0][0]
            t0 = time.perf_counter()
            try:
                if len(items) == 1 and rows <= 4:
                    proba, _ = self.scorer.score(Xb)                      # tiny: skip the thread hop
                else:
                    proba, _ = await loop.run_in_executor(None, self.scorer.score, Xb)
            except Exception as e:                                       # pragma: no cover
                for _, f in items:
                    if not f.done():
                        f.set_exception(e)
                continue
            dt = time.perf_counter() - t0
            self.launches += 1
            self.rows += rows
            off = 0
            for Xi, f in items:
                k = Xi.shape[0]
                if not f.done():
                    f.set_result((proba[off:off + k], dt))
                off += k


class SeldonServer:
    def __init__(self, scorer, model_name: str = "modelfull", token: Optional[str] = None,
                 max_batch: int = 4096, max_delay_us: int = 200, metrics: Optional[ModelMetrics] = None,
                 output_names: Optional[List[str]] = None, matrix_scorer: bool = False):
        self.scorer = scorer
        self.model_name = model_name
        self.token = token
        self.metrics = metrics or ModelMetrics(deployment=model_name, predictor=model_name, model_name=model_name)
        self.batcher = _Batcher(scorer, max_batch, max_delay_us) if not matrix_scorer else None
        self.output_names = output_names
        self.matrix_scorer = matrix_scorer      # scorer.predict_proba(X) -> [n, k] (user-task model)
        self.app = web.Application(client_max_size=64 * 1024 * 1024)
        r = self.app.router
        for path in ("/api/v0.1/predictions", "/api/v1.0/predictions", "/predict", "/api/v0.1/predict"):
            r.add_post(path, self.predict)
        r.add_get("/prometheus", self.prometheus)
        r.add_get("/metrics", self.prometheus)
        for path in ("/health/ping", "/ping", "/live", "/ready", "/health/status"):
            r.add_get(path, self.health)
        self.app.on_startup.append(self._startup)
        self.app.on_cleanup.append(self._cleanup)

    async def _startup(self, _app):
        if self.batcher:
            self.batcher.start()

    async def _cleanup(self, _app):
        if self.batcher:
            await self.batcher.stop()

    def _authorized(self, request: web.Request) -> bool:
        if not self.token:
            return True
        h = request.headers.get("Authorization", "")
        return h == f"Bearer {self.token}" or request.query.get("access_token") == self.token

    async def _body(self, request: web.Request):
        ctype = request.content_type or ""
        if ctype.startswith("application/x-www-form-urlencoded") or ctype.startswith("multipart/"):
            form = await request.post()
            return json.loads(form.get("json", "{}"))
        raw = await request.read()
        return json.loads(raw) if raw else {}

    async def predict(self, request: web.Request) -> web.Response:
        t0 = time.perf_counter()
        if not self._authorized(request):
            self.metrics.observe_request(time.perf_counter() - t0, 401)
            return web.json_response(seldon.error_response(401, "unauthorized"), status=401)
        try:
            body = await self._body(request)
            X, _names = seldon.parse_request(body)
        except (seldon.SeldonError, json.JSONDecodeError, ValueError, KeyError) as e:
            self.metrics.observe_request(time.perf_counter() - t0, 400)
            return web.json_response(seldon.error_response(400, str(e)), status=400)
        tensor = "tensor" in body.get("data", {})
        if self.matrix_scorer:
            mat = self.scorer.predict_proba(X)
            resp = seldon.build_matrix_response(mat, self.output_names or [], self.model_name)
            model_dt = time.perf_counter() - t0
        else:
            if X.shape[1] != 30:
                self.metrics.observe_request(time.perf_counter() - t0, 400)
                return web.json_response(seldon.error_response(400, "expected 30 features"), status=400)
            proba, model_dt = await self.batcher.submit(X)
            resp = seldon.build_response(proba, self.model_name, tensor=tensor)
            self.metrics.set_last(X[-1], float(proba[-1]))
        self.metrics.observe_request(time.perf_counter() - t0, 200, model_dt)
        return web.json_response(resp)

    async def prometheus(self, _request: web.Request) -> web.Response:
        return web.Response(body=self.metrics.expose(), headers={"Content-Type": CONTENT_TYPE})

    async def health(self, _request: web.Request) -> web.Response:
        st = {"status": "ok", "model": self.model_name, "device": getattr(self.scorer, "device", "cpu")}
        if self.batcher:
            st.update(launches=self.batcher.launches, rows=self.batcher.rows)
        return web.json_response(st)


def usertask_server(token: Optional[str] = None) -> SeldonServer:
    """The second model slot: ``ccfd-seldon-model`` for the jBPM prediction service."""
    from ..models.usertask import OUTCOMES, UserTaskModel
    return SeldonServer(UserTaskModel(), model_name="ccfd-seldon-model", token=token,
                        output_names=list(OUTCOMES), matrix_scorer=True)


def run(server: SeldonServer, host: str = "0.0.0.0", port: int = 8000) -> None:
    web.run_app(server.app, host=host, port=port, print=None, access_log=None)
