"""Seldon REST client used by the router (remote-scoring mode) and the KIE prediction
service: ``POST {SELDON_URL}/{SELDON_ENDPOINT}`` with optional bearer token, request
timeout ``SELDON_TIMEOUT`` (ms) and connection pool ``SELDON_POOL_SIZE``
(deploy/router.yaml:63-68; README.md:366-393)."""
from __future__ import annotations

import json
from typing import Optional

import aiohttp
import requests
from requests.adapters import HTTPAdapter


def _url(base: str, endpoint: str) -> str:
    if not base.startswith("http"):
        base = "http://" + base
    return base.rstrip("/") + "/" + endpoint.lstrip("/")


class SeldonClient:
    def __init__(self, url: str, endpoint: str = "api/v0.1/predictions", token: Optional[str] = None,
                 timeout_ms: int = 5000, pool_size: int = 5):
        self.url = _url(url, endpoint)
        self.token = token
        self.timeout_s = timeout_ms / 1000.0
        self.pool_size = pool_size
        self._session = requests.Session()
        ad = HTTPAdapter(pool_connections=pool_size, pool_maxsize=pool_size)
        self._session.mount("http://", ad)
        self._session.mount("https://", ad)
        self._aio: Optional[aiohttp.ClientSession] = None

    def _headers(self):
        h = {"Content-Type": "application/json"}
        if self.token:
            h["Authorization"] = f"Bearer {self.token}"
        return h

    def predict_sync(self, body: dict) -> dict:
        r = self._session.post(self.url, data=json.dumps(body), headers=self._headers(), timeout=self.timeout_s)
        r.raise_for_status()
        return r.json()

    async def predict(self, body: dict) -> dict:
        if self._aio is None or self._aio.closed:
            self._aio = aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=self.pool_size),
                                              timeout=aiohttp.ClientTimeout(total=self.timeout_s))
        async with self._aio.post(self.url, data=json.dumps(body), headers=self._headers()) as r:
            r.raise_for_status()
            return await r.json()

    async def aclose(self):
        if self._aio is not None:
            await self._aio.close()

    def close(self):
        self._session.close()
