"""KIE-Server-compatible REST front of the process engine (replaces ``ccd-service``:
deploy/ccd-service.yaml, port 8090; metrics at ``/rest/metrics``, README.md:509-514).

KIE Server REST paths ([EXT], container/process/signal ids configurable):
  POST /services/rest/server/containers/{c}/processes/{p}/instances            -> instance id
  POST /services/rest/server/containers/{c}/processes/instances/{i}/signal/{s} -> signal
  GET  /services/rest/server/containers/{c}/processes/instances/{i}            -> instance
  GET  /services/rest/server/queries/tasks/instances/pot-owners                -> task list
  GET  /services/rest/server/containers/{c}/tasks/{t}                          -> task
  PUT  /services/rest/server/containers/{c}/tasks/{t}/states/completed         -> complete
  GET  /rest/metrics                                                           -> Prometheus
Extensions for the GPU engine's router:
  POST .../containers/{c}/processes/{p}/instances/batch       many starts in one request
  POST .../containers/{c}/processes/{p}/instances/committed   the engine's committed offsets
       (frees commit-gated dedupe keys, process/engine.py note_committed)
  POST .../containers/{c}/processes/instances/signal/batch    many signals in one request
  GET  .../containers/{c}/processes/instances/by-transaction/{tx}[?deep=1]
       the process a transaction started -- standard ones too, which are counted, not
       retained as instances (process/engine.py find_transaction)
A background task fires process timers (``ProcessEngine.tick``).

Sharded tier (process/sharding.py): a server is shard ``engine.shard`` of ``engine.shards``.
A start whose transaction hashes to another shard, or a signal / task / instance request for
an id another shard owns, is answered ``421 Misdirected Request`` -- a misconfigured router
surfaces (the hand-off dead-letters it) instead of silently breaking per-shard idempotency.
"""
from __future__ import annotations

import asyncio
import json
import time
from dataclasses import asdict
from typing import Optional

import requests
from aiohttp import web

from ..metrics.exporter import CONTENT_TYPE
from ..utils.lathist import LatHist
from .dedupe import DedupeFull
from .engine import ProcessEngine

BASE = "/services/rest/server"


COLUMNS_CT = "application/x-ccfd-columns"
IDS_CT = "application/x-ccfd-ids"          # response: the instance ids as raw int64 LE
MISDIRECTED = 421
_COL_DT = {"q": "<i8", "d": "<f8", "f": "<f4", "I": "<u4"}


def encode_columns(cols) -> bytes:
    """Column batch -> binary body: b"CCOL", u32 rows, u32 columns, then per column u8 name
    length, name, u8 dtype code (q i64 / d f64 / f f32 / I u32) and the raw little-endian
    array.  ~20x cheaper to build and parse than the JSON list form at 4096 rows."""
    import struct

    import numpy as np
    arrs = {k: np.asarray(v) for k, v in cols.items()}
    n = len(next(iter(arrs.values()))) if arrs else 0
    parts = [b"CCOL", struct.pack("<II", n, len(arrs))]
    for k, a in arrs.items():
        code = {"i": "q", "u": "q", "f": "f" if a.dtype.itemsize <= 4 else "d"}.get(a.dtype.kind)
        if code is None or len(a) != n:
            raise ValueError(f"column {k!r}: numeric columns of one length only")
        kb = k.encode()
        parts += [struct.pack("<B", len(kb)), kb, code.encode(), np.ascontiguousarray(a, _COL_DT[code]).tobytes()]
    return b"".join(parts)


def decode_columns(body: bytes):
    import struct

    import numpy as np
    if body[:4] != b"CCOL":
        raise ValueError("not a CCOL column batch")
    n, k = struct.unpack_from("<II", body, 4)
    o, cols = 12, {}
    for _ in range(k):
        ln = body[o]
        name = body[o + 1:o + 1 + ln].decode()
        dt = np.dtype(_COL_DT[chr(body[o + 1 + ln])])
        o += 2 + ln
        cols[name] = np.frombuffer(body, dt, n, o)
        o += n * dt.itemsize
    if o != len(body):
        raise ValueError("CCOL body length mismatch")
    return cols


class KieServer:
    def __init__(self, engine: ProcessEngine, container_id: str = "ccd-fraud-kjar",
                 fraud_process_id: str = "ccd-fraud-kjar.CCDProcess",
                 standard_process_id: str = "ccd-fraud-kjar.StandardProcess", tick_s: float = 0.05):
        self.engine = engine
        self.container_id = container_id
        self.fraud_pid = fraud_process_id
        self.standard_pid = standard_process_id
        self.tick_s = tick_s
        self.app = web.Application()
        r = self.app.router
        r.add_post(BASE + "/containers/{c}/processes/{p}/instances", self.start)
        r.add_post(BASE + "/containers/{c}/processes/{p}/instances/batch", self.start_batch)
        r.add_post(BASE + "/containers/{c}/processes/{p}/instances/committed", self.committed)
        r.add_get(BASE + "/containers/{c}/processes/instances/by-transaction/{tx}", self.by_transaction)
        r.add_post(BASE + "/containers/{c}/processes/instances/signal/batch", self.signal_batch)
        r.add_post(BASE + "/containers/{c}/processes/instances/{i}/signal/{s}", self.signal)
        r.add_get(BASE + "/containers/{c}/processes/instances/{i}", self.get_instance)
        r.add_get(BASE + "/queries/tasks/instances/pot-owners", self.tasks)
        r.add_get(BASE + "/containers/{c}/tasks/{t}", self.get_task)
        r.add_put(BASE + "/containers/{c}/tasks/{t}/states/completed", self.complete_task)
        r.add_get("/rest/metrics", self.metrics)
        r.add_get("/rest/stats", self.stats)
        r.add_get(BASE, self.info)
        self.app.on_startup.append(self._startup)
        self.app.on_cleanup.append(self._cleanup)
        self._ticker: Optional[asyncio.Task] = None
        # scored -> started, the server's share: a start request's arrival after its rows were
        # scored (engine hand-off queue + network), the handler's own time, the timer tick's
        # time, and how late the event loop wakes the ticker (everything else on the loop)
        self.recv_after_scored = LatHist()
        self.handler_time = LatHist()
        self.tick_time = LatHist()
        self.loop_lag = LatHist()
        self.gc_pauses = LatHist()          # filled when the service tracks GC (cmd_kie)

    def attribution(self) -> dict:
        return {"received_after_scored_us": self.recv_after_scored.summary_us(),
                "start_handler_us": self.handler_time.summary_us(),
                "timer_tick_us": self.tick_time.summary_us(),
                "event_loop_lag_us": self.loop_lag.summary_us(),
                "journal_write_us": self.engine.journal_time.summary_us(),
                "gc_pause_us": self.gc_pauses.summary_us()}

    async def _startup(self, _app):
        async def loop():
            while True:
                t0 = time.monotonic_ns()
                self.engine.tick()
                t1 = time.monotonic_ns()
                self.tick_time.add(t1 - t0)
                await asyncio.sleep(self.tick_s)
                self.loop_lag.add(time.monotonic_ns() - t1 - int(self.tick_s * 1e9))
        self._ticker = asyncio.get_running_loop().create_task(loop())

    async def _cleanup(self, _app):
        if self._ticker:
            self._ticker.cancel()

    def _check_container(self, request) -> Optional[web.Response]:
        c = request.match_info.get("c")
        if c is not None and c != self.container_id:
            return web.json_response({"type": "FAILURE", "msg": f"Container {c} is not instantiated."}, status=404)
        return None

    @property
    def shard(self) -> int:
        return getattr(self.engine, "shard", 0)

    @property
    def shards(self) -> int:
        return getattr(self.engine, "shards", 1)

    def _misdirected(self, what: str) -> web.Response:
        return web.json_response({"type": "FAILURE", "msg": f"{what} belongs to another KIE shard "
                                  f"(this is shard {self.shard} of {self.shards})"}, status=MISDIRECTED)

    def _foreign_txs(self, items) -> int:
        """How many of a start request's transactions hash to another shard."""
        if self.shards <= 1:
            return 0
        from .sharding import shard_of_tx
        if isinstance(items, dict):
            tx = items.get("transaction_id", items.get("tx_id"))
            if tx is None:
                return 0
            import numpy as np
            t = np.asarray(tx)
            if t.dtype.kind not in "iu":
                t = np.asarray([int(x) for x in tx], np.int64)
            return int((shard_of_tx(t, self.shards) != self.shard).sum())
        n = 0
        for v in items:
            tx = v.get("transaction_id", v.get("tx_id")) if isinstance(v, dict) else None
            if isinstance(tx, (int, float)) and shard_of_tx(int(tx), self.shards) != self.shard:
                n += 1
        return n

    def _foreign_id(self, iid) -> bool:
        return self.shards > 1 and int(iid) % self.shards != self.shard

    async def info(self, _request):
        return web.json_response({"type": "SUCCESS", "msg": "Kie Server info",
                                  "result": {"kie-server-info": {"id": "ccd-service", "version": "ccfd-mi355x",
                                                                  "capabilities": ["BPM", "DMN", "Prometheus"]}}})

    async def start(self, request: web.Request):
        bad = self._check_container(request)
        if bad:
            return bad
        pid = request.match_info["p"]
        raw = await request.read()
        variables = json.loads(raw) if raw else {}
        if self._foreign_txs([variables]):
            return self._misdirected("transaction")
        if pid == self.standard_pid:
            iid = self.engine.start_standard(variables)
        elif pid == self.fraud_pid:
            iid = self.engine.start_fraud(variables)
        else:
            return web.json_response({"type": "FAILURE", "msg": f"Could not find process definition {pid}"},
                                     status=404)
        return web.json_response(iid, status=201)

    async def start_batch(self, request: web.Request):
        """Extension for the GPU engine's router: start one instance per element of a JSON
        list in ONE request (the engine hands off every fraud-routed row of a scoring step
        together; one HTTP round trip per transaction would cap the hand-off at ~1K/s)."""
        bad = self._check_container(request)
        if bad:
            return bad
        pid = request.match_info["p"]
        t_in, t0 = time.time_ns(), time.monotonic_ns()
        raw = await request.read()
        try:
            # a JSON list of variable objects, JSON columns {"transaction_id": [...], ...}, or a
            # binary column batch (COLUMNS_CT: the router's standard-route hand-off)
            items = decode_columns(raw) if request.content_type == COLUMNS_CT else json.loads(raw or b"[]")
        except (ValueError, KeyError, IndexError) as e:
            return web.json_response({"type": "FAILURE", "msg": f"bad batch body: {e}"}, status=400)
        if not isinstance(items, (list, dict)):
            return web.json_response({"type": "FAILURE", "msg": "expected a JSON list or columns"}, status=400)
        try:
            foreign = self._foreign_txs(items)
        except (ValueError, TypeError) as e:
            return web.json_response({"type": "FAILURE", "msg": f"bad batch: {e}"}, status=400)
        if foreign:
            return self._misdirected(f"{foreign} transaction(s) of the batch")
        try:
            if pid == self.standard_pid:
                ids = self.engine.start_standard_array(items) if hasattr(self.engine, "start_standard_array") \
                    else self.engine.start_standard_many(items)
            elif pid == self.fraud_pid:
                ids = self.engine.start_fraud_many(items)
            else:
                ids = None
        except DedupeFull as e:
            # every dedupe key may still be re-delivered: refuse (retried by the hand-off) rather
            # than evict one -- back-pressure until the engine's commits free room
            return web.json_response({"type": "FAILURE", "msg": str(e)}, status=503)
        except (ValueError, TypeError, AttributeError) as e:
            return web.json_response({"type": "FAILURE", "msg": f"bad batch: {e}"}, status=400)
        if ids is None:
            return web.json_response({"type": "FAILURE", "msg": f"Could not find process definition {pid}"},
                                     status=404)
        self._note_request(items, t_in, len(ids))
        if IDS_CT in request.headers.get("Accept", ""):
            import numpy as np                  # binary ids: no JSON list of 4096 ints to build
            body = np.asarray(ids, np.int64).astype("<i8", copy=False).tobytes()
            self.handler_time.add(time.monotonic_ns() - t0)
            return web.Response(body=body, status=201, content_type=IDS_CT)
        if hasattr(ids, "tolist"):
            ids = ids.tolist()
        self.handler_time.add(time.monotonic_ns() - t0)
        return web.json_response(ids, status=201)

    async def committed(self, request: web.Request):
        """The engine's committed Kafka offsets ({"offsets": {partition: offset}})."""
        bad = self._check_container(request)
        if bad:
            return bad
        try:
            body = json.loads(await request.read() or b"{}")
            offs = {int(p): int(o) for p, o in body.get("offsets", {}).items()}
        except (ValueError, TypeError, AttributeError) as e:
            return web.json_response({"type": "FAILURE", "msg": f"bad offsets: {e}"}, status=400)
        note = getattr(self.engine, "note_committed", None)
        if note is not None:
            note(offs)
        return web.json_response({"type": "SUCCESS"}, status=200)

    async def by_transaction(self, request: web.Request):
        bad = self._check_container(request)
        if bad:
            return bad
        try:
            tx = int(request.match_info["tx"])
        except ValueError:
            return web.json_response({"type": "FAILURE", "msg": "transaction id must be an integer"}, status=400)
        if self.shards > 1:
            from .sharding import shard_of_tx
            if shard_of_tx(tx, self.shards) != self.shard:
                return self._misdirected("transaction")
        deep = request.query.get("deep", "0") not in ("0", "", "false")
        if deep:                                # journal scan: off the event loop
            rec = await asyncio.get_running_loop().run_in_executor(None, self.engine.find_transaction, tx, True)
        else:
            rec = self.engine.find_transaction(tx)
        if rec is None:
            return web.json_response({"type": "FAILURE", "msg": f"no process for transaction {tx} on this shard "
                                      "within the retention" + ("" if deep else " (try ?deep=1)")}, status=404)
        return web.json_response(rec)

    def _note_request(self, items, t_in: int, n: int) -> None:
        sc = None
        if isinstance(items, dict):
            col = items.get("scored_ns")
            sc = int(col[0]) if col is not None and len(col) else None
        elif items and isinstance(items[0], dict):
            sc = items[0].get("scored_ns")
        if sc:
            self.recv_after_scored.add(t_in - int(sc), n)

    async def signal(self, request: web.Request):
        bad = self._check_container(request)
        if bad:
            return bad
        raw = await request.read()
        payload = json.loads(raw) if raw else None
        if self._foreign_id(request.match_info["i"]):
            return self._misdirected("process instance")
        ok = self.engine.signal(int(request.match_info["i"]), request.match_info["s"], payload)
        return web.Response(status=200 if ok else 404)

    async def signal_batch(self, request: web.Request):
        """Extension for the engine's hand-off: many customer-response signals in ONE request
        (a JSON list of {"instance_id", "signal", "payload"}); answers a list of booleans
        (False: the instance was no longer waiting -- timer fired, duplicate, unknown)."""
        bad = self._check_container(request)
        if bad:
            return bad
        items = json.loads(await request.read() or b"[]")
        if not isinstance(items, list):
            return web.json_response({"type": "FAILURE", "msg": "expected a JSON list"}, status=400)
        if any(self._foreign_id(it["instance_id"]) for it in items):
            return self._misdirected("a process instance of the batch")
        return web.json_response([bool(self.engine.signal(int(it["instance_id"]), it.get("signal", "customerResponse"),
                                                          it.get("payload"))) for it in items])

    async def get_instance(self, request: web.Request):
        if self._foreign_id(request.match_info["i"]):
            return self._misdirected("process instance")
        inst = self.engine.get(int(request.match_info["i"]))
        if inst is None:
            return web.json_response({"type": "FAILURE"}, status=404)
        d = asdict(inst)
        d["state"] = inst.state.value
        return web.json_response({"process-instance-id": inst.id, "process-id": inst.process_id,
                                  "process-instance-state": 1 if inst.state.value != "completed" else 2,
                                  "variables": inst.variables, "outcome": inst.outcome, "detail": d},
                                 dumps=lambda o: json.dumps(o, default=str))

    async def tasks(self, request: web.Request):
        status = request.query.get("status", "Ready")
        ts = self.engine.list_tasks(None if status == "all" else status)
        return web.json_response({"task-summary": [
            {"task-id": t.id, "task-name": t.name, "task-status": t.status, "task-proc-inst-id": t.instance_id,
             "task-container-id": self.container_id, "suggested-outcome": t.suggested_outcome,
             "confidence": t.confidence} for t in ts]})

    async def get_task(self, request: web.Request):
        if self._foreign_id(request.match_info["t"]):
            return self._misdirected("task")
        t = self.engine.tasks.get(int(request.match_info["t"]))
        if t is None:
            return web.json_response({"type": "FAILURE"}, status=404)
        return web.json_response(asdict(t), dumps=lambda o: json.dumps(o, default=str))

    async def complete_task(self, request: web.Request):
        if self._foreign_id(request.match_info["t"]):
            return self._misdirected("task")
        raw = await request.read()
        out = json.loads(raw) if raw else {}
        outcome = out.get("outcome", out.get("approved"))
        ok = self.engine.complete_task(int(request.match_info["t"]), str(outcome))
        return web.Response(status=201 if ok else 404)

    async def stats(self, _request):
        """Process counts (deployment checks: every fraud-routed transaction started once)."""
        e = self.engine
        with e._lock:
            fraud = sum(1 for i in e.instances.values() if i.process_id == e.FRAUD)
            body = {"shard": self.shard, "shards": self.shards,
                    "fraud_instances_retained": fraud, "fraud_started": getattr(e, "fraud_count", len(e._by_tx)),
                    "duplicates": e.duplicates, "notified": getattr(e, "notified_count", 0),
                    "standard_started": e.standard_count, "standard_duplicates": e.standard_duplicates,
                    "scored_to_started_us": e.handoff_latency_us(),
                    "handoff_attribution": self.attribution(),
                    "active": sum(1 for i in e.instances.values() if i.state.value != "completed"),
                    "waiting_customer": sum(1 for i in e.instances.values() if i.state.value == "waiting_customer"),
                    "outcomes": dict(e.outcome_counts), "outcome_digest": f"{e.outcome_digest:016x}",
                    "next_instance_id": None}
        if hasattr(e, "dedupe_stats"):
            body["standard_dedupe"] = e.dedupe_stats()
        return web.json_response(body)

    async def metrics(self, _request):
        m = self.engine.metrics
        body = m.expose() if m is not None else b""
        return web.Response(body=body, headers={"Content-Type": CONTENT_TYPE})


class KieClient:
    """HTTP client with the ProcessEngine hand-off interface (router -> KIE, README.md:552,569).

    Pooled: each calling thread (e.g. the KieHandoff workers, router/handoff.py) gets its own
    keep-alive session with up to ``pool_size`` connections -- the KIE analogue of the
    reference's SELDON_POOL_SIZE / SELDON_TIMEOUT client settings (README.md:386-393)."""

    def __init__(self, url: str, container_id: str = "ccd-fraud-kjar",
                 fraud_process_id: str = "ccd-fraud-kjar.CCDProcess",
                 standard_process_id: str = "ccd-fraud-kjar.StandardProcess",
                 signal_name: str = "customerResponse", timeout_s: float = 5.0, pool_size: int = 5):
        import threading
        self.base = url.rstrip("/") + BASE
        self.c = container_id
        self.fraud_pid = fraud_process_id
        self.standard_pid = standard_process_id
        self.signal_name = signal_name
        self.timeout = timeout_s
        self.pool_size = max(1, int(pool_size))
        self._tls = threading.local()

    @property
    def s(self) -> requests.Session:
        sess = getattr(self._tls, "session", None)
        if sess is None:
            sess = requests.Session()
            ad = requests.adapters.HTTPAdapter(pool_connections=1, pool_maxsize=self.pool_size)
            sess.mount("http://", ad)
            sess.mount("https://", ad)
            self._tls.session = sess
        return sess

    def _start(self, pid: str, variables) -> int:
        r = self.s.post(f"{self.base}/containers/{self.c}/processes/{pid}/instances",
                        data=json.dumps(variables), headers={"Content-Type": "application/json"},
                        timeout=self.timeout)
        r.raise_for_status()
        return int(r.json())

    def start_fraud(self, variables) -> int:
        return self._start(self.fraud_pid, variables)

    def start_fraud_many(self, items) -> list:
        """One request for many fraud instances (``/instances/batch`` extension)."""
        if not items:
            return []
        r = self.s.post(f"{self.base}/containers/{self.c}/processes/{self.fraud_pid}/instances/batch",
                        data=json.dumps(items), headers={"Content-Type": "application/json"}, timeout=self.timeout)
        r.raise_for_status()
        return [int(x) for x in r.json()]

    def start_standard(self, variables) -> int:
        return self._start(self.standard_pid, variables)

    def start_standard_many(self, items) -> list:
        """One request for many standard instances (``/instances/batch`` extension); ``items``
        may be columns ``{"transaction_id": [...], "customer_id": [...], "amount": [...],
        "proba": [...]}`` -- ~4x smaller and faster to encode than a list of objects."""
        if isinstance(items, dict):
            if not any(len(v) for v in items.values()):
                return []
            body, ct = encode_columns(items), COLUMNS_CT
        else:
            if not items:
                return []
            body, ct = json.dumps(items), "application/json"
        r = self.s.post(f"{self.base}/containers/{self.c}/processes/{self.standard_pid}/instances/batch",
                        data=body, headers={"Content-Type": ct, "Accept": f"{IDS_CT}, application/json"},
                        timeout=self.timeout)
        r.raise_for_status()
        if r.headers.get("Content-Type", "").startswith(IDS_CT):
            import numpy as np
            return np.frombuffer(r.content, "<i8").tolist()
        return [int(x) for x in r.json()]

    def note_committed(self, offsets) -> None:
        """Tell the shard the engine committed these offsets (``/instances/committed``)."""
        r = self.s.post(f"{self.base}/containers/{self.c}/processes/{self.standard_pid}/instances/committed",
                        data=json.dumps({"offsets": {str(int(p)): int(o) for p, o in offsets.items()}}),
                        headers={"Content-Type": "application/json"}, timeout=self.timeout)
        r.raise_for_status()

    def find_transaction(self, tx_id: int, deep: bool = False):
        """The process transaction ``tx_id`` started on this shard (None: none in retention)."""
        r = self.s.get(f"{self.base}/containers/{self.c}/processes/instances/by-transaction/{int(tx_id)}",
                       params={"deep": "1"} if deep else None, timeout=max(self.timeout, 60.0 if deep else 0))
        if r.status_code == 404:
            return None
        r.raise_for_status()
        return r.json()

    def signal_many(self, items) -> list:
        """Many signals in one request (``signal/batch`` extension): items of
        (instance_id, name, payload); returns one bool per item."""
        if not items:
            return []
        body = [{"instance_id": int(i), "signal": n or self.signal_name, "payload": p} for i, n, p in items]
        r = self.s.post(f"{self.base}/containers/{self.c}/processes/instances/signal/batch",
                        data=json.dumps(body), headers={"Content-Type": "application/json"}, timeout=self.timeout)
        r.raise_for_status()
        return [bool(x) for x in r.json()]

    def signal(self, instance_id: int, name: str, payload) -> bool:
        r = self.s.post(f"{self.base}/containers/{self.c}/processes/instances/{instance_id}/signal/{name or self.signal_name}",
                        data=json.dumps(payload), headers={"Content-Type": "application/json"}, timeout=self.timeout)
        if r.status_code >= 500 or r.status_code == MISDIRECTED:
            r.raise_for_status()              # 5xx transient: retried; 421 misrouted: dead-lettered
        return r.status_code == 200
