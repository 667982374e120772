"""Tracing: host-side spans exported as Chrome/Perfetto trace JSON, mirrored into roctx
ranges when the ROCm tracer library is loadable, so ``rocprofv3 --marker-trace`` shows the
framework's stages (ingest, pump, routing, all-reduce) on the same timeline as the kernels
(SURVEY.md §5 "Tracing / profiling": the reference has none).

    from ccfd_demo_summit_amd.utils.tracing import tracer
    with tracer.span("pump", batches=256):
        engine.pump(256)
    tracer.dump("trace.json")      # open in chrome://tracing or ui.perfetto.dev
"""
from __future__ import annotations

import ctypes
import json
import os
import threading
import time
from contextlib import contextmanager
from typing import Any, Dict, List, Optional


def _load_roctx():
    for name in ("libroctx64.so", "libroctx64.so.4"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePop.restype = ctypes.c_int
            return lib
        except OSError:
            continue
    try:
        import torch
        p = os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so")
        lib = ctypes.CDLL(p)
        lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
        return lib
    except Exception:
        return None


class Tracer:
    def __init__(self, enabled: Optional[bool] = None, max_events: int = 1_000_000, roctx: Optional[bool] = None):
        self.enabled = bool(int(os.environ.get("CCFD_TRACE", "0"))) if enabled is None else enabled
        self.max_events = max_events
        self._events: List[Dict[str, Any]] = []
        self._lock = threading.Lock()
        self._t0 = time.perf_counter_ns()
        use_roctx = bool(int(os.environ.get("CCFD_ROCTX", "0"))) if roctx is None else roctx
        self._roctx = _load_roctx() if use_roctx else None

    def enable(self, on: bool = True) -> None:
        self.enabled = on

    @contextmanager
    def span(self, name: str, cat: str = "ccfd", **args):
        if not self.enabled:
            yield
            return
        if self._roctx is not None:
            self._roctx.roctxRangePushA(name.encode())
        t = time.perf_counter_ns()
        try:
            yield
        finally:
            dur = time.perf_counter_ns() - t
            if self._roctx is not None:
                self._roctx.roctxRangePop()
            self._add({"name": name, "cat": cat, "ph": "X", "ts": (t - self._t0) / 1e3, "dur": dur / 1e3,
                       "pid": os.getpid(), "tid": threading.get_ident() & 0xFFFF, "args": args})

    def instant(self, name: str, cat: str = "ccfd", **args) -> None:
        if self.enabled:
            self._add({"name": name, "cat": cat, "ph": "i", "s": "t", "ts": (time.perf_counter_ns() - self._t0) / 1e3,
                       "pid": os.getpid(), "tid": threading.get_ident() & 0xFFFF, "args": args})

    def counter(self, name: str, **values) -> None:
        if self.enabled:
            self._add({"name": name, "ph": "C", "ts": (time.perf_counter_ns() - self._t0) / 1e3,
                       "pid": os.getpid(), "args": values})

    def _add(self, ev: Dict[str, Any]) -> None:
        with self._lock:
            if len(self._events) < self.max_events:
                self._events.append(ev)

    def events(self) -> List[Dict[str, Any]]:
        with self._lock:
            return list(self._events)

    def dump(self, path: str) -> str:
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events(), "displayTimeUnit": "ms"}, f)
        return path

    def clear(self) -> None:
        with self._lock:
            self._events.clear()


tracer = Tracer()


def batch_trace_events(trace, pid: int = 0, name: str = "engine") -> List[Dict[str, Any]]:
    """Chrome trace events of an engine's per-batch stage trace (``StreamEngine.read_trace``):
    one track per stage -- ``queued`` (ring arrival -> submit), ``in flight`` (submit ->
    completion record in host memory), ``device`` (first item claimed -> last item done,
    aligned to the host clock) and ``hand-off`` (landed -> retired by the engine thread).

    The device clock has its own epoch: it is aligned by the smallest ``t_landed - dev_end``
    over the trace (the fastest observed completion-record round trip), so device spans sit
    just before the host saw their completion and never after it."""
    import numpy as np
    tr = np.asarray(trace)
    ev: List[Dict[str, Any]] = [{"name": "process_name", "ph": "M", "pid": pid, "args": {"name": name}}]
    for tid, label in enumerate(("queued", "in flight", "device", "hand-off")):
        ev.append({"name": "thread_name", "ph": "M", "pid": pid, "tid": tid, "args": {"name": label}})
    if tr.size == 0:
        return ev
    dev = tr["dev_end"] > 0
    off = int((tr["t_landed"][dev] - tr["dev_end"][dev]).min()) if dev.any() else 0
    t0 = int(min(tr["t_submit"].min(), tr["t_arrival"][tr["t_arrival"] > 0].min()
                 if (tr["t_arrival"] > 0).any() else tr["t_submit"].min()))

    def span(tid, a, b, e):
        ev.append({"name": f"batch {int(e['seq'])}", "ph": "X", "pid": pid, "tid": tid, "ts": (a - t0) / 1e3,
                   "dur": max(0, b - a) / 1e3, "args": {"rows": int(e["rows"]), "partition": int(e["partition"]),
                                                        "flagged": int(e["flagged"])}})
    for e in tr:
        if e["t_arrival"] > 0:
            span(0, int(e["t_arrival"]), int(e["t_submit"]), e)
        span(1, int(e["t_submit"]), int(e["t_landed"]), e)
        if e["dev_end"] > 0:
            span(2, int(e["dev_start"]) + off, int(e["dev_end"]) + off, e)
        span(3, int(e["t_landed"]), int(e["t_complete"]), e)
    return ev


def dump_batch_trace(trace, path: str, **kw) -> str:
    with open(path, "w") as f:
        json.dump({"traceEvents": batch_trace_events(trace, **kw), "displayTimeUnit": "ns"}, f)
    return path
