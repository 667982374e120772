"""Progress watchdog for long collective runs (bench.py, engine ranks).

A rank that stops making progress -- a peer that died inside an RCCL collective, a
persistent kernel whose doorbell never rings, a hand-off that blocks -- otherwise sits until
the process-group timeout or an outer kill, and says nothing about where it stopped.  The
watchdog is a daemon thread: the main loop calls ``beat(label)`` whenever it completes a unit
of work; when no beat arrives for ``timeout_s`` the thread prints a one-line JSON diagnostic
(``state()`` of the caller: posted/completed batches, epoch ticks, reducer busy, last
collective, ...) to stderr and ends the process with ``os._exit(code)``.

It never re-execs, never touches the GPU and never waits on a lock the stalled thread might
hold: ``state`` must read plain attributes only (a stalled main thread may hold the GIL-free
native call the watchdog would otherwise block behind).  Reference analogue: the
DeploymentConfig's ``activeDeadlineSeconds`` / ``timeoutSeconds`` (deploy/router.yaml:11-20),
which kill a rollout that stops progressing.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from typing import Callable, Dict, Optional

EXIT_STALLED = 5


class Watchdog:
    def __init__(self, timeout_s: float, state: Optional[Callable[[], Dict]] = None, rank: int = 0,
                 name: str = "bench", code: int = EXIT_STALLED, exit_fn: Callable[[int], None] = os._exit,
                 poll_s: Optional[float] = None, on_fire: Optional[Callable[[], object]] = None):
        self.timeout_s = float(timeout_s)
        self.state = state
        self.rank = rank
        self.name = name
        self.code = code
        self.exit_fn = exit_fn
        self.poll_s = poll_s if poll_s is not None else max(0.05, min(5.0, self.timeout_s / 10))
        self.last_beat = time.monotonic()
        self.last_label = "start"
        self.beats = 0
        self.fired = False
        self.report: Optional[Dict] = None
        # last action before the exit: e.g. StreamEngine.emergency_stop, so no persistent
        # kernel is left resident when the process ends
        self.on_fire = on_fire
        self._stop = threading.Event()
        self._th: Optional[threading.Thread] = None

    def beat(self, label: str = "") -> None:
        self.last_beat = time.monotonic()
        self.beats += 1
        if label:
            self.last_label = label

    def start(self) -> "Watchdog":
        if self.timeout_s <= 0:
            return self
        self._th = threading.Thread(target=self._run, daemon=True, name=f"{self.name}-watchdog")
        self._th.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._th is not None:
            self._th.join(1.0)

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            idle = time.monotonic() - self.last_beat
            if idle < self.timeout_s:
                continue
            self.fired = True
            rep = {"watchdog": self.name, "rank": self.rank, "stalled_s": round(idle, 1),
                   "timeout_s": self.timeout_s, "beats": self.beats, "last_progress": self.last_label}
            try:
                rep["state"] = self.state() if self.state is not None else {}
            except Exception as e:          # the diagnostic must not mask the stall
                rep["state_error"] = repr(e)
            self.report = rep
            print(f"[watchdog] rank {self.rank}: no progress for {idle:.1f} s -- "
                  + json.dumps(rep, default=str), file=sys.stderr, flush=True)
            if self.on_fire is not None:
                try:
                    rc = self.on_fire()
                    print(f"[watchdog] rank {self.rank}: exit hook returned {rc!r}", file=sys.stderr, flush=True)
                except Exception as e:
                    print(f"[watchdog] rank {self.rank}: exit hook failed: {e!r}", file=sys.stderr, flush=True)
            self.exit_fn(self.code)
            return
