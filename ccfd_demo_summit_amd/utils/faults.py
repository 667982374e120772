"""Fault-injection hooks ("Fault-injection hooks: drop, delay, or crash a
rank"; §4.1 fault-injection tests).

The reference's only injected fault is the notification service's simulated "no reply"
(README.md:414,562-565), which drives the fraud process's timer branch; that lives in
``process/notifier.py``.  This module injects faults into the scoring ranks themselves so the
recovery paths (lease failover, at-least-once re-delivery, exactly-once committed counts,
X2 pairing under skew) can be exercised on purpose:

* ``drop``  -- a fetched batch is discarded before it is scored and committed (the consumer
  "loses" it); at-least-once delivery must re-fetch it from the committed offset;
* ``delay`` -- the rank stalls for ``ms`` before a step (a slow or descheduled rank; peers must
  not block on it);
* ``crash`` -- the rank dies: ``mode=exit`` ends the process with ``os._exit`` (no cleanup,
  like SIGKILL), ``mode=raise`` raises :class:`InjectedCrash` (in-process tests);
* ``stall`` -- the rank hangs for good at ``after_steps`` (a peer wedged in a collective or a
  kernel that never completes): nothing but a watchdog (utils/watchdog.py) or a kill ends it.

A plan is a ``;``-separated list of ``kind:key=value,...`` clauses, from ``CCFD_FAULTS`` or
code, each optionally restricted to one rank::

    CCFD_FAULTS="drop:p=0.01;delay:ms=20,p=0.05,rank=1;crash:after_steps=500,rank=2,mode=exit"

Decisions come from a seeded RNG per (plan, rank), so a run is reproducible.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np


class InjectedCrash(RuntimeError):
    """Raised by a ``crash`` clause with ``mode=raise``."""


@dataclass
class FaultClause:
    kind: str                                  # drop | delay | crash | stall
    p: float = 1.0                             # per-step probability (drop, delay)
    ms: float = 0.0                            # delay length
    rank: Optional[int] = None                 # None: every rank
    after_steps: Optional[int] = None          # crash / stall: at this step count
    after_s: Optional[float] = None            # crash: this long after the plan was armed
    mode: str = "raise"                        # crash: raise | exit


@dataclass
class FaultPlan:
    clauses: List[FaultClause] = field(default_factory=list)
    seed: int = 0
    rank: int = 0
    steps: int = 0
    injected: Dict[str, int] = field(default_factory=lambda: {"drop": 0, "delay": 0, "crash": 0, "stall": 0})

    def __post_init__(self):
        self._rng = np.random.default_rng(self.seed * 1_000_003 + self.rank)
        # called right before a crash clause's os._exit: the GPU state a crashed rank must not
        # leave behind (the engine service stops its persistent kernel here)
        self.before_exit = None
        self._t0 = time.monotonic()

    @classmethod
    def parse(cls, spec: str, rank: int = 0, seed: int = 0) -> "FaultPlan":
        clauses = []
        for part in filter(None, (s.strip() for s in spec.split(";"))):
            kind, _, args = part.partition(":")
            kind = kind.strip()
            if kind not in ("drop", "delay", "crash", "stall"):
                raise ValueError(f"unknown fault kind {kind!r}")
            c = FaultClause(kind)
            for kv in filter(None, (s.strip() for s in args.split(","))):
                k, _, v = kv.partition("=")
                if k in ("p", "ms", "after_s"):
                    setattr(c, k, float(v))
                elif k in ("rank", "after_steps"):
                    setattr(c, k, int(v))
                elif k == "mode":
                    if v not in ("raise", "exit"):
                        raise ValueError(f"crash mode must be raise|exit, got {v!r}")
                    c.mode = v
                else:
                    raise ValueError(f"unknown fault option {k!r} in {part!r}")
            clauses.append(c)
        return cls(clauses, seed=seed, rank=rank)

    @classmethod
    def from_env(cls, rank: int = 0) -> Optional["FaultPlan"]:
        spec = os.environ.get("CCFD_FAULTS", "").strip()
        if not spec:
            return None
        return cls.parse(spec, rank=rank, seed=int(os.environ.get("CCFD_FAULTS_SEED", "0")))

    def _mine(self, c: FaultClause) -> bool:
        return c.rank is None or c.rank == self.rank

    def step(self) -> None:
        """Call once per scoring step: applies delay and crash clauses."""
        self.steps += 1
        for c in self.clauses:
            if not self._mine(c):
                continue
            if c.kind == "delay" and c.ms > 0 and self._rng.random() < c.p:
                self.injected["delay"] += 1
                time.sleep(c.ms / 1e3)
            elif c.kind == "stall" and (c.after_steps is None or self.steps >= c.after_steps):
                self.injected["stall"] += 1
                while True:                             # wedged: only a watchdog / kill ends it
                    time.sleep(3600)
            elif c.kind == "crash":
                due = (c.after_steps is not None and self.steps >= c.after_steps) or \
                      (c.after_s is not None and time.monotonic() - self._t0 >= c.after_s)
                if due:
                    self.injected["crash"] += 1
                    if c.mode == "exit":
                        if self.before_exit is not None:
                            self.before_exit()          # e.g. stop a resident persistent kernel
                        os._exit(17)                    # no cleanup, no commit: like SIGKILL
                    raise InjectedCrash(f"injected crash on rank {self.rank} at step {self.steps}")

    def drop(self) -> bool:
        """True when the batch just fetched should be discarded (not scored, not committed)."""
        for c in self.clauses:
            if c.kind == "drop" and self._mine(c) and self._rng.random() < c.p:
                self.injected["drop"] += 1
                return True
        return False
