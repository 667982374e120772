"""Membership generations + communicator re-formation on rank failure / rejoin
(SURVEY.md §5 "Failure detection / elastic recovery": "The RCCL communicator is
re-initialised on membership change").

The reference only has platform-level recovery (``restartPolicy: Always``, rolling
DeploymentConfigs: deploy/router.yaml:11-20,75-76, deploy/ccd-service.yaml:11-20,71-72).
Here the job's ranks share a KV store that outlives any single rank (the launcher's or the
test's ``TCPStore``; rank 0's store would die with rank 0) and:

* every rank bumps a heartbeat counter ``hb/<r>`` from its own thread (so a blocking group
  build never makes it look dead); an observer calls a rank dead
  when ITS OWN monotonic clock saw no change of that counter for ``ttl`` (no cross-host
  clock comparison), and a never-seen rank only after a start-up grace;
* the lowest live rank proposes generation ``g+1 = sorted(live ranks)`` with one
  compare-and-set on ``gen`` whenever the live set differs from generation ``g``'s members
  (a rank dying, a restarted rank heartbeating again);
* every member of the new generation builds a FRESH process group for it on a
  ``PrefixStore("g<g>/")`` -- gloo, or RCCL (``ProcessGroupNCCL``) for GPU tensors -- and
  aborts the previous one, so a collective stuck on a dead peer is cancelled instead of
  hanging the survivors.  A build that times out (a member died mid-rendezvous) bumps the
  generation with one CAS so every member retries on fresh keys.  ``torch.distributed``'s
  default group is never touched.

Collectives are only ever issued asynchronously and polled (``ElasticGroup.poll``): a
failure shows up as an exception (gloo: peer connection reset) or as a generation change
while the work is pending (RCCL: the stuck collective is aborted with the old group).
``ElasticCounterReducer`` keeps a failed epoch's local contribution and re-submits it in
the next generation, so the survivors' X2 totals lose no locally-counted rows.  (Rows the
dead rank counted but never reduced are recovered by the lease/commit layer,
parallel/elastic.py, which stays the exactly-once source of truth.)
"""
from __future__ import annotations

import datetime
import threading
import time
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist


def _get(store, key: str) -> Optional[bytes]:
    try:
        if hasattr(store, "check") and not store.check([key]):
            return None
        return store.get(key)
    except (KeyError, RuntimeError):
        return None


def _parse_gen(raw: Optional[bytes], world: int) -> Tuple[int, List[int]]:
    if not raw:
        return 0, list(range(world))
    g, m = raw.decode().split(":")
    return int(g), [int(x) for x in m.split(",") if x != ""]


class Membership:
    """Heartbeats + generation proposals over a shared store."""

    def __init__(self, store, rank: int, world: int, ttl_s: float = 2.0, grace_s: Optional[float] = None,
                 prefix: str = "ccfd/mem/", clock=time.monotonic):
        self.store = store
        self.rank = rank
        self.world = world                     # rank ids are 0..world-1 (a restarted rank reuses its id)
        self.ttl = float(ttl_s)
        self.grace = float(grace_s if grace_s is not None else 3 * ttl_s)
        self.prefix = prefix
        self.clock = clock
        self.t0 = clock()
        self._seen: Dict[int, Tuple[int, float]] = {}     # rank -> (last counter, local time it changed)

    def heartbeat(self) -> None:
        self.store.add(f"{self.prefix}hb/{self.rank}", 1)

    def live(self) -> List[int]:
        now = self.clock()
        out = []
        for r in range(self.world):
            if r == self.rank:
                out.append(r)
                continue
            raw = _get(self.store, f"{self.prefix}hb/{r}")
            v = int(raw) if raw else 0
            last = self._seen.get(r)
            if last is None or last[0] != v:
                self._seen[r] = (v, now)
                last = self._seen[r]
            if v == 0:
                if now - self.t0 < self.grace:        # not started yet: give it the start-up grace
                    out.append(r)
            elif now - last[1] < self.ttl:
                out.append(r)
        return out

    def view(self) -> Tuple[int, List[int]]:
        return _parse_gen(_get(self.store, f"{self.prefix}gen"), self.world)

    def propose(self) -> Optional[Tuple[int, List[int]]]:
        """Lowest live rank: publish generation g+1 = live set if it differs from g's members."""
        live = self.live()
        key = f"{self.prefix}gen"
        raw = _get(self.store, key)
        gen, members = _parse_gen(raw, self.world)
        if self.rank != min(live) or live == members:
            return None
        new = f"{gen + 1}:{','.join(str(r) for r in live)}"
        got = self.store.compare_set(key, raw.decode() if raw else "", new)
        got = got.decode() if isinstance(got, (bytes, bytearray)) else str(got)
        return (gen + 1, live) if got == new else None


class ElasticGroup:
    """A process group per membership generation (gloo or RCCL), re-formed on change."""

    def __init__(self, store, rank: int, world: int, backend: str = "gloo",
                 device: Optional[torch.device] = None, ttl_s: float = 2.0, timeout_s: float = 30.0,
                 prefix: str = "ccfd/mem/", grace_s: Optional[float] = None, heartbeat_thread: bool = True):
        self.store = store
        self.rank = rank
        self.backend = backend
        self.device = device if device is not None else torch.device("cpu")
        self.timeout = datetime.timedelta(seconds=timeout_s)
        self.prefix = prefix
        self.membership = Membership(store, rank, world, ttl_s=ttl_s, grace_s=grace_s, prefix=prefix)
        self.gen = -1
        self.members: List[int] = []
        self.pg = None
        self.regroups = 0
        self.build_failures = 0
        # Heartbeats from their own thread: building a group for a new generation blocks until
        # every member has joined, and a rank that stopped heartbeating meanwhile would be
        # declared dead by the others (generation flapping).
        self._stop = threading.Event()
        self._hb = None
        if heartbeat_thread:
            self.membership.heartbeat()
            self._hb = threading.Thread(target=self._beat, name=f"ccfd-hb-{rank}", daemon=True)
            self._hb.start()

    def _beat(self) -> None:
        period = max(0.01, self.membership.ttl / 5)
        while not self._stop.wait(period):
            try:
                self.membership.heartbeat()
            except Exception:
                return                      # store gone: the job is over

    @property
    def member(self) -> bool:
        return self.pg is not None

    @property
    def size(self) -> int:
        return len(self.members)

    def _build(self, gen: int, members: List[int]):
        idx = members.index(self.rank)
        st = dist.PrefixStore(f"{self.prefix}g{gen}/", self.store)
        if self.backend == "nccl":
            opts = dist.ProcessGroupNCCL.Options()
            return dist.ProcessGroupNCCL(st, idx, len(members), opts)
        return dist.ProcessGroupGloo(st, idx, len(members), self.timeout)

    def _drop(self) -> None:
        if self.pg is None:
            return
        try:
            self.pg.abort()            # cancels a collective stuck on a dead peer (RCCL) / closes sockets
        except Exception:
            pass
        self.pg = None

    def tick(self) -> bool:
        """Heartbeat, propose if leader, and follow the published generation.  Returns True
        when this call switched generations (the caller must treat in-flight work as lost)."""
        if self._hb is None:
            self.membership.heartbeat()
        self.membership.propose()
        gen, members = self.membership.view()
        if gen == self.gen:
            return False
        self._drop()
        self.gen, self.members = gen, members
        self.regroups += 1
        if self.rank in members:
            try:
                self.pg = self._build(gen, members)
            except Exception:
                # a member never joined generation `gen` (it died, or moved on): bump the
                # generation with one CAS so every member retries on a fresh key prefix
                self.pg = None
                self.build_failures += 1
                key = f"{self.prefix}gen"
                cur = f"{gen}:{','.join(str(r) for r in members)}"
                self.store.compare_set(key, cur, f"{gen + 1}:{','.join(str(r) for r in members)}")
        return True

    def all_reduce(self, t: torch.Tensor):
        """Asynchronous SUM over the current generation; None if this rank is not a member."""
        if self.pg is None:
            return None
        return self.pg.allreduce([t])

    @staticmethod
    def poll(work) -> str:
        """'done' | 'pending' | 'failed' for a Work returned by all_reduce."""
        if work is None:
            return "failed"
        if not work.is_completed():
            return "pending"
        try:
            work.wait()
        except Exception:
            return "failed"
        return "done"

    def close(self) -> None:
        self._stop.set()
        self._drop()


class ElasticCounterReducer:
    """X2 over an ElasticGroup: cumulative global totals that survive rank failures.

    ``submit(v)`` adds the local epoch vector ``v`` (int64) and starts an async all-reduce of
    everything not yet reduced; ``progress()`` polls it: on success the reduced vector is
    folded into ``totals``; on failure, or when ``group.tick()`` reports a new generation
    while it is pending, the LOCAL part is kept and re-sent in the next generation."""

    def __init__(self, group: ElasticGroup, k: int, device: Optional[torch.device] = None):
        self.group = group
        self.device = device if device is not None else group.device
        self.totals = torch.zeros(k, dtype=torch.int64, device=self.device)
        self.unsent = torch.zeros(k, dtype=torch.int64, device=self.device)    # local, not yet reduced
        self._buf: Optional[torch.Tensor] = None
        self._local: Optional[torch.Tensor] = None
        self._work = None
        self.completed = 0
        self.failed = 0

    def submit(self, v: torch.Tensor) -> None:
        self.unsent += v.to(self.device, torch.int64)

    def _start(self) -> None:
        if self._work is not None or not self.group.member:
            return
        self._local = self.unsent.clone()
        self.unsent.zero_()
        self._buf = self._local.clone()
        self._work = self.group.all_reduce(self._buf)

    def progress(self) -> str:
        """One non-blocking step (call every tick AFTER group.tick()); returns the state."""
        if self._work is None:
            self._start()
            return "idle" if self._work is None else "started"
        st = ElasticGroup.poll(self._work)
        if st == "pending":
            return st
        if st == "done":
            self.totals += self._buf
            self.completed += 1
        else:
            self.unsent += self._local            # keep our rows for the next generation
            self.failed += 1
        self._work = self._buf = self._local = None
        self._start()
        return st

    def on_regroup(self) -> None:
        """The group switched generations: in-flight work belongs to a dead communicator."""
        if self._work is not None:
            self.unsent += self._local
            self.failed += 1
            self._work = self._buf = self._local = None
