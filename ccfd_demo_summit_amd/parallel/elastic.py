"""Elastic partition ownership: failure detection + re-assignment of a dead rank's stream
partitions (SURVEY.md §5 "Failure detection / elastic recovery", §4.1 fault-injection).

The reference relies on the platform (``restartPolicy: Always``, Kafka consumer-group
rebalance).  Here every rank holds a time-limited LEASE per partition in a shared KV store
(``torch.distributed.TCPStore`` of the job, or ``MemoryStore`` in tests):

    lease/<p>  = "<rank>:<expiry_ms>"          renewed by the owner every tick
    commit/<p> = "<offset>,<rows>,<fraud>"     written by the owner with every offset commit

* home partitions (``p % world == rank``) are claimed at start;
* a partition whose lease has been expired for ``ttl`` (its owner stopped renewing: crash,
  hang, lost GPU) is taken over by the first live rank that sees it, which resumes from the
  partition's committed offset (at-least-once) -- rows scored but not committed by the dead
  rank are scored again, and the committed per-partition counts make the global counters
  exactly-once (each offset range is counted by exactly one commit);
* the process engine de-duplicates fraud processes by transaction id, so a re-scored
  transaction never starts a second business process.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple


class MemoryStore:
    """In-process stand-in for ``torch.distributed.TCPStore`` (same method subset)."""

    def __init__(self):
        self._d: Dict[str, bytes] = {}
        self._lock = threading.Lock()

    def set(self, key: str, value) -> None:
        with self._lock:
            self._d[key] = value.encode() if isinstance(value, str) else bytes(value)

    def get(self, key: str) -> bytes:
        with self._lock:
            if key not in self._d:
                raise KeyError(key)
            return self._d[key]

    def add(self, key: str, amount: int) -> int:
        with self._lock:
            v = int(self._d.get(key, b"0")) + int(amount)
            self._d[key] = str(v).encode()
            return v

    def check(self, keys: List[str]) -> bool:
        with self._lock:
            return all(k in self._d for k in keys)

    def compare_set(self, key: str, expected, desired) -> bytes:
        exp = expected.encode() if isinstance(expected, str) else bytes(expected)
        des = desired.encode() if isinstance(desired, str) else bytes(desired)
        with self._lock:
            cur = self._d.get(key)
            if (cur is None and exp == b"") or cur == exp:
                self._d[key] = des
                return des
            return cur if cur is not None else b""


def _get(store, key: str) -> Optional[bytes]:
    try:
        if hasattr(store, "check") and not store.check([key]):
            return None
        return store.get(key)
    except (KeyError, RuntimeError):
        return None


@dataclass
class Lease:
    owner: int
    expiry_ms: int

    @classmethod
    def parse(cls, raw: Optional[bytes]) -> Optional["Lease"]:
        if not raw:
            return None
        o, e = raw.decode().split(":")
        return cls(int(o), int(e))

    def encode(self) -> str:
        return f"{self.owner}:{self.expiry_ms}"


class PartitionLeases:
    def __init__(self, store, rank: int, world: int, n_partitions: int, ttl_s: float = 2.0,
                 clock=time.time):
        self.store = store
        self.rank = rank
        self.world = world
        self.n = n_partitions
        self.ttl_ms = int(ttl_s * 1000)
        self.clock = clock
        self._owned: Dict[int, Lease] = {}
        self._t0: Optional[int] = None

    def _now_ms(self) -> int:
        return int(self.clock() * 1000)

    def owned(self) -> List[int]:
        return sorted(self._owned)

    def tick(self) -> Tuple[List[int], List[int]]:
        """Renew owned leases and claim claimable partitions.  Returns (gained, lost).

        home partition     claimable when unleased or its lease has expired;
        foreign partition  claimable when its lease expired more than one ttl ago, or when
                           nobody has ever leased it for 2 ttl since this rank started."""
        now = self._now_ms()
        if self._t0 is None:
            self._t0 = now
        gained, lost = [], []
        for p, lease in list(self._owned.items()):
            new = Lease(self.rank, now + self.ttl_ms)
            if self.store.compare_set(f"lease/{p}", lease.encode(), new.encode()) == new.encode().encode():
                self._owned[p] = new
            else:
                del self._owned[p]             # someone took it: we were presumed dead
                lost.append(p)
        for p in range(self.n):
            if p in self._owned:
                continue
            cur_raw = _get(self.store, f"lease/{p}")
            cur = Lease.parse(cur_raw)
            if p % self.world == self.rank:
                claimable = cur is None or cur.expiry_ms < now
            elif cur is None:
                claimable = now - self._t0 > 2 * self.ttl_ms
            else:
                claimable = cur.expiry_ms + self.ttl_ms < now
            if not claimable:
                continue
            new = Lease(self.rank, now + self.ttl_ms)
            if self.store.compare_set(f"lease/{p}", cur_raw or b"", new.encode()) == new.encode().encode():
                self._owned[p] = new
                gained.append(p)
        return gained, lost

    def release(self) -> None:
        for p, lease in list(self._owned.items()):
            self.store.compare_set(f"lease/{p}", lease.encode(), Lease(-1, 0).encode())
        self._owned.clear()

    # ------------------------------------------------------------------ commits
    def commit(self, p: int, offset: int, rows: int, fraud: int) -> bool:
        """Record an offset commit with the cumulative counts of the partition; only the
        current lease holder may commit."""
        if p not in self._owned:
            return False
        self.store.set(f"commit/{p}", f"{offset},{rows},{fraud}")
        return True

    def committed(self, p: int) -> Tuple[int, int, int]:
        raw = _get(self.store, f"commit/{p}")
        if not raw:
            return 0, 0, 0
        o, r, f = raw.decode().split(",")
        return int(o), int(r), int(f)

    def global_counts(self) -> Tuple[int, int]:
        rows = fraud = 0
        for p in range(self.n):
            _, r, f = self.committed(p)
            rows += r
            fraud += f
        return rows, fraud
