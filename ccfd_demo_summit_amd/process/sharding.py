"""KIE scale-out: the business-process tier as K shard processes.

The reference runs ONE KIE server (``ccd-service``, deploy/ccd-service.yaml:32 ``replicas:
1``) and its router starts a process for EVERY transaction (README.md:552; router.yaml:63-64).
At 1e6 tx/s that is 1e6 starts a second, more than one event loop absorbs, so the tier is
sharded:

* a process start goes to shard ``shard_of_tx(transaction_id, K)`` (a fixed 64-bit mix of
  the id -- the same on every engine rank, so a re-delivered start reaches the shard that
  deduplicates it);
* instance ids encode their shard: ``iid = shard + K * n`` (and task ids likewise), so a
  customer-response signal (which carries only the process id, README.md:569,605) and a
  task completion reach the owner: ``shard_of_id(iid, K) = iid % K``;
* every shard keeps its own journal (recovery), its own dedupe window, and -- on the engine
  side -- its own hand-off queue and dead-letter journal (router/handoff.py ShardedHandoff);
* each shard serves the reference's ``/rest/metrics`` histograms for its own instances;
  Prometheus sums them across the shard pods, so the KIE dashboard's queries
  (deploy/grafana/KIE.json) are unchanged.

``KIE_SERVER_URL`` names the shards: a comma-separated list (shard order), or one URL with
a ``{shard}`` placeholder expanded for ``kie.shards`` shards (the operator renders
``http://ccd-service-{shard}.ccd-service:8090`` for its StatefulSet pods).
"""
from __future__ import annotations

import os
import re
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

_MIX = np.uint64(0x9E3779B97F4A7C15)


def shard_of_tx(tx, shards: int):
    """Shard of a transaction id (scalar -> int, array -> int64 array).  Fibonacci hashing
    of the 64-bit id (high bits of id * 2^64/phi), so ids that share their low bits (the
    producers' ``(i + 1) << 40`` ranges) still spread evenly."""
    if shards <= 1:
        return 0 if np.isscalar(tx) or isinstance(tx, int) else np.zeros(len(tx), np.int64)
    if isinstance(tx, (int, np.integer)):
        h = (int(tx) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        return (h >> 32) % shards
    a = np.asarray(tx).astype(np.uint64, copy=False)
    with np.errstate(over="ignore"):
        h = a * _MIX
    return ((h >> np.uint64(32)) % np.uint64(shards)).astype(np.int64)


def shard_of_id(iid, shards: int):
    """Shard that owns a process instance (or user task) id."""
    if shards <= 1:
        return 0 if isinstance(iid, (int, np.integer)) else np.zeros(len(iid), np.int64)
    if isinstance(iid, (int, np.integer)):
        return int(iid) % shards
    return np.asarray(iid).astype(np.int64) % shards


def kie_urls(url: str, shards: int = 1) -> List[str]:
    """The shard URLs from KIE_SERVER_URL: a comma list, or ``{shard}`` expanded ``shards``
    times.  A single plain URL with shards > 1 is refused (the shards would be unreachable)."""
    url = (url or "").strip()
    if "{shard}" in url:
        return [url.replace("{shard}", str(k)) for k in range(max(1, int(shards)))]
    urls = [u.strip() for u in url.split(",") if u.strip()]
    if not urls:
        raise ValueError("KIE_SERVER_URL is empty")
    if shards > 1 and len(urls) != shards:
        raise ValueError(f"kie.shards={shards} but KIE_SERVER_URL names {len(urls)} server(s): give one URL "
                         "per shard (comma-separated) or a {shard} template")
    return urls


def shard_from_env(explicit: Optional[int] = None, hostname: Optional[str] = None) -> int:
    """This KIE process's shard: ``--shard``, else CCFD_KIE_SHARD, else the StatefulSet pod
    ordinal at the end of the host name (``ccd-service-3`` -> 3), else 0."""
    if explicit is not None and explicit >= 0:
        return int(explicit)
    env = os.environ.get("CCFD_KIE_SHARD")
    if env not in (None, ""):
        return int(env)
    m = re.search(r"-(\d+)$", hostname if hostname is not None else os.environ.get("HOSTNAME", ""))
    return int(m.group(1)) if m else 0


def split_columns(cols: Dict[str, Any], shard: np.ndarray, shards: int) -> List[Optional[Dict[str, Any]]]:
    """Columns -> one column dict per shard (None where a shard gets no row)."""
    out: List[Optional[Dict[str, Any]]] = []
    arrs = {k: np.asarray(v) for k, v in cols.items()}
    for k in range(shards):
        m = shard == k
        if not m.any():
            out.append(None)
            continue
        out.append({name: a[m] for name, a in arrs.items()})
    return out


def tx_column(cols: Dict[str, Any]):
    t = cols.get("transaction_id")
    return cols.get("tx_id") if t is None else t


class ShardedKieClient:
    """The ProcessEngine hand-off interface over K KIE shards (one KieClient each): starts
    split by transaction-id shard (ids merged back in request order), signals by instance id.
    With K = 1 it is a thin pass-through to the one client."""

    def __init__(self, clients: Sequence[Any]):
        if not clients:
            raise ValueError("no KIE shard clients")
        self.clients = list(clients)
        self.shards = len(self.clients)
        c0 = self.clients[0]
        self.signal_name = getattr(c0, "signal_name", "customerResponse")

    @classmethod
    def from_config(cls, kie_cfg, timeout_s: float = 5.0, pool_size: int = 5) -> "ShardedKieClient":
        from .kie_server import KieClient
        urls = kie_urls(kie_cfg.url, getattr(kie_cfg, "shards", 1))
        return cls([KieClient(u, kie_cfg.container_id, kie_cfg.fraud_process_id, kie_cfg.standard_process_id,
                              kie_cfg.signal_name, timeout_s=timeout_s, pool_size=pool_size) for u in urls])

    def client_for_tx(self, tx) -> Any:
        return self.clients[shard_of_tx(int(tx), self.shards)]

    def client_for_id(self, iid) -> Any:
        return self.clients[shard_of_id(int(iid), self.shards)]

    # -- starts
    def start_fraud(self, variables) -> int:
        tx = variables.get("transaction_id", variables.get("tx_id"))
        c = self.clients[0] if tx is None else self.client_for_tx(tx)
        return c.start_fraud(variables)

    def start_standard(self, variables) -> int:
        tx = variables.get("transaction_id", variables.get("tx_id"))
        c = self.clients[0] if tx is None else self.client_for_tx(tx)
        return c.start_standard(variables)

    def start_fraud_many(self, items) -> list:
        if self.shards == 1:
            return self.clients[0].start_fraud_many(items)
        groups: Dict[int, List[int]] = {}
        for i, v in enumerate(items):
            tx = v.get("transaction_id", v.get("tx_id"))
            groups.setdefault(0 if tx is None else shard_of_tx(int(tx), self.shards), []).append(i)
        out = [None] * len(items)
        for k, idx in groups.items():
            ids = self.clients[k].start_fraud_many([items[i] for i in idx]) if len(idx) > 1 else \
                [self.clients[k].start_fraud(items[idx[0]])]
            for i, iid in zip(idx, ids):
                out[i] = iid
        return out

    def start_standard_many(self, cols) -> list:
        if self.shards == 1:
            return self.clients[0].start_standard_many(cols)
        if not isinstance(cols, dict):
            from .engine import columns_of
            cols = columns_of(cols)
        tx = tx_column(cols)
        sh = shard_of_tx(np.asarray(tx), self.shards)
        out = np.full(len(sh), -1, np.int64)
        for k, sub in enumerate(split_columns(cols, sh, self.shards)):
            if sub is not None:
                out[sh == k] = np.asarray(self.clients[k].start_standard_many(sub), np.int64)
        return out.tolist()

    # -- commit watermark / audit
    def note_committed(self, offsets) -> None:
        for c in self.clients:
            c.note_committed(offsets)

    def find_transaction(self, tx_id: int, deep: bool = False):
        return self.client_for_tx(tx_id).find_transaction(tx_id, deep=deep)

    # -- signals
    def signal(self, instance_id: int, name: str, payload) -> bool:
        return self.client_for_id(instance_id).signal(instance_id, name, payload)

    def signal_many(self, items) -> list:
        if self.shards == 1 and hasattr(self.clients[0], "signal_many"):
            return self.clients[0].signal_many(items)
        groups: Dict[int, List[int]] = {}
        for i, (iid, _n, _p) in enumerate(items):
            groups.setdefault(shard_of_id(int(iid), self.shards), []).append(i)
        out = [False] * len(items)
        for k, idx in groups.items():
            c = self.clients[k]
            many = getattr(c, "signal_many", None)
            sub = [items[i] for i in idx]
            res = many(sub) if many is not None else [c.signal(iid, n, p) for iid, n, p in sub]
            for i, r in zip(idx, res):
                out[i] = r
        return out
