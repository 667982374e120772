"""Runtime model hot swap across the DP ranks ("Weights are RCCL-broadcast
from rank 0 at load and at hot swap"; §5 checkpoint/resume: versioned weights + hot swap).

The reference bakes the model into its Seldon image and rolls pods to change it
(deploy/model/modelfull.json:24-25, ``imagePullPolicy: Always``).  Here a new model is
published to a running job without stopping ingest:

* rank 0 (or whoever holds the new weights) calls :meth:`HotSwap.offer`;
* the offer is announced in the control words of the next X2 counter all-reduce
  (``EpochPipeline(ctrl=hotswap)``): {version, blob bytes, 2-word checksum}, summed over
  ranks with only the source contributing -- no extra collective and no host wait;
* when that reduction completes, every rank (in the same collective order) starts an
  ASYNC broadcast of the blob; ``poll()`` swaps the engine's weights once it has landed and
  the checksum matches (``StreamEngine.swap_model``: in-flight batches finish on the old
  weights).  Nothing on the scoring thread waits for a slower rank.

:meth:`tick` is the standalone, blocking form of the same protocol (one header all-reduce,
then the broadcast), for callers without an epoch pipeline.

Optionally rank 0 watches a safetensors file (``models.save_model``) and offers it whenever
its mtime changes.
"""
from __future__ import annotations

import os
import threading
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .dp import N_CTRL_SLOTS, DistContext, _checksum


def _checksum_np(blob: bytes) -> np.ndarray:
    """Host twin of ``dp._checksum``: {sum of bytes, position-weighted sum} as int64."""
    b = np.frombuffer(blob, np.uint8).astype(np.int64)
    idx = np.arange(b.size, dtype=np.int64)
    return np.array([b.sum(), (b * (idx % 65521 + 1)).sum()], np.int64)


class HotSwap:
    def __init__(self, ctx: DistContext, engine, watch_path: Optional[str] = None, src: int = 0, group=None):
        self.ctx = ctx
        self.group = group
        self.engine = engine
        self.src = src
        self.version = 0
        self.watch_path = watch_path
        self._mtime = os.path.getmtime(watch_path) if watch_path and os.path.exists(watch_path) else None
        self._lock = threading.Lock()
        self._offer: Optional[bytes] = None
        self._announced: Optional[bytes] = None     # src: blob whose header is in flight
        self._inflight = None                       # (work, tensor, version, checksum)
        self.swaps = 0

    def offer(self, model) -> None:
        """Queue ``model`` (same kind as the running one) for the next announcement.  Rank ``src``.
        G32 / G20 engines (GBDT): the ensemble is packed against the LIVE bin table, so the
        partition logs need no re-encoding; ValueError if a split threshold is not one of its
        edges (a retrain that moves thresholds needs a new table: restart with re-encoding)."""
        bins = getattr(self.engine, "bins", None)
        if bins is not None:
            blob = model.pack(bins=bins)
        else:
            blob = model.pack(wire=True) if getattr(self.engine, "wire", False) else model.pack()
        with self._lock:
            self._offer = blob

    def _poll_watch(self) -> None:
        if not self.watch_path or self.ctx.rank != self.src:
            return
        try:
            m = os.path.getmtime(self.watch_path)
        except OSError:
            return
        if self._mtime is None or m > self._mtime:
            self._mtime = m
            from ..models import load_model
            self.offer(load_model(self.watch_path))

    # ---------------------------------------------------------------- pipeline protocol
    def contribute(self) -> np.ndarray:
        """Control words for the next reduction (all zero except on an announcing source)."""
        v = np.zeros(N_CTRL_SLOTS, np.int64)
        self._poll_watch()
        if self.ctx.rank != self.src or self._announced is not None or self._inflight is not None:
            return v
        with self._lock:
            blob, self._offer = self._offer, None
        if blob is None:
            return v
        self._announced = blob
        v[0], v[1] = self.version + 1, len(blob)
        v[2:4] = _checksum_np(blob)
        return v

    def on_reduced(self, v: np.ndarray) -> None:
        """Every rank, same order: the reduced control words of a completed reduction."""
        new_version, nbytes = int(v[0]), int(v[1])
        if new_version <= self.version:
            return
        dev = self.ctx.device
        if self.ctx.rank == self.src:
            t = torch.from_numpy(np.frombuffer(self._announced, np.uint8).copy()).to(dev)
            self._announced = None
        else:
            t = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        work = dist.broadcast(t, self.src, group=self.group, async_op=True) if self.ctx.initialized else None
        self._inflight = (work, t, new_version, np.asarray(v[2:4], np.int64))

    def poll(self, block: bool = False) -> bool:
        """Swap once the announced blob has arrived.  Returns True when this call swapped."""
        if self._inflight is None:
            return False
        work, t, new_version, ck = self._inflight
        if work is not None:
            if not block and not work.is_completed():
                return False
            work.wait()
        if t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()   # the engine reads it from its own streams
        self._inflight = None
        got = _checksum(t).cpu().numpy()
        if not np.array_equal(got, ck):
            raise RuntimeError("hot swap: model blob checksum mismatch after broadcast")
        self._swap(t)
        self.version = new_version
        self.swaps += 1
        return True

    # ---------------------------------------------------------------- standalone form
    def tick(self) -> bool:
        """Collective on every rank (blocking): announce + broadcast + swap.  True if swapped."""
        v = self.contribute()
        if self.ctx.initialized:
            hdr = torch.from_numpy(v).to(self.ctx.device)
            dist.all_reduce(hdr, group=self.group)
            v = hdr.cpu().numpy()
        self.on_reduced(v)
        return self.poll(block=True)

    def _swap(self, blob: torch.Tensor) -> None:
        from ..ops.kernels import DeviceModel
        cur = self.engine.dm
        dm = DeviceModel.from_blob(cur.kind, blob, cur.trees, cur.depth, wire=getattr(cur, "wire", False),
                                   bins=getattr(cur, "bins", None))
        self.engine.swap_model(dm)
