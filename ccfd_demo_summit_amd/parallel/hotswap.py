"""Runtime model hot swap across the DP ranks ("Weights are RCCL-broadcast
from rank 0 at load and at hot swap"; §5 checkpoint/resume: versioned weights + hot swap).

The reference bakes the model into its Seldon image and rolls pods to change it
(deploy/model/modelfull.json:24-25, ``imagePullPolicy: Always``).  Here a new model is
published to a running job without stopping ingest:

* rank 0 (or whoever holds the new weights) calls :meth:`HotSwap.offer`;
* every rank calls :meth:`HotSwap.tick` at the same point of its loop (the epoch tick,
  already a collective point).  ``tick`` broadcasts a 2-word header {version, blob bytes}
  from rank 0; when the version moved, the packed blob follows as one RCCL broadcast with a
  checksum agreement (``dp.broadcast_blob``), and each rank swaps its engine's weights
  between two micro-batches (``StreamEngine.swap_model``: in-flight batches finish on the old
  weights).

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

from .dp import DistContext, broadcast_blob


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
        self.swaps = 0

    def offer(self, model) -> None:
        """Queue ``model`` (same kind as the running one) for the next ``tick``.  Rank ``src``."""
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

    def tick(self) -> bool:
        """Collective on every rank.  Returns True when this call swapped the weights."""
        self._poll_watch()
        dev = self.ctx.device
        with self._lock:
            blob = self._offer if self.ctx.rank == self.src else None
            if self.ctx.rank == self.src:
                self._offer = None
        hdr = torch.zeros(2, dtype=torch.int64, device=dev)
        if self.ctx.rank == self.src and blob is not None:
            hdr[0] = self.version + 1
            hdr[1] = len(blob)
        if self.ctx.initialized:
            dist.broadcast(hdr, self.src, group=self.group)
        new_version, nbytes = int(hdr[0].item()), int(hdr[1].item())
        if new_version <= self.version:
            return False
        t = (torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).to(dev)
             if self.ctx.rank == self.src else None)
        t = broadcast_blob(self.ctx, t, self.src, group=self.group)
        if t.numel() != nbytes:
            raise RuntimeError("hot swap: blob size mismatch after broadcast")
        self._swap(t)
        self.version = new_version
        self.swaps += 1
        return True

    def _swap(self, blob: torch.Tensor) -> None:
        from ..ops.kernels import DeviceModel
        cur = self.engine.dm
        dm = DeviceModel.from_blob(cur.kind, blob, cur.trees, cur.depth, wire=getattr(cur, "wire", False))
        self.engine.swap_model(dm)
