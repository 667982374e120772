"""Scoring back-ends behind predict() and the compat (JSON-topic) router path.

* ``CpuScorer``  -- NumPy model on the host; config 1 (LR, batch=1) and the CPU oracle.
* ``GpuScorer``  -- the fused HIP kernels through a native StreamEngine slot set
                    (pageable host input is staged by DMA; results come back pinned).

Both return ``(proba_1 float32[n], route uint8[n])`` with route = proba >= threshold.
"""
from __future__ import annotations

import threading
import weakref
from typing import Tuple

import numpy as np


class CpuScorer:
    device = "cpu"

    def __init__(self, model, threshold: float = 0.5):
        self.model = model
        self.threshold = float(threshold)

    def score(self, X: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        p = self.model.predict_proba(np.asarray(X, np.float32)).astype(np.float32)
        return p, (p >= self.threshold).astype(np.uint8)


class GpuScorer:
    device = "gpu"
    _resident = weakref.WeakSet()            # persistent scorers of this process

    def __init__(self, model, threshold: float = 0.5, max_batch: int = 4096, depth: int = 2,
                 device_index: int = 0, exec_mode: str = "launch"):
        """``exec_mode="persistent"`` (MLP / LR): the scoring kernel stays resident between
        requests and a call is a descriptor post instead of a kernel launch.  It holds one of
        the process's GPU_MAX_HW_QUEUES hardware queues while the scorer lives."""
        import torch
        from ..engine import StreamEngine
        from ..ops.kernels import DeviceModel
        self.threshold = float(threshold)
        self.dm = DeviceModel(model, torch.device("cuda", device_index))
        if exec_mode == "persistent" and getattr(model, "kind", None) == "gbdt":
            exec_mode = "launch"                   # the persistent GBDT kernel reads G32 rows only
        self.engine = StreamEngine(self.dm, batch=max_batch, depth=depth, streams=1,
                                   input_mode="dma", output_mode="zerocopy", threshold=threshold,
                                   device=device_index, exec_mode=exec_mode)
        self.exec_mode = exec_mode
        self._lock = threading.Lock()
        if exec_mode == "persistent":
            self.engine.keep_resident(True)
            GpuScorer._resident.add(self)

    def score(self, X: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        with self._lock:
            return self.engine.score(X)

    def close(self):
        # hipFree synchronises the device and a resident kernel never finishes: halt every
        # resident scorer of the process first (each under its lock, so not mid-request; the
        # next request relaunches its kernel), then free this one
        for sc in list(GpuScorer._resident):
            with sc._lock:
                if sc.engine is not None:
                    sc.engine.halt()
        GpuScorer._resident.discard(self)
        with self._lock:
            if self.engine is not None:
                self.engine.close()
                self.engine = None


def make_scorer(model, threshold: float = 0.5, device: str = "auto", **kw):
    if device in ("auto", "gpu"):
        try:
            import torch
            if torch.cuda.is_available() and getattr(model, "kind", None) in ("lr", "mlp", "gbdt"):
                return GpuScorer(model, threshold, **kw)
        except Exception:
            if device == "gpu":
                raise
        if device == "gpu":
            raise RuntimeError("GPU scorer requested but no GPU is available")
    return CpuScorer(model, threshold)
