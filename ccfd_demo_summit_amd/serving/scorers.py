"""Scoring back-ends behind predict() and the compat (JSON-topic) router path.

* ``CpuScorer``  -- NumPy model on the host; config 1 (LR, batch=1) and the CPU oracle.
* ``GpuScorer``  -- the fused HIP kernels through a native StreamEngine slot set
                    (pageable host input is staged by DMA; results come back pinned).

Both return ``(proba_1 float32[n], route uint8[n])`` with route = proba >= threshold.
"""
from __future__ import annotations

import threading
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

    def __init__(self, model, threshold: float = 0.5, max_batch: int = 4096, depth: int = 2,
                 device_index: int = 0):
        import torch
        from ..engine import StreamEngine
        from ..ops.kernels import DeviceModel
        self.threshold = float(threshold)
        self.dm = DeviceModel(model, torch.device("cuda", device_index))
        self.engine = StreamEngine(self.dm, batch=max_batch, depth=depth, streams=1,
                                   input_mode="dma", output_mode="zerocopy", threshold=threshold,
                                   device=device_index)
        self._lock = threading.Lock()

    def score(self, X: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        with self._lock:
            return self.engine.score(X)

    def close(self):
        self.engine.close()


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
