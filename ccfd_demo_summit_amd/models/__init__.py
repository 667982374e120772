"""Model families: logistic regression, 3-layer MLP, oblivious GBDT, user-task model.

Versioned weight files are safetensors (``kind`` + ``version`` in the metadata) --
the replacement for the reference's "model baked into the image, imagePullPolicy
Always" rollout (deploy/model/modelfull.json:24-25; SURVEY.md §5 checkpoint/resume).
"""
from __future__ import annotations

from typing import Union

import numpy as np

from .common import Normalizer, bf16_round, sigmoid
from .gbdt import ObliviousGBDT
from .lr import LogisticModel
from .mlp import MLPModel
from .usertask import UserTaskModel

AnyModel = Union[LogisticModel, MLPModel, ObliviousGBDT]
KINDS = {"lr": LogisticModel, "mlp": MLPModel, "gbdt": ObliviousGBDT}


def build_model(kind: str, seed: int = 0, X_ref=None, calibrate_rate=None, threshold: float = 0.5,
                gbdt_trees: int = 100, gbdt_depth: int = 6) -> AnyModel:
    """Random-init model of the named architecture.  If ``X_ref`` is given the
    normaliser is fitted on it; if ``calibrate_rate`` is given the output bias is shifted
    so that this fraction of ``X_ref`` routes to the fraud process."""
    norm = Normalizer.fit(X_ref) if X_ref is not None else None
    if kind == "lr":
        m = LogisticModel.random_init(seed, norm)
    elif kind == "mlp":
        m = MLPModel.random_init(seed, norm)
    elif kind == "gbdt":
        m = ObliviousGBDT.random_init(gbdt_trees, gbdt_depth, seed, X_ref)
    else:
        raise ValueError(f"unknown model kind {kind!r}")
    if calibrate_rate is not None and X_ref is not None:
        m.calibrate_bias(X_ref, calibrate_rate, threshold)
    return m


def save_model(model: AnyModel, path: str, version: str = "1") -> None:
    from safetensors.numpy import save_file
    st = {k: np.ascontiguousarray(v) for k, v in model.state_dict().items()}
    save_file(st, path, metadata={"kind": model.kind, "version": str(version)})


def load_model(path: str) -> AnyModel:
    from safetensors import safe_open
    with safe_open(path, framework="numpy") as f:
        meta = f.metadata() or {}
        st = {k: f.get_tensor(k) for k in f.keys()}
    kind = meta.get("kind")
    if kind not in KINDS:
        raise ValueError(f"{path}: unknown model kind {kind!r}")
    return KINDS[kind].from_state_dict(st)


__all__ = ["Normalizer", "LogisticModel", "MLPModel", "ObliviousGBDT", "UserTaskModel",
           "build_model", "save_model", "load_model", "KINDS", "bf16_round", "sigmoid"]
