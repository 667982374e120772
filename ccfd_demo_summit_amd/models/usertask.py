"""User-task outcome model (replaces ``ruivieira/ccfd-seldon-usertask-model``, README.md:347-353).

The jBPM prediction service asks it, for an open "Assign case" investigation task, what
the investigator's outcome will be and how confident it is (README.md:571-581).  The
reference image's internals are not available; we model it as a small logistic model over
task features ``[proba_1, log1p(amount)]`` returning class probabilities for the outcomes
``["approved", "rejected"]`` (Seldon ``ndarray`` with those ``names``).  The prediction
service takes the arg-max as outcome and the max as confidence ([EXT] assumption about
``SeldonPredictionService`` parsing).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .common import sigmoid

OUTCOMES = ("approved", "rejected")


@dataclass
class UserTaskModel:
    w: np.ndarray = None
    b: float = 0.0
    kind: str = "usertask"

    def __post_init__(self):
        if self.w is None:
            # high fraud probability and high amount -> more likely "rejected"
            self.w = np.array([6.0, 0.4], np.float32)
            self.b = -4.0

    @staticmethod
    def features(proba_1, amount) -> np.ndarray:
        p = np.asarray(proba_1, np.float32).reshape(-1)
        a = np.asarray(amount, np.float32).reshape(-1)
        return np.stack([p, np.log1p(np.maximum(a, 0))], axis=1)

    def predict_proba(self, F: np.ndarray) -> np.ndarray:
        """Returns [n, 2] probabilities over OUTCOMES."""
        F = np.asarray(F, np.float32)
        if F.ndim == 1:
            F = F.reshape(1, -1)
        p_rej = sigmoid(F[:, :2].astype(np.float64) @ self.w.astype(np.float64) + self.b)
        return np.stack([1.0 - p_rej, p_rej], axis=1).astype(np.float32)

    def state_dict(self) -> dict:
        return {"usertask.w": self.w, "usertask.b": np.array([self.b], np.float32)}
