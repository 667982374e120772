"""jBPM prediction service for the investigation User Task (README.md:370-402, 571-581;
deploy/ccd-service.yaml:65-66 ``-Dorg.jbpm.task.prediction.service=SeldonPredictionService``).

For a new "Assign case" task the service asks the user-task model for the most likely
outcome.  If the confidence is >= ``CONFIDENCE_THRESHOLD`` (default 1.0, README.md:395-402)
the task is completed automatically with that outcome; otherwise the outcome is only
pre-filled and the task stays open for the investigator.  ``train()`` receives the
investigator's final outcome (jBPM calls it on task completion); we record it for
retraining the user-task model (train/).

The model is either in-process (UserTaskModel) or remote over the Seldon protocol
(``SELDON_URL``/``SELDON_ENDPOINT`` with ``SELDON_TOKEN``, ``SELDON_TIMEOUT`` ms and
``SELDON_POOL_SIZE`` connections, README.md:372-393).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

import numpy as np

from ..models.usertask import OUTCOMES, UserTaskModel


@dataclass
class PredictionOutcome:
    outcome: Optional[str]
    confidence: float
    present: bool = True

    @property
    def as_dict(self) -> Dict[str, Any]:
        return {"outcome": self.outcome, "confidence": self.confidence}


class PredictionService:
    def __init__(self, confidence_threshold: float = 1.0, model: Optional[UserTaskModel] = None,
                 client=None):
        self.confidence_threshold = float(confidence_threshold)
        self.model = model if (model is not None or client is not None) else UserTaskModel()
        self.client = client
        self.training: List[Dict[str, Any]] = []
        self._lock = threading.Lock()

    def predict(self, task_inputs: Dict[str, Any]) -> PredictionOutcome:
        proba = float(task_inputs.get("proba", task_inputs.get("fraud_probability", 0.0)))
        amount = float(task_inputs.get("amount", 0.0))
        try:
            if self.client is not None:
                from ..contracts import seldon
                F = UserTaskModel.features(proba, amount)
                resp = self.client.predict_sync(seldon.build_request(F, names=["proba_1", "log_amount"]))
                mat, names = seldon.parse_response(resp)
                probs = np.asarray(mat, np.float64).reshape(-1)
                labels = list(names) if names else list(OUTCOMES)
            else:
                probs = self.model.predict_proba(UserTaskModel.features(proba, amount))[0].astype(np.float64)
                labels = list(OUTCOMES)
        except Exception:
            # jBPM semantics: a failing prediction service leaves the task to the human
            return PredictionOutcome(None, 0.0, present=False)
        k = int(np.argmax(probs))
        return PredictionOutcome(labels[k], float(probs[k]))

    def should_auto_complete(self, pred: PredictionOutcome) -> bool:
        return pred.present and pred.confidence >= self.confidence_threshold

    def train(self, task_inputs: Dict[str, Any], outputs: Dict[str, Any]) -> None:
        with self._lock:
            self.training.append({"inputs": dict(task_inputs), "outputs": dict(outputs)})
