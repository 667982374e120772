"""Business processes (KIE replacement): fraud/standard BP, DMN, prediction service, notifier."""
from .dmn import Decision, investigation_decision, investigation_decision_batch
from .engine import ProcessEngine, ProcessInstance, State, UserTask
from .notifier import NotificationService
from .prediction_service import PredictionOutcome, PredictionService

__all__ = ["Decision", "investigation_decision", "investigation_decision_batch", "ProcessEngine",
           "ProcessInstance", "State", "UserTask", "NotificationService", "PredictionOutcome",
           "PredictionService"]
