"""DMN "Start investigation" decision of the fraud process (README.md:592-596).

"If the fraud probability is below a certain threshold, and the transaction amount is
sufficiently small, it is accepted.  If the transaction amount is large or the
probability is above a certain threshold, the BP proceeds with the creation of a User
Task, assigned to a fraud investigator."  The numeric thresholds are not in the
reference; they are config (KieConfig.dmn_probability_threshold / dmn_amount_threshold).
Also vectorised for the batch path.
"""
from __future__ import annotations

import enum

import numpy as np


class Decision(str, enum.Enum):
    APPROVE = "approve"
    INVESTIGATE = "investigate"


def investigation_decision(proba: float, amount: float, p_threshold: float, amount_threshold: float) -> Decision:
    if proba < p_threshold and amount < amount_threshold:
        return Decision.APPROVE
    return Decision.INVESTIGATE


def investigation_decision_batch(proba: np.ndarray, amount: np.ndarray, p_threshold: float,
                                 amount_threshold: float) -> np.ndarray:
    """True where the DMN sends the transaction to investigation."""
    proba = np.asarray(proba)
    amount = np.asarray(amount)
    return ~((proba < p_threshold) & (amount < amount_threshold))
