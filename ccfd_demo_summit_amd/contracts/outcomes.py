"""Routing decisions and business-process terminal outcomes.

Routes: the Camel/Drools router picks the *standard* or *fraud* process
(README.md:427,552; metric label ``type`` in README.md:525-526).

Fraud BP outcomes (docs/process-fraud.png; README.md:583-605):
  * ``APPROVED_BY_CUSTOMER`` -- customer signalled ``true`` before the timer
  * ``CANCELLED``            -- customer signalled ``false``
  * ``APPROVED_LOW_AMOUNT``  -- timer expired, DMN accepted (low prob and small amount)
  * ``INVESTIGATION``        -- timer expired, DMN -> User Task "Assign case"
Standard BP terminates as ``STANDARD`` (README.md:552).
"""
from __future__ import annotations

import enum


class Route(enum.IntEnum):
    STANDARD = 0
    FRAUD = 1

    @property
    def label(self) -> str:
        return "standard" if self is Route.STANDARD else "fraud"


class Outcome(str, enum.Enum):
    STANDARD = "standard"
    APPROVED_BY_CUSTOMER = "approved_by_customer"
    CANCELLED = "cancelled"
    APPROVED_LOW_AMOUNT = "approved_low_amount"
    INVESTIGATION = "investigation"
    # terminal states of the investigation User Task (prediction service / investigator)
    INVESTIGATION_CLOSED_FRAUD = "investigation_closed_fraud"
    INVESTIGATION_CLOSED_LEGIT = "investigation_closed_legit"


class CustomerResponse(str, enum.Enum):
    """Payload of ``ccd-customer-response`` (README.md:597: ``true`` = made the tx)."""
    APPROVED = "approved"          # metric label notifications_incoming{response="approved"}
    NON_APPROVED = "non_approved"  # README.md:528-530

    @classmethod
    def from_bool(cls, made_tx: bool) -> "CustomerResponse":
        return cls.APPROVED if made_tx else cls.NON_APPROVED
