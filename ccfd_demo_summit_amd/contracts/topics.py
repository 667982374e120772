"""Kafka topic names (reference: deploy/router.yaml:57-62, deploy/ccd-service.yaml:57-58,
deploy/kafka/ProducerDeployment.yaml:88-89, README.md:547,560,567).

| topic                     | producer                | consumer            |
|---------------------------|-------------------------|---------------------|
| ``odh-demo``              | transaction producer    | router / engine     |
| ``ccd-customer-outgoing`` | fraud BP notification   | notification svc    |
| ``ccd-customer-response`` | notification svc        | router -> BP signal |
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Topics:
    transactions: str = "odh-demo"                       # KAFKA_TOPIC (router.yaml:61-62)
    customer_outgoing: str = "ccd-customer-outgoing"     # CUSTOMER_NOTIFICATION_TOPIC (router.yaml:57-58)
    customer_response: str = "ccd-customer-response"     # CUSTOMER_RESPONSE_TOPIC (router.yaml:59-60)

    @classmethod
    def from_env(cls, environ=None) -> "Topics":
        e = os.environ if environ is None else environ
        d = cls()
        return cls(
            transactions=e.get("KAFKA_TOPIC", e.get("topic", d.transactions)),
            customer_outgoing=e.get("CUSTOMER_NOTIFICATION_TOPIC", d.customer_outgoing),
            customer_response=e.get("CUSTOMER_RESPONSE_TOPIC", d.customer_response),
        )


DEFAULT_TOPICS = Topics()
