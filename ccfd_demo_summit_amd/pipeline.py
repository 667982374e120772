"""End-to-end wiring of the whole demo in one process (events-1/2/3):

    producer -> topic odh-demo -> [consume batch] -> scorer (GPU kernels | CPU) -> router
      -> fraud process (KIE replacement) -> topic ccd-customer-outgoing -> notifier
      -> topic ccd-customer-response -> router -> process signal
      -> timer -> DMN -> user task -> prediction service

This is the compat path (JSON or TXB1 messages through a broker); the multi-GPU hot path
is the native engine over pinned partition logs (bench.py / launch/serve.py).  Offsets are
committed only after a batch has been scored and routed (at-least-once); the process
engine ignores duplicate signals.
"""
from __future__ import annotations


import time
from dataclasses import dataclass
from typing import Callable, Dict, Optional


from .config import Config
from .ingest.broker import InProcBroker
from .ingest.codec import decode_records
from .metrics.exporter import MetricsHub
from .process.engine import ProcessEngine
from .process.notifier import NotificationService, encode_notification
from .process.prediction_service import PredictionService
from .router.router import Router
from .router.rules import RuleSet


@dataclass
class PipelineStats:
    consumed: int = 0
    batches: int = 0
    responses: int = 0
    score_s: float = 0.0


class FraudPipeline:
    def __init__(self, cfg: Config, scorer, broker: Optional[InProcBroker] = None,
                 clock: Callable[[], float] = time.monotonic, rules: Optional[RuleSet] = None,
                 metrics: Optional[MetricsHub] = None, journal_path: Optional[str] = None,
                 max_poll: int = 4096):
        self.cfg = cfg
        self.scorer = scorer
        self.broker = broker or InProcBroker(default_partitions=cfg.kafka.partitions)
        self.clock = clock
        self.metrics = metrics or MetricsHub()
        self.max_poll = max_poll
        k = cfg.kafka
        for t in (k.transactions_topic, k.notification_topic, k.response_topic):
            self.broker.create_topic(t)
        self.processes = ProcessEngine(
            cfg.kie.notification_timeout_s, cfg.kie.dmn_probability_threshold, cfg.kie.dmn_amount_threshold,
            publish_notification=self._publish_notification, kie_metrics=self.metrics.kie,
            prediction=PredictionService(cfg.kie.confidence_threshold), clock=clock, journal_path=journal_path)
        self.router = Router(rules or RuleSet.from_config(cfg.router), self.processes,
                             self.metrics.router)
        self.notifier = NotificationService(self._publish_response, cfg.notifier.p_reply, cfg.notifier.p_approve,
                                            cfg.notifier.mean_delay_s, cfg.notifier.seed, clock)
        self.tx_consumer = self.broker.consumer(k.group_id, [k.transactions_topic])
        self.resp_consumer = self.broker.consumer(k.group_id + "-responses", [k.response_topic])
        self.notif_consumer = self.broker.consumer("notification-service", [k.notification_topic])
        self.stats = PipelineStats()

    # ------------------------------------------------------------------ publishers
    def _publish_notification(self, msg: Dict) -> None:
        self.broker.produce(self.cfg.kafka.notification_topic, encode_notification(msg),
                            key=str(msg.get("customer_id")).encode())
        self.router.on_notification_sent(msg)

    def _publish_response(self, raw: bytes, key: Optional[bytes]) -> None:
        self.broker.produce(self.cfg.kafka.response_topic, raw, key=key)

    # ------------------------------------------------------------------ loop
    def step(self, timeout: float = 0.0) -> int:
        """One iteration of every service loop; returns the number of transactions scored."""
        recs = self.tx_consumer.poll(timeout=timeout, max_records=self.max_poll)
        n = 0
        if recs:
            X, ids, cust = decode_records([r.value for r in recs])
            t0 = time.perf_counter()
            proba, route = self.scorer.score(X)
            self.stats.score_s += time.perf_counter() - t0
            self.router.on_scored(ids, cust, proba, X=X, routes=route)
            if len(X):
                self.metrics.model.set_last(X[-1], float(proba[-1]))
            self.tx_consumer.commit()                      # at-least-once: commit after routing
            n = len(X)
            self.stats.consumed += n
            self.stats.batches += 1
        for r in self.notif_consumer.poll(max_records=100_000):
            self.notifier.handle(r.value)
        self.notif_consumer.commit()
        self.notifier.tick()
        for r in self.resp_consumer.poll(max_records=100_000):
            self.router.on_response(r.value)
            self.stats.responses += 1
        self.resp_consumer.commit()
        self.processes.tick()
        return n

    def run_until_idle(self, max_iters: int = 100_000) -> None:
        for _ in range(max_iters):
            n = self.step()
            if n == 0 and self.broker.lag(self.cfg.kafka.group_id, self.cfg.kafka.transactions_topic) == 0 \
                    and self.notifier.pending() == 0 and \
                    self.broker.lag("notification-service", self.cfg.kafka.notification_topic) == 0 and \
                    self.broker.lag(self.cfg.kafka.group_id + "-responses", self.cfg.kafka.response_topic) == 0:
                return

    def close(self):
        for c in (self.tx_consumer, self.resp_consumer, self.notif_consumer):
            c.close()
        self.processes.close()
