"""Customer notification service (replaces ``ruivieira/ccfd-notification-service``,
deploy/notification-service.yaml; README.md:410-422, 556-569; docs/images/events-2).

Consumes ``ccd-customer-outgoing``; "sends" the SMS/e-mail (simulated); the customer
replies with probability ``p_reply`` after an exponential delay (mean ``mean_delay_s``),
approving with probability ``p_approve``; replies go to ``ccd-customer-response``.  The
reference "randomly generate[s] a reply (or no reply)" (README.md:414,565) -- the no-reply
branch is what drives the fraud process's timer path (SURVEY.md §5 fault injection).
Seeded RNG and an injected clock keep it deterministic for tests.
"""
from __future__ import annotations

import heapq
import json
import threading
import time
from typing import Any, Callable, Dict, List, Optional

import numpy as np


def encode_notification(d: Dict[str, Any]) -> bytes:
    return json.dumps(d, separators=(",", ":"), default=float).encode()


def decode_message(raw: bytes) -> Dict[str, Any]:
    return json.loads(raw)


class NotificationService:
    def __init__(self, publish_response: Callable[[bytes, Optional[bytes]], None], p_reply: float = 0.8,
                 p_approve: float = 0.5, mean_delay_s: float = 0.5, seed: int = 0,
                 clock: Callable[[], float] = time.monotonic):
        self.publish_response = publish_response
        self.p_reply = p_reply
        self.p_approve = p_approve
        self.mean_delay_s = mean_delay_s
        self.rng = np.random.default_rng(seed)
        self.clock = clock
        self._pending: List = []
        self._lock = threading.Lock()
        self._seq = 0
        self.sent = 0
        self.replied = 0
        self.no_reply = 0

    def handle(self, raw: bytes, now: Optional[float] = None) -> None:
        msg = decode_message(raw)
        now = self.clock() if now is None else now
        self.sent += 1                         # "send" SMS / e-mail
        if self.rng.random() >= self.p_reply:
            self.no_reply += 1
            return
        approve = bool(self.rng.random() < self.p_approve)
        delay = float(self.rng.exponential(self.mean_delay_s)) if self.mean_delay_s > 0 else 0.0
        resp = {"customer_id": msg.get("customer_id"), "transaction_id": msg.get("transaction_id"),
                "process_id": msg.get("process_id"), "response": approve}
        with self._lock:
            self._seq += 1
            heapq.heappush(self._pending, (now + delay, self._seq, resp))

    def tick(self, now: Optional[float] = None) -> int:
        now = self.clock() if now is None else now
        out = []
        with self._lock:
            while self._pending and self._pending[0][0] <= now:
                out.append(heapq.heappop(self._pending)[2])
        for resp in out:
            key = str(resp.get("customer_id")).encode()
            self.publish_response(encode_notification(resp), key)
            self.replied += 1
        return len(out)

    def pending(self) -> int:
        with self._lock:
            return len(self._pending)
