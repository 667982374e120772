"""Customer notification service (replaces ``ruivieira/ccfd-notification-service``,
deploy/notification-service.yaml; README.md:410-422, 556-569; docs/images/events-2).

Consumes ``ccd-customer-outgoing``; "sends" the SMS/e-mail (simulated); the customer
replies with probability ``p_reply`` after an exponential delay (mean ``mean_delay_s``),
approving with probability ``p_approve``; replies go to ``ccd-customer-response``.  The
reference "randomly generate[s] a reply (or no reply)" (README.md:414,565) -- the no-reply
branch is what drives the fraud process's timer path (SURVEY.md §5 fault injection).

Crash safety:

* the customer's behaviour is a pure function of ``(seed, transaction id)`` (the process id
  when a message carries no transaction id): a re-delivered notification gets the SAME reply
  and delay, so a crashed-and-restarted notifier changes no outcome -- and two runs over the
  same input with the same seed end in the same ``kie.outcomes``.  (The transaction id, not
  the process id, is the key: instance ids depend on arrival order at a sharded KIE tier.)
* notifications are deduplicated by process id over a bounded window: the KIE outbox
  re-publishes after a KIE restart, and each process is answered once;
* ``committable()`` is what the consumer may commit: per partition, the lowest offset whose
  reply is not yet acknowledged by the broker (``on_published``).  A crash re-delivers every
  notification whose reply might not have gone out; none is lost.
"""
from __future__ import annotations

import collections
import heapq
import json
import math
import threading
import time
import zlib
from typing import Any, Callable, Dict, List, Optional, Tuple

_M64 = (1 << 64) - 1


def encode_notification(d: Dict[str, Any]) -> bytes:
    return json.dumps(d, separators=(",", ":"), default=float).encode()


def decode_message(raw: bytes) -> Dict[str, Any]:
    return json.loads(raw)


def _mix64(x: int) -> int:
    x &= _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def _uniform(seed: int, key: int, draw: int) -> float:
    """A uniform in [0, 1) that depends only on (seed, key, draw)."""
    x = _mix64(_mix64(seed * 0x9E3779B97F4A7C15 + key) + draw * 0xD1B54A32D192ED03)
    return (x >> 11) * (1.0 / (1 << 53))


def _key(msg: Dict[str, Any], raw: bytes) -> int:
    for k in ("transaction_id", "process_id"):
        v = msg.get(k)
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            return int(v) & _M64
        if isinstance(v, str) and v:
            return zlib.crc32(v.encode()) | (1 << 40)
    return zlib.crc32(raw) | (1 << 41)


Offset = Tuple[str, int, int]                 # (topic, partition, offset) of a consumed message


class NotificationService:
    def __init__(self, publish_response: Callable[..., None], p_reply: float = 0.8,
                 p_approve: float = 0.5, mean_delay_s: float = 0.5, seed: int = 0,
                 clock: Callable[[], float] = time.monotonic, ack_async: bool = False,
                 dedupe_window: int = 1 << 20):
        """``publish_response(raw, key)``; with ``ack_async`` it is ``publish_response(raw, key,
        token)`` and the publisher reports acknowledged tokens to ``on_published`` (a consumed
        offset is committable only after that)."""
        self.publish_response = publish_response
        self.p_reply = p_reply
        self.p_approve = p_approve
        self.mean_delay_s = mean_delay_s
        self.seed = int(seed)
        self.clock = clock
        self.ack_async = bool(ack_async)
        self._pending: List = []
        self._lock = threading.Lock()
        self._seq = 0
        self.sent = 0                          # distinct notifications "sent" to a customer
        self.replied = 0                       # replies handed to the publisher
        self.no_reply = 0
        self.duplicates = 0                    # notifications of an already answered process
        self.published_acked = 0               # replies the broker acknowledged (ack_async)
        self.dedupe_window = int(dedupe_window)
        self._seen: Dict[Any, bool] = {}
        self._seen_order: collections.deque = collections.deque()
        # offsets whose reply is not yet acknowledged, per partition (min-heap + live set)
        self._open: Dict[Tuple[str, int], List[int]] = {}
        self._open_live: Dict[Tuple[str, int], set] = {}
        self._high: Dict[Tuple[str, int], int] = {}    # last handled offset + 1

    # ------------------------------------------------------------------ decisions
    def decide(self, msg: Dict[str, Any], raw: bytes = b"") -> Tuple[bool, bool, float]:
        """(replies?, approves?, delay s): deterministic per (seed, transaction id)."""
        k = _key(msg, raw)
        if _uniform(self.seed, k, 0) >= self.p_reply:
            return False, False, 0.0
        approve = _uniform(self.seed, k, 1) < self.p_approve
        delay = -self.mean_delay_s * math.log1p(-_uniform(self.seed, k, 2)) if self.mean_delay_s > 0 else 0.0
        return True, approve, delay

    # ------------------------------------------------------------------ offsets
    def _open_offset(self, off: Optional[Offset]) -> None:
        if off is None:
            return
        tp = (off[0], off[1])
        heapq.heappush(self._open.setdefault(tp, []), off[2])
        self._open_live.setdefault(tp, set()).add(off[2])

    def _close_offset(self, off: Optional[Offset]) -> None:
        if off is None:
            return
        live = self._open_live.get((off[0], off[1]))
        if live is not None:
            live.discard(off[2])

    def _handled(self, off: Optional[Offset]) -> None:
        if off is not None:
            tp = (off[0], off[1])
            self._high[tp] = max(self._high.get(tp, 0), off[2] + 1)

    def committable(self) -> Dict[Tuple[str, int], int]:
        """Per consumed partition, the offset the consumer may commit: below it every message
        was answered with no reply, or its reply was acknowledged by the broker."""
        out = {}
        with self._lock:
            for tp, high in self._high.items():
                h, live = self._open.get(tp, []), self._open_live.get(tp, set())
                while h and h[0] not in live:
                    heapq.heappop(h)
                out[tp] = h[0] if h else high
        return out

    def on_published(self, tokens) -> None:
        """Publisher thread: these replies (their consumed offsets) are on the topic."""
        with self._lock:
            for off in tokens:
                self._close_offset(off)
            self.published_acked += len(tokens)

    # ------------------------------------------------------------------ messages
    def _seen_before(self, pid) -> bool:
        if pid is None:
            return False
        if pid in self._seen:
            return True
        self._seen[pid] = True
        self._seen_order.append(pid)
        if len(self._seen_order) > self.dedupe_window:
            self._seen.pop(self._seen_order.popleft(), None)
        return False

    def handle(self, raw: bytes, now: Optional[float] = None, offset: Optional[Offset] = None) -> None:
        msg = decode_message(raw)
        now = self.clock() if now is None else now
        with self._lock:
            self._handled(offset)
            if self._seen_before(msg.get("process_id")):
                self.duplicates += 1           # the KIE outbox re-published it: answered once
                return
            self.sent += 1                     # "send" SMS / e-mail
            reply, approve, delay = self.decide(msg, raw)
            if not reply:
                self.no_reply += 1
                return
            resp = {"customer_id": msg.get("customer_id"), "transaction_id": msg.get("transaction_id"),
                    "process_id": msg.get("process_id"), "response": approve}
            self._open_offset(offset)
            self._seq += 1
            heapq.heappush(self._pending, (now + delay, self._seq, resp, offset))

    def tick(self, now: Optional[float] = None) -> int:
        now = self.clock() if now is None else now
        out = []
        with self._lock:
            while self._pending and self._pending[0][0] <= now:
                out.append(heapq.heappop(self._pending))
        for _due, _s, resp, off in out:
            key = str(resp.get("customer_id")).encode()
            if self.ack_async:
                self.publish_response(encode_notification(resp), key, off)
            else:
                self.publish_response(encode_notification(resp), key)
                with self._lock:
                    self._close_offset(off)
            self.replied += 1
        return len(out)

    def pending(self) -> int:
        with self._lock:
            return len(self._pending)

    def stats(self) -> Dict[str, Any]:
        with self._lock:
            return {"sent": self.sent, "replied": self.replied, "no_reply": self.no_reply,
                    "duplicates": self.duplicates, "pending": len(self._pending),
                    "published_acked": self.published_acked}
