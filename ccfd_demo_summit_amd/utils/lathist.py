"""Thread-safe log-bucket latency histogram for the host services' own timings.

Same bucketing as the engine's device histograms (``parallel.dp.hist_quantile``): bucket i
holds ns values in [2^(i/4), 2^((i+1)/4)), 256 buckets, so 1 ns .. ~1.8e19 ns.  Used for the
hand-off attribution (queue wait, request time on the engine side; request arrival, handler
time and event-loop lag on the KIE side), where a p99 has to be split into where it was spent.
"""
from __future__ import annotations

import math
import threading
import time
from typing import Dict, Optional


class LatHist:
    N = 256

    def __init__(self):
        self.h = [0] * self.N
        self.max_ns = 0
        self.max_at = 0.0                    # wall clock (time.time()) of the largest value
        self._lock = threading.Lock()

    def add(self, ns: int, n: int = 1) -> None:
        if ns <= 0 or n <= 0:
            return
        i = min(self.N - 1, int(4.0 * math.log2(ns)))
        with self._lock:
            self.h[i] += n
            if ns > self.max_ns:
                self.max_ns = ns
                self.max_at = time.time()

    def count(self) -> int:
        return sum(self.h)

    def quantile_ns(self, q: float) -> Optional[float]:
        with self._lock:
            h = list(self.h)
        tot = sum(h)
        if not tot:
            return None
        target, c = q * tot, 0
        for i, v in enumerate(h):
            if c + v >= target and v:
                frac = (target - c) / v
                return 2.0 ** ((i + frac) / 4.0)
            c += v
        return 2.0 ** (self.N / 4.0)

    def summary_us(self) -> Dict[str, float]:
        """{"n", "p50", "p99", "max"} in microseconds (p50/p99 interpolated in the bucket), and
        "max_at": the wall-clock second the max was seen (to place it in a run's timeline)."""
        n = self.count()
        if not n:
            return {"n": 0}
        mx = self.max_ns                     # interpolation never reports beyond the max seen
        return {"n": n, "p50": round(min(self.quantile_ns(0.5), mx) / 1e3, 1),
                "p99": round(min(self.quantile_ns(0.99), mx) / 1e3, 1), "max": round(mx / 1e3, 1),
                "max_at": round(self.max_at, 3)}


def merged(hists) -> LatHist:
    """One histogram holding the samples of several (a sharded hand-off's per-shard queues)."""
    m = LatHist()
    for h in hists:
        with h._lock:
            m.h = [a + b for a, b in zip(m.h, h.h)]
            if h.max_ns > m.max_ns:
                m.max_ns, m.max_at = h.max_ns, h.max_at
    return m
