"""Request-rate tracking.

Reference: scheduler.py:115-179 RequestTracker -- its get_rate() RESETS the
window once it has elapsed, so every caller (monitor thread, metrics thread)
perturbs the estimate.  Here the rate is a pure read over a sliding window of
time buckets; recording is O(1) and thread-safe.
"""
from __future__ import annotations

import threading
import time
from typing import Callable, Optional


class RateTracker:
    def __init__(self, window_s: float = 1.0, bucket_s: float = 0.05, clock: Optional[Callable[[], float]] = None):
        self.window_s = window_s
        self.bucket_s = bucket_s
        self.n = max(1, int(round(window_s / bucket_s)))
        self.counts = [0] * self.n
        self.stamp = [-1] * self.n
        self.total = 0
        self._clock = clock or time.monotonic
        self._start = self._clock()
        self._lock = threading.Lock()

    def record(self, n: int = 1) -> None:
        t = int(self._clock() / self.bucket_s)
        i = t % self.n
        with self._lock:
            if self.stamp[i] != t:
                self.stamp[i] = t
                self.counts[i] = 0
            self.counts[i] += n
            self.total += n

    def rate(self) -> float:
        """Requests/s over the last window (shorter right after start)."""
        now = self._clock()
        t = int(now / self.bucket_s)
        with self._lock:
            c = sum(cnt for cnt, st in zip(self.counts, self.stamp) if t - self.n < st <= t)
        span = min(self.window_s, max(now - self._start, self.bucket_s))
        return c / span

    def total_requests(self) -> int:
        return self.total
