"""Synthetic request-rate patterns and load drivers.

Reference generators:
* test_scheduler.py:57-96 WorkloadGenerator -- linear ramp rate = elapsed*slope
  (then hold), fired once per second (and, by mistake, synchronously);
* venkat-code/test_scheduler.py:67-153,323-361 -- sinusoidal, step, random,
  spike, constant patterns;
* milind-code/request_simulator.py -- per-model sender threads at 1/rate
  spacing with live rate changes (rate 0 stops).
Here a pattern is a pure function rate(t); ``PatternDriver`` runs patterns on
real threads with Poisson or uniform arrivals and accepts live rate overrides.
The native closed/open-loop generator for throughput runs is runtime LoadGen.
"""
from __future__ import annotations

import math
import random
import threading
import time
from dataclasses import dataclass
from typing import Callable, Dict, Optional


@dataclass
class Pattern:
    kind: str = "constant"
    base: float = 10.0
    amplitude: float = 0.0
    period_s: float = 60.0
    slope: float = 1.0          # ramp: req/s per second
    ramp_s: float = 40.0        # ramp: hold after this
    step_at_s: float = 30.0
    step_to: float = 20.0
    spike_at_s: float = 30.0
    spike_len_s: float = 5.0
    spike_rate: float = 100.0
    seed: int = 0

    def rate(self, t: float) -> float:
        k = self.kind
        if k == "constant":
            return self.base
        if k == "ramp":
            return self.base + self.slope * min(t, self.ramp_s)
        if k == "sinusoidal":
            return max(0.0, self.base + self.amplitude * math.sin(2 * math.pi * t / self.period_s))
        if k == "step":
            return self.base if t < self.step_at_s else self.step_to
        if k == "spike":
            return self.spike_rate if self.spike_at_s <= t < self.spike_at_s + self.spike_len_s else self.base
        if k == "random":
            # piecewise-constant random rate, new value every period_s (deterministic per seed)
            rng = random.Random(self.seed * 1000003 + int(t // self.period_s))
            return max(0.0, self.base + self.amplitude * (2 * rng.random() - 1))
        raise ValueError(f"unknown pattern {k!r}")


PATTERNS = ("constant", "ramp", "sinusoidal", "step", "spike", "random")


class PatternDriver:
    """Fire requests for several models following their patterns.

    submit(model) is called once per request (any callable: a serve handle's
    remote, SLOScheduler.submit, ...).  Arrivals are Poisson (default) or
    evenly spaced.  ``set_rate(model, r)`` overrides a pattern live (r=0 stops
    that model), like the fork's interactive simulator."""

    def __init__(self, submit: Callable[[str], object], patterns: Dict[str, Pattern], poisson: bool = True,
                 seed: int = 0):
        self.submit = submit
        self.patterns = dict(patterns)
        self.poisson = poisson
        self.overrides: Dict[str, Optional[float]] = {}
        self.sent: Dict[str, int] = {m: 0 for m in patterns}
        self._stop = threading.Event()
        self._threads = []
        self._rng = random.Random(seed)
        self.t0 = 0.0

    def set_rate(self, model: str, rate: Optional[float]) -> None:
        self.overrides[model] = rate

    def rate(self, model: str, t: float) -> float:
        o = self.overrides.get(model)
        return o if o is not None else self.patterns[model].rate(t)

    def _run(self, model: str, duration_s: float) -> None:
        rng = random.Random(self._rng.random())
        next_t = 0.0
        while not self._stop.is_set():
            now = time.perf_counter() - self.t0
            if now >= duration_s:
                return
            r = self.rate(model, now)
            if r <= 0:
                self._stop.wait(0.05)
                next_t = time.perf_counter() - self.t0
                continue
            gap = rng.expovariate(r) if self.poisson else 1.0 / r
            next_t = max(next_t, now - 1.0) + gap   # bounded catch-up after stalls
            wait = next_t - (time.perf_counter() - self.t0)
            if wait > 0:
                self._stop.wait(wait)
            if self._stop.is_set():
                return
            self.submit(model)
            self.sent[model] += 1

    def start(self, duration_s: float) -> "PatternDriver":
        self.t0 = time.perf_counter()
        for m in self.patterns:
            t = threading.Thread(target=self._run, args=(m, duration_s), daemon=True, name=f"load-{m}")
            t.start()
            self._threads.append(t)
        return self

    def join(self, timeout: Optional[float] = None) -> None:
        for t in self._threads:
            t.join(timeout)

    def stop(self) -> None:
        self._stop.set()
        self.join(2)
