"""Queue-length autoscaling policy (reference: serve/autoscaling_policy.py:12-156,
serve/_private/autoscaling_state.py).

    error   = total_ongoing / (target_ongoing_requests * running)
    desired = ceil(running * (1 + (error - 1) * smoothing))   smoothing = up/down factor

clamped to [min_replicas, max_replicas]; when the smoothing keeps a downscale
stuck at `running`, step down by one; with 0 running replicas and queued
requests, scale straight to >= 1.  A decision only takes effect after it has
held for upscale_delay_s / downscale_delay_s worth of consecutive control-loop
ticks (CONTROL_LOOP_INTERVAL_S = 0.1 s).

The request count the policy sees is NOT one instantaneous queue-depth sample:
``AutoscalingMetrics`` samples every replica's ongoing count every
``min(0.5 s, metrics_interval_s)``, and every ``metrics_interval_s`` a replica
"pushes" its average over the last ``look_back_period_s``; the policy sums the
latest pushed averages of the running replicas (plus the handle-queued count
only while no replica runs).  Reference: replica.py:170-230
(_add_autoscaling_metrics_point / _push_autoscaling_metrics),
metrics_utils.py:119-200 (InMemoryMetricsStore.window_average) and
autoscaling_state.py:179-193, 289-300 (record / get_total_num_requests).
"""
from __future__ import annotations

import bisect
import math
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, Hashable, Iterable, List, Optional, Tuple

from .config import CONTROL_LOOP_INTERVAL_S, AutoscalingConfig


def calculate_desired_num_replicas(cfg: AutoscalingConfig, total_num_requests: float, num_running_replicas: int,
                                   override_min_replicas: float = None) -> int:
    lo = cfg.min_replicas if override_min_replicas is None else override_min_replicas
    if num_running_replicas == 0:
        # cold start: any queued work needs a replica
        return max(1 if total_num_requests > 0 else 0, int(lo))
    error_ratio = total_num_requests / (cfg.target_ongoing_requests * num_running_replicas)
    if error_ratio >= 1:
        factor = cfg.get_upscaling_factor()
    else:
        factor = cfg.get_downscaling_factor()
    smoothed = 1 + (error_ratio - 1) * factor
    desired = math.ceil(num_running_replicas * smoothed)
    if error_ratio < 1 and desired == num_running_replicas and num_running_replicas > 0 and smoothed < 1:
        # smoothing made a real downscale round back to "no change"
        desired = num_running_replicas - 1
    return int(min(cfg.max_replicas, max(lo, desired)))


@dataclass
class AutoscalingState:
    cfg: AutoscalingConfig
    decision_counter: int = 0

    def step(self, total_num_requests: float, num_running: int, current_target: int) -> int:
        """One control-loop tick -> new target replica count."""
        desired = calculate_desired_num_replicas(self.cfg, total_num_requests, num_running)
        up_ticks = round(self.cfg.upscale_delay_s / CONTROL_LOOP_INTERVAL_S)
        down_ticks = round(self.cfg.downscale_delay_s / CONTROL_LOOP_INTERVAL_S)
        if num_running == 0 and desired > 0:
            self.decision_counter = 0
            return max(current_target, desired)
        if desired > current_target:
            self.decision_counter = self.decision_counter + 1 if self.decision_counter > 0 else 1
            if self.decision_counter > up_ticks:
                self.decision_counter = 0
                return desired
        elif desired < current_target:
            self.decision_counter = self.decision_counter - 1 if self.decision_counter < 0 else -1
            if -self.decision_counter > down_ticks:
                self.decision_counter = 0
                return desired
        else:
            self.decision_counter = 0
        return current_target


RECORD_PERIOD_S = 0.5     # reference RAY_SERVE_REPLICA_AUTOSCALING_METRIC_RECORD_PERIOD_S


class MetricsStore:
    """Time-stamped samples per key with a window average (reference
    InMemoryMetricsStore): the average of every point at or after the window
    start; the last point before the window stands in when none falls in it."""

    def __init__(self):
        self.data: Dict[Hashable, List[Tuple[float, float]]] = {}

    def add(self, key: Hashable, value: float, ts: float) -> None:
        bisect.insort(self.data.setdefault(key, []), (ts, float(value)))

    def window_average(self, key: Hashable, start: float, compact: bool = True) -> Optional[float]:
        pts = self.data.get(key)
        if not pts:
            return None
        i = bisect.bisect_left(pts, (start, float("-inf")))
        if i >= len(pts):              # nothing new since the window opened: keep the last value
            i = len(pts) - 1
        if compact and i > 0:
            del pts[:i]
            i = 0
        win = pts[i:]
        return sum(v for _, v in win) / len(win)

    def drop(self, key: Hashable) -> None:
        self.data.pop(key, None)


@dataclass
class _Report:
    avg: float
    ts: float


@dataclass
class AutoscalingMetrics:
    """Per-deployment look-back aggregation of replica ongoing-request counts.

    ``tick(now, ongoing_by_replica)`` is called every control-loop tick with the
    current ongoing count of each live replica; it records a sample per replica
    every RECORD_PERIOD_S (capped at metrics_interval_s) and, every
    metrics_interval_s, replaces that replica's report with its window average
    over look_back_period_s.  ``total_num_requests(running, queued_at_handles)``
    is the policy input."""
    cfg: object
    store: MetricsStore = field(default_factory=MetricsStore)
    reports: Dict[Hashable, _Report] = field(default_factory=dict)
    _last_record: Dict[Hashable, float] = field(default_factory=dict)
    _last_push: Dict[Hashable, float] = field(default_factory=dict)

    def record_period(self) -> float:
        return min(RECORD_PERIOD_S, self.cfg.metrics_interval_s)

    def tick(self, now: float, ongoing: Dict[Hashable, float]) -> None:
        for rid, n in ongoing.items():
            if now - self._last_record.get(rid, float("-inf")) >= self.record_period() - 1e-9:
                self.store.add(rid, n, now)
                self._last_record[rid] = now
            if now - self._last_push.get(rid, float("-inf")) >= self.cfg.metrics_interval_s - 1e-9:
                avg = self.store.window_average(rid, now - self.cfg.look_back_period_s)
                if avg is not None:
                    self.reports[rid] = _Report(avg, now)
                self._last_push[rid] = now
        for rid in [r for r in self.reports if r not in ongoing]:   # replica gone
            self.forget(rid)

    def forget(self, rid: Hashable) -> None:
        self.reports.pop(rid, None)
        self.store.drop(rid)
        self._last_record.pop(rid, None)
        self._last_push.pop(rid, None)

    def total_num_requests(self, running: Iterable[Hashable], queued_at_handles: float = 0.0) -> float:
        running = list(running)
        if not running:
            return float(queued_at_handles)
        return sum(self.reports[r].avg for r in running if r in self.reports)
