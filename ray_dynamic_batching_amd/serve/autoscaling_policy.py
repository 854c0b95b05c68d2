"""Queue-length autoscaling policy (reference: serve/autoscaling_policy.py:12-156,
serve/_private/autoscaling_state.py).

    error   = total_ongoing / (target_ongoing_requests * running)
    desired = ceil(running * (1 + (error - 1) * smoothing))   smoothing = up/down factor

clamped to [min_replicas, max_replicas]; when the smoothing keeps a downscale
stuck at `running`, step down by one; with 0 running replicas and queued
requests, scale straight to >= 1.  A decision only takes effect after it has
held for upscale_delay_s / downscale_delay_s worth of consecutive control-loop
ticks (CONTROL_LOOP_INTERVAL_S = 0.1 s).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

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
