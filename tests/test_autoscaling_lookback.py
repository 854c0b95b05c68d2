"""Autoscaling over a look-back window, on a fake clock (no cluster).

Mirrors python/ray/serve/tests/unit/test_autoscaling_policy.py (policy cases)
and adds the look-back aggregation the reference performs in the replica
(replica.py:170-230) and controller (autoscaling_state.py:179-193, 289-300):
ongoing counts sampled every min(0.5 s, metrics_interval_s), averaged over
look_back_period_s, pushed every metrics_interval_s."""
import math
import random

import pytest

from ray_dynamic_batching_amd.serve.autoscaling_policy import (AutoscalingMetrics, AutoscalingState, MetricsStore,
                                                               calculate_desired_num_replicas)
from ray_dynamic_batching_amd.serve.config import CONTROL_LOOP_INTERVAL_S, AutoscalingConfig


def test_metrics_store_window_average_and_compaction():
    st = MetricsStore()
    for t, v in [(0.0, 1), (1.0, 3), (2.0, 5), (3.0, 7)]:
        st.add("r", v, t)
    assert st.window_average("r", 1.5, compact=False) == 6.0       # points at 2 and 3
    assert st.window_average("r", 0.0, compact=False) == 4.0
    assert st.window_average("r", 10.0) == 7.0                      # nothing new: last value stands in
    assert st.window_average("missing", 0.0) is None
    st.add("r", 9, 4.0)
    assert st.window_average("r", 3.5) == 9.0
    assert len(st.data["r"]) == 1                                   # compacted


def test_samples_and_pushes_follow_the_configured_periods():
    cfg = AutoscalingConfig(min_replicas=1, max_replicas=10, metrics_interval_s=2.0, look_back_period_s=4.0)
    m = AutoscalingMetrics(cfg)
    now = 0.0
    pushes = []
    while now < 10.0 - 1e-9:
        m.tick(now, {"a": now})              # ongoing == current time: easy to average by hand
        pushes.append(m.reports["a"].ts)
        now = round(now + CONTROL_LOOP_INTERVAL_S, 6)
    assert sorted(set(pushes)) == [0.0, 2.0, 4.0, 6.0, 8.0]
    # at t=8 the store holds samples every 0.5 s; the push averages those in [4, 8]
    assert m.reports["a"].avg == pytest.approx(sum(x * 0.5 for x in range(8, 17)) / 9)
    assert len(m.store.data["a"]) <= (4.0 + 2.0) / 0.5 + 1     # compacted at every push


def test_bursty_load_does_not_flap_the_decision():
    """One raw sample per 0.1 s tick of a bursty queue (2 or 10 ongoing at
    random) swings the policy between 1 and 3 replicas; the look-back average
    over the default 30 s window (about 6, target 4) holds one decision."""
    rng = random.Random(0)
    cfg = AutoscalingConfig(min_replicas=1, max_replicas=10, target_ongoing_requests=4, upscale_delay_s=0.0,
                            downscale_delay_s=0.0, metrics_interval_s=0.5)
    assert cfg.look_back_period_s == 30.0
    m = AutoscalingMetrics(cfg)
    raw, smooth = set(), set()
    now = 0.0
    for i in range(900):
        n = 10 if rng.random() < 0.5 else 2
        m.tick(now, {"r0": n})
        raw.add(calculate_desired_num_replicas(cfg, n, 1))
        if now >= cfg.look_back_period_s:
            smooth.add(calculate_desired_num_replicas(cfg, m.total_num_requests(["r0"]), 1))
        now = round(now + CONTROL_LOOP_INTERVAL_S, 6)
    assert raw == {1, 3}
    assert smooth == {2}


def test_running_zero_uses_handle_queue_and_gone_replicas_are_forgotten():
    cfg = AutoscalingConfig(min_replicas=0, max_replicas=4, metrics_interval_s=1.0, look_back_period_s=2.0)
    m = AutoscalingMetrics(cfg)
    assert m.total_num_requests([], queued_at_handles=7) == 7
    m.tick(0.0, {"a": 4, "b": 2})
    assert m.total_num_requests(["a", "b"]) == 6
    assert m.total_num_requests(["a"]) == 4                          # b not running (yet / any more)
    m.tick(0.1, {"a": 4})
    assert "b" not in m.reports and "b" not in m.store.data


def test_scale_up_over_look_back_then_down_after_delay():
    """Load steps from 40 ongoing to 2: the averaged total falls over the
    look-back window, and the downscale happens only after the delay."""
    cfg = AutoscalingConfig(min_replicas=1, max_replicas=8, target_ongoing_requests=10, upscale_delay_s=0.0,
                            downscale_delay_s=2.0, metrics_interval_s=0.5, look_back_period_s=3.0)
    m, state = AutoscalingMetrics(cfg), AutoscalingState(cfg)
    target, now, history = 1, 0.0, []
    for i in range(200):
        per = 40.0 / target if now < 5.0 else 2.0 / target
        ids = [f"r{k}" for k in range(target)]
        m.tick(now, {r: per for r in ids})
        target = state.step(m.total_num_requests(ids), target, target)
        history.append((now, target))
        now = round(now + CONTROL_LOOP_INTERVAL_S, 6)
    up = next(t for t, n in history if n >= 4)
    assert up <= 0.5
    down = next(t for t, n in history if t > 5.0 and n == 1)
    assert down >= 5.0 + 2.0                      # the delay holds the downscale
    assert history[-1][1] == 1


# -- reference policy cases (test_autoscaling_policy.py) ----------------------------
@pytest.mark.parametrize("delay_s", [0.0, 0.5])
def test_fluctuating_ongoing_requests(delay_s):
    cfg = AutoscalingConfig(min_replicas=1, max_replicas=10, upscale_delay_s=delay_s, downscale_delay_s=delay_s,
                            target_ongoing_requests=50)
    st = AutoscalingState(cfg)
    for trial in range(1000):
        if trial % 2 == 0:
            n = st.step(100, 1, 1)
            assert n == (1 if delay_s > 0 else 2), trial
        else:
            n = st.step(40, 2, 2)
            assert n == (2 if delay_s > 0 else 1), trial


@pytest.mark.parametrize("ongoing", [20, 100, 10])
def test_single_replica_receives_all_requests(ongoing):
    cfg = AutoscalingConfig(min_replicas=1, max_replicas=50, target_ongoing_requests=5, upscale_delay_s=0.0,
                            downscale_delay_s=0.0)
    assert AutoscalingState(cfg).step(ongoing, 4, 4) == ongoing / 5


@pytest.mark.parametrize("target", [0.5, 1.0, 1.5])
def test_scale_up_and_down(target):
    cfg = AutoscalingConfig(min_replicas=0, max_replicas=100, target_ongoing_requests=target)
    assert calculate_desired_num_replicas(cfg, 2 * target * 10, 10) == 20
    assert calculate_desired_num_replicas(cfg, 0.5 * target * 10, 10) == 5
    assert math.isclose(calculate_desired_num_replicas(cfg, target * 10, 10), 10)
