"""End-to-end SLO scheduler runtime on CPU: rate tracking -> squishy plan ->
per-model queues on 2 'GPUs' -> duty-cycle executors -> SLO metrics."""
import time

import numpy as np
import pytest
import torch

from ray_dynamic_batching_amd.models.mlp import MLP
from ray_dynamic_batching_amd.planner import synthetic_profile
from ray_dynamic_batching_amd.planner.scheduler import SLOScheduler
from ray_dynamic_batching_amd.serve.servable import TensorCodec


def make_sched(**kw):
    prof = {"a": synthetic_profile(2, 0.1, 50, 1, batches=range(1, 33)),
            "b": synthetic_profile(3, 0.2, 80, 2, batches=range(1, 33))}
    codecs = {m: TensorCodec((32,), torch.float32, (8,), torch.float32) for m in prof}
    return SLOScheduler(prof, {"a": 200.0, "b": 300.0}, {"a": MLP, "b": lambda: MLP(seed=1)}, codecs, num_gpus=2,
                        monitoring_interval=0.2, **kw)


def test_scheduler_places_models_and_serves_within_slo():
    s = make_sched()
    try:
        x = np.random.rand(32).astype(np.float32)
        rids = []
        # before any plan: requests are held, then flushed once the model is placed
        rids.append(s.submit("a", x))
        s.check_and_update({"a": 100.0, "b": 50.0})
        assert {m for n in s.slots if n for m in n.models()} == {"a", "b"}
        t0 = time.perf_counter()
        for i in range(150):   # ~150 req/s paced arrivals (planned 100 + 50)
            rids.append(s.submit("a" if i % 3 else "b", x))
            time.sleep(max(0.0, t0 + (i + 1) / 150.0 - time.perf_counter()))
        got = {}
        deadline = time.time() + 20
        while len(got) < len(rids) and time.time() < deadline:
            for c in s.poll(1024, 0.1):
                got[c[0]] = c[1]
        assert len(got) == len(rids)
        assert all(st in (0, 1) for st in got.values())
        assert sum(1 for st in got.values() if st == 0) >= 0.9 * len(got)
        st = s.get_stats()
        assert st["a"]["completed"] + st["b"]["completed"] >= 150
        assert st["a"]["slo_violations"] == 0 and st["b"]["slo_violations"] == 0
    finally:
        s.shutdown()


def test_replan_on_rate_change_and_thresholds():
    s = make_sched()
    try:
        assert s.check_and_update({"a": 100.0})
        n1 = len(s.changes)
        assert not s.check_and_update({"a": 103.0})      # +3% < 5%
        assert not s.check_and_update({"a": 92.0})       # -8% < 10% (decreases need 2x)
        assert s.check_and_update({"a": 120.0})          # +20%
        assert len(s.changes) == n1 + 1
        assert s.changes[-1].transfers == 0              # model stays where it was
    finally:
        s.shutdown()


def test_plan_checkpoint_and_resume(tmp_path):
    """every applied plan is checkpointed; a restarted scheduler
    resumes it (same placement) before any rate sample arrives."""
    path = str(tmp_path / "plan.json")
    s = make_sched(plan_path=path)
    try:
        s.check_and_update({"a": 100.0, "b": 50.0})
        before = [n.as_tuples() if n else [] for n in s.slots]
        assert (tmp_path / "plan.json").exists()
    finally:
        s.shutdown()
    s2 = make_sched(plan_path=path)
    try:
        assert [n.as_tuples() if n else [] for n in s2.slots] == before
        assert s2.changes and s2.changes[-1].reason == {"restored": 1.0}
        assert set(s2.sessions) == {"a", "b"}
        # the restored plan serves: requests routed to the placed queues complete
        x = np.random.rand(32).astype(np.float32)
        rid = s2.submit("a", x)
        got = {}
        deadline = time.time() + 10
        while rid not in got and time.time() < deadline:
            for c in s2.poll(64, 0.1):
                got[c[0]] = c[1]
        assert got.get(rid) == 0
        # a plan for a different node shape is refused
        st = s2.plan_state()
        st["num_gpus"] = 3
        assert not s2.restore_plan(st)
    finally:
        s2.shutdown()


def test_stale_requests_are_dropped_with_deadline():
    s = make_sched()
    try:
        s.check_and_update({"a": 10.0})
        x = np.zeros(32, dtype=np.float32)
        rid = s.submit("a", x, deadline_s=1e-7)
        got = {}
        deadline = time.time() + 10
        while rid not in got and time.time() < deadline:
            for c in s.poll(64, 0.1):
                got[c[0]] = c[1]
        assert got[rid] == 1  # DROPPED_STALE
        assert s.get_stats()["a"]["dropped_requests"] >= 1
    finally:
        s.shutdown()
