"""Deployment / handle / router / controller tests (local and process mode, CPU)."""
import time

import numpy as np
import pytest

from ray_dynamic_batching_amd import serve
from ray_dynamic_batching_amd.serve.autoscaling_policy import AutoscalingState, calculate_desired_num_replicas
from ray_dynamic_batching_amd.serve.config import AutoscalingConfig, DeploymentConfig


@pytest.fixture(autouse=True)
def _shutdown():
    yield
    serve.shutdown()


def test_config_schema_compatible_fields():
    c = DeploymentConfig(num_replicas=2, max_ongoing_requests=7, ray_actor_options={"num_gpus": 0.5},
                         slo_ms=40.0, health_check_period_s=1)
    assert c.initial_num_replicas() == 2 and c.num_gpus == 0.5
    with pytest.raises(ValueError):
        DeploymentConfig(max_ongoing_requests=0)
    with pytest.raises(ValueError):
        DeploymentConfig(max_queued_requests=0)
    with pytest.raises(ValueError):
        DeploymentConfig(ray_actor_options={"num_gpus": 1.5})
    a = DeploymentConfig(num_replicas="auto")
    assert a.autoscaling_config is not None
    with pytest.raises(ValueError):
        AutoscalingConfig(min_replicas=3, max_replicas=2)


def test_deployment_decorator_and_options():
    @serve.deployment(num_replicas=3, max_ongoing_requests=11)
    class A:
        pass
    assert A.name == "A" and A.num_replicas == 3 and A.max_ongoing_requests == 11
    B = A.options(name="B", num_replicas=1, user_config={"x": 1})
    assert B.name == "B" and B.num_replicas == 1 and B.user_config == {"x": 1}
    with pytest.raises(TypeError):
        A.options(not_a_field=1)
    with pytest.raises(RuntimeError):
        A()


def test_mlp_plumbing_two_replicas_local():
    """BASELINE config 1: 2-layer MLP, 2 CPU replicas, dyn-batch <= 4 / 10 ms."""
    import torch

    from ray_dynamic_batching_amd.models.mlp import MLP

    @serve.deployment(num_replicas=2, max_ongoing_requests=16)
    class MLPDep:
        def __init__(self):
            self.m = MLP()
            self.sizes = []

        @serve.batch(max_batch_size=4, batch_wait_timeout_s=0.01)
        async def __call__(self, xs):
            self.sizes.append(len(xs))
            return list(self.m(torch.stack(xs)).unbind(0))

        def batch_sizes(self):
            return self.sizes

    h = serve.run(MLPDep.bind(), _local_testing_mode=True)
    m = MLP()
    xs = m.example_input(32)
    outs = [h.remote(xs[i]) for i in range(32)]
    got = torch.stack([o.result() for o in outs])
    assert torch.allclose(got, m(xs), atol=1e-5)
    sizes = [h.batch_sizes.remote().result() for _ in range(8)]
    flat = [s for ss in sizes for s in ss]
    assert max(flat) <= 4 and max(flat) > 1


def test_handle_methods_await_composition_and_function_deployment():
    @serve.deployment
    def double(x):
        return 2 * x

    @serve.deployment
    class Adder:
        def __init__(self, doubler):
            self.doubler = doubler

        async def __call__(self, x):
            return await self.doubler.remote(x) + 1

        def plain(self, x):
            return x - 1

    h = serve.run(Adder.bind(double.bind()), _local_testing_mode=True)
    assert h.remote(5).result() == 11
    assert h.plain.remote(5).result() == 4
    assert h.options(method_name="plain").remote(7).result() == 6

    import asyncio

    async def go():
        return await h.remote(1)
    assert asyncio.new_event_loop().run_until_complete(go()) == 3
    # composition: pass a response as an argument
    d = serve.get_deployment_handle("double", "default")
    assert h.plain.remote(d.remote(10)).result() == 19


def test_streaming_handle_local():
    @serve.deployment
    class G:
        def stream(self, n):
            for i in range(n):
                yield i * i

    h = serve.run(G.bind(), _local_testing_mode=True)
    assert list(h.options(method_name="stream", stream=True).remote(4)) == [0, 1, 4, 9]


def test_max_ongoing_and_backpressure():
    import threading

    gate = threading.Event()

    @serve.deployment(max_ongoing_requests=1, max_queued_requests=1)
    class Slow:
        def __call__(self):
            gate.wait(5)
            return "ok"

    h = serve.run(Slow.bind(), _local_testing_mode=True)
    r1 = h.remote()
    time.sleep(0.1)
    r2 = h.remote()         # queued at the router
    time.sleep(0.1)
    r3 = h.remote()         # exceeds max_queued_requests
    with pytest.raises(serve.BackPressureError):
        r3.result(timeout_s=2)
    gate.set()
    assert r1.result(timeout_s=5) == "ok" and r2.result(timeout_s=5) == "ok"


def test_pow2_router_balances_local():
    @serve.deployment(num_replicas=4, max_ongoing_requests=100)
    class Who:
        def __call__(self):
            time.sleep(0.002)
            return serve.get_replica_context().replica_index

    h = serve.run(Who.bind(), _local_testing_mode=True)
    counts = {}
    rs = [h.remote() for _ in range(200)]
    for r in rs:
        i = r.result()
        counts[i] = counts.get(i, 0) + 1
    assert len(counts) == 4 and min(counts.values()) > 20


def test_user_config_reconfigure_and_status():
    @serve.deployment(user_config={"k": 5})
    class U:
        def reconfigure(self, cfg):
            self.k = cfg["k"]

        def __call__(self):
            return self.k

    h = serve.run(U.bind(), name="app1", _local_testing_mode=True)
    assert h.remote().result() == 5
    st = serve.status()["applications"]["app1"]
    assert st["deployments"]["U"]["status"] == "HEALTHY"
    assert serve.get_app_handle("app1").remote().result() == 5
    serve.delete("app1")
    assert "app1" not in serve.status()["applications"]


def test_multiplexing_lru_and_affinity():
    @serve.deployment(num_replicas=1)
    class Mux:
        def __init__(self):
            self.loads = []

        @serve.multiplexed(max_num_models_per_replica=2)
        async def get_model(self, model_id):
            self.loads.append(model_id)
            return f"model-{model_id}"

        async def __call__(self):
            mid = serve.get_multiplexed_model_id()
            return await self.get_model(mid)

        def loaded(self):
            return self.loads

    h = serve.run(Mux.bind(), _local_testing_mode=True)
    for mid in ["a", "b", "a", "c", "a", "b"]:
        assert h.options(multiplexed_model_id=mid).remote().result() == f"model-{mid}"
    # capacity 2: a, b loaded; c evicts b (LRU: a was used more recently); b reload evicts c
    assert h.loaded.remote().result() == ["a", "b", "c", "b"]


def test_autoscaling_policy_math():
    cfg = AutoscalingConfig(min_replicas=1, max_replicas=10, target_ongoing_requests=2, upscale_delay_s=0,
                            downscale_delay_s=0)
    assert calculate_desired_num_replicas(cfg, 20, 2) == 10        # 5x overloaded, capped
    assert calculate_desired_num_replicas(cfg, 8, 2) == 4
    assert calculate_desired_num_replicas(cfg, 2, 4) == 1
    assert calculate_desired_num_replicas(cfg, 0, 0) == 1
    cfg2 = AutoscalingConfig(min_replicas=0, max_replicas=5, target_ongoing_requests=1, downscale_smoothing_factor=0.1)
    assert calculate_desired_num_replicas(cfg2, 3, 4) == 3         # smoothing stuck -> step down by one
    s = AutoscalingState(AutoscalingConfig(min_replicas=1, max_replicas=5, target_ongoing_requests=1,
                                           upscale_delay_s=0.3, downscale_delay_s=0.5))
    tgt = 1
    ticks = 0
    while tgt == 1:
        tgt = s.step(10, 1, tgt)
        ticks += 1
    assert tgt == 5 and ticks == 4  # delay 0.3 s = 3 ticks, decision on the 4th


def test_autoscaling_local_scales_up_and_down():
    import threading

    gate = threading.Event()

    @serve.deployment(max_ongoing_requests=2, autoscaling_config=dict(
        min_replicas=1, max_replicas=3, target_ongoing_requests=1, upscale_delay_s=0.0, downscale_delay_s=0.3,
        metrics_interval_s=0.1, look_back_period_s=0.3))
    class AS:
        def __call__(self):
            gate.wait(10)
            return 1

    h = serve.run(AS.bind(), _local_testing_mode=True)
    rs = [h.remote() for _ in range(6)]
    deadline = time.time() + 5
    while time.time() < deadline and serve.status()["applications"]["default"]["deployments"]["AS"]["target_replicas"] < 3:
        time.sleep(0.05)
    assert serve.status()["applications"]["default"]["deployments"]["AS"]["target_replicas"] == 3
    gate.set()
    assert sum(r.result(timeout_s=10) for r in rs) == 6
    deadline = time.time() + 5
    while time.time() < deadline and serve.status()["applications"]["default"]["deployments"]["AS"]["target_replicas"] > 1:
        time.sleep(0.05)
    assert serve.status()["applications"]["default"]["deployments"]["AS"]["target_replicas"] == 1


def test_unhealthy_replica_is_replaced_local():
    @serve.deployment(num_replicas=1, health_check_period_s=0.05, health_check_timeout_s=1)
    class H:
        def __init__(self):
            self.calls = 0

        def check_health(self):
            self.calls += 1
            if self.calls >= 2:
                raise RuntimeError("sick")

        def __call__(self):
            return id(self)

    h = serve.run(H.bind(), _local_testing_mode=True)
    first = h.remote().result()
    deadline = time.time() + 5
    while time.time() < deadline and h.remote().result() == first:
        time.sleep(0.05)
    assert h.remote().result() != first


def test_logging_config_validation_and_app_default():
    from ray_dynamic_batching_amd.serve.logging_utils import LoggingConfig

    with pytest.raises(Exception):
        serve.deployment(logging_config={"encoding": "XML"})(lambda x: x)
    with pytest.raises(Exception):
        LoggingConfig(log_level="LOUD")
    d = serve.deployment(logging_config=LoggingConfig(encoding="json", log_level="DEBUG"))(lambda x: x)
    assert d.config.logging_config["encoding"] == "JSON"
    assert d.config.get_logging_config().level() == 10


def test_access_log_text_and_json_local(tmp_path):
    """Per-replica component log + one access-log line per request (reference
    replica.py:430-437, logging_utils.py:274); JSON encoding carries the
    request fields; enable_access_log=False silences it; serve.run's
    logging_config is the application default."""
    import json as _json
    import logging as _logging

    @serve.deployment(num_replicas=1)
    class Greeter:
        def __call__(self, x):
            _logging.getLogger("ray.serve.replica.default.Greeter.0").warning("user says %s", x)
            return f"hi {x}"

        def boom(self):
            raise ValueError("no")

    h = serve.run(Greeter.bind(), _local_testing_mode=True,
                  logging_config={"encoding": "JSON", "logs_dir": str(tmp_path)})
    assert h.remote("a").result() == "hi a"
    with pytest.raises(ValueError):
        h.boom.remote().result()
    path = tmp_path / "replica_default_Greeter_0.log"
    lines = [_json.loads(line) for line in path.read_text().splitlines()]
    access = [x for x in lines if "latency_ms" in x]
    assert [(x["method"], x["status"]) for x in access] == [("__call__", "OK"), ("boom", "ERROR")]
    assert all(x["deployment"] == "Greeter" and x["replica"] == "default#Greeter#0" for x in lines)
    assert any(x["message"] == "user says a" for x in lines)
    serve.shutdown()

    @serve.deployment(logging_config={"enable_access_log": False, "logs_dir": str(tmp_path / "quiet")})
    class Quiet:
        def __call__(self, x):
            return x

    h = serve.run(Quiet.bind(), _local_testing_mode=True)
    assert h.remote(1).result() == 1
    assert (tmp_path / "quiet" / "replica_default_Quiet_0.log").read_text() == ""
    serve.shutdown()

    @serve.deployment(logging_config={"encoding": "TEXT", "logs_dir": str(tmp_path / "t")})
    class Texty:
        def __call__(self, x):
            return x

    h = serve.run(Texty.bind(), _local_testing_mode=True)
    h.remote(2).result()
    txt = (tmp_path / "t" / "replica_default_Texty_0.log").read_text()
    assert "Texty default#Texty#0" in txt and "CALL __call__ OK" in txt and "ms" in txt
