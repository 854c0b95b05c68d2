"""Process-mode serving on CPU: replica processes + shm rings (no GPU needed)."""
import os
import signal
import time

import pytest

from ray_dynamic_batching_amd import serve


@pytest.fixture(autouse=True)
def _shutdown():
    yield
    serve.shutdown()


@serve.deployment(num_replicas=2, max_ongoing_requests=16)
class Echo:
    def __init__(self, k):
        self.k = k

    @serve.batch(max_batch_size=4, batch_wait_timeout_s=0.01)
    async def __call__(self, xs):
        return [x * self.k for x in xs]

    def pid(self):
        return os.getpid()

    def stream(self, n):
        for i in range(n):
            yield i

    def fail(self):
        raise KeyError("nope")


def test_process_mode_roundtrip_stream_errors():
    h = serve.run(Echo.bind(7), mode="process")
    rs = [h.remote(i) for i in range(50)]
    assert [r.result(timeout_s=20) for r in rs] == [7 * i for i in range(50)]
    pids = {h.pid.remote().result(timeout_s=10) for _ in range(20)}
    assert len(pids) == 2 and os.getpid() not in pids
    assert list(h.options(method_name="stream", stream=True).remote(5)) == [0, 1, 2, 3, 4]
    with pytest.raises(KeyError):
        h.fail.remote().result(timeout_s=10)
    st = serve.status()["applications"]["default"]["deployments"]["Echo"]
    assert st["mode"] == "process" and st["running_replicas"] == 2
    assert sum(r["queue"]["completed"] for r in st["replicas"]) >= 50


@serve.deployment(num_replicas=1)
class Down:
    def __call__(self, x):
        return x + 1


@serve.deployment(num_replicas=1)
class Up:
    def __init__(self, down):
        self.down = down

    async def __call__(self, x):
        return await self.down.remote(x) * 10


def test_process_mode_composition_across_processes():
    h = serve.run(Up.bind(Down.bind()), mode="process")
    assert h.remote(4).result(timeout_s=20) == 50


def test_replica_crash_is_restarted_and_requests_retried():
    h = serve.run(Echo.options(num_replicas=1, health_check_timeout_s=2).bind(2), mode="process")
    pid = h.pid.remote().result(timeout_s=10)
    os.kill(pid, signal.SIGKILL)
    t = time.time()
    # a request sent while the replica is dead is retried after the restart
    assert h.remote(21).result(timeout_s=60) == 42
    new_pid = h.pid.remote().result(timeout_s=10)
    assert new_pid != pid
    st = serve.status()["applications"]["default"]["deployments"]["Echo"]
    assert st["replicas"][0]["restarts"] >= 1


_CRASHING_DRIVER = r"""
import os, sys
sys.path.insert(0, {repo!r})
from ray_dynamic_batching_amd import serve

@serve.deployment(num_replicas=2, max_ongoing_requests=16)
class Scaled:
    def __init__(self, k):
        self.k = k

    def __call__(self, x):
        return x * self.k

h = serve.run(Scaled.bind(3), name="calc", route_prefix="/calc", mode="process")
assert h.remote(5).result(timeout_s=30) == 15
# a later options() change is part of the checkpointed config
h = serve.run(Scaled.options(num_replicas=1).bind(4), name="calc", route_prefix="/calc", mode="process")
assert h.remote(5).result(timeout_s=30) == 20
print("deployed", flush=True)
os._exit(0)          # controller dies: no shutdown, no checkpoint clean-up
"""


def test_controller_recovers_applications_from_checkpoint(tmp_path, monkeypatch):
    """A controller started on the same checkpoint location (RDB_SERVE_KV:
    the agent's persistent KV + JSON, the GCS-KV role) after the previous one
    died redeploys its applications -- graph, configs, route prefix, mode
    (reference serve/_private/controller.py:510-563)."""
    import subprocess
    import sys

    kv = str(tmp_path / "serve_kv.json")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RDB_SERVE_KV=kv, RDB_SERVE_DISCOVERY=str(tmp_path / "disc.json"))
    r = subprocess.run([sys.executable, "-c", _CRASHING_DRIVER.format(repo=repo)], env=env,
                       capture_output=True, text=True, timeout=180)
    assert "deployed" in r.stdout, r.stdout + r.stderr
    assert os.path.exists(kv) and os.path.exists(kv + ".agent.bin")
    monkeypatch.setenv("RDB_SERVE_KV", kv)
    monkeypatch.setenv("RDB_SERVE_DISCOVERY", str(tmp_path / "disc2.json"))
    from ray_dynamic_batching_amd.serve.controller import get_controller

    ctrl = get_controller()
    assert ctrl.recovered == ["calc"]
    h = serve.get_app_handle("calc")
    assert h.remote(6).result(timeout_s=30) == 24          # the later config (k=4) came back
    st = serve.status()["applications"]["calc"]["deployments"]["Scaled"]
    assert st["mode"] == "process" and st["running_replicas"] == 1
    assert ctrl.route_prefixes["calc"] == "/calc"
    # an explicit shutdown empties the checkpoint: the next controller starts clean
    serve.shutdown()
    assert get_controller().recovered == []


def test_controller_recovery_disabled(tmp_path, monkeypatch):
    from ray_dynamic_batching_amd.serve.controller import ServeController

    monkeypatch.setenv("RDB_SERVE_KV", str(tmp_path / "kv.json"))
    monkeypatch.setenv("RDB_SERVE_DISCOVERY", str(tmp_path / "d.json"))
    serve.run(Down.bind(), name="d1", mode="local")
    assert serve.get_app_handle("d1").remote(1).result(timeout_s=10) == 2
    doc = serve.api._controller().read_checkpoint()
    assert "d1" in doc["applications"] and doc["applications"]["d1"]["app"].get("pickle")


@serve.deployment(num_replicas=3, max_ongoing_requests=8)
class MuxModels:
    def __init__(self):
        self.loads = 0

    @serve.multiplexed(max_num_models_per_replica=2)
    async def get_model(self, model_id):
        self.loads += 1
        return f"{model_id}@{os.getpid()}"

    async def __call__(self):
        return await self.get_model(serve.get_multiplexed_model_id())

    def num_loads(self):
        return self.loads


def test_process_mode_multiplexed_affinity_through_native_router():
    """Replicas publish the multiplexed ids they hold into their shm queue
    state; the native router sends a request for a held id to that replica
    (reference pow_2_scheduler.py:396-443), so each model loads once."""
    h = serve.run(MuxModels.bind(), name="mux", mode="process")
    where = {}
    for rnd in range(6):
        for mid in ("m1", "m2", "m3"):
            out = h.options(multiplexed_model_id=mid).remote().result(timeout_s=30)
            assert out.startswith(mid + "@")
            where.setdefault(mid, set()).add(out)
            time.sleep(0.01)
    assert all(len(v) == 1 for v in where.values()), where      # every id stuck to one replica
    total = sum(h.num_loads.remote().result(timeout_s=10) for _ in range(30))
    # num_loads is routed to random replicas; the sum over replicas is 3 (one load per id)
    ctrl = serve.api._controller()
    job = ctrl.jobs["mux"]
    held = [job.queue_models(q) for q in range(3)]
    assert sorted(len(x) for x in held) in ([0, 1, 2], [1, 1, 1]) and sum(len(x) for x in held) == 3
    assert total > 0


def test_process_mode_replica_logs_and_access_log(tmp_path):
    """Replica processes write their component log + access log per
    logging_config; user records on the 'ray.serve' logger land there too."""
    import json as _json

    @serve.deployment(num_replicas=1, logging_config={"encoding": "JSON", "logs_dir": str(tmp_path)})
    class Logged:
        def __call__(self, x):
            import logging as _logging

            _logging.getLogger("ray.serve").info("handling %s", x)
            return x + 1

    h = serve.run(Logged.bind(), name="lg", mode="process")
    assert [h.remote(i).result(timeout_s=30) for i in range(3)] == [1, 2, 3]
    path = tmp_path / "replica_lg_Logged_0.log"
    deadline = time.time() + 10
    while time.time() < deadline:
        lines = [_json.loads(x) for x in path.read_text().splitlines()] if path.exists() else []
        if sum("latency_ms" in x for x in lines) >= 3:
            break
        time.sleep(0.1)
    access = [x for x in lines if "latency_ms" in x]
    assert len(access) == 3 and all(x["status"] == "OK" and x["method"] == "__call__" for x in access)
    assert sum(x["message"].startswith("handling") for x in lines) == 3
    assert any("replica starting" in x["message"] for x in lines)
