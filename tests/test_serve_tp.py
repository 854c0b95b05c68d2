"""Tensor-parallel replicas deployed through Serve (CPU, gloo).

``serve.model_deployment(factory, ..., tensor_parallel_size=N)``: the node
agent gang-reserves N placement bundles, spawns N rank processes (one group),
the ranks rendezvous through the agent's KV (no torchrun), rank 0 serves the
replica's queue, and when any rank dies the agent kills and restarts the whole
group while the router re-dispatches the requests that were in flight.
Reference: placement_group_bundles (python/ray/serve/api.py:240-259), the
collective rendezvous through a named store
(python/ray/util/collective/collective_group/nccl_collective_group.py:555-577).
"""
import threading
import time

import numpy as np
import pytest

from ray_dynamic_batching_amd import serve
from ray_dynamic_batching_amd.models import factories
from ray_dynamic_batching_amd.models.tp_echo import TPEcho


@pytest.fixture(autouse=True)
def _shutdown():
    yield
    serve.shutdown()


def _deploy(world: int, **kw):
    app = serve.model_deployment(factories.tp_echo(d=16), "tpecho", max_batch_size=4, batch_wait_timeout_s=0.002,
                                 tensor_parallel_size=world, **kw)
    return serve.run(app.bind(), mode="process")


def _group(world):
    from ray_dynamic_batching_amd.serve.controller import get_controller

    c = get_controller()
    st = c.apps["default"]["tpecho"]
    rep = st.proc_replicas[0]
    info = c.agent.group_info(rep.group_id)
    assert len(info["members"]) == world
    return c, info


@pytest.mark.parametrize("world", [2, 4, 8])
def test_tp_deployment_serves_through_serve_run(world):
    h = _deploy(world)
    rng = np.random.default_rng(world)
    xs = [rng.standard_normal(16).astype(np.float32) for _ in range(24)]
    outs = [h.remote(x) for x in xs]
    w = TPEcho(16, 8).w_full.numpy()
    for x, o in zip(xs, outs):
        y = o.result(timeout_s=60)
        np.testing.assert_allclose(y[:8], x @ w.T, rtol=1e-4, atol=1e-4)   # sum of the N row-parallel partials
        assert y[8] == world                                               # every rank contributed
    c, info = _group(world)
    deadline = time.time() + 10           # the agent's monitor marks the gang RUNNING on its next pass
    while info["state"] != "RUNNING" and time.time() < deadline:
        time.sleep(0.05)
        info = c.agent.group_info(info["id"])
    assert info["state"] == "RUNNING" and info["epoch"] == 0 and all(p > 0 for p in info["pids"])
    # the store address was published under the group's epoch in the agent KV
    assert any(k.startswith("tp/default#tpecho#") and k.endswith("/0/store") for k in c.agent.kv_keys("tp/"))
    st = serve.status()["applications"]["default"]["deployments"]["tpecho"]
    assert st["running_replicas"] == 1


def test_killing_one_rank_restarts_the_whole_group_and_requests_complete():
    world = 4
    h = _deploy(world)
    w = TPEcho(16, 8).w_full.numpy()
    c, info = _group(world)
    old_pids = list(info["pids"])
    results, errors = [], []
    stop = threading.Event()

    def load():
        rng = np.random.default_rng(0)
        while not stop.is_set():
            x = rng.standard_normal(16).astype(np.float32)
            try:
                results.append((x, h.remote(x).result(timeout_s=90)))
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))
    threads = [threading.Thread(target=load) for _ in range(4)]
    for t in threads:
        t.start()
    time.sleep(1.0)
    before = len(results)
    c.agent.kill(info["members"][2], 9)                   # SIGKILL rank 2 mid-traffic
    deadline = time.time() + 60
    while time.time() < deadline:
        g = c.agent.group_info(info["id"])
        if g["restarts"] >= 1 and g["state"] == "RUNNING" and len(results) > before + 20:
            break
        time.sleep(0.1)
    stop.set()
    for t in threads:
        t.join(120)
    g = c.agent.group_info(info["id"])
    assert not errors, errors[:3]
    assert g["restarts"] >= 1 and g["epoch"] >= 1, g
    assert all(p > 0 and p not in old_pids for p in g["pids"]), (old_pids, g["pids"])   # the whole gang restarted
    assert "rank 2" in g["last_exit"]
    assert len(results) > before + 20
    for x, y in results:
        np.testing.assert_allclose(y[:8], x @ w.T, rtol=1e-4, atol=1e-4)
        assert y[8] == world
    # the old epoch's rendezvous key is gone, the new one is there
    keys = c.agent.kv_keys("tp/")
    assert not any(k.endswith("/0/store") for k in keys) and any(k.endswith(f"/{g['epoch']}/store") for k in keys)


def test_tp_config_validation():
    with pytest.raises(ValueError):
        serve.deployment(tensor_parallel_size=0)(TPEcho)
    with pytest.raises(ValueError):
        serve.deployment(tensor_parallel_size=2, placement_group_bundles=[{"GPU": 1}])(TPEcho)
    d = serve.deployment(tensor_parallel_size=4, ray_actor_options={"num_gpus": 1})(TPEcho)
    assert d.config.tp_bundles() == [(1.0, 0.0)] * 4


def test_bad_request_gets_an_error_and_the_group_keeps_running():
    """A request that is not one model row (wrong shape -> the router falls back
    to a pickled payload) is answered with an error by rank 0; the group never
    restarts and the next good requests are served (one bad client
    request must not crash-loop a TP deployment)."""
    from ray_dynamic_batching_amd.serve.exceptions import RayServeException

    h = _deploy(2)
    good = np.ones(16, np.float32)
    assert h.remote(good).result(timeout_s=60)[8] == 2
    bad = h.remote(np.ones(5, np.float32))
    with pytest.raises((RayServeException, RuntimeError, ValueError)):
        bad.result(timeout_s=60)
    outs = [h.remote(good) for _ in range(6)]
    assert all(o.result(timeout_s=60)[8] == 2 for o in outs)
    c, info = _group(2)
    assert info["restarts"] == 0 and info["epoch"] == 0


def test_stopping_a_tp_replica_forgets_its_group():
    """Deleting the deployment stops the gang and erases the agent's Group entry
    (every TP stop leaked one Group)."""
    h = _deploy(2)
    assert h.remote(np.ones(16, np.float32)).result(timeout_s=60)[8] == 2
    from ray_dynamic_batching_amd.serve.controller import get_controller

    c = get_controller()
    assert c.agent.num_groups() == 1
    serve.delete("default")
    deadline = time.time() + 30
    while c.agent.num_groups() and time.time() < deadline:
        time.sleep(0.1)
    assert c.agent.num_groups() == 0
