"""Chaos tests: replica killer, injected message loss and
router rejections, all through env knobs inherited by replica processes."""
import os

import pytest

from ray_dynamic_batching_amd import serve
from ray_dynamic_batching_amd.utils import faults


@serve.deployment(num_replicas=2, max_ongoing_requests=16)
class Mul:
    def __init__(self, k):
        self.k = k

    @serve.batch(max_batch_size=4, batch_wait_timeout_s=0.005)
    async def __call__(self, xs):
        return [x * self.k for x in xs]


@pytest.fixture
def env_knobs():
    saved = dict(os.environ)
    yield os.environ
    serve.shutdown()
    os.environ.clear()
    os.environ.update(saved)
    faults.reset()


def test_replica_killer_agent_restarts_and_requests_complete(env_knobs):
    env_knobs["RDB_FAULT_KILL_AFTER_BATCHES"] = "6"
    # restarts back off 0.5 s doubling per restart (cap 30 s): a replica killed every
    # 6 batches restarts ~8 times for 120 requests, whose doubling delays alone can
    # outlast the 60 s re-dispatch window when batches are small (CPU load) -- cap them
    env_knobs["RDB_RESTART_BACKOFF_MAX_S"] = "1.0"
    # a replica that dies every 6 batches takes every request it holds with it:
    # give them a re-dispatch budget above the default 3 (the cap exists for a
    # request that kills every replica it reaches, tests/test_router_retry.py)
    h = serve.run(Mul.options(health_check_timeout_s=5, max_request_retries=20).bind(3), mode="process")
    outs = [h.remote(i) for i in range(120)]
    assert [o.result(timeout_s=120) for o in outs] == [3 * i for i in range(120)]
    from ray_dynamic_batching_amd.serve.controller import get_controller

    # the agent notices the death asynchronously (exit reaping + back-off); under
    # CPU load the re-dispatched requests can finish before it does
    import time

    deadline = time.time() + 30
    procs = get_controller().agent.list()
    while sum(p["restarts"] for p in procs) < 1 and time.time() < deadline:
        time.sleep(0.1)
        procs = get_controller().agent.list()
    assert sum(p["restarts"] for p in procs) >= 1, procs


def test_injected_message_loss_is_redispatched(env_knobs):
    env_knobs["RDB_FAULT_DROP_EVERY"] = "5"
    # a re-dispatched request can land on the 5th slot again: budget above the default 3
    h = serve.run(Mul.options(max_request_retries=20).bind(2), mode="process")
    outs = [h.remote(i) for i in range(60)]
    assert [o.result(timeout_s=60) for o in outs] == [2 * i for i in range(60)]


def test_router_rejections_retry(env_knobs):
    env_knobs["RDB_FAULT_REJECT_EVERY"] = "3"
    inj = faults.reset()
    assert inj.reject_every == 3
    h = serve.run(Mul.bind(5), mode="process")
    outs = [h.remote(i) for i in range(40)]
    assert [o.result(timeout_s=60) for o in outs] == [5 * i for i in range(40)]
    assert inj._n_submit >= 40
