"""Re-dispatch of requests whose replica died is capped: a request
that kills every replica it reaches fails with ReplicaDiedError after
``max_request_retries`` re-dispatches instead of being replayed into every
restarted replica for the whole retry window; other requests keep working.
A cancelled stream request still waiting in the router's FIFO is never sent."""
import os
import time

import pytest

from ray_dynamic_batching_amd import serve
from ray_dynamic_batching_amd.serve.exceptions import ReplicaDiedError


@pytest.fixture(autouse=True)
def _shutdown():
    yield
    serve.shutdown()


@serve.deployment(max_request_retries=2, request_retry_timeout_s=120.0, health_check_timeout_s=60)
class Poisonable:
    def __call__(self, x):
        if x == "poison":
            os._exit(7)            # the replica dies while running this request
        return x * 2


def test_poison_request_fails_after_retry_budget():
    h = serve.run(Poisonable.bind(), mode="process")
    assert h.remote(21).result(timeout_s=60) == 42
    t0 = time.time()
    with pytest.raises(ReplicaDiedError):
        h.remote("poison").result(timeout_s=120)
    assert time.time() - t0 < 90                 # not the 120 s window: the budget ran out first
    from ray_dynamic_batching_amd.serve.controller import get_controller

    # 1 first dispatch + 2 re-dispatches = 3 replica deaths, then the request failed
    deaths = sum(p["restarts"] for p in get_controller().agent.list())
    assert deaths == 3, deaths
    assert h.remote(5).result(timeout_s=60) == 10


def test_retry_fields_round_trip_yaml():
    from ray_dynamic_batching_amd.serve.config import DeploymentConfig

    c = Poisonable.config
    assert (c.max_request_retries, c.request_retry_timeout_s) == (2, 120.0)
    assert DeploymentConfig(**c.model_dump(mode="json")).max_request_retries == 2
    with pytest.raises(ValueError):
        DeploymentConfig(name="x", max_request_retries=-1)


def test_cancelled_queued_stream_request_is_not_sent():
    from ray_dynamic_batching_amd.serve.handle import StreamSink
    from ray_dynamic_batching_amd.serve.router import _ShmClientHub

    # the hub's FIFO logic without a job: a fake hub object with the real methods
    hub = _ShmClientHub.__new__(_ShmClientHub)
    import collections
    import threading

    hub.lock = threading.Lock()
    hub.inflight = {}
    hub.pending = collections.deque()
    hub._pending_by_model = collections.Counter()
    hub._deferred = []
    hub._deferred_lock = threading.Lock()
    sink = ("stream", StreamSink())
    other = ("unary", __import__("concurrent.futures").futures.Future())
    hub.pending.append((7, b"a", 1, sink, None, (time.monotonic() + 9, 3)))
    hub.pending.append((7, b"b", 1, other, None, (time.monotonic() + 9, 3)))
    hub._pending_by_model[7] = 2
    hub.cancel(sink)
    assert [it[3] for it in hub.pending] == [other] and hub._pending_by_model[7] == 1
    assert _ShmClientHub._sink_cancelled(sink)
