"""The native power-of-two router (runtime.cpp Client::choose_queue) and the
Python dispatch hub above it (serve/router.py _ShmClientHub), driven with
synthetic queue depths and replica states -- the cases of the reference's
python/ray/serve/tests/unit/test_pow_2_replica_scheduler.py (fake replicas):
shortest-of-two choice, full-scan fallback, saturation, dead / starting /
draining replica exclusion, inactive queues, per-model isolation,
multiplexed-model affinity tiers, FIFO dispatch under rejection and
back-pressure per deployment."""
import collections
import concurrent.futures

import pytest

from ray_dynamic_batching_amd.runtime import job as rjob
from ray_dynamic_batching_amd.serve.router import mux_hash

READY, STARTING, DRAINING, DEAD = 2, 1, 3, 4


@pytest.fixture
def job():
    name = rjob.unique_job_name("rt")
    j = rjob.Job(name, create=True, n_replicas=8, n_queues=8, n_clients=4, req_capacity=64, req_slot_bytes=128,
                 cmp_slot_bytes=64)
    for q in range(8):
        j.configure_queue(q, q, 0 if q < 6 else 1, 4, 0.0, True)     # queues 0-5: model 0, 6-7: model 1
        j.set_replica_status(q, READY, -1, 0)
    yield j
    j.close()


def _choices(c, model, n=400, mux=0):
    return collections.Counter(c.choose_queue(model, mux) for _ in range(n))


def test_never_picks_the_deepest_of_several(job):
    c = rjob.Client(job, 1, seed=7)
    for q, d in enumerate([0, 1, 2, 2, 2, 3]):
        job._test_set_queue_depth(q, d)
    got = _choices(c, 0)
    assert 5 not in got and got[0] > got[2]            # the unique deepest never wins a pair
    # two distinct samples: with 2 candidates the shorter always wins
    for q in range(2, 6):
        job.configure_queue(q, q, 0, 4, 0.0, False)
    assert set(_choices(c, 0)) == {0}


def test_equal_depths_spread_over_all_candidates(job):
    c = rjob.Client(job, 1, seed=3)
    got = _choices(c, 0, n=3000)
    assert set(got) == set(range(6))
    assert min(got.values()) > 300          # roughly uniform (500 expected each)


def test_second_sample_uniform_over_the_other_candidates(job):
    """The pair is two DISTINCT uniform samples (reference random.sample): when
    the deep queue 0 is drawn first, its partner is uniform over queues 1-5 --
    no neighbour of queue 0 gets the collision mass."""
    c = rjob.Client(job, 1, seed=5)
    job._test_set_queue_depth(0, 3)
    n = 30000
    got = _choices(c, 0, n=n)
    assert 0 not in got
    expect = n / 5                              # 1/6 + 1/6 * 1/5 per shallow queue
    assert max(abs(got[q] - expect) for q in range(1, 6)) < 0.05 * expect, got


def test_full_scan_fallback_when_sampled_pair_is_full(job):
    c = rjob.Client(job, 1, seed=11)
    for q in range(6):
        job._test_set_queue_depth(q, 4)     # at max_ongoing
    job._test_set_queue_depth(5, 1)         # the only one with capacity
    assert set(_choices(c, 0)) == {5}


def test_all_saturated_returns_minus_one(job):
    c = rjob.Client(job, 1)
    for q in range(6):
        job._test_set_queue_depth(q, 4)
    assert set(_choices(c, 0, n=50)) == {-1}


def test_unbounded_max_ongoing(job):
    c = rjob.Client(job, 1)
    for q in range(6):
        job.configure_queue(q, q, 0, 0, 0.0, True)       # 0 = no admission bound
        job._test_set_queue_depth(q, 10_000)
    assert -1 not in _choices(c, 0, n=50)


def test_unknown_model_and_inactive_queues(job):
    c = rjob.Client(job, 1)
    assert c.choose_queue(7) == -2                      # nothing serves model 7
    for q in (6, 7):
        job.configure_queue(q, q, 1, 4, 0.0, False)
    assert c.choose_queue(1) == -2                      # model 1's queues all inactive


def test_models_are_isolated(job):
    c = rjob.Client(job, 1)
    assert set(_choices(c, 1)) == {6, 7}
    assert set(_choices(c, 0)) <= set(range(6))


@pytest.mark.parametrize("status", [STARTING, DRAINING, DEAD])
def test_not_ready_replicas_are_excluded(job, status):
    c = rjob.Client(job, 1)
    for q in range(5):
        job.set_replica_status(q, status, -1, 0)
    assert set(_choices(c, 0)) == {5}
    job.set_replica_status(5, status, -1, 0)
    assert set(_choices(c, 0, n=20)) == {-1}           # queues exist, no replica ready: hold


def test_single_candidate(job):
    c = rjob.Client(job, 1)
    assert set(_choices(c, 1, n=20)) <= {6, 7}
    job.configure_queue(7, 7, 1, 4, 0.0, False)
    assert c.choose_queue(1) == 6
    job._test_set_queue_depth(6, 4)
    assert c.choose_queue(1) == -1


def test_multiplexed_affinity_tiers(job):
    c = rjob.Client(job, 1, seed=5)
    h = mux_hash("llama-lora-7")
    job.set_queue_models(2, [mux_hash("other"), h])
    job._test_set_queue_depth(2, 3)                     # deeper than everyone else, still preferred
    assert set(_choices(c, 0, mux=h)) == {2}
    # holder full -> replicas with the fewest models loaded (free cache slots)
    job._test_set_queue_depth(2, 4)
    job.set_queue_models(0, [mux_hash("a")])
    job.set_queue_models(1, [mux_hash("b"), mux_hash("c")])
    assert set(_choices(c, 0, mux=h)) == {3, 4, 5}
    # two holders: power-of-two between them
    job._test_set_queue_depth(2, 0)
    job.set_queue_models(4, [h])
    job._test_set_queue_depth(4, 2)
    assert set(_choices(c, 0, mux=h)) == {2}
    # ids are published and cleared by the replica; at most 16 slots
    job.set_queue_models(2, [])
    assert job.queue_models(2) == []
    job.set_queue_models(3, list(range(1, 40)))
    assert len(job.queue_models(3)) == 16
    assert mux_hash("") == 0 and mux_hash("x") == mux_hash("x") != 0


def test_submit_ring_full_and_too_large(job):
    c = rjob.Client(job, 1)
    assert c.submit(0, b"x" * 200) == -3               # larger than the slot
    n = 0
    while c.submit(0, b"x" * 16) > 0:
        n += 1
    assert n == 64                                      # ring capacity, then -1 (back-pressure)


class _Sink(list):
    pass


def test_hub_dispatches_pending_fifo_under_rejection(job):
    """Every replica at max_ongoing: requests wait in the hub's FIFO; as
    capacity frees they are dispatched in arrival order (reference
    pow_2_scheduler: pending requests fulfilled FIFO)."""
    from ray_dynamic_batching_amd.serve.router import _ShmClientHub

    for q in range(8):
        job.configure_queue(q, q, 0 if q == 0 else 1, 2, 0.0, True)
    hub = _ShmClientHub(job.info()["name"])
    try:
        futs = []
        for i in range(6):
            f = concurrent.futures.Future()
            futs.append(f)
            hub.submit(0, b"p%02d" % i + b"-" * 13, 1, ("unary", f), None, 0)
        assert len(hub.pending) == 4 and hub.pending_for(0) == 4       # 2 admitted (max_ongoing 2)
        cons = rjob.Consumer(job, [0])
        order = []
        for _ in range(20):
            reqs = cons.pop(8, 10_000_000)
            for r in reqs:
                order.append(r[6][:3])
                cons.complete(r[2], r[0], r[1], 0, r[4], b"")
            hub.kick()
            if len(order) == 6:
                break
        assert order == [b"p%02d" % i for i in range(6)]
        assert hub.pending_for(0) == 0
    finally:
        hub.close()


def test_backpressure_is_per_deployment(job):
    """max_queued_requests counts only the deployment's own pending requests."""
    from ray_dynamic_batching_amd.serve.exceptions import BackPressureError
    from ray_dynamic_batching_amd.serve.handle import RequestMeta
    from ray_dynamic_batching_amd.serve.router import ShmRouter

    for q in range(8):
        job.configure_queue(q, q, 0 if q == 0 else 1, 1, 0.0, True)
    job._test_set_queue_depth(0, 1)                     # model 0 saturated: everything pends
    name = job.info()["name"]
    r0 = ShmRouter(name, 0, "A", 2, None)
    r1 = ShmRouter(name, 1, "B", 2, None)
    try:
        meta = lambda i: RequestMeta(i, "__call__", "", False, "app", "A")  # noqa: E731
        rs = [r0.assign(meta(i), (i,), {}) for i in range(3)]
        with pytest.raises(BackPressureError):
            rs[2].result(timeout_s=5)
        assert r0.metrics.num_rejected_backpressure == 1
        # deployment B still admits
        r1.assign(RequestMeta(9, "__call__", "", False, "app", "B"), (1,), {})
        assert r1.metrics.num_rejected_backpressure == 0
    finally:
        job._test_set_queue_depth(0, 0)
