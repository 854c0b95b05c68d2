"""core.util.placement_group (reference python/ray/util/placement_group.py:145,
scheduling_strategies.py:41): gang reservation with the per-GPU strategy
reading shared with Serve's bundles, actors scheduled into bundles (GPU
pinning, capacity), waiting / failing reservations, removal."""
import os
import sys
import uuid

import cloudpickle
import pytest

import ray_dynamic_batching_amd.core as ray
from ray_dynamic_batching_amd.core.util import (get_placement_group, placement_group, placement_group_table,
                                                 remove_placement_group)
from ray_dynamic_batching_amd.core.util.scheduling_strategies import PlacementGroupSchedulingStrategy
from ray_dynamic_batching_amd.runtime.resources import GpuAllocator

cloudpickle.register_pickle_by_value(sys.modules[__name__])


def test_allocator_bundle_strategies():
    a = GpuAllocator(4)
    sp = a.allocate_bundles("p", [0.5, 0.25], "STRICT_PACK")
    assert sp[0].gpus == sp[1].gpus                      # one GPU
    ss = a.allocate_bundles("s", [1, 1, 0.5], "STRICT_SPREAD")
    used = [g for x in ss for g in x.gpus]
    assert len(used) == len(set(used)) == 3
    assert a.allocate_bundles("y", [1, 1], "PACK") is None                 # no two whole GPUs left
    pk = a.allocate_bundles("z", [0.125, 0.125], "PACK")                   # packs onto one GPU
    assert pk is not None and pk[0].gpus == pk[1].gpus
    assert a.allocate_bundles("x", [0.5, 0.5, 0.5], "STRICT_SPREAD") is None
    for i in range(2):
        a.release(f"p/{i}")
        a.release(f"z/{i}")
    assert a.allocate_bundles("y2", [1], "PACK")[0].gpus == [0]
    with pytest.raises(ValueError):
        a.allocate_bundles("bad", [1.5], "PACK")


@pytest.fixture(params=["process", "local"])
def rt(request):
    ray.init(num_gpus=4, local_mode=request.param == "local", namespace="p" + uuid.uuid4().hex[:8])
    yield request.param
    ray.shutdown()


class Pinned:
    def gpus(self):
        import ray_dynamic_batching_amd.core as r

        return r.get_gpu_ids(), os.environ.get("HIP_VISIBLE_DEVICES")


def test_placement_group_actors(rt):
    pg = placement_group([{"GPU": 1}, {"GPU": 1}], strategy="STRICT_SPREAD", name="tp2")
    assert ray.get(pg.ready()) is pg and pg.wait(5)
    assert ray.available_resources()["GPU"] == 2
    A = ray.remote(Pinned)
    a0 = A.options(num_gpus=1, scheduling_strategy=PlacementGroupSchedulingStrategy(pg, 0)).remote()
    a1 = A.options(num_gpus=1, placement_group=pg, placement_group_bundle_index=1).remote()
    g0, g1 = ray.get(a0.gpus.remote())[0], ray.get(a1.gpus.remote())[0]
    assert g0 == pg.bundle_gpus[0] and g1 == pg.bundle_gpus[1] and g0 != g1
    with pytest.raises(ValueError):          # bundle 0 is full
        A.options(num_gpus=1, scheduling_strategy=PlacementGroupSchedulingStrategy(pg, 0)).remote()
    assert ray.available_resources()["GPU"] == 2    # actors in the group do not take free GPUs
    assert get_placement_group("tp2") is pg
    assert placement_group_table(pg)["state"] == "CREATED"
    # fractional bundles: two half-GPU actors share one packed GPU
    half = placement_group([{"GPU": 0.5}, {"GPU": 0.5}], strategy="STRICT_PACK")
    assert half.wait(5) and half.bundle_gpus[0] == half.bundle_gpus[1]
    h = [A.options(num_gpus=0.5, scheduling_strategy=PlacementGroupSchedulingStrategy(half)).remote()
         for _ in range(2)]
    assert ray.get(h[0].gpus.remote())[0] == ray.get(h[1].gpus.remote())[0] == half.bundle_gpus[0]
    remove_placement_group(pg)
    assert ray.available_resources()["GPU"] == 3.0
    with pytest.raises(ray.RayError):
        ray.get(a0.gpus.remote(), timeout=10)   # members die with their group
    # a group that cannot fit fails its ready()
    big = placement_group([{"GPU": 1}] * 5, strategy="STRICT_SPREAD", _timeout_s=0.5)
    assert not big.wait(3) and big.state == "FAILED"


def test_remove_races_reservation():
    """remove_placement_group() landing while the reserve thread is inside
    allocate_bundles: the bundles it then takes are given back, the group stays
    REMOVED and ready() raises (no InvalidStateError in the thread, no leak)."""
    import threading

    ray.init(num_gpus=2, local_mode=True, namespace="r" + uuid.uuid4().hex[:8])
    try:
        ctx = ray._require_ctx()
        inside, go = threading.Event(), threading.Event()
        real = ctx.allocator.allocate_bundles

        def slow(owner, amounts, strategy="PACK"):
            inside.set()
            go.wait(10)
            return real(owner, amounts, strategy)

        ctx.allocator.allocate_bundles = slow
        pg = placement_group([{"GPU": 1}, {"GPU": 1}], strategy="SPREAD")
        assert inside.wait(10)
        remove_placement_group(pg)
        go.set()
        with pytest.raises(RuntimeError):
            ray.get(pg.ready(), timeout=10)
        import time

        deadline = time.monotonic() + 5
        while time.monotonic() < deadline and ray.available_resources()["GPU"] != 2:
            time.sleep(0.02)
        assert pg.state == "REMOVED"
        assert ray.available_resources()["GPU"] == 2        # nothing leaked
    finally:
        ray.shutdown()


class Sq:
    def __init__(self, d):
        self.d = d

    def f(self, x):
        import time

        time.sleep(self.d * (x % 3))
        return x * x


def test_actor_pool(rt):
    from ray_dynamic_batching_amd.core.util import ActorPool

    S = ray.remote(Sq)
    pool = ActorPool([S.remote(0.01), S.remote(0.01)])
    assert list(pool.map(lambda a, v: a.f.remote(v), range(8))) == [x * x for x in range(8)]
    assert sorted(pool.map_unordered(lambda a, v: a.f.remote(v), range(8))) == sorted(x * x for x in range(8))
    for v in range(5):
        pool.submit(lambda a, v: a.f.remote(v), v)          # 3 of them queue behind 2 actors
    assert [pool.get_next() for _ in range(5)] == [0, 1, 4, 9, 16]
    assert not pool.has_next() and pool.has_free()
    a = pool.pop_idle()
    with pytest.raises(ValueError):
        pool.push(pool._idle[0])
    pool.push(a)


def test_python_bundle_allocator_matches_native_agent():
    """Differential: core placement groups (Python GpuAllocator.allocate_bundles)
    and Serve bundles (native NodeAgent.allocate_bundles) place the same random
    gang requests on the same GPUs, or both refuse them."""
    import random

    from ray_dynamic_batching_amd.runtime import agent as ragent

    rng = random.Random(11)
    nat = ragent.NodeAgent(8, 288.0)
    py = GpuAllocator(8)
    live = []
    try:
        for step in range(200):
            if live and rng.random() < 0.35:
                name, n = live.pop(rng.randrange(len(live)))
                assert nat.release(name)
                for i in range(n):
                    py.release(f"{name}/{i}")
                continue
            n = rng.randint(1, 3)
            amounts = [rng.choice([0.25, 0.5, 1, 2, 0.125]) for _ in range(n)]
            strategy = rng.choice(["PACK", "SPREAD", "STRICT_PACK", "STRICT_SPREAD"])
            name = f"g{step}"
            got_n = nat.allocate_bundles(name, [(a, 0) for a in amounts], strategy)
            got_p = py.allocate_bundles(name, amounts, strategy)
            assert (got_n is None) == (got_p is None), (step, amounts, strategy, got_n, got_p)
            if got_n is not None:
                assert got_n["bundle_gpus"] == [a.gpus for a in got_p], (step, amounts, strategy)
                live.append((name, n))
            assert [round(g["used"], 6) for g in nat.resources()] == [round(s.used, 6) for s in py.slots], step
    finally:
        nat.shutdown()


def test_timeline(rt, tmp_path):
    import json

    S = ray.remote(Sq)
    a = S.remote(0.0)
    ray.get([a.f.remote(i) for i in range(4)])
    sq = ray.remote(lambda x: x + 1)
    assert ray.get(sq.remote(1)) == 2
    ev = ray.timeline(str(tmp_path / "tl.json"))
    names = [e["name"] for e in ev]
    assert names.count("Sq.f") >= 4 and "<lambda>" in names
    assert all(e["ph"] == "X" and e["dur"] >= 0 for e in ev)
    assert json.load(open(tmp_path / "tl.json")) == ev
