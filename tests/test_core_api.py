"""Ray-core-compatible API (ray_dynamic_batching_amd.core): actors as pinned
processes (and in local mode), ordering, errors, named actors across drivers,
tasks, put/get/wait, util.queue.Queue semantics, and the fork's structure --
GPU worker actors draining per-model RayQueues (293-project/src/scheduler.py)."""
import os
import subprocess
import sys
import textwrap
import time
import uuid

import cloudpickle
import pytest

import ray_dynamic_batching_amd.core as ray
from ray_dynamic_batching_amd.core.util.queue import Empty, Full, Queue

cloudpickle.register_pickle_by_value(sys.modules[__name__])


@pytest.fixture(params=["process", "local"])
def rt(request):
    ray.init(num_gpus=2, local_mode=request.param == "local", namespace="t" + uuid.uuid4().hex[:8])
    yield request.param
    ray.shutdown()


class Counter:
    def __init__(self, start=0):
        self.n = start

    def incr(self, k=1):
        self.n += k
        return self.n

    def gpus(self):
        import ray_dynamic_batching_amd.core as r

        return r.get_gpu_ids(), os.environ.get("HIP_VISIBLE_DEVICES")

    def boom(self):
        raise ValueError("bad input")

    async def aget(self):
        return self.n


def test_actor_calls_ordering_errors_and_gpu_pinning(rt):
    C = ray.remote(num_gpus=1)(Counter)
    a, b = C.remote(10), C.options(name="second").remote()
    refs = [a.incr.remote() for _ in range(50)]
    assert ray.get(refs) == list(range(11, 61))                      # per-caller FIFO
    assert ray.get(a.aget.remote()) == 60                            # async method
    ga, gb = ray.get(a.gpus.remote()), ray.get(b.gpus.remote())
    assert sorted([ga[0], gb[0]]) == [[0], [1]]                       # whole GPUs, first-fit
    if rt == "process":
        assert ga[1] == str(ga[0][0])                                # HIP_VISIBLE_DEVICES pinned
    assert ray.available_resources()["GPU"] == 0.0
    with pytest.raises(ray.RayTaskError) as e:
        ray.get(a.boom.remote())
    assert isinstance(e.value.cause, ValueError) and "bad input" in str(e.value)
    # no GPU left: creation waits, then fails; killing an actor frees its GPU
    os.environ["RDB_CORE_PENDING_TIMEOUT_S"] = "0.3"
    try:
        with pytest.raises(ray.RayError):
            C.remote()
        ray.kill(b)
        c = C.remote(5)
        assert ray.get(c.incr.remote()) == 6
    finally:
        del os.environ["RDB_CORE_PENDING_TIMEOUT_S"]
    # fractional GPUs co-locate best-fit on the freed... fully used -> none left
    assert ray.available_resources()["GPU"] == 0.0


class Log:
    def __init__(self):
        self.seen = []

    def put(self, x):
        self.seen.append(x)
        return x

    def seen_all(self):
        return list(self.seen)


def test_remote_never_blocks_on_arg_refs(rt):
    """.remote() with an unresolved ref argument returns at once (reference:
    ray.remote submission is asynchronous; the dependency resolves before the
    call runs); calls on one actor keep their submission order even when an
    earlier one waits for its argument; an upstream failure surfaces at get()
    on the dependent ref, not at submit time."""
    import threading
    from concurrent.futures import Future

    L = ray.remote(Log).remote()
    gate: Future = Future()
    slow = ray.ObjectRef(gate)
    t0 = time.monotonic()
    r1 = L.put.remote(slow)          # waits for `slow`
    r2 = L.put.remote("b")           # no deps, but queued behind r1
    assert time.monotonic() - t0 < 0.5
    threading.Timer(0.2, lambda: gate.set_result("a")).start()
    assert ray.get([r1, r2], timeout=30) == ["a", "b"]
    assert ray.get(L.seen_all.remote())[-2:] == ["a", "b"]
    # failure propagates through the dependent ref
    bad = ray.ObjectRef(Future())
    r3 = L.put.remote(bad)
    bad._fut.set_exception(ValueError("upstream"))
    with pytest.raises(ValueError):
        ray.get(r3, timeout=30)
    assert ray.get(L.put.remote("c"), timeout=30) == "c"
    # tasks chain the same way
    sq = ray.remote(lambda x: x * x)
    g2: Future = Future()
    r4 = sq.remote(ray.ObjectRef(g2))
    g2.set_result(7)
    assert ray.get(r4, timeout=30) == 49


def test_tasks_put_get_wait(rt):
    @ray.remote
    def add(x, y):
        time.sleep(0.01 * y)
        return x + y

    r = ray.put(40)
    refs = [add.remote(r, i) for i in range(5)]                      # ObjectRef args resolved
    ready, rest = ray.wait(refs, num_returns=2, timeout=5)
    assert len(ready) == 2 and len(rest) == 3
    assert ray.get(refs) == [40, 41, 42, 43, 44]
    with pytest.raises(ray.GetTimeoutError):
        ray.get(add.remote(0, 100), timeout=0.05)


def test_queue_semantics(rt):
    q = Queue(maxsize=2)
    assert q.empty() and not q.full()
    q.put(1)
    q.put_nowait(2)
    assert q.full() and q.qsize() == 2
    with pytest.raises(Full):
        q.put_nowait(3)
    with pytest.raises(Full):
        q.put(3, timeout=0.05)
    assert q.get() == 1 and q.get_nowait() == 2
    with pytest.raises(Empty):
        q.get(timeout=0.05)
    with pytest.raises(Empty):
        q.get_nowait()
    q.put_nowait_batch([7, 8])
    with pytest.raises(Full):
        q.put_nowait_batch([9])
    with pytest.raises(Empty):
        q.get_nowait_batch(3)
    assert q.get_nowait_batch(2) == [7, 8]
    q.shutdown()


class GPUWorker:
    """The fork's worker shape: pinned to one GPU, drains its model queues."""

    def __init__(self, name):
        self.name = name

    def execute(self, queues, n):
        import ray_dynamic_batching_amd.core as r

        # nested refs stay refs (Ray semantics): the worker gets them, as the fork's executor does
        queues = {m: r.get(q) if isinstance(q, r.ObjectRef) else q for m, q in queues.items()}
        out = []
        while True:       # drain until every model queue is empty (n: batch size cap)
            took = 0
            for model, q in queues.items():
                try:
                    got = q.get_nowait_batch(min(q.qsize(), n))
                except Empty:          # another worker emptied it meanwhile
                    got = []
                out.extend((model, x) for x in got)
                took += len(got)
            if not took and all(q.empty() for q in queues.values()):
                return self.name, r.get_gpu_ids(), out


def test_fork_structure_workers_drain_model_queues(rt):
    queues = {"resnet": Queue(maxsize=64), "vit": Queue(maxsize=64)}
    W = ray.remote(num_gpus=1)(GPUWorker)
    workers = [W.options(name=f"gpu{i}").remote(f"gpu{i}") for i in range(2)]
    qrefs = {m: ray.put(q) for m, q in queues.items()}                # ray.put(queue) as the fork does
    for i in range(10):
        queues["resnet"].put(i)
        queues["vit"].put(100 + i)
    futs = [w.execute.remote(qrefs, 4) for w in workers]
    res = ray.get(futs, timeout=60)
    got = sorted(x for _, _, out in res for _, x in out)
    assert got == sorted(list(range(10)) + [100 + i for i in range(10)])
    assert sorted(g[0] for _, g, _ in res) == [0, 1]
    acts = ray.state.actors()
    assert {a["Name"] for a in acts.values()} >= {"gpu0", "gpu1"}
    assert all(a["State"] == "ALIVE" for a in acts.values())


def test_named_actor_from_another_driver():
    ns = "x" + uuid.uuid4().hex[:8]
    ray.init(num_gpus=0, namespace=ns)
    try:
        h = ray.remote(Counter).options(name="tracker", lifetime="detached").remote(3)
        assert ray.get(h.incr.remote()) == 4
        with pytest.raises(ValueError):
            ray.remote(Counter).options(name="tracker").remote()
        code = textwrap.dedent(f"""
            import ray_dynamic_batching_amd.core as ray
            ray.init(address="auto", namespace="{ns}")
            h = ray.get_actor("tracker")
            print(ray.get(h.incr.remote(10)))
            ray.shutdown()
        """)
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                             env=dict(os.environ, PYTHONPATH=os.getcwd()))
        assert out.returncode == 0, out.stderr
        assert out.stdout.strip().splitlines()[-1] == "14"
        assert ray.get(h.incr.remote()) == 15
        ray.kill(h)
        with pytest.raises(ValueError):
            ray.get_actor("tracker")
    finally:
        ray.shutdown()


def test_actor_death_fails_pending_calls():
    ray.init(num_gpus=0, namespace="d" + uuid.uuid4().hex[:8])
    try:
        class Slow:
            def sleep(self, s):
                time.sleep(s)
                return s

            def pid(self):
                return os.getpid()

        h = ray.remote(Slow).remote()
        pid = ray.get(h.pid.remote())
        ref = h.sleep.remote(30)
        time.sleep(0.2)
        os.kill(pid, 9)
        with pytest.raises(ray.RayActorError):
            ray.get(ref, timeout=30)
        with pytest.raises(ray.RayActorError):
            ray.get(h.pid.remote(), timeout=30)
    finally:
        ray.shutdown()


def test_nodes_runtime_context_and_node_affinity():
    """ray.nodes() / get_runtime_context() / NodeAffinitySchedulingStrategy on the
    single node: affinity to this node schedules, to an unknown node fails the ref
    (hard) or falls back to this node (soft); string strategies DEFAULT / SPREAD."""
    import pytest

    from ray_dynamic_batching_amd import core
    from ray_dynamic_batching_amd.core.util.scheduling_strategies import NodeAffinitySchedulingStrategy

    core.init(num_gpus=0, local_mode=True, ignore_reinit_error=True)
    try:
        ns = core.nodes()
        assert len(ns) == 1 and ns[0]["Alive"]
        me = core.get_runtime_context().get_node_id()
        assert ns[0]["NodeID"] == me and len(me) == 56

        @core.remote
        def where():
            return core.get_runtime_context().get_node_id()

        assert core.get(where.options(scheduling_strategy=NodeAffinitySchedulingStrategy(me, soft=False)).remote()) == me
        assert core.get(where.options(scheduling_strategy="SPREAD").remote()) == me
        bad = NodeAffinitySchedulingStrategy("ff" * 28, soft=False)
        with pytest.raises(core.TaskUnschedulableError):
            core.get(where.options(scheduling_strategy=bad).remote())
        soft = NodeAffinitySchedulingStrategy("ff" * 28, soft=True)
        assert core.get(where.options(scheduling_strategy=soft).remote()) == me
        with pytest.raises(ValueError):
            where.options(scheduling_strategy="PACKED_TIGHT").remote()

        @core.remote
        class A:
            def node(self):
                return core.get_runtime_context().get_node_id()

        a = A.options(scheduling_strategy=NodeAffinitySchedulingStrategy(me, soft=False)).remote()
        assert core.get(a.node.remote()) == me
        with pytest.raises(core.TaskUnschedulableError):
            A.options(scheduling_strategy=bad).remote()
        assert core.get_runtime_context().get_accelerator_ids() == {"GPU": []}
    finally:
        core.shutdown()
