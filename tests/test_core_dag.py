"""core.dag: actor DAGs (reference python/ray/dag/dag_node.py:153,
compiled_dag_node.py:113,549,1956) -- bind / execute, MultiOutputNode,
InputNode attributes, compiled pipelining of a 1F1B-style two-stage pipeline
with per-stage ordering, error propagation and teardown."""
import sys
import time
import uuid

import cloudpickle
import pytest

import ray_dynamic_batching_amd.core as ray
from ray_dynamic_batching_amd.core.dag import InputNode, MultiOutputNode

cloudpickle.register_pickle_by_value(sys.modules[__name__])


@pytest.fixture(params=["process", "local"])
def rt(request):
    ray.init(num_gpus=2, local_mode=request.param == "local", namespace="g" + uuid.uuid4().hex[:8])
    yield request.param
    ray.shutdown()


class Stage:
    def __init__(self, k):
        self.k, self.seen = k, []

    def fwd(self, x):
        time.sleep(0.002)
        self.seen.append(x)
        return x * self.k + 1

    def add(self, a, b=0):
        return a + b

    def fail(self, x):
        raise ValueError(f"stage failed on {x}")

    def history(self):
        return list(self.seen)


def test_dag_execute_and_compile(rt):
    S = ray.remote(num_gpus=1)(Stage)
    a, b = S.remote(2), S.remote(10)
    with InputNode() as inp:
        y = b.fwd.bind(a.fwd.bind(inp))
    assert ray.get(y.execute(3)) == (3 * 2 + 1) * 10 + 1
    # multi-output + fan-in + input attributes / kwargs
    with InputNode() as inp:
        h = a.fwd.bind(inp[0])
        s = b.add.bind(h, b=inp[1])
        dag = MultiOutputNode([h, s])
    assert ray.get(dag.execute(1, 5)) == [3, 8]
    # compiled, pipelined: 16 executions in flight through the two stages
    with InputNode() as inp:
        pipe = b.fwd.bind(a.fwd.bind(inp))
    cd = pipe.experimental_compile(_max_inflight_executions=16)
    refs = [cd.execute(i) for i in range(16)]
    assert ray.get(refs) == [(i * 2 + 1) * 10 + 1 for i in range(16)]
    hist_b = ray.get(b.history.remote())
    assert hist_b[-16:] == [i * 2 + 1 for i in range(16)]       # stage order == submission order
    cd.teardown()
    with pytest.raises(ray.RayError):
        cd.execute(0)
    # a failing stage fails that execution's output, not the next ones
    with InputNode() as inp:
        bad = b.fwd.bind(a.fail.bind(inp))
    cbad = bad.experimental_compile()
    with pytest.raises(ray.RayTaskError):
        ray.get(cbad.execute(1))
    cbad.teardown()


def test_dag_submit_failure_releases_slot(rt):
    """A stage whose submission itself raises (a typo'd method) fails that
    execution's ref; the compiled DAG's in-flight slot is released, so later
    executions still run (one slot: a leak would block the second execute)."""
    S = ray.remote(num_gpus=1)(Stage)
    a = S.remote(2)
    with InputNode() as inp:
        bad = a.no_such_method.bind(inp)
    cd = bad.experimental_compile(_max_inflight_executions=1)
    for i in range(3):
        with pytest.raises(Exception):
            ray.get(cd.execute(i), timeout=30)
    cd.teardown(timeout=5)
    with InputNode() as inp:
        good = a.fwd.bind(inp)
    cg = good.experimental_compile(_max_inflight_executions=1)
    assert [ray.get(cg.execute(i), timeout=30) for i in range(3)] == [1, 3, 5]
    cg.teardown()


def test_dag_validation():
    with pytest.raises(ValueError):
        MultiOutputNode([])
    with InputNode() as inp:
        pass
    with pytest.raises(ValueError):
        inp.experimental_compile()            # no actor node


class Big:
    def make(self, n):
        import numpy as np

        return np.arange(n, dtype=np.float64)

    def total(self, arr, scale=1.0):
        return float(arr.sum()) * scale


def test_compiled_dag_shm_channels_actor_to_actor(rt):
    """Compiled DAGs run on shared-memory channels (reference
    experimental/channel/shared_memory_channel.py): each actor's execution
    loop reads its inputs from shm rings and writes its outputs to the next
    actor's ring -- the intermediate arrays never reach the driver."""
    from ray_dynamic_batching_amd.core.dag import ChannelCompiledDAG

    A = ray.remote(num_gpus=1)(Big)
    a, b = A.remote(), A.remote()
    with InputNode() as inp:
        arr = a.make.bind(inp["n"])
        out = MultiOutputNode([b.total.bind(arr, scale=inp["s"]), a.total.bind(arr)])
    cd = out.experimental_compile(_max_inflight_executions=4)
    assert isinstance(cd, ChannelCompiledDAG)
    n = 32 * 1024                                     # 256 KB per intermediate value
    refs = [cd.execute({"n": n + i, "s": 2.0}) for i in range(12)]
    for i, (r1, r2) in enumerate(refs):
        want = float(sum(range(n + i)))
        assert ray.get(r1, timeout=60) == 2 * want and ray.get(r2, timeout=60) == want
    # the edge a.make -> b.total carried 12 values written by actor a, not the driver
    st = [cd.job.queue_stats(q)["submitted"] for q in range(cd.job.info()["n_queues"])]
    assert st.count(12) == len(st) and len(st) == 6   # 2 input edges, 2 inter-actor edges, 2 outputs
    cd.teardown()
    with pytest.raises(ray.RayError):
        cd.execute({"n": 1, "s": 1.0})
    # a value larger than the channel buffer fails that execution, loudly
    with InputNode() as inp:
        big = b.total.bind(a.make.bind(inp))
    small = big.experimental_compile(_buffer_size_bytes=1024)
    with pytest.raises(Exception):
        ray.get(small.execute(10_000), timeout=30)
    small.teardown(timeout=5)
    # the driver-routed interpreter stays available
    drv = big.experimental_compile(_channel="driver")
    assert ray.get(drv.execute(4), timeout=30) == 6.0
    drv.teardown()


class TensorStage:
    def make(self, n):
        import torch

        return {"x": torch.arange(n, dtype=torch.float64), "meta": ("n", n), "ids": [torch.ones(3, dtype=torch.int64)]}

    def total(self, d, scale=1.0):
        assert d["meta"] == ("n", d["x"].numel())
        return (d["x"] * scale).sum() + d["ids"][0].sum()

    def big(self, n):
        import torch

        return torch.zeros(n, dtype=torch.float64)


def test_compiled_dag_tensor_transport_host_ring(rt):
    """``with_tensor_transport()``: the tensors of a node's values travel through
    the reader's staging ring (here host shared memory: CPU tensors) and only
    descriptors cross the shm ring (nested containers, mixed tensors and
    plain values, an actor -> actor edge and an actor -> driver edge)."""
    import torch

    from ray_dynamic_batching_amd.core.dag import TorchTensorType

    A = ray.remote(num_gpus=1)(TensorStage)
    a, b = A.remote(), A.remote()
    n = 24 * 1024                                       # 192 KB of tensor per value
    with InputNode() as inp:
        made = a.make.bind(inp).with_tensor_transport()
        out = b.total.bind(made, scale=2.0).with_type_hint(TorchTensorType(transport="shm"))
    cd = out.experimental_compile(_max_inflight_executions=3, _buffer_size_bytes=256 * 1024)
    refs = [cd.execute(n + i) for i in range(8)]
    for i, r in enumerate(refs):
        got = ray.get(r, timeout=60)
        assert isinstance(got, torch.Tensor) and float(got) == 2.0 * sum(range(n + i)) + 3
    cd.teardown()
    # a tensor larger than a ring slot fails that execution, loudly, and the next ones still run
    with InputNode() as inp:
        big = b.total.bind(a.make.bind(inp).with_tensor_transport())
    small = big.experimental_compile(_max_inflight_executions=1, _buffer_size_bytes=64 * 1024)
    with pytest.raises(Exception, match="slot|buffer"):
        ray.get(small.execute(32 * 1024), timeout=30)
    assert float(ray.get(small.execute(10), timeout=30)) == 45.0 + 3
    small.teardown(timeout=5)
    with pytest.raises(ValueError):
        TorchTensorType(transport="carrier-pigeon")


def test_tensor_ring_slot_reuse_protocol():
    """Ring slots are indexed by message sequence number on both sides; a
    value's tensors are cloned out, so a later write into the same slot does
    not change a value already read."""
    import torch

    from ray_dynamic_batching_amd.core.channel import (TensorRing, _TRef, create_rings, decode_tensors,
                                                       encode_tensors, release_rings)

    job = "t" + uuid.uuid4().hex[:8]
    exp = create_rings(job, [(0, 3, 4096)], ("cpu",))
    w = {"cpu": TensorRing.attach(exp[0]["cpu"])}
    r = {"cpu": w["cpu"]}
    try:
        enc = encode_tensors([torch.full((4,), 7.0), 5, torch.empty(0)], w, seq=4)
        assert isinstance(enc[0], _TRef) and enc[1] == 5 and enc[2].nbytes == 0
        import cloudpickle

        assert len(cloudpickle.dumps(encode_tensors(torch.zeros(1000), w, seq=0))) < 300   # descriptor only
        got = decode_tensors(enc, r, seq=4)
        encode_tensors([torch.full((4,), -1.0)], w, seq=7)        # 7 % 3 == 4 % 3: same slot, rewritten
        assert got[0].tolist() == [7.0] * 4 and got[2].numel() == 0
        assert decode_tensors(enc, r, seq=7)[0].tolist() == [-1.0] * 4
    finally:
        release_rings(job)


class BlobStage:
    def make(self, n):
        import torch

        if n < 0:
            return b"x" * (-n)                 # a large NON-tensor value on a tensor edge
        return {"x": torch.arange(n, dtype=torch.float64)}

    def total(self, d):
        return float(d["x"].sum())

    def echo(self, x):
        return len(x)


def test_oversized_input_raises_before_queueing_and_next_execution_is_right(rt):
    """An input larger than the channel buffer raises from execute() with no
    channel written and no future queued; the next execution gets ITS result
    (advisor finding: futures / slots used to stay queued on a failed write)."""
    A = ray.remote(num_gpus=1)(BlobStage)
    a = A.remote()
    with InputNode() as inp:
        out = a.echo.bind(inp)
    cd = out.experimental_compile(_max_inflight_executions=2, _buffer_size_bytes=4096)
    with pytest.raises(ValueError, match="exceeds"):
        cd.execute(b"y" * 100_000)
    for i in range(5):                          # more executions than in-flight slots: none leaked
        assert ray.get(cd.execute(b"z" * (10 + i)), timeout=30) == 10 + i
    cd.teardown(timeout=5)


def test_oversized_plain_value_on_tensor_edge_keeps_slots_in_step(rt):
    """A non-tensor value too large for a tensor edge's message becomes an error
    for that execution only; the writer's slot numbering stays in step with the
    reader, so the next tensor value is decoded from the right ring slot."""
    A = ray.remote(num_gpus=1)(BlobStage)
    a, b = A.remote(), A.remote()
    with InputNode() as inp:
        out = b.total.bind(a.make.bind(inp).with_tensor_transport())
    cd = out.experimental_compile(_max_inflight_executions=1, _buffer_size_bytes=32 * 1024)
    assert ray.get(cd.execute(100), timeout=30) == float(sum(range(100)))
    with pytest.raises(Exception, match="exceeds|buffer"):
        ray.get(cd.execute(-200_000), timeout=30)
    for n in (10, 300, 77):
        assert ray.get(cd.execute(n), timeout=30) == float(sum(range(n)))
    cd.teardown(timeout=5)
