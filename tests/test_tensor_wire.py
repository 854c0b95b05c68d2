"""Raw-tensor calls for Python-worker deployments: an
array / CPU tensor argument crosses the shm ring as header + raw bytes (never
cloudpickled), arrays come back the same way, and ``@serve.batch`` methods get
the arrays; ``stack_to_device`` assembles the batch."""
import numpy as np
import pytest
import torch

from ray_dynamic_batching_amd import serve
from ray_dynamic_batching_amd.serve import tensor_wire


@pytest.fixture(autouse=True)
def _shutdown():
    yield
    serve.shutdown()


@pytest.mark.parametrize("x", [np.arange(12, dtype=np.float32).reshape(3, 4), np.arange(5, dtype=np.uint8),
                               torch.arange(6, dtype=torch.int64).reshape(2, 3),
                               torch.randn(4, 8).to(torch.bfloat16), np.zeros((0, 3), np.float16)])
def test_round_trip(x):
    p = tensor_wire.encode_call("__call__", x, "mux-a", "rid-1")
    method, y, mux, rid, stream = tensor_wire.decode_call(p)
    assert (method, mux, rid, stream) == ("__call__", "mux-a", "rid-1", False)
    assert type(y) is type(x) and tuple(y.shape) == tuple(x.shape)
    if isinstance(x, torch.Tensor):
        assert y.dtype == x.dtype and torch.equal(y, x)
    else:
        assert y.dtype == x.dtype and np.array_equal(y, x)
    r = tensor_wire.decode_result(tensor_wire.encode_result(x))
    assert tuple(r.shape) == tuple(x.shape)


def test_what_is_encodable():
    assert tensor_wire.encodable((np.ones(3),), {})
    assert not tensor_wire.encodable((np.ones(3),), {"k": 1})            # kwargs: pickled
    assert not tensor_wire.encodable((np.ones(3), 2), {})                # two args: pickled
    assert not tensor_wire.encodable((np.array(["a"], dtype=object),), {})
    assert not tensor_wire.encodable(([1, 2],), {})


@serve.deployment(max_ongoing_requests=64)
class Doubler:
    def __init__(self):
        self.kinds = []

    @serve.batch(max_batch_size=8, batch_wait_timeout_s=0.01)
    async def __call__(self, xs):
        self.kinds.extend(type(x).__name__ for x in xs)
        batch = serve.stack_to_device(xs, "cpu")       # on a GPU replica: pinned staging + async H2D
        return [row * 2 for row in batch.numpy()]

    def seen(self):
        return sorted(set(self.kinds))


def test_process_mode_batch_gets_raw_arrays_not_pickles(monkeypatch):
    h = serve.run(Doubler.bind(), mode="process")
    xs = [np.full((4, 4), i, np.float32) for i in range(24)]
    outs = [h.remote(x) for x in xs]
    for i, o in enumerate(outs):
        np.testing.assert_array_equal(o.result(timeout_s=60), xs[i] * 2)
    assert h.seen.remote().result(timeout_s=60) == ["ndarray"]
    from ray_dynamic_batching_amd.serve.controller import get_controller

    router = get_controller().apps["default"]["Doubler"].router
    assert router.metrics.num_raw_tensor_calls == 24


def test_router_never_pickles_an_array_argument(monkeypatch):
    """The encoding decision itself: cloudpickle.dumps must not be reached."""
    import cloudpickle

    h = serve.run(Doubler.bind(), mode="process")
    assert h.remote(np.ones((2, 2), np.float32)).result(timeout_s=60).sum() == 8     # warm
    real = cloudpickle.dumps

    def guard(obj, *a, **k):
        if isinstance(obj, tuple) and any(isinstance(v, np.ndarray) for v in obj[1] if isinstance(obj[1], tuple)):
            raise AssertionError("an array argument was pickled")
        return real(obj, *a, **k)

    monkeypatch.setattr(cloudpickle, "dumps", guard)
    assert h.remote(np.ones((2, 2), np.float32)).result(timeout_s=60).sum() == 8


def test_native_client_drives_a_batch_deployment():
    """The native load generator's client submits encoded calls (kind 0 + the
    wire magic) straight to the deployment's queue; the Python worker decodes
    them as raw arrays (bench/serve_batch_slice.py --native-client)."""
    import time

    from ray_dynamic_batching_amd.runtime import job as rjob
    from ray_dynamic_batching_amd.serve.controller import get_controller

    h = serve.run(Doubler.bind(), mode="process")
    assert h.remote(np.ones((2, 2), np.float32)).result(timeout_s=60).sum() == 8
    ctrl = get_controller()
    st = ctrl.apps["default"]["Doubler"]
    c = rjob.Client(ctrl.jobs["default"])
    q = c.choose_queue(st.model_id, 0)
    x = np.arange(16, dtype=np.float32).reshape(4, 4)
    rid = c.submit(q, tensor_wire.encode_call("__call__", x))
    got = None
    t_end = time.time() + 30
    while got is None and time.time() < t_end:
        for comp in c.poll(16, 0.2):
            if comp[0] == rid:
                got = comp
    assert got is not None and got[1] == 0 and got[6] == tensor_wire.KIND_TENSOR_RESULT
    np.testing.assert_array_equal(tensor_wire.decode_result(got[7]), x * 2)
