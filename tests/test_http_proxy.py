"""HTTP ingress: route-prefix routing, JSON in/out, back-pressure -> 503,
servable tensor deployments over HTTP (local and process mode)."""
import json
import urllib.error
import urllib.request

import numpy as np
import pytest

from ray_dynamic_batching_amd import serve


@pytest.fixture(autouse=True)
def _shutdown():
    yield
    serve.shutdown()


def _post(url, obj):
    req = urllib.request.Request(url, data=json.dumps(obj).encode(), method="POST",
                                 headers={"content-type": "application/json"})
    with urllib.request.urlopen(req, timeout=30) as r:
        return r.status, r.read()


@serve.deployment(num_replicas=2, max_ongoing_requests=8)
class Adder:
    def __init__(self, k):
        self.k = k

    @serve.batch(max_batch_size=4, batch_wait_timeout_s=0.005)
    async def add(self, xs):
        return [x + self.k for x in xs]

    async def __call__(self, request):
        body = await request.json()
        return {"y": await self.add(body["x"]), "path": request.path, "q": request.query_params.get("tag")}


@serve.deployment
class Boom:
    async def __call__(self, request):
        raise ValueError("bad input")


@pytest.mark.parametrize("mode", ["local", "process"])
def test_http_routes_and_json(mode):
    serve.start(http_options={"host": "127.0.0.1", "port": 0})
    port = serve.http_port()
    serve.run(Adder.bind(10), name="adder", route_prefix="/add", mode=mode)
    serve.run(Boom.bind(), name="boom", route_prefix="/boom", mode=mode)
    st, body = _post(f"http://127.0.0.1:{port}/add/sub?tag=t1", {"x": 5})
    out = json.loads(body)
    assert st == 200 and out == {"y": 15, "path": "/add/sub", "q": "t1"}
    with pytest.raises(urllib.error.HTTPError) as e:
        _post(f"http://127.0.0.1:{port}/boom", {})
    assert e.value.code == 500 and b"bad input" in e.value.read()
    with pytest.raises(urllib.error.HTTPError) as e:
        _post(f"http://127.0.0.1:{port}/nowhere", {})
    assert e.value.code == 404
    routes = json.loads(urllib.request.urlopen(f"http://127.0.0.1:{port}/-/routes", timeout=10).read())
    assert routes == {"/add": "adder", "/boom": "boom"}


def test_http_tensor_servable_local():
    from ray_dynamic_batching_amd.models import factories
    from ray_dynamic_batching_amd.models.mlp import MLP

    serve.start(http_options={"host": "127.0.0.1", "port": 0})
    port = serve.http_port()
    d = serve.model_deployment(factories.mlp(), "mlp", max_batch_size=4, batch_wait_timeout_s=0.005)
    serve.run(d.bind(), name="mlp", route_prefix="/mlp", mode="local")
    x = np.random.default_rng(0).standard_normal(32).astype(np.float32)
    st, body = _post(f"http://127.0.0.1:{port}/mlp", {"inputs": x.tolist()})
    got = np.asarray(json.loads(body)["outputs"], dtype=np.float32)
    import torch

    ref = MLP(device="cpu")(torch.from_numpy(x)[None])[0].numpy()
    assert st == 200 and np.allclose(got, ref, atol=1e-5)
