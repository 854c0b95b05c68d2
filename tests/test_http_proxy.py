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


import sys  # noqa: E402

import cloudpickle  # noqa: E402

cloudpickle.register_pickle_by_value(sys.modules[__name__])   # replica processes cannot import tests/

try:     # module level: pydantic keeps the defining namespace of a model, so a model
    # (and app) defined inside a function would drag the app into the pickle
    from fastapi import FastAPI, HTTPException
    from pydantic import BaseModel

    api = FastAPI()

    class Item(BaseModel):
        x: int
        tag: str = "none"

    @serve.deployment(num_replicas=2)
    @serve.ingress(api)
    class Api:
        def __init__(self, k):
            self.k = k

        @api.get("/hello")
        def hello(self, name: str = "world"):
            return {"msg": f"hi {name}", "k": self.k}

        @api.post("/items/{item_id}")
        async def put(self, item_id: int, item: Item):
            return {"id": item_id, "y": item.x * self.k, "tag": item.tag}

        @api.get("/fail")
        def fail(self):
            raise HTTPException(status_code=418, detail="teapot")
except ImportError:      # pragma: no cover
    Api = None


@pytest.mark.parametrize("mode", ["local", "process"])
def test_serve_ingress_fastapi_class_routes(mode):
    """@serve.ingress(FastAPI app): class-method routes bound to the replica
    instance, path/query/body validation, status codes from the app."""
    if Api is None:
        pytest.skip("fastapi not installed")
    serve.start(http_options={"host": "127.0.0.1", "port": 0})
    port = serve.http_port()
    serve.run(Api.bind(3), name="api", route_prefix="/api", mode=mode)
    with urllib.request.urlopen(f"http://127.0.0.1:{port}/api/hello?name=mi355x", timeout=30) as r:
        assert r.status == 200 and json.loads(r.read()) == {"msg": "hi mi355x", "k": 3}
    st, body = _post(f"http://127.0.0.1:{port}/api/items/7", {"x": 5, "tag": "t"})
    assert st == 200 and json.loads(body) == {"id": 7, "y": 15, "tag": "t"}
    with pytest.raises(urllib.error.HTTPError) as e:
        _post(f"http://127.0.0.1:{port}/api/items/7", {"tag": "no x"})       # pydantic validation
    assert e.value.code == 422
    with pytest.raises(urllib.error.HTTPError) as e:
        urllib.request.urlopen(f"http://127.0.0.1:{port}/api/fail", timeout=30)
    assert e.value.code == 418 and b"teapot" in e.value.read()
    with pytest.raises(urllib.error.HTTPError) as e:
        urllib.request.urlopen(f"http://127.0.0.1:{port}/api/missing", timeout=30)
    assert e.value.code == 404
