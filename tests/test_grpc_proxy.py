"""gRPC ingress (serve/grpc_proxy.py): routing by the ``application`` metadata
key and method name, raw-bytes and registered-message requests, server
streaming, the RayServeAPIService built-ins and status-code mapping."""
import json
import sys

import cloudpickle
import grpc
import pytest

from ray_dynamic_batching_amd import serve

# replica processes cannot import this test module: ship its classes by value
cloudpickle.register_pickle_by_value(sys.modules[__name__])


@pytest.fixture(autouse=True)
def _shutdown():
    yield
    serve.shutdown()


class Msg:
    """Stand-in for a generated protobuf message (FromString / SerializeToString)."""

    def __init__(self, text: str):
        self.text = text

    @classmethod
    def FromString(cls, data: bytes) -> "Msg":
        return cls(data.decode())

    def SerializeToString(self) -> bytes:
        return self.text.encode()


@serve.deployment(num_replicas=2, max_ongoing_requests=8)
class Echo:
    @serve.batch(max_batch_size=4, batch_wait_timeout_s=0.005)
    async def Upper(self, msgs):
        return [Msg(m.text.upper()) for m in msgs]

    async def Count(self, data):             # raw bytes in, generator out (server streaming)
        for i in range(int(data.decode())):
            yield f"tick {i}".encode()

    async def Fail(self, data):
        raise ValueError("bad request")

    async def __call__(self, data):
        return {"len": len(data)}


@serve.deployment
class Other:
    async def __call__(self, data):
        return b"other:" + data


def _pb_strings(data: bytes):
    """Decode a message made of repeated string field 1 (single-byte lengths)."""
    out, i = [], 0
    while i < len(data):
        assert data[i] == 0x0A
        n = data[i + 1]
        out.append(data[i + 2:i + 2 + n].decode())
        i += 2 + n
    return out


@pytest.mark.parametrize("mode", ["local", "process"])
def test_grpc_routing_streaming_and_builtins(mode):
    serve.start(grpc_options={"port": 0, "request_types": {"/demo.Echo/Upper": Msg},
                              "streaming_methods": ["Count"]})
    port = serve.grpc_port()
    serve.run(Echo.bind(), name="echo", route_prefix=None, mode=mode)
    serve.run(Other.bind(), name="other", route_prefix=None, mode=mode)
    ch = grpc.insecure_channel(f"127.0.0.1:{port}")
    md = (("application", "echo"),)
    upper = ch.unary_unary("/demo.Echo/Upper")
    assert upper(b"hello", metadata=md, timeout=60) == b"HELLO"
    # unknown method on the ingress -> __call__
    assert json.loads(ch.unary_unary("/demo.Echo/Anything")(b"abc", metadata=md, timeout=60)) == {"len": 3}
    assert ch.unary_unary("/x.Y/Z")(b"q", metadata=(("application", "other"),), timeout=60) == b"other:q"
    ticks = list(ch.unary_stream("/demo.Echo/Count")(b"3", metadata=md, timeout=60))
    assert ticks == [b"tick 0", b"tick 1", b"tick 2"]
    with pytest.raises(grpc.RpcError) as e:
        ch.unary_unary("/demo.Echo/Fail")(b"", metadata=md, timeout=60)
    assert e.value.code() == grpc.StatusCode.INTERNAL and "bad request" in e.value.details()
    with pytest.raises(grpc.RpcError) as e:     # two apps and no metadata -> NOT_FOUND
        upper(b"x", timeout=60)
    assert e.value.code() == grpc.StatusCode.NOT_FOUND
    with pytest.raises(grpc.RpcError) as e:
        upper(b"x", metadata=(("application", "nope"),), timeout=60)
    assert e.value.code() == grpc.StatusCode.NOT_FOUND
    apps = ch.unary_unary("/ray.serve.RayServeAPIService/ListApplications")(b"", timeout=30)
    assert _pb_strings(apps) == ["echo", "other"]
    assert _pb_strings(ch.unary_unary("/ray.serve.RayServeAPIService/Healthz")(b"", timeout=30)) == ["success"]
    ch.close()
