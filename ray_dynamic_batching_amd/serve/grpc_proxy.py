"""gRPC ingress (reference: serve/_private/proxy.py gRPCProxy, serve/config.py
gRPCOptions; routing by the ``application`` metadata key, method name ->
deployment method, ``ray.serve.RayServeAPIService`` ListApplications /
Healthz).

No generated stubs are needed on the server: one generic handler accepts every
``/<package.Service>/<Method>`` path with raw-bytes (de)serialisation.

* The target application comes from the ``application`` metadata key (or the
  only application when there is exactly one), the deployment method from the
  RPC's method name (``__call__`` if the ingress has no such method).
* The method receives the request message: an instance of the class
  registered for that RPC path in ``grpc_options["request_types"]`` (its
  ``FromString`` is called), else the raw request ``bytes``.
* The reply is serialised with ``SerializeToString()`` when it has one, else
  ``bytes`` pass through, ``str`` is UTF-8 encoded and anything else JSON.
* Methods listed in ``grpc_options["streaming_methods"]`` are server-streaming:
  the deployment method is called with ``stream=True`` and every yielded item
  is one reply message.
* Errors: unknown application -> NOT_FOUND, back-pressure / dropped request ->
  UNAVAILABLE, user exception -> INTERNAL with the message.
"""
from __future__ import annotations

import json
import logging
from concurrent import futures
from typing import Any, Callable, Dict, Iterable, Optional

logger = logging.getLogger("ray_dynamic_batching_amd.serve")

SERVE_API_SERVICE = "ray.serve.RayServeAPIService"


def _pb_string_field(field: int, s: str) -> bytes:
    """Protobuf wire encoding of one length-delimited (string) field."""
    data = s.encode()
    out = bytearray([(field << 3) | 2])
    n = len(data)
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            break
    return bytes(out) + data


def _encode_reply(result: Any) -> bytes:
    if hasattr(result, "SerializeToString"):
        return result.SerializeToString()
    if isinstance(result, (bytes, bytearray)):
        return bytes(result)
    if isinstance(result, str):
        return result.encode()
    if hasattr(result, "tolist"):
        result = result.tolist()
    return json.dumps(result, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o)).encode()


class GRPCProxy:
    def __init__(self, controller, host: str = "127.0.0.1", port: int = 9000,
                 request_types: Optional[Dict[str, Any]] = None, streaming_methods: Iterable[str] = (),
                 max_workers: int = 32, timeout_s: float = 600.0):
        self.controller = controller
        self.host = host
        self.port = port
        self.request_types = dict(request_types or {})
        self.streaming_methods = set(streaming_methods)
        self.max_workers = max_workers
        self.timeout_s = timeout_s
        self.server = None
        self.num_requests = 0
        self.num_errors = 0

    # -- routing -----------------------------------------------------------
    def _app_for(self, context) -> Optional[str]:
        md = dict(context.invocation_metadata() or ())
        app = md.get("application")
        if app:
            return app if app in self.controller.apps else None
        apps = list(self.controller.apps)
        return apps[0] if len(apps) == 1 else None

    def _target(self, app: str, method: str):
        handle = self.controller.get_app_handle(app)
        ingress = self.controller.apps[app][self.controller.ingress[app]]
        cls = ingress.deployment.func_or_class
        name = method if isinstance(cls, type) and hasattr(cls, method) else "__call__"
        return handle, name

    def _decode(self, path: str, data: bytes):
        t = self.request_types.get(path)
        return t.FromString(data) if t is not None else data

    def _fail(self, context, e: Exception):
        import grpc

        from .exceptions import BackPressureError, RequestDroppedError

        self.num_errors += 1
        if isinstance(e, (BackPressureError, RequestDroppedError)):
            context.abort(grpc.StatusCode.UNAVAILABLE, str(e))
        context.abort(grpc.StatusCode.INTERNAL, f"{type(e).__name__}: {e}")

    # -- handlers ------------------------------------------------------------
    def _unary(self, path: str, method: str) -> Callable:
        import grpc

        def call(data: bytes, context):
            self.num_requests += 1
            app = self._app_for(context)
            if app is None:
                context.abort(grpc.StatusCode.NOT_FOUND, "application not found: set the 'application' metadata key "
                              f"to one of {sorted(self.controller.apps)}")
            try:
                handle, name = self._target(app, method)
                res = handle.options(method_name=name).remote(self._decode(path, data)).result(timeout_s=self.timeout_s)
                return _encode_reply(res)
            except Exception as e:  # noqa: BLE001 - mapped to a status code
                self._fail(context, e)

        return call

    def _stream(self, path: str, method: str) -> Callable:
        import grpc

        def call(data: bytes, context):
            self.num_requests += 1
            app = self._app_for(context)
            if app is None:
                context.abort(grpc.StatusCode.NOT_FOUND, "application not found")
            try:
                handle, name = self._target(app, method)
                for item in handle.options(method_name=name, stream=True).remote(self._decode(path, data)):
                    yield _encode_reply(item)
            except Exception as e:  # noqa: BLE001
                self._fail(context, e)

        return call

    def _builtin(self, method: str) -> Callable:
        def call(data: bytes, context):
            if method == "ListApplications":   # ListApplicationsResponse{repeated string application_names = 1}
                return b"".join(_pb_string_field(1, a) for a in sorted(self.controller.apps))
            return _pb_string_field(1, "success")  # HealthzResponse{string message = 1}

        return call

    def _generic(self):
        import grpc

        proxy = self

        class Handler(grpc.GenericRpcHandler):
            def service(self, details):
                path = details.method                    # "/package.Service/Method"
                try:
                    service, method = path.rsplit("/", 1)
                except ValueError:
                    return None
                service = service.lstrip("/")
                if service == SERVE_API_SERVICE and method in ("ListApplications", "Healthz"):
                    return grpc.unary_unary_rpc_method_handler(proxy._builtin(method))
                if method in proxy.streaming_methods or path in proxy.streaming_methods:
                    return grpc.unary_stream_rpc_method_handler(proxy._stream(path, method))
                return grpc.unary_unary_rpc_method_handler(proxy._unary(path, method))

        return Handler()

    def start(self) -> "GRPCProxy":
        import grpc

        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=self.max_workers),
                                  handlers=[self._generic()])
        bound = self.server.add_insecure_port(f"{self.host}:{self.port}")
        if bound == 0:
            raise RuntimeError(f"gRPC proxy could not bind {self.host}:{self.port}")
        self.port = bound
        self.server.start()
        return self

    def stop(self, grace_s: float = 1.0) -> None:
        if self.server is not None:
            self.server.stop(grace_s).wait(grace_s + 5)
            self.server = None
