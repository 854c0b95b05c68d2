"""HTTP ingress (reference: serve/_private/proxy.py:136-1153 HTTPProxy over
uvicorn/ASGI; back-pressure -> HTTP 503, serve/api.py:299-303).

One proxy per controller, on a uvicorn thread.  A request to
``<route_prefix>/...`` is routed (longest prefix) to that application's
ingress deployment through the normal DeploymentHandle path:

* Python deployments receive an :class:`HTTPRequest` (picklable, starlette-like:
  ``await request.json()``, ``await request.body()``, ``.query_params``,
  ``.headers``, ``.method``, ``.path``);
* servable-model deployments (tensor codec) receive the JSON body as an array
  (``{"inputs": [...]}`` or a bare list) and answer ``{"outputs": [...]}``.

Results: dict / list / str / numbers -> JSON; numpy arrays -> JSON lists;
bytes -> application/octet-stream.
"""
from __future__ import annotations

import asyncio
import json
import logging
import threading
import time
from typing import Any, Dict, Optional

logger = logging.getLogger("ray_dynamic_batching_amd.serve")


class HTTPRequest:
    """Picklable subset of starlette's Request handed to the ingress deployment."""

    def __init__(self, method: str, path: str, query_params: Dict[str, str], headers: Dict[str, str], body: bytes,
                 route_path: str = ""):
        self.method = method
        self.path = path
        self.url_path = path
        self.route_path = route_path or path      # path below the application's route prefix
        self.query_params = query_params
        self.headers = headers
        self._body = body

    async def body(self) -> bytes:
        return self._body

    async def json(self) -> Any:
        return json.loads(self._body or b"null")

    def json_sync(self) -> Any:
        return json.loads(self._body or b"null")

    def __repr__(self) -> str:
        return f"HTTPRequest({self.method} {self.path}, {len(self._body)} bytes)"


def _encode(result: Any):
    import numpy as np

    if isinstance(result, (bytes, bytearray)):
        return bytes(result), "application/octet-stream"
    if isinstance(result, np.ndarray):
        result = result.tolist()
    elif hasattr(result, "detach"):
        result = result.detach().cpu().tolist()
    if isinstance(result, str):
        return result.encode(), "text/plain; charset=utf-8"
    return json.dumps(result, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o)).encode(), \
        "application/json"


class HTTPProxy:
    def __init__(self, controller, host: str = "127.0.0.1", port: int = 8000):
        self.controller = controller
        self.host = host
        self.port = port
        self.server = None
        self.thread: Optional[threading.Thread] = None
        self.num_requests = 0
        self.num_errors = 0

    # -- routing
    def _match(self, path: str):
        best = None
        for app, prefix in self.controller.route_prefixes.items():
            if prefix is None:
                continue
            p = prefix.rstrip("/")
            if path == p or path.startswith(p + "/") or p == "":
                if best is None or len(p) > len(best[1]):
                    best = (app, p)
        return best

    def _asgi_app(self):
        from starlette.applications import Starlette
        from starlette.responses import JSONResponse, Response
        from starlette.routing import Route

        from .exceptions import BackPressureError, RequestDroppedError

        async def handle(request):
            self.num_requests += 1
            m = self._match(request.url.path)
            if m is None:
                return JSONResponse({"error": f"no application at {request.url.path}"}, status_code=404)
            app_name, prefix = m
            try:
                handle_ = self.controller.get_app_handle(app_name)
                body = await request.body()
                ingress = self.controller.apps[app_name][self.controller.ingress[app_name]]
                if ingress.codec is not None or getattr(ingress.deployment, "servable", None) is not None:
                    # tensor servable: JSON array in, JSON array out
                    import numpy as np

                    data = json.loads(body or b"null")
                    arr = np.asarray(data["inputs"] if isinstance(data, dict) else data)
                    result = await handle_.remote(arr)
                    payload, ctype = _encode({"outputs": result})
                else:
                    sub = request.url.path[len(prefix):] or "/"
                    req = HTTPRequest(request.method, request.url.path, dict(request.query_params),
                                      dict(request.headers), body, route_path=sub)
                    result = await handle_.remote(req)
                    from .ingress import ASGIResponse

                    if isinstance(result, ASGIResponse):        # @serve.ingress app: its own status / headers
                        hdrs = {k.decode(): v.decode() for k, v in result.headers if k.lower() != b"content-length"}
                        return Response(result.body, status_code=result.status, headers=hdrs)
                    payload, ctype = _encode(result)
                return Response(payload, media_type=ctype)
            except BackPressureError as e:
                self.num_errors += 1
                return JSONResponse({"error": str(e)}, status_code=503)
            except RequestDroppedError as e:
                self.num_errors += 1
                return JSONResponse({"error": str(e)}, status_code=503)
            except Exception as e:  # user error -> 500 with the message
                self.num_errors += 1
                return JSONResponse({"error": f"{type(e).__name__}: {e}"}, status_code=500)

        async def health(request):
            return Response(b"success", media_type="text/plain")

        async def routes(request):
            return JSONResponse({p or "/": a for a, p in self.controller.route_prefixes.items() if p is not None})

        async def metrics(request):
            from starlette.responses import PlainTextResponse

            return PlainTextResponse(self.controller.metrics_text(), media_type="text/plain; version=0.0.4")

        return Starlette(routes=[Route("/-/healthz", health), Route("/-/routes", routes), Route("/-/metrics", metrics),
                                 Route("/{path:path}", handle, methods=["GET", "POST", "PUT", "DELETE"])])

    def start(self, timeout_s: float = 30.0) -> "HTTPProxy":
        import uvicorn

        cfg = uvicorn.Config(self._asgi_app(), host=self.host, port=self.port, log_level="warning", lifespan="off",
                             loop="asyncio")
        self.server = uvicorn.Server(cfg)
        self.server.install_signal_handlers = lambda: None   # run off the main thread
        self.thread = threading.Thread(target=self._serve, name="rdb-http-proxy", daemon=True)
        self.thread.start()
        t_end = time.time() + timeout_s
        while not self.server.started and time.time() < t_end:
            if not self.thread.is_alive():
                raise RuntimeError(f"HTTP proxy failed to start on {self.host}:{self.port}")
            time.sleep(0.01)
        if self.server.started and self.port == 0:
            self.port = self.server.servers[0].sockets[0].getsockname()[1]
        return self

    def _serve(self):
        loop = asyncio.new_event_loop()
        asyncio.set_event_loop(loop)
        try:
            loop.run_until_complete(self.server.serve())
        finally:
            loop.close()

    def stop(self):
        if self.server is not None:
            self.server.should_exit = True
        if self.thread is not None and self.thread.is_alive():
            self.thread.join(5.0)
        self.server = None
