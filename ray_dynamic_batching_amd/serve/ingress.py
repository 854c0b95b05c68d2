"""``@serve.ingress(fastapi_app)``: a deployment class whose HTTP surface is a
FastAPI (or any ASGI) app.

Reference: ``python/ray/serve/api.py`` ``ingress`` and
``serve/_private/http_util.py`` ``make_fastapi_class_based_view`` -- route
handlers written as methods of the deployment class (``def f(self, ...)``)
run with ``self`` bound to the replica instance.  Here:

* the decorator records the app on the class and gives it an async
  ``__call__(request)``;
* each replica builds its OWN copy of the app on first use, re-registering
  every route whose endpoint is a method of the class as the bound method (so
  FastAPI's signature analysis sees the parameters without ``self``, and
  dependency injection, validation, response models keep working);
* the proxy's :class:`~.http_proxy.HTTPRequest` (route prefix stripped) is
  replayed through the app as one ASGI ``http`` request, and the complete
  response (status, headers, body) goes back to the proxy as an
  :class:`ASGIResponse`.
"""
from __future__ import annotations

import types
from typing import Any, List, Tuple
from urllib.parse import urlencode


class ASGIResponse:
    """A finished HTTP response produced inside the replica."""

    def __init__(self, status: int, headers: List[Tuple[bytes, bytes]], body: bytes):
        self.status = status
        self.headers = headers
        self.body = body

    def header(self, name: str, default: str = "") -> str:
        n = name.lower().encode()
        for k, v in self.headers:
            if k.lower() == n:
                return v.decode()
        return default

    def json(self) -> Any:
        import json

        return json.loads(self.body or b"null")

    def __repr__(self) -> str:
        return f"ASGIResponse({self.status}, {len(self.body)} bytes)"


async def call_asgi(app, method: str, path: str, query: str, headers, body: bytes) -> ASGIResponse:
    scope = {"type": "http", "asgi": {"version": "3.0", "spec_version": "2.3"}, "http_version": "1.1",
             "method": method.upper(), "scheme": "http", "path": path or "/", "raw_path": (path or "/").encode(),
             "root_path": "", "query_string": query.encode(),
             "headers": [(str(k).lower().encode(), str(v).encode()) for k, v in dict(headers).items()],
             "client": ("127.0.0.1", 0), "server": ("127.0.0.1", 80)}
    pending = [{"type": "http.request", "body": body or b"", "more_body": False}]
    out = {"status": 500, "headers": [], "body": b""}

    async def receive():
        return pending.pop(0) if pending else {"type": "http.disconnect"}

    async def send(msg):
        if msg["type"] == "http.response.start":
            out["status"], out["headers"] = msg["status"], list(msg.get("headers", []))
        elif msg["type"] == "http.response.body":
            out["body"] += msg.get("body", b"")

    await app(scope, receive, send)
    return ASGIResponse(out["status"], out["headers"], out["body"])


def _route_recipe(app):
    """The app's routes as plain data + functions (a FastAPI app object does
    not survive pickling -- starlette's ``State`` recurses in ``__getattr__``
    while unpickling -- so replica processes rebuild it from this)."""
    from fastapi.routing import APIRoute

    routes = []
    for r in app.router.routes:
        if isinstance(r, APIRoute):
            routes.append(dict(path=r.path, endpoint=r.endpoint, methods=sorted(r.methods or ["GET"]),
                               response_model=r.response_model, status_code=r.status_code, name=r.name,
                               response_class=r.response_class))
    handlers = dict(getattr(app, "exception_handlers", {}))
    return dict(title=getattr(app, "title", "FastAPI"), routes=routes, handlers=handlers)


def _bind_app(recipe, cls, instance):
    """A per-replica FastAPI app with class-method routes bound to ``instance``."""
    from fastapi import FastAPI

    own = FastAPI(title=recipe["title"])
    members = set()
    for klass in cls.__mro__:
        members |= {id(v) for v in vars(klass).values() if isinstance(v, types.FunctionType)}
    for r in recipe["routes"]:
        ep = r["endpoint"]
        if id(ep) in members:
            ep = types.MethodType(ep, instance)
        own.add_api_route(r["path"], ep, methods=r["methods"], response_model=r["response_model"],
                          status_code=r["status_code"], name=r["name"], response_class=r["response_class"])
    for exc, handler in recipe["handlers"].items():
        if getattr(handler, "__module__", "").startswith(("fastapi", "starlette")):
            continue                     # the new app installs the framework's defaults itself
        own.add_exception_handler(exc, handler)
    return own


def ingress(app):
    """Class decorator: serve ``app`` (FastAPI / Starlette / any ASGI callable)
    as this deployment's HTTP interface."""

    def deco(cls):
        if not isinstance(cls, type):
            raise TypeError("@serve.ingress decorates a deployment class")
        if "__call__" in vars(cls):
            raise ValueError("an @serve.ingress class must not define __call__ (the app handles requests)")
        # routes are read HERE: the class body (whose @app.get(...) methods
        # register them) runs after ``ingress(app)`` is evaluated
        try:
            from fastapi import FastAPI
            recipe = _route_recipe(app) if isinstance(app, FastAPI) else None
        except ImportError:
            recipe = None

        async def __call__(self, request):
            asgi = self.__dict__.get("_rdb_asgi_app")
            if asgi is None:
                asgi = _bind_app(recipe, type(self), self) if recipe is not None else type(self).__serve_asgi_app__
                self.__dict__["_rdb_asgi_app"] = asgi
            path = getattr(request, "route_path", None) or request.path
            return await call_asgi(asgi, request.method, path, urlencode(request.query_params), request.headers,
                                   await request.body())

        cls.__call__ = __call__
        if recipe is None:
            cls.__serve_asgi_app__ = app     # a plain ASGI app must be picklable itself
        return cls

    return deco
