"""DeploymentHandle / DeploymentResponse / DeploymentResponseGenerator
(reference: python/ray/serve/handle.py:129-856).

* ``handle.remote(*args, **kwargs)`` returns immediately with a
  ``DeploymentResponse`` (awaitable, ``.result(timeout_s)``, ``.cancel()``);
* ``handle.options(method_name=, multiplexed_model_id=, stream=)`` and
  ``handle.<method>.remote(...)`` select the target;
* a ``DeploymentResponse`` passed as an argument to another handle call is
  resolved to its value before the request is sent (composition);
* handles are picklable: a handle shipped to another replica re-binds to the
  deployment's router in that process.
"""
from __future__ import annotations

import asyncio
import collections
import concurrent.futures
import itertools
import queue as _queue
import threading
from dataclasses import dataclass, replace
from typing import Any, Optional

from .exceptions import RayServeException, RequestCancelledError

_req_counter = itertools.count(1)


@dataclass(frozen=True)
class HandleOptions:
    method_name: str = "__call__"
    multiplexed_model_id: str = ""
    stream: bool = False


@dataclass
class RequestMeta:
    request_id: int
    method_name: str
    multiplexed_model_id: str
    stream: bool
    app_name: str
    deployment: str


class DeploymentResponse:
    def __init__(self, fut: concurrent.futures.Future, meta: Optional[RequestMeta] = None, cancel_cb=None):
        self._fut = fut
        self._meta = meta
        self._cancel_cb = cancel_cb

    @property
    def request_id(self) -> int:
        return self._meta.request_id if self._meta else 0

    def result(self, timeout_s: Optional[float] = None, *, _skip_asyncio_check: bool = False) -> Any:
        if not _skip_asyncio_check:
            try:
                asyncio.get_running_loop()
                in_loop = True
            except RuntimeError:
                in_loop = False
            if in_loop and not self._fut.done():
                raise RayServeException("Sync methods should not be called from within an asyncio event loop; "
                                        "use `await response` instead of `response.result()`.")
        try:
            return self._fut.result(timeout=timeout_s)
        except concurrent.futures.TimeoutError:
            raise TimeoutError(f"request {self.request_id} did not finish within {timeout_s}s") from None
        except concurrent.futures.CancelledError:
            raise RequestCancelledError(f"request {self.request_id} was cancelled") from None

    def __await__(self):
        async def _wait():
            try:
                return await asyncio.wrap_future(self._fut)
            except (asyncio.CancelledError, concurrent.futures.CancelledError):
                if self._fut.cancelled():
                    raise RequestCancelledError(f"request {self.request_id} was cancelled") from None
                raise
        return _wait().__await__()

    def cancel(self) -> None:
        if self._cancel_cb is not None:
            self._cancel_cb()
        self._fut.cancel()

    def cancelled(self) -> bool:
        return self._fut.cancelled()

    def done(self) -> bool:
        return self._fut.done()


_END = object()


class StreamSink:
    """Thread-safe FIFO of ``(kind, value)`` stream events that a consumer can
    wait on synchronously (``get``) or from any asyncio loop (``aget``) without
    parking an executor thread per pending item.

    The producer (a router's dispatcher thread or loop) calls ``put``; each
    waiting coroutine is woken with ``call_soon_threadsafe`` on its own loop.
    Reference behaviour: the streaming ObjectRefGenerator a
    ``DeploymentResponseGenerator`` wraps (python/ray/serve/handle.py:620-743)
    is awaited natively on the caller's loop."""

    __slots__ = ("_items", "_cv", "_waiters", "cancelled")

    def __init__(self):
        self.cancelled = False            # set by the router's cancel(): a queued request is never sent
        self._items: collections.deque = collections.deque()
        self._cv = threading.Condition(threading.Lock())
        self._waiters: list = []          # [(loop, future)] of async consumers

    def put(self, ev) -> None:
        with self._cv:
            self._items.append(ev)
            self._cv.notify()
            waiters, self._waiters = self._waiters, []
        for loop, fut in waiters:
            try:
                loop.call_soon_threadsafe(_wake_future, fut)
            except RuntimeError:          # the consumer's loop is closed
                pass

    # queue.Queue-compatible producer / consumer names
    put_nowait = put

    def get(self, timeout: Optional[float] = None):
        with self._cv:
            if not self._cv.wait_for(lambda: self._items, timeout):
                raise _queue.Empty
            return self._items.popleft()

    def get_nowait(self):
        with self._cv:
            if not self._items:
                raise _queue.Empty
            return self._items.popleft()

    async def aget(self):
        loop = asyncio.get_running_loop()
        while True:
            with self._cv:
                if self._items:
                    return self._items.popleft()
                fut = loop.create_future()
                self._waiters.append((loop, fut))
            await fut

    def qsize(self) -> int:
        with self._cv:
            return len(self._items)

    def empty(self) -> bool:
        return self.qsize() == 0


def _wake_future(fut) -> None:
    if not fut.done():
        fut.set_result(None)


class DeploymentResponseGenerator:
    """Streaming response: iterate (sync or async) over the items the
    replica's generator yields.  ``async for`` awaits the sink on the caller's
    own loop (no thread per pending item)."""

    def __init__(self, q: "StreamSink", meta: Optional[RequestMeta] = None, cancel_cb=None):
        self._q = q
        self._meta = meta
        self._cancel_cb = cancel_cb
        self._done = False

    def _take(self, ev):
        kind, val = ev
        if kind == "item":
            return val
        self._done = True
        if kind == "error":
            raise val
        raise StopIteration

    def _next(self, timeout=None):
        if self._done:
            raise StopIteration
        return self._take(self._q.get(timeout=timeout))

    def __iter__(self):
        return self

    def __next__(self):
        return self._next()

    def __aiter__(self):
        return self

    async def __anext__(self):
        if self._done:
            raise StopAsyncIteration
        if isinstance(self._q, StreamSink):
            ev = await self._q.aget()
        else:                              # a plain queue.Queue from user code
            ev = await asyncio.get_running_loop().run_in_executor(None, self._q.get)
        try:
            return self._take(ev)
        except StopIteration:
            raise StopAsyncIteration from None

    def cancel(self) -> None:
        if self._cancel_cb:
            self._cancel_cb()
        self._done = True


class DeploymentHandle:
    def __init__(self, deployment_name: str, app_name: str = "default", options: HandleOptions = HandleOptions(),
                 _router=None):
        self.deployment_name = deployment_name
        self.app_name = app_name
        self._options = options
        self._router = _router
        self._lock = threading.Lock()

    # -- routing -----------------------------------------------------------
    def _get_router(self):
        if self._router is None:
            with self._lock:
                if self._router is None:
                    from .controller import lookup_router

                    self._router = lookup_router(self.app_name, self.deployment_name)
        return self._router

    def options(self, *, method_name: Optional[str] = None, multiplexed_model_id: Optional[str] = None,
                stream: Optional[bool] = None, **unsupported) -> "DeploymentHandle":
        if unsupported:
            unknown = set(unsupported) - {"use_new_handle_api", "_prefer_local_routing"}
            if unknown:
                raise TypeError(f"unsupported handle options: {sorted(unknown)}")
        o = self._options
        o = replace(o, method_name=method_name if method_name is not None else o.method_name,
                    multiplexed_model_id=multiplexed_model_id if multiplexed_model_id is not None else o.multiplexed_model_id,
                    stream=stream if stream is not None else o.stream)
        return DeploymentHandle(self.deployment_name, self.app_name, o, self._router)

    def remote(self, *args, **kwargs):
        meta = RequestMeta(next(_req_counter), self._options.method_name, self._options.multiplexed_model_id,
                           self._options.stream, self.app_name, self.deployment_name)
        return self._get_router().assign(meta, args, kwargs)

    def __getattr__(self, name: str):
        if name.startswith("_"):
            raise AttributeError(name)
        return self.options(method_name=name)

    def __reduce__(self):
        return (DeploymentHandle, (self.deployment_name, self.app_name, self._options))

    def __repr__(self) -> str:
        return f"DeploymentHandle(deployment={self.deployment_name!r}, app={self.app_name!r})"
