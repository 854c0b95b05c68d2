"""Replica: hosts one instance of the user's deployment class/function.

Reference behaviour (serve/_private/replica.py:233-1270): all user code runs
on a dedicated user-code event loop (sync methods block it, as in Serve);
``reconfigure(user_config)`` is called at start and on config updates;
``check_health()`` is the user health hook; generators stream.

``UserCallable`` is shared by both execution modes:
* ``LocalReplica`` -- in-process, own event-loop thread (local mode);
* the replica process main loop (replica_main.py) -- one process per GPU slot.
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import inspect
import logging
import threading
import time
import traceback
from typing import Any, Dict, Optional

from .context import ReplicaContext, RequestContext, _set_replica_context, _set_request_context
from .handle import RequestMeta, StreamSink

logger = logging.getLogger("ray_dynamic_batching_amd.serve")


class UserCallable:
    def __init__(self, func_or_class, init_args, init_kwargs, user_config=None, access_log=None):
        from .logging_utils import AccessLog

        self.access = access_log or AccessLog(None, False)
        self.is_function = not inspect.isclass(func_or_class)
        self.func_or_class = func_or_class
        if self.is_function:
            self.obj = None
        else:
            self.obj = func_or_class(*init_args, **init_kwargs)
            if user_config is not None:
                self.reconfigure(user_config)

    def reconfigure(self, user_config) -> None:
        if self.obj is None:
            return
        fn = getattr(self.obj, "reconfigure", None)
        if fn is None:
            raise ValueError("user_config given but the deployment class has no reconfigure() method")
        r = fn(user_config)
        if inspect.isawaitable(r):
            asyncio.get_event_loop().run_until_complete(r) if not asyncio.get_event_loop().is_running() else None

    def resolve(self, method_name: str):
        if self.is_function:
            return self.func_or_class
        m = getattr(self.obj, method_name, None)
        if m is None:
            raise AttributeError(f"deployment has no method {method_name!r}")
        return m

    async def call(self, meta: RequestMeta, args, kwargs) -> Any:
        token = _set_request_context(RequestContext(meta.request_id, meta.multiplexed_model_id, meta.method_name))
        t0 = time.perf_counter()
        status = "ERROR"
        try:
            fn = self.resolve(meta.method_name)
            r = fn(*args, **kwargs)
            if inspect.isawaitable(r):
                r = await r
            status = "OK"
            return r
        except asyncio.CancelledError:
            status = "CANCELLED"
            raise
        finally:
            self.access.record(meta, status, time.perf_counter() - t0)
            from .context import _request_ctx

            _request_ctx.reset(token)

    async def call_stream(self, meta: RequestMeta, args, kwargs, emit) -> None:
        """Drive a (sync or async) generator method; emit(kind, value)."""
        token = _set_request_context(RequestContext(meta.request_id, meta.multiplexed_model_id, meta.method_name))
        t0 = time.perf_counter()
        status = "ERROR"
        try:
            fn = self.resolve(meta.method_name)
            g = fn(*args, **kwargs)
            if inspect.isasyncgen(g):
                async for item in g:
                    emit("item", item)
            elif inspect.isgenerator(g):
                for item in g:
                    emit("item", item)
            else:
                if inspect.isawaitable(g):
                    g = await g
                emit("item", g)
            emit("end", None)
            status = "OK"
        except Exception as e:
            emit("error", e)
        finally:
            self.access.record(meta, status, time.perf_counter() - t0)
            from .context import _request_ctx

            _request_ctx.reset(token)

    async def check_health(self) -> None:
        fn = getattr(self.obj, "check_health", None) if self.obj is not None else None
        if fn is not None:
            r = fn()
            if inspect.isawaitable(r):
                await r

    def destroy(self) -> None:
        fn = getattr(self.obj, "__del__", None) if self.obj is not None else None
        if fn is not None:
            try:
                fn()
            except Exception:  # pragma: no cover
                pass


class LocalReplica:
    """In-process replica with its own user-code event-loop thread."""

    def __init__(self, app_name: str, deployment: str, index: int, func_or_class, init_args, init_kwargs,
                 config, gpu: Optional[int] = None):
        self.app_name = app_name
        self.deployment = deployment
        self.index = index
        self.replica_id = f"{app_name}#{deployment}#{index}"
        self.config = config
        self.max_ongoing = config.max_ongoing_requests
        self.ongoing = 0              # owned by the router loop
        self.loaded_models: set = set()
        self.healthy = True
        self.dead = False
        self.started_at = time.time()
        self.processed = 0
        self.errors = 0
        self._loop = asyncio.new_event_loop()
        ready = concurrent.futures.Future()
        self.ctx = ReplicaContext(app_name, deployment, self.replica_id, index, None, self.max_ongoing, gpu)
        from .logging_utils import AccessLog, configure_replica_logger

        lcfg = config.get_logging_config()
        self.logger = configure_replica_logger(app_name, deployment, index, self.replica_id, lcfg)
        access = AccessLog(self.logger, lcfg is None or lcfg.enable_access_log)

        def run():
            asyncio.set_event_loop(self._loop)
            _set_replica_context(self.ctx)
            try:
                self.user = UserCallable(func_or_class, init_args, init_kwargs, config.user_config, access)
                self.ctx.servable_object = self.user.obj
                ready.set_result(True)
            except BaseException as e:  # constructor failure
                ready.set_exception(e)
                return
            self._loop.run_forever()

        self._thread = threading.Thread(target=run, name=f"replica-{self.replica_id}", daemon=True)
        self._thread.start()
        ready.result()

    def call(self, meta: RequestMeta, args, kwargs) -> concurrent.futures.Future:
        return asyncio.run_coroutine_threadsafe(self._wrapped(meta, args, kwargs), self._loop)

    async def _wrapped(self, meta, args, kwargs):
        try:
            r = await self.user.call(meta, args, kwargs)
            self.processed += 1
            if meta.multiplexed_model_id:
                self.loaded_models.add(meta.multiplexed_model_id)
            return r
        except Exception:
            self.errors += 1
            raise

    def call_stream(self, meta: RequestMeta, args, kwargs) -> "StreamSink":
        q = StreamSink()
        asyncio.run_coroutine_threadsafe(self.user.call_stream(meta, args, kwargs, lambda k, v: q.put((k, v))),
                                         self._loop)
        return q

    def poll_health(self, now: float, period_s: float, timeout_s: float) -> Optional[bool]:
        """Non-blocking health check for the controller loop (the reference's
        controller awaits ``check_health`` actor calls with a timeout and never
        blocks its loop on one): starts a check every ``period_s``; returns
        True / False once a check finished or timed out, None while none did."""
        if self.dead:
            return False
        f = getattr(self, "_hc_future", None)
        if f is not None:
            if f.done():
                self._hc_future = None
                try:
                    f.result()
                    return True
                except Exception:
                    logger.warning("health check failed for %s:\n%s", self.replica_id, traceback.format_exc())
                    return False
            if now - self._hc_started > timeout_s:
                self._hc_future = None
                f.cancel()
                logger.warning("health check of %s timed out after %.1fs", self.replica_id, timeout_s)
                return False
            return None
        if now - getattr(self, "_hc_started", float("-inf")) >= period_s:
            self._hc_started = now
            self._hc_future = asyncio.run_coroutine_threadsafe(self.user.check_health(), self._loop)
        return None

    def check_health(self, timeout_s: float) -> bool:
        if self.dead:
            return False
        try:
            asyncio.run_coroutine_threadsafe(self.user.check_health(), self._loop).result(timeout_s)
            return True
        except Exception:
            logger.warning("health check failed for %s:\n%s", self.replica_id, traceback.format_exc())
            return False

    def reconfigure(self, user_config) -> None:
        async def _rc():
            fn = getattr(self.user.obj, "reconfigure", None)
            if fn is not None:
                r = fn(user_config)
                if inspect.isawaitable(r):
                    await r
        asyncio.run_coroutine_threadsafe(_rc(), self._loop).result(30)

    def shutdown(self, graceful_timeout_s: float = 5.0) -> None:
        if self.dead:
            return
        deadline = time.time() + graceful_timeout_s
        while self.ongoing > 0 and time.time() < deadline:
            time.sleep(0.01)
        self.dead = True

        async def _stop():
            self.user.destroy()
            # cancel the @batch queue loops (and any other background tasks) so the
            # loop stops with nothing pending
            me = asyncio.current_task()
            rest = [t for t in asyncio.all_tasks() if t is not me]
            for t in rest:
                t.cancel()
            await asyncio.gather(*rest, return_exceptions=True)
        try:
            asyncio.run_coroutine_threadsafe(_stop(), self._loop).result(2)
        except Exception:  # pragma: no cover
            pass
        self._loop.call_soon_threadsafe(self._loop.stop)

    def stats(self) -> Dict[str, Any]:
        return dict(replica_id=self.replica_id, ongoing=self.ongoing, processed=self.processed, errors=self.errors,
                    healthy=self.healthy and not self.dead, uptime_s=time.time() - self.started_at)
