"""Request routers: power-of-two-choices by queue depth, FIFO pending queue,
``max_ongoing_requests`` admission, ``max_queued_requests`` back-pressure,
model-multiplexing affinity, retry on replica death.

Reference: serve/_private/router.py:313-566 and
replica_scheduler/pow_2_scheduler.py:346-835.  Differences by design:
* the queue length of a replica is read from memory (local mode) or from two
  shm atomics (process mode, via the native Client) -- there is no probe RPC,
  no queue-length cache and no probe back-off to tune;
* process-mode routing and submission are native (runtime.cpp Client).
"""
from __future__ import annotations

import asyncio
import collections
import concurrent.futures
import logging
import random
import threading
import time
import traceback
from typing import Any, Callable, Deque, Dict, List, Optional, Tuple

from .exceptions import (BackPressureError, DeploymentUnavailableError, RayServeException, ReplicaDiedError,
                         RequestCancelledError)
from . import tensor_wire
from .handle import DeploymentResponse, DeploymentResponseGenerator, RequestMeta, StreamSink

logger = logging.getLogger("ray_dynamic_batching_amd.serve")


def _has_response_args(args, kwargs) -> bool:
    return any(isinstance(a, DeploymentResponse) for a in args) or any(
        isinstance(v, DeploymentResponse) for v in kwargs.values())


async def _resolve_args(args, kwargs):
    """Composition: DeploymentResponse arguments are replaced by their values."""
    if not _has_response_args(args, kwargs):
        return args, kwargs
    args = list(args)
    for i, a in enumerate(args):
        if isinstance(a, DeploymentResponse):
            args[i] = await a
    kwargs = dict(kwargs)
    for k, v in kwargs.items():
        if isinstance(v, DeploymentResponse):
            kwargs[k] = await v
    return tuple(args), kwargs


class _LoopThread:
    """A private asyncio loop on a daemon thread (Serve's router loop)."""

    _shared: Optional["_LoopThread"] = None
    _lock = threading.Lock()

    def __init__(self, name="rdb-router"):
        self.loop = asyncio.new_event_loop()
        self.thread = threading.Thread(target=self._run, name=name, daemon=True)
        self.thread.start()

    def _run(self):
        asyncio.set_event_loop(self.loop)
        self.loop.run_forever()

    @classmethod
    def shared(cls) -> "_LoopThread":
        with cls._lock:
            if cls._shared is None or not cls._shared.thread.is_alive():
                cls._shared = _LoopThread()
            return cls._shared


class RouterMetrics:
    """serve_num_router_requests / serve_deployment_queued_queries equivalents."""

    def __init__(self):
        self.num_router_requests = 0
        self.num_queued = 0
        self.num_rejected_backpressure = 0
        self.num_retries = 0
        self.num_raw_tensor_calls = 0     # array arguments sent as raw bytes (tensor_wire), not pickled


class LocalRouter:
    """Routes to in-process LocalReplica objects."""

    def __init__(self, deployment: str, max_queued_requests: int = -1, seed: Optional[int] = None):
        self.deployment = deployment
        self.max_queued = max_queued_requests
        self.replicas: List = []
        self._lt = _LoopThread.shared()
        self._waiters: Deque[asyncio.Future] = collections.deque()
        self._rng = random.Random(seed)
        self.metrics = RouterMetrics()
        self._pending_count = 0

    # replica set updates come from the controller thread
    def update_replicas(self, replicas: List) -> None:
        def _set():
            self.replicas = [r for r in replicas if not r.dead]
            self._wake()
        self._lt.loop.call_soon_threadsafe(_set)

    def set_max_queued_requests(self, v: int) -> None:
        self.max_queued = v

    def num_queued(self) -> int:
        return self._pending_count

    def total_ongoing(self) -> int:
        return sum(r.ongoing for r in self.replicas) + self._pending_count

    # --- replica choice (runs on the router loop) -------------------------
    def _choose(self, meta: RequestMeta):
        cands = [r for r in self.replicas if not r.dead and r.ongoing < r.max_ongoing]
        if not cands:
            return None
        if meta.multiplexed_model_id:
            with_model = [r for r in cands if meta.multiplexed_model_id in r.loaded_models]
            if with_model:
                cands = with_model
        if len(cands) == 1:
            return cands[0]
        a, b = self._rng.sample(cands, 2)
        return a if a.ongoing <= b.ongoing else b

    def _wake(self) -> None:
        while self._waiters:
            w = self._waiters.popleft()
            if not w.done():
                w.set_result(None)
                return

    async def _acquire(self, meta: RequestMeta):
        r = self._choose(meta)
        if r is not None and not self._waiters:
            return r
        self._pending_count += 1
        self.metrics.num_queued += 1
        try:
            while True:
                w = self._lt.loop.create_future()
                self._waiters.append(w)
                await w
                r = self._choose(meta)
                if r is not None:
                    if self._waiters:  # keep the FIFO moving
                        self._lt.loop.call_soon(self._wake)
                    return r
        finally:
            self._pending_count -= 1

    async def _assign(self, meta: RequestMeta, args, kwargs, attempt: int = 0):
        args, kwargs = await _resolve_args(args, kwargs)
        r = await self._acquire(meta)
        r.ongoing += 1
        try:
            if r.dead:
                raise ReplicaDiedError(r.replica_id)
            return await asyncio.wrap_future(r.call(meta, args, kwargs))
        except ReplicaDiedError:
            if attempt < 3:
                self.metrics.num_retries += 1
                return await self._assign(meta, args, kwargs, attempt + 1)
            raise
        finally:
            r.ongoing -= 1
            self._wake()

    async def _assign_stream(self, meta, args, kwargs, out_q: StreamSink):
        try:
            args, kwargs = await _resolve_args(args, kwargs)
            r = await self._acquire(meta)
        except Exception as e:
            out_q.put(("error", e))
            return
        r.ongoing += 1
        try:
            src = r.call_stream(meta, args, kwargs)
            while True:
                kind, val = await src.aget()
                out_q.put((kind, val))
                if kind != "item":
                    break
        finally:
            r.ongoing -= 1
            self._wake()

    def _check_backpressure(self) -> None:
        if self.max_queued != -1 and self._pending_count >= self.max_queued:
            # only when no replica has capacity right now
            if not any(not r.dead and r.ongoing < r.max_ongoing for r in self.replicas):
                self.metrics.num_rejected_backpressure += 1
                raise BackPressureError(self._pending_count, self.max_queued)

    def assign(self, meta: RequestMeta, args, kwargs):
        self.metrics.num_router_requests += 1
        if meta.stream:
            q = StreamSink()
            try:
                self._check_backpressure()
            except BackPressureError as e:
                q.put(("error", e))
                return DeploymentResponseGenerator(q, meta)
            asyncio.run_coroutine_threadsafe(self._assign_stream(meta, args, kwargs, q), self._lt.loop)
            return DeploymentResponseGenerator(q, meta)
        fut: concurrent.futures.Future
        try:
            self._check_backpressure()
        except BackPressureError as e:
            fut = concurrent.futures.Future()
            fut.set_exception(e)
            return DeploymentResponse(fut, meta)
        fut = asyncio.run_coroutine_threadsafe(self._assign(meta, args, kwargs), self._lt.loop)
        return DeploymentResponse(fut, meta, cancel_cb=lambda: self._lt.loop.call_soon_threadsafe(fut.cancel))


# ---------------------------------------------------------------------------
# Process mode: routing through the shared-memory job segment.
# ---------------------------------------------------------------------------
KIND_TENSOR = 0
KIND_PICKLE = 1
KIND_STREAM_ITEM = 2
KIND_STREAM_END = 3


class ShmRouter:
    """Routes to replica processes of one deployment (model id) through the
    job segment.  One instance per (process, job, deployment); a single
    dispatcher thread drains this process's completion ring for all routers
    sharing the client."""

    _clients: Dict[str, "_ShmClientHub"] = {}
    _clients_lock = threading.Lock()

    def __init__(self, job_name: str, model_id: int, deployment: str, max_queued_requests: int = -1,
                 tensor_codec=None, retry_timeout_s: float = 60.0, max_retries: int = 3):
        self.job_name = job_name
        self.model_id = model_id
        self.deployment = deployment
        self.max_queued = max_queued_requests
        self.codec = tensor_codec
        # Requests whose replica died are re-dispatched at most `max_retries`
        # times AND only until `retry_timeout_s` after their submission, then
        # fail with ReplicaDiedError: a request that kills its replica is not
        # replayed into every restarted replica (the reference retries only
        # scheduling, python/ray/serve/_private/router.py:452-496; replaying an
        # accepted request assumes an idempotent forward, hence the cap).
        # DeploymentConfig.request_retry_timeout_s / max_request_retries set both.
        self.retry_timeout_s = retry_timeout_s
        self.max_retries = max_retries
        self.metrics = RouterMetrics()
        with ShmRouter._clients_lock:
            hub = ShmRouter._clients.get(job_name)
            if hub is None or hub.closed:
                hub = _ShmClientHub(job_name)
                ShmRouter._clients[job_name] = hub
        self.hub = hub

    def num_queued(self) -> int:
        return self.hub.pending_for(self.model_id)

    def set_max_queued_requests(self, v: int) -> None:
        self.max_queued = v

    def update_replicas(self, replicas) -> None:  # replica set lives in shm
        self.hub.kick()

    def assign(self, meta: RequestMeta, args, kwargs):
        self.metrics.num_router_requests += 1
        if self.max_queued != -1 and self.hub.pending_for(self.model_id) >= self.max_queued:
            self.metrics.num_rejected_backpressure += 1
            err = BackPressureError(self.hub.pending_for(self.model_id), self.max_queued)
            if meta.stream:
                q = StreamSink()
                q.put(("error", err))
                return DeploymentResponseGenerator(q, meta)
            f = concurrent.futures.Future()
            f.set_exception(err)
            return DeploymentResponse(f, meta)
        if _has_response_args(args, kwargs):
            return self._assign_composed(meta, args, kwargs)
        return self._assign_resolved(meta, args, kwargs)

    def _assign_composed(self, meta: RequestMeta, args, kwargs):
        """Composition without a thread per request: a done-callback on every
        upstream response counts them down; the last one to finish (on whatever
        thread completed it -- the dispatcher for process-mode upstreams)
        substitutes the values and submits this request into the SAME future /
        stream sink the caller already holds.  An upstream error fails the
        request; cancelling the composed response before submission means it is
        never sent, after submission the hub drops it if still queued.
        Reference: argument resolution in python/ray/serve/_private/utils.py:605-660."""
        ups = [a for a in args if isinstance(a, DeploymentResponse)] + \
              [v for v in kwargs.values() if isinstance(v, DeploymentResponse)]
        sink = ("stream", StreamSink()) if meta.stream else ("unary", concurrent.futures.Future())
        state = {"left": len(ups), "cancelled": False}
        lock = threading.Lock()

        def submit():
            try:
                a = tuple(x._fut.result() if isinstance(x, DeploymentResponse) else x for x in args)
                k = {kk: (v._fut.result() if isinstance(v, DeploymentResponse) else v) for kk, v in kwargs.items()}
            except concurrent.futures.CancelledError:
                _settle_sink(sink, "error", RayServeException("an upstream response of a composed request was cancelled"))
                return
            except BaseException as e:      # an upstream failed: so does this request
                _settle_sink(sink, "error", e)
                return
            if not state["cancelled"]:
                self._assign_resolved(meta, a, k, sink)

        def on_done(_f):
            with lock:
                state["left"] -= 1
                last = state["left"] == 0
            if last:
                submit()

        def cancel_cb():
            state["cancelled"] = True
            self.hub.cancel(sink)

        for u in ups:
            u._fut.add_done_callback(on_done)
        if meta.stream:
            return DeploymentResponseGenerator(sink[1], meta, cancel_cb=cancel_cb)
        return DeploymentResponse(sink[1], meta, cancel_cb=cancel_cb)

    def _assign_resolved(self, meta: RequestMeta, args, kwargs, sink=None):
        if self.codec is not None and not meta.stream and meta.method_name == "__call__" and len(args) == 1 \
                and not kwargs and self.codec.accepts(args[0]):
            payload, kind = self.codec.encode(args[0]), KIND_TENSOR
        elif self.codec is None and tensor_wire.encodable(args, kwargs):
            # one array / CPU tensor argument to a Python deployment (the @serve.batch
            # GPU idiom): header + raw bytes in the ring slot, never cloudpickled
            payload = tensor_wire.encode_call(meta.method_name, args[0], meta.multiplexed_model_id or "",
                                              meta.request_id or "", meta.stream)
            kind = tensor_wire.KIND_TENSOR_CALL
            self.metrics.num_raw_tensor_calls += 1
        else:
            import cloudpickle

            payload = cloudpickle.dumps((meta.method_name, args, kwargs, meta.multiplexed_model_id, meta.stream,
                                         meta.request_id))
            kind = KIND_PICKLE
        route = _Route(self.model_id, mux_hash(meta.multiplexed_model_id)) if meta.multiplexed_model_id \
            else self.model_id
        budget = (time.monotonic() + self.retry_timeout_s, self.max_retries)   # (deadline, retries left)
        if sink is None:
            sink = ("stream", StreamSink()) if meta.stream else ("unary", concurrent.futures.Future())
        self.hub.submit(route, payload, kind, sink, self.codec, budget)
        if meta.stream:
            return DeploymentResponseGenerator(sink[1], meta, cancel_cb=lambda: self.hub.cancel(sink))
        return DeploymentResponse(sink[1], meta, cancel_cb=lambda: self.hub.cancel(sink))


def mux_hash(model_id: str) -> int:
    """64-bit id of a multiplexed model id as replicas publish it in shm (0 = none)."""
    import hashlib

    if not model_id:
        return 0
    return int.from_bytes(hashlib.blake2b(model_id.encode(), digest_size=8).digest(), "little") or 1


class _Route(int):
    """A deployment's model id (an int: pending counts and retries key on it)
    carrying the request's multiplexed-model hash for the native router."""

    def __new__(cls, model_id: int, mux: int = 0):
        o = super().__new__(cls, model_id)
        o.mux = mux
        return o


class _ShmClientHub:
    """Per-process native Client + dispatcher thread for one job segment.

    Request state (pending FIFO, in-flight table) is guarded by ``lock``; the
    futures / stream sinks of callers are settled only AFTER the lock is
    released (``_settle`` defers, ``_flush`` runs), so a done-callback that
    submits a composed request -- possibly into another hub -- never runs
    under this hub's lock (no lock-order inversion between hubs)."""

    def __init__(self, job_name: str):
        from ..runtime import job as rjob
        from ..runtime.job import Status

        self.Status = Status
        self.job = rjob.Job(job_name, create=False)
        self.client = rjob.Client(self.job)
        self.lock = threading.Lock()
        self.inflight: Dict[int, Tuple] = {}
        self.retries = 0
        self.pending: Deque[Tuple] = collections.deque()
        self.closed = False
        self._pending_by_model: Dict[int, int] = collections.Counter()
        self._deferred: List[Callable[[], None]] = []
        self._deferred_lock = threading.Lock()
        from ..utils.faults import injector

        self.faults = injector()
        self.thread = threading.Thread(target=self._run, name=f"rdb-dispatch-{job_name}", daemon=True)
        self.thread.start()

    # -- settlement outside the lock ------------------------------------------
    def _settle(self, fn: Callable[[], None]) -> None:
        with self._deferred_lock:
            self._deferred.append(fn)

    def _flush(self) -> None:
        while True:
            with self._deferred_lock:
                todo, self._deferred = self._deferred, []
            if not todo:
                return
            for fn in todo:
                try:
                    fn()
                except Exception:  # pragma: no cover - a user callback raised
                    logger.exception("completion callback failed")

    def _fail(self, sink, exc) -> None:
        self._settle(lambda: _settle_sink(sink, "error", exc))

    # -- public entry points ---------------------------------------------------
    def pending_for(self, model_id: int) -> int:
        return self._pending_by_model[model_id]

    def kick(self) -> None:
        with self.lock:
            self._drain_pending()
        self._flush()

    def submit(self, model_id, payload, kind, sink, codec, retry_deadline) -> None:
        with self.lock:
            item = (model_id, payload, kind, sink, codec, retry_deadline)
            if self.pending or not self._try_submit(*item):
                self.pending.append(item)
                self._pending_by_model[model_id] += 1
                self._drain_pending()
        self._flush()

    def cancel(self, sink) -> None:
        """Cancel a request: a queued one is never sent; an in-flight one's
        result is discarded (the replica still finishes the batch it is in)."""
        kind, obj = sink
        if kind == "unary":
            obj.cancel()
        else:
            obj.cancelled = True              # _sink_cancelled: still-queued items are dropped, not sent
            obj.put(("error", RequestCancelledError("stream cancelled")))
        with self.lock:
            for rid in [r for r, e in self.inflight.items() if e[3] is sink]:
                del self.inflight[rid]
            if self.pending:                  # drop it from the FIFO now (and its pending count)
                keep = collections.deque()
                for item in self.pending:
                    if item[3] is sink:
                        self._pending_by_model[item[0]] -= 1
                    else:
                        keep.append(item)
                self.pending = keep

    # -- internals (lock held) -------------------------------------------------
    @staticmethod
    def _sink_cancelled(sink) -> bool:
        return sink[1].cancelled() if sink[0] == "unary" else bool(getattr(sink[1], "cancelled", False))

    def _retry(self, entry, why: str) -> None:
        """Re-dispatch a request whose replica died, at the front of the FIFO,
        while it has retries left and its retry deadline has not passed; fail it
        with ReplicaDiedError after that."""
        model_id, payload, kind, sink, codec, budget = entry[:6]
        if self._sink_cancelled(sink):
            return
        deadline, left = budget
        if left > 0 and time.monotonic() < deadline:
            self.retries += 1
            self.pending.appendleft((model_id, payload, kind, sink, codec, (deadline, left - 1)))
            self._pending_by_model[model_id] += 1
        else:
            what = "retry window exhausted" if left > 0 else "retried too often"
            self._fail(sink, ReplicaDiedError(f"{why}; {what}"))

    def _try_submit(self, model_id, payload, kind, sink, codec, retry_deadline) -> bool:
        if self._sink_cancelled(sink):
            return True                    # cancelled while queued: drop it
        q = self.client.choose_queue(int(model_id), getattr(model_id, "mux", 0))
        if q == -2:
            self._fail(sink, DeploymentUnavailableError(f"no replica serves model id {int(model_id)}"))
            return True
        if q < 0:
            return False
        if self.faults.reject_submit():   # injected rejection: exercises the pending/retry path
            return False
        rid = self.client.submit(q, payload, kind)
        if rid == -3:
            self._fail(sink, RayServeException("request payload larger than the ring slot "
                                               "(raise engine.request_slot_bytes)"))
            return True
        if rid < 0:
            return False
        rep = self.job.queue_replica(q)
        self.inflight[rid] = (model_id, payload, kind, sink, codec, retry_deadline, q, rep,
                              self.job.replica_generation(rep))
        return True

    def _drain_pending(self) -> None:
        while self.pending:
            item = self.pending[0]
            if not self._try_submit(*item):
                break
            self.pending.popleft()
            self._pending_by_model[item[0]] -= 1

    def _complete(self, entry, st, kind, payload) -> None:
        import cloudpickle

        St = self.Status
        sink, codec = entry[3], entry[4]
        try:
            if st == St.OK:
                if sink[0] == "stream":
                    self._settle(lambda: _settle_sink(sink, "end", None))
                else:
                    if kind == KIND_TENSOR:
                        val = codec.decode(payload)
                    elif kind == tensor_wire.KIND_TENSOR_RESULT:
                        val = tensor_wire.decode_result(payload)
                    else:
                        val = cloudpickle.loads(payload) if payload else None
                    self._settle(lambda: _settle_sink(sink, "ok", val))
            elif st == St.ERROR:
                self._fail(sink, cloudpickle.loads(payload) if payload else RayServeException("replica error"))
            elif st == St.DROPPED_STALE:
                from .exceptions import RequestDroppedError

                self._fail(sink, RequestDroppedError("request dropped: its SLO deadline could not be met"))
            elif st in (St.REPLICA_DIED, St.SHUTDOWN):
                self._retry(entry, f"replica failed the request (status {int(st)})")
            elif st == St.TOO_LARGE:
                self._fail(sink, RayServeException("result larger than the completion slot"))
            else:
                self._fail(sink, ReplicaDiedError(f"request failed with status {int(st)}"))
        except Exception as e:  # pragma: no cover - decode failure
            self._fail(sink, e)

    def _run(self) -> None:
        import cloudpickle

        St = self.Status
        last_check = time.time()
        while not self.closed:
            try:
                comps = self.client.poll(1024, 0.05)
            except Exception:  # pragma: no cover - job torn down
                break
            if time.time() - last_check > 0.1:
                last_check = time.time()
                with self.lock:
                    self._reap_lost()
                self._flush()
            if not comps:
                if self.pending:
                    self.kick()
                continue
            with self.lock:
                for rid, st, q, ts, td, tr, kind, payload in comps:
                    entry = self.inflight.get(rid)
                    if entry is None:
                        continue              # cancelled, or already retried
                    if kind == KIND_STREAM_ITEM and st == St.OK:
                        item = cloudpickle.loads(payload)
                        entry[3][1].put(("item", item))   # stream sinks are thread-safe
                        continue
                    del self.inflight[rid]
                    self._complete(entry, st, kind, payload)
                self._drain_pending()
            self._flush()

    def _reap_lost(self) -> None:
        """Requests a replica popped but never answered because it died (its
        generation changed or it is DEAD) are re-dispatched (idempotent forward)
        within their retry window."""
        lost = []
        for rid, e in self.inflight.items():
            rep, gen = e[7], e[8]
            if self.job.replica_generation(rep) != gen or self.job.replica_status(rep) == 4:
                lost.append(rid)
        for rid in lost:
            self._retry(self.inflight.pop(rid), "replica died while processing the request")
        if lost:
            self._drain_pending()

    def close(self) -> None:
        self.closed = True
        if self.thread.is_alive() and self.thread is not threading.current_thread():
            self.thread.join(2.0)


def _settle_sink(sink, what: str, val) -> None:
    kind, obj = sink
    if kind == "unary":
        if obj.done():
            return
        if what == "ok":
            obj.set_result(val)
        else:
            obj.set_exception(val)
    else:
        obj.put(("error", val) if what == "error" else ("end", None))


def _close_all_hubs() -> None:
    for hub in list(ShmRouter._clients.values()):
        hub.close()


import atexit as _atexit  # noqa: E402

_atexit.register(_close_all_hubs)
