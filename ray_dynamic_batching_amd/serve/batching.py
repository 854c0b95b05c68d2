"""``@serve.batch``: dynamic request batching inside a replica.

Semantics kept compatible with Ray Serve (reference:
python/ray/serve/batching.py:529-678, _BatchQueue 80-333):

* the decorated function is ``async`` and takes ``List[T]`` (one entry per
  caller, for every positional / keyword argument) and returns ``List[R]`` of
  the same length -- or is an async generator yielding such lists;
* callers pass a single item and await their own result;
* a batch is flushed when it holds ``max_batch_size`` items or
  ``batch_wait_timeout_s`` after its FIRST item arrived, whichever is first;
* an exception raised by the batch function is delivered to every caller of
  that batch; a result of the wrong length raises ``RayServeException``;
* ``set_max_batch_size`` / ``set_batch_wait_timeout_s`` change the knobs at run
  time; ``_get_max_batch_size`` / ``_get_batch_wait_timeout_s`` read them.

This is the *generic* Python batching path used for arbitrary user code.  GPU
models registered as servable models bypass it: the replica engine
(ops/csrc/engine.cpp) batches natively with the same flush rule.
"""
from __future__ import annotations

import asyncio
import functools
import inspect
import logging
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from .exceptions import RayServeException

logger = logging.getLogger("ray_dynamic_batching_amd.serve")


@dataclass
class _SingleRequest:
    self_arg: Any
    args: Tuple
    kwargs: Dict[str, Any]
    future: asyncio.Future
    enqueue_time: float = 0.0


def _validate_max_batch_size(v) -> None:
    if not isinstance(v, int) or isinstance(v, bool):
        raise TypeError(f"max_batch_size must be an integer >= 1, got {v!r}")
    if v < 1:
        raise ValueError(f"max_batch_size must be an integer >= 1, got {v}")


def _validate_timeout(v) -> None:
    if not isinstance(v, (int, float)) or isinstance(v, bool):
        raise TypeError(f"batch_wait_timeout_s must be a non-negative number, got {v!r}")
    if v < 0:
        raise ValueError(f"batch_wait_timeout_s must be a non-negative number, got {v}")


def _transpose_args(batch: List[_SingleRequest]) -> Tuple[List[List[Any]], Dict[str, List[Any]]]:
    """Turn N calls f(a_i, b_i, k=c_i) into f([a..], [b..], k=[c..]).
    Every call must use the same arity and keyword names."""
    n_args = len(batch[0].args)
    keys = tuple(sorted(batch[0].kwargs))
    for r in batch:
        if len(r.args) != n_args or tuple(sorted(r.kwargs)) != keys:
            raise ValueError("all calls in a batch must pass the same number of positional arguments "
                             "and the same keyword arguments")
    args = [[r.args[i] for r in batch] for i in range(n_args)]
    kwargs = {k: [r.kwargs[k] for r in batch] for k in keys}
    return args, kwargs


class _BatchQueue:
    """Per-(replica, method) queue + the background task that forms batches."""

    def __init__(self, max_batch_size: int, batch_wait_timeout_s: float, handle_fn: Callable,
                 is_generator: bool, batch_started_hook: Optional[Callable] = None):
        self.queue: asyncio.Queue = asyncio.Queue()
        self.max_batch_size = max_batch_size
        self.batch_wait_timeout_s = batch_wait_timeout_s
        self._handle_fn = handle_fn
        self._is_generator = is_generator
        self._arrival = asyncio.Event()
        self._hook = batch_started_hook
        self.batches_processed = 0
        self.last_batch_sizes: List[int] = []
        self.loop = asyncio.get_running_loop()
        # The batching task runs only while requests are queued: it is started
        # by put() and returns once the queue is drained, so an idle queue (or
        # one whose event loop is closed without cancelling its tasks) leaves no
        # pending task behind -- the reference cancels its long-lived task from
        # __del__ (python/ray/serve/batching.py:323-333), which a closed loop
        # can no longer run.
        self._task: Optional[asyncio.Task] = None
        self._crashed: Optional[BaseException] = None   # what ended the batching loop abnormally
        self._shut = False
        self.current_iteration_start: Optional[float] = None

    def put(self, req: _SingleRequest) -> None:
        self.queue.put_nowait(req)
        self._arrival.set()
        if self._task is None or self._task.done():
            self._task = self.loop.create_task(self._loop())

    def is_alive(self) -> bool:
        """Whether the batching loop can still serve: True while a batch task runs
        AND while the queue is idle (the task is started again by the next put),
        False only once the loop died of an exception or the queue was shut
        down -- the reference's long-lived task reports exactly that
        (python/ray/serve/batching.py:400-410), so a health check can tell a
        crashed loop from an idle one."""
        return self._crashed is None and not self._shut and not self.loop.is_closed()

    def task_stack(self) -> Optional[str]:
        """Formatted stack of the running batch task (reference
        ``_get_handling_task_stack``), or None when idle."""
        if self._task is None or self._task.done():
            return None
        import io

        buf = io.StringIO()
        self._task.print_stack(file=buf)
        return buf.getvalue()

    async def wait_for_batch(self) -> List[_SingleRequest]:
        """Block for the first item, then keep adding until full or until
        batch_wait_timeout_s has elapsed since that first item."""
        batch = [await self.queue.get()]
        # the event loop's clock (monotonic; a test loop may virtualise it)
        clock = asyncio.get_running_loop().time
        max_bs = self.max_batch_size
        timeout = self.batch_wait_timeout_s
        deadline = clock() + timeout
        while len(batch) < max_bs:
            while len(batch) < max_bs and not self.queue.empty():
                batch.append(self.queue.get_nowait())
            if len(batch) >= max_bs:
                break
            remaining = deadline - clock()
            if remaining <= 0:
                break
            self._arrival.clear()
            try:
                await asyncio.wait_for(self._arrival.wait(), remaining)
            except asyncio.TimeoutError:
                pass
        return batch

    async def _loop(self) -> None:
        try:
            await self._loop_body()
        except asyncio.CancelledError:
            raise
        except BaseException as e:   # the loop itself died: report it, fail the queued callers
            self._crashed = e
            logger.exception("batching loop crashed: %s", e)
            while not self.queue.empty():
                r = self.queue.get_nowait()
                if not r.future.done():
                    r.future.set_exception(e)
            raise

    async def _loop_body(self) -> None:
        while not self.queue.empty():
            batch = await self.wait_for_batch()
            # drop requests whose caller already gave up (cancelled)
            batch = [r for r in batch if not r.future.done()]
            if not batch:
                continue
            self.current_iteration_start = asyncio.get_running_loop().time()
            self.batches_processed += 1
            self.last_batch_sizes = (self.last_batch_sizes + [len(batch)])[-1000:]
            if self._hook:
                try:
                    self._hook(len(batch))
                except Exception:  # pragma: no cover
                    pass
            try:
                if self._is_generator:
                    await self._run_generator(batch)
                else:
                    await self._run_once(batch)
            except Exception as e:  # pragma: no cover - defensive
                logger.exception("batch loop error: %s", e)
            finally:
                self.current_iteration_start = None

    async def _run_once(self, batch: List[_SingleRequest]) -> None:
        try:
            args, kwargs = _transpose_args(batch)
            if batch[0].self_arg is not None:
                results = await self._handle_fn(batch[0].self_arg, *args, **kwargs)
            else:
                results = await self._handle_fn(*args, **kwargs)
            if not isinstance(results, (list, tuple)) or len(results) != len(batch):
                raise RayServeException(
                    f"batched function must return a list of length {len(batch)} (one result per "
                    f"request), got {type(results).__name__}"
                    + (f" of length {len(results)}" if hasattr(results, "__len__") else ""))
            for r, out in zip(batch, results):
                if not r.future.done():
                    r.future.set_result(out)
        except Exception as e:
            for r in batch:
                if not r.future.done():
                    r.future.set_exception(e)

    async def _run_generator(self, batch: List[_SingleRequest]) -> None:
        # each caller's future resolves to an asyncio.Queue of its items
        queues = [asyncio.Queue() for _ in batch]
        for r, q in zip(batch, queues):
            if not r.future.done():
                r.future.set_result(q)
        try:
            args, kwargs = _transpose_args(batch)
            gen = (self._handle_fn(batch[0].self_arg, *args, **kwargs) if batch[0].self_arg is not None
                   else self._handle_fn(*args, **kwargs))
            async for results in gen:
                if not isinstance(results, (list, tuple)) or len(results) != len(batch):
                    raise RayServeException(f"batched generator must yield lists of length {len(batch)}")
                for q, item in zip(queues, results):
                    if item is not StopIteration:  # StopIteration marks an early-finished caller
                        q.put_nowait(("item", item))
                    else:
                        q.put_nowait(("end", None))
            for q in queues:
                q.put_nowait(("end", None))
        except Exception as e:
            for q in queues:
                q.put_nowait(("error", e))

    def shutdown(self) -> None:
        self._shut = True
        if self._task is not None and not self._task.done() and not self.loop.is_closed():
            self._task.cancel()


class _LazyBatchQueue:
    """The asyncio queue must be created on the replica's event loop, lazily
    (a decorated method's object may be pickled to a replica process first)."""

    def __init__(self, max_batch_size: int, batch_wait_timeout_s: float, fn: Callable, is_generator: bool):
        self.max_batch_size = max_batch_size
        self.batch_wait_timeout_s = batch_wait_timeout_s
        self._fn = fn
        self._gen = is_generator
        self._queues: Dict[int, _BatchQueue] = {}  # per event loop

    def queue(self, owner=None) -> _BatchQueue:
        """One queue per (event loop, bound instance): replicas never share a batch."""
        key = (id(asyncio.get_running_loop()), id(owner))
        q = self._queues.get(key)
        if q is not None and q.loop is not asyncio.get_running_loop():
            q = None   # a closed loop's id was reused
        if q is None:
            self._prune()
            q = _BatchQueue(self.max_batch_size, self.batch_wait_timeout_s, self._fn, self._gen)
            self._warn_if_ongoing_too_small()
            self._queues[key] = q
        return q

    def _prune(self) -> None:
        """Forget the queues of closed event loops (their pending items can never run)."""
        for k in [k for k, q in self._queues.items() if q.loop.is_closed()]:
            q = self._queues.pop(k)
            while not q.queue.empty():
                r = q.queue.get_nowait()
                r.future.cancel() if not r.future.done() and not q.loop.is_closed() else None

    def set_max_batch_size(self, v: int) -> None:
        _validate_max_batch_size(v)
        self.max_batch_size = v
        for q in self._queues.values():
            q.max_batch_size = v

    def set_batch_wait_timeout_s(self, v: float) -> None:
        _validate_timeout(v)
        self.batch_wait_timeout_s = v
        for q in self._queues.values():
            q.batch_wait_timeout_s = v

    def _warn_if_ongoing_too_small(self) -> None:
        # reference batching.py:121-135: a replica never sees a full batch if
        # max_ongoing_requests < max_batch_size
        from .context import get_replica_context_or_none

        ctx = get_replica_context_or_none()
        if ctx is not None and ctx.max_ongoing_requests is not None and ctx.max_ongoing_requests < self.max_batch_size:
            logger.warning("max_batch_size (%d) > max_ongoing_requests (%d): batches will never be full",
                           self.max_batch_size, ctx.max_ongoing_requests)

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_queues"] = {}
        return d

    # debugging hooks (reference _LazyBatchQueueWrapper)
    def _get_curr_iteration_start_times(self):
        return [q.current_iteration_start for q in self._queues.values()]

    def _is_batching_task_alive(self) -> bool:
        """False only if a queue's batching loop crashed or was shut down; a
        queue not created yet (no request so far) counts as alive, as the
        reference creates its queue on first access."""
        return all(q.is_alive() for q in self._queues.values() if not q.loop.is_closed())

    def _get_handling_task_stack(self) -> Optional[str]:
        for q in self._queues.values():
            st = q.task_stack()
            if st:
                return st
        return None


def batch(_func: Optional[Callable] = None, /, max_batch_size: int = 10, batch_wait_timeout_s: float = 0.0):
    """Decorator (usable bare or with arguments) turning an async
    ``List[T] -> List[R]`` function/method into a per-call ``T -> R`` one."""
    if _func is not None:
        if not callable(_func):
            raise TypeError("@serve.batch can only decorate functions or methods; "
                            "pass max_batch_size / batch_wait_timeout_s as keyword arguments")
        if not (inspect.iscoroutinefunction(_func) or inspect.isasyncgenfunction(_func)):
            raise TypeError("functions decorated with @serve.batch must be 'async def'")
    _validate_max_batch_size(max_batch_size)
    _validate_timeout(batch_wait_timeout_s)

    def deco(fn: Callable) -> Callable:
        if not (inspect.iscoroutinefunction(fn) or inspect.isasyncgenfunction(fn)):
            raise TypeError("functions decorated with @serve.batch must be 'async def'")
        is_gen = inspect.isasyncgenfunction(fn)
        lazy = _LazyBatchQueue(max_batch_size, batch_wait_timeout_s, fn, is_gen)
        params = list(inspect.signature(fn).parameters)
        is_method = bool(params) and params[0] == "self"

        def _enqueue(args, kwargs) -> asyncio.Future:
            self_arg = None
            if is_method:
                self_arg, args = args[0], args[1:]
            fut = asyncio.get_running_loop().create_future()
            lazy.queue(self_arg).put(_SingleRequest(self_arg, tuple(args), dict(kwargs), fut,
                                                    asyncio.get_running_loop().time()))
            return fut

        if is_gen:
            @functools.wraps(fn)
            async def gen_wrapper(*args, **kwargs):
                q = await _enqueue(args, kwargs)
                while True:
                    kind, val = await q.get()
                    if kind == "item":
                        yield val
                    elif kind == "error":
                        raise val
                    else:
                        return

            wrapper = gen_wrapper
        else:
            @functools.wraps(fn)
            async def wrapper(*args, **kwargs):
                return await _enqueue(args, kwargs)

        wrapper.set_max_batch_size = lazy.set_max_batch_size
        wrapper.set_batch_wait_timeout_s = lazy.set_batch_wait_timeout_s
        wrapper._get_max_batch_size = lambda: lazy.max_batch_size
        wrapper._get_batch_wait_timeout_s = lambda: lazy.batch_wait_timeout_s
        wrapper._get_curr_iteration_start_times = lazy._get_curr_iteration_start_times
        wrapper._is_batching_task_alive = lazy._is_batching_task_alive
        wrapper._get_handling_task_stack = lazy._get_handling_task_stack
        wrapper._rdb_batch_queue = lazy
        return wrapper

    return deco(_func) if _func is not None else deco


class _PinnedStager:
    """Per-thread pinned host staging buffer + side stream for ``stack_to_device``."""

    def __init__(self):
        self.buf = None
        self.stream = None
        self.event = None


_stagers = threading.local()


def stack_to_device(items, device="cuda", dtype=None):
    """Assemble a ``@serve.batch`` batch of same-shape arrays / CPU tensors in a
    pinned host staging buffer and copy it to ``device`` with
    ``non_blocking=True`` on a side stream; the caller's current stream waits on
    that copy (an event), so the returned device tensor is ready for the next
    kernel without a host sync.  The staging buffer is reused across batches
    (grown when needed); the copy of batch k is retired before batch k+1 rewrites
    it.  On a CPU ``device`` it is a plain ``torch.stack``.

    The reference idiom (release/serve_tests/workloads/resnet_50.py:50-57) does
    ``torch.stack(images).cuda()``: a pageable, synchronous H2D per batch."""
    import numpy as np
    import torch

    xs = [torch.from_numpy(np.asarray(x)) if not isinstance(x, torch.Tensor) else x for x in items]
    if not xs:
        raise ValueError("stack_to_device: empty batch")
    dev = torch.device(device)
    if dev.type != "cuda":
        out = torch.stack(xs)
        return out.to(dtype) if dtype is not None else out
    st = getattr(_stagers, "s", None)
    if st is None:
        st = _stagers.s = _PinnedStager()
        st.stream = torch.cuda.Stream(device=dev)
        st.event = torch.cuda.Event()
    shape = (len(xs),) + tuple(xs[0].shape)
    n = int(np.prod(shape))
    src_dtype = xs[0].dtype
    if st.buf is None or st.buf.numel() < n or st.buf.dtype != src_dtype:
        st.event.synchronize()
        st.buf = torch.empty(max(n, 1), dtype=src_dtype, pin_memory=True)
    st.event.synchronize()                         # the previous batch's copy has left the buffer
    host = st.buf[:n].view(shape)
    torch.stack(xs, out=host)
    cur = torch.cuda.current_stream(dev)
    st.stream.wait_stream(cur)                     # the destination's allocator order
    with torch.cuda.stream(st.stream):
        out = host.to(dev, non_blocking=True)
        st.event.record(st.stream)
    cur.wait_event(st.event)
    out.record_stream(cur)
    return out.to(dtype) if dtype is not None else out
