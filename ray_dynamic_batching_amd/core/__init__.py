"""Ray-core-compatible task / actor / object API for one MI355X node.

The fork drives its Nexus scheduler through Ray core directly
(reference: ``293-project/src/scheduler.py:374`` ``@ray.remote(num_gpus=1) class
GPUWorker``, ``:393`` ``ray.get_gpu_ids()``, ``test_scheduler.py:124``
``ray.init(...)``, ``venkat-code/schedule_executor.py:363-383`` ``ray.put`` /
``ray.get``, ``slo_viewer.py:184-197`` ``ray.state.actors()`` /
``ray.get_actor``) and ``ray.util.queue.Queue``.  This module is that surface
(SURVEY.md §2.3), so such code runs with ``import ray_dynamic_batching_amd.core
as ray``:

* ``init`` / ``is_initialized`` / ``shutdown`` / ``remote`` (functions and
  classes, ``.options(...)``) / ``get`` / ``put`` / ``wait`` / ``kill`` /
  ``get_actor`` / ``get_gpu_ids`` / ``cluster_resources`` /
  ``available_resources``; ``state.actors()``; ``util.queue.Queue``; ``data``
  (offline batch inference: ``map_batches`` on GPU actor pools).
* An actor is ONE process (spawned, not forked: a GPU runtime must never be
  forked) pinned to the GPUs the node's slot allocator gave it
  (``runtime/resources.py``: whole GPUs first-fit, fractional best-fit, the
  rule of Ray's ``resource_instance_set.cc:93-187``) through
  ``HIP_VISIBLE_DEVICES``.  Method calls travel over a Unix socket with
  cloudpickle; each caller's calls run in submission order
  (``max_concurrency`` > 1: threaded actor).  ``init(local_mode=True)`` hosts
  actors in-process on threads instead (CPU tests, debugging).
* Named actors live in a per-namespace registry directory, so another driver
  (``init(address="auto", namespace=...)``) finds them with ``get_actor``.
* Tasks (remote functions) run on a driver thread pool; a task that asks for
  GPUs runs in a one-shot pinned process.

This is the control-plane API of the fork.  The request path of the
framework does NOT go through it: serving uses the shm rings and the native
replica engine (``serve`` / ``runtime``).
"""
from __future__ import annotations

import atexit
import json
import multiprocessing as mp
import os
import secrets
import shutil
import tempfile
import threading
import time
import uuid
from concurrent.futures import Future, ThreadPoolExecutor
from concurrent.futures import TimeoutError as _FutTimeout
from multiprocessing.connection import Client as _ConnClient
from typing import Any, Dict, List, Optional, Sequence, Tuple

__all__ = ["init", "is_initialized", "shutdown", "remote", "get", "put", "wait", "kill", "get_actor",
           "get_gpu_ids", "cluster_resources", "available_resources", "timeline", "ObjectRef", "ActorHandle",
           "nodes", "get_runtime_context", "RayError", "RayTaskError", "RayActorError", "GetTimeoutError",
           "TaskUnschedulableError", "state", "util", "data", "dag"]


class RayError(Exception):
    pass


class RayTaskError(RayError):
    """A task or actor method raised; ``cause`` is the original exception."""

    def __init__(self, cause: BaseException, remote_tb: str = ""):
        super().__init__(f"{type(cause).__name__}: {cause}\n{remote_tb}".rstrip())
        self.cause = cause
        self.remote_traceback = remote_tb


class RayActorError(RayError):
    pass


class GetTimeoutError(RayError, TimeoutError):
    pass


class TaskUnschedulableError(RayError):
    """A hard scheduling constraint no node satisfies (e.g. node affinity to an unknown node)."""


# ---------------------------------------------------------------------------
# process-wide state
# ---------------------------------------------------------------------------
_ctx: Optional["_Context"] = None
_ctx_lock = threading.Lock()
_WORKER: Dict[str, str] = {}          # set in actor processes (GPU ids, namespace)
_tls = threading.local()              # local mode: the env of the actor running on this thread


def _set_worker_context(env: Dict[str, str]) -> None:
    _WORKER.update(env)


def _registry_root(namespace: str) -> str:
    return os.path.join(tempfile.gettempdir(), f"rdb_core_{os.getuid()}", namespace or "default")


class _Context:
    def __init__(self, num_gpus: Optional[int], num_cpus: Optional[int], local_mode: bool, namespace: str,
                 connect_only: bool):
        from ..runtime.resources import GpuAllocator, detect_num_gpus

        self.local_mode = local_mode
        self.namespace = namespace or "default"
        self.num_gpus = detect_num_gpus() if num_gpus is None else int(num_gpus)
        self.num_cpus = (os.cpu_count() or 1) if num_cpus is None else int(num_cpus)
        self.allocator = GpuAllocator(self.num_gpus)
        self.registry = _registry_root(self.namespace)
        os.makedirs(os.path.join(self.registry, "_actors"), exist_ok=True)
        self.sock_dir = tempfile.mkdtemp(prefix="rdb_core_sock_")
        self.owned: List["ActorHandle"] = []
        self.procs: Dict[str, Any] = {}
        self.tasks = ThreadPoolExecutor(max(4, min(64, self.num_cpus)), thread_name_prefix="rdb-task")
        self.connect_only = connect_only
        self.lock = threading.Lock()


def _require_ctx() -> "_Context":
    if _ctx is None:
        init()
    return _ctx


def init(address: Optional[str] = None, *, num_cpus: Optional[int] = None, num_gpus: Optional[int] = None,
         local_mode: bool = False, namespace: Optional[str] = None, ignore_reinit_error: bool = False,
         **_unused) -> dict:
    """Start (or, with ``address="auto"``, attach to the named-actor registry of)
    this node's runtime.  ``num_gpus`` overrides detection (logical GPUs, as in
    Ray's ``cluster_utils`` fake GPUs)."""
    global _ctx
    with _ctx_lock:
        if _ctx is not None:
            if ignore_reinit_error:
                return {"namespace": _ctx.namespace}
            raise RuntimeError("init() called twice; pass ignore_reinit_error=True")
        _ctx = _Context(num_gpus, num_cpus, local_mode, namespace or "default", connect_only=address == "auto")
    atexit.register(shutdown)
    return {"namespace": _ctx.namespace, "num_gpus": _ctx.num_gpus}


def is_initialized() -> bool:
    return _ctx is not None


def shutdown() -> None:
    """Kill every non-detached actor this driver created; drop its registry entries."""
    global _ctx
    with _ctx_lock:
        ctx, _ctx = _ctx, None
    if ctx is None:
        return
    for h in list(ctx.owned):
        if not h._detached:
            try:
                kill(h, _ctx_override=ctx)
            except Exception:
                pass
    from .util import _pg_mod as _pgm

    with _pgm._lock:        # reservations die with this driver's allocator
        for g in _pgm._groups.values():
            g.state = "REMOVED"
        _pgm._groups.clear()
    ctx.tasks.shutdown(wait=False, cancel_futures=True)
    shutil.rmtree(ctx.sock_dir, ignore_errors=True)


def cluster_resources() -> Dict[str, float]:
    ctx = _require_ctx()
    return {"CPU": float(ctx.num_cpus), "GPU": float(ctx.num_gpus)}


def available_resources() -> Dict[str, float]:
    ctx = _require_ctx()
    free = sum(s["free"] for s in ctx.allocator.snapshot())
    return {"CPU": float(ctx.num_cpus), "GPU": float(free)}


def _node_id() -> str:
    """This host's node id (56 hex chars, like Ray's NodeID): derived from the
    hostname and the kernel boot id, so every process on the node agrees."""
    import hashlib
    import socket

    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    return hashlib.sha256(f"{socket.gethostname()}/{boot}".encode()).hexdigest()[:56]


def nodes() -> List[Dict[str, Any]]:
    """``ray.nodes()``: this single node (multi-node is out of scope)."""
    import socket

    return [{"NodeID": _node_id(), "Alive": True, "NodeManagerAddress": "127.0.0.1",
             "NodeManagerHostname": socket.gethostname(), "Resources": cluster_resources()}]


class RuntimeContext:
    """``ray.get_runtime_context()`` subset: node / job ids, namespace and the
    accelerators this worker was pinned to."""

    def get_node_id(self) -> str:
        return _node_id()

    def get_job_id(self) -> str:
        env = getattr(_tls, "env", None) or _WORKER
        return env.get("RDB_CORE_JOB_ID", os.environ.get("RDB_CORE_JOB_ID", f"{os.getpid():08x}"))

    @property
    def namespace(self) -> str:
        env = getattr(_tls, "env", None) or _WORKER
        return env.get("RDB_CORE_NAMESPACE", _ctx.namespace if _ctx is not None else "default")

    def get_accelerator_ids(self) -> Dict[str, List[str]]:
        return {"GPU": [str(g) for g in get_gpu_ids()]}


def get_runtime_context() -> RuntimeContext:
    return RuntimeContext()


def get_gpu_ids() -> List[int]:
    """The (physical) GPU indices this actor / task was pinned to; [] in a driver."""
    env = getattr(_tls, "env", None) or _WORKER
    ids = env.get("RDB_CORE_GPU_IDS", os.environ.get("RDB_CORE_GPU_IDS", ""))
    return [int(x) for x in ids.split(",") if x != ""]


# ---------------------------------------------------------------------------
# objects
# ---------------------------------------------------------------------------
class ObjectRef:
    """A future value.  Pickling a ref (passing it inside a container to an
    actor) ships its value, waiting for it if needed."""

    __slots__ = ("_fut", "_id")

    def __init__(self, fut: Future):
        self._fut = fut
        self._id = uuid.uuid4().hex[:16]

    def future(self) -> Future:
        return self._fut

    def hex(self) -> str:
        return self._id

    def __await__(self):
        import asyncio

        return asyncio.wrap_future(self._fut).__await__()

    def __reduce__(self):
        return (_resolved_ref, (_result(self, None),))

    def __repr__(self) -> str:
        return f"ObjectRef({self._id})"


def _resolved_ref(value) -> ObjectRef:
    f: Future = Future()
    f.set_result(value)
    return ObjectRef(f)


def _failed_ref(exc: BaseException) -> ObjectRef:
    f: Future = Future()
    f.set_exception(exc)
    return ObjectRef(f)


def _result(ref: ObjectRef, timeout: Optional[float]):
    try:
        return ref._fut.result(timeout)
    except _FutTimeout:
        raise GetTimeoutError(f"get timed out after {timeout} s") from None


def put(value: Any) -> ObjectRef:
    if isinstance(value, ObjectRef):
        raise TypeError("put() of an ObjectRef is not allowed")
    return _resolved_ref(value)


def get(refs, *, timeout: Optional[float] = None):
    """Value(s) of one ref or a list of refs; a remote exception is re-raised as
    RayTaskError (its ``cause`` is the original)."""
    deadline = None if timeout is None else time.monotonic() + timeout
    if isinstance(refs, ObjectRef):
        return _result(refs, timeout)
    if not isinstance(refs, (list, tuple)):
        raise TypeError("get() takes an ObjectRef or a list of ObjectRefs")
    out = []
    for r in refs:
        left = None if deadline is None else max(0.0, deadline - time.monotonic())
        out.append(_result(r, left))
    return out


def wait(refs: Sequence[ObjectRef], *, num_returns: int = 1, timeout: Optional[float] = None,
         fetch_local: bool = True) -> Tuple[List[ObjectRef], List[ObjectRef]]:
    refs = list(refs)
    if num_returns > len(refs):
        raise ValueError("num_returns cannot exceed the number of refs")
    deadline = None if timeout is None else time.monotonic() + timeout
    while True:
        ready = [r for r in refs if r._fut.done()]
        if len(ready) >= num_returns or (deadline is not None and time.monotonic() >= deadline):
            ready = ready[:num_returns] if len(ready) > num_returns else ready
            rs = set(id(r) for r in ready)
            return ready, [r for r in refs if id(r) not in rs]
        time.sleep(0.001)


# ---------------------------------------------------------------------------
# timeline (reference: ``ray.timeline`` -> _private/state.py:948, profiling.py:84)
# ---------------------------------------------------------------------------
_timeline: List[dict] = []
_timeline_lock = threading.Lock()
_TIMELINE_CAP = 100000


def _traced(ref: ObjectRef, name: str, lane: str) -> ObjectRef:
    """Record submit -> completion of an actor call / task as one span."""
    t0 = time.time()

    def done(f: Future):
        ev = dict(name=name, cat="actor_call" if lane != "tasks" else "task", ph="X", ts=t0 * 1e6,
                  dur=(time.time() - t0) * 1e6, pid="rdb-core", tid=lane,
                  args={"ok": f.exception() is None})
        with _timeline_lock:
            if len(_timeline) < _TIMELINE_CAP:
                _timeline.append(ev)

    ref._fut.add_done_callback(done)
    return ref


def timeline(filename: Optional[str] = None) -> List[dict]:
    """Chrome-trace events (``chrome://tracing`` / Perfetto) of the actor calls
    and tasks this driver submitted, submit to completion, one row per actor;
    written to ``filename`` as JSON if given (like ``ray timeline``)."""
    with _timeline_lock:
        events = list(_timeline)
    if filename:
        with open(filename, "w") as f:
            json.dump(events, f)
    return events


def _resolve_args(args, kwargs):
    """Top-level ObjectRef arguments are passed by value (Ray semantics)."""
    args = tuple(get(a) if isinstance(a, ObjectRef) else a for a in args)
    kwargs = {k: get(v) if isinstance(v, ObjectRef) else v for k, v in kwargs.items()}
    return args, kwargs


def _pending_deps(args, kwargs) -> List[Future]:
    return [a._fut for a in list(args) + list(kwargs.values()) if isinstance(a, ObjectRef) and not a._fut.done()]


def _upstream_error(args, kwargs) -> Optional[BaseException]:
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, ObjectRef) and a._fut.done() and a._fut.exception() is not None:
            return a._fut.exception()
    return None


def _all_done(futs: List[Future], fn) -> None:
    if not futs:
        fn()
        return
    left = [len(futs)]
    lock = threading.Lock()

    def one(_f):
        with lock:
            left[0] -= 1
            last = left[0] == 0
        if last:
            fn()

    for f in futs:
        f.add_done_callback(one)


# per-actor tail of deferred submissions: a call made while an earlier call on
# the same actor still waits for its arguments is queued behind it, so actor
# calls keep their submission order (Ray's per-caller actor-task ordering)
_submit_tails: Dict[str, Future] = {}
_submit_tails_lock = threading.Lock()


def _deferred_submit(args, kwargs, submit_now, order_key: Optional[str] = None) -> Optional[ObjectRef]:
    """``.remote()`` never blocks on argument refs (reference: ``ray.remote``
    returns at once; dependencies resolve before the task runs): with every
    argument ref resolved (or none), returns None and the caller submits at
    once; otherwise the submission is chained on the pending refs and the
    returned ref resolves with the call's result -- or with the upstream
    exception, raised at ``get()`` like Ray's failed dependency."""
    tail_prev: Optional[Future] = None
    deps = _pending_deps(args, kwargs)
    if order_key is not None:
        with _submit_tails_lock:
            tail_prev = _submit_tails.get(order_key)
            if tail_prev is not None and tail_prev.done():
                tail_prev = None
                _submit_tails.pop(order_key, None)
            if not deps and tail_prev is None:
                return None
            tail: Future = Future()
            _submit_tails[order_key] = tail
    elif not deps:
        return None
    else:
        tail = Future()
    out: Future = Future()

    def go():
        try:
            err = _upstream_error(args, kwargs)
            if err is not None:
                out.set_exception(err)
                return
            a, kw = _resolve_args(args, kwargs)
            try:
                ref = submit_now(a, kw)
            except BaseException as e:  # noqa: BLE001
                out.set_exception(e)
                return
            ref._fut.add_done_callback(lambda r: out.set_exception(r.exception()) if r.exception() is not None
                                       else out.set_result(r.result()))
        finally:
            tail.set_result(None)

    _all_done(deps + ([tail_prev] if tail_prev is not None else []), go)
    return ObjectRef(out)


# ---------------------------------------------------------------------------
# actors
# ---------------------------------------------------------------------------
class _Channel:
    """One caller process's connection to one actor: sends calls, a reader
    thread resolves their futures."""

    def __init__(self, address: str, authkey: bytes):
        self.conn = _ConnClient(address, family="AF_UNIX", authkey=authkey)
        self.lock = threading.Lock()
        self.pending: Dict[int, Future] = {}
        self.next_id = 0
        self.dead: Optional[BaseException] = None
        threading.Thread(target=self._reader, daemon=True).start()

    def _reader(self):
        import cloudpickle

        while True:
            try:
                call_id, ok, val = cloudpickle.loads(self.conn.recv_bytes())
            except (EOFError, OSError) as e:
                self._fail(RayActorError(f"the actor process died or closed its connection ({type(e).__name__})"))
                return
            except Exception as e:  # noqa: BLE001 - undecodable reply
                self._fail(RayActorError(f"bad reply from actor: {e}"))
                return
            with self.lock:
                fut = self.pending.pop(call_id, None)
            if fut is None:
                continue
            if ok:
                fut.set_result(val)
            else:
                exc, tb = val
                fut.set_exception(RayTaskError(exc, tb))

    def _fail(self, exc: BaseException):
        with self.lock:
            self.dead = exc
            pend, self.pending = self.pending, {}
        for f in pend.values():
            if not f.done():
                f.set_exception(exc)

    def call(self, method: str, args, kwargs) -> Future:
        import cloudpickle

        fut: Future = Future()
        with self.lock:
            if self.dead is not None:
                fut.set_exception(self.dead)
                return fut
            cid = self.next_id
            self.next_id += 1
            self.pending[cid] = fut
            try:
                self.conn.send_bytes(cloudpickle.dumps((cid, method, args, kwargs)))
            except (OSError, EOFError) as e:
                self.pending.pop(cid, None)
                self.dead = RayActorError(f"cannot reach the actor: {e}")
                fut.set_exception(self.dead)
        return fut

    def close(self):
        try:
            self.conn.close()
        except OSError:
            pass


_channels: Dict[str, _Channel] = {}
_channels_lock = threading.Lock()
_local_actors: Dict[str, Tuple[Any, ThreadPoolExecutor, Dict[str, str]]] = {}


class ActorHandle:
    def __init__(self, actor_id: str, class_name: str, address: str = "", authkey: bytes = b"",
                 name: Optional[str] = None, detached: bool = False):
        self._actor_id = actor_id
        self._class_name = class_name
        self._address = address
        self._authkey = authkey
        self._name = name
        self._detached = detached

    def _channel(self) -> _Channel:
        with _channels_lock:
            ch = _channels.get(self._actor_id)
            if ch is None or ch.dead is not None:
                ch = _Channel(self._address, self._authkey)
                _channels[self._actor_id] = ch
            return ch

    def _call(self, method: str, args, kwargs) -> ObjectRef:
        deferred = _deferred_submit(args, kwargs, lambda a, kw: self._call_now(method, a, kw),
                                    order_key=self._actor_id)
        if deferred is not None:
            return deferred
        err = _upstream_error(args, kwargs)
        if err is not None:
            return _failed_ref(err)
        return self._call_now(method, *_resolve_args(args, kwargs))

    def _call_now(self, method: str, args, kwargs) -> ObjectRef:
        if self._actor_id in _local_actors:
            obj, pool, env = _local_actors[self._actor_id]
            fn = getattr(obj, method)

            def run():
                _tls.env = env
                try:
                    res = fn(*args, **kwargs)
                    if hasattr(res, "__await__"):
                        import asyncio

                        from ._worker import _await

                        res = asyncio.run(_await(res))
                    return res
                except BaseException as e:  # noqa: BLE001
                    import traceback

                    raise RayTaskError(e, traceback.format_exc()) from e

            return _traced(ObjectRef(pool.submit(run)), f"{self._class_name}.{method}", self._actor_id)
        if not self._address:
            return _failed_ref(RayActorError(f"actor {self._actor_id} is not reachable from this process"))
        try:
            return _traced(ObjectRef(self._channel().call(method, args, kwargs)), f"{self._class_name}.{method}",
                           self._actor_id)
        except (OSError, EOFError, ConnectionRefusedError) as e:
            return _failed_ref(RayActorError(f"cannot connect to actor {self._actor_id}: {e}"))

    def __getattr__(self, name: str):
        if name.startswith("_"):
            raise AttributeError(name)
        return _ActorMethod(self, name)

    def __reduce__(self):
        return (ActorHandle, (self._actor_id, self._class_name, self._address, self._authkey, self._name,
                              self._detached))

    def __repr__(self) -> str:
        return f"Actor({self._class_name}, {self._actor_id})"


class _ActorMethod:
    def __init__(self, handle: ActorHandle, name: str):
        self._handle, self._name = handle, name

    def remote(self, *args, **kwargs) -> ObjectRef:
        return self._handle._call(self._name, args, kwargs)

    def options(self, **_ignored) -> "_ActorMethod":
        return self


def _pending_timeout() -> float:
    return float(os.environ.get("RDB_CORE_PENDING_TIMEOUT_S", "30"))


def _pg_option(o: Dict[str, Any]):
    """(placement group, bundle index) from ``scheduling_strategy=`` or the
    legacy ``placement_group=`` / ``placement_group_bundle_index=`` options."""
    st = o.get("scheduling_strategy")
    if isinstance(st, str):
        if st not in ("DEFAULT", "SPREAD"):
            raise ValueError(f"unknown scheduling_strategy {st!r} (DEFAULT, SPREAD or a strategy object)")
        return None, -1
    if st is not None and hasattr(st, "node_id"):    # NodeAffinitySchedulingStrategy
        if st.node_id != _node_id() and not st.soft:
            raise TaskUnschedulableError(f"node affinity to {st.node_id!r}: no such alive node "
                                         f"(this node is {_node_id()})")
        return None, -1
    if st is not None and hasattr(st, "placement_group"):
        return st.placement_group, int(st.placement_group_bundle_index)
    if o.get("placement_group") not in (None, "default"):
        return o["placement_group"], int(o.get("placement_group_bundle_index", -1))
    return None, -1


def _allocate(ctx: _Context, owner: str, num_gpus: float, pg=None, bundle_index: int = -1):
    from ..runtime.resources import visible_devices_env

    if pg is not None:       # carve the demand out of a reserved bundle
        from ..runtime.resources import Allocation

        _, gpus = pg._take(owner, float(num_gpus or 0), bundle_index)
        gpus = gpus if num_gpus else []
        env = dict(visible_devices_env(gpus)) if num_gpus else {}
        env["RDB_CORE_GPU_IDS"] = ",".join(str(g) for g in gpus)
        env["RDB_CORE_NAMESPACE"] = ctx.namespace
        return Allocation(owner, gpus, float(num_gpus or 0), 0), env

    deadline = time.monotonic() + _pending_timeout()
    while True:   # like Ray, a creation that does not fit yet waits for resources
        a = ctx.allocator.allocate(owner, float(num_gpus or 0))
        if a is not None:
            break
        if time.monotonic() > deadline:
            raise RayError(f"{owner}: {num_gpus} GPU(s) not available within {_pending_timeout():.0f} s "
                           f"(allocator: {ctx.allocator.snapshot()})")
        time.sleep(0.05)
    env = dict(visible_devices_env(a.gpus)) if num_gpus else {}
    env["RDB_CORE_GPU_IDS"] = ",".join(str(g) for g in a.gpus)
    env["RDB_CORE_NAMESPACE"] = ctx.namespace
    return a, env


class ActorClass:
    def __init__(self, cls, options: Dict[str, Any]):
        self._cls = cls
        self._options = dict(options)
        self.__name__ = getattr(cls, "__name__", "Actor")

    def options(self, **opts) -> "ActorClass":
        o = dict(self._options)
        o.update(opts)
        return ActorClass(self._cls, o)

    def remote(self, *args, **kwargs) -> ActorHandle:
        ctx = _require_ctx()
        o = self._options
        name = o.get("name")
        detached = o.get("lifetime") == "detached"
        if name:
            if o.get("get_if_exists"):
                try:
                    return get_actor(name, o.get("namespace"))
                except ValueError:
                    pass
            if os.path.exists(_name_path(ctx, name, o.get("namespace"))):
                try:
                    get_actor(name, o.get("namespace"))
                    raise ValueError(f"an actor named {name!r} already exists")
                except ValueError as e:
                    if "already exists" in str(e):
                        raise
        args, kwargs = _resolve_args(args, kwargs)
        actor_id = uuid.uuid4().hex[:16]
        maxc = int(o.get("max_concurrency", 1))
        pg, bidx = _pg_option(o)
        a, env = _allocate(ctx, actor_id, o.get("num_gpus", 0), pg, bidx)
        try:
            if ctx.local_mode:
                prev = getattr(_tls, "env", None)
                _tls.env = env
                try:
                    obj = self._cls(*args, **kwargs)
                finally:
                    _tls.env = prev
                _local_actors[actor_id] = (obj, ThreadPoolExecutor(maxc, thread_name_prefix="rdb-lactor"), env)
                h = ActorHandle(actor_id, self.__name__, name=name, detached=detached)
                pid = os.getpid()
            else:
                h, pid = self._spawn(ctx, actor_id, args, kwargs, env, maxc, name, detached)
        except BaseException:
            ctx.allocator.release(actor_id)
            if pg is not None:
                pg._give_back(actor_id)
            raise
        ctx.owned.append(h)
        _register(ctx, h, pid, o.get("namespace"), a.gpus)
        return h

    def _spawn(self, ctx, actor_id, args, kwargs, env, maxc, name, detached):
        import sys

        import cloudpickle

        from ._worker import actor_main

        address = os.path.join(ctx.sock_dir, actor_id + ".sock")
        authkey = secrets.token_bytes(16)
        payload = cloudpickle.dumps((self._cls, args, kwargs))
        mpctx = mp.get_context("spawn")
        r, w = mpctx.Pipe(duplex=False)
        p = mpctx.Process(target=actor_main, args=(payload, list(sys.path), address, authkey, env, maxc, w),
                          daemon=not detached, name=f"rdb-actor-{self.__name__}")
        p.start()
        w.close()
        if not r.poll(float(os.environ.get("RDB_CORE_START_TIMEOUT_S", "120"))):
            p.terminate()
            raise RayActorError(f"actor {self.__name__} did not start")
        status, info = r.recv()
        if status != "ok":
            p.join(5)
            raise RayActorError(f"actor {self.__name__} failed in __init__: {info}")
        ctx.procs[actor_id] = p
        return ActorHandle(actor_id, self.__name__, address, authkey, name, detached), p.pid


def _name_path(ctx: _Context, name: str, namespace: Optional[str]) -> str:
    root = _registry_root(namespace) if namespace else ctx.registry
    return os.path.join(root, name + ".json")


def _register(ctx: _Context, h: ActorHandle, pid: int, namespace: Optional[str], gpus: List[int]) -> None:
    rec = dict(actor_id=h._actor_id, class_name=h._class_name, address=h._address, authkey=h._authkey.hex(),
               name=h._name, pid=pid, detached=h._detached, gpus=gpus, local=not h._address)
    root = _registry_root(namespace) if namespace else ctx.registry
    os.makedirs(os.path.join(root, "_actors"), exist_ok=True)
    with open(os.path.join(root, "_actors", h._actor_id + ".json"), "w") as f:
        json.dump(rec, f)
    if h._name:
        tmp = os.path.join(root, f".{h._name}.{h._actor_id}.tmp")
        with open(tmp, "w") as f:
            json.dump(rec, f)
        os.replace(tmp, os.path.join(root, h._name + ".json"))


def _unregister(ctx: _Context, h: ActorHandle) -> None:
    for root in {ctx.registry}:
        try:
            os.remove(os.path.join(root, "_actors", h._actor_id + ".json"))
        except OSError:
            pass
        if h._name:
            p = os.path.join(root, h._name + ".json")
            try:
                with open(p) as f:
                    if json.load(f).get("actor_id") == h._actor_id:
                        os.remove(p)
            except (OSError, ValueError):
                pass


def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except OSError:
        return False


def get_actor(name: str, namespace: Optional[str] = None) -> ActorHandle:
    ctx = _require_ctx()
    try:
        with open(_name_path(ctx, name, namespace)) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        raise ValueError(f"Failed to look up actor with name {name!r}") from None
    if not rec.get("local") and not _pid_alive(int(rec["pid"])):
        raise ValueError(f"Failed to look up actor with name {name!r} (its process is gone)")
    if rec.get("local") and rec["actor_id"] not in _local_actors:
        raise ValueError(f"actor {name!r} is a local-mode actor of another process")
    return ActorHandle(rec["actor_id"], rec["class_name"], rec["address"], bytes.fromhex(rec["authkey"]),
                       rec.get("name"), rec.get("detached", False))


def kill(actor: ActorHandle, *, no_restart: bool = True, _ctx_override: Optional[_Context] = None) -> None:
    from ._worker import TERMINATE

    ctx = _ctx_override or _require_ctx()
    if actor._actor_id in _local_actors:
        _, pool, _ = _local_actors.pop(actor._actor_id)
        pool.shutdown(wait=False, cancel_futures=True)
    else:
        p = ctx.procs.pop(actor._actor_id, None)
        try:
            actor._channel().call(TERMINATE, (), {}).result(2.0)
        except Exception:
            pass
        if p is not None:
            p.join(2.0)
            if p.is_alive():
                p.terminate()
                p.join(2.0)
        else:   # an actor of another driver: signal its process
            try:
                with open(os.path.join(ctx.registry, "_actors", actor._actor_id + ".json")) as f:
                    os.kill(int(json.load(f)["pid"]), 15)
            except (OSError, ValueError):
                pass
        with _channels_lock:
            ch = _channels.pop(actor._actor_id, None)
        if ch is not None:
            ch.close()
    ctx.allocator.release(actor._actor_id)
    from .util.placement_group import _owner_group

    g = _owner_group(actor._actor_id)
    if g is not None:
        g._give_back(actor._actor_id)
    _unregister(ctx, actor)
    if actor in ctx.owned:
        ctx.owned.remove(actor)


# ---------------------------------------------------------------------------
# tasks
# ---------------------------------------------------------------------------
class _FnHost:
    def __init__(self, fn):
        self.fn = fn

    def run(self, args, kwargs):
        return self.fn(*args, **kwargs)


class RemoteFunction:
    def __init__(self, fn, options: Dict[str, Any]):
        self._fn = fn
        self._options = dict(options)
        self.__name__ = getattr(fn, "__name__", "task")

    def options(self, **opts) -> "RemoteFunction":
        o = dict(self._options)
        o.update(opts)
        return RemoteFunction(self._fn, o)

    def remote(self, *args, **kwargs) -> ObjectRef:
        ctx = _require_ctx()
        deferred = _deferred_submit(args, kwargs, lambda a, kw: self._remote_now(ctx, a, kw))
        if deferred is not None:
            return deferred
        err = _upstream_error(args, kwargs)
        if err is not None:
            return _failed_ref(err)
        return self._remote_now(ctx, *_resolve_args(args, kwargs))

    def _remote_now(self, ctx, args, kwargs) -> ObjectRef:
        num_gpus = self._options.get("num_gpus", 0)
        try:
            _pg_option(self._options)          # validates scheduling_strategy (node affinity)
        except TaskUnschedulableError as e:
            return _failed_ref(e)
        if not num_gpus:
            fn = self._fn

            def run():
                try:
                    return fn(*args, **kwargs)
                except BaseException as e:  # noqa: BLE001
                    import traceback

                    raise RayTaskError(e, traceback.format_exc()) from e

            return _traced(ObjectRef(ctx.tasks.submit(run)), self.__name__, "tasks")
        # a GPU task runs in a one-shot process pinned to its GPUs
        host_opts = {"num_gpus": num_gpus}
        for k in ("scheduling_strategy", "placement_group", "placement_group_bundle_index"):
            if k in self._options:
                host_opts[k] = self._options[k]
        host = ActorClass(_FnHost, host_opts).remote(self._fn)
        ref = host.run.remote(args, kwargs)
        ref._fut.add_done_callback(lambda _f: threading.Thread(target=kill, args=(host,), daemon=True).start())
        return ref

    def __call__(self, *a, **kw):
        raise TypeError(f"remote function {self.__name__} must be called with .remote()")


def remote(*args, **options):
    """``@remote`` / ``@remote(num_gpus=1, max_concurrency=4, name=...)`` on a
    function (task) or a class (actor)."""
    def wrap(obj):
        if isinstance(obj, type):
            return ActorClass(obj, options)
        if callable(obj):
            return RemoteFunction(obj, options)
        raise TypeError("remote() decorates functions and classes")

    if len(args) == 1 and not options and (callable(args[0]) or isinstance(args[0], type)):
        return wrap(args[0])
    if args:
        raise TypeError("remote() takes keyword options only")
    return wrap


from . import dag, data, state, util  # noqa: E402  (submodules use the names above)
