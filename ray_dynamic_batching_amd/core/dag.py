"""Actor DAGs: ``InputNode`` / ``actor.method.bind(...)`` / ``MultiOutputNode``
with interpreted ``execute`` and ``experimental_compile()``.

Reference: ``python/ray/dag/dag_node.py:153`` (bind / execute),
``dag/compiled_dag_node.py:113,549,1956`` (compile, execute, teardown) --
static actor pipelines, used by the reference's tests to model 1F1B pipeline
parallelism.  Here:

* ``execute(*args)`` walks the graph once per call and chains actor calls
  through future callbacks, so the submitting thread never blocks and
  independent branches run concurrently; it returns an ``ObjectRef`` (a list
  of them for a ``MultiOutputNode``).
* ``experimental_compile(_max_inflight_executions=N)`` validates and orders
  the graph ONCE (topological schedule, argument slots resolved to node
  indices), then ``CompiledDAG.execute`` replays that schedule.  Up to ``N``
  executions are in flight; each actor runs its calls in submission order (the
  per-caller ordering of ``core``), so consecutive executions pipeline across
  the stages like microbatches in 1F1B.  ``teardown()`` waits for in-flight
  executions and rejects new ones.

Compiled DAGs move values over shared-memory channels (``core/channel.py``,
reference ``experimental/channel/shared_memory_channel.py``): each edge is a
native shm ring, each actor runs an execution loop over its nodes, and only
the DAG's inputs and outputs touch the driver.  ``_channel="driver"`` keeps the
interpreted path (values hop actor -> driver -> actor).  A node marked
``.with_tensor_transport()`` (or ``.with_type_hint(TorchTensorType())``,
reference ``dag_node.py`` ``with_tensor_transport`` / ``with_type_hint``)
sends the torch tensors of its values through the reader's staging ring --
GPU memory exported with HIP IPC (device-to-device copies, over xGMI between
GPUs), shared memory for host tensors -- with only descriptors in the shm
ring (``core/channel.py`` ``TensorRing``).
"""
from __future__ import annotations

import threading
from concurrent.futures import Future
from typing import Any, Dict, List, Optional, Sequence, Tuple

from . import ObjectRef, RayError, _ActorMethod
from .channel import TorchTensorType

__all__ = ["DAGNode", "InputNode", "InputAttributeNode", "ClassMethodNode", "MultiOutputNode", "CompiledDAG",
           "TorchTensorType"]


class DAGNode:
    _type_hint: Optional[TorchTensorType] = None

    def _deps(self) -> List["DAGNode"]:
        return []

    def with_tensor_transport(self, transport: str = "auto", _static_shape: bool = False,
                              _direct_return: bool = False) -> "DAGNode":
        """Ship the torch tensors of this node's outputs through staging rings
        (compiled DAGs; see core/channel.py).  Returns the node."""
        self._type_hint = TorchTensorType(transport, _static_shape, _direct_return)
        return self

    def with_type_hint(self, hint) -> "DAGNode":
        if hint is not None and not isinstance(hint, TorchTensorType):
            raise TypeError("with_type_hint expects a TorchTensorType")
        self._type_hint = hint
        return self

    def execute(self, *args, **kwargs):
        return _Schedule(self).run(args, kwargs, None)

    def experimental_compile(self, _max_inflight_executions: int = 10, _buffer_size_bytes: int = 1 << 20,
                             _channel: str = "shm", **_ignored) -> "CompiledDAG":
        """``_channel="shm"`` (default): every edge becomes a shared-memory
        channel and each actor runs an execution loop (values never pass
        through the driver); ``"driver"``: the interpreted schedule replayed
        per execution (values hop through the driver)."""
        if _channel == "shm":
            return ChannelCompiledDAG(self, _max_inflight_executions, _buffer_size_bytes)
        return CompiledDAG(self, _max_inflight_executions)


class InputNode(DAGNode):
    """The DAG's argument(s); usable as a context manager like Ray's."""

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def __getitem__(self, key):
        return InputAttributeNode(self, key, "item")

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return InputAttributeNode(self, name, "attr")


class InputAttributeNode(DAGNode):
    def __init__(self, inp: InputNode, key, how: str):
        self.inp, self.key, self.how = inp, key, how

    def _deps(self):
        return [self.inp]


class ClassMethodNode(DAGNode):
    def __init__(self, method: _ActorMethod, args: Tuple, kwargs: Dict):
        self.method, self.args, self.kwargs = method, args, kwargs

    def _deps(self):
        return [a for a in list(self.args) + list(self.kwargs.values()) if isinstance(a, DAGNode)]


class MultiOutputNode(DAGNode):
    def __init__(self, outputs: Sequence[DAGNode]):
        if not outputs:
            raise ValueError("MultiOutputNode needs at least one output")
        self.outputs = list(outputs)

    def _deps(self):
        return list(self.outputs)


def _bind(self: _ActorMethod, *args, **kwargs) -> ClassMethodNode:
    return ClassMethodNode(self, args, kwargs)


_ActorMethod.bind = _bind           # actor.method.bind(...) builds a DAG node


class _Schedule:
    """Topological order of a DAG with each node's inputs as node indices."""

    def __init__(self, root: DAGNode):
        order: List[DAGNode] = []
        state: Dict[int, int] = {}

        def visit(n: DAGNode):
            s = state.get(id(n), 0)
            if s == 1:
                raise ValueError("the DAG has a cycle")
            if s == 2:
                return
            state[id(n)] = 1
            for d in n._deps():
                visit(d)
            state[id(n)] = 2
            order.append(n)

        visit(root)
        inputs = [n for n in order if isinstance(n, InputNode)]
        if len(inputs) > 1:
            raise ValueError("a DAG takes exactly one InputNode")
        self.order, self.root = order, root
        self.index = {id(n): i for i, n in enumerate(order)}

    def run(self, args, kwargs, on_done) -> Any:
        vals: List[Optional[Future]] = [None] * len(self.order)
        for i, n in enumerate(self.order):
            vals[i] = self._launch(n, vals, args, kwargs)
        if isinstance(self.root, MultiOutputNode):
            outs = [vals[self.index[id(o)]] for o in self.root.outputs]
            if on_done is not None:
                _when_all(outs, on_done)
            return [ObjectRef(f) for f in outs]
        out = vals[self.index[id(self.root)]]
        if on_done is not None:
            out.add_done_callback(lambda _f: on_done())
        return ObjectRef(out)

    def _launch(self, n: DAGNode, vals, args, kwargs) -> Future:
        f: Future = Future()
        if isinstance(n, InputNode):
            f.set_result(args[0] if len(args) == 1 and not kwargs else _Args(args, kwargs))
            return f
        if isinstance(n, InputAttributeNode):
            src = vals[self.index[id(n.inp)]].result()
            try:
                if isinstance(src, _Args):
                    v = src.args[n.key] if isinstance(n.key, int) else src.kwargs[n.key]
                else:
                    v = src[n.key] if n.how == "item" else getattr(src, n.key)
                f.set_result(v)
            except Exception as e:  # noqa: BLE001
                f.set_exception(RayError(f"DAG input has no {n.key!r}: {e}"))
            return f
        if isinstance(n, MultiOutputNode):
            f.set_result(None)
            return f
        deps = [vals[self.index[id(d)]] for d in n._deps()]

        def submit():
            try:
                a = tuple(vals[self.index[id(x)]].result() if isinstance(x, DAGNode) else x for x in n.args)
                kw = {k: (vals[self.index[id(x)]].result() if isinstance(x, DAGNode) else x)
                      for k, x in n.kwargs.items()}
            except BaseException as e:  # noqa: BLE001 - upstream failure propagates
                f.set_exception(e)
                return
            # submit() runs as a Future done-callback, where concurrent.futures
            # would log and swallow a synchronous failure (a missing method, a
            # killed actor): route it into the node's future instead, so get()
            # raises and the compiled DAG's in-flight slot is released
            try:
                ref = n.method.remote(*a, **kw)
            except BaseException as e:  # noqa: BLE001
                f.set_exception(e if isinstance(e, Exception) else RayError(repr(e)))
                return
            ref._fut.add_done_callback(lambda r: f.set_exception(r.exception()) if r.exception() is not None
                                       else f.set_result(r.result()))

        _when_all(deps, submit)
        return f


class _Args:
    def __init__(self, args, kwargs):
        self.args, self.kwargs = args, kwargs


def _when_all(futs: List[Future], fn) -> None:
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


class CompiledDAG:
    def __init__(self, root: DAGNode, max_inflight: int):
        if max_inflight < 1:
            raise ValueError("_max_inflight_executions must be >= 1")
        self._sched = _Schedule(root)
        if not any(isinstance(n, InputNode) for n in self._sched.order):
            raise ValueError("a compiled DAG needs an InputNode")
        if not any(isinstance(n, ClassMethodNode) for n in self._sched.order):
            raise ValueError("a compiled DAG needs at least one actor method node")
        self._slots = threading.BoundedSemaphore(max_inflight)
        self._inflight = 0
        self._cv = threading.Condition()
        self._closed = False

    def execute(self, *args, **kwargs):
        if self._closed:
            raise RayError("this compiled DAG was torn down")
        self._slots.acquire()
        with self._cv:
            self._inflight += 1

        def done():
            self._slots.release()
            with self._cv:
                self._inflight -= 1
                self._cv.notify_all()

        return self._sched.run(args, kwargs, done)

    def teardown(self, timeout: Optional[float] = 30.0) -> None:
        self._closed = True
        with self._cv:
            self._cv.wait_for(lambda: self._inflight == 0, timeout)


class ChannelCompiledDAG:
    """A compiled DAG on shared-memory channels (see module doc)."""

    def __init__(self, root: DAGNode, max_inflight: int, buffer_size: int):
        import collections
        import uuid

        from . import _local_actors
        from ..runtime import job as rjob
        from .channel import ChannelReader, ChannelWriter, start_exec_loop
        from ._worker import DAG_EXEC

        if max_inflight < 1:
            raise ValueError("_max_inflight_executions must be >= 1")
        sched = _Schedule(root)
        if not any(isinstance(n, InputNode) for n in sched.order):
            raise ValueError("a compiled DAG needs an InputNode")
        nodes = [n for n in sched.order if isinstance(n, ClassMethodNode)]
        if not nodes:
            raise ValueError("a compiled DAG needs at least one actor method node")
        outs = root.outputs if isinstance(root, MultiOutputNode) else [root]
        if not all(isinstance(o, ClassMethodNode) for o in outs):
            raise ValueError("compiled DAG outputs must be actor method nodes")
        nq = [0]
        producers: Dict[int, List[int]] = collections.defaultdict(list)
        self._inputs: List[Tuple[int, DAGNode]] = []      # driver-written channels
        # tensor channels: queue -> (reader actor id or None = driver, ring devices)
        tensor_q: Dict[int, Tuple[Optional[str], Tuple[str, ...]]] = {}

        def devs_of(a: DAGNode) -> Optional[Tuple[str, ...]]:
            h = getattr(a, "_type_hint", None)
            if h is None:
                return None
            return ("cpu",) if h.transport == "shm" else ("cpu", "cuda")

        def chan(a: DAGNode, reader: Optional[str]) -> Tuple[str, int]:
            q = nq[0]
            nq[0] += 1
            if isinstance(a, (InputNode, InputAttributeNode)):
                self._inputs.append((q, a))
            elif isinstance(a, ClassMethodNode):
                producers[id(a)].append(q)
                if devs_of(a):
                    tensor_q[q] = (reader, devs_of(a))
            else:
                raise ValueError(f"unsupported DAG argument node {type(a).__name__}")
            return ("chan", q)

        specs = []
        for n in nodes:
            rd = n.method._handle._actor_id
            args = [chan(a, rd) if isinstance(a, DAGNode) else ("const", a) for a in n.args]
            kwargs = {k: (chan(a, rd) if isinstance(a, DAGNode) else ("const", a)) for k, a in n.kwargs.items()}
            specs.append((n, args, kwargs))
        self._outputs = []
        for o in outs:
            q = nq[0]
            nq[0] += 1
            producers[id(o)].append(q)
            self._outputs.append(q)
            if devs_of(o):
                tensor_q[q] = (None, devs_of(o))
        self.multi = isinstance(root, MultiOutputNode)
        cap = 4
        while cap < max_inflight + 2:
            cap *= 2
        self.job_name = rjob.unique_job_name("dag")
        actors = {n.method._handle._actor_id: n.method._handle for n in nodes}
        self.job = rjob.Job(self.job_name, create=True, n_replicas=1, n_queues=nq[0], n_clients=len(actors) + 2,
                            req_capacity=cap, req_slot_bytes=buffer_size + 64, cmp_capacity=4, cmp_slot_bytes=64)
        per_actor: Dict[str, List[dict]] = collections.defaultdict(list)
        for n, args, kwargs in specs:
            in_q = [a[1] for a in args if a[0] == "chan"] + [a[1] for a in kwargs.values() if a[0] == "chan"]
            per_actor[n.method._handle._actor_id].append(dict(method=n.method._name, args=args, kwargs=kwargs,
                                                             in_queues=in_q, out_queues=producers[id(n)]))
        self._local_stops = []
        try:
            # tensor rings: allocated by each tensor channel's reader, attached by its writer
            from .channel import create_rings
            from ._worker import DAG_SETUP

            slots = cap + 2
            rings: Dict[int, Dict[str, dict]] = {}
            for q, (rd, devs) in tensor_q.items():
                spec = (self.job_name, [(q, slots, buffer_size)], devs)
                if rd is None or rd in _local_actors:
                    rings.update(create_rings(*spec))
                else:
                    rings.update(actors[rd]._call_now(DAG_SETUP, spec, {})._fut.result(60))
            pending = []
            for aid, ops in per_actor.items():
                outq = [q for op in ops for q in op["out_queues"]]
                plan = dict(job=self.job_name, ops=ops, rings={q: rings[q] for q in outq if q in rings})
                if aid in _local_actors:
                    self._local_stops.append(start_exec_loop(_local_actors[aid][0], plan))
                else:
                    pending.append(actors[aid]._call_now(DAG_EXEC, (plan,), {}))
            for ref in pending:
                ref._fut.result(60)
        except BaseException:
            from .channel import release_rings

            release_rings(self.job_name)
            self.job.close()
            raise
        self._client = rjob.Client(self.job)
        self._writers = [(ChannelWriter(self.job, q, self._client), src) for q, src in self._inputs]
        self._readers = [ChannelReader(self.job, q, self.job_name) for q in self._outputs]
        self._slots = threading.BoundedSemaphore(max_inflight)
        self._pending: "collections.deque" = collections.deque()
        self._cv = threading.Condition()
        self._stop = threading.Event()
        self._closed = False
        self._broken: Optional[str] = None
        self._reader = threading.Thread(target=self._collect, daemon=True, name="rdb-dag-out")
        self._reader.start()

    @staticmethod
    def _input_value(src: DAGNode, args, kwargs):
        whole = args[0] if len(args) == 1 and not kwargs else _Args(args, kwargs)
        if isinstance(src, InputNode):
            return whole
        if isinstance(whole, _Args):
            return whole.args[src.key] if isinstance(src.key, int) else whole.kwargs[src.key]
        return whole[src.key] if src.how == "item" else getattr(whole, src.key)

    def execute(self, *args, **kwargs):
        if self._closed:
            raise RayError("this compiled DAG was torn down")
        if self._broken is not None:
            raise RayError(f"this compiled DAG is broken ({self._broken}); tear it down")
        # Every input is pickled and size-checked BEFORE an in-flight slot is
        # taken and the execution's futures are queued: an oversized input
        # raises here with no channel written, so channels and futures stay
        # paired one message per execution.
        data = []
        for w, src in self._writers:
            try:
                v = ("val", self._input_value(src, args, kwargs))
            except Exception as e:  # noqa: BLE001
                v = ("err", RayError(f"DAG input has no {getattr(src, 'key', '?')!r}: {e}"))
            data.append(w.pack(*v))
        self._slots.acquire()
        futs = [Future() for _ in self._readers]
        with self._cv:
            self._pending.append(futs)
            self._cv.notify_all()
        for w_src, d in zip(self._writers, data):
            try:
                w_src[0].write("", None, self._stop, data=d)
            except BaseException as e:
                # A channel stayed full (or the DAG is stopping): that channel has
                # no message for this execution, so later executions would pair
                # values of different calls.  The DAG is unusable from here on.
                self._broken = f"input channel write failed: {e}"
                for f in futs:
                    if not f.done():
                        f.set_exception(RayError(self._broken))
                raise
        refs = [ObjectRef(f) for f in futs]
        return refs if self.multi else refs[0]

    def _collect(self) -> None:
        while True:
            with self._cv:
                while not self._pending and not self._stop.is_set():
                    self._cv.wait(0.1)
                if not self._pending:
                    return
                futs = self._pending[0]
            msgs = []
            for r in self._readers:
                m = r.read(self._stop)
                if m is None:
                    return
                msgs.append(m)
            with self._cv:
                self._pending.popleft()
            for f, (kind, val) in zip(futs, msgs):
                if f.done():        # failed at submission (broken DAG)
                    continue
                if kind == "val":
                    f.set_result(val)
                elif kind == "err":
                    f.set_exception(val)
                else:
                    f.set_exception(RayError("compiled DAG stopped"))
            self._slots.release()

    def teardown(self, timeout: Optional[float] = 30.0) -> None:
        if self._closed:
            return
        self._closed = True
        import time as _t

        t_end = _t.monotonic() + (timeout or 30.0)
        with self._cv:
            while self._pending and _t.monotonic() < t_end:
                self._cv.wait(0.05)
        for w, _src in self._writers:
            try:
                w.write("stop", None, None, timeout_s=5.0)
            except Exception:  # noqa: BLE001
                pass
        for r in self._readers:          # loops forward STOP to the outputs once they have drained
            r.read(None, timeout_s=max(0.1, t_end - _t.monotonic()))
        self._stop.set()
        for s in self._local_stops:
            s.set()
        self._reader.join()          # it polls the stop flag: never unmap under a reading thread
        from .channel import release_rings

        release_rings(self.job_name, list(self._outputs))
        self.job.close()
