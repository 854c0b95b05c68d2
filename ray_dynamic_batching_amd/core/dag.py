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

Values move actor -> driver -> actor over the core actor channels; GPU tensors
between replicas move with ``parallel.collective`` send / recv (RCCL over
xGMI), not through the DAG.
"""
from __future__ import annotations

import threading
from concurrent.futures import Future
from typing import Any, Dict, List, Optional, Sequence, Tuple

from . import ObjectRef, RayError, _ActorMethod

__all__ = ["DAGNode", "InputNode", "InputAttributeNode", "ClassMethodNode", "MultiOutputNode", "CompiledDAG"]


class DAGNode:
    def _deps(self) -> List["DAGNode"]:
        return []

    def execute(self, *args, **kwargs):
        return _Schedule(self).run(args, kwargs, None)

    def experimental_compile(self, _max_inflight_executions: int = 10, **_ignored) -> "CompiledDAG":
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
