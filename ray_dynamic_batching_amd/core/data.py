"""Offline batch inference: the ``ray.data`` subset the fork's models need.

SURVEY.md §2.3 lists Ray Data's ``Dataset.map_batches(fn, batch_size,
num_gpus, compute=ActorPoolStrategy)`` (reference: ``python/ray/data/
dataset.py:391``, ``data/_internal/compute.py:53``,
``execution/operators/actor_pool_map_operator.py:34,415,561``) as the offline
counterpart of serving: a stream of blocks goes through a pool of GPU-pinned
actors, each of which loads the model once and runs it batch by batch.  This
module keeps that API and builds it on ``core`` (one spawned process per pool
actor, pinned through the node's GPU slot allocator):

* sources: ``from_items``, ``range``, ``from_numpy``, ``from_pandas``;
* lazy transforms: ``map_batches`` (function, or callable class on an actor
  pool with ``compute=ActorPoolStrategy(size | min_size, max_size)`` or
  ``concurrency=``), ``map``, ``flat_map``, ``filter``, ``limit``,
  ``repartition``;
* consumption: ``iter_batches`` / ``iter_rows`` / ``take`` / ``take_all`` /
  ``take_batch`` / ``count`` / ``schema`` / ``to_pandas`` / ``materialize``.

Rows are dicts; ``batch_format="numpy"`` (default) hands the UDF a dict of
column arrays, ``"pandas"`` a DataFrame.  Execution streams blocks: a pool
stage keeps at most ``max_tasks_in_flight_per_actor`` blocks queued per actor
(least-loaded dispatch) and yields results in input order, so a consumer sees
the first batches while later ones are still on the GPUs.
"""
from __future__ import annotations

import builtins
import collections
import itertools
from dataclasses import dataclass
from typing import Any, Callable, Dict, Iterator, List, Optional, Sequence

import numpy as np

from . import ActorClass, get, kill

__all__ = ["Dataset", "ActorPoolStrategy", "TaskPoolStrategy", "from_items", "range", "from_numpy",
           "from_pandas"]

Block = List[Dict[str, Any]]          # a block is a list of rows


@dataclass
class ActorPoolStrategy:
    """``compute=ActorPoolStrategy(size=n)`` or ``(min_size=, max_size=)``;
    the pool starts at ``min_size`` actors and grows up to ``max_size`` while
    every actor has a full in-flight window."""
    size: Optional[int] = None
    min_size: int = 1
    max_size: Optional[int] = None
    max_tasks_in_flight_per_actor: int = 2

    def __post_init__(self):
        if self.size is not None:
            if self.size < 1:
                raise ValueError("size must be >= 1")
            self.min_size = self.max_size = self.size
        if self.max_size is None:
            self.max_size = self.min_size
        if self.min_size < 1 or self.max_size < self.min_size:
            raise ValueError("need 1 <= min_size <= max_size")
        if self.max_tasks_in_flight_per_actor < 1:
            raise ValueError("max_tasks_in_flight_per_actor must be >= 1")


@dataclass
class TaskPoolStrategy:
    """Stateless function UDFs run in the driver process (tasks)."""
    size: Optional[int] = None


# ---------------------------------------------------------------------------
# batch formats
# ---------------------------------------------------------------------------
def _rows_to_batch(rows: Block, fmt: str):
    if fmt in ("numpy", "default"):
        keys = list(rows[0].keys()) if rows else []
        return {k: np.asarray([r[k] for r in rows]) for k in keys}
    if fmt == "pandas":
        import pandas as pd

        return pd.DataFrame(rows)
    if fmt in (None, "rows"):
        return list(rows)
    raise ValueError(f"unknown batch_format {fmt!r}")


def _batch_to_rows(batch) -> Block:
    if isinstance(batch, list):
        return [r if isinstance(r, dict) else {"item": r} for r in batch]
    try:
        import pandas as pd

        if isinstance(batch, pd.DataFrame):
            return batch.to_dict("records")
    except ImportError:   # pragma: no cover
        pass
    if isinstance(batch, dict):
        cols = {k: (v if isinstance(v, (np.ndarray, list)) else np.asarray(v)) for k, v in batch.items()}
        lens = {len(v) for v in cols.values()}
        if len(lens) > 1:
            raise ValueError(f"map_batches UDF returned columns of different lengths {sorted(lens)}")
        n = lens.pop() if lens else 0
        return [{k: v[i] for k, v in cols.items()} for i in builtins.range(n)]
    raise TypeError(f"map_batches UDF must return a dict of arrays, a DataFrame or a list, got {type(batch)}")


def _rebatch(blocks: Iterator[Block], batch_size: Optional[int]) -> Iterator[Block]:
    """Re-cut a block stream into batches of exactly ``batch_size`` rows (the
    last may be short); ``None`` keeps the block boundaries."""
    if batch_size is None:
        for b in blocks:
            if b:
                yield b
        return
    buf: Block = []
    for b in blocks:
        buf.extend(b)
        while len(buf) >= batch_size:
            yield buf[:batch_size]
            buf = buf[batch_size:]
    if buf:
        yield buf


# ---------------------------------------------------------------------------
# stages
# ---------------------------------------------------------------------------
class _Stage:
    def run(self, blocks: Iterator[Block]) -> Iterator[Block]:
        raise NotImplementedError


class _RowStage(_Stage):
    def __init__(self, kind: str, fn: Callable):
        self.kind, self.fn = kind, fn

    def run(self, blocks):
        for b in blocks:
            if self.kind == "map":
                out = [self.fn(r) for r in b]
            elif self.kind == "flat_map":
                out = [o for r in b for o in self.fn(r)]
            else:
                out = [r for r in b if self.fn(r)]
            yield [o if isinstance(o, dict) else {"item": o} for o in out]


class _BatchUDF:
    """Runs inside a pool actor (or in the driver for function UDFs)."""

    def __init__(self, fn, fn_args, fn_kwargs, ctor_args, ctor_kwargs, is_class, batch_format):
        self.fn = fn(*ctor_args, **ctor_kwargs) if is_class else fn
        self.fn_args, self.fn_kwargs, self.batch_format = fn_args, fn_kwargs, batch_format

    def apply(self, rows: Block) -> Block:
        out = self.fn(_rows_to_batch(rows, self.batch_format), *self.fn_args, **self.fn_kwargs)
        if hasattr(out, "__next__") or (hasattr(out, "__iter__") and not isinstance(out, (dict, list))
                                        and type(out).__name__ != "DataFrame"):
            return [r for part in out for r in _batch_to_rows(part)]     # generator UDF
        return _batch_to_rows(out)

    def ready(self) -> bool:
        return True


class _MapBatches(_Stage):
    def __init__(self, fn, batch_size, batch_format, compute, num_gpus, fn_args, fn_kwargs, ctor_args,
                 ctor_kwargs):
        self.fn, self.batch_size, self.batch_format = fn, batch_size, batch_format
        self.is_class = isinstance(fn, type)
        if self.is_class and not isinstance(compute, ActorPoolStrategy):
            raise ValueError("a callable-class UDF needs compute=ActorPoolStrategy(...) or concurrency=")
        if not self.is_class and (ctor_args or ctor_kwargs):
            raise ValueError("fn_constructor_args / kwargs only apply to callable-class UDFs")
        self.compute, self.num_gpus = compute, num_gpus
        self.udf_args = (fn, fn_args, fn_kwargs, ctor_args, ctor_kwargs, self.is_class, batch_format)

    def run(self, blocks):
        batches = _rebatch(blocks, self.batch_size)
        if not isinstance(self.compute, ActorPoolStrategy):
            udf = _BatchUDF(*self.udf_args)
            for b in batches:
                yield udf.apply(b)
            return
        yield from _ActorPool(self.compute, self.num_gpus, self.udf_args).map(batches)


class _ActorPool:
    def __init__(self, strategy: ActorPoolStrategy, num_gpus: float, udf_args):
        self.s, self.num_gpus, self.udf_args = strategy, num_gpus, udf_args
        self.actors: List[Any] = []
        self.inflight: Dict[int, int] = {}

    def _add_actor(self):
        opts = {"num_gpus": self.num_gpus} if self.num_gpus else {}
        a = ActorClass(_BatchUDF, opts).remote(*self.udf_args)
        get(a.ready.remote())             # the model is loaded before the actor takes work
        self.inflight[len(self.actors)] = 0
        self.actors.append(a)

    def map(self, batches: Iterator[Block]) -> Iterator[Block]:
        window = self.s.max_tasks_in_flight_per_actor
        pending: "collections.deque" = collections.deque()     # (actor idx, ref) in input order
        try:
            for _ in builtins.range(self.s.min_size):
                self._add_actor()
            for b in batches:
                idx = min(self.inflight, key=self.inflight.get)
                if self.inflight[idx] >= window and len(self.actors) < self.s.max_size:
                    self._add_actor()          # every actor saturated: grow the pool
                    idx = len(self.actors) - 1
                while self.inflight[idx] >= window:
                    yield self._pop(pending)
                    idx = min(self.inflight, key=self.inflight.get)
                pending.append((idx, self.actors[idx].apply.remote(b)))
                self.inflight[idx] += 1
            while pending:
                yield self._pop(pending)
        finally:
            for a in self.actors:
                kill(a)

    def _pop(self, pending) -> Block:
        idx, ref = pending.popleft()
        try:
            return get(ref)
        finally:
            self.inflight[idx] -= 1


class _Limit(_Stage):
    def __init__(self, n: int):
        self.n = n

    def run(self, blocks):
        left = self.n
        for b in blocks:
            if left <= 0:
                return
            yield b[:left]
            left -= len(b)


class _Repartition(_Stage):
    def __init__(self, n: int):
        self.n = n

    def run(self, blocks):
        rows = [r for b in blocks for r in b]
        for part in np.array_split(np.arange(len(rows)), self.n):
            yield [rows[i] for i in part]


# ---------------------------------------------------------------------------
# Dataset
# ---------------------------------------------------------------------------
class Dataset:
    def __init__(self, source: Callable[[], Iterator[Block]], stages: Sequence[_Stage] = ()):
        self._source, self._stages = source, list(stages)

    def _then(self, stage: _Stage) -> "Dataset":
        return Dataset(self._source, self._stages + [stage])

    # -- transforms (lazy) --------------------------------------------------
    def map_batches(self, fn, *, batch_size: Optional[int] = 1024, batch_format: str = "numpy",
                    compute=None, concurrency=None, num_gpus: float = 0, fn_args=(), fn_kwargs=None,
                    fn_constructor_args=(), fn_constructor_kwargs=None, **_ray_remote_args) -> "Dataset":
        if batch_size is not None and batch_size < 1:
            raise ValueError("batch_size must be >= 1 or None")
        if compute is None and concurrency is not None:
            if isinstance(concurrency, tuple):
                compute = ActorPoolStrategy(min_size=concurrency[0], max_size=concurrency[1])
            elif isinstance(fn, type):
                compute = ActorPoolStrategy(size=int(concurrency))
        if compute is None and isinstance(fn, type):
            raise ValueError("callable-class UDFs need compute=ActorPoolStrategy(...) or concurrency=")
        return self._then(_MapBatches(fn, batch_size, batch_format, compute, num_gpus, tuple(fn_args),
                                      dict(fn_kwargs or {}), tuple(fn_constructor_args),
                                      dict(fn_constructor_kwargs or {})))

    def map(self, fn: Callable[[Dict], Dict]) -> "Dataset":
        return self._then(_RowStage("map", fn))

    def flat_map(self, fn: Callable[[Dict], List[Dict]]) -> "Dataset":
        return self._then(_RowStage("flat_map", fn))

    def filter(self, fn: Callable[[Dict], bool]) -> "Dataset":
        return self._then(_RowStage("filter", fn))

    def limit(self, n: int) -> "Dataset":
        return self._then(_Limit(int(n)))

    def repartition(self, num_blocks: int) -> "Dataset":
        if num_blocks < 1:
            raise ValueError("num_blocks must be >= 1")
        return self._then(_Repartition(int(num_blocks)))

    # -- execution -----------------------------------------------------------
    def _blocks(self) -> Iterator[Block]:
        it = self._source()
        for st in self._stages:
            it = st.run(it)
        return it

    def materialize(self) -> "Dataset":
        blocks = [b for b in self._blocks() if b]
        return Dataset(lambda: iter(blocks))

    def iter_rows(self) -> Iterator[Dict[str, Any]]:
        for b in self._blocks():
            yield from b

    def iter_batches(self, *, batch_size: Optional[int] = 256, batch_format: str = "numpy",
                     drop_last: bool = False):
        for b in _rebatch(self._blocks(), batch_size):
            if drop_last and batch_size is not None and len(b) < batch_size:
                return
            yield _rows_to_batch(b, batch_format)

    def take(self, limit: int = 20) -> List[Dict[str, Any]]:
        return list(itertools.islice(self.iter_rows(), limit))

    def take_all(self) -> List[Dict[str, Any]]:
        return list(self.iter_rows())

    def take_batch(self, batch_size: int = 20, *, batch_format: str = "numpy"):
        return _rows_to_batch(self.take(batch_size), batch_format)

    def count(self) -> int:
        return sum(len(b) for b in self._blocks())

    def schema(self) -> Dict[str, str]:
        first = self.take(1)
        return {k: type(v).__name__ if not isinstance(v, np.generic) else str(v.dtype)
                for k, v in (first[0].items() if first else [])}

    def columns(self) -> List[str]:
        return list(self.schema())

    def to_pandas(self):
        import pandas as pd

        return pd.DataFrame(self.take_all())

    def num_blocks(self) -> int:
        return sum(1 for _ in self._blocks())

    def __repr__(self):
        return f"Dataset(stages={[type(s).__name__.lstrip('_') for s in self._stages]})"


def _blocked(rows: List[Dict[str, Any]], parallelism: int) -> Callable[[], Iterator[Block]]:
    n = max(1, min(parallelism, len(rows) or 1))
    bounds = np.linspace(0, len(rows), n + 1).astype(int)
    blocks = [rows[bounds[i]:bounds[i + 1]] for i in builtins.range(n)]
    return lambda: iter(blocks)


def from_items(items: Sequence[Any], *, override_num_blocks: int = 8) -> Dataset:
    rows = [it if isinstance(it, dict) else {"item": it} for it in items]
    return Dataset(_blocked(rows, override_num_blocks))


def range(n: int, *, override_num_blocks: int = 8) -> Dataset:   # noqa: A001 - Ray's name
    return Dataset(_blocked([{"id": i} for i in builtins.range(n)], override_num_blocks))


def from_numpy(arr, *, column: str = "data", override_num_blocks: int = 8) -> Dataset:
    arr = np.asarray(arr)
    return Dataset(_blocked([{column: arr[i]} for i in builtins.range(len(arr))], override_num_blocks))


def from_pandas(df, *, override_num_blocks: int = 8) -> Dataset:
    return Dataset(_blocked(df.to_dict("records"), override_num_blocks))
