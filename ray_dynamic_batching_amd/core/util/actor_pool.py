"""``ray.util.ActorPool`` (reference ``python/ray/util/actor_pool.py``): a
fixed set of actors fed work items; ``map`` keeps input order,
``map_unordered`` yields as results finish, ``submit`` / ``get_next`` for
manual pipelining.  ``fn(actor, value)`` must return an ObjectRef
(``lambda a, v: a.method.remote(v)``)."""
from __future__ import annotations

import collections
import time
from typing import Any, Callable, Dict, Iterable, List, Optional

from .. import GetTimeoutError, ObjectRef, get, wait

__all__ = ["ActorPool"]


class ActorPool:
    def __init__(self, actors: List[Any]):
        self._idle = list(actors)
        self._future_to_actor: Dict[int, tuple] = {}     # seq -> (ref, actor)
        self._index_to_future: Dict[int, ObjectRef] = {}
        self._next_task = 0
        self._next_return = 0
        self._pending: "collections.deque" = collections.deque()

    def submit(self, fn: Callable[[Any, Any], ObjectRef], value: Any) -> None:
        if self._idle:
            actor = self._idle.pop()
            ref = fn(actor, value)
            self._future_to_actor[self._next_task] = (ref, actor)
            self._index_to_future[self._next_task] = ref
            self._next_task += 1
        else:
            self._pending.append((fn, value))

    def has_next(self) -> bool:
        return bool(self._index_to_future)

    def has_free(self) -> bool:
        return bool(self._idle) and not self._pending

    def _return_actor(self, seq: int) -> None:
        _, actor = self._future_to_actor.pop(seq)
        self._idle.append(actor)
        if self._pending:
            self.submit(*self._pending.popleft())

    def get_next(self, timeout: Optional[float] = None, ignore_if_timedout: bool = False) -> Any:
        """Next result in submission order."""
        if not self.has_next():
            raise StopIteration("no more results to get")
        seq = self._next_return
        while seq not in self._index_to_future:     # consumed out of order by get_next_unordered
            seq += 1
        ref = self._index_to_future[seq]
        try:
            value = get(ref, timeout=timeout)
        except GetTimeoutError:
            if ignore_if_timedout:
                return None
            raise TimeoutError("timed out waiting for result") from None
        finally:
            if ref._fut.done():
                del self._index_to_future[seq]
                self._next_return = seq + 1
                self._return_actor(seq)
        return value

    def get_next_unordered(self, timeout: Optional[float] = None) -> Any:
        """Whichever result finishes first."""
        if not self.has_next():
            raise StopIteration("no more results to get")
        refs = list(self._index_to_future.values())
        ready, _ = wait(refs, num_returns=1, timeout=timeout)
        if not ready:
            raise TimeoutError("timed out waiting for result")
        seq = next(s for s, r in self._index_to_future.items() if r is ready[0])
        del self._index_to_future[seq]
        self._return_actor(seq)
        return get(ready[0])

    def map(self, fn: Callable[[Any, Any], ObjectRef], values: Iterable[Any]):
        while self.has_next():            # drain earlier work first (Ray semantics)
            self.get_next_unordered()
        for v in values:
            self.submit(fn, v)
        while self.has_next():
            yield self.get_next()

    def map_unordered(self, fn: Callable[[Any, Any], ObjectRef], values: Iterable[Any]):
        while self.has_next():
            self.get_next_unordered()
        for v in values:
            self.submit(fn, v)
        while self.has_next():
            yield self.get_next_unordered()

    def pop_idle(self) -> Optional[Any]:
        return self._idle.pop() if self.has_free() else None

    def push(self, actor: Any) -> None:
        busy = [a for _, a in self._future_to_actor.values()]
        if actor in self._idle or actor in busy:
            raise ValueError("actor already belongs to this pool")
        self._idle.append(actor)
        if self._pending:
            self.submit(*self._pending.popleft())
