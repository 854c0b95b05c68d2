"""``ray.util.queue.Queue`` (reference: ``python/ray/util/queue.py:20-305``): a
FIFO hosted by an actor, so a queue handle can be passed to other actors and
every operation is a call on that actor -- the structure the fork's request
queues use (``293-project/src/scheduler.py:194`` ``RayQueue(maxsize=...)``).

Blocking ``put`` / ``get`` block inside the queue actor (on one of its
``max_concurrency`` threads), with Ray's ``block`` / ``timeout`` semantics and
``Empty`` / ``Full`` errors; ``put_nowait_batch`` / ``get_nowait_batch`` are
all-or-nothing.  (The framework's own request path uses the native shm rings,
``runtime/csrc/shm.h``, not this.)
"""
from __future__ import annotations

import queue as _q
import threading
from typing import Any, Iterable, List, Optional


class Empty(_q.Empty):
    pass


class Full(_q.Full):
    pass


class _QueueActor:
    def __init__(self, maxsize: int):
        self.maxsize = maxsize
        self.items: List[Any] = []
        self.cv = threading.Condition()

    def _full(self) -> bool:
        return self.maxsize > 0 and len(self.items) >= self.maxsize

    def qsize(self) -> int:
        with self.cv:
            return len(self.items)

    def empty(self) -> bool:
        return self.qsize() == 0

    def full(self) -> bool:
        with self.cv:
            return self._full()

    def put(self, item, block: bool = True, timeout: Optional[float] = None) -> None:
        with self.cv:
            if not block:
                if self._full():
                    raise Full
            elif not self.cv.wait_for(lambda: not self._full(), timeout):
                raise Full
            self.items.append(item)
            self.cv.notify_all()

    def get(self, block: bool = True, timeout: Optional[float] = None):
        with self.cv:
            if not block:
                if not self.items:
                    raise Empty
            elif not self.cv.wait_for(lambda: bool(self.items), timeout):
                raise Empty
            item = self.items.pop(0)
            self.cv.notify_all()
            return item

    def put_nowait_batch(self, items: List[Any]) -> None:
        with self.cv:
            if self.maxsize > 0 and len(self.items) + len(items) > self.maxsize:
                raise Full(f"cannot add {len(items)} items to a queue of size {len(self.items)} "
                           f"and maxsize {self.maxsize}")
            self.items.extend(items)
            self.cv.notify_all()

    def get_nowait_batch(self, num_items: int) -> List[Any]:
        with self.cv:
            if num_items > len(self.items):
                raise Empty(f"cannot get {num_items} items from a queue of size {len(self.items)}")
            out, self.items = self.items[:num_items], self.items[num_items:]
            self.cv.notify_all()
            return out


def _unwrap(fn, *a, **kw):
    from .. import RayTaskError, get

    try:
        return get(fn.remote(*a, **kw))
    except RayTaskError as e:
        if isinstance(e.cause, (_q.Empty, _q.Full)):
            raise (Empty if isinstance(e.cause, _q.Empty) else Full)(str(e.cause)) from None
        raise


class Queue:
    def __init__(self, maxsize: int = 0, actor_options: Optional[dict] = None, _actor=None):
        from .. import remote

        self.maxsize = maxsize
        if _actor is not None:
            self.actor = _actor
        else:
            opts = dict(actor_options or {})
            opts.setdefault("max_concurrency", 128)   # blocked put/get hold one thread each
            self.actor = remote(_QueueActor).options(**opts).remote(maxsize)

    def __reduce__(self):
        return (Queue, (self.maxsize, None, self.actor))

    def __len__(self) -> int:
        return self.size()

    def size(self) -> int:
        return _unwrap(self.actor.qsize)

    qsize = size

    def empty(self) -> bool:
        return _unwrap(self.actor.empty)

    def full(self) -> bool:
        return _unwrap(self.actor.full)

    def put(self, item: Any, block: bool = True, timeout: Optional[float] = None) -> None:
        if timeout is not None and timeout < 0:
            raise ValueError("'timeout' must be a non-negative number")
        _unwrap(self.actor.put, item, block, timeout)

    def get(self, block: bool = True, timeout: Optional[float] = None) -> Any:
        if timeout is not None and timeout < 0:
            raise ValueError("'timeout' must be a non-negative number")
        return _unwrap(self.actor.get, block, timeout)

    def put_nowait(self, item: Any) -> None:
        self.put(item, block=False)

    def get_nowait(self) -> Any:
        return self.get(block=False)

    def put_nowait_batch(self, items: Iterable) -> None:
        if not isinstance(items, list):
            raise TypeError("Argument 'items' must be a list")
        _unwrap(self.actor.put_nowait_batch, items)

    def get_nowait_batch(self, num_items: int) -> List[Any]:
        if not isinstance(num_items, int) or num_items < 0:
            raise ValueError("'num_items' must be a nonnegative integer")
        return _unwrap(self.actor.get_nowait_batch, num_items)

    def shutdown(self, force: bool = False, grace_period_s: int = 5) -> None:
        from .. import kill

        if self.actor is not None:
            kill(self.actor)
        self.actor = None
