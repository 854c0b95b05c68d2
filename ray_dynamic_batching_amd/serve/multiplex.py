"""Model multiplexing (reference: serve/multiplex.py:22-258).

``@serve.multiplexed(max_num_models_per_replica=N)`` on an async
``get_model(model_id)`` method turns it into a per-replica LRU cache: a model
is loaded on first use and the least recently used one is evicted (its
``__del__`` runs) when more than N are resident.  ``get_multiplexed_model_id()``
returns the id the caller set with ``handle.options(multiplexed_model_id=...)``;
the router prefers replicas that already hold that model.
"""
from __future__ import annotations

import asyncio
import collections
import functools
import inspect
from typing import Callable, Optional

from .context import get_request_context


def get_multiplexed_model_id() -> str:
    return get_request_context().multiplexed_model_id


# Replica-side publication of the loaded model ids (process mode: the replica
# sets a publisher that writes their hashes into its queue's shm slots, where
# the native router's choose_queue looks for them).
_caches: "list" = []
_publisher: Optional[Callable] = None


def set_publisher(fn: Optional[Callable]) -> None:
    global _publisher
    _publisher = fn
    _publish()


def loaded_model_ids() -> list:
    out = []
    for c in _caches:
        for m in c.models:
            if m not in out:
                out.append(m)
    return out


def _publish() -> None:
    if _publisher is not None:
        try:
            _publisher(loaded_model_ids())
        except Exception:  # pragma: no cover - routing hint only
            pass


class _ModelCache:
    def __init__(self, loader: Callable, max_models: int):
        self.loader = loader
        self.max_models = max_models
        self.models: "collections.OrderedDict[str, object]" = collections.OrderedDict()
        self.loading: dict = {}
        self.num_loads = 0
        self.num_evictions = 0
        _caches.append(self)

    async def get(self, owner, model_id: str):
        if model_id in self.models:
            self.models.move_to_end(model_id)
            return self.models[model_id]
        if model_id in self.loading:
            return await self.loading[model_id]
        fut = asyncio.get_running_loop().create_future()
        self.loading[model_id] = fut
        try:
            while len(self.models) >= self.max_models:
                _, old = self.models.popitem(last=False)
                self.num_evictions += 1
                _publish()
                d = getattr(old, "__del__", None)
                if d is not None:
                    try:
                        d()
                    except Exception:
                        pass
            r = self.loader(owner, model_id) if owner is not None else self.loader(model_id)
            if inspect.isawaitable(r):
                r = await r
            self.models[model_id] = r
            self.num_loads += 1
            _publish()
            fut.set_result(r)
            return r
        except Exception as e:
            fut.set_exception(e)
            raise
        finally:
            self.loading.pop(model_id, None)


def multiplexed(func: Optional[Callable] = None, max_num_models_per_replica: int = 3):
    if max_num_models_per_replica != -1 and max_num_models_per_replica < 1:
        raise ValueError("max_num_models_per_replica must be positive or -1")

    def deco(fn):
        if not inspect.iscoroutinefunction(fn):
            raise TypeError("@serve.multiplexed functions must be 'async def'")
        is_method = list(inspect.signature(fn).parameters)[:1] == ["self"]
        cap = max_num_models_per_replica if max_num_models_per_replica != -1 else 1 << 30

        @functools.wraps(fn)
        async def wrapper(*args):
            if is_method:
                owner, model_id = args[0], (args[1] if len(args) > 1 else get_multiplexed_model_id())
                cache = owner.__dict__.get("_rdb_model_cache_" + fn.__name__)
                if cache is None:
                    cache = _ModelCache(fn, cap)
                    owner.__dict__["_rdb_model_cache_" + fn.__name__] = cache
            else:
                owner, model_id = None, (args[0] if args else get_multiplexed_model_id())
                cache = wrapper.__dict__.setdefault("_cache", _ModelCache(fn, cap))
            if not isinstance(model_id, str) or not model_id:
                raise ValueError("a non-empty model id string is required")
            return await cache.get(owner, model_id)
        return wrapper

    return deco(func) if func is not None else deco
