"""Replica context (reference: serve/context.py, get_replica_context)."""
from __future__ import annotations

import contextvars
import threading
from dataclasses import dataclass
from typing import Optional


@dataclass
class ReplicaContext:
    app_name: str
    deployment: str
    replica_id: str
    replica_index: int
    servable_object: object = None
    max_ongoing_requests: Optional[int] = None
    gpu: Optional[int] = None
    logger: object = None           # the replica's component logger (serve.logging_utils)


_local = threading.local()
_request_ctx: contextvars.ContextVar = contextvars.ContextVar("rdb_request_ctx", default=None)


def _set_replica_context(ctx: Optional[ReplicaContext]) -> None:
    _local.ctx = ctx


def get_replica_context_or_none() -> Optional[ReplicaContext]:
    return getattr(_local, "ctx", None)


def get_replica_context() -> ReplicaContext:
    ctx = get_replica_context_or_none()
    if ctx is None:
        from .exceptions import RayServeException

        raise RayServeException("get_replica_context() may only be called from within a replica")
    return ctx


@dataclass
class RequestContext:
    request_id: int = 0
    multiplexed_model_id: str = ""
    method_name: str = "__call__"


def _set_request_context(ctx: RequestContext):
    return _request_ctx.set(ctx)


def get_request_context() -> RequestContext:
    return _request_ctx.get() or RequestContext()
