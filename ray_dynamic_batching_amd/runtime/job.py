"""Thin Python layer over the native job segment (``_rdb_runtime``)."""
from __future__ import annotations

import enum
import os
import uuid

from ..utils.native import load_runtime


class Status(enum.IntEnum):
    OK = 0
    DROPPED_STALE = 1
    ERROR = 2
    REJECTED = 3
    TOO_LARGE = 4
    SHUTDOWN = 5
    REPLICA_DIED = 6


class ReplicaStatus(enum.IntEnum):
    UNUSED = 0
    STARTING = 1
    READY = 2
    DRAINING = 3
    DEAD = 4


def unique_job_name(prefix: str = "job") -> str:
    return f"{prefix}_{os.getpid()}_{uuid.uuid4().hex[:8]}"


def Job(name: str, create: bool = False, **kw):
    """Create (create=True) or attach to a job segment.  kwargs: n_replicas,
    n_queues, n_clients, req_capacity, req_slot_bytes, cmp_capacity,
    cmp_slot_bytes, attach_timeout_s."""
    return load_runtime().Job(name, create, **kw)


def Client(job, client_id: int = -1, seed: int = 0):
    return load_runtime().Client(job, client_id, seed)


def LoadGen(client, model: int, payloads):
    return load_runtime().LoadGen(client, model, list(payloads))


def Consumer(job, queues):
    return load_runtime().Consumer(job, list(queues))


def EchoServer(job, replica: int, queues, max_batch: int = 32, service_us: float = 0.0, per_item_us: float = 0.0,
               out_bytes: int = 8):
    """Native fake replica (C++ threads): batches up to ``max_batch`` requests per
    queue, busy-waits ``service_us + per_item_us*B`` and echoes ``out_bytes``."""
    return load_runtime().EchoServer(job, replica, list(queues), max_batch, service_us, per_item_us, out_bytes)
