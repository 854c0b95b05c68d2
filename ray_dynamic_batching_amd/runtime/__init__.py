"""Native data plane: shm job segments, rings, router/clients, replica engine.

See ``csrc/shm.h`` for the segment layout and ``ops/csrc/engine.cpp`` for the
GPU replica engine.
"""
from .job import Job, Client, LoadGen, Consumer, Status, ReplicaStatus, unique_job_name  # noqa: F401
