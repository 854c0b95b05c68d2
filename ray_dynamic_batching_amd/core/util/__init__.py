"""``ray.util`` surface of :mod:`ray_dynamic_batching_amd.core`: ``queue``;
collectives live in :mod:`ray_dynamic_batching_amd.parallel.collective`."""
from . import queue  # noqa: F401
