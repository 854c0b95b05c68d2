"""``ray.util`` surface of :mod:`ray_dynamic_batching_amd.core`: ``queue``,
``placement_group`` / ``scheduling_strategies``; collectives live in
:mod:`ray_dynamic_batching_amd.parallel.collective`."""
from . import placement_group as _pg_mod  # noqa: F401
from . import queue, scheduling_strategies  # noqa: F401
from .actor_pool import ActorPool  # noqa: F401
from .placement_group import (PlacementGroup, get_placement_group, placement_group,  # noqa: F401
                              placement_group_table, remove_placement_group)
