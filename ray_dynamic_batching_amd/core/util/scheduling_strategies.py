"""``ray.util.scheduling_strategies`` (reference ``util/scheduling_strategies.py:15,41``)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any

__all__ = ["PlacementGroupSchedulingStrategy"]


@dataclass
class PlacementGroupSchedulingStrategy:
    placement_group: Any
    placement_group_bundle_index: int = -1
    placement_group_capture_child_tasks: bool = False
