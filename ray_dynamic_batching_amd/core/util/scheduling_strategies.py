"""``ray.util.scheduling_strategies`` (reference ``util/scheduling_strategies.py:15,41,135``).

Single node: ``NodeAffinitySchedulingStrategy`` to this node (``core.get_runtime_context().get_node_id()``
or an entry of ``core.nodes()``) schedules normally; to any other node id it fails the submission with
``TaskUnschedulableError`` unless ``soft=True``, which falls back to this node as Ray does when the
target is unavailable.  The string strategies ``"DEFAULT"`` and ``"SPREAD"`` are accepted (one node:
both place locally)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any

__all__ = ["PlacementGroupSchedulingStrategy", "NodeAffinitySchedulingStrategy"]


@dataclass
class PlacementGroupSchedulingStrategy:
    placement_group: Any
    placement_group_bundle_index: int = -1
    placement_group_capture_child_tasks: bool = False


@dataclass
class NodeAffinitySchedulingStrategy:
    node_id: str
    soft: bool
    _spill_on_unavailable: bool = False
    _fail_on_unavailable: bool = False
