"""``ray.util.placement_group``: gang reservation of GPU bundles that actors are
then scheduled into.

Reference: ``python/ray/util/placement_group.py:145`` (``placement_group``,
``PlacementGroup.ready/wait``, ``remove_placement_group``,
``placement_group_table``), ``util/scheduling_strategies.py:15,41``
(``PlacementGroupSchedulingStrategy``), SURVEY.md §2.3.  On one MI355X node
the strategies are read per GPU, as the native agent does for Serve's
``placement_group_bundles`` (``GpuAllocator.allocate_bundles``): STRICT_PACK =
all bundles on one GPU, STRICT_SPREAD = one GPU per bundle, PACK / SPREAD =
best effort.  A bundle is ``{"GPU": x, "CPU": y}``; CPU is accounted only as a
label (processes are not CPU-pinned).  An actor created with
``scheduling_strategy=PlacementGroupSchedulingStrategy(pg, i)`` (or the legacy
``placement_group=pg, placement_group_bundle_index=i`` options) takes its
``num_gpus`` out of bundle ``i``'s reservation (``-1``: the first bundle with
room) and is pinned to that bundle's GPUs.
"""
from __future__ import annotations

import threading
import time
import uuid
from concurrent.futures import Future
from typing import Dict, List, Optional

__all__ = ["PlacementGroup", "placement_group", "remove_placement_group", "get_placement_group",
           "placement_group_table"]

_EPS = 1e-9
_groups: Dict[str, "PlacementGroup"] = {}
_lock = threading.Lock()


class PlacementGroup:
    def __init__(self, bundles: List[Dict[str, float]], strategy: str, name: str):
        self.id = uuid.uuid4().hex[:16]
        self.bundle_specs = [dict(b) for b in bundles]
        self.strategy = strategy
        self.name = name
        self.state = "PENDING"
        self._ready: Future = Future()
        self.bundle_gpus: List[List[int]] = [[] for _ in bundles]
        self._used = [0.0] * len(bundles)
        self._members: Dict[str, tuple] = {}

    @property
    def bundle_count(self) -> int:
        return len(self.bundle_specs)

    def ready(self):
        from .. import ObjectRef

        return ObjectRef(self._ready)

    def wait(self, timeout_seconds: float = 30) -> bool:
        try:
            self._ready.result(timeout_seconds)
            return True
        except Exception:
            return False

    # -- actor placement inside the group
    def _take(self, owner: str, num_gpus: float, index: int):
        if self.state != "CREATED":
            if not self.wait(30):
                raise RuntimeError(f"placement group {self.id} is not ready ({self.state})")
        with _lock:
            idxs = [index] if index >= 0 else range(self.bundle_count)
            for i in idxs:
                if i >= self.bundle_count:
                    raise ValueError(f"bundle index {i} out of range ({self.bundle_count} bundles)")
                cap = float(self.bundle_specs[i].get("GPU", 0))
                if self._used[i] + num_gpus <= cap + _EPS:
                    self._used[i] += num_gpus
                    self._members[owner] = (i, num_gpus)
                    return i, list(self.bundle_gpus[i])
        raise ValueError(f"no bundle of placement group {self.id} has {num_gpus} GPU(s) free "
                         f"(bundles {self.bundle_specs}, used {self._used})")

    def _give_back(self, owner: str) -> bool:
        with _lock:
            m = self._members.pop(owner, None)
            if m is None:
                return False
            self._used[m[0]] -= m[1]
            return True

    def __repr__(self):
        return f"PlacementGroup({self.id}, {self.strategy}, {self.bundle_specs}, {self.state})"


def placement_group(bundles: List[Dict[str, float]], strategy: str = "PACK", name: str = "",
                    lifetime: Optional[str] = None, _timeout_s: float = 30.0) -> PlacementGroup:
    """Reserve ``bundles`` all-or-nothing; returns at once, ``ready()`` resolves
    when the reservation is made (it waits for GPUs like a pending Ray PG)."""
    from .. import _require_ctx

    if not bundles or not all(isinstance(b, dict) and b for b in bundles):
        raise ValueError("bundles must be a non-empty list of non-empty dicts")
    for b in bundles:
        if any(v < 0 for v in b.values()):
            raise ValueError("bundle resources must be >= 0")
    if strategy not in ("PACK", "SPREAD", "STRICT_PACK", "STRICT_SPREAD"):
        raise ValueError(f"invalid placement strategy {strategy!r}")
    ctx = _require_ctx()
    pg = PlacementGroup(bundles, strategy, name)
    with _lock:
        if name and any(g.name == name and g.state != "REMOVED" for g in _groups.values()):
            raise ValueError(f"a placement group named {name!r} already exists")
        _groups[pg.id] = pg
    amounts = [float(b.get("GPU", 0)) for b in bundles]

    def settle(state: str, result=None, exc: Optional[BaseException] = None) -> bool:
        # state change + future resolution under _lock, and only while PENDING:
        # remove_placement_group() may have run concurrently (it resolves the
        # future itself and releases only what a CREATED group holds)
        with _lock:
            if pg.state != "PENDING":
                return False
            pg.state = state
            if not pg._ready.done():
                if exc is not None:
                    pg._ready.set_exception(exc)
                else:
                    pg._ready.set_result(result)
            return True

    def reserve():
        deadline = time.monotonic() + _timeout_s
        while pg.state == "PENDING":
            try:
                allocs = ctx.allocator.allocate_bundles("pg:" + pg.id, amounts, strategy)
            except ValueError as e:
                settle("FAILED", exc=e)
                return
            if allocs is not None:
                with _lock:
                    if pg.state == "PENDING":
                        pg.bundle_gpus = [a.gpus for a in allocs]
                committed = settle("CREATED", result=pg)
                if not committed:
                    # removed while allocate_bundles ran: give back what it just took
                    for i in range(len(amounts)):
                        ctx.allocator.release(f"pg:{pg.id}/{i}")
                return
            if time.monotonic() > deadline:
                settle("FAILED", exc=RuntimeError(
                    f"placement group {bundles} ({strategy}) not satisfiable within {_timeout_s:.0f} s "
                    f"(allocator: {ctx.allocator.snapshot()})"))
                return
            time.sleep(0.05)

    threading.Thread(target=reserve, daemon=True, name="rdb-pg-reserve").start()
    return pg


def remove_placement_group(pg: PlacementGroup) -> None:
    """Release the reservation; actors scheduled into the group are killed (Ray semantics)."""
    from .. import _ctx, kill

    with _lock:
        members = list(pg._members)
        prev, pg.state = pg.state, "REMOVED"
        if not pg._ready.done():
            pg._ready.set_exception(RuntimeError("placement group removed"))
    if _ctx is not None:
        for h in list(_ctx.owned):
            if h._actor_id in members:
                try:
                    kill(h)
                except Exception:
                    pass
        if prev == "CREATED":
            for i in range(pg.bundle_count):
                _ctx.allocator.release(f"pg:{pg.id}/{i}")
    if not pg._ready.done():
        pg._ready.set_exception(RuntimeError("placement group removed"))


def get_placement_group(name: str) -> PlacementGroup:
    with _lock:
        for g in _groups.values():
            if g.name == name and g.state != "REMOVED":
                return g
    raise ValueError(f"no placement group named {name!r}")


def placement_group_table(pg: Optional[PlacementGroup] = None) -> Dict:
    def row(g: PlacementGroup):
        return dict(placement_group_id=g.id, name=g.name, strategy=g.strategy, state=g.state,
                    bundles={i: b for i, b in enumerate(g.bundle_specs)},
                    bundles_to_gpus={i: gs for i, gs in enumerate(g.bundle_gpus)})
    if pg is not None:
        return row(pg)
    with _lock:
        return {g.id: row(g) for g in _groups.values()}


def _owner_group(owner: str) -> Optional[PlacementGroup]:
    with _lock:
        for g in _groups.values():
            if owner in g._members:
                return g
    return None
