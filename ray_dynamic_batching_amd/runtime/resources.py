"""GPU slot allocator of the node agent.

Same rule as Ray's unit-instance GPU resource
(src/ray/common/scheduling/resource_instance_set.cc:93-187): a demand >= 1
takes whole free GPUs first-fit; a fractional demand goes BEST-FIT to the GPU
with the least remaining capacity that still fits (that is how num_gpus=0.5
co-locates two replicas on one GPU).  Extended with an HBM budget per GPU
(288 GB on MI355X) so planner-packed models are also checked for memory.
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional

MI355X_HBM_BYTES = 288 * 10**9
_EPS = 1e-9


@dataclass
class GpuSlot:
    index: int
    capacity: float = 1.0
    hbm_total: int = MI355X_HBM_BYTES
    used: float = 0.0
    hbm_used: int = 0
    holders: Dict[str, float] = field(default_factory=dict)

    @property
    def free(self) -> float:
        return self.capacity - self.used


@dataclass
class Allocation:
    owner: str
    gpus: List[int]
    fraction: float
    hbm_bytes: int


class GpuAllocator:
    def __init__(self, num_gpus: Optional[int] = None, hbm_bytes: int = MI355X_HBM_BYTES):
        if num_gpus is None:
            num_gpus = detect_num_gpus()
        self.slots = [GpuSlot(i, hbm_total=hbm_bytes) for i in range(num_gpus)]
        self.allocs: Dict[str, Allocation] = {}
        self._lock = threading.Lock()

    def allocate(self, owner: str, num_gpus: float, hbm_bytes: int = 0) -> Optional[Allocation]:
        """Returns None if the demand cannot be met right now."""
        if num_gpus <= 0:
            a = Allocation(owner, [], 0.0, 0)
            self.allocs[owner] = a
            return a
        with self._lock:
            if owner in self.allocs:
                raise ValueError(f"{owner} already holds GPUs")
            if num_gpus >= 1:
                if abs(num_gpus - round(num_gpus)) > _EPS:
                    raise ValueError("num_gpus > 1 must be an integer")
                need = int(round(num_gpus))
                free = [s for s in self.slots if s.used <= _EPS and s.hbm_total - s.hbm_used >= hbm_bytes // need]
                if len(free) < need:
                    return None
                chosen = free[:need]
                for s in chosen:
                    s.used = s.capacity
                    s.hbm_used += hbm_bytes // need
                    s.holders[owner] = s.capacity
                a = Allocation(owner, [s.index for s in chosen], 1.0, hbm_bytes)
            else:
                fits = [s for s in self.slots if s.free + _EPS >= num_gpus and s.hbm_total - s.hbm_used >= hbm_bytes]
                if not fits:
                    return None
                best = min(fits, key=lambda s: (s.free - num_gpus, s.index))
                best.used += num_gpus
                best.hbm_used += hbm_bytes
                best.holders[owner] = num_gpus
                a = Allocation(owner, [best.index], num_gpus, hbm_bytes)
            self.allocs[owner] = a
            return a

    def allocate_bundles(self, owner: str, amounts: List[float], strategy: str = "PACK") -> Optional[List[Allocation]]:
        """Gang (all-or-nothing) reservation of placement-group bundles, the
        same per-GPU reading of the strategies as the native agent's
        ``allocate_bundles`` (node_agent.cpp): STRICT_PACK = every bundle on one
        GPU, STRICT_SPREAD = each bundle on its own GPU(s), PACK / SPREAD = try
        the strict form, else place bundles one by one (best fit).  Bundle ``i``
        is held as owner ``f"{owner}/{i}"``.  None if it does not fit now."""
        if strategy not in ("PACK", "SPREAD", "STRICT_PACK", "STRICT_SPREAD"):
            raise ValueError(f"unknown placement strategy {strategy!r}")
        for a in amounts:
            if a < 0 or (a > 1 and abs(a - round(a)) > _EPS):
                raise ValueError("bundle GPU amounts must be fractions <= 1 or whole numbers")
        with self._lock:
            free = [s.free for s in self.slots]
            plan = None
            if strategy in ("STRICT_PACK", "PACK"):
                plan = self._plan_pack(amounts, free)
            elif strategy in ("STRICT_SPREAD", "SPREAD"):
                plan = self._plan_spread(amounts, free)
            if plan is None and strategy in ("PACK", "SPREAD"):
                plan = self._plan_each(amounts, free)
            if plan is None:
                return None
            out = []
            for i, (gpus, per) in enumerate(plan):
                name = f"{owner}/{i}"
                for g in gpus:
                    self.slots[g].used += per
                    self.slots[g].holders[name] = per
                a = Allocation(name, gpus, per if gpus else 0.0, 0)
                self.allocs[name] = a
                out.append(a)
            return out

    @staticmethod
    def _plan_pack(amounts, free):
        total = sum(amounts)
        if total <= _EPS:
            return [([], 0.0) for _ in amounts]
        if total > 1 + _EPS:
            return None                     # one GPU holds at most 1.0
        fits = [g for g, f in enumerate(free) if f + _EPS >= total]
        if not fits:
            return None
        g = min(fits, key=lambda i: (free[i] - total, i))
        return [([g], a) if a > 0 else ([], 0.0) for a in amounts]

    @staticmethod
    def _plan_spread(amounts, free):
        free, taken, plan = list(free), set(), [None] * len(amounts)
        for i in sorted(range(len(amounts)), key=lambda j: -amounts[j]):
            a = amounts[i]
            if a <= _EPS:
                plan[i] = ([], 0.0)
                continue
            need = int(round(a)) if a >= 1 else 1
            per = 1.0 if a >= 1 else a
            cand = sorted((g for g, f in enumerate(free) if g not in taken and f + _EPS >= per),
                          key=lambda g: (free[g] - per, g))
            if len(cand) < need:
                return None
            gs = cand[:need]
            for g in gs:
                free[g] -= per
                taken.add(g)
            plan[i] = (gs, per)
        return plan

    @staticmethod
    def _plan_each(amounts, free):
        free, plan = list(free), []
        for a in amounts:
            if a <= _EPS:
                plan.append(([], 0.0))
                continue
            if a >= 1:
                gs = [g for g, f in enumerate(free) if f >= 1 - _EPS][:int(round(a))]
                if len(gs) < int(round(a)):
                    return None
                for g in gs:
                    free[g] = 0.0
                plan.append((gs, 1.0))
            else:
                fits = [g for g, f in enumerate(free) if f + _EPS >= a]
                if not fits:
                    return None
                g = min(fits, key=lambda i: (free[i] - a, i))
                free[g] -= a
                plan.append(([g], a))
        return plan

    def release(self, owner: str) -> None:
        with self._lock:
            a = self.allocs.pop(owner, None)
            if a is None:
                return
            for g in a.gpus:
                s = self.slots[g]
                s.used = max(0.0, s.used - s.holders.pop(owner, 0.0))
                s.hbm_used = max(0, s.hbm_used - (a.hbm_bytes // max(1, len(a.gpus)) if a.fraction >= 1 else a.hbm_bytes))

    def snapshot(self) -> List[dict]:
        with self._lock:
            return [dict(gpu=s.index, used=round(s.used, 4), free=round(s.free, 4), hbm_used=s.hbm_used,
                         holders=dict(s.holders)) for s in self.slots]


def detect_num_gpus() -> int:
    env = os.environ.get("RDB_NUM_GPUS")
    if env is not None:
        return int(env)
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


def visible_devices_env(gpus: List[int]) -> Dict[str, str]:
    """Environment that pins a replica process to its GPUs (reference:
    _private/accelerators/amd_gpu.py:99-107 sets ROCR_VISIBLE_DEVICES).  The
    native node agent (runtime/csrc/node_agent.cpp) owns the live allocator;
    the Python GpuAllocator above is the reference model its tests pin."""
    # Only HIP_VISIBLE_DEVICES: it indexes the devices ROCR already exposes, so an
    # inherited ROCR_VISIBLE_DEVICES (e.g. from a cluster scheduler) keeps working.
    v = ",".join(str(g) for g in gpus)
    return {"HIP_VISIBLE_DEVICES": v} if gpus else {"HIP_VISIBLE_DEVICES": "", "RDB_NO_GPU": "1"}
