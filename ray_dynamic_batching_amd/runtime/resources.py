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
        """Gang (all-or-nothing) reservation of placement-group bundles with the
        native agent's algorithm (``GpuAllocator::allocate_bundles`` in
        runtime/csrc/node_agent.cpp; the differential test pins them together):
        bundles in order; a whole-GPU bundle takes free GPUs first-fit; a
        fractional one goes best-fit with this group's GPUs preferred (PACK) or
        avoided (SPREAD); STRICT_PACK keeps every bundle on one GPU, STRICT_SPREAD
        never reuses a GPU of the group.  Bundle ``i`` is held as owner
        ``f"{owner}/{i}"``.  None if the gang does not fit now."""
        unit = 10000
        if strategy not in ("PACK", "SPREAD", "STRICT_PACK", "STRICT_SPREAD"):
            raise ValueError(f"unknown placement strategy {strategy!r}")
        spread = strategy in ("SPREAD", "STRICT_SPREAD")
        with self._lock:
            used = [int(round(sl.used * unit)) for sl in self.slots]
            mine: List[int] = []
            plan = []
            pack_gpu = -1
            for amount in amounts:
                units = int(round(amount * unit))
                if units <= 0:
                    plan.append(([], 0.0))
                    continue
                if units >= unit:
                    if units % unit:
                        raise ValueError("bundle GPU amounts > 1 must be whole numbers")
                    need = units // unit
                    if strategy == "STRICT_PACK" and (len(amounts) > 1 or need > 1):
                        return None
                    got = [g for g in range(len(used)) if used[g] == 0][:need]
                    if len(got) < need:
                        return None
                    for g in got:
                        used[g] = unit
                        if g not in mine:
                            mine.append(g)
                    plan.append((got, 1.0))
                    continue
                best, best_key = -1, None
                for g in range(len(used)):
                    left = unit - used[g] - units
                    if left < 0:
                        continue
                    if strategy == "STRICT_PACK" and pack_gpu >= 0 and g != pack_gpu:
                        continue
                    if strategy == "STRICT_SPREAD" and g in mine:
                        continue
                    pref = (1 if spread else 0) if g in mine else (0 if spread else 1)
                    key = pref * 2 * unit + left
                    if best_key is None or key < best_key:
                        best, best_key = g, key
                if best < 0:
                    return None
                used[best] += units
                if best not in mine:
                    mine.append(best)
                if strategy == "STRICT_PACK":
                    pack_gpu = best
                plan.append(([best], units / unit))
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
