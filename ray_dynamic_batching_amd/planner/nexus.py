"""SLO-aware multi-model GPU planner: Nexus "squishy bin packing" (Nexus §6.1).

Reference behaviour: 293-project/src/nexus.py:17-296 (session / node /
scheduleSaturate / scheduleResidue / mergeNodes).  This is a re-implementation
with two modes:

* ``compat=True`` reproduces the reference planner's decisions (SURVEY.md
  Appendix A goldens): batch choice by ``bisect`` over the profile rows (even
  where latencies are not monotonic), SLO/2 for saturated nodes, occupancy-only
  + memory merge test, 11 GB memory cap -- minus its object-aliasing bug (every
  saturated node is a distinct object);
* default mode fixes the reference's gaps: infeasible SLOs are flagged (the
  session is still placed at batch 1 so capacity is reserved, and listed in
  ``plan.infeasible``), a merge must keep every moved session within its SLO
  (``duty + lat(b') <= SLO`` -- the Nexus condition absent in nexus.py:203-229),
  batch sizes missing from the profile use the next profiled batch, zero
  residual rates are skipped, and the memory cap defaults to MI355X's 288 GB.

Profiles: ``{model: {batch: {"avg_latency_ms": ms, "peak_memory_mb": MB}}}`` as
written by profiler/ModelProfiler (CSV contract of ModelProfiler.py:350-366).
"""
from __future__ import annotations

import bisect
import copy
import math
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

Profile = Dict[str, Dict[int, Dict[str, float]]]

MI355X_HBM_GB = 288.0
A6000_COMPAT_GB = 11.0


@dataclass
class Session:
    """A model's serving demand: <model, SLO (ms), request rate (req/s), batch>."""
    model_name: str
    latency_slo: float
    request_rate: float
    batch_size: int = 0
    created: float = field(default_factory=time.time)

    def __post_init__(self):
        if not isinstance(self.model_name, str) or not self.model_name:
            raise ValueError("model name must be a non-empty string")
        if not isinstance(self.latency_slo, (int, float)) or self.latency_slo <= 0:
            raise ValueError("latency SLO must be a positive number (ms)")
        if not isinstance(self.request_rate, (int, float)) or self.request_rate < 0:
            raise ValueError("request rate must be non-negative")
        if not isinstance(self.batch_size, int) or self.batch_size < 0:
            raise ValueError("batch size must be a non-negative integer")

    def to_dict(self) -> dict:
        return dict(model_name=self.model_name, latency_SLO=self.latency_slo, request_rate=self.request_rate,
                    batch_size=self.batch_size)


@dataclass
class Node:
    """One GPU (a bin): sessions with their occupancy of the duty cycle."""
    sessions: List[Tuple[Session, float]] = field(default_factory=list)
    duty_cycle: float = float("inf")      # ms
    gpu_type: str = "MI355X"
    gpu_mem: float = MI355X_HBM_GB

    def occupancy(self) -> float:
        return sum(o for _, o in self.sessions)

    def models(self) -> List[str]:
        return [s.model_name for s, _ in self.sessions]

    def memory_gb(self, profile: Profile) -> float:
        return sum(_row(profile, s.model_name, s.batch_size)["peak_memory_mb"] / 1024.0 for s, _ in self.sessions)

    def describe(self) -> str:
        lines = [f"GPU {self.gpu_type} ({self.gpu_mem:g} GB) duty cycle {self.duty_cycle:.1f} ms, "
                 f"occupancy {self.occupancy() * 100:.1f}%"]
        for s, o in self.sessions:
            lines.append(f"  {s.model_name}: batch {s.batch_size}, rate {s.request_rate:.1f} req/s, "
                         f"occupancy {o * 100:.1f}%, SLO {s.latency_slo:.0f} ms")
        return "\n".join(lines)

    def as_tuples(self) -> List[Tuple[str, int, float, float]]:
        return [(s.model_name, s.batch_size, round(s.request_rate, 1), round(o, 3)) for s, o in self.sessions]


@dataclass
class Plan:
    nodes: List[Node]
    infeasible: List[str] = field(default_factory=list)

    def __iter__(self):
        return iter(self.nodes)

    def __len__(self):
        return len(self.nodes)

    def __getitem__(self, i):
        return self.nodes[i]


def _batches(profile: Profile, model: str) -> List[int]:
    return list(profile[model].keys())  # CSV row order (ascending batch)


def _row(profile: Profile, model: str, b: int) -> Dict[str, float]:
    rows = profile[model]
    if b in rows:
        return rows[b]
    larger = [k for k in rows if k >= b]
    if not larger:
        return rows[max(rows)]
    return rows[min(larger)]


class SquishyPlanner:
    def __init__(self, profile: Profile, gpu_mem_gb: Optional[float] = None, compat: bool = False,
                 gpu_type: str = "MI355X"):
        self.profile = profile
        self.compat = compat
        self.gpu_mem = gpu_mem_gb if gpu_mem_gb is not None else (A6000_COMPAT_GB if compat else MI355X_HBM_GB)
        self.gpu_type = gpu_type

    # ------------------------------------------------------------------ API
    def plan(self, sessions: List[Session]) -> Plan:
        infeasible: List[str] = []
        nodes, residual = self.schedule_saturate(sessions, infeasible)
        nodes.extend(self.schedule_residue(residual, infeasible))
        return Plan(nodes, infeasible)

    # --------------------------------------------------------- saturate step
    def _largest_batch(self, model: str, lat_bound_ms: float) -> Tuple[int, float, bool]:
        """Largest profiled batch with latency <= bound and memory <= cap.
        Returns (batch, latency, feasible)."""
        bs = _batches(self.profile, model)
        lats = [self.profile[model][b]["avg_latency_ms"] for b in bs]
        mems = [self.profile[model][b]["peak_memory_mb"] / 1024.0 for b in bs]
        if self.compat:
            i_lat = bisect.bisect(lats, lat_bound_ms)
            i_mem = bisect.bisect(mems, self.gpu_mem)
            i = min(i_lat, i_mem)
            feasible = i > 0
            i = max(i, 1)
            return bs[i - 1], lats[i - 1], feasible
        best = None
        for b, l, m in zip(bs, lats, mems):
            if l <= lat_bound_ms and m <= self.gpu_mem:
                if best is None or b > best[0]:
                    best = (b, l)
        if best is None:
            return bs[0], lats[0], False
        return best[0], best[1], True

    def schedule_saturate(self, sessions: List[Session], infeasible: List[str]):
        nodes: List[Node] = []
        residual: List[Session] = []
        for s in sessions:
            b, lat, ok = self._largest_batch(s.model_name, s.latency_slo / 2.0)
            if not ok and not self.compat:
                infeasible.append(s.model_name)
            thr = b / lat * 1000.0
            n, r = divmod(s.request_rate, thr)
            for _ in range(int(n)):  # distinct objects (the reference aliases one node n times)
                nodes.append(Node([(Session(s.model_name, s.latency_slo, thr, b), 1.0)], duty_cycle=lat,
                                  gpu_type=self.gpu_type, gpu_mem=self.gpu_mem))
            residual.append(Session(s.model_name, s.latency_slo, r))
        return nodes, residual

    # ---------------------------------------------------------- residue step
    def _residual_node(self, s: Session, infeasible: List[str]) -> Optional[Node]:
        if s.request_rate <= 0:
            return None
        bs = _batches(self.profile, s.model_name)
        lats = [self.profile[s.model_name][b]["avg_latency_ms"] for b in bs]
        worst = [l + b / s.request_rate * 1000.0 for b, l in zip(bs, lats)]
        if self.compat:
            i = max(bisect.bisect(worst, s.latency_slo), 1)
            b, lat = bs[i - 1], lats[i - 1]
        else:
            ok = [(b, l) for b, l, w in zip(bs, lats, worst) if w <= s.latency_slo
                  and self.profile[s.model_name][b]["peak_memory_mb"] / 1024.0 <= self.gpu_mem]
            if ok:
                b, lat = max(ok)
            else:
                b, lat = bs[0], lats[0]
                if s.model_name not in infeasible:
                    infeasible.append(s.model_name)
        duty = b / s.request_rate * 1000.0
        sess = Session(s.model_name, s.latency_slo, s.request_rate, b)
        return Node([(sess, lat / duty)], duty_cycle=duty, gpu_type=self.gpu_type, gpu_mem=self.gpu_mem)

    def merge(self, a: Node, b: Node) -> Optional[Node]:
        """Fold the longer-duty node's sessions into the shorter duty cycle."""
        base, other = (a, b) if a.duty_cycle <= b.duty_cycle else (b, a)
        if self.compat and a.duty_cycle == b.duty_cycle:
            base, other = b, a  # reference keeps node2 as the base on ties
        new = Node([(copy.copy(s), o) for s, o in base.sessions], base.duty_cycle, base.gpu_type, base.gpu_mem)
        d = base.duty_cycle
        for s, _ in other.sessions:
            nb = int(math.ceil(d * s.request_rate / 1000.0))
            nb = max(nb, 1)
            if self.compat and nb not in self.profile[s.model_name]:
                return None  # the reference would raise KeyError here
            lat = _row(self.profile, s.model_name, nb)["avg_latency_ms"]
            if not self.compat and d + lat > s.latency_slo:
                return None  # moved session would miss its SLO
            new.sessions.append((Session(s.model_name, s.latency_slo, s.request_rate, nb), lat / d))
        if new.occupancy() > 1.0:
            return None
        if new.memory_gb(self.profile) > new.gpu_mem:
            return None
        return new

    def schedule_residue(self, sessions: List[Session], infeasible: List[str]) -> List[Node]:
        singles = [n for n in (self._residual_node(s, infeasible) for s in sessions) if n is not None]
        singles.sort(key=lambda n: n.occupancy(), reverse=True)
        nodes: List[Node] = []
        for cand in singles:
            best, best_i, best_occ = None, None, 0.0
            for i, n in enumerate(nodes):
                m = self.merge(n, cand)
                if m is not None and m.occupancy() > best_occ:
                    best, best_i, best_occ = m, i, m.occupancy()
            if best is not None:
                nodes[best_i] = best
            else:
                nodes.append(cand)
        return nodes


# ---------------------------------------------------------------------------
# Plan-to-GPU assignment minimising model moves (reference: the O(n!)
# permutation search of scheduler.py:821-891 -> Hungarian assignment).
# ---------------------------------------------------------------------------
def count_transfers(old_models: List[str], new_models: List[str]) -> int:
    return sum(1 for m in new_models if m not in old_models)


def assign_to_slots(old: List[Optional[Node]], new: List[Node]) -> List[Optional[Node]]:
    """Place the new nodes on GPU slots (old[i] is what slot i runs now) so that
    the number of model loads is minimal.  Returns the per-slot node list
    (length >= len(old); extra nodes go to new slots, freed slots get None)."""
    from scipy.optimize import linear_sum_assignment
    import numpy as np

    n_slots = max(len(old), len(new))
    old_models = [(o.models() if o is not None else []) for o in old] + [[]] * (n_slots - len(old))
    cost = np.zeros((n_slots, n_slots))
    for i in range(n_slots):          # slot
        for j in range(n_slots):      # new node (or an empty placeholder)
            cost[i, j] = count_transfers(old_models[i], new[j].models()) if j < len(new) else 0
    rows, cols = linear_sum_assignment(cost)
    out: List[Optional[Node]] = [None] * n_slots
    for i, j in zip(rows, cols):
        out[i] = new[j] if j < len(new) else None
    return out


def total_transfers(old: List[Optional[Node]], placed: List[Optional[Node]]) -> int:
    t = 0
    for i, n in enumerate(placed):
        if n is None:
            continue
        prev = old[i].models() if i < len(old) and old[i] is not None else []
        t += count_transfers(prev, n.models())
    return t
