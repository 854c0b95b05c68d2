"""SLO-aware multi-model scheduler runtime (the fork's NexusScheduler + GPUWorker,
293-project/src/scheduler.py:374-930, re-designed on the shm data plane).

* Per-model request queues: the job segment has one queue per (GPU, model);
  a queue is ACTIVE only on the GPUs the current plan places that model on,
  so the native router's power-of-two choice follows the plan automatically
  (no per-request RPC, no RayQueue actors).
* Executors, one per GPU:
    - ``DutyCycleExecutor`` (Python; CPU tests and arbitrary torch models):
      the fork's duty-cycle loop -- for each (session, occupancy) take up to
      ``batch`` requests, drop stale ones, run, then wait out the time slice
      (scheduler.py:525-588, without its inverted end-of-cycle sleep);
    - the native engine (GPU): same sessions handed to ops/csrc/engine.cpp,
      which serves them EDF/priority-first with stale dropping in C++.
* Monitoring: request rates from RateTrackers; a model triggers re-planning
  when it is new or its rate moved by more than ``rate_change_threshold``
  (2x that threshold for decreases), as in scheduler.py:773-819.  The new
  plan is placed on GPU slots with minimal model moves (Hungarian assignment)
  and applied at batch boundaries (models loaded/unloaded by the executor).
"""
from __future__ import annotations

import collections
import copy
import logging
import math
import threading
import time
import warnings
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import numpy as np

from ..runtime import job as rjob
from .nexus import Node, Plan, Session, SquishyPlanner, assign_to_slots, total_transfers
from .rates import RateTracker

logger = logging.getLogger("ray_dynamic_batching_amd.planner")


@dataclass
class ScheduleChange:
    time: float
    reason: Dict[str, float]
    nodes: List[List[tuple]]
    transfers: int


class DutyCycleExecutor(threading.Thread):
    """One GPU worker (CPU-capable): serves the sessions of its plan node."""

    def __init__(self, sched: "SLOScheduler", gpu: int):
        super().__init__(name=f"executor-{gpu}", daemon=True)
        self.sched = sched
        self.gpu = gpu
        self.node: Optional[Node] = None
        self._new: Optional[Node] = None
        self._lock = threading.Lock()
        self.models: Dict[str, Any] = {}
        self.stop_flag = threading.Event()
        self.stats = dict(processed_batches=0, total_requests=0, dropped=0, processing_ms=[])
        self.consumers: Dict[str, Any] = {}
        self.footprint: Dict[str, int] = {}
        self.loads = 0
        self.unloads = 0
        self.rerouted = 0
        self.failed_on_unload = 0      # leftovers failed because no GPU serves the model any more

    def resident_bytes(self) -> int:
        return sum(self.footprint.get(m, 0) for m in self.models)

    def estimate_bytes(self, m: str) -> int:
        return self.footprint.get(m) or self.sched.footprint_estimate(m)

    def update(self, node: Optional[Node]) -> None:
        with self._lock:
            self._new = node if node is not None else Node([], 1.0)

    def _apply_update(self) -> None:
        with self._lock:
            new, self._new = self._new, None
        if new is None:
            return
        new_models = set(new.models())
        for m in list(self.models):
            if m not in new_models:           # unload (fork: .cpu(); del; empty_cache)
                cons = self.consumers.pop(m, None)
                del self.models[m]
                self.unloads += 1
                if cons is not None:
                    # queued requests follow the model to a GPU that serves it
                    moved = self.sched._reroute_queue(self.sched.queue_id(self.gpu, m), m, cons)
                    if moved >= 0:
                        self.rerouted += moved
                    else:
                        self.failed_on_unload += -moved
        for m in new_models:
            if m not in self.models:          # load
                self.models[m] = self.sched.model_factories[m]()
                self.footprint[m] = model_footprint_bytes(self.models[m])
                self.loads += 1
                q = self.sched.queue_id(self.gpu, m)
                self.consumers[m] = rjob.Consumer(self.sched.job, [q])
        self.node = new

    def run(self) -> None:
        S = self.sched
        while not self.stop_flag.is_set():
            self._apply_update()
            node = self.node
            if node is None or not node.sessions:
                time.sleep(0.01)
                continue
            cycle_start = time.perf_counter()
            for s, occ in node.sessions:
                slice_s = node.duty_cycle * occ / 1000.0
                t0 = time.perf_counter()
                self._serve(s)
                spent = time.perf_counter() - t0
                if spent < slice_s:
                    time.sleep(min(slice_s - spent, 0.25))
                if self.stop_flag.is_set() or self._new is not None:
                    break
            # end of duty cycle: idle out the remainder (the fork's sign-inverted sleep, fixed)
            rem = node.duty_cycle / 1000.0 - (time.perf_counter() - cycle_start)
            if rem > 0 and self._new is None:
                self.stop_flag.wait(min(rem, 0.25))

    def _serve(self, s: Session) -> None:
        S = self.sched
        cons = self.consumers.get(s.model_name)
        model = self.models.get(s.model_name)
        if cons is None or model is None:
            return
        reqs = cons.pop(max(1, s.batch_size), 0)
        if not reqs:
            return
        est_ms = S.latency_ms(s.model_name, len(reqs))
        from ..utils.native import load_runtime

        now = load_runtime().now_ns()
        keep, xs = [], []
        for r in reqs:
            rid, q, client, kind, t_sub, dl, payload = r
            deadline = dl or (t_sub + int(S.slos[s.model_name] * 1e6))
            if S.drop_stale and now + est_ms * 1e6 > deadline:
                cons.complete(client, rid, q, int(rjob.Status.DROPPED_STALE), t_sub, b"", 0)
                self.stats["dropped"] += 1
                continue
            keep.append(r)
            xs.append(np.frombuffer(payload, dtype=S.codecs[s.model_name].in_np).reshape(S.codecs[s.model_name].input_shape))
        if not keep:
            return
        import torch

        t0 = time.perf_counter()
        with torch.no_grad():
            y = model.forward(torch.from_numpy(np.stack(xs)))
        y = y.cpu().numpy()
        dt = (time.perf_counter() - t0) * 1e3
        for r, out in zip(keep, y):
            rid, q, client, kind, t_sub, dl, payload = r
            cons.complete(client, rid, q, 0, t_sub, np.ascontiguousarray(out, dtype=S.codecs[s.model_name].out_np).tobytes(), 0)
        self.stats["processed_batches"] += 1
        self.stats["total_requests"] += len(keep)
        self.stats["processing_ms"] = (self.stats["processing_ms"] + [dt])[-100:]


def model_footprint_bytes(model: Any) -> int:
    """Resident bytes of a model's parameters and buffers (torch modules, or
    objects exposing ``parameters()`` / ``footprint_bytes()``); 0 if unknown."""
    fb = getattr(model, "footprint_bytes", None)
    if callable(fb):
        return int(fb())
    total = 0
    seen = set()
    for attr in ("parameters", "buffers"):
        fn = getattr(model, attr, None)
        if not callable(fn):
            continue
        try:
            for t in fn():
                if id(t) not in seen:
                    seen.add(id(t))
                    total += t.numel() * t.element_size()
        except TypeError:
            pass
    if total == 0 and hasattr(model, "__dict__"):
        import torch

        for v in vars(model).values():
            if isinstance(v, torch.Tensor) and id(v) not in seen:
                seen.add(id(v))
                total += v.numel() * v.element_size()
    return total


class PlanRejected(RuntimeError):
    """A plan whose per-GPU resident model set exceeds the GPU's HBM budget."""


class EngineExecutor:
    """GPU worker on the native replica engine (ops/csrc/engine.cpp) with the
    Nexus duty-cycle policy in C++.  Models are loaded and unloaded as plans
    move them (the fork's ``_check_for_updates``, 293-project/src/scheduler.py:
    483-523: ``.to(device)`` on load, ``.cpu(); del; empty_cache`` on unload):

    * arriving model: weights created on this GPU, graphs captured into private
      pools BESIDE the sessions that keep serving, session registered inactive
      (``prepare``), activated once the router sends its queue traffic
      (``update``);
    * leaving model: its queue is already inactive in the router, so the engine
      drains what is queued, retires the session at a batch boundary (no batch
      in flight), drops graphs + weights and empties the cache: the HBM really
      returns (``resident_bytes`` / ``torch.cuda.memory_allocated`` drop).
      Requests that reached the queue after the drain are re-routed to a GPU
      that serves the model.

    Every load records its measured footprint (allocated bytes across weights +
    capture) and capture time; the scheduler refuses plans whose per-GPU
    resident set would exceed ``hbm_budget_bytes``."""

    def __init__(self, sched: "SLOScheduler", gpu: int, device: int, max_batch: Dict[str, int],
                 compute_streams: int = 1, policy: str = "duty"):
        """``policy``: "duty" (Nexus duty cycle: each session's planned batch per
        cycle within its GPU-time share, work-conserving backfill) or
        "priority" (no cycle: highest priority, then earliest deadline first)."""
        import torch

        from ..runtime.engine import EngineRunner

        self.sched = sched
        self.gpu = gpu
        self.device = device
        self.node: Optional[Node] = None
        self.max_batch = dict(max_batch)
        self.models: Dict[str, Any] = {}
        self.index: Dict[str, int] = {}            # model -> EngineRunner.sessions index (resident)
        self.footprint: Dict[str, int] = {}        # model -> measured resident bytes
        self.capture_s: Dict[str, float] = {}      # model -> last load + capture time
        self.loads = 0
        self.unloads = 0
        self.rerouted = 0
        self.failed_on_unload = 0
        with torch.cuda.device(device):
            if policy not in ("duty", "priority"):
                raise ValueError(f"engine policy must be 'duty' or 'priority', got {policy!r}")
            self.policy = policy
            self.runner = EngineRunner(sched.job_name, gpu, [], pipeline_depth=2, device=device,
                                       policy=(EngineRunner.POLICY_DUTY_CYCLE if policy == "duty"
                                               else EngineRunner.POLICY_PRIORITY_EDF),
                                       compute_streams=compute_streams)
            self.runner.tune_in_context = False
            self.runner.pools = [torch.cuda.graph_pool_handle() for _ in range(self.runner.compute_streams)]
        self.runner.start()

    # ------------------------------------------------------------ memory
    def resident_bytes(self) -> int:
        return sum(self.footprint.get(m, 0) for m in self.index)

    def estimate_bytes(self, m: str) -> int:
        return self.footprint.get(m) or self.sched.footprint_estimate(m)

    # ------------------------------------------------------------ load / unload
    def load(self, m: str) -> None:
        """Load + capture ``m`` (inactive until ``update`` activates it)."""
        import torch

        from ..runtime.engine import SessionSpec

        if m in self.index:
            return
        t0 = time.perf_counter()
        with torch.cuda.device(self.device):
            torch.cuda.synchronize(self.device)
            before = torch.cuda.memory_allocated(self.device)
            model = self.sched.model_factories[m](device=f"cuda:{self.device}")
            spec = SessionSpec(model=model, queue=self.sched.queue_id(self.gpu, m), max_batch=self.max_batch[m],
                               max_wait_s=0.0, slo_ms=float(self.sched.slos[m]), drop_stale=self.sched.drop_stale,
                               name=m)
            idx = self.runner.add_session(spec, activate=False)
            torch.cuda.synchronize(self.device)
            self.footprint[m] = max(1, torch.cuda.memory_allocated(self.device) - before)
        self.models[m] = model
        self.index[m] = idx
        self.capture_s[m] = time.perf_counter() - t0
        self.loads += 1

    def unload(self, m: str, drain_timeout_s: float = 10.0) -> bool:
        """Drain, retire at a batch boundary, free.  False if it could not drain."""
        if m not in self.index:
            return True
        idx = self.index[m]
        sid = self.runner.sessions[idx].sid
        eng = self.runner.engine
        t_end = time.monotonic() + drain_timeout_s
        while time.monotonic() < t_end and (eng.session_pending(sid) > 0 or eng.session_inflight(sid) > 0):
            time.sleep(0.002)
        if not self.runner.retire_session(idx, max(0.1, t_end - time.monotonic())):
            return False
        self.models.pop(m, None)
        del self.index[m]
        self.unloads += 1
        # requests routed here after the drain: hand them to a GPU serving m
        moved = self.sched._reroute_queue(self.sched.queue_id(self.gpu, m), m)
        if moved >= 0:
            self.rerouted += moved
        else:
            self.failed_on_unload += -moved
        return True

    def prepare(self, node: Optional[Node]) -> None:
        """Phase 1 of a plan change (before the router's queues flip): load the
        models arriving on this GPU."""
        for m in (node.models() if node else []):
            if m not in self.index:
                self.load(m)

    def update(self, node: Optional[Node]) -> None:
        """Phase 2 (after the queues flipped): activate the planned sessions with
        their batch sizes and GPU-time shares, unload the models that left."""
        self.node = node
        planned = set(node.models()) if node else set()
        for m in planned:
            if m not in self.index:
                self.load(m)
        shares = {}
        for m in planned:
            sess = [(s, occ) for s, occ in node.sessions if s.model_name == m]
            spec = self.runner.sessions[self.index[m]]
            b = max(1, min(self.max_batch[m], max(s.batch_size for s, _ in sess)))
            self.runner.engine.set_max_batch(spec.sid, b)
            shares[m] = node.duty_cycle * sum(occ for _, occ in sess)
            self.runner.engine.set_duty_share(spec.sid, shares[m])
        self.runner.engine.set_duty_cycle(node.duty_cycle if node else 0.0)
        for m in planned:
            self.runner.engine.set_session_active(self.runner.sessions[self.index[m]].sid, True)
        for m in list(self.index):
            if m not in planned:
                self.unload(m)

    @property
    def stats(self) -> Dict[str, Any]:
        st = dict(self.runner.stats())
        st.update(resident_models=sorted(self.index), resident_bytes=self.resident_bytes(),
                  loads=self.loads, unloads=self.unloads, rerouted=self.rerouted,
                  failed_on_unload=self.failed_on_unload,
                  capture_s=dict(self.capture_s))
        return st

    def stop(self) -> None:
        self.runner.stop()


class SLOScheduler:
    def __init__(self, profiles: Dict[str, Dict[int, Dict[str, float]]], slos_ms: Dict[str, float],
                 model_factories: Dict[str, Callable[[], Any]], codecs: Dict[str, Any], num_gpus: int = 2,
                 monitoring_interval: float = 1.0, rate_change_threshold: float = 0.05, rate_window_s: float = 1.0,
                 compat: bool = False, slo_divisor: float = 1.0, drop_stale: bool = True,
                 gpu_mem_gb: Optional[float] = None, queue_capacity: int = 2048, job_name: Optional[str] = None,
                 executor: str = "python", devices: Optional[List[int]] = None,
                 max_batch: Optional[Dict[str, int]] = None, plan_path: Optional[str] = None,
                 hbm_budget_gb: Optional[float] = None, model_footprint_gb: Optional[Dict[str, float]] = None,
                 compute_streams: int = 1, engine_policy: str = "duty"):
        """``executor``: "python" (DutyCycleExecutor threads; CPU / arbitrary torch
        models) or "engine" (native GPU engines, one per entry of ``devices``;
        ``max_batch`` = largest batch captured per model).  ``plan_path``: every
        applied plan is checkpointed there, and a plan found there at start-up
        is restored (resume after a restart).  ``hbm_budget_gb``: per-GPU bytes
        the resident models may take (default: the node agent's per-GPU HBM
        budget, 288 GB on MI355X); a plan whose per-GPU resident set -- measured
        footprints of loaded models, else ``model_footprint_gb`` estimates, else
        the parameter bytes of a probe instance -- exceeds it is refused and the
        current plan stays (``rejected_plans``); the fork's planner caps the same
        way at packing time (293-project/src/nexus.py:223-227)."""
        self.plan_path = plan_path
        from ..runtime.resources import MI355X_HBM_BYTES as DEFAULT_HBM_BYTES

        # Several engine executors ("GPU slots") on one device: the planner packs
        # whole GPUs, so it must see each slot as 1/k of its device -- its
        # per-batch latencies are planned k times longer (the duty cycles then
        # leave the other slots' share of every cycle idle on this one)
        self.slot_share = 1.0
        if executor == "engine":
            devices = list(devices if devices is not None else range(num_gpus))
            counts = collections.Counter(devices)
            k = max(counts.values())
            if k > 1:
                if len(set(counts.values())) > 1:
                    warnings.warn(f"uneven GPU slots per device {dict(counts)}: planning every slot as 1/{k}")
                self.slot_share = 1.0 / k
                profiles = {m: {b: dict(r, avg_latency_ms=r["avg_latency_ms"] * k) for b, r in p.items()}
                            for m, p in profiles.items()}

        self.hbm_budget_bytes = int((hbm_budget_gb * 1e9) if hbm_budget_gb is not None else DEFAULT_HBM_BYTES)
        self._footprint_hint = {m: int(v * 1e9) for m, v in (model_footprint_gb or {}).items()}
        self.rejected_plans: List[Dict[str, Any]] = []
        self.swapped_first: List[Any] = []      # (gpu, [models]) retired before their arrivals loaded
        self.profiles = profiles
        self.slos = dict(slos_ms)
        self.model_factories = model_factories
        self.codecs = codecs
        self.models = sorted(slos_ms)
        self.num_gpus = num_gpus
        self.monitoring_interval = monitoring_interval
        self.threshold = rate_change_threshold
        self.slo_divisor = slo_divisor
        self.drop_stale = drop_stale
        if gpu_mem_gb is None and hbm_budget_gb is not None:
            gpu_mem_gb = hbm_budget_gb      # the planner packs against the same per-GPU cap
        self.planner = SquishyPlanner(profiles, gpu_mem_gb=gpu_mem_gb, compat=compat)
        self.trackers = {m: RateTracker(rate_window_s) for m in self.models}
        self.sessions: Dict[str, Session] = {}
        self.slots: List[Optional[Node]] = [None] * num_gpus
        self.changes: List[ScheduleChange] = []
        self.unplaced_nodes = 0
        slot_bytes = max(c.in_bytes for c in codecs.values())
        cmp_bytes = max(c.out_bytes for c in codecs.values())
        self.job_name = job_name or rjob.unique_job_name("sched")
        self.job = rjob.Job(self.job_name, create=True, n_replicas=num_gpus, n_queues=num_gpus * len(self.models),
                            n_clients=8, req_capacity=queue_capacity, req_slot_bytes=slot_bytes,
                            cmp_capacity=max(4096, queue_capacity * 2), cmp_slot_bytes=cmp_bytes)
        for g in range(num_gpus):
            self.job.set_replica_status(g, 2, g, 0)
            for m in self.models:
                self.job.configure_queue(self.queue_id(g, m), g, self.model_id(m), 0,
                                         float(self.slos[m]), False)
        self.client = rjob.Client(self.job)
        self._client_lock = threading.Lock()
        self._backlog: List[tuple] = []
        self._backlog_ids = 0
        if executor == "engine":
            devices = list(devices if devices is not None else range(num_gpus))
            mb = {m: (max_batch or {}).get(m, 32) for m in self.models}
            self.executors = [EngineExecutor(self, g, devices[g], mb, compute_streams=compute_streams,
                                             policy=engine_policy) for g in range(num_gpus)]
        else:
            self.executors = [DutyCycleExecutor(self, g) for g in range(num_gpus)]
            for e in self.executors:
                e.start()
        self._monitor: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self.lock = threading.Lock()
        if plan_path:
            saved = self.load_plan(plan_path)
            if saved and self.restore_plan(saved):
                logger.info("restored the last plan from %s", plan_path)

    # --------------------------------------------------------------- ids
    def model_id(self, m: str) -> int:
        return self.models.index(m)

    def queue_id(self, gpu: int, m: str) -> int:
        return gpu * len(self.models) + self.model_id(m)

    def latency_ms(self, model: str, b: int) -> float:
        rows = self.profiles[model]
        ks = [k for k in rows if k >= b]
        return rows[min(ks) if ks else max(rows)]["avg_latency_ms"]

    # ------------------------------------------------------------ ingress
    def submit_request(self, model_name: str, request_id: Any = None, input_tensor=None) -> bool:
        """Fork API (scheduler.py:734-751): enqueue one request; False if dropped."""
        return self.submit(model_name, input_tensor) > 0

    def submit(self, model_name: str, x, deadline_s: float = 0.0) -> int:
        if model_name not in self.trackers:
            return -2
        self.trackers[model_name].record()
        payload = self.codecs[model_name].encode(x)
        with self._client_lock:
            q = self.client.choose_queue(self.model_id(model_name))
            if q == -2:
                # model not placed yet: hold the request until the next plan places it
                rid = self._next_backlog_id()
                self._backlog.append((model_name, payload, deadline_s, rid))
                return rid
            if q < 0:
                q = self._least_loaded_active(model_name)
            return self.client.submit(q, payload, 0, deadline_s)

    def _least_loaded_active(self, model_name: str) -> int:
        qs = [self.queue_id(g, model_name) for g in range(self.num_gpus)
              if self.slots[g] is not None and model_name in self.slots[g].models()]
        return min(qs, key=self.job.queue_depth) if qs else self.queue_id(0, model_name)

    def _next_backlog_id(self) -> int:
        self._backlog_ids += 1
        return 1 << 62 | self._backlog_ids

    def _flush_backlog(self) -> None:
        with self._client_lock:
            keep = []
            for model_name, payload, dl, rid in self._backlog:
                q = self.client.choose_queue(self.model_id(model_name))
                if q == -2:
                    keep.append((model_name, payload, dl, rid))
                    continue
                if q < 0:
                    q = self._least_loaded_active(model_name)
                self.client.submit(q, payload, 0, dl, rid)
            self._backlog = keep

    def poll(self, max_n: int = 1024, timeout_s: float = 0.0):
        # never block while holding the client lock: submitters (ingress threads)
        # would starve behind a waiting poller
        deadline = time.perf_counter() + timeout_s
        while True:
            with self._client_lock:
                out = self.client.poll(max_n, 0)
            if out or time.perf_counter() >= deadline:
                return out
            time.sleep(0.0002)

    # ----------------------------------------------------------- planning
    def start_monitoring(self) -> None:
        if self._monitor is not None:
            return
        self._stop.clear()
        self._monitor = threading.Thread(target=self._monitor_loop, name="rate-monitor", daemon=True)
        self._monitor.start()

    def stop_monitoring(self) -> None:
        self._stop.set()
        if self._monitor is not None:
            self._monitor.join()
            self._monitor = None

    def _monitor_loop(self) -> None:
        while not self._stop.wait(self.monitoring_interval):
            try:
                self.check_and_update()
            except Exception:  # pragma: no cover
                logger.exception("monitor error")

    def check_and_update(self, rates: Optional[Dict[str, float]] = None) -> bool:
        rates = rates or {m: t.rate() for m, t in self.trackers.items()}
        update = {}
        with self.lock:
            for m, r in rates.items():
                if r <= 0:
                    continue
                if m not in self.sessions:
                    update[m] = r
                    continue
                prev = self.sessions[m].request_rate
                diff = r - prev
                thr = self.threshold * (2 if diff < 0 else 1)
                if prev > 0 and abs(diff) / prev > thr:
                    update[m] = r
        if update:
            try:
                self.replan(update)
            except PlanRejected:
                return False        # the current plan stays (rejected_plans records why)
            return True
        return False

    def footprint_estimate(self, m: str) -> int:
        """Resident bytes of model ``m`` on one GPU: measured by an executor that
        loaded it, else the user's hint, else the profile's peak memory (the
        fork's profiler records torch.cuda.max_memory_allocated per batch,
        weights included: 293-project/profiling/ModelProfiler.py:114-178)."""
        for e in self.executors:
            fp = getattr(e, "footprint", {}).get(m)
            if fp:
                return fp
        if m in self._footprint_hint:
            return self._footprint_hint[m]
        rows = self.profiles.get(m, {})
        return int(max((r.get("peak_memory_mb", 0.0) for r in rows.values()), default=0.0) * 2**20)

    def over_budget(self, placed: List[Optional[Node]]) -> Dict[int, Dict[str, Any]]:
        """GPUs whose planned resident set exceeds the HBM budget."""
        out = {}
        for g, node in enumerate(placed):
            if node is None:
                continue
            need = {m: self.footprint_estimate(m) for m in set(node.models())}
            if sum(need.values()) > self.hbm_budget_bytes:
                out[g] = dict(models=need, total=sum(need.values()), budget=self.hbm_budget_bytes)
        return out

    def swap_first(self, placed: List[Optional[Node]]) -> List[int]:
        """GPUs whose plan change would hold the leaving AND the arriving models
        at once above the HBM budget (arrivals are loaded before departures are
        unloaded, so the transition peaks at current + arriving).  _apply
        retires their leaving models first on those GPUs."""
        out = []
        for g, node in enumerate(placed):
            if not hasattr(self.executors[g], "unload"):
                continue        # the Python executor already unloads before it loads
            cur = set(getattr(self.executors[g], "index", {}) or {})
            planned = set(node.models()) if node else set()
            arriving = planned - cur
            if not arriving or not (cur - planned):
                continue
            peak = sum(self.footprint_estimate(m) for m in cur | arriving)
            if peak > self.hbm_budget_bytes:
                out.append(g)
        return out

    def _reroute_queue(self, q: int, m: str, consumer: Any = None) -> int:
        """Move the requests left in queue ``q`` (model ``m`` just left that GPU)
        to the least-loaded GPU queue that serves ``m`` (native
        ``Consumer.forward``: headers kept, completions reach the original
        client).  If no GPU serves ``m`` in the new plan the leftovers are
        failed at once with ST_ERROR ("model unloaded") and the count is
        returned negated (-failed), so callers can tell moved from failed."""
        targets = [self.queue_id(g, m) for g in range(self.num_gpus)
                   if self.queue_id(g, m) != q and self.slots[g] is not None and m in self.slots[g].models()]
        cons = consumer if consumer is not None else rjob.Consumer(self.job, [q])
        if not targets:
            # no GPU serves m any more (it left the plan): fail the leftovers
            # fast instead of leaving their clients to time out on a retired ring
            failed = 0
            while True:
                got = cons.pop(256, 0)
                if not got:
                    return 0 if not failed else -failed
                for rid, queue, client, _kind, t_sub, _dl, _payload in got:
                    cons.complete(client, rid, queue, 2, t_sub, b"model unloaded: no GPU serves it")  # ST_ERROR
                    failed += 1
        to = min(targets, key=self.job.queue_depth)
        return int(cons.forward(to))

    def replan(self, update: Dict[str, float]) -> Plan:
        plan = self._replan_locked(update)
        if self.plan_path:
            self.save_plan(self.plan_path)       # checkpoint every applied plan
        return plan

    def _replan_locked(self, update: Dict[str, float]) -> Plan:
        with self.lock:
            sessions = []
            for m, s in self.sessions.items():
                ns = copy.copy(s)
                if m in update:
                    ns.request_rate = update[m]
                if ns.request_rate > 0:
                    sessions.append(ns)
            for m, r in update.items():
                if m not in self.sessions and r > 0:
                    sessions.append(Session(m, self.slos[m] / self.slo_divisor, r))
            plan = self.planner.plan(sessions)
            nodes = plan.nodes
            if len(nodes) > self.num_gpus:
                # more GPUs needed than the node has: keep the most loaded ones (the fork
                # silently ignored the shortage, scheduler.py:927-929; we count it)
                self.unplaced_nodes = len(nodes) - self.num_gpus
                nodes = sorted(nodes, key=lambda n: n.occupancy(), reverse=True)[: self.num_gpus]
            else:
                self.unplaced_nodes = 0
            placed = assign_to_slots(self.slots, nodes)[: self.num_gpus]
            placed += [None] * (self.num_gpus - len(placed))
            over = self.over_budget(placed)
            if over:
                self.rejected_plans.append(dict(time=time.time(), update=dict(update), over=over))
                logger.warning("plan refused: resident models exceed the HBM budget on GPU(s) %s", over)
                raise PlanRejected(f"plan exceeds the per-GPU HBM budget ({self.hbm_budget_bytes / 1e9:.1f} GB): "
                                   f"{over}")
            transfers = total_transfers(self.slots, placed)
            self.sessions = {s.model_name: s for s in sessions}
            self.slots = placed
            self._apply(placed)
            self._flush_backlog()
            self.changes.append(ScheduleChange(time.time(), dict(update),
                                               [n.as_tuples() if n else [] for n in placed], transfers))
            logger.info("new schedule (%d transfers):\n%s", transfers,
                        "\n".join(n.describe() if n else "(idle)" for n in placed))
            return plan

    def _apply(self, placed: List[Optional[Node]]) -> None:
        # phase 0: on a GPU where old + new models would not fit the HBM budget
        # together, the leaving models are taken off the router, drained and
        # unloaded BEFORE the arrivals load (their requests are forwarded to
        # another GPU serving them, or failed fast if none does)
        for g in self.swap_first(placed):
            ex = self.executors[g]
            planned = set(placed[g].models()) if placed[g] else set()
            leaving = [m for m in list(getattr(ex, "index", {})) if m not in planned]
            for m in leaving:
                self.job.configure_queue(self.queue_id(g, m), g, self.model_id(m), 0, float(self.slos[m]), False)
            for m in leaving:
                if not ex.unload(m):
                    logger.warning("GPU %d: %s did not drain before the swap; the transition may exceed "
                                   "the HBM budget", g, m)
            self.swapped_first.append((g, leaving))
        # phase 1: models arriving on a GPU are loaded + captured (inactive)
        # while every session keeps serving; only then does the router see their
        # queues, so no request waits for a capture
        for g, node in enumerate(placed):
            prep = getattr(self.executors[g], "prepare", None)
            if prep is not None:
                prep(node)
        # phase 2: flip the router's queues, then activate / drain + unload
        for g, node in enumerate(placed):
            models = set(node.models()) if node else set()
            for m in self.models:
                batch = 0
                if node:
                    batch = max((s.batch_size for s, _ in node.sessions if s.model_name == m), default=0)
                self.job.configure_queue(self.queue_id(g, m), g, self.model_id(m), 0, float(self.slos[m]),
                                         m in models)
            self.executors[g].update(node)
        # requests parked on queues that are no longer active stay there until a
        # plan re-activates them; move them forward by re-submitting is unnecessary
        # because every model keeps at least one active queue while its rate > 0.

    # ---------------------------------------------------- checkpoint/resume
    # the reference keeps its plan only in memory (scheduler.py:
    # 894-897); here the last applied plan is a JSON document that the node
    # agent's persistent KV (or a file) holds, and a restarted scheduler
    # re-applies it before the first rate sample arrives.
    def plan_state(self) -> Dict[str, Any]:
        with self.lock:
            def sess(s: Session) -> Dict[str, Any]:
                return dict(model=s.model_name, slo_ms=s.latency_slo, rate=s.request_rate, batch=s.batch_size)

            return dict(version=1, models=list(self.models), num_gpus=self.num_gpus,
                        sessions={m: sess(s) for m, s in self.sessions.items()},
                        slots=[None if n is None else dict(duty_cycle=n.duty_cycle, gpu_type=n.gpu_type,
                                                           gpu_mem=n.gpu_mem,
                                                           sessions=[dict(sess(s), occupancy=o) for s, o in n.sessions])
                               for n in self.slots])

    def save_plan(self, path: Optional[str] = None, agent_socket: Optional[str] = None,
                  key: str = "planner/last_plan") -> str:
        import json

        blob = json.dumps(self.plan_state())
        if path:
            import os

            tmp = path + ".tmp"
            with open(tmp, "w") as f:
                f.write(blob)
            os.replace(tmp, path)
        if agent_socket:
            from ..runtime import agent as ragent

            ragent.request(agent_socket, f"KV_PUT {key} {blob}")
        return blob

    def restore_plan(self, state: Any) -> bool:
        """Re-apply a plan from ``plan_state()`` (dict or JSON text).  Returns False
        when it does not fit this scheduler (different models or GPU count)."""
        import json

        if isinstance(state, (str, bytes)):
            state = json.loads(state)
        if not state or state.get("version") != 1 or state.get("num_gpus") != self.num_gpus:
            return False
        if any(m not in self.slos for m in state["sessions"]):
            return False

        def mk(d: Dict[str, Any]) -> Session:
            return Session(d["model"], float(d["slo_ms"]), float(d["rate"]), int(d["batch"]))

        slots: List[Optional[Node]] = []
        for n in state["slots"]:
            if n is None:
                slots.append(None)
                continue
            slots.append(Node([(mk(s), float(s["occupancy"])) for s in n["sessions"]], float(n["duty_cycle"]),
                              n.get("gpu_type", "MI355X"), float(n.get("gpu_mem", 288.0))))
        if self.over_budget(slots):
            return False
        with self.lock:
            self.sessions = {m: mk(d) for m, d in state["sessions"].items()}
            self.slots = slots
            self._apply(slots)
            self._flush_backlog()
            self.changes.append(ScheduleChange(time.time(), {"restored": 1.0},
                                               [n.as_tuples() if n else [] for n in slots], 0))
        return True

    @staticmethod
    def load_plan(path: Optional[str] = None, agent_socket: Optional[str] = None,
                  key: str = "planner/last_plan") -> Optional[str]:
        if path:
            try:
                with open(path) as f:
                    return f.read()
            except FileNotFoundError:
                return None
        if agent_socket:
            from ..runtime import agent as ragent

            r = ragent.request(agent_socket, f"KV_GET {key}")
            return r[3:] if r.startswith("OK ") else None
        return None

    # ------------------------------------------------------------- metrics
    def get_stats(self) -> Dict[str, Dict[str, Any]]:
        """Per-model stats with the fork's metrics.json keys (scheduler.py:343-372)."""
        out = {}
        for m in self.models:
            tot = dict(total_requests=0, dropped_requests=0, slo_violations=0, queue_size=0, completed=0)
            lat_p = []
            for g in range(self.num_gpus):
                st = self.job.queue_stats(self.queue_id(g, m))
                tot["total_requests"] += st["submitted"]
                tot["dropped_requests"] += st["dropped"]
                tot["slo_violations"] += st["slo_violations"]
                tot["queue_size"] += st["ring_depth"]
                tot["completed"] += st["completed"]
                if st["e2e"]["count"]:
                    lat_p.append(st["e2e"])
            n = sum(h["count"] for h in lat_p)
            tot["avg_latency"] = sum(h["mean_ms"] * h["count"] for h in lat_p) / n if n else 0.0
            tot["p95_latency"] = max((h["p95_ms"] for h in lat_p), default=0.0)
            tot["p99_latency"] = max((h["p99_ms"] for h in lat_p), default=0.0)
            tot["request_rate"] = self.trackers[m].rate()
            tot["slo_ms"] = self.slos[m]
            out[m] = tot
        return out

    def shutdown(self) -> None:
        self.stop_monitoring()
        for e in self.executors:
            if isinstance(e, EngineExecutor):
                e.stop()
            else:
                e.stop_flag.set()
        for e in self.executors:
            if not isinstance(e, EngineExecutor):
                e.join(2)
        self.job.set_shutdown(True)
        self.job.close()
