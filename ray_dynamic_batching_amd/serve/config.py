"""Deployment configuration schema, field names kept compatible with Ray Serve
(reference: serve/_private/config.py:81-170 DeploymentConfig, serve/config.py:33-78
AutoscalingConfig, serve/_private/constants.py:107-110 health-check defaults),
plus the Nexus fields of the fork (SLO-aware planning: ``slo_ms``,
``profile_csv``, ``priority``) and the MI355X engine knobs."""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Union

from pydantic import BaseModel, Field, field_validator, model_validator

DEFAULT_MAX_ONGOING_REQUESTS = 5
DEFAULT_HEALTH_CHECK_PERIOD_S = 10.0
DEFAULT_HEALTH_CHECK_TIMEOUT_S = 30.0
DEFAULT_HEALTH_CHECK_FAILURE_THRESHOLD = 3
DEFAULT_GRACEFUL_SHUTDOWN_WAIT_LOOP_S = 2.0
DEFAULT_GRACEFUL_SHUTDOWN_TIMEOUT_S = 20.0
CONTROL_LOOP_INTERVAL_S = 0.1


class AutoscalingConfig(BaseModel):
    """Queue-length autoscaling (serve/config.py:33-78)."""
    min_replicas: int = 1
    initial_replicas: Optional[int] = None
    max_replicas: int = 1
    target_ongoing_requests: float = 2.0
    metrics_interval_s: float = 10.0
    look_back_period_s: float = 30.0
    smoothing_factor: float = 1.0
    upscale_smoothing_factor: Optional[float] = None
    downscale_smoothing_factor: Optional[float] = None
    upscaling_factor: Optional[float] = None
    downscaling_factor: Optional[float] = None
    downscale_delay_s: float = 600.0
    upscale_delay_s: float = 30.0

    @model_validator(mode="after")
    def _check(self):
        if self.min_replicas < 0:
            raise ValueError("min_replicas must be >= 0")
        if self.max_replicas < max(1, self.min_replicas):
            raise ValueError("max_replicas must be >= max(1, min_replicas)")
        if self.initial_replicas is not None and not (self.min_replicas <= self.initial_replicas <= self.max_replicas):
            raise ValueError("initial_replicas must be within [min_replicas, max_replicas]")
        if self.target_ongoing_requests <= 0:
            raise ValueError("target_ongoing_requests must be > 0")
        return self

    def get_upscaling_factor(self) -> float:
        return self.upscaling_factor or self.upscale_smoothing_factor or self.smoothing_factor

    def get_downscaling_factor(self) -> float:
        return self.downscaling_factor or self.downscale_smoothing_factor or self.smoothing_factor


class EngineConfig(BaseModel):
    """MI355X replica-engine knobs for servable (natively executed) models.

    Every knob the headline replica (``bench.py``) runs with travels here, from
    the deployment (decorator options / YAML ``engine:``) to the replica process
    that builds the engine (``serve/replica_main._run_engine``), the way Serve's
    DeploymentConfig carries every replica knob (reference:
    python/ray/serve/_private/config.py:81-170).  Defaults = the benchmarked
    BERT replica: three compute streams, each on its own HIP hardware queue
    (runtime/queues.py), x pipeline depth 6, the shipped MI355X tile table for
    the model's signature, NUMA-pinned process and ring."""
    buckets: Optional[List[int]] = None          # padded batch sizes captured as hipGraphs
    pipeline_depth: int = 6                      # batches in flight (H2D of k+1 under compute of k)
    compute_streams: int = 3                     # batches executing concurrently on the GPU
    batch_policy: str = "timeout"                # "timeout" (@serve.batch semantics) or "idle"
    stagger_us: int = 0                          # hold an idle-starting stream behind the other (latency knob)
    tile_table: str = "auto"                     # "auto" (shipped table for the model signature), "none", or a path
    numa_pin: bool = True                        # node agent pins the replica to its GPU's CPUs, ring mbind-ed there
    warm_s: Optional[float] = None               # device warm-up replays before READY (default 0.25 s)
    zero_copy: bool = True                       # GPU gathers payloads straight from pinned shm
    request_slot_bytes: Optional[int] = None     # per-request payload bytes (default: model input size)

    @model_validator(mode="after")
    def _check(self):
        if self.pipeline_depth < 1:
            raise ValueError("engine.pipeline_depth must be >= 1")
        if self.compute_streams < 1:
            raise ValueError("engine.compute_streams must be >= 1")
        if self.compute_streams > self.pipeline_depth:
            raise ValueError("engine.compute_streams must be <= engine.pipeline_depth (one slot per running batch)")
        if self.batch_policy not in ("timeout", "idle"):
            raise ValueError("engine.batch_policy must be 'timeout' or 'idle'")
        if self.stagger_us < 0:
            raise ValueError("engine.stagger_us must be >= 0")
        if self.buckets is not None and (not self.buckets or any(int(b) < 1 for b in self.buckets)):
            raise ValueError("engine.buckets must be a non-empty list of positive batch sizes")
        return self


class DeploymentConfig(BaseModel):
    name: str = ""
    num_replicas: Union[int, str, None] = 1
    max_ongoing_requests: int = DEFAULT_MAX_ONGOING_REQUESTS
    max_queued_requests: int = -1
    user_config: Optional[Any] = None
    autoscaling_config: Optional[AutoscalingConfig] = None
    graceful_shutdown_wait_loop_s: float = DEFAULT_GRACEFUL_SHUTDOWN_WAIT_LOOP_S
    graceful_shutdown_timeout_s: float = DEFAULT_GRACEFUL_SHUTDOWN_TIMEOUT_S
    health_check_period_s: float = DEFAULT_HEALTH_CHECK_PERIOD_S
    health_check_timeout_s: float = DEFAULT_HEALTH_CHECK_TIMEOUT_S
    health_check_failure_threshold: int = DEFAULT_HEALTH_CHECK_FAILURE_THRESHOLD
    ray_actor_options: Dict[str, Any] = Field(default_factory=dict)
    placement_group_bundles: Optional[List[Dict[str, float]]] = None
    placement_group_strategy: Optional[str] = None
    max_replicas_per_node: Optional[int] = None
    logging_config: Optional[Dict[str, Any]] = None   # serve.logging_utils.LoggingConfig fields
    # Nexus / fork extensions
    slo_ms: Optional[float] = None
    profile_csv: Optional[str] = None
    priority: int = 0
    drop_stale: bool = False
    # router: re-dispatch of a request whose replica died (serve/router.py ShmRouter)
    max_request_retries: int = 3
    request_retry_timeout_s: float = 60.0
    engine: EngineConfig = Field(default_factory=EngineConfig)
    # Tensor-parallel replica: the node agent gang-spawns `tensor_parallel_size`
    # rank processes (one per placement bundle; default: that many bundles of
    # ray_actor_options' num_gpus / hbm each), they rendezvous through the
    # agent's KV, rank 0 serves the replica's queue and the group restarts as one.
    tensor_parallel_size: int = 1
    tp_backend: Optional[str] = None       # "nccl" (= RCCL) / "gloo"; default: nccl when ranks hold GPUs

    @field_validator("logging_config", mode="before")
    @classmethod
    def _logging(cls, v):
        # validated here (bad encoding / level fail at definition time), kept as
        # a plain dict so the config stays JSON-checkpointable
        from .logging_utils import as_logging_config

        c = as_logging_config(v)
        return None if c is None else c.model_dump()

    def get_logging_config(self):
        from .logging_utils import as_logging_config

        return as_logging_config(self.logging_config)

    @field_validator("max_ongoing_requests")
    @classmethod
    def _pos(cls, v):
        if v <= 0:
            raise ValueError("max_ongoing_requests must be > 0")
        return v

    @field_validator("max_queued_requests")
    @classmethod
    def _queued(cls, v):
        if v != -1 and v <= 0:
            raise ValueError("max_queued_requests must be -1 (no limit) or > 0")
        return v

    @model_validator(mode="after")
    def _replicas(self):
        if self.num_replicas == "auto":
            if self.autoscaling_config is None:
                self.autoscaling_config = AutoscalingConfig(min_replicas=1, max_replicas=8, initial_replicas=1)
        elif self.num_replicas is not None:
            if not isinstance(self.num_replicas, int) or self.num_replicas < 0:
                raise ValueError("num_replicas must be a non-negative int or 'auto'")
            if self.autoscaling_config is not None and self.num_replicas not in (None, 1):
                raise ValueError("num_replicas and autoscaling_config cannot both be set")
        g = self.ray_actor_options.get("num_gpus", 0)
        if not isinstance(g, (int, float)) or g < 0:
            raise ValueError("ray_actor_options.num_gpus must be a non-negative number")
        if g > 1 and g != int(g):
            raise ValueError("fractional num_gpus must be < 1")
        # placement groups (serve/api.py:299-303 + deployment_scheduler.py validation)
        if self.placement_group_strategy is not None and self.placement_group_bundles is None:
            raise ValueError("placement_group_strategy needs placement_group_bundles")
        if self.placement_group_bundles is not None:
            b = self.placement_group_bundles
            if not isinstance(b, list) or not b or not all(isinstance(x, dict) and x for x in b):
                raise ValueError("placement_group_bundles must be a non-empty list of non-empty dicts")
            for x in b:
                for k, v in x.items():
                    if not isinstance(v, (int, float)) or v < 0:
                        raise ValueError(f"bundle resource {k} must be a non-negative number")
                gb = float(x.get("GPU", 0))
                if gb > 1 and gb != int(gb):
                    raise ValueError("fractional bundle GPU must be < 1")
            if g > float(b[0].get("GPU", 0)) + 1e-9:
                raise ValueError("the replica (ray_actor_options.num_gpus) must fit in the first bundle")
            st = self.placement_group_strategy or "PACK"
            if st not in ("PACK", "SPREAD", "STRICT_PACK", "STRICT_SPREAD"):
                raise ValueError("placement_group_strategy must be PACK, SPREAD, STRICT_PACK or STRICT_SPREAD")
        if not isinstance(self.tensor_parallel_size, int) or self.tensor_parallel_size < 1:
            raise ValueError("tensor_parallel_size must be an int >= 1")
        if self.tensor_parallel_size > 1 and self.placement_group_bundles is not None \
                and len(self.placement_group_bundles) != self.tensor_parallel_size:
            raise ValueError("a tensor-parallel deployment needs one placement bundle per rank")
        if self.tp_backend is not None and self.tp_backend not in ("nccl", "rccl", "gloo"):
            raise ValueError("tp_backend must be nccl / rccl / gloo")
        if self.max_request_retries < 0 or self.request_retry_timeout_s < 0:
            raise ValueError("max_request_retries / request_retry_timeout_s must be >= 0")
        if self.max_replicas_per_node is not None and not (1 <= self.max_replicas_per_node <= 100):
            raise ValueError("max_replicas_per_node must be in [1, 100]")
        return self

    def initial_num_replicas(self) -> int:
        if self.autoscaling_config is not None:
            a = self.autoscaling_config
            n = a.initial_replicas if a.initial_replicas is not None else a.min_replicas
        else:
            n = int(self.num_replicas or 0)
        return self.cap_replicas(n)

    def cap_replicas(self, n: int) -> int:
        """One node: ``max_replicas_per_node`` caps the whole deployment."""
        return min(n, self.max_replicas_per_node) if self.max_replicas_per_node else n

    def placement_bundles(self):
        """[(num_gpus, hbm_gb), ...] of the placement group, or None."""
        if not self.placement_group_bundles:
            return None
        return [(float(b.get("GPU", 0)), float(b.get("hbm_gb", b.get("memory_gb", 0)) or 0))
                for b in self.placement_group_bundles]

    def tp_bundles(self):
        """[(num_gpus, hbm_gb)] per rank of a tensor-parallel replica."""
        return self.placement_bundles() or [(self.num_gpus, self.hbm_gb)] * self.tensor_parallel_size

    @property
    def num_gpus(self) -> float:
        return float(self.ray_actor_options.get("num_gpus", 0) or 0)

    @property
    def hbm_gb(self) -> float:
        """HBM the replica reserves on its GPU(s) for placement (ray_actor_options
        ``memory_gb`` / ``hbm_gb``; 0 = unconstrained)."""
        o = self.ray_actor_options
        return float(o.get("hbm_gb", o.get("memory_gb", 0)) or 0)
