"""Public Serve-compatible API: ``@serve.deployment``, ``Deployment.bind``,
``serve.run`` and friends (reference: python/ray/serve/api.py:240-514,
serve/deployment.py).

Execution model (MI355X-native):
* ``serve.run`` hands the application graph to the in-process controller
  (controller.py), which starts the replicas:
    - ``local`` mode: replicas are in-process objects, each on its own
      user-code event-loop thread (Serve's ``_local_testing_mode`` / Ray's
      ``local_mode`` plumbing, BASELINE config 1);
    - ``process`` mode (default when a deployment asks for GPUs): one replica
      process per GPU slot, pinned with ``HIP_VISIBLE_DEVICES``; requests and
      results travel through the shared-memory job segment (no RPC).
* A deployment whose class is a *servable model* (``__rdb_servable__ = True``,
  see models/servable.py) is executed by the native replica engine: batching,
  H2D, hipGraph replay and completion all happen in C++.
"""
from __future__ import annotations

import inspect
from typing import Any, Callable, Dict, List, Optional, Union

from .config import AutoscalingConfig, DeploymentConfig, EngineConfig


class Deployment:
    """A deployment definition (a class or function plus its config)."""

    def __init__(self, func_or_class: Union[Callable, type], config: DeploymentConfig, name: str):
        self.func_or_class = func_or_class
        self.config = config
        self._name = name

    @property
    def name(self) -> str:
        return self._name

    @property
    def num_replicas(self):
        return self.config.num_replicas

    @property
    def max_ongoing_requests(self) -> int:
        return self.config.max_ongoing_requests

    @property
    def user_config(self):
        return self.config.user_config

    @property
    def ray_actor_options(self) -> Dict[str, Any]:
        return self.config.ray_actor_options

    def options(self, **kw) -> "Deployment":
        """Return a copy with some config fields overridden (Deployment.options)."""
        name = kw.pop("name", self._name)
        func = kw.pop("func_or_class", self.func_or_class)
        data = self.config.model_dump()
        for k, v in kw.items():
            if k not in DeploymentConfig.model_fields:
                raise TypeError(f"unknown deployment option {k!r}")
            if isinstance(v, (AutoscalingConfig, EngineConfig)):
                v = v.model_dump()
            elif k == "engine" and isinstance(v, dict):
                # partial engine overrides (YAML `engine: {compute_streams: 1}`) keep
                # the other engine fields (model_deployment's slot size, buckets, ...)
                v = {**(data.get("engine") or {}), **v}
            data[k] = v
        if "num_replicas" in kw and kw["num_replicas"] != "auto" and "autoscaling_config" not in kw:
            data["autoscaling_config"] = None
        data["name"] = name
        d = Deployment(func, DeploymentConfig(**data), name)
        if hasattr(self, "servable"):
            d.servable = self.servable
        return d

    def _with_config(self, config: DeploymentConfig) -> "Deployment":
        """Copy with a whole config replaced (controller recovery)."""
        d = Deployment(self.func_or_class, config, self._name)
        if hasattr(self, "servable"):
            d.servable = self.servable
        return d

    def bind(self, *args, **kwargs) -> "Application":
        return Application(self, args, kwargs)

    def __call__(self, *a, **k):
        raise RuntimeError("Deployments cannot be constructed directly; use .bind() and serve.run()")

    def __repr__(self) -> str:
        return f"Deployment(name={self._name!r}, num_replicas={self.config.num_replicas})"


class Application:
    """A bound deployment: the root of an application graph.  Init args may
    themselves be Applications; they become DeploymentHandles in the replica
    (model composition)."""

    def __init__(self, deployment: Deployment, init_args: tuple, init_kwargs: dict):
        self.deployment = deployment
        self.init_args = init_args
        self.init_kwargs = init_kwargs

    def walk(self) -> List["Application"]:
        """All applications in the graph, dependencies first."""
        seen: List[Application] = []

        def visit(a: "Application"):
            for x in list(a.init_args) + list(a.init_kwargs.values()):
                if isinstance(x, Application):
                    visit(x)
            if all(a is not s for s in seen):
                seen.append(a)

        visit(self)
        return seen


_DEPLOYMENT_FIELDS = set(DeploymentConfig.model_fields) - {"name", "engine"}


def deployment(_func_or_class: Optional[Union[Callable, type]] = None, *, name: Optional[str] = None,
               num_replicas: Union[int, str, None] = None, ray_actor_options: Optional[Dict] = None,
               placement_group_bundles=None, placement_group_strategy=None, max_replicas_per_node=None,
               user_config=None, max_ongoing_requests: Optional[int] = None, max_queued_requests: Optional[int] = None,
               autoscaling_config: Union[Dict, AutoscalingConfig, None] = None,
               graceful_shutdown_wait_loop_s: Optional[float] = None, graceful_shutdown_timeout_s: Optional[float] = None,
               health_check_period_s: Optional[float] = None, health_check_timeout_s: Optional[float] = None,
               logging_config=None, slo_ms: Optional[float] = None, profile_csv: Optional[str] = None,
               priority: Optional[int] = None, drop_stale: Optional[bool] = None,
               max_request_retries: Optional[int] = None, request_retry_timeout_s: Optional[float] = None,
               engine: Union[Dict, EngineConfig, None] = None, tensor_parallel_size: Optional[int] = None,
               tp_backend: Optional[str] = None):
    """Decorator turning a class or function into a Deployment
    (signature of serve/api.py:240-259 plus the Nexus SLO fields)."""
    given = {k: v for k, v in dict(
        num_replicas=num_replicas, ray_actor_options=ray_actor_options,
        placement_group_bundles=placement_group_bundles, placement_group_strategy=placement_group_strategy,
        max_replicas_per_node=max_replicas_per_node, user_config=user_config,
        max_ongoing_requests=max_ongoing_requests, max_queued_requests=max_queued_requests,
        autoscaling_config=autoscaling_config, graceful_shutdown_wait_loop_s=graceful_shutdown_wait_loop_s,
        graceful_shutdown_timeout_s=graceful_shutdown_timeout_s, health_check_period_s=health_check_period_s,
        health_check_timeout_s=health_check_timeout_s, logging_config=logging_config, slo_ms=slo_ms,
        profile_csv=profile_csv, priority=priority, drop_stale=drop_stale, engine=engine,
        max_request_retries=max_request_retries, request_retry_timeout_s=request_retry_timeout_s,
        tensor_parallel_size=tensor_parallel_size, tp_backend=tp_backend).items() if v is not None}
    if isinstance(given.get("autoscaling_config"), AutoscalingConfig):
        given["autoscaling_config"] = given["autoscaling_config"].model_dump()
    if isinstance(given.get("engine"), EngineConfig):
        given["engine"] = given["engine"].model_dump()

    def deco(fc):
        if not (inspect.isclass(fc) or callable(fc)):
            raise TypeError("@serve.deployment must decorate a class or a function")
        dname = name or getattr(fc, "__name__", "deployment")
        cfg = DeploymentConfig(name=dname, **given)
        return Deployment(fc, cfg, dname)

    if _func_or_class is not None:
        return deco(_func_or_class)
    return deco


# ---------------------------------------------------------------------------
# module-level functions (serve/__init__.py exports)
# ---------------------------------------------------------------------------
def _controller(create: bool = True):
    from .controller import get_controller

    return get_controller(create)


def start(http_options: Optional[Dict[str, Any]] = None, grpc_options: Optional[Dict[str, Any]] = None,
          **kwargs) -> None:
    """Start the (in-process) serve controller.  kwargs: mode="auto"|"local"|"process";
    ``http_options={"host": ..., "port": ...}`` also starts the HTTP proxy
    (port 0 = pick a free port; see ``serve.http_port()``); ``grpc_options=
    {"host", "port", "request_types": {"/pkg.Svc/Method": MsgClass}, "streaming_methods": [...]}``
    starts the gRPC proxy (``serve.grpc_port()``)."""
    _controller().configure(http_options=http_options, grpc_options=grpc_options, **kwargs)


def http_port() -> Optional[int]:
    ctrl = _controller(create=False)
    return ctrl.proxy.port if ctrl is not None and ctrl.proxy is not None else None


def grpc_port() -> Optional[int]:
    ctrl = _controller(create=False)
    return ctrl.grpc_proxy.port if ctrl is not None and ctrl.grpc_proxy is not None else None


def run(target: Application, blocking: bool = False, name: str = "default", route_prefix: Optional[str] = "/",
        logging_config=None, _local_testing_mode: bool = False, mode: Optional[str] = None):
    """Deploy an application and return a DeploymentHandle to its ingress."""
    if isinstance(target, Deployment):
        target = target.bind()
    if not isinstance(target, Application):
        raise TypeError("serve.run expects an Application (Deployment.bind(...))")
    if logging_config is not None:
        # application-level default: deployments without their own config take it
        from .logging_utils import as_logging_config

        lc = as_logging_config(logging_config).model_dump()
        for node in target.walk():
            if node.deployment.config.logging_config is None:
                node.deployment = node.deployment.options(logging_config=lc)
    ctrl = _controller()
    handle = ctrl.deploy_application(target, name=name, route_prefix=route_prefix,
                                     mode=("local" if _local_testing_mode else mode))
    if blocking:  # pragma: no cover - interactive
        import time

        try:
            while True:
                time.sleep(1)
        except KeyboardInterrupt:
            shutdown()
    return handle


def shutdown() -> None:
    ctrl = _controller(create=False)
    if ctrl is not None:
        ctrl.shutdown()


def delete(name: str, _blocking: bool = True) -> None:
    ctrl = _controller(create=False)
    if ctrl is not None:
        ctrl.delete_application(name)


def metrics_text() -> str:
    """Prometheus text of the running instance (user metrics + serving counters)."""
    return _controller().metrics_text()


def status():
    ctrl = _controller(create=False)
    return ctrl.status() if ctrl is not None else {"applications": {}}


def get_app_handle(name: str):
    return _controller().get_app_handle(name)


def get_deployment_handle(deployment_name: str, app_name: Optional[str] = None):
    return _controller().get_deployment_handle(deployment_name, app_name)
