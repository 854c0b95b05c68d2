"""YAML / JSON application config (reference: serve/schema.py:261,476,689
DeploymentSchema / ServeApplicationSchema / ServeDeploySchema).

    applications:
      - name: default
        route_prefix: /
        import_path: my_module:app          # module:Application
        args: {}                            # passed to a builder function
        deployments:                        # per-deployment overrides
          - name: Model
            num_replicas: 2
            max_ongoing_requests: 16
            ray_actor_options: {num_gpus: 1}
"""
from __future__ import annotations

import importlib
from typing import Any, Dict, List, Optional

import yaml
from pydantic import BaseModel, Field

from .config import DeploymentConfig


class DeploymentSchema(BaseModel):
    name: str
    num_replicas: Optional[Any] = None
    max_ongoing_requests: Optional[int] = None
    max_queued_requests: Optional[int] = None
    user_config: Optional[Any] = None
    autoscaling_config: Optional[Dict[str, Any]] = None
    graceful_shutdown_wait_loop_s: Optional[float] = None
    graceful_shutdown_timeout_s: Optional[float] = None
    health_check_period_s: Optional[float] = None
    health_check_timeout_s: Optional[float] = None
    ray_actor_options: Optional[Dict[str, Any]] = None
    slo_ms: Optional[float] = None
    priority: Optional[int] = None
    drop_stale: Optional[bool] = None
    max_request_retries: Optional[int] = None
    request_retry_timeout_s: Optional[float] = None
    engine: Optional[Dict[str, Any]] = None

    def overrides(self) -> Dict[str, Any]:
        return {k: v for k, v in self.model_dump().items() if v is not None and k != "name"}


class ServeApplicationSchema(BaseModel):
    name: str = "default"
    route_prefix: Optional[str] = "/"
    import_path: str
    args: Dict[str, Any] = Field(default_factory=dict)
    runtime_env: Dict[str, Any] = Field(default_factory=dict)
    deployments: List[DeploymentSchema] = Field(default_factory=list)
    mode: Optional[str] = None


class ServeDeploySchema(BaseModel):
    applications: List[ServeApplicationSchema]
    # proxies (serve/schema.py ServeDeploySchema.http_options / grpc_options)
    http_options: Optional[Dict[str, Any]] = None     # {"host": ..., "port": ...}
    grpc_options: Optional[Dict[str, Any]] = None     # {"host": ..., "port": ..., "streaming_methods": [...]}

    @classmethod
    def from_yaml(cls, path: str) -> "ServeDeploySchema":
        with open(path) as f:
            data = yaml.safe_load(f)
        return cls(**data)


def import_attr(path: str):
    if ":" in path:
        mod, attr = path.split(":", 1)
    else:
        mod, _, attr = path.rpartition(".")
    obj = importlib.import_module(mod)
    for part in attr.split("."):
        obj = getattr(obj, part)
    return obj


def build_application(app_schema: ServeApplicationSchema):
    """Import the target, call it with ``args`` if it is a builder, apply the
    per-deployment overrides to every matching node of the graph."""
    from .api import Application

    target = import_attr(app_schema.import_path)
    if not isinstance(target, Application):
        if callable(target):
            target = target(app_schema.args) if app_schema.args else target()
        if not isinstance(target, Application):
            raise TypeError(f"{app_schema.import_path} is not an Application (or a builder returning one)")
    overrides = {d.name: d.overrides() for d in app_schema.deployments}
    for node in target.walk():
        ov = overrides.pop(node.deployment.name, None)
        if ov:
            node.deployment = node.deployment.options(**ov)
    if overrides:
        raise ValueError(f"deployments {sorted(overrides)} not found in {app_schema.import_path}")
    target._import_path = app_schema.import_path       # the controller checkpoints how to rebuild it
    target._import_args = dict(app_schema.args or {})
    return target


def deploy_config(schema: ServeDeploySchema):
    from .api import run

    handles = {}
    for app in schema.applications:
        handles[app.name] = run(build_application(app), name=app.name, route_prefix=app.route_prefix, mode=app.mode)
    return handles
