"""Ray-Serve-compatible serving API on the MI355X-native runtime.

    from ray_dynamic_batching_amd import serve

    @serve.deployment(num_replicas=2, max_ongoing_requests=16)
    class Model:
        @serve.batch(max_batch_size=4, batch_wait_timeout_s=0.01)
        async def __call__(self, xs): ...

    handle = serve.run(Model.bind())
    handle.remote(x).result()
"""
from .api import Application, Deployment, delete, deployment, get_app_handle, get_deployment_handle, grpc_port, \
    http_port, metrics_text, run, shutdown, start, status
from .batching import batch, stack_to_device
from .config import AutoscalingConfig, DeploymentConfig, EngineConfig
from .context import get_replica_context
from .exceptions import BackPressureError, RayServeException, RequestCancelledError, RequestDroppedError
from .handle import DeploymentHandle, DeploymentResponse, DeploymentResponseGenerator
from .http_proxy import HTTPRequest
from .ingress import ingress
from .multiplex import get_multiplexed_model_id, multiplexed
from .servable import TensorCodec, model_deployment

__all__ = [
    "ingress",
    "Application", "Deployment", "deployment", "batch", "stack_to_device", "run", "start", "shutdown", "delete", "status",
    "get_app_handle", "get_deployment_handle", "get_replica_context", "multiplexed", "get_multiplexed_model_id",
    "DeploymentHandle", "DeploymentResponse", "DeploymentResponseGenerator", "AutoscalingConfig",
    "DeploymentConfig", "EngineConfig", "BackPressureError", "RayServeException", "RequestCancelledError",
    "RequestDroppedError", "model_deployment", "TensorCodec", "HTTPRequest", "http_port", "grpc_port", "metrics_text",
]
