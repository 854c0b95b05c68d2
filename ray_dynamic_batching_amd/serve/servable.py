"""Servable-model deployments: the GPU fast path.

``serve.model_deployment(factory, ...)`` declares a deployment whose replicas
run the native replica engine instead of Python code: requests are raw tensor
bytes in shm ring slots, batching / H2D gather / hipGraph replay / completion
are all C++ (ops/csrc/engine.cpp).  The handle API is unchanged:
``handle.remote(np_or_torch_array).result()`` returns the per-request output.

In local mode (no GPU, tests, BASELINE config 1) the same deployment runs the
model eagerly behind ``@serve.batch`` with the same batching knobs.
"""
from __future__ import annotations

from typing import Any, Callable, List, Optional, Sequence

import numpy as np

from .api import Deployment, deployment
from .batching import batch

_NP = {
    "torch.int32": np.int32, "torch.int64": np.int64, "torch.float32": np.float32, "torch.float16": np.float16,
    "torch.uint8": np.uint8, "torch.bfloat16": None,
}


class TensorCodec:
    """Fixed-shape request/response encoding for servable models."""

    def __init__(self, input_shape, input_dtype, output_shape, output_dtype):
        self.input_shape = tuple(int(s) for s in input_shape)
        self.output_shape = tuple(int(s) for s in output_shape)
        self.in_np = _NP.get(str(input_dtype), None)
        self.out_np = _NP.get(str(output_dtype), None)
        if self.in_np is None or self.out_np is None:
            raise TypeError(f"unsupported servable dtypes {input_dtype} / {output_dtype}")
        self.in_bytes = int(np.prod(self.input_shape)) * np.dtype(self.in_np).itemsize
        self.out_bytes = int(np.prod(self.output_shape)) * np.dtype(self.out_np).itemsize

    @classmethod
    def for_model(cls, m) -> "TensorCodec":
        return cls(m.input_shape, m.input_dtype, m.output_shape, m.output_dtype)

    def accepts(self, x) -> bool:
        try:
            a = self._as_np(x)
        except Exception:
            return False
        return a.shape == self.input_shape

    def _as_np(self, x):
        if hasattr(x, "detach"):
            x = x.detach().cpu().numpy()
        return np.ascontiguousarray(np.asarray(x, dtype=self.in_np))

    def encode(self, x) -> bytes:
        a = self._as_np(x)
        if a.shape != self.input_shape:
            raise ValueError(f"input shape {a.shape} != {self.input_shape}")
        return a.tobytes()

    def decode(self, b: bytes):
        return np.frombuffer(b, dtype=self.out_np).reshape(self.output_shape).copy()


class _EagerServable:
    """Local-mode body of a model deployment: eager forward behind @serve.batch."""

    __rdb_servable__ = True

    def __init__(self, factory: Callable, max_batch_size: int, batch_wait_timeout_s: float, device: str = "cpu"):
        import torch

        self.model = factory(device=device) if _accepts_device(factory) else factory()
        self.torch = torch
        self.call.set_max_batch_size(max_batch_size)
        self.call.set_batch_wait_timeout_s(batch_wait_timeout_s)

    @batch(max_batch_size=32, batch_wait_timeout_s=0.005)
    async def call(self, xs: List[Any]) -> List[Any]:
        torch = self.torch
        m = self.model
        dev = getattr(m, "device", torch.device("cpu"))
        x = torch.stack([torch.as_tensor(np.asarray(v)).to(m.input_dtype) for v in xs]).to(dev)
        y = m.forward(x)
        return [r.cpu().numpy() for r in y.unbind(0)]

    async def __call__(self, x):
        return await self.call(x)


def _accepts_device(f) -> bool:
    import inspect

    try:
        return "device" in inspect.signature(f).parameters
    except (TypeError, ValueError):
        return False


def model_deployment(factory: Callable, name: str, *, max_batch_size: int = 32, batch_wait_timeout_s: float = 0.005,
                     buckets: Optional[Sequence[int]] = None, pipeline_depth: Optional[int] = None,
                     compute_streams: Optional[int] = None, io_spec=None, **deployment_options) -> Deployment:
    """Declare a GPU servable-model deployment.  ``factory(device=...)`` returns a
    model exposing ``input_shape/input_dtype/output_shape/output_dtype`` and
    ``forward(x[B, ...])``; ``io_spec`` (or ``factory.io_spec``) =
    (input_shape, input_dtype, output_shape, output_dtype) lets the router encode
    requests without instantiating the model (see models/factories.py).
    ``engine={...}`` takes every ``EngineConfig`` field (compute streams, batch
    policy, tile table, NUMA pinning, ...); ``pipeline_depth`` /
    ``compute_streams`` are shorthands for two of them.  The defaults are the
    benchmarked replica's (3 streams x depth 6, shipped tile table)."""
    if io_spec is not None:
        factory.io_spec = tuple(io_spec)
    eng = dict(deployment_options.pop("engine", {}) or {})
    eng.setdefault("buckets", list(buckets) if buckets else None)
    if pipeline_depth is not None:
        eng.setdefault("pipeline_depth", pipeline_depth)
    if compute_streams is not None:
        eng.setdefault("compute_streams", compute_streams)
    if eng.get("pipeline_depth") is not None and eng.get("compute_streams") is None:
        # an explicit shallow pipeline cannot hold more running batches than slots
        from .config import EngineConfig

        eng["compute_streams"] = min(EngineConfig.model_fields["compute_streams"].default, int(eng["pipeline_depth"]))
    spec = getattr(factory, "io_spec", None)
    if spec is not None and not eng.get("request_slot_bytes"):
        eng["request_slot_bytes"] = TensorCodec(*spec).in_bytes
    d = deployment(_EagerServable, name=name, engine=eng, **deployment_options)
    d.servable = dict(factory=factory, max_batch_size=max_batch_size, batch_wait_timeout_s=batch_wait_timeout_s)
    return d
