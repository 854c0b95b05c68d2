"""fp32 numerics anchor for every model of the zoo.

``fp32_reference(model)`` returns the SAME model -- the same weights, bf16 /
fp16 values upcast exactly -- evaluated by the plain PyTorch path in fp32.  The
HIP kernels are then checked against an fp32 computation of identical weights,
so a test measures the kernels' arithmetic (bf16 storage of activations, fp32
MFMA accumulation) and not a second bf16 implementation's rounding.  Also
reachable as ``models.create(name, backend="torch32")``.

Reference counterpart: the fork serves torchvision models under AMP autocast
(293-project/profiling/ModelProfiler.py:101); its numerics are those of cuDNN /
cuBLAS in fp16 -- the fp32 path here is the stricter anchor.
"""
from __future__ import annotations

import copy

import torch

__all__ = ["fp32_reference", "eager_reference", "rel_err", "parity_bound"]


def _up(v):
    if isinstance(v, torch.Tensor):
        return v.float() if v.is_floating_point() else v
    if isinstance(v, list):
        return [_up(x) for x in v]
    if isinstance(v, tuple):
        return tuple(_up(x) for x in v)
    if isinstance(v, dict):
        return {k: _up(x) for k, x in v.items()}
    return v


# attributes that are caches of kernel-layout weights (the torch path never reads them)
_KERNEL_CACHES = ("_packed", "_folded", "_deferred", "_folded_key", "_workspace", "_ws")


def fp32_reference(model):
    """A shallow copy of ``model`` whose floating tensors are fp32 and whose
    forward runs the PyTorch reference path (``backend="torch"``)."""
    ref = copy.copy(model)
    for k, v in vars(model).items():
        if k in _KERNEL_CACHES:
            setattr(ref, k, None)
            continue
        setattr(ref, k, _up(v))
    ref.dtype = torch.float32
    ref.backend = "torch"
    return ref


def rel_err(y: torch.Tensor, ref: torch.Tensor) -> float:
    """||y - ref||_inf / ||ref||_inf (both upcast to fp32)."""
    y, ref = y.float(), ref.float()
    return float((y - ref).abs().max() / ref.abs().max().clamp_min(1e-12))


def eager_reference(model):
    """A shallow copy of ``model`` on the PyTorch path in the model's OWN dtype
    (bf16 / fp16 eager): its distance to ``fp32_reference`` is the rounding
    error any bf16 implementation of the network pays, the yardstick for the
    HIP kernels' error (``parity_bound``)."""
    ref = copy.copy(model)
    for k in _KERNEL_CACHES:
        if k in vars(model):
            setattr(ref, k, None)
    ref.backend = "torch"
    return ref


def parity_bound(eager_err: float, floor: float = 2e-2, factor: float = 1.75) -> float:
    """Relative-error bound for a HIP forward against the fp32 anchor: the
    ``floor`` or ``factor`` x the PyTorch eager error at the same dtype,
    whichever is larger (bf16 logits of a 12-layer encoder sit ~2 % from fp32
    in eager PyTorch already; a kernel bug of a few percent still fails)."""
    return max(floor, factor * eager_err)
