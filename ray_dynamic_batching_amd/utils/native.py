"""Loading of the in-tree native extensions.

On a machine with a GPU the HIP extension is REQUIRED: ``load_ops()`` builds it
if it is missing or stale and raises if that fails -- there is no silent
fallback to eager PyTorch on the GPU path.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
import threading

_lock = threading.Lock()
_ops = None
_rt = None


def _gpu_present() -> bool:
    # device_count() does not initialise the HIP runtime on this image.
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:  # pragma: no cover
        return False


def load_runtime():
    """The host runtime (_rdb_runtime): shm rings, router, load generator."""
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is None:
            from .. import _build

            alt = os.environ.get("RDB_RUNTIME_SO", "")
            if alt:
                # a sanitizer build (python -m ray_dynamic_batching_amd._build --sanitize thread):
                # loaded from its own path, the production extension is never replaced
                spec = importlib.util.spec_from_file_location("ray_dynamic_batching_amd._rdb_runtime", alt)
                _rt = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(_rt)
                sys.modules["ray_dynamic_batching_amd._rdb_runtime"] = _rt
                return _rt
            if os.environ.get("RDB_NO_AUTOBUILD") != "1":
                _build.build_runtime()
            _rt = importlib.import_module("ray_dynamic_batching_amd._rdb_runtime")
    return _rt


def load_ops():
    """The gfx950 kernels + replica engine (_rdb_ops)."""
    global _ops
    if _ops is not None:
        return _ops
    with _lock:
        if _ops is None:
            import torch  # noqa: F401  (shares its HIP runtime)
            from .. import _build

            alt = os.environ.get("RDB_OPS_SO", "")
            if alt:
                # A/B runs: a variant build (python -m ray_dynamic_batching_amd._build --variant X -D ...)
                spec = importlib.util.spec_from_file_location("ray_dynamic_batching_amd._rdb_ops", alt)
                _ops = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(_ops)
                sys.modules["ray_dynamic_batching_amd._rdb_ops"] = _ops
                return _ops
            if os.environ.get("RDB_NO_AUTOBUILD") != "1":
                _build.build_ops()
            _ops = importlib.import_module("ray_dynamic_batching_amd._rdb_ops")
    return _ops


def native_available() -> bool:
    try:
        load_ops()
        return True
    except Exception:
        return False


def require_gpu_ops():
    """Load the HIP extension; raise loudly on a GPU box if it cannot be loaded."""
    try:
        return load_ops()
    except Exception as e:  # pragma: no cover - only on broken GPU boxes
        if _gpu_present():
            raise RuntimeError(f"ray_dynamic_batching_amd: HIP extension failed to load on a GPU host: {e}") from e
        raise
