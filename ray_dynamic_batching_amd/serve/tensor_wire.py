"""Raw-tensor wire format for Python-worker deployments (the reference's own
GPU idiom: ``@serve.deployment(ray_actor_options={"num_gpus": 1})`` + a
``@serve.batch`` method on a torch model, release/serve_tests/workloads/
resnet_50.py:50-57; python/ray/serve/batching.py:529-678).

A call whose only argument is a numpy array or a CPU torch tensor travels as
ONE header + the array's bytes in the request's shm ring slot -- never
cloudpickled -- and a result that is an array / tensor comes back the same way.
The replica decodes the argument as a view of the popped payload; the batch
helper ``stack_to_device`` (serve/batching.py) assembles a batch in a pinned
staging buffer and copies it H2D with ``non_blocking=True`` on a side stream.

    header = MAGIC(4) | version u8 | flags u8 (1 = torch, 2 = stream) | ndim u8 |
             dtype-name len u8 | method len u16 | mux len u16 | rid len u16 |
             shape (ndim x i64) | dtype name | method | mux id | request id | raw bytes
"""
from __future__ import annotations

import struct
from typing import Any, Optional, Tuple

import numpy as np

KIND_TENSOR_CALL = 4      # request: header + raw array bytes (ShmRouter -> Python replica)
KIND_TENSOR_RESULT = 5    # result: header + raw array bytes (Python replica -> ShmRouter)
MAGIC = b"RDBT"
_HDR = struct.Struct("<4sBBBBHHH")
F_TORCH, F_STREAM = 1, 2

_NP_OK = {"float16", "float32", "float64", "int8", "int16", "int32", "int64", "uint8", "uint16", "uint32",
          "uint64", "bool"}
_TORCH_RAW = {"bfloat16": "int16"}        # torch dtypes numpy cannot hold: moved as their bit pattern


def _torch():
    try:
        import torch

        return torch
    except ImportError:  # pragma: no cover
        return None


def _as_array(x) -> Optional[Tuple[np.ndarray, bool, str]]:
    """(contiguous ndarray of the raw bytes, is_torch, dtype name) or None."""
    if isinstance(x, np.ndarray):
        if x.dtype.name not in _NP_OK or x.dtype.hasobject:
            return None
        return np.ascontiguousarray(x), False, x.dtype.name
    t = _torch()
    if t is not None and isinstance(x, t.Tensor):
        if x.is_cuda or x.requires_grad or x.is_sparse or x.is_complex():
            return None
        name = str(x.dtype).replace("torch.", "")
        c = x.detach().contiguous()
        if name in _TORCH_RAW:
            return c.view(getattr(t, _TORCH_RAW[name])).numpy(), True, name
        if name not in _NP_OK:
            return None
        return c.numpy(), True, name
    return None


def encodable(args, kwargs) -> bool:
    """One positional array / CPU tensor argument and nothing else."""
    return len(args) == 1 and not kwargs and _as_array(args[0]) is not None


def _pack(arr: np.ndarray, is_torch: bool, dtype: str, method: str = "", mux: str = "", rid: str = "",
          stream: bool = False) -> bytes:
    d, m, x, r = dtype.encode(), method.encode(), str(mux or "").encode(), str(rid if rid is not None else "").encode()
    flags = (F_TORCH if is_torch else 0) | (F_STREAM if stream else 0)
    head = _HDR.pack(MAGIC, 1, flags, arr.ndim, len(d), len(m), len(x), len(r))
    shape = struct.pack(f"<{arr.ndim}q", *arr.shape)
    return b"".join((head, shape, d, m, x, r, arr.tobytes()))


def _unpack(payload) -> Tuple[Any, str, str, str, bool]:
    mv = memoryview(payload)
    magic, ver, flags, ndim, ld, lm, lx, lr = _HDR.unpack_from(mv, 0)
    if magic != MAGIC or ver != 1:
        raise ValueError("not a raw-tensor payload")
    o = _HDR.size
    shape = struct.unpack_from(f"<{ndim}q", mv, o)
    o += 8 * ndim
    dtype = bytes(mv[o:o + ld]).decode()
    o += ld
    method = bytes(mv[o:o + lm]).decode()
    o += lm
    mux = bytes(mv[o:o + lx]).decode()
    o += lx
    rid = bytes(mv[o:o + lr]).decode()
    rid = int(rid) if rid.isdigit() else rid          # handles number their requests
    o += lr
    store = _TORCH_RAW.get(dtype, dtype)
    arr = np.frombuffer(mv[o:], dtype=np.dtype(store)).reshape(shape)     # a view of the payload, no copy
    val: Any = arr
    if flags & F_TORCH:
        t = _torch()
        val = t.from_numpy(arr.copy() if not arr.flags.writeable else arr)
        if dtype in _TORCH_RAW:
            val = val.view(getattr(t, dtype))
    return val, method, mux, rid, bool(flags & F_STREAM)


def encode_call(method: str, x, mux: str = "", rid: str = "", stream: bool = False) -> bytes:
    arr, is_torch, dtype = _as_array(x)
    return _pack(arr, is_torch, dtype, method, mux, rid, stream)


def decode_call(payload):
    """-> (method, arg, multiplexed model id, request id, stream)."""
    val, method, mux, rid, stream = _unpack(payload)
    return method, val, mux, rid, stream


def result_encodable(x) -> bool:
    if _as_array(x) is not None:
        return True
    t = _torch()
    return t is not None and isinstance(x, t.Tensor) and x.is_cuda and not x.requires_grad


def encode_result(x) -> bytes:
    t = _torch()
    if t is not None and isinstance(x, t.Tensor) and x.is_cuda:
        x = x.detach().cpu()          # a GPU result crosses to the caller as its raw bytes
    arr, is_torch, dtype = _as_array(x)
    return _pack(arr, is_torch, dtype)


def decode_result(payload):
    return _unpack(payload)[0]
