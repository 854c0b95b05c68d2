"""Collective-communication API with the surface of ``ray.util.collective``
(reference: python/ray/util/collective/collective.py:40-789; NCCLGroup via
cupy, GLOOGroup via pygloo).

MI355X-native: one process per GPU, ``torch.distributed`` with the ``nccl``
backend, which IS RCCL on ROCm, over the xGMI full mesh (7 links x ~153 GB/s
per GPU); ``gloo`` for CPU groups.  Named groups map to torch process groups;
the rendezvous is torch's TCP store (the reference used a detached named actor
``NCCLUniqueIDStore``).  Multi-tensor "multigpu" variants are not provided:
one process drives one GPU.
"""
from __future__ import annotations

import enum
import os
import threading
from typing import Dict, List, Optional

import torch
import torch.distributed as dist


class ReduceOp(enum.Enum):
    SUM = 0
    PRODUCT = 1
    MIN = 2
    MAX = 3


_TORCH_OP = {ReduceOp.SUM: dist.ReduceOp.SUM, ReduceOp.PRODUCT: dist.ReduceOp.PRODUCT,
             ReduceOp.MIN: dist.ReduceOp.MIN, ReduceOp.MAX: dist.ReduceOp.MAX}


class _Group:
    def __init__(self, name: str, world_size: int, rank: int, backend: str, pg):
        self.name = name
        self.world_size = world_size
        self.rank = rank
        self.backend = backend
        self.pg = pg
        self.xgmi = None   # optional parallel.xgmi.XgmiCommunicator (enable_xgmi)


_groups: Dict[str, _Group] = {}
_lock = threading.Lock()


def _backend(backend: str) -> str:
    b = backend.lower()
    if b in ("nccl", "rccl"):
        return "nccl"
    if b == "gloo":
        return "gloo"
    raise ValueError(f"unsupported backend {backend!r} (nccl/rccl or gloo)")


def init_collective_group(world_size: int, rank: int, backend: str = "nccl", group_name: str = "default",
                          master_addr: Optional[str] = None, master_port: Optional[int] = None,
                          store=None) -> None:
    """Join a named collective group.  The first group initialises the default
    torch process group (rendezvous via ``store`` -- e.g. the node agent's
    ``parallel.rendezvous.agent_store`` -- or MASTER_ADDR/MASTER_PORT / the args)."""
    b = _backend(backend)
    with _lock:
        if group_name in _groups:
            raise RuntimeError(f"collective group {group_name!r} already initialised")
        if not dist.is_initialized():
            if master_addr:
                os.environ["MASTER_ADDR"] = master_addr
            if master_port:
                os.environ["MASTER_PORT"] = str(master_port)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {} if store is None else {"store": store}
            if b == "nccl":
                dev = torch.device("cuda", torch.cuda.current_device())
                kw["device_id"] = dev
            dist.init_process_group(b, rank=rank, world_size=world_size, **kw)
            pg = dist.group.WORLD
        else:
            if dist.get_world_size() == world_size:
                pg = dist.group.WORLD if dist.get_backend() == b else dist.new_group(backend=b)
            else:
                raise RuntimeError("sub-groups of a different size need create_collective_group with ranks")
        _groups[group_name] = _Group(group_name, world_size, rank, b, pg)


def create_collective_group(ranks: List[int], backend: str = "nccl", group_name: str = "default") -> None:
    """Sub-group of an initialised world (every world rank must call it)."""
    b = _backend(backend)
    pg = dist.new_group(ranks=ranks, backend=b)
    me = dist.get_rank()
    with _lock:
        if me in ranks:
            _groups[group_name] = _Group(group_name, len(ranks), ranks.index(me), b, pg)


def is_group_initialized(group_name: str = "default") -> bool:
    return group_name in _groups


def destroy_collective_group(group_name: str = "default") -> None:
    with _lock:
        g = _groups.pop(group_name, None)
    if g is not None and g.xgmi is not None:
        g.xgmi.close()
        g.xgmi = None
    if g is not None and g.pg is not dist.group.WORLD:
        dist.destroy_process_group(g.pg)
    if not _groups and dist.is_initialized() and g is not None and g.pg is dist.group.WORLD:
        dist.destroy_process_group()


def _g(name: str) -> _Group:
    g = _groups.get(name)
    if g is None:
        raise RuntimeError(f"collective group {name!r} is not initialised in this process")
    return g


def get_rank(group_name: str = "default") -> int:
    return _g(group_name).rank if group_name in _groups else -1


def get_collective_group_size(group_name: str = "default") -> int:
    return _g(group_name).world_size if group_name in _groups else -1


def get_group_handle(group_name: str = "default"):
    return _g(group_name).pg


def enable_xgmi(group_name: str = "default", **kw):
    """Attach the custom xGMI all-reduce (``parallel.xgmi``) to a GPU group: from
    then on ``allreduce`` of bf16/f16 tensors up to ``max_elems`` goes through
    it instead of RCCL.  Every rank of the group must call it.  Returns the
    communicator (or None -- RCCL stays in use -- when IPC is unavailable)."""
    g = _g(group_name)
    if getattr(g, "xgmi", None) is not None:
        return g.xgmi
    from .xgmi import XgmiCommunicator

    try:
        g.xgmi = XgmiCommunicator.create(group_name, **kw)
    except RuntimeError as e:  # no IPC / uncached memory on this platform: RCCL fallback
        import warnings

        warnings.warn(f"xgmi all-reduce unavailable, using RCCL: {e}")
        g.xgmi = None
    return g.xgmi


def get_xgmi(group_name: str = "default"):
    g = _groups.get(group_name)
    return getattr(g, "xgmi", None) if g is not None else None


def _xgmi_rows(n: int) -> int:
    for d in (4096, 8192, 2048, 1024, 512, 256, 128, 64, 32, 16, 8):
        if n % d == 0:
            return d
    return 0


def allreduce(tensor: torch.Tensor, group_name: str = "default", op: ReduceOp = ReduceOp.SUM) -> torch.Tensor:
    g = _g(group_name)
    xg = getattr(g, "xgmi", None)
    if (xg is not None and op == ReduceOp.SUM and tensor.is_cuda and tensor.dtype == xg.dtype
            and tensor.is_contiguous() and 0 < tensor.numel() <= xg.max_elems and _xgmi_rows(tensor.numel())):
        d = _xgmi_rows(tensor.numel())
        out = xg.all_reduce(tensor.view(-1, d))
        tensor.view(-1, d).copy_(out)
        return tensor
    dist.all_reduce(tensor, op=_TORCH_OP[op], group=g.pg)
    return tensor


def barrier(group_name: str = "default") -> None:
    g = _g(group_name)
    if g.backend == "nccl":
        dist.barrier(group=g.pg, device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier(group=g.pg)


def _global(g: _Group, group_rank: int) -> int:
    return dist.get_global_rank(g.pg, group_rank) if g.pg is not dist.group.WORLD else group_rank


def reduce(tensor: torch.Tensor, dst_rank: int = 0, group_name: str = "default",
           op: ReduceOp = ReduceOp.SUM) -> torch.Tensor:
    g = _g(group_name)
    dist.reduce(tensor, dst=_global(g, dst_rank), op=_TORCH_OP[op], group=g.pg)
    return tensor


def broadcast(tensor: torch.Tensor, src_rank: int = 0, group_name: str = "default") -> torch.Tensor:
    g = _g(group_name)
    dist.broadcast(tensor, src=_global(g, src_rank), group=g.pg)
    return tensor


def allgather(tensor_list: List[torch.Tensor], tensor: torch.Tensor, group_name: str = "default") -> List[torch.Tensor]:
    g = _g(group_name)
    if len(tensor_list) != g.world_size:
        raise ValueError("allgather: tensor_list must have world_size entries")
    dist.all_gather(tensor_list, tensor, group=g.pg)
    return tensor_list


def allgather_into(out: torch.Tensor, tensor: torch.Tensor, group_name: str = "default") -> torch.Tensor:
    """Single-buffer all-gather (out = concat over ranks along dim 0)."""
    dist.all_gather_into_tensor(out, tensor, group=_g(group_name).pg)
    return out


def reducescatter(tensor: torch.Tensor, tensor_list: List[torch.Tensor], group_name: str = "default",
                  op: ReduceOp = ReduceOp.SUM) -> torch.Tensor:
    g = _g(group_name)
    if len(tensor_list) != g.world_size:
        raise ValueError("reducescatter: tensor_list must have world_size entries")
    if g.backend == "gloo":  # gloo has no reduce_scatter: all-reduce the stack, keep our slice
        full = torch.stack([t.clone() for t in tensor_list])
        dist.all_reduce(full, op=_TORCH_OP[op], group=g.pg)
        tensor.copy_(full[g.rank])
        return tensor
    dist.reduce_scatter(tensor, tensor_list, op=_TORCH_OP[op], group=g.pg)
    return tensor


def send(tensor: torch.Tensor, dst_rank: int, group_name: str = "default") -> None:
    g = _g(group_name)
    dist.send(tensor, dst=_global(g, dst_rank), group=g.pg)


def recv(tensor: torch.Tensor, src_rank: int, group_name: str = "default") -> torch.Tensor:
    g = _g(group_name)
    dist.recv(tensor, src=_global(g, src_rank), group=g.pg)
    return tensor


def synchronize(gpu_id: Optional[int] = None) -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize(gpu_id)


def xgmi_allreduce_time_model(bytes_: int, world: int = 8, link_gbps: float = 153.0) -> dict:
    """Bandwidth model used to size TP all-reduce buckets on the MI355X xGMI
    full mesh: a ring uses one link per GPU, a direct
    reduce-scatter + all-gather uses all world-1 links."""
    ring = 2 * (world - 1) / world * bytes_ / (link_gbps * 1e9)
    direct = 2 * (world - 1) / world * bytes_ / ((world - 1) * link_gbps * 1e9)
    return dict(ring_us=ring * 1e6, direct_us=direct * 1e6)
