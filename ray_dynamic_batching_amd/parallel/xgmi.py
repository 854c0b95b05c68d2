"""Custom all-reduce over xGMI peer memory for tensor-parallel groups inside one
node ("custom xGMI one-shot /
two-shot all-reduce, fused with residual + RMSNorm, RCCL fallback").

The reference exposes all-reduce through ``ray.util.collective`` on NCCL
(``python/ray/util/collective/collective.py:258``,
``collective_group/nccl_collective_group.py:188``); this module is the
MI355X-native fast path behind the same call (``parallel.collective.allreduce``
uses it when enabled) and the fused ``all_reduce_rmsnorm`` the TP Llama uses.

Every rank allocates three fine-grained uncached device buffers (receive
slots, gather buffer = all-reduced output, signal block), exports them as HIP
IPC handles, and maps every peer's buffers; the kernel (``ops/csrc/xgmi.hip``)
pushes data straight into peers' memory over the xGMI mesh and synchronises
with per-block flags.  One-shot (one barrier) below ``one_shot_max_bytes``,
two-shot (reduce-scatter + all-gather, two barriers) above it.

``XgmiCommunicator.create(group)`` builds a real group (one process per GPU,
handles exchanged over the torch.distributed group); ``local_group(world)``
builds ``world`` communicators inside ONE process on ONE GPU (no IPC), used by
tests to exercise the protocol on a single-GPU box.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

_DT = {torch.bfloat16: 0, torch.float16: 1}


def _ops():
    from .. import ops

    return ops._ops()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


class _Buffers:
    """One rank's uncached buffers: recv [2][world][slot], gather [slot_max], signal."""

    def __init__(self, world: int, slot_elems: int, gather_elems: int, elem_bytes: int):
        o = _ops()
        self.recv_bytes = 2 * world * slot_elems * elem_bytes
        self.gather_bytes = gather_elems * elem_bytes
        self.recv = o.xgmi_alloc_uncached(self.recv_bytes)
        self.gather = o.xgmi_alloc_uncached(self.gather_bytes)
        self.sig = o.xgmi_alloc_uncached(o.xgmi_signal_bytes())

    def handles(self) -> Tuple[bytes, bytes, bytes]:
        o = _ops()
        return o.xgmi_ipc_handle(self.recv), o.xgmi_ipc_handle(self.gather), o.xgmi_ipc_handle(self.sig)

    def free(self):
        o = _ops()
        for p in (self.recv, self.gather, self.sig):
            if p:
                o.xgmi_free(p)
        self.recv = self.gather = self.sig = 0


class _PtrArray:
    """Minimal ``__cuda_array_interface__`` so torch can view a raw device buffer."""

    def __init__(self, ptr: int, shape, typestr: str):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (ptr, False),
                                         "version": 3, "strides": None}


class XgmiCommunicator:
    """All-reduce (and all-reduce + RMSNorm) over the xGMI mesh for one TP group."""

    def __init__(self, rank: int, world: int, mine: _Buffers, recv: Sequence[int], gather: Sequence[int],
                 sig: Sequence[int], slot_elems: int, max_elems: int, dtype: torch.dtype, device: torch.device,
                 one_shot_max_bytes: int, timeout_s: float, opened: Sequence[int] = (), owns: bool = True):
        if not 1 <= world <= 8:
            raise ValueError("xgmi: 1..8 ranks")
        self.rank, self.world = rank, world
        self.mine = mine
        self.recv, self.gather, self.sig = list(recv), list(gather), list(sig)
        self.slot_elems = slot_elems
        self.max_elems = max_elems
        self.dtype = dtype
        self.device = device
        self.one_shot_max_bytes = one_shot_max_bytes
        self.timeout_ticks = int(timeout_s * _ops().xgmi_ticks_per_second())
        self._opened = list(opened)
        self._owns = owns
        self.calls = 0
        self.poisoned = False
        # Store flavour of the fused-norm output: 0 plain (default), 1 nontemporal, 2
        # write-through (sc1).  Plain stores keep the normalised rows in the XCD's L2
        # for the GEMM that reads them next.  (Round 2 made sc1 the default after a
        # graph-replay test read "unwritten" rows; tools/archive/gpu_xgmi_cause*.sh showed the
        # rows were unwritten because the two in-process ranks' streams shared one
        # hardware queue and the barrier timed out -- every store flavour and both
        # copy engines pass once the ranks run concurrently, tests/test_xgmi_gpu.py.)
        import os

        self.norm_store = int(os.environ.get("RDB_XGMI_NORM_STORE", "0"))
        # cap on the kernel's blocks (rows are grid-strided; every rank of a group
        # must use the same cap: barriers are per block).  A TP group rehearsed on
        # ONE GPU sets it low (RDB_XGMI_MAX_GRID=8): ranks spinning in the kernel
        # then hold at most world x 8 CU slots, never every CU a peer's GEMM needs.
        self.max_grid = max(1, min(256, int(os.environ.get("RDB_XGMI_MAX_GRID", "256"))))
        self.debug_ptr = 0          # set by enable_debug(): per-block launch-view records

    # -- construction ---------------------------------------------------------
    @staticmethod
    def _sizes(world: int, max_elems: int, one_shot_max_bytes: int, elem_bytes: int):
        one_shot_elems = one_shot_max_bytes // elem_bytes
        slot = max(min(one_shot_elems, max_elems), -(-max_elems // world) + 8192)  # + one 8k row of slack
        return slot

    @classmethod
    def create(cls, group_name: str = "default", max_elems: int = 1 << 23, dtype: torch.dtype = torch.bfloat16,
               one_shot_max_bytes: int = 512 << 10, timeout_s: float = 30.0) -> "XgmiCommunicator":
        """Collective over the torch.distributed group behind ``group_name``
        (``parallel.collective``); every rank of the group must call it."""
        import torch.distributed as dist

        from . import collective as col

        g = col._g(group_name)
        world, rank = g.world_size, g.rank
        eb = torch.finfo(dtype).bits // 8
        slot = cls._sizes(world, max_elems, one_shot_max_bytes, eb)
        mine = _Buffers(world, slot, max_elems, eb)
        handles: List[Optional[Tuple[bytes, bytes, bytes]]] = [None] * world
        dist.all_gather_object(handles, mine.handles(), group=g.pg)
        o = _ops()
        recv, gather, sig, opened = [], [], [], []
        for p in range(world):
            if p == rank:
                recv.append(mine.recv), gather.append(mine.gather), sig.append(mine.sig)
                continue
            ptrs = [o.xgmi_ipc_open(h) for h in handles[p]]
            opened += ptrs
            recv.append(ptrs[0]), gather.append(ptrs[1]), sig.append(ptrs[2])
        dist.barrier(group=g.pg)
        return cls(rank, world, mine, recv, gather, sig, slot, max_elems, dtype,
                   torch.device("cuda", torch.cuda.current_device()), one_shot_max_bytes, timeout_s, opened)

    @classmethod
    def local_group(cls, world: int, max_elems: int = 1 << 20, dtype: torch.dtype = torch.bfloat16,
                    one_shot_max_bytes: int = 512 << 10, timeout_s: float = 10.0) -> List["XgmiCommunicator"]:
        """``world`` ranks inside this process on the current GPU (tests): the
        kernels of different ranks must run concurrently (one stream each)."""
        eb = torch.finfo(dtype).bits // 8
        slot = cls._sizes(world, max_elems, one_shot_max_bytes, eb)
        bufs = [_Buffers(world, slot, max_elems, eb) for _ in range(world)]
        dev = torch.device("cuda", torch.cuda.current_device())
        return [cls(r, world, bufs[r], [b.recv for b in bufs], [b.gather for b in bufs], [b.sig for b in bufs],
                    slot, max_elems, dtype, dev, one_shot_max_bytes, timeout_s) for r in range(world)]

    # -- ops --------------------------------------------------------------------
    def output_view(self, rows: int, cols: int) -> torch.Tensor:
        """The gather buffer as a [rows, cols] tensor: where every call writes
        its all-reduced x (valid until the next call on this communicator)."""
        if rows * cols > self.max_elems:
            raise ValueError("xgmi: view exceeds the gather buffer")
        t = torch.as_tensor(_PtrArray(self.mine.gather, (rows * cols,), "<i2"), device=self.device)
        return t.view(self.dtype).view(rows, cols)

    def _launch(self, x: torch.Tensor, gamma: Optional[torch.Tensor], eps: float,
                norm_out: Optional[torch.Tensor], two_shot: Optional[bool]) -> None:
        if self.poisoned:
            raise RuntimeError("xgmi: communicator poisoned by an earlier barrier timeout; rebuild the group")
        if x.dtype != self.dtype or not x.is_cuda or not x.is_contiguous() or x.dim() != 2:
            raise ValueError("xgmi: x must be a contiguous 2-D tensor of the communicator dtype on the GPU")
        T, D = x.shape
        if T * D > self.max_elems:
            raise ValueError(f"xgmi: message of {T * D} elements exceeds max_elems={self.max_elems}")
        nbytes = T * D * x.element_size()
        if two_shot is None:
            two_shot = self.world > 1 and nbytes > self.one_shot_max_bytes
        rows_per_block = -(-T // self.world) if two_shot else T
        grid = max(1, min(self.max_grid, rows_per_block))
        _ops().xgmi_allreduce(_DT[self.dtype], self.recv, self.gather, self.sig, self.rank, x.data_ptr(),
                              norm_out.data_ptr() if norm_out is not None else 0,
                              gamma.data_ptr() if gamma is not None else 0, float(eps), T, D, self.slot_elems,
                              int(two_shot), grid, self.timeout_ticks, _stream(), self.debug_ptr,
                              self.norm_store)
        self.calls += 1

    def all_reduce(self, x: torch.Tensor, two_shot: Optional[bool] = None) -> torch.Tensor:
        """Sum of ``x`` [T, D] over the group; returns a view of the gather buffer."""
        self._launch(x, None, 0.0, None, two_shot)
        return self.output_view(*x.shape)

    def all_reduce_rmsnorm(self, x: torch.Tensor, gamma: torch.Tensor, eps: float = 1e-5,
                           norm_out: Optional[torch.Tensor] = None,
                           two_shot: Optional[bool] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """(s, rmsnorm(s) * gamma) with s = sum of ``x`` over the group.  ``s`` is a
        view of the gather buffer (valid until the next call)."""
        if gamma.dtype != self.dtype or gamma.numel() != x.shape[-1] or not gamma.is_contiguous():
            raise ValueError("xgmi: gamma must be a contiguous [D] tensor of the communicator dtype")
        if norm_out is None:
            norm_out = torch.empty_like(x)
        self._launch(x, gamma, eps, norm_out, two_shot)
        return self.output_view(*x.shape), norm_out

    def error(self) -> int:
        """Nonzero when a barrier of this rank timed out (a peer never arrived)."""
        return _ops().xgmi_read_error(self.mine.sig)

    def check(self) -> None:
        """Raise (and poison the communicator) if any barrier of this rank timed
        out.  A timed-out call returned partial sums; the kernel still advanced
        its epochs so the protocol stays in step, but the results of that call
        (and of the captured graph replay it was part of) are garbage.
        Synchronises with the device (reads the signal block)."""
        if self.poisoned:
            raise RuntimeError("xgmi: communicator poisoned by an earlier barrier timeout")
        e = self.error()
        if e:
            self.poisoned = True
            raise RuntimeError(f"xgmi: barrier {'A' if e == 1 else 'B'} timed out on rank {self.rank} "
                               f"(a peer never arrived); communicator poisoned")

    def enable_debug(self, max_blocks: int = 256) -> None:
        """Every later launch records, per block, the pointers / shape / epoch /
        XCC id it actually ran with (``debug_records``)."""
        if not self.debug_ptr:
            self._dbg_bytes = max_blocks * 64
            self.debug_ptr = _ops().xgmi_alloc_uncached(self._dbg_bytes)

    def debug_records(self, blocks: int) -> List[Tuple[int, ...]]:
        if not self.debug_ptr:
            return []
        t = torch.as_tensor(_PtrArray(self.debug_ptr, (blocks * 8,), "<i8"), device=self.device).cpu()
        return [tuple(int(v) for v in t[b * 8:(b + 1) * 8]) for b in range(blocks)]

    def close(self) -> None:
        o = _ops()
        if self.debug_ptr:
            o.xgmi_free(self.debug_ptr)
            self.debug_ptr = 0
        for p in self._opened:
            o.xgmi_ipc_close(p)
        self._opened = []
        if self._owns and self.mine is not None:
            self.mine.free()
        self.mine = None


def algorithm_time_model(nbytes: int, world: int, link_GBps: float = 153.0, barrier_us: float = 3.0) -> dict:
    """First-order time of the two algorithms on the 7-link mesh (for bucket /
    threshold sizing): one-shot pushes (N-1) copies, two-shot 2 (N-1)/N."""
    if world <= 1:
        return {"one_shot_us": 0.0, "two_shot_us": 0.0}
    per_link = link_GBps * 1e3  # bytes / us
    one = nbytes / per_link + barrier_us
    two = 2 * nbytes / world / per_link + 2 * barrier_us
    return {"one_shot_us": one, "two_shot_us": two}
