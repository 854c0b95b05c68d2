"""Shared-memory channels for compiled actor DAGs (``core.dag``).

Reference: ``python/ray/experimental/channel/shared_memory_channel.py`` (and
the mutable-object manager behind it, ``core_worker/experimental_mutable_
object_manager.cc``): once a DAG is compiled, every edge is a shared-memory
channel and each actor runs an execution loop over its nodes, so values move
actor -> actor without the driver.

Here a channel is one request ring of a native job segment
(``runtime/csrc/shm.h``: MPSC ring, seq-numbered slots, futex doorbell); the
writer is a native ``Client`` (``submit``), the reader a native ``Consumer``
(``pop``).  Values are cloudpickled into the slot (``buffer_size_bytes`` per
value).

Tensor edges (reference ``experimental/channel/torch_tensor_type.py``,
``torch_tensor_nccl_channel.py``): a node marked
``.with_tensor_transport()`` / ``.with_type_hint(TorchTensorType())`` ships
the torch tensors inside its values through a ``TensorRing`` owned by the
channel's READER -- device memory exported once with HIP IPC for GPU tensors
(the writer's copy goes HBM -> HBM, over xGMI when the reader sits on a peer
GPU), a POSIX shared-memory segment for host tensors -- and only a small
descriptor (slot offset, dtype, shape) travels through the shm ring.  A ring
has ``ring capacity + 2`` slots: at most ``capacity`` messages are queued, one
more is being cloned out by the reader and one is being written, so a slot is
never overwritten while it is still read.
"""
from __future__ import annotations

import threading
import time
import traceback
from typing import Any, Dict, List, Optional, Tuple

STOP = ("stop",)
_ALIGN = 256                          # tensor placement inside a ring slot


class TorchTensorType:
    """Type hint of a DAG edge whose values carry torch tensors (reference
    ``ray.experimental.channel.torch_tensor_type.TorchTensorType``).
    ``transport``: "auto" / "device" / "nccl" -- GPU tensors through the
    reader's device ring (HIP IPC; xGMI between GPUs), host tensors through a
    shared-memory ring; "shm" -- the same, host tensors only (GPU tensors are
    pickled inline)."""

    def __init__(self, transport: str = "auto", _static_shape: bool = False, _direct_return: bool = False):
        if transport not in ("auto", "device", "nccl", "shm"):
            raise ValueError(f"unknown tensor transport {transport!r}")
        self.transport = transport

    def __repr__(self):
        return f"TorchTensorType(transport={self.transport!r})"


class _TRef:
    """Descriptor of a tensor placed in a ring slot."""
    __slots__ = ("dev", "off", "nbytes", "dtype", "shape")

    def __init__(self, dev, off, nbytes, dtype, shape):
        self.dev, self.off, self.nbytes, self.dtype, self.shape = dev, off, nbytes, dtype, shape

    def __reduce__(self):
        return (_TRef, (self.dev, self.off, self.nbytes, self.dtype, self.shape))


class _PtrArray:
    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3,
                                         "strides": None}


_RINGS: Dict[Tuple[str, int, str], "TensorRing"] = {}     # this process's rings by (job, queue, dev)
_RING_LOCK = threading.Lock()


class TensorRing:
    """``slots`` x ``slot_bytes`` staging buffer for one channel's tensors.
    ``dev="cuda"``: device memory of the creating process's current GPU
    (``xgmi_alloc_uncached``, exported with hipIpcGetMemHandle); ``"cpu"``: a
    POSIX shared-memory segment.  Created by the reader, attached by the
    writer from ``export()``."""

    def __init__(self, job: str, queue: int, dev: str, slots: int, slot_bytes: int, _attach: Optional[dict] = None):
        import os

        import torch

        self.job, self.queue, self.dev = job, queue, dev
        self.slots, self.slot_bytes = int(slots), int(slot_bytes)
        n = self.slots * self.slot_bytes
        self._shm = None
        self._ptr = 0
        self._owner = _attach is None
        self.pid = os.getpid() if _attach is None else _attach["pid"]
        if dev == "cpu":
            from multiprocessing import shared_memory

            if _attach is None:
                self._shm = shared_memory.SharedMemory(create=True, size=n)
            else:
                self._shm = shared_memory.SharedMemory(name=_attach["name"])
                _untrack(self._shm)
            self.buf = torch.frombuffer(self._shm.buf, dtype=torch.uint8, count=n)
        else:
            from .. import ops

            o = ops._ops()
            if _attach is None:
                self._ptr = o.xgmi_alloc_uncached(n)
                self._handle = o.xgmi_ipc_handle(self._ptr)
            else:
                self._ptr = o.xgmi_ipc_open(_attach["handle"])
            self.buf = torch.as_tensor(_PtrArray(self._ptr, n), device=torch.device("cuda", torch.cuda.current_device()))

    def export(self) -> dict:
        d = dict(job=self.job, queue=self.queue, dev=self.dev, slots=self.slots, slot_bytes=self.slot_bytes,
                 pid=self.pid)
        if self.dev == "cpu":
            d["name"] = self._shm.name
        else:
            d["handle"] = self._handle
        return d

    @staticmethod
    def attach(desc: dict) -> "TensorRing":
        import os

        key = (desc["job"], desc["queue"], desc["dev"])
        if desc["pid"] == os.getpid():                  # same process (local-mode actor, driver)
            with _RING_LOCK:
                return _RINGS[key]
        return TensorRing(desc["job"], desc["queue"], desc["dev"], desc["slots"], desc["slot_bytes"], _attach=desc)

    def slot(self, seq: int):
        base = (seq % self.slots) * self.slot_bytes
        return self.buf[base:base + self.slot_bytes]

    def close(self) -> None:
        self.buf = None
        if self._shm is not None:
            try:
                self._shm.close()
                if self._owner:
                    self._shm.unlink()
            except (OSError, BufferError):
                pass
            self._shm = None
        if self._ptr:
            from .. import ops

            o = ops._ops()
            try:
                if self._owner:
                    import torch

                    torch.cuda.synchronize()
                    o.xgmi_free(self._ptr)
                else:
                    o.xgmi_ipc_close(self._ptr)
            except Exception:  # noqa: BLE001 - teardown
                pass
            self._ptr = 0


def _untrack(shm) -> None:
    """An attached segment is the creator's to unlink: keep this process's
    resource tracker from unlinking it at exit."""
    try:
        from multiprocessing import resource_tracker

        resource_tracker.unregister(shm._name, "shared_memory")   # noqa: SLF001
    except Exception:  # noqa: BLE001
        pass


def create_rings(job: str, specs: List[Tuple[int, int, int]], devs: Tuple[str, ...]) -> Dict[int, Dict[str, dict]]:
    """Reader side: allocate the rings of this process's inbound tensor
    channels; ``specs`` = [(queue, slots, slot_bytes)]. Returns
    {queue: {dev: export}}."""
    import torch

    out: Dict[int, Dict[str, dict]] = {}
    for q, slots, nbytes in specs:
        out[q] = {}
        for dev in devs:
            if dev == "cuda" and not torch.cuda.is_available():
                continue
            r = TensorRing(job, q, dev, slots, nbytes)
            with _RING_LOCK:
                _RINGS[(job, q, dev)] = r
            out[q][dev] = r.export()
    return out


def release_rings(job: str, queues: Optional[List[int]] = None) -> None:
    """Free this process's rings of ``job`` (only those of ``queues`` if given)."""
    with _RING_LOCK:
        keys = [k for k in _RINGS if k[0] == job and (queues is None or k[1] in queues)]
        rings = [_RINGS.pop(k) for k in keys]
    for r in rings:
        r.close()


def _walk(v, fn):
    """Rebuild ``v`` with ``fn`` applied to every leaf of lists / tuples / dicts."""
    if isinstance(v, list):
        return [_walk(x, fn) for x in v]
    if isinstance(v, tuple) and type(v) is tuple:
        return tuple(_walk(x, fn) for x in v)
    if isinstance(v, dict) and type(v) is dict:
        return {k: _walk(x, fn) for k, x in v.items()}
    return fn(v)


def encode_tensors(value, rings: Dict[str, "TensorRing"], seq: int):
    """Writer side: copy every tensor of ``value`` whose device has a ring into
    slot ``seq`` of that ring and replace it with a descriptor."""
    import torch

    used = {d: 0 for d in rings}
    sync = [False]

    def put(x):
        if not isinstance(x, torch.Tensor):
            return x
        dev = "cuda" if x.is_cuda else "cpu"
        ring = rings.get(dev)
        if ring is None:
            return x
        nbytes = x.numel() * x.element_size()
        off = used[dev]
        if off + nbytes > ring.slot_bytes:
            raise ValueError(f"tensors of {off + nbytes} bytes exceed the channel's {ring.slot_bytes}-byte slot "
                             "(compile with a larger _buffer_size_bytes)")
        used[dev] = (off + nbytes + _ALIGN - 1) // _ALIGN * _ALIGN
        if nbytes:
            src = x.detach().contiguous().reshape(-1).view(torch.uint8)
            ring.slot(seq)[off:off + nbytes].copy_(src)
            sync[0] |= dev == "cuda"
        return _TRef(dev, off, nbytes, x.dtype, tuple(x.shape))

    out = _walk(value, put)
    if sync[0]:
        torch.cuda.current_stream().synchronize()     # the bytes land before the descriptor is sent
    return out


def decode_tensors(value, rings: Dict[str, "TensorRing"], seq: int):
    """Reader side: materialise the descriptors of slot ``seq`` as tensors
    owned by this process (cloned out of the ring before the slot is reused)."""
    import torch

    sync = [False]

    def get(x):
        if not isinstance(x, _TRef):
            return x
        ring = rings[x.dev]
        if x.nbytes == 0:
            t = torch.empty(x.shape, dtype=x.dtype, device=ring.buf.device)
        else:
            t = ring.slot(seq)[x.off:x.off + x.nbytes].view(x.dtype).view(x.shape).clone()
        sync[0] |= x.dev == "cuda"
        return t

    out = _walk(value, get)
    if sync[0]:
        torch.cuda.current_stream().synchronize()     # cloned out before the next message frees the slot
    return out


def _pack(kind: str, value: Any = None) -> bytes:
    import cloudpickle

    return cloudpickle.dumps((kind, value))


def _unpack(b: bytes):
    import cloudpickle

    return cloudpickle.loads(b)


class ChannelWriter:
    def __init__(self, job, queue: int, client, rings: Optional[Dict[str, dict]] = None):
        self.job, self.queue, self.client = job, queue, client
        self.client_max = int(job.info()["req_payload_bytes"])
        self.rings = {d: TensorRing.attach(desc) for d, desc in (rings or {}).items()}
        self.seq = 0

    def _encode(self, kind: str, value: Any, seq: int) -> bytes:
        if self.rings and kind == "val":
            try:
                value = encode_tensors(value, self.rings, seq)
            except ValueError as e:
                from . import RayError

                kind, value = "err", RayError(str(e)[:512])
        data = _pack(kind, value)
        if kind == "err" and len(data) > self.client_max:
            from . import RayError

            data = _pack("err", RayError(f"{type(value).__name__}: {str(value)[:256]}"))
        return data

    def _too_big(self, n: int) -> ValueError:
        return ValueError(f"value of {n} bytes exceeds the channel buffer "
                          "(compile with a larger _buffer_size_bytes)")

    def pack(self, kind: str, value: Any = None) -> bytes:
        """The message bytes of (kind, value), size-checked, WITHOUT sending it
        (raises ValueError if it can never fit).  For ring-less edges only: a
        tensor edge encodes into the slot of the message actually sent."""
        assert not self.rings, "pack() is for edges without tensor rings"
        data = self._encode(kind, value, self.seq)
        if len(data) > self.client_max:
            raise self._too_big(len(data))
        return data

    def write(self, kind: str, value: Any = None, stop: Optional[threading.Event] = None,
              timeout_s: float = 60.0, data: Optional[bytes] = None) -> None:
        """Send one message.  The slot number (which the reader counts the same
        way, one per message it pops) is taken only once the message is in the
        ring: a value that is too large, or a ring that stays full, raises and
        leaves the writer in step with its reader."""
        seq = self.seq
        if data is None:
            data = self._encode(kind, value, seq)
        if len(data) > self.client_max:
            raise self._too_big(len(data))
        t_end = time.monotonic() + timeout_s
        delay = 0.0
        while True:
            rid = self.client.submit(self.queue, data)
            if rid > 0:
                self.seq = seq + 1
                return
            if rid == -3:
                raise self._too_big(len(data))
            if (stop is not None and stop.is_set()) or time.monotonic() > t_end:
                raise TimeoutError("channel full: the reader is not consuming")
            time.sleep(delay)                      # ring full: back off
            delay = min(0.002, delay + 5e-5)


class ChannelReader:
    def __init__(self, job, queue: int, job_name: str = ""):
        from ..runtime import job as rjob

        self.queue = queue
        self.cons = rjob.Consumer(job, [queue])
        with _RING_LOCK:
            self.rings = {k[2]: r for k, r in _RINGS.items() if k[0] == job_name and k[1] == queue}
        self.seq = 0

    def read(self, stop: Optional[threading.Event] = None, timeout_s: Optional[float] = None):
        """(kind, value) of the next message; None on stop / timeout."""
        t_end = None if timeout_s is None else time.monotonic() + timeout_s
        while True:
            got = self.cons.pop(1, 50_000_000)
            if got:
                seq = self.seq
                self.seq += 1
                kind, value = _unpack(got[0][6])
                if self.rings and kind == "val":
                    value = decode_tensors(value, self.rings, seq)
                return kind, value
            if (stop is not None and stop.is_set()) or (t_end is not None and time.monotonic() > t_end):
                return None


def exec_loop(instance, plan: Dict[str, Any], stop: threading.Event) -> None:
    """The per-actor execution loop of a compiled DAG: per execution, for each
    of this actor's nodes in topological order, read one value from every input
    channel, call the method, write the result to every output channel.  An
    upstream error skips the call and flows on; STOP is forwarded and ends it."""
    from ..runtime import job as rjob

    job = rjob.Job(plan["job"], create=False)
    client = rjob.Client(job)
    rings = plan.get("rings", {})
    ops = []
    for op in plan["ops"]:
        readers = {q: ChannelReader(job, q, plan["job"]) for q in op["in_queues"]}
        writers = [ChannelWriter(job, q, client, rings.get(q)) for q in op["out_queues"]]
        ops.append((op, readers, writers))
    try:
        while not stop.is_set():
            for op, readers, writers in ops:
                vals: Dict[int, Tuple] = {}
                for q, r in readers.items():
                    m = r.read(stop)
                    if m is None:
                        return
                    vals[q] = m
                if any(m[0] == "stop" for m in vals.values()):
                    for w in writers:
                        w.write("stop", None, stop)
                    if op is ops[-1][0]:
                        return
                    continue
                err = next((m for m in vals.values() if m[0] == "err"), None)
                if err is not None:
                    out = err
                else:
                    def arg(spec):
                        return vals[spec[1]][1] if spec[0] == "chan" else spec[1]
                    a = tuple(arg(s) for s in op["args"])
                    kw = {k: arg(s) for k, s in op["kwargs"].items()}
                    try:
                        res = getattr(instance, op["method"])(*a, **kw)
                        if hasattr(res, "__await__"):
                            import asyncio

                            res = asyncio.run(_await(res))
                        out = ("val", res)
                    except BaseException as e:  # noqa: BLE001 - shipped downstream
                        from . import RayTaskError

                        out = ("err", RayTaskError(e, traceback.format_exc()))
                for w in writers:
                    try:
                        w.write(out[0], out[1], stop)
                    except ValueError as e:          # value larger than the channel buffer
                        from . import RayError

                        w.write("err", RayError(str(e)[:512]), stop)
    finally:
        for _op, _r, writers in ops:
            for w in writers:
                for r in w.rings.values():
                    if not r._owner and r.pid != _getpid():
                        r.close()
        release_rings(plan["job"], [q for op, _r, _w in ops for q in op["in_queues"]])
        job.close()


def _getpid() -> int:
    import os

    return os.getpid()


async def _await(aw):
    return await aw


def start_exec_loop(instance, plan: Dict[str, Any]) -> threading.Event:
    stop = threading.Event()
    threading.Thread(target=exec_loop, args=(instance, plan, stop), daemon=True,
                     name=f"rdb-dag-{plan['job'][-8:]}").start()
    return stop
