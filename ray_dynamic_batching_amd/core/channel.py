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
value); GPU tensors between replicas travel with ``parallel.collective`` (RCCL
over xGMI), not through a channel.
"""
from __future__ import annotations

import threading
import time
import traceback
from typing import Any, Dict, List, Optional, Tuple

STOP = ("stop",)


def _pack(kind: str, value: Any = None) -> bytes:
    import cloudpickle

    return cloudpickle.dumps((kind, value))


def _unpack(b: bytes):
    import cloudpickle

    return cloudpickle.loads(b)


class ChannelWriter:
    def __init__(self, job, queue: int, client):
        self.job, self.queue, self.client = job, queue, client
        self.client_max = int(job.info()["req_payload_bytes"])

    def write(self, kind: str, value: Any = None, stop: Optional[threading.Event] = None,
              timeout_s: float = 60.0) -> None:
        data = _pack(kind, value)
        if kind == "err" and len(data) > self.client_max:
            from . import RayError

            data = _pack("err", RayError(f"{type(value).__name__}: {str(value)[:256]}"))
        t_end = time.monotonic() + timeout_s
        delay = 0.0
        while True:
            rid = self.client.submit(self.queue, data)
            if rid > 0:
                return
            if rid == -3:
                raise ValueError(f"value of {len(data)} bytes exceeds the channel buffer "
                                 "(compile with a larger _buffer_size_bytes)")
            if (stop is not None and stop.is_set()) or time.monotonic() > t_end:
                raise TimeoutError("channel full: the reader is not consuming")
            time.sleep(delay)                      # ring full: back off
            delay = min(0.002, delay + 5e-5)


class ChannelReader:
    def __init__(self, job, queue: int):
        from ..runtime import job as rjob

        self.queue = queue
        self.cons = rjob.Consumer(job, [queue])

    def read(self, stop: Optional[threading.Event] = None, timeout_s: Optional[float] = None):
        """(kind, value) of the next message; None on stop / timeout."""
        t_end = None if timeout_s is None else time.monotonic() + timeout_s
        while True:
            got = self.cons.pop(1, 50_000_000)
            if got:
                return _unpack(got[0][6])
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
    ops = []
    for op in plan["ops"]:
        readers = {q: ChannelReader(job, q) for q in op["in_queues"]}
        writers = [ChannelWriter(job, q, client) for q in op["out_queues"]]
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
        job.close()


async def _await(aw):
    return await aw


def start_exec_loop(instance, plan: Dict[str, Any]) -> threading.Event:
    stop = threading.Event()
    threading.Thread(target=exec_loop, args=(instance, plan, stop), daemon=True,
                     name=f"rdb-dag-{plan['job'][-8:]}").start()
    return stop
