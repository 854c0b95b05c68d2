"""Tensor-parallel replica group (BASELINE config 4: Llama-3-8B, TP over the
node's GPUs, prefill of <= 8 prompts).

One process per GPU; the group is ONE replica of the serving job.  Two serving
loops share one protocol -- rank 0 forms each batch from the replica's shm
queue (first-arrival timeout like @serve.batch), publishes (bucket, n) + the n
request rows on the group's broadcast ring (``runtime/csrc/tp_bcast.h``, one
record per batch), every rank runs its shard's forward (collectives inside),
rank 0 answers:

* ``NativeTP`` (GPU, hipGraphs): one native replica Engine per rank
  (``ops/csrc/engine.cpp`` TP leader / follower roles).  Rank 0's engine forms
  the batch, gathers it zero-copy on its copy stream and publishes it; each
  follower's engine copies the rows H2D on its own copy stream and replays the
  same (bucket, slot) graph with the RCCL / xGMI all-reduces captured inside,
  while batch k+1 is being formed.  No Python and no host sync per batch.
* ``TPReplica`` (eager forwards: CPU / gloo tests, one-GPU rehearsals whose
  ranks must line up before each all-reduce): the same ring from Python.

Both validate requests before batching: a payload that is not a raw tensor row
of the model's input size (a pickled call, a wrong shape) is answered with an
error status and left out of the batch -- never allowed to crash the group.

Used by Serve's tensor-parallel deployments (``serve.model_deployment(...,
tensor_parallel_size=N)``: the node agent gang-spawns the ranks and they meet
through its KV, serve/replica_main.py ``_run_tp``), by bench/llama_tp_bench.py
--serve and by tests.
"""
from __future__ import annotations

import re
from typing import Dict, List, Optional

import torch

KIND_TENSOR, KIND_PICKLE = 0, 1
ST_OK, ST_ERROR = 0, 2
BCAST_BATCH, BCAST_STOP = 0, 1


def bcast_name(group: str, epoch: int) -> str:
    """Shared-memory name of a TP group's broadcast ring (one per epoch: a
    restarted group never attaches to its predecessor's ring)."""
    return f"{re.sub(r'[^A-Za-z0-9_]', '_', group)[-80:]}_e{epoch}"


def _error_payload(msg: str) -> bytes:
    import cloudpickle

    from ..serve.exceptions import RayServeException

    return cloudpickle.dumps(RayServeException(msg))


class TPReplica:
    def __init__(self, model, job_name: Optional[str], replica: int, queue: int, buckets: List[int],
                 group: Optional[str] = None, max_wait_s: float = 0.002, use_graphs: bool = True,
                 gpu_index: int = -1, ring: Optional[str] = None, attach_timeout_s: float = 120.0):
        """``use_graphs=False`` runs each batch eagerly instead of replaying the
        bucket's hipGraph (tests with several TP ranks sharing one GPU).
        ``ring``: the group's broadcast-ring name (``bcast_name``; default from
        the group name), created by rank 0 and attached by the others."""
        from ..parallel import collective as col
        from ..utils.native import load_runtime

        self.model = model
        self.col = col
        self.group = group
        self.rank = col.get_rank(group) if group else 0
        self.world = col.get_collective_group_size(group) if group else 1
        self.buckets = sorted(buckets)
        self.max_wait_s = max_wait_s
        self.queue = queue
        self.replica = replica
        self.dev = torch.device(getattr(model, "device", "cpu"))
        self.in_shape = tuple(model.input_shape)
        self.in_dtype = model.input_dtype
        self.row_bytes = int(torch.empty(self.in_shape, dtype=self.in_dtype).numel()) * \
            torch.empty((), dtype=self.in_dtype).element_size()
        self.gpu_index = gpu_index if gpu_index >= 0 else (
            torch.cuda.current_device() if self.dev.type == "cuda" else -1)
        self.ids: Dict[int, torch.Tensor] = {b: torch.zeros(b, *self.in_shape, dtype=self.in_dtype, device=self.dev)
                                             for b in self.buckets}
        pin = self.dev.type == "cuda"
        self.stage = torch.zeros(self.buckets[-1], *self.in_shape, dtype=self.in_dtype, pin_memory=pin)
        # the pinned stage is rewritten only after the previous batch's H2D copy ran
        self._h2d = torch.cuda.Event() if pin else None
        self.out: Dict[int, torch.Tensor] = {}
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.job = None
        self.cons = None
        if self.rank == 0 and job_name:
            from . import job as rjob

            self.job = rjob.Job(job_name, create=False)
            self.cons = rjob.Consumer(self.job, [queue])
        self.bcast = None
        if self.world > 1:
            rt = load_runtime()
            name = ring or bcast_name(group or "tp", 0)
            if self.rank == 0:
                self.bcast = rt.TPBcast(name, True, n_readers=self.world - 1, n_slots=8,
                                        payload_bytes=self.buckets[-1] * self.row_bytes)
            else:
                self.bcast = rt.TPBcast(name, False, attach_timeout_s=attach_timeout_s)
            col.barrier(group)               # every rank attached: the name can go
            if self.rank == 0:
                self.bcast.unlink()
        self.batches = 0
        self.requests = 0
        self.rejected = 0
        self.use_graphs = use_graphs

    def capture(self) -> "TPReplica":
        if not self.use_graphs:
            if self.job is not None:
                self.job.set_replica_status(self.replica, 2, self.gpu_index, 0)
            return self
        with torch.no_grad():
            for b in self.buckets:
                x = self.ids[b]
                x.copy_(self.model.example_input(b, seed=b, device=self.dev))
                for _ in range(2):
                    self.model(x)
                torch.cuda.synchronize()
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    self.model(x)
                torch.cuda.current_stream().wait_stream(side)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self.out[b] = self.model(x)
                self.graphs[b] = g
        torch.cuda.synchronize()
        if self.job is not None:
            self.job.set_replica_status(self.replica, 2, self.gpu_index, 0)
        return self

    def _bucket(self, n: int) -> int:
        for b in self.buckets:
            if b >= n:
                return b
        return self.buckets[-1]

    def _valid(self, reqs):
        """Rank 0: keep raw tensor rows of the model's input size; answer every
        other request with an error (the router falls back to a pickled payload
        for a wrong shape or a kwargs call -- that must not crash the group)."""
        ok = []
        for r in reqs:
            rid, q, client, kind, t_sub, dl, payload = r
            if kind == KIND_TENSOR and len(payload) == self.row_bytes:
                ok.append(r)
                continue
            self.rejected += 1
            why = (f"tensor-parallel replica: request must be one {tuple(self.in_shape)} {self.in_dtype} row "
                   f"({self.row_bytes} bytes), got kind {kind} with {len(payload)} bytes")
            self.cons.complete(client, rid, q, ST_ERROR, t_sub, _error_payload(why), KIND_PICKLE)
        return ok

    def step(self, timeout_s: float = 0.05) -> int:
        """One serving step on every rank; returns the number of prompts served
        (0 = idle, -1 = stop)."""
        reqs = []
        if self.rank == 0:
            t_end = time_now() + timeout_s
            reqs = self._valid(self.cons.pop(self.buckets[-1], int(timeout_s * 1e9)))
            if reqs:   # first-arrival timeout: keep filling until max batch or max_wait
                t_flush = time_now() + self.max_wait_s
                while len(reqs) < self.buckets[-1] and time_now() < min(t_flush, t_end):
                    reqs += self._valid(self.cons.pop(self.buckets[-1] - len(reqs), 100_000))
            n = len(reqs)
            if n == 0:
                return 0
            b = self._bucket(n)
            payload = b"".join(r[6] for r in reqs)
            if self.bcast is not None and not self.bcast.publish(BCAST_BATCH, b, n, 0, n, payload, -1.0):
                return -1                                       # ring closed: a follower is gone
        else:
            rec = self.bcast.take(self.rank - 1, timeout_s)
            if rec is None:
                return -1 if self.bcast.closed() else 0
            kind, b, n, _, _, payload = rec
            if kind == BCAST_STOP:
                return -1
        host = self.stage[:n]
        if self._h2d is not None:
            self._h2d.synchronize()
        host.view(-1).view(torch.uint8)[: n * self.row_bytes].copy_(
            torch.frombuffer(bytearray(payload), dtype=torch.uint8))
        x = self.ids[b]
        x[:n].copy_(host, non_blocking=True)
        if self._h2d is not None:
            self._h2d.record()
        if b > n:
            x[n:].zero_()
        if self.use_graphs:
            self.graphs[b].replay()
        else:
            with torch.no_grad():
                self.out[b] = self.model(x)
        xg = self.col.get_xgmi(self.group) if self.world > 1 else None
        if xg is not None:
            # a timed-out xGMI barrier leaves partial sums in this replay's output:
            # fail loudly (and poison the communicator) rather than answer with them
            xg.check()
        if self.rank == 0:
            out = self.out[b][:n].cpu().numpy()
            q = self.queue
            for r, o in zip(reqs, out):
                rid, q, client, kind, t_sub, dl, _ = r
                self.cons.complete(client, rid, q, ST_OK, t_sub, o.tobytes(), KIND_TENSOR)
            self.cons.record_batch(self.replica, n, 0.0, q)
        self.batches += 1
        self.requests += n
        return n

    def stop_all(self) -> None:
        """Rank 0: tell the other ranks to leave their serving loop."""
        if self.rank == 0 and self.bcast is not None:
            self.bcast.publish(BCAST_STOP, 0, 0, 0, 0, b"", 1.0)
            self.bcast.close()


def time_now() -> float:
    import time

    return time.perf_counter()


class NativeTP:
    """One rank of a TP replica on the native engine (GPU, hipGraphs): rank 0
    is a TP leader engine serving the replica's queue, ranks 1..N-1 are
    follower engines fed by the group's broadcast ring (module docstring)."""

    def __init__(self, model, job_name: str, replica: int, buckets: List[int], rank: int, world: int,
                 group: Optional[str], ring: str, max_batch: int, max_wait_s: float, pipeline_depth: int = 2,
                 batch_policy: str = "timeout", attach_timeout_s: float = 120.0, compute_streams: int = 1):
        from ..parallel import collective as col
        from .engine import EngineRunner, SessionSpec

        # one compute stream when world > 1: every rank must launch the same graphs (all-reduces
        # inside) in the same order; a TP = 1 replica has no collectives and may overlap batches
        if world > 1 and compute_streams != 1:
            raise ValueError("NativeTP: a TP group runs one compute stream per rank (collectives in order)")
        self.rank, self.world, self.group = rank, world, group
        spec = SessionSpec(model=model, queue=replica, max_batch=max_batch, max_wait_s=max_wait_s, buckets=buckets)
        self.runner = EngineRunner(job_name, replica, [spec], pipeline_depth=max(2, pipeline_depth, compute_streams),
                                   zero_copy=rank == 0, compute_streams=compute_streams, batch_policy=batch_policy,
                                   tile_table="")
        # whole-forward tile tuning and the timed warm-up replay different numbers
        # of forwards per rank -- with collectives inside they would not pair up
        self.runner.tune_in_context = False
        self.runner.build(warm_s=0.0)
        eng = self.runner.engine
        if world == 1:
            pass                              # TP = 1: a plain engine, nothing to publish
        elif rank == 0:
            eng.set_tp_leader(ring, world - 1, 8)
        else:
            eng.set_tp_follower(ring, rank - 1, attach_timeout_s)
        if group is not None:
            if world > 1:
                col.barrier(group)            # every follower attached: the name can go
            if rank == 0 and world > 1:
                eng.unlink_tp()
        # (group None: ranks in one process -- tests; the caller unlinks via unlink())
        self.xg = col.get_xgmi(group) if (group and world > 1) else None

    def unlink(self) -> None:
        if self.world > 1:
            self.runner.engine.unlink_tp()

    def start(self) -> "NativeTP":
        self.runner.start()                   # rank 0: replica READY in shm
        return self

    def check(self) -> str:
        """'' while serving; else why this rank must leave (engine error, the
        leader's STOP on a follower, a poisoned xGMI communicator)."""
        err = self.runner.error()
        if err:
            return err
        if self.xg is not None:
            try:
                self.xg.check()
            except RuntimeError as e:
                return str(e)
        if not self.runner.engine.running():
            return "stopped"
        return ""

    def stop(self) -> None:
        self.runner.stop()

    def stats(self) -> dict:
        return self.runner.stats()
