"""Tensor-parallel replica group (BASELINE config 4: Llama-3-8B, TP over the
node's GPUs, prefill of <= 8 prompts).

One process per GPU (torchrun); the group is ONE replica of the serving job:

* rank 0 is the front end: it pops up to ``max_batch`` prompts from the
  replica's shm queue (first-arrival timeout like @serve.batch), pads to a
  bucket and broadcasts (bucket, n) + token ids over RCCL;
* every rank replays the hipGraph of its shard's prefill for that bucket
  (column/row-parallel linears with RCCL all-reduces captured in the graph);
* rank 0 writes each prompt's next-token id into the completion ring.

Used by Serve's tensor-parallel deployments (``serve.model_deployment(...,
tensor_parallel_size=N)``: the node agent gang-spawns the ranks and they meet
through its KV, serve/replica_main.py ``_run_tp``), by bench/llama_tp_bench.py
--serve and by tests.  Any servable works: requests are ``input_shape`` x
``input_dtype`` tensors, results ``output_shape`` x ``output_dtype`` rows.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import torch


class TPReplica:
    def __init__(self, model, job_name: Optional[str], replica: int, queue: int, buckets: List[int],
                 group: Optional[str] = None, max_wait_s: float = 0.002, use_graphs: bool = True,
                 gpu_index: int = -1):
        """``use_graphs=False`` runs each batch eagerly instead of replaying the
        bucket's hipGraph (tests with several TP ranks sharing one GPU)."""
        from ..parallel import collective as col

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
        self.gpu_index = gpu_index if gpu_index >= 0 else (
            torch.cuda.current_device() if self.dev.type == "cuda" else -1)
        self.ids: Dict[int, torch.Tensor] = {b: torch.zeros(b, *self.in_shape, dtype=self.in_dtype, device=self.dev)
                                             for b in self.buckets}
        self.out: Dict[int, torch.Tensor] = {}
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.hdr = torch.zeros(2, dtype=torch.int32, device=self.dev)      # (bucket, n) broadcast header
        self.job = None
        self.cons = None
        if self.rank == 0 and job_name:
            from . import job as rjob

            self.job = rjob.Job(job_name, create=False)
            self.cons = rjob.Consumer(self.job, [queue])
        self.batches = 0
        self.requests = 0
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

    def step(self, timeout_s: float = 0.05) -> int:
        """One serving step on every rank; returns the number of prompts served
        (0 = idle, -1 = stop)."""
        reqs = []
        if self.rank == 0:
            t_end = time.perf_counter() + timeout_s
            reqs = self.cons.pop(self.buckets[-1], int(timeout_s * 1e9))
            if reqs:   # first-arrival timeout: keep filling until max batch or max_wait
                t_flush = time.perf_counter() + self.max_wait_s
                while len(reqs) < self.buckets[-1] and time.perf_counter() < min(t_flush, t_end):
                    reqs += self.cons.pop(self.buckets[-1] - len(reqs), 100_000)
            n = len(reqs)
            b = self._bucket(n) if n else 0
            self.hdr[0], self.hdr[1] = b, n
            if n:
                host = torch.zeros(b, *self.in_shape, dtype=self.in_dtype)
                for i, r in enumerate(reqs):
                    host[i] = torch.frombuffer(bytearray(r[6]), dtype=self.in_dtype).view(self.in_shape)
                self.ids[b].copy_(host, non_blocking=False)
        if self.world > 1:
            self.col.broadcast(self.hdr, 0, self.group)
        b, n = int(self.hdr[0].item()), int(self.hdr[1].item())
        if n < 0:
            return -1
        if n == 0:
            return 0
        if self.world > 1:
            self.col.broadcast(self.ids[b], 0, self.group)
        if self.use_graphs:
            self.graphs[b].replay()
        else:
            with torch.no_grad():
                self.out[b] = self.model(self.ids[b])
        xg = self.col.get_xgmi(self.group) if self.world > 1 else None
        if xg is not None:
            # a timed-out xGMI barrier leaves partial sums in this replay's output:
            # fail loudly (and poison the communicator) rather than answer with them
            xg.check()
        if self.rank == 0:
            out = self.out[b][:n].cpu().numpy()
            for r, o in zip(reqs, out):
                rid, q, client, kind, t_sub, dl, payload = r
                self.cons.complete(client, rid, q, 0, t_sub, o.tobytes(), 0)
            self.cons.record_batch(self.replica, n, 0.0, q)
        self.batches += 1
        self.requests += n
        return n

    def stop_all(self) -> None:
        """Rank 0: tell the other ranks to leave their serving loop."""
        if self.rank == 0:
            self.hdr[0], self.hdr[1] = 0, -1
        if self.world > 1:
            self.col.broadcast(self.hdr, 0, self.group)
