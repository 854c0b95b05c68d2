#!/usr/bin/env python3
"""Headline benchmark: whole-node req/s vs p99 latency, BERT-base seq128 bf16,
dynamic batching <= 32, one replica per MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Both forms run N ranks: without a launcher (no WORLD_SIZE in the environment)
and N > 1, this process touches no GPU and starts the N ranks itself as ONE
child ``torch.distributed.run`` (127.0.0.1 rendezvous on a free port), whose
rank 0 prints the JSON line; the parent exits with the child's code.  This is
the fork's one-invocation fan-out (``ray.init(num_gpus=N)`` + one GPUWorker
per GPU, 293-project/src/scheduler.py:671-693).  Under a launcher,
``--gpus`` must equal WORLD_SIZE.

Every rank is one replica process pinned to its GPU (LOCAL_RANK).  Rank 0
creates the shared-memory job; every rank runs an ingress: a native
closed-loop load generator whose requests go through the power-of-two-choices
router over the shm queue depths of ALL replicas (`--ingress rank0` keeps one
node-wide ingress on rank 0).  Each request is one 128-token sequence
(synthetic token ids, random-init weights); each replica's native engine
coalesces up to 32 requests or 5 ms, pads to a bucket, gathers the payloads
H2D on a side stream, replays the hipGraph of the batched forward, and returns
per-request logits through the completion ring.

One "step" = 32 x N completed requests (one full dynamic batch per replica).
Untimed set-up: model load, tile table, graph capture, then the engine's device
warm-up (EngineRunner.build: ~0.25 s of graph replays, so serving starts at
steady clocks, as a production replica does before it reports ready), then the
W warm-up steps.  The timed region is bracketed by barrier +
torch.cuda.synchronize() on every rank and contains exactly K steps of the full
request path; the reported time is the max over ranks.  Latency percentiles are
client-side end-to-end (submit -> result received).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

METRIC = "req/s (whole node) vs p99 latency, BERT-base dyn-batch<=32, at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one replica per GPU); default: WORLD_SIZE under a launcher, else 1")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--max-batch", type=int, default=32)
    ap.add_argument("--max-wait-ms", type=float, default=5.0)
    ap.add_argument("--concurrency", type=int, default=96, help="closed-loop requests in flight per GPU")
    ap.add_argument("--rate", type=float, default=0.0, help="open-loop Poisson rate per GPU (req/s); 0 = closed loop")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--backend", default="hip", choices=["hip", "torch", "echo"],
                    help="echo = CPU rehearsal of the multi-rank path (native fake replicas, gloo)")
    ap.add_argument("--echo-service-us", type=float, default=1400.0, help="echo backend: batch service time")
    ap.add_argument("--batch-policy", default="timeout", choices=["timeout", "idle"],
                    help="timeout: @serve.batch semantics (full or max-wait after the first request); idle: also "
                         "dispatch a partial batch as soon as a compute stream is idle")
    # 3 streams x depth 6 (each stream on its own HIP hardware queue, runtime/queues.py): every batch of the
    # 96-request closed loop has a stream -- 37.5k req/s at p99 2.7 ms vs 34.8k at 3.67 ms for 2 x 4
    # (profiles/hw_queues_compute_streams_r6.json)
    ap.add_argument("--pipeline-depth", type=int, default=6)
    ap.add_argument("--compute-streams", type=int, default=3, help="batches executing concurrently per GPU")
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--tune-streams", type=int, default=0,
                    help="GEMM tile autotuning objective: throughput with this many concurrent streams "
                         "(0 = --compute-streams)")
    ap.add_argument("--ingress", default="per-rank", choices=["per-rank", "rank0"],
                    help="per-rank: every rank runs a load generator routing over all replicas; "
                         "rank0: one node-wide ingress on rank 0")
    ap.add_argument("--ingress-threads", type=int, default=0,
                    help="load-generator threads per ingress, each with its own client / completion ring "
                         "(0 = 1 per rank with --ingress per-rank; one per 2 GPUs, at most 4, with rank0)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="rehearsal only: every rank's replica on cuda:0, gloo instead of RCCL (a 1-GPU box "
                         "running the N-rank protocol with real engines); never a measurement")
    ap.add_argument("--tile-table", default="auto",
                    help="GEMM tile table to replay (auto = the MI355X table shipped for this config when it "
                         "exists; none = tune per shape and in context at start-up)")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--trace-out", default="", help="write a Chrome trace of the replicas' batches")
    ap.add_argument("--stamps-out", default="",
                    help="diagnostic: with the RDB_BLOCK_STAMPS kernel build (RDB_OPS_SO), save every block's start / "
                         "end / CU of the timed region to this .npy (bench/stamp_timeline.py); never a measurement")
    return ap.parse_args()


class _EchoRunner:
    """CPU stand-in for EngineRunner (native EchoServer fake replica)."""

    def __init__(self, srv):
        self.srv = srv

    def start(self):
        self.srv.start()

    def stop(self):
        self.srv.stop()

    def error(self):
        return ""


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _fan_out(n: int) -> int:
    """Start the N ranks as one child launcher and relay its output.  Runs
    before anything here touches the GPU (the parent never initialises HIP: it
    only waits), so no process that owns a GPU context is ever replaced."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    here = os.path.dirname(os.path.abspath(__file__))
    env["PYTHONPATH"] = here + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    launched = "WORLD_SIZE" in os.environ
    if not launched and (args.gpus or 1) > 1:
        sys.exit(_fan_out(args.gpus))
    if launched and args.gpus is not None and args.gpus != int(os.environ["WORLD_SIZE"]):
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={os.environ['WORLD_SIZE']} ranks",
              file=sys.stderr)
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    echo = args.backend == "echo"
    # one HIP hardware queue per engine stream (compute streams + copy + current),
    # set before anything initialises HIP (runtime/queues.py)
    from ray_dynamic_batching_amd.runtime.queues import ensure_hw_queues

    ensure_hw_queues(args.compute_streams)
    # NUMA placement BEFORE the HIP runtime or any native thread starts: this
    # rank's process (engine launcher, completer, load generator threads all
    # inherit it) is pinned to its own share of the CPUs local to its GPU
    from ray_dynamic_batching_amd.runtime import numa

    rank_gpus = [0] * world if (args.rehearse_one_gpu or world == 1) else list(range(world))
    try:
        placement = dict(rank=rank, gpu=rank_gpus[rank], **numa.place_rank(rank, rank_gpus))
    except Exception as e:  # noqa: BLE001 -- placement is an optimisation: never fail the bench on it
        placement = dict(rank=rank, gpu=rank_gpus[rank], numa_node=-1, cpus="", pinned=False, error=str(e)[:200])
    import torch
    import torch.distributed as dist

    if echo:
        if world > 1:
            dist.init_process_group("gloo")
    elif world > 1 and args.rehearse_one_gpu:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
    elif world > 1:
        torch.cuda.set_device(local)
        # RCCL default group, created lazily: DP replicas issue no device
        # collectives (requests are routed, not reduced), so no communicator is
        # built and no RCCL proxy thread competes with the replica engine
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)

    def sync():
        if not echo:
            torch.cuda.synchronize()

    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification
    from ray_dynamic_batching_amd.runtime import job as rjob
    from ray_dynamic_batching_amd.runtime.engine import EngineRunner, SessionSpec

    # Host-side rendezvous runs over a gloo group: an RCCL barrier would leave a
    # spinning all-reduce kernel on ranks 1..N-1 (occupying CUs their replica
    # engine serves on) for the whole timed region, while rank 0 drives load.
    host_pg = dist.new_group(backend="gloo") if (world > 1 and not echo and not args.rehearse_one_gpu) else None

    def barrier():
        if world > 1:
            dist.barrier(group=host_pg)

    port = os.environ.get("MASTER_PORT", str(os.getpid()))
    name = f"bench_{port}"
    n = world
    if rank == 0:
        # request rings deferred: each rank first-touches its own ring from its
        # pinned CPUs, with the pages bound to its GPU's NUMA node
        job = rjob.Job(name, create=True, n_replicas=n, n_queues=n, n_clients=max(8, n * max(4, args.ingress_threads)), req_capacity=4096,
                       req_slot_bytes=args.seq * 4, cmp_capacity=16384, cmp_slot_bytes=64, defer_req_rings=True)
    barrier()
    if rank != 0:
        job = rjob.Job(name, create=False)
    # each rank owns queue `rank` (model 0) on replica `rank`
    placement["arena_mbind"] = job.init_req_ring(rank, placement["numa_node"])
    job.configure_queue(rank, rank, 0, args.concurrency * 2, 0.0, True)

    cfg = BertConfig(seq_len=args.seq, layers=args.layers)
    # The ingress: every rank runs G native generator threads (GIL released
    # inside run()), each with its own client and completion ring, all routing
    # through the power-of-two choice over EVERY replica's queue depth -- like
    # Serve, where each proxy / handle owns a router over all replicas.  One
    # ingress per rank keeps submission and completion draining spread over
    # the node's processes instead of funnelling 8 GPUs' traffic through rank 0.
    # `--ingress rank0` keeps the single node-wide ingress on rank 0.  Built
    # BEFORE the engine: the engine's device warm-up (EngineRunner.build) is then
    # followed only by the W warm-up steps, not by host-side set-up.
    from concurrent.futures import ThreadPoolExecutor

    drivers = range(n) if args.ingress == "per-rank" else [0]
    n_drv = len(drivers)
    is_driver = rank in drivers
    G = args.ingress_threads or (1 if args.ingress == "per-rank" else min(4, max(1, n // 2)))
    if is_driver:
        g = torch.Generator().manual_seed(1234 + rank)
        payloads = []
        for _ in range(256):
            ids = torch.randint(1, cfg.vocab_size, (args.seq,), generator=g, dtype=torch.int32)
            ids[0] = 101
            payloads.append(ids.numpy().tobytes())
        clients = [rjob.Client(job, seed=1234 + 64 * rank + i) for i in range(G)]
        gens = [rjob.LoadGen(c, 0, payloads) for c in clients]
        pool = ThreadPoolExecutor(G)
        slot = list(drivers).index(rank)
    os.environ.setdefault("RDB_TUNE_STREAMS", str(args.tune_streams or args.compute_streams))
    if echo:
        runner = _EchoRunner(rjob.EchoServer(job, rank, [rank], args.max_batch, args.echo_service_us, 0.0, 8))
    else:
        from ray_dynamic_batching_amd.runtime.engine import resolve_tile_table

        model = BertForSequenceClassification(cfg, device="cuda", backend=args.backend)
        # replay the tile table selected on MI355X for this configuration
        # (ops/tuned/README.md) instead of tuning at start-up: start-up tuning is
        # timed on a few replays, so its picks -- and the served throughput --
        # vary run to run by up to ~10 %.  The same resolution as a Serve-deployed
        # replica's EngineConfig.tile_table="auto"; RDB_TUNE_FILE set by the caller wins.
        tile_table = os.environ.get("RDB_TUNE_FILE") or resolve_tile_table(
            args.tile_table, model, args.max_batch, args.compute_streams, args.pipeline_depth)
        if tile_table:
            os.environ["RDB_TUNE_FILE"] = tile_table
        spec = SessionSpec(model=model, queue=rank, max_batch=args.max_batch, max_wait_s=args.max_wait_ms / 1e3)
        runner = EngineRunner(name, rank, [spec], pipeline_depth=args.pipeline_depth,
                              compute_streams=args.compute_streams, batch_policy=args.batch_policy,
                              tile_table=tile_table).build()
    runner.start()
    if not echo and getattr(runner, "tuning_changes", None):
        print(json.dumps({"rank": rank, "in_context_tile_changes": {str(k[2:5]): v for k, v in runner.tuning_changes.items()}}),
              file=sys.stderr, flush=True)
    barrier()

    result = {}
    per_step = args.max_batch * n
    if is_driver:
        def share(total, k, i):
            return total // k + (1 if i < total % k else 0)

        conc = share(args.concurrency * n, n_drv, slot)
        rate = args.rate * n / n_drv

        def drive(total, record, timeout_s):
            total = share(total, n_drv, slot)
            futs = [pool.submit(gens[i].run, share(total, G, i), max(1, share(conc, G, i)), rate / G, 0.0,
                                record, timeout_s) for i in range(G)]
            res = [f.result() for f in futs]
            if record:
                for lg_i in gens[1:]:
                    gens[0].merge_from(lg_i)
            return {k: sum(r[k] for r in res) for k in ("ok", "completed", "dropped", "errors", "issued")}

        drive(args.warmup * per_step, False, 600.0)
    stamps = None
    if args.stamps_out:
        from ray_dynamic_batching_amd import ops as _ops_mod

        stamps = _ops_mod.BlockStamps()
    barrier()
    sync()
    if stamps is not None:
        stamps.reset()
    if rank == 0:
        job.reset_stats()
        rep0 = [job.replica_stats(r) for r in range(n)]
    barrier()
    t0 = time.perf_counter()
    if is_driver:
        result = drive(args.steps * per_step, True, 1200.0)
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if stamps is not None:
        import numpy as np

        path = args.stamps_out if world == 1 else args.stamps_out.replace(".npy", f".rank{rank}.npy")
        np.save(path, stamps.read())
        print(json.dumps({"rank": rank, "stamps": path, "dropped": stamps.dropped}), file=sys.stderr, flush=True)
        stamps.close()
    barrier()
    err = runner.error()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=host_pg)
        elapsed = t.item()
        if n_drv > 1:
            # whole-node counts and latency histogram: every rank's ingress folded into rank 0's
            counts = [result.get(k, 0) for k in ("ok", "completed", "dropped", "errors", "issued")]
            c = torch.tensor(counts, dtype=torch.float64)
            dist.all_reduce(c, group=host_pg)
            result = dict(zip(("ok", "completed", "dropped", "errors", "issued"), (int(v) for v in c.tolist())))
            states = [None] * world
            dist.all_gather_object(states, gens[0].hist_state() if is_driver else None, group=host_pg)
            if rank == 0:
                for r, st in enumerate(states):
                    if r != 0 and st is not None:
                        gens[0].merge_state(*st)
    placements = [placement]
    if world > 1:
        placements = [None] * world
        dist.all_gather_object(placements, placement, group=host_pg)
    if rank == 0:
        result["latency"] = gens[0].latency()
    if rank == 0 and args.trace_out:
        from ray_dynamic_batching_amd.utils.tracing import collect, export_chrome_trace, summarize

        export_chrome_trace(job, args.trace_out)
        print(json.dumps({"trace_summary": summarize(collect(job))}), file=sys.stderr)
    if rank == 0:
        rep1 = [job.replica_stats(r) for r in range(n)]
        rep = [{k: rep1[i][k] - rep0[i][k] for k in ("batches", "batch_items", "busy_ms")} for i in range(n)]
        ok = result["ok"]
        value = ok / elapsed
        lat = result["latency"]
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "req/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random token ids, random-init weights)",
            "config": {"model": "bert-base (12L, 768H, 12 heads), sequence classification",
                       "global_batch": args.max_batch * n, "seq_len": args.seq,
                       "parallelism": f"dp{n}", "max_batch": args.max_batch,
                       "batch_wait_timeout_ms": args.max_wait_ms, "backend": args.backend,
                       "batch_policy": args.batch_policy, "compute_streams": args.compute_streams,
                       "pipeline_depth": args.pipeline_depth,
                       "hip_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "load": (f"closed-loop x{args.concurrency}/GPU" if args.rate <= 0 else f"poisson {args.rate}/s/GPU"),
                       "tile_table": os.path.basename(os.environ.get("RDB_TUNE_FILE", "")) or "tuned at start-up"},
            "p50_ms": round(lat["p50_ms"], 3),
            "p99_ms": round(lat["p99_ms"], 3),
            "p999_ms": round(lat["p999_ms"], 3),
            "mean_ms": round(lat["mean_ms"], 3),
            "completed": result["completed"],
            "dropped": result["dropped"],
            "errors": result["errors"],
            "mean_batch": round(sum(r["batch_items"] for r in rep) / max(1, sum(r["batches"] for r in rep)), 2),
            "gpu_busy_frac": round(sum(r["busy_ms"] for r in rep) / (n * elapsed * 1e3), 3) if elapsed > 0 else None,
            "per_replica_requests": [r["batch_items"] for r in rep],
            "ingress": f"{args.ingress} x{G} thread(s)",
            "placement": placements,
        }
        if os.environ.get("RDB_ABLATE"):
            line["metric"] = f"ABLATION (skips {os.environ['RDB_ABLATE']}: wrong outputs, not a measurement): " + METRIC
            line["vs_baseline"] = None
        if args.rehearse_one_gpu:
            line["metric"] = "REHEARSAL (all ranks on one GPU, gloo): " + METRIC
            line["vs_baseline"] = None
        if args.stamps_out:
            line["metric"] = "DIAGNOSTIC (block-stamp kernel build; barriers added per block): " + METRIC
            line["vs_baseline"] = None
        if err:
            line["engine_error"] = err
        print(json.dumps(line), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(line, f, indent=1)
    if is_driver:
        pool.shutdown()
    runner.stop()
    barrier()
    job.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
