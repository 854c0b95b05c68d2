"""BASELINE config 4: Llama-3-8B bf16, tensor parallel over the node's GPUs
(one process per GPU, RCCL over xGMI), prefill of <= 8 prompts.

Each rank holds a 1/TP shard (column-parallel QKV / gate-up, row-parallel O /
down with an all-reduce each, vocab-parallel LM head + all-gathered argmax).
The whole prefill (kernels + RCCL collectives) is captured in ONE hipGraph per
batch bucket and replayed; rank 0 is the serving front: it batches prompts,
broadcasts the token ids over RCCL and returns next-token ids.

    python bench/llama_tp_bench.py                      # TP=1 on one GPU
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/llama_tp_bench.py
Reports per-batch prefill latency (p50 over replays) and prompts/s for
batches 1, 2, 4, 8 of --seq tokens.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--batches", default="1,2,4,8")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--serve", action="store_true", help="serve prompts through the shm rings (TPReplica)")
    ap.add_argument("--requests", type=int, default=400)
    ap.add_argument("--concurrency", type=int, default=16)
    ap.add_argument("--loop", default="native", choices=["native", "python"],
                    help="--serve: the native engine TP loop (NativeTP) or the Python TPReplica loop")
    ap.add_argument("--max-wait-ms", type=float, default=2.0, help="--serve: first-arrival batch timeout")
    ap.add_argument("--compute-streams", type=int, default=1,
                    help="--serve --loop native at TP = 1: batches overlapping on the GPU (TP > 1 runs one)")
    ap.add_argument("--pipeline-depth", type=int, default=2)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--checkpoint", default="", help="Hugging Face Llama checkpoint dir (each rank loads its shard)")
    ap.add_argument("--allreduce", default="xgmi", choices=["xgmi", "rccl"],
                    help="TP all-reduce: custom push-based xGMI kernel (fused RMSNorm) or RCCL")
    a = ap.parse_args(argv)
    from ray_dynamic_batching_amd.runtime.queues import ensure_hw_queues

    ensure_hw_queues(a.compute_streams)       # one HIP hardware queue per engine stream, before HIP starts

    import torch
    import torch.distributed as dist

    from ray_dynamic_batching_amd.models.llama import LlamaConfig, LlamaTP
    from ray_dynamic_batching_amd.parallel import collective as col

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        col.init_collective_group(world, rank, "nccl", "tp")
        if a.allreduce == "xgmi":
            # 8 prompts x seq tokens x hidden bf16 per all-reduce
            col.enable_xgmi("tp", max_elems=8 * a.seq * 4096)
    cfg = LlamaConfig.llama3_8b(seq_len=a.seq, layers=a.layers)
    t0 = time.time()
    if a.checkpoint:
        from ray_dynamic_batching_amd.models.weights import llama_from_hf

        m = llama_from_hf(a.checkpoint, seq_len=a.seq, tp_rank=rank, tp_size=world,
                          group_name="tp" if world > 1 else None, device=f"cuda:{local}")
        cfg = m.cfg
    else:
        m = LlamaTP(cfg, rank, world, "tp" if world > 1 else None, device=f"cuda:{local}", init="shard")
    init_s = time.time() - t0
    if a.serve:
        return _serve(a, m, world, rank)
    results = []
    for b in [int(x) for x in a.batches.split(",")]:
        ids = m.example_input(b, seed=b)
        if world > 1:                      # rank 0 is the front end: it owns the prompts
            col.broadcast(ids, 0, "tp")
        with torch.no_grad():
            for _ in range(2):
                out = m(ids)
            torch.cuda.synchronize()
            if not a.no_graph:
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    m(ids)
                torch.cuda.current_stream().wait_stream(side)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    out = m(ids)
                step = g.replay
            else:
                def step():
                    m(ids)
            if world > 1:
                dist.barrier()
            times = []
            for _ in range(a.iters):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                step()
                e.record()
                torch.cuda.synchronize()
                times.append(s.elapsed_time(e))
        times.sort()
        p50 = times[len(times) // 2]
        t = torch.tensor([p50], device="cuda")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        p50 = t.item()
        tokens = b * a.seq
        flops = 2 * 8.0e9 * tokens * (a.layers / 32)
        results.append(dict(batch=b, prefill_ms=round(p50, 3), prompts_per_s=round(b / p50 * 1e3, 1),
                            tokens_per_s=round(tokens / p50 * 1e3, 1), tflops_whole_node=round(flops / p50 / 1e9, 1),
                            next_token=int(out[0, 0].item())))
    if rank == 0:
        rep = dict(metric="Llama-3-8B bf16 TP prefill latency", tp=world, allreduce=a.allreduce if world > 1 else "none", seq_len=a.seq, layers=a.layers,
                   graph=not a.no_graph, init_s=round(init_s, 1), results=results,
                   data="synthetic token ids, random-init weights")
        print(json.dumps(rep), flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                json.dump(rep, f, indent=1)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _serve(a, m, world, rank):
    """Config 4 serving: prompts -> shm queue -> rank-0 batching (<= 8) -> RCCL
    broadcast -> graph replay on every TP rank -> next-token completions."""
    import threading

    import torch
    import torch.distributed as dist

    from ray_dynamic_batching_amd.runtime import job as rjob
    from ray_dynamic_batching_amd.runtime.tp_replica import TPReplica

    name = f"llama_tp_{os.environ.get('MASTER_PORT', os.getpid())}"
    job = None
    if rank == 0:
        job = rjob.Job(name, create=True, n_replicas=1, n_queues=1, n_clients=2, req_capacity=1024,
                       req_slot_bytes=a.seq * 4, cmp_capacity=2048, cmp_slot_bytes=64)
        job.configure_queue(0, 0, 0, 1024, 0.0, True)
    buckets = [1, 2, 4, 8]
    if a.loop == "native":
        return _serve_native(a, m, world, rank, name, job, buckets)
    rep = TPReplica(m, name if rank == 0 else None, 0, 0, buckets, "tp" if world > 1 else None,
                    ring=f"{name}_ring").capture()
    if world > 1:
        dist.barrier()
    if rank != 0:
        while rep.step() >= 0:
            pass
        dist.barrier()
        dist.destroy_process_group()
        return
    ids = m.example_input(64, seed=3).cpu()
    payloads = [ids[i].numpy().tobytes() for i in range(64)]
    res = {}

    def drive():
        c = rjob.Client(job, 1)
        lg = rjob.LoadGen(c, 0, payloads)
        lg.run(min(64, a.requests), a.concurrency, 0.0, 0.0, False, 600.0)   # warmup
        res.update(lg.run(a.requests, a.concurrency, 0.0, 0.0, True, 600.0))

    t = threading.Thread(target=drive)
    t.start()
    while t.is_alive():
        rep.step(0.01)
    rep.stop_all()
    lat = res["latency"]
    rep_out = dict(metric="Llama-3-8B bf16 TP prefill serving (<= 8 prompts / batch)", tp=world, allreduce=a.allreduce if world > 1 else "none", seq_len=a.seq,
                   layers=a.layers, prompts_per_s=round(res["ok"] / res["elapsed_s"], 1),
                   p50_ms=round(lat["p50_ms"], 3), p99_ms=round(lat["p99_ms"], 3), ok=res["ok"],
                   mean_batch=round(job.replica_stats(0)["batch_items"] / max(1, job.replica_stats(0)["batches"]), 2),
                   data="synthetic token ids, random-init weights")
    print(json.dumps(rep_out), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(rep_out, f, indent=1)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    job.close()


def _serve_native(a, m, world, rank, name, job, buckets):
    """The native TP loop (runtime/tp_replica.py NativeTP): rank 0's engine forms
    batches (first-arrival timeout), gathers them zero-copy on its copy stream and
    publishes them on the group's broadcast ring; followers copy + replay the same
    bucket graph; batch k+1 is formed and copied while batch k computes."""
    import torch.distributed as dist

    from ray_dynamic_batching_amd.runtime import job as rjob
    from ray_dynamic_batching_amd.runtime.tp_replica import NativeTP

    if world > 1:
        dist.barrier()                        # rank 0 created the job
    ntp = NativeTP(m, name, 0, buckets, rank, world, "tp" if world > 1 else None, f"{name}_ring", 8,
                   a.max_wait_ms / 1e3, pipeline_depth=max(a.pipeline_depth, a.compute_streams),
                   compute_streams=a.compute_streams if world == 1 else 1)
    if world == 1:
        ntp.unlink()                          # no follower to wait for: drop the ring's name now
    ntp.start()
    if world > 1:
        dist.barrier()
    if rank != 0:
        while ntp.check() == "":
            time.sleep(0.05)
        ntp.stop()
        dist.barrier()
        dist.destroy_process_group()
        return
    ids = m.example_input(64, seed=3).cpu()
    payloads = [ids[i].numpy().tobytes() for i in range(64)]
    c = rjob.Client(job, 1)
    lg = rjob.LoadGen(c, 0, payloads)
    lg.run(min(64, a.requests), a.concurrency, 0.0, 0.0, False, 600.0)   # warmup
    job.reset_stats()
    res = lg.run(a.requests, a.concurrency, 0.0, 0.0, True, 600.0)
    err = ntp.check()
    st = job.replica_stats(0)
    ntp.stop()                                # STOP record: the followers leave
    lat = res["latency"]
    rep_out = dict(metric="Llama-3-8B bf16 TP prefill serving (<= 8 prompts / batch)", loop="native engine",
                   compute_streams=a.compute_streams if world == 1 else 1,
                   tp=world, allreduce=a.allreduce if world > 1 else "none", seq_len=a.seq, layers=a.layers,
                   prompts_per_s=round(res["ok"] / res["elapsed_s"], 1), p50_ms=round(lat["p50_ms"], 3),
                   p99_ms=round(lat["p99_ms"], 3), ok=res["ok"], errors=res.get("errors", 0),
                   mean_batch=round(st["batch_items"] / max(1, st["batches"]), 2), engine_error=err,
                   data="synthetic token ids, random-init weights")
    print(json.dumps(rep_out), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(rep_out, f, indent=1)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    job.close()


if __name__ == "__main__":
    main()
