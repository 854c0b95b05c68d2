"""Single-GPU serving curves through the native replica engine:
req/s vs p50/p99 latency for any servable model of the zoo.

BASELINE config 2 (ResNet-50 fp16, 1 GPU, dyn-batch <= 32 / 5 ms, Poisson; one
replica engine running three batches at a time on three compute streams, like bench.py):
    python bench/serve_bench.py --model resnet50 --rates 8000,16000,32000,46000
    python bench/serve_bench.py --model resnet50 --closed 128   # a 4th batch forms while 3 run
Closed-loop saturation throughput:
    python bench/serve_bench.py --model bert-base --closed 96
The same replica deployed through Serve (serve.run(model_deployment(...)) in
process mode: node agent, NUMA placement, EngineConfig from the deployment),
driven by native clients on the deployment's own shm queues:
    python bench/serve_bench.py --model bert-base --closed 96 --via-serve

Requests carry synthetic inputs of the model's per-request shape (uint8
224x224x3 images for the CNNs / ViT, 128 token ids for BERT) through the shm
rings -> zero-copy H2D gather -> hipGraph replay -> completion ring, exactly
as in bench.py.  Latency is client-side end to end, measured from the
scheduled Poisson arrival (so client-side backlog counts).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--rates", default="", help="comma-separated Poisson rates (req/s)")
    ap.add_argument("--closed", type=int, default=0, help="closed-loop concurrency (0 = off)")
    ap.add_argument("--seconds", type=float, default=5.0, help="measurement length per point")
    ap.add_argument("--max-batch", type=int, default=32)
    ap.add_argument("--max-wait-ms", type=float, default=5.0)
    ap.add_argument("--backend", default="hip")
    ap.add_argument("--pipeline-depth", type=int, default=6)
    ap.add_argument("--compute-streams", type=int, default=3, help="batches executing concurrently on the GPU")
    ap.add_argument("--via-serve", action="store_true",
                    help="deploy the replica with serve.run(serve.model_deployment(...)) instead of building an "
                         "EngineRunner here; the load generator drives the deployment's queues")
    ap.add_argument("--replicas", type=int, default=1, help="--via-serve: num_replicas (one GPU each)")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--stamps-out", default="", help="diagnostic: block-stamp records of the closed-loop run (.npy; needs "
                    "the RDB_BLOCK_STAMPS kernel build via RDB_OPS_SO, bench/stamp_timeline.py reads them)")
    a = ap.parse_args(argv)
    from ray_dynamic_batching_amd.runtime.queues import ensure_hw_queues

    ensure_hw_queues(a.compute_streams)       # one HIP hardware queue per engine stream, before HIP starts

    import numpy as np
    import torch

    from ray_dynamic_batching_amd import models
    from ray_dynamic_batching_amd.runtime import job as rjob
    from ray_dynamic_batching_amd.runtime.engine import EngineRunner, SessionSpec, resolve_tile_table

    if a.via_serve:
        return _via_serve(a)
    torch.cuda.set_device(0)
    m = models.create(a.model, device="cuda", backend=a.backend)
    # replay the tile table shipped for this (model, max batch, streams, depth) when there is
    # one (ops/tuned/README.md; the resolution a Serve replica's tile_table="auto" uses);
    # RDB_TUNE_FILE set by the caller wins
    table = os.environ.get("RDB_TUNE_FILE") or resolve_tile_table("auto", m, a.max_batch, a.compute_streams,
                                                                   a.pipeline_depth)
    if table:
        os.environ["RDB_TUNE_FILE"] = table
    in_bytes = int(np.prod(m.input_shape)) * torch.tensor([], dtype=m.input_dtype).element_size()
    name = rjob.unique_job_name("sbench")
    cap = 512 if in_bytes > 8192 else 4096
    j = rjob.Job(name, create=True, n_replicas=1, n_queues=1, n_clients=2, req_capacity=cap,
                 req_slot_bytes=in_bytes + 64, cmp_capacity=8192, cmp_slot_bytes=128)
    j.configure_queue(0, 0, 0, cap, 0.0, True)
    runner = EngineRunner(name, 0, [SessionSpec(model=m, queue=0, max_batch=a.max_batch,
                                                max_wait_s=a.max_wait_ms / 1e3)],
                          pipeline_depth=a.pipeline_depth, compute_streams=a.compute_streams,
                          tile_table=table).build()
    runner.start()
    try:
        x = m.example_input(64, seed=3).cpu()
        payloads = [x[i].contiguous().numpy().tobytes() for i in range(64)]
        points = _drive(a, j, 0, payloads, in_bytes, stats=lambda: [j.replica_stats(0)])
        assert runner.error() == "", runner.error()
    finally:
        runner.stop()
        j.close()
    _report(a, points, os.path.basename(os.environ.get("RDB_TUNE_FILE", "")) or "tuned at start-up")


def _drive(a, j, model_id, payloads, in_bytes, stats):
    """Warm-up, then the closed-loop and Poisson points through a native load
    generator on job ``j`` routing over the queues of ``model_id``."""
    import numpy as np
    import torch

    from ray_dynamic_batching_amd.runtime import job as rjob

    points = []
    c = rjob.Client(j)
    lg = rjob.LoadGen(c, model_id, payloads)
    lg.run(2000 if in_bytes <= 8192 else 500, 64, 0.0, 0.0, False, 300.0)
    runs = [("closed", a.closed)] if a.closed else []
    runs += [("poisson", float(r)) for r in a.rates.split(",") if r]
    for kind, v in runs:
        j.reset_stats()
        before = stats()
        if kind == "closed":
            total = int(max(2000, 20000 * a.seconds / 5))
            stamps = None
            if a.stamps_out:
                from ray_dynamic_batching_amd import ops as _ops_mod

                stamps = _ops_mod.BlockStamps()
                total = min(total, 4096)          # ~30k records per batch: stay inside the stamp buffer
                torch.cuda.synchronize()
                stamps.reset()
            res = lg.run(total, int(v), 0.0, 0.0, True, 600.0)
            if stamps is not None:
                torch.cuda.synchronize()
                np.save(a.stamps_out, stamps.read())
                print(json.dumps({"stamps": a.stamps_out, "dropped": stamps.dropped}), flush=True)
                stamps.close()
        else:
            total = int(v * a.seconds)
            res = lg.run(total, 0, v, 0.0, True, 600.0)
        after = stats()
        items = sum(x["batch_items"] - y["batch_items"] for x, y in zip(after, before))
        nb = sum(x["batches"] - y["batches"] for x, y in zip(after, before))
        lat = res["latency"]
        pt = {"load": kind, "offered": v, "req_per_s": round(res["ok"] / res["elapsed_s"], 1),
              "p50_ms": round(lat["p50_ms"], 3), "p99_ms": round(lat["p99_ms"], 3),
              "p999_ms": round(lat["p999_ms"], 3), "mean_batch": round(items / max(1, nb), 2),
              "ok": res["ok"], "errors": res.get("errors", 0)}
        points.append(pt)
        print(json.dumps(pt), flush=True)
    return points


def _report(a, points, table, **extra):
    out = {"model": a.model, "backend": a.backend, "max_batch": a.max_batch, "max_wait_ms": a.max_wait_ms,
           "pipeline_depth": a.pipeline_depth, "compute_streams": a.compute_streams, "tile_table": table,
           "via_serve": bool(a.via_serve), "points": points, **extra}
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


def _via_serve(a):
    """serve.run(serve.model_deployment(factory, num_replicas=R, num_gpus=1)) in
    process mode -- the node agent spawns the replica process(es) pinned to their
    GPUs' NUMA CPUs, each builds its engine from the deployment's EngineConfig --
    then native clients drive the deployment's queues (the router's pow-2 choice
    over its replicas' queue depths), exactly like the direct path's load."""
    import numpy as np

    from ray_dynamic_batching_amd import models, serve
    from ray_dynamic_batching_amd.models import factories
    from ray_dynamic_batching_amd.serve.controller import get_controller

    fac = {"bert-base": factories.bert_base(backend=a.backend), "resnet50": factories.resnet50(backend=a.backend),
           "vit-b16": factories.vit_b16(backend=a.backend)}[a.model]
    dep = serve.model_deployment(fac, "model", max_batch_size=a.max_batch, batch_wait_timeout_s=a.max_wait_ms / 1e3,
                                 num_replicas=a.replicas, ray_actor_options={"num_gpus": 1},
                                 max_ongoing_requests=4096, health_check_timeout_s=120,
                                 engine=dict(compute_streams=a.compute_streams, pipeline_depth=a.pipeline_depth))
    try:
        serve.run(dep.bind(), name="sbench", mode="process")
        ctrl = get_controller()
        st = ctrl.apps["sbench"]["model"]
        j = ctrl.jobs["sbench"]
        # inputs of the model's per-request shape, made on the CPU (this process never touches the GPU)
        m = models.create(a.model, device="cpu", backend="torch") if a.model != "bert-base" else None
        if m is not None:
            x = m.example_input(64, seed=3).cpu()
            payloads = [x[i].contiguous().numpy().tobytes() for i in range(64)]
        else:
            rng = np.random.default_rng(3)
            ids = rng.integers(1, 30522, size=(64, 128)).astype(np.int32)
            ids[:, 0] = 101
            payloads = [ids[i].tobytes() for i in range(64)]
        in_bytes = len(payloads[0])
        points = _drive(a, j, st.model_id, payloads, in_bytes,
                        stats=lambda: [j.replica_stats(s) for s in st.slots])
        logs = sorted(os.path.join(ctrl.workdir, f) for f in os.listdir(ctrl.workdir) if f.endswith(".log"))
        engine_line = ""
        for lp in logs:
            with open(lp, errors="replace") as f:
                for line in f:
                    if "engine:" in line:
                        engine_line = line.strip()
        places = [p for p in (ctrl.agent.list() or [])]
        _report(a, points, engine_line.split("tile table ")[-1] if engine_line else "?",
                replicas=a.replicas, replica_engine_log=engine_line,
                agent_procs=[dict(owner=p.get("owner"), restarts=p.get("restarts")) for p in places])
    finally:
        serve.shutdown()


if __name__ == "__main__":
    main()
