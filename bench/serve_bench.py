"""Single-GPU serving curves through the native replica engine:
req/s vs p50/p99 latency for any servable model of the zoo.

BASELINE config 2 (ResNet-50 fp16, 1 GPU, dyn-batch <= 32 / 5 ms, Poisson; one
replica engine running two batches at a time on two compute streams, like bench.py):
    python bench/serve_bench.py --model resnet50 --rates 2000,4000,8000,12000
Closed-loop saturation throughput:
    python bench/serve_bench.py --model bert-base --closed 96

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
    ap.add_argument("--pipeline-depth", type=int, default=4)
    ap.add_argument("--compute-streams", type=int, default=2, help="batches executing concurrently on the GPU")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--stamps-out", default="", help="diagnostic: block-stamp records of the closed-loop run (.npy; needs "
                    "the RDB_BLOCK_STAMPS kernel build via RDB_OPS_SO, bench/stamp_timeline.py reads them)")
    a = ap.parse_args(argv)

    import numpy as np
    import torch

    from ray_dynamic_batching_amd import models
    from ray_dynamic_batching_amd.runtime import job as rjob
    from ray_dynamic_batching_amd.runtime.engine import EngineRunner, SessionSpec

    torch.cuda.set_device(0)
    # replay the tile table shipped for this (model, max batch, depth) when there is one
    # (ops/tuned/README.md); RDB_TUNE_FILE set by the caller wins
    tuned = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ray_dynamic_batching_amd",
                         "ops", "tuned")
    shipped = os.path.join(tuned, f"mi355x_{a.model}_B{a.max_batch}_cs{a.compute_streams}_d{a.pipeline_depth}.json")
    if not os.path.exists(shipped) and a.compute_streams == 1:
        shipped = os.path.join(tuned, f"mi355x_{a.model}_B{a.max_batch}_d{a.pipeline_depth}.json")   # round-3 name
    if a.backend == "hip" and "RDB_TUNE_FILE" not in os.environ and os.path.exists(shipped):
        os.environ["RDB_TUNE_FILE"] = shipped
    m = models.create(a.model, device="cuda", backend=a.backend)
    in_bytes = int(np.prod(m.input_shape)) * torch.tensor([], dtype=m.input_dtype).element_size()
    name = rjob.unique_job_name("sbench")
    cap = 512 if in_bytes > 8192 else 4096
    j = rjob.Job(name, create=True, n_replicas=1, n_queues=1, n_clients=2, req_capacity=cap,
                 req_slot_bytes=in_bytes + 64, cmp_capacity=8192, cmp_slot_bytes=128)
    j.configure_queue(0, 0, 0, cap, 0.0, True)
    runner = EngineRunner(name, 0, [SessionSpec(model=m, queue=0, max_batch=a.max_batch,
                                                max_wait_s=a.max_wait_ms / 1e3)],
                          pipeline_depth=a.pipeline_depth, compute_streams=a.compute_streams).build()
    runner.start()
    points = []
    try:
        x = m.example_input(64, seed=3).cpu()
        payloads = [x[i].contiguous().numpy().tobytes() for i in range(64)]
        c = rjob.Client(j)
        lg = rjob.LoadGen(c, 0, payloads)
        lg.run(2000 if in_bytes <= 8192 else 500, 64, 0.0, 0.0, False, 300.0)
        runs = [("closed", a.closed)] if a.closed else []
        runs += [("poisson", float(r)) for r in a.rates.split(",") if r]
        for kind, v in runs:
            j.reset_stats()
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
            rs = j.replica_stats(0)
            lat = res["latency"]
            pt = {"load": kind, "offered": v, "req_per_s": round(res["ok"] / res["elapsed_s"], 1),
                  "p50_ms": round(lat["p50_ms"], 3), "p99_ms": round(lat["p99_ms"], 3),
                  "p999_ms": round(lat["p999_ms"], 3), "mean_batch": round(rs["batch_items"] / max(1, rs["batches"]), 2),
                  "ok": res["ok"], "errors": res.get("errors", 0)}
            points.append(pt)
            print(json.dumps(pt), flush=True)
        assert runner.error() == "", runner.error()
    finally:
        runner.stop()
        j.close()
    out = {"model": a.model, "backend": a.backend, "max_batch": a.max_batch, "max_wait_ms": a.max_wait_ms,
           "pipeline_depth": a.pipeline_depth, "compute_streams": a.compute_streams,
           "tile_table": os.path.basename(os.environ.get("RDB_TUNE_FILE", "")) or "tuned at start-up",
           "points": points}
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
