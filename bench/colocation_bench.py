"""BASELINE config 5: ResNet-50 + BERT-base co-located on one MI355X with
per-model queues, the Nexus planner and the native duty-cycle engine.

  1. profile every model on this GPU (graph mode, the fork's CSV contract;
     written to --profile-dir),
  2. plan the requested rates with squishy bin packing (SLO/2 saturate,
     residue merge) -> per-GPU (model, batch, occupancy, duty cycle),
  3. serve open-loop Poisson traffic for every model at once through the
     shm router into the engine's duty-cycle executor,
  4. report per-model throughput, p50/p99 latency, SLO violations and drops.

    python bench/colocation_bench.py --models resnet50,bert-base --rates 4000,8000 --slos 30,30
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,bert-base")
    ap.add_argument("--rates", default="4000,8000", help="req/s per model")
    ap.add_argument("--slos", default="30,30", help="SLO ms per model")
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--batches", default="1,2,4,8,16,32")
    ap.add_argument("--profile-dir", default="gpurun_out/colocation_profiles")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)

    import torch

    from ray_dynamic_batching_amd import models
    from ray_dynamic_batching_amd.planner.profiles import write_profile_csv
    from ray_dynamic_batching_amd.planner.scheduler import SLOScheduler
    from ray_dynamic_batching_amd.profiler.model_profiler import ModelProfiler
    from ray_dynamic_batching_amd.runtime import job as rjob
    from ray_dynamic_batching_amd.serve.servable import TensorCodec

    names = a.models.split(",")
    rates = dict(zip(names, map(float, a.rates.split(","))))
    slos = dict(zip(names, map(float, a.slos.split(","))))
    batches = [int(b) for b in a.batches.split(",")]
    os.makedirs(a.profile_dir, exist_ok=True)
    torch.cuda.set_device(0)

    profiles, codecs, payloads = {}, {}, {}
    for n in names:
        m = models.create(n, device="cuda:0")
        prof = ModelProfiler(m, [m.input_shape], batch_sizes=batches, mode="graph", device="cuda:0",
                             input_fn=lambda b, m=m: [m.example_input(b)], output_dir=a.profile_dir)
        res = prof.profile_all()
        write_profile_csv(os.path.join(a.profile_dir, f"{n}_summary.csv"), res)
        profiles[n] = {r["batch_size"]: dict(avg_latency_ms=r["avg_latency_ms"], peak_memory_mb=r["peak_memory_mb"])
                       for r in res if r["status"] == "success"}
        codecs[n] = TensorCodec.for_model(m)
        x = m.example_input(32, seed=7).cpu()
        payloads[n] = [x[i].contiguous().numpy().tobytes() for i in range(32)]
        del m, prof
        torch.cuda.empty_cache()

    factories = {n: (lambda device, n=n: models.create(n, device=device)) for n in names}
    sched = SLOScheduler(profiles, slos, factories, codecs, num_gpus=1, executor="engine", devices=[0],
                         max_batch={n: max(batches) for n in names}, queue_capacity=4096)
    out = {"models": names, "rates": rates, "slos_ms": slos, "profiles": profiles}
    try:
        sched.check_and_update(rates)
        node = sched.slots[0]
        out["plan"] = dict(duty_cycle_ms=node.duty_cycle if node else None,
                           sessions=[dict(model=s.model_name, batch=s.batch_size, rate=s.request_rate, occupancy=occ)
                                     for s, occ in (node.sessions if node else [])],
                           unplaced_nodes=sched.unplaced_nodes)
        print(json.dumps({"plan": out["plan"]}), flush=True)
        results = {}

        def drive(i, n):
            c = rjob.Client(sched.job, 1 + i)
            lg = rjob.LoadGen(c, sched.model_id(n), payloads[n])
            results[n] = lg.run(int(rates[n] * a.seconds), 0, rates[n], 0.0, True, a.seconds * 4 + 60)

        ts = [threading.Thread(target=drive, args=(i, n)) for i, n in enumerate(names)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        st = sched.get_stats()
        out["results"] = {}
        for n in names:
            r = results[n]
            lat = r["latency"]
            out["results"][n] = dict(offered_rps=rates[n], served_rps=round(r["ok"] / r["elapsed_s"], 1),
                                     p50_ms=round(lat["p50_ms"], 3), p99_ms=round(lat["p99_ms"], 3),
                                     ok=r["ok"], dropped=r["dropped"], errors=r["errors"],
                                     slo_violations=st[n]["slo_violations"],
                                     slo_compliance=round(1 - (st[n]["slo_violations"] + r["dropped"])
                                                          / max(1, r["completed"]), 4))
        out["engine"] = sched.executors[0].stats
        print(json.dumps(out["results"], indent=1), flush=True)
    finally:
        sched.shutdown()
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1, default=str)


if __name__ == "__main__":
    main()
