#!/usr/bin/env python3
"""Config 5 with LIVE re-planning on the GPU: ResNet-50 + BERT-base served by
the native engine executors while their arrival rates ramp, the way the fork
drives its scheduler (293-project/src/test_scheduler.py:57-96: per-model rate
patterns; scheduler.py:763-904: monitor -> 5 % / 10 % thresholds -> re-plan ->
move / load / unload models at batch boundaries).

Each phase offers Poisson traffic per model (native load generators through the
shm router).  A monitor thread measures every model's arrival rate from the
queues' submitted counters (1 s window, sampled every 0.5 s) and calls
``SLOScheduler.check_and_update`` -- measured rates, not the offered schedule,
drive the plan.  Recorded per phase and model: offered / served req/s, p50 /
p99, SLO compliance (completed within the SLO, stale drops counted as
violations), drops, errors; and per run: every re-plan (time, rates,
placement, transfers), model loads / unloads with their load + capture time,
forwarded requests.

``--slots 2`` runs two engine executors ("GPU slots") on the ONE device a box
has, so a plan change can MOVE a model between executors (load + capture on
the new one while the old one serves, then drain, retire, free); ``--slots 1``
keeps both models on one executor (re-plans change batch sizes and duty
shares).  ``--policy priority`` replaces the Nexus duty cycle by the engine's
priority / earliest-deadline-first policy.

    python bench/colocation_replan_bench.py --slots 2 --json-out gpurun_out/replan.json

Offered load: ``--load`` phases as fractions of the device's measured solo
capacity per model (from the same profiles), or absolute ``--phases``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# the fork's ramp (test_scheduler.py:57-96) as fractions of the GPU's measured
# capacity: utilisation 0.3 -> 0.8 -> 0.35, the mix shifting between the models
DEFAULT_LOAD = "0.3:0.5,0.5:0.4,0.7:0.4,0.8:0.5,0.75:0.25,0.35:0.4"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,bert-base")
    ap.add_argument("--slos", default="30,30", help="SLO ms per model")
    ap.add_argument("--phases", default="", help="comma list of per-phase 'rate_m0:rate_m1' req/s (absolute)")
    ap.add_argument("--load", default=DEFAULT_LOAD,
                    help="comma list of per-phase 'utilisation:share_m0' of the GPU's measured capacity (used when "
                         "--phases is empty): model 0 gets share_m0 of the utilisation, model 1 the rest")
    ap.add_argument("--compute-streams", type=int, default=1)
    ap.add_argument("--phase-s", type=float, default=4.0)
    ap.add_argument("--slots", type=int, default=2, help="engine executors (GPU slots) on device 0")
    ap.add_argument("--policy", default="duty", choices=["duty", "priority"])
    ap.add_argument("--batches", default="1,2,4,8,16,32")
    ap.add_argument("--profile-dir", default="gpurun_out/replan_profiles")
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

    # solo capacity of each model on the device (req/s at its best profiled batch)
    capacity = {n: max(b / (r["avg_latency_ms"] / 1e3) for b, r in p.items()) for n, p in profiles.items()}
    if a.phases:
        phases = [dict(zip(names, map(float, p.split(":")))) for p in a.phases.split(",")]
    else:
        phases = []
        for p in a.load.split(","):
            u, sh = map(float, p.split(":"))
            phases.append({names[0]: round(u * sh * capacity[names[0]]),
                           names[1]: round(u * (1 - sh) * capacity[names[1]])})
    utilisation = [round(sum(ph[n] / capacity[n] for n in names), 3) for ph in phases]
    # ``--slots`` executors share ONE device: SLOScheduler plans each as 1/slots
    # of it (its ``slot_share``: per-batch latencies planned slots x longer)
    factories = {n: (lambda device, n=n: models.create(n, device=device)) for n in names}
    sched = SLOScheduler(profiles, slos, factories, codecs, num_gpus=a.slots, executor="engine",
                         devices=[0] * a.slots, max_batch={n: max(batches) for n in names}, queue_capacity=8192,
                         engine_policy=a.policy, compute_streams=a.compute_streams)
    out = dict(models=names, slos_ms=slos, phases=phases, phase_s=a.phase_s, slots=a.slots, policy=a.policy,
               capacity_rps={n: round(c) for n, c in capacity.items()}, offered_utilisation=utilisation,
               slot_note=f"{a.slots} engine executor(s) on one MI355X; the planner sees each as "
                         f"{sched.slot_share:.3g} of it (profiled latencies x {a.slots})",
               profiles={n: {b: r["avg_latency_ms"] for b, r in p.items()} for n, p in profiles.items()})
    print(json.dumps(dict(capacity_rps=out["capacity_rps"], phases=phases, offered_utilisation=utilisation)), flush=True)
    replans, stop = [], threading.Event()
    t0 = time.time()

    def placement():
        return [[(s.model_name, s.batch_size, round(occ, 3)) for s, occ in n.sessions] if n else []
                for n in sched.slots]

    def monitor():
        """measured arrival rates (queue submitted counters) -> check_and_update"""
        def submitted():
            return {m: sum(sched.job.queue_stats(sched.queue_id(g, m))["submitted"] for g in range(sched.num_gpus))
                    for m in names}
        hist = [(time.time(), submitted())]
        while not stop.wait(0.5):
            now, cur = time.time(), submitted()
            hist.append((now, cur))
            while len(hist) > 2 and now - hist[0][0] > 1.0:
                hist.pop(0)
            t_old, old = hist[0]
            rates = {m: (cur[m] - old[m]) / max(1e-3, now - t_old) for m in names}
            n_before = len(sched.changes)
            try:
                changed = sched.check_and_update(rates)
            except Exception as e:  # noqa: BLE001 -- recorded, the run goes on
                replans.append(dict(t=round(now - t0, 2), error=repr(e)))
                continue
            if changed and len(sched.changes) > n_before:
                ch = sched.changes[-1]
                replans.append(dict(t=round(now - t0, 2), measured={m: round(r) for m, r in rates.items()},
                                    transfers=ch.transfers, placement=placement()))

    # initial plan from the first phase's offered rates (the fork starts from its profile-based plan)
    sched.check_and_update(phases[0])
    replans.append(dict(t=0.0, measured=dict(phases[0]), transfers=None, placement=placement(), initial=True))
    mon = threading.Thread(target=monitor, daemon=True)
    mon.start()
    results = []
    try:
        for pi, rates in enumerate(phases):
            res = {}

            def drive(i, n):
                c = rjob.Client(sched.job, 1 + i)
                lg = rjob.LoadGen(c, sched.model_id(n), payloads[n])
                total = int(rates[n] * a.phase_s)
                res[n] = lg.run(total, 8192, rates[n], 0.0, True, a.phase_s * 3 + 30) if total else None

            ts = [threading.Thread(target=drive, args=(i, n)) for i, n in enumerate(names)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            row = dict(phase=pi, t_end=round(time.time() - t0, 2), offered=rates, utilisation=utilisation[pi],
                       models={})
            for n in names:
                r = res[n]
                if r is None:
                    continue
                lat = r["latency"]
                within = r.get("ok", 0)
                row["models"][n] = dict(offered_rps=rates[n], served_rps=round(r["ok"] / r["elapsed_s"], 1),
                                        p50_ms=round(lat["p50_ms"], 3), p99_ms=round(lat["p99_ms"], 3),
                                        ok=r["ok"], dropped=r["dropped"], errors=r["errors"],
                                        completed=r["completed"],
                                        p99_within_slo=lat["p99_ms"] <= slos[n])
                del within
            results.append(row)
            print(json.dumps(row), flush=True)
    finally:
        stop.set()
        mon.join(5)
        st = sched.get_stats()
        out["results"] = results
        out["replans"] = replans
        out["slo_violations"] = {m: st[m]["slo_violations"] for m in names}
        out["executors"] = [dict(loads=e.loads, unloads=e.unloads, rerouted=e.rerouted,
                                 failed_on_unload=getattr(e, "failed_on_unload", 0),
                                 capture_s={k: round(v, 3) for k, v in e.capture_s.items()},
                                 footprint_mb={k: round(v / 2**20, 1) for k, v in e.footprint.items()},
                                 batches=e.runner.stats().get("batches"), backfill=e.runner.stats().get("backfill_batches"))
                            for e in sched.executors]
        tot = {m: dict(completed=sum(r["models"].get(m, {}).get("completed", 0) for r in results),
                       errors=sum(r["models"].get(m, {}).get("errors", 0) for r in results),
                       dropped=sum(r["models"].get(m, {}).get("dropped", 0) for r in results)) for m in names}
        for m in names:
            c = max(1, tot[m]["completed"])
            tot[m]["slo_compliance"] = round(1 - (out["slo_violations"][m] + tot[m]["dropped"]) / c, 4)
        out["totals"] = tot
        sched.shutdown()
    print(json.dumps(dict(replans=len(replans) - 1, totals=out["totals"], executors=out["executors"])), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1, default=str)


if __name__ == "__main__":
    main()
