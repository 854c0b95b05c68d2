"""Runtime microbenchmarks: the request path with the GPU taken out.

Mirrors Ray's core microbenchmarks that bound the reference's request path
(release/perf_metrics/microbenchmark.json:2-13,78-81 -- 1:1 sync actor calls
1,934.5/s, 1:1 async 8,761.3/s, n:n async 27,090.4/s on m5.16xlarge; the fork
pays 3 such RPCs per request on ingress) and adds the batched
serving path used by bench.py (N queues, dyn-batch <= 32), so the N-GPU bench
can be checked for load-generator headroom.

    python bench/runtime_microbench.py [--queues 8] [--seconds 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ray_dynamic_batching_amd.runtime import job as rjob  # noqa: E402

RAY_REF = {"1:1 sync": 1934.5, "1:1 async": 8761.3, "n:n async": 27090.4}


def _run(n_queues, n_clients, concurrency, max_batch, total, service_us=0.0, per_item_us=0.0):
    name = rjob.unique_job_name("ubench")
    j = rjob.Job(name, create=True, n_replicas=n_queues, n_queues=n_queues, n_clients=n_clients,
                 req_capacity=4096, req_slot_bytes=512, cmp_capacity=8192, cmp_slot_bytes=64)
    for q in range(n_queues):
        j.configure_queue(q, q, 0, 4096, 0.0, True)
    servers = [rjob.EchoServer(j, q, [q], max_batch, service_us, per_item_us) for q in range(n_queues)]
    for s in servers:
        s.start()
    payload = [bytes(512 - 64)]
    try:
        clients = [rjob.Client(j, c) for c in range(n_clients)]
        gens = [rjob.LoadGen(c, 0, payload) for c in clients]
        for g in gens:  # warmup
            g.run(min(2000, total // 10 + 1), concurrency, 0.0, 0.0, False, 30.0)
        res = [None] * n_clients

        def go(i):
            res[i] = gens[i].run(total, concurrency, 0.0, 0.0, True, 120.0)

        ts = [threading.Thread(target=go, args=(i,)) for i in range(n_clients)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        dt = time.perf_counter() - t0
        ok = sum(r["ok"] for r in res)
        batches = sum(j.replica_stats(q)["batches"] for q in range(n_queues))
        items = sum(j.replica_stats(q)["batch_items"] for q in range(n_queues))
        return {"req_per_s": ok / dt, "p50_us": res[0]["latency"]["p50_ms"] * 1e3, "p99_us": res[0]["latency"]["p99_ms"] * 1e3,
                "mean_batch": items / max(1, batches), "ok": ok}
    finally:
        for s in servers:
            s.stop()
        j.close()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--queues", type=int, default=8)
    ap.add_argument("--total", type=int, default=100000)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)
    out = {}
    out["1:1 sync"] = _run(1, 1, 1, 1, a.total // 5)
    out["1:1 async"] = _run(1, 1, 100, 1, a.total)
    out["n:n async"] = _run(4, 4, 100, 1, a.total // 2)
    out[f"serve path {a.queues}q dyn-batch<=32"] = _run(a.queues, 1, 96 * a.queues, 32, a.total * 2)
    for k, v in out.items():
        ref = RAY_REF.get(k)
        v["ray_ref_per_s"] = ref
        v["x_vs_ray"] = (v["req_per_s"] / ref) if ref else None
        print(f"{k:34s} {v['req_per_s']:>12,.0f} /s  p50 {v['p50_us']:8.1f} us  p99 {v['p99_us']:8.1f} us  "
              f"batch {v['mean_batch']:5.1f}" + (f"  ({v['x_vs_ray']:.1f}x Ray)" if ref else ""))
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
