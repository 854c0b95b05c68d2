"""Reference-equivalent baseline for the headline metric.

The reference publishes no serving numbers, so we measure what its stack does
on the same MI355X: Ray Serve's ``@serve.batch(max_batch_size=32,
batch_wait_timeout_s)`` semantics (our faithful re-implementation,
serve/batching.py <- python/ray/serve/batching.py:529-678) wrapped around an
eager PyTorch-ROCm BERT-base forward (``torch.stack(...).cuda()`` -> model ->
``.cpu()``, as in the fork's GPUWorker.process_batch, scheduler.py:435-475).
Everything runs in ONE process on one asyncio loop with zero Ray RPC / plasma
hops, so this is an UPPER bound on what the reference could reach per GPU
(whole node = N x this number at best).

    python bench/baseline_serve.py [--backend torch|hip] [--requests 20000]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=20000)
    ap.add_argument("--warmup", type=int, default=2000)
    ap.add_argument("--concurrency", type=int, default=96)
    ap.add_argument("--max-batch", type=int, default=32)
    ap.add_argument("--max-wait-ms", type=float, default=5.0)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--backend", default="torch", choices=["torch", "hip"],
                    help="torch = eager PyTorch-ROCm (reference); hip = our kernels, eager (no graphs, no engine)")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)

    import numpy as np
    import torch

    from ray_dynamic_batching_amd import serve
    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification

    model = BertForSequenceClassification(BertConfig(seq_len=a.seq, layers=a.layers), device="cuda",
                                          backend=a.backend)
    ids = model.example_input(256, seed=1).cpu()
    reqs = [ids[i] for i in range(256)]

    class Replica:
        @serve.batch(max_batch_size=a.max_batch, batch_wait_timeout_s=a.max_wait_ms / 1e3)
        async def __call__(self, xs):
            x = torch.stack(xs).cuda()
            with torch.no_grad():
                y = model(x)
            y = y.cpu()
            return list(y.unbind(0))

    rep = Replica()
    lat = []
    batches = []

    async def client(n, rec):
        for i in range(n):
            t = time.perf_counter()
            await rep(reqs[i % 256])
            if rec:
                lat.append(time.perf_counter() - t)

    async def run(total, rec):
        per = total // a.concurrency
        await asyncio.gather(*[client(per, rec) for _ in range(a.concurrency)])
        return per * a.concurrency

    loop = asyncio.new_event_loop()
    loop.run_until_complete(run(a.warmup, False))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = loop.run_until_complete(run(a.requests, True))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    pending = asyncio.all_tasks(loop)
    for t in pending:
        t.cancel()
    if pending:   # (an idle @serve.batch queue leaves no task behind)
        loop.run_until_complete(asyncio.gather(*pending, return_exceptions=True))
    loop.close()
    lat_ms = np.array(lat) * 1e3
    out = {"metric": "baseline req/s (1 GPU, Python @serve.batch + eager forward, no RPC)", "backend": a.backend,
           "value": round(done / dt, 2), "unit": "req/s", "p50_ms": float(np.percentile(lat_ms, 50)),
           "p99_ms": float(np.percentile(lat_ms, 99)), "mean_ms": float(lat_ms.mean()), "requests": done,
           "concurrency": a.concurrency, "max_batch": a.max_batch, "max_wait_ms": a.max_wait_ms,
           "config": {"model": "bert-base", "seq_len": a.seq, "dtype": "bf16", "layers": a.layers}}
    print(json.dumps(out))
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
