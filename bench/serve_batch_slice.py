"""SURVEY §7.3 slice: the reference's own GPU idiom on MI355X -- a Python
``@serve.deployment(ray_actor_options={"num_gpus": 1})`` class with a
``@serve.batch`` method on ResNet-50 fp16 (this repo's HIP kernels, eager
forward), deployed with ``serve.run`` and driven by ``handle.remote`` calls
(reference: release/serve_tests/workloads/resnet_50.py:50-57).

Each request is one uint8 224x224x3 image; it crosses the shm ring as raw bytes
(serve/tensor_wire.py: no cloudpickle), the batch is assembled in pinned
memory and copied H2D on a side stream (serve.stack_to_device), the top-5
(probabilities, ids) row comes back raw.  Closed loop: ``--concurrency``
caller threads each keep one request in flight.

    python bench/serve_batch_slice.py --seconds 10 --concurrency 64 --json-out out.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from ray_dynamic_batching_amd import serve  # noqa: E402


@serve.deployment(ray_actor_options={"num_gpus": 1}, max_ongoing_requests=256, health_check_timeout_s=120,
                  engine={"request_slot_bytes": 224 * 224 * 3 + 1024})   # one raw image + the wire header per slot
class ResNet50Batch:
    def __init__(self, max_batch: int = 32, wait_s: float = 0.005, backend: str = "hip"):
        import torch

        from ray_dynamic_batching_amd import models

        torch.cuda.set_device(0)
        self.torch = torch
        self.model = models.create("resnet50", device="cuda", backend=backend)
        self.classify.set_max_batch_size(max_batch)
        self.classify.set_batch_wait_timeout_s(wait_s)
        with torch.no_grad():                       # per-shape kernel tuning happens here, not under load
            for b in (1, 2, 4, 8, 16, 24, max_batch):
                self.model.forward(self.model.example_input(b, seed=b, device="cuda"))
        torch.cuda.synchronize()
        self.batches = 0
        self.items = 0

    @serve.batch(max_batch_size=32, batch_wait_timeout_s=0.005)
    async def classify(self, images):
        x = serve.stack_to_device(images, "cuda")   # pinned staging + non-blocking H2D on a side stream
        with self.torch.no_grad():
            y = self.model.forward(x)
        rows = y.cpu().numpy()
        self.batches += 1
        self.items += len(images)
        return list(rows)

    async def __call__(self, image):
        return await self.classify(image)

    def stats(self):
        return {"batches": self.batches, "items": self.items}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--warmup-s", type=float, default=3.0)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--max-batch", type=int, default=32)
    ap.add_argument("--max-wait-ms", type=float, default=5.0)
    ap.add_argument("--backend", default="hip")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--native-client", action="store_true",
                    help="also drive the deployment's queue with the native closed-loop client")
    ap.add_argument("--native-concurrency", type=int, default=96)
    a = ap.parse_args(argv)

    h = serve.run(ResNet50Batch.bind(a.max_batch, a.max_wait_ms / 1e3, a.backend), name="slice", mode="process")
    rng = np.random.default_rng(0)
    imgs = [rng.integers(0, 256, size=(224, 224, 3), dtype=np.uint8) for _ in range(32)]
    lat: list = []
    lock = threading.Lock()
    state = {"record": False, "stop": False, "ok": 0, "err": 0}

    def caller(i):
        k = i
        while not state["stop"]:
            t0 = time.perf_counter()
            try:
                h.remote(imgs[k % len(imgs)]).result(timeout_s=60)
                ok = True
            except Exception as e:  # noqa: BLE001
                ok = False
                state.setdefault("first_error", repr(e)[:500])
            dt = time.perf_counter() - t0
            k += 1
            if state["record"]:
                with lock:
                    if ok:
                        state["ok"] += 1
                        lat.append(dt)
                    else:
                        state["err"] += 1

    ts = [threading.Thread(target=caller, args=(i,), daemon=True) for i in range(a.concurrency)]
    for t in ts:
        t.start()
    time.sleep(a.warmup_s)
    s0 = h.stats.remote().result(timeout_s=60)
    state["record"] = True
    t0 = time.perf_counter()
    time.sleep(a.seconds)
    state["record"] = False
    el = time.perf_counter() - t0
    s1 = h.stats.remote().result(timeout_s=60)
    state["stop"] = True
    for t in ts:
        t.join(70)
    lat_ms = np.array(lat) * 1e3 if lat else np.array([float("nan")])
    if state.get("first_error"):
        print("first error:", state["first_error"], file=sys.stderr, flush=True)
    from ray_dynamic_batching_amd.serve.controller import get_controller

    router = get_controller().apps["slice"]["ResNet50Batch"].router
    out = {
        "what": "SURVEY 7.3 slice: @serve.deployment(num_gpus=1) + @serve.batch(32, 5 ms) on ResNet-50 fp16 "
                "(this repo's HIP kernels, eager forward), serve.run process mode, handle.remote closed loop",
        "req_per_s": round(state["ok"] / el, 1), "p50_ms": round(float(np.percentile(lat_ms, 50)), 3),
        "p99_ms": round(float(np.percentile(lat_ms, 99)), 3), "ok": state["ok"], "errors": state["err"],
        "concurrency": a.concurrency, "seconds": round(el, 2),
        "mean_batch": round((s1["items"] - s0["items"]) / max(1, s1["batches"] - s0["batches"]), 2),
        "raw_tensor_calls": router.metrics.num_raw_tensor_calls, "router_requests": router.metrics.num_router_requests,
    }
    if a.native_client:
        # the same deployment driven by the native closed-loop client on its shm queue (the encoded
        # call payloads the router would send): the replica's own capacity, without this process's
        # Python handle threads in the loop
        from ray_dynamic_batching_amd.runtime import job as rjob
        from ray_dynamic_batching_amd.serve import tensor_wire

        ctrl = get_controller()
        st = ctrl.apps["slice"]["ResNet50Batch"]
        j = ctrl.jobs["slice"]
        lg = rjob.LoadGen(rjob.Client(j), st.model_id, [tensor_wire.encode_call("__call__", im) for im in imgs])
        lg.run(1000, a.native_concurrency, 0.0, 0.0, False, 300.0)
        s0 = h.stats.remote().result(timeout_s=60)
        res = lg.run(int(max(2000, 6000 * a.seconds / 5)), a.native_concurrency, 0.0, 0.0, True, 600.0)
        s1 = h.stats.remote().result(timeout_s=60)
        lat = res["latency"]
        out["native_client"] = {"req_per_s": round(res["ok"] / res["elapsed_s"], 1), "p50_ms": round(lat["p50_ms"], 3),
                                "p99_ms": round(lat["p99_ms"], 3), "ok": res["ok"], "errors": res.get("errors", 0),
                                "concurrency": a.native_concurrency,
                                "mean_batch": round((s1["items"] - s0["items"]) / max(1, s1["batches"] - s0["batches"]), 2)}
    print(json.dumps(out), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)
    serve.shutdown()


if __name__ == "__main__":
    main()
