"""Offline per-batch profiles of the fork's models on MI355X (the reference's
only published numbers: RTX A6000 ModelProfiler CSVs) -- same CSV
contract (profiler/model_profiler.py), graph mode, plus a side-by-side
comparison with the A6000 rows kept in tests/fixtures/a6000_profiles/.

    python bench/profile_models.py --models resnet50,shufflenet-v2,efficientnet-v2s,vit-g16 \
        --out profiles/mi355x_model_profiles
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

A6000 = {"resnet50": "resnet50", "shufflenet-v2": "shufflenet", "efficientnet-v2s": "efficientnetv2",
         "vit-g16": "vit_g16"}


def a6000_rows(model: str):
    pat = os.path.join(ROOT, "tests", "fixtures", "a6000_profiles", f"{A6000.get(model, model)}_*summary.csv")
    files = glob.glob(pat)
    if not files:
        return {}
    out = {}
    with open(files[0]) as f:
        for r in csv.DictReader(f):
            try:
                out[int(r["batch_size"])] = float(r["avg_latency_ms"])
            except (KeyError, ValueError):
                pass
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,shufflenet-v2,efficientnet-v2s,vit-g16")
    ap.add_argument("--batches", default="1,8,16,32,64,128,256")
    ap.add_argument("--out", default="gpurun_out/model_profiles")
    ap.add_argument("--include-h2d", action="store_true")
    a = ap.parse_args(argv)

    import torch

    from ray_dynamic_batching_amd import models
    from ray_dynamic_batching_amd.planner.profiles import write_profile_csv
    from ray_dynamic_batching_amd.profiler.model_profiler import ModelProfiler

    os.makedirs(a.out, exist_ok=True)
    batches = [int(b) for b in a.batches.split(",")]
    summary = {}
    for name in a.models.split(","):
        m = models.create(name, device="cuda:0")
        prof = ModelProfiler(m, [m.input_shape], batch_sizes=batches, mode="graph", device="cuda:0",
                             include_h2d=a.include_h2d, input_fn=lambda b, m=m: [m.example_input(b, device="cpu")],
                             output_dir=a.out, warmup_runs=3, num_runs=10)
        res = prof.profile_all()
        write_profile_csv(os.path.join(a.out, f"{name}_summary.csv"), res)
        ref = a6000_rows(name)
        rows = []
        for r in res:
            if r["status"] != "success":
                rows.append(dict(batch=r["batch_size"], status=r["status"]))
                continue
            b = r["batch_size"]
            row = dict(batch=b, mi355x_ms=round(r["avg_latency_ms"], 3), mi355x_img_s=round(r["throughput"], 1),
                       peak_mb=round(r["peak_memory_mb"], 1))
            if b in ref:
                row.update(a6000_ms=ref[b], a6000_img_s=round(b * 1000 / ref[b], 1),
                           speedup=round(ref[b] / r["avg_latency_ms"], 2))
            rows.append(row)
        summary[name] = rows
        print(json.dumps({name: rows}), flush=True)
        del m, prof
        torch.cuda.empty_cache()
    with open(os.path.join(a.out, "comparison.json"), "w") as f:
        json.dump(dict(include_h2d=a.include_h2d, note="MI355X: this framework's HIP kernels, f16, hipGraph; "
                       "A6000: reference ModelProfiler CSVs (AMP autocast, no H2D)", models=summary), f, indent=1)


if __name__ == "__main__":
    main()
