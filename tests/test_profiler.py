import csv
import os

from ray_dynamic_batching_amd.models.mlp import MLP
from ray_dynamic_batching_amd.planner import load_profile_csv, Session, SquishyPlanner
from ray_dynamic_batching_amd.planner.profiles import CSV_FIELDS
from ray_dynamic_batching_amd.profiler import ModelProfiler


def test_profiler_cpu_writes_planner_contract(tmp_path):
    m = MLP()
    p = ModelProfiler(m, [(32,)], min_batch_size=1, max_batch_size=8, batch_size_step=1, warmup_runs=1, num_runs=3,
                      output_dir=str(tmp_path), device="cpu")
    res = p.profile_all()
    assert len(res) == 8 and all(r["status"] == "success" for r in res)
    paths = p.save_results(res, "mlp")
    with open(paths["csv"]) as f:
        rows = list(csv.DictReader(f))
    assert list(rows[0].keys()) == CSV_FIELDS and len(rows) == 8
    prof = load_profile_csv(paths["csv"])
    assert set(prof) == set(range(1, 9))
    plan = SquishyPlanner({"mlp": prof}).plan([Session("mlp", 100.0, 500.0)])
    assert len(plan) >= 1
    assert "Best throughput" in open(paths["report"]).read()
    # the reference's 4-panel figure (run_profiler.py:110-156)
    assert os.path.getsize(paths["plot"]) > 10_000 and open(paths["plot"], "rb").read(4) == b"\x89PNG"


def test_profiler_stops_after_three_failures(tmp_path):
    class Bad:
        input_dtype = None

        def forward(self, x):
            raise RuntimeError("nope")

    import torch

    p = ModelProfiler(Bad(), [(4,)], 1, 10, warmup_runs=0, num_runs=1, output_dir=str(tmp_path), device="cpu",
                      input_dtype=torch.float32)
    res = p.profile_all()
    assert len(res) == 3 and all(r["status"] == "error" for r in res)
