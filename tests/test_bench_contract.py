"""bench.py driver contract, rehearsed on CPU: torchrun with 2 ranks (gloo),
native fake replicas standing in for the GPU engines; rank 0 prints exactly
one JSON line with the required keys and a whole-job value."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


@pytest.mark.parametrize("ingress", ["per-rank", "rank0"])
def test_bench_two_ranks_echo_backend(ingress):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(29000 + os.getpid() % 1000), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "40", "--warmup", "4", "--backend", "echo", "--echo-service-us", "800",
           "--ingress", ingress]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT,
                         env=dict(os.environ, PYTHONPATH=ROOT))
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert KEYS <= set(d)
    assert d["n_gpus"] == 2 and d["steps"] == 40 and d["config"]["parallelism"] == "dp2"
    assert d["completed"] == 40 * 32 * 2 and d["errors"] == 0
    assert abs(d["value"] - d["completed"] / (d["ms_per_step"] * d["steps"] / 1e3)) / d["value"] < 0.01
    assert min(d["per_replica_requests"]) > 0
    assert d["ingress"].startswith(ingress)
    assert 0 < d["p50_ms"] <= d["p99_ms"]


def test_bench_resolves_shipped_tile_table():
    """bench.py's default (--tile-table auto) replays the MI355X table shipped for
    the headline config -- through the same resolver a Serve-deployed replica uses
    (runtime.engine.resolve_tile_table, keyed by the model's tile signature);
    other configs / 'none' / non-HIP backends tune at start-up."""
    from types import SimpleNamespace

    from ray_dynamic_batching_amd.models.bert import BertConfig, bert_tile_signature
    from ray_dynamic_batching_amd.runtime.engine import resolve_tile_table

    def model(layers=12, backend="hip"):
        return SimpleNamespace(tile_signature=bert_tile_signature(BertConfig(layers=layers, seq_len=128), backend))

    p = resolve_tile_table("auto", model(), 32, 2, 4)
    assert p.endswith("mi355x_bert_L12_S128_B32_cs2_d4.json") and os.path.exists(p)
    table = json.load(open(p))
    assert any(k[0] == "gemm" and k[2:5] == [4096, 3072, 768] for k, _ in table)      # the bs32 FFN-up entry
    assert resolve_tile_table("auto", model(layers=2), 32, 2, 4) == ""
    assert resolve_tile_table("none", model(), 32, 2, 4) == ""
    assert resolve_tile_table("auto", model(backend="torch"), 32, 2, 4) == ""
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")).read()
    assert "resolve_tile_table(" in src


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_gpus_flag_launches_ranks_itself(n):
    """`python bench.py --gpus N` with no launcher (the driver's command shape)
    starts N ranks itself: n_gpus == N and every replica served requests."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "20", "--warmup", "2",
           "--backend", "echo", "--echo-service-us", "800"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["config"]["parallelism"] == f"dp{n}"
    assert len(d["per_replica_requests"]) == n and min(d["per_replica_requests"]) > 0
    assert d["errors"] == 0 and d["completed"] == 20 * 32 * n


def test_bench_gpus_must_match_launcher_world_size():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "2", "--backend", "echo"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=ROOT,
                         env=dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert out.returncode == 2 and "WORLD_SIZE=2" in out.stderr
