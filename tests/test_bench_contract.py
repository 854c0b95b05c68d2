"""bench.py driver contract, rehearsed on CPU: torchrun with 2 ranks (gloo),
native fake replicas standing in for the GPU engines; rank 0 prints exactly
one JSON line with the required keys and a whole-job value."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def test_bench_two_ranks_echo_backend():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(29000 + os.getpid() % 1000), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "40", "--warmup", "4", "--backend", "echo", "--echo-service-us", "800"]
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
