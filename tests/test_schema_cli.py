import os
import subprocess
import sys

import pytest
import torch

from ray_dynamic_batching_amd import serve
from ray_dynamic_batching_amd.serve.schema import ServeDeploySchema, build_application, deploy_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _shutdown():
    yield
    serve.shutdown()


def test_yaml_deploy_applies_overrides():
    sys.path.insert(0, ROOT)
    sch = ServeDeploySchema.from_yaml(os.path.join(ROOT, "configs", "mlp_local.yaml"))
    app = build_application(sch.applications[0])
    assert app.deployment.config.num_replicas == 2 and app.deployment.config.max_ongoing_requests == 16
    h = deploy_config(sch)["mlp"]
    y = h.remote(torch.zeros(32)).result(timeout_s=10)
    assert tuple(y.shape) == (8,)
    assert serve.status()["applications"]["mlp"]["deployments"]["MLPDeployment"]["running_replicas"] == 2


def test_cli_build_and_run():
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-m", "ray_dynamic_batching_amd.serve.cli", "build", "examples.mlp_app:app"],
                         capture_output=True, text=True, env=env, cwd=ROOT, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "import_path: examples.mlp_app:app" in out.stdout and "num_replicas: 2" in out.stdout
    out = subprocess.run([sys.executable, "-m", "ray_dynamic_batching_amd.serve.cli", "run", "examples.mlp_app:app",
                          "--mode", "local", "--duration", "0.5"], capture_output=True, text=True, env=env, cwd=ROOT,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    assert "HEALTHY" in out.stdout


def test_cli_status_queries_live_node_agent(tmp_path):
    from ray_dynamic_batching_amd import serve
    from ray_dynamic_batching_amd.serve.cli import _status

    disc = tmp_path / "disc.json"
    os.environ["RDB_SERVE_DISCOVERY"] = str(disc)
    try:
        from examples.mlp_app import app

        serve.run(app, mode="local")
        st = _status("", "")
        assert "procs" in st and "gpus" in st
        assert "default" in st["checkpoint"]["applications"]
    finally:
        serve.shutdown()
        os.environ.pop("RDB_SERVE_DISCOVERY", None)


def test_cli_start_remote_deploy_status_shutdown(tmp_path):
    """`serve start` in one process; `serve deploy` hands the YAML to it over the
    node agent's control socket; `serve shutdown` stops it (reference:
    serve/scripts.py start/deploy/shutdown against a running instance)."""
    env = dict(os.environ, PYTHONPATH=ROOT, RDB_SERVE_DISCOVERY=str(tmp_path / "disc.json"))
    cli = [sys.executable, "-m", "ray_dynamic_batching_amd.serve.cli"]
    inst = subprocess.Popen(cli + ["start", "--duration", "120"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                            text=True, env=env, cwd=ROOT)
    try:
        import time

        t_end = time.time() + 60
        while not (tmp_path / "disc.json").exists() and time.time() < t_end:
            time.sleep(0.1)
        assert (tmp_path / "disc.json").exists(), "instance never published its discovery record"
        out = subprocess.run(cli + ["deploy", os.path.join(ROOT, "configs", "mlp_local.yaml")], capture_output=True,
                             text=True, env=env, cwd=ROOT, timeout=120)
        assert out.returncode == 0 and "running instance" in out.stdout, out.stdout + out.stderr
        out = subprocess.run(cli + ["status"], capture_output=True, text=True, env=env, cwd=ROOT, timeout=60)
        assert out.returncode == 0 and '"mlp"' in out.stdout, out.stdout + out.stderr
        out = subprocess.run(cli + ["shutdown", "-y"], capture_output=True, text=True, env=env, cwd=ROOT, timeout=60)
        assert out.returncode == 0 and "shut down" in out.stdout, out.stdout + out.stderr
        assert inst.wait(timeout=60) == 0
    finally:
        if inst.poll() is None:
            inst.kill()
            inst.wait(10)
