"""The Serve-deployed replica engine is the benchmarked one:
every EngineConfig knob travels from the deployment (decorator / YAML) to the
EngineRunner the replica process builds, the shipped MI355X tile table is
resolved by model signature exactly as bench.py resolves it, and the node
agent starts the replica pinned to its GPU's CPUs.  CPU only: a fake runner
records what it was given."""
import os

import pytest
import yaml

from ray_dynamic_batching_amd import serve
from ray_dynamic_batching_amd.models import factories
from ray_dynamic_batching_amd.runtime.engine import TUNED_DIR, resolve_tile_table, shipped_tile_table
from ray_dynamic_batching_amd.serve.config import DeploymentConfig, EngineConfig
from ray_dynamic_batching_amd.serve.replica_main import build_engine_runner
from ray_dynamic_batching_amd.serve.schema import ServeApplicationSchema, build_application


class _FakeBert:
    tile_signature = "bert_L12_S128"


class _FakeRunner:
    def __init__(self, job, replica, sessions, **kw):
        self.job, self.replica, self.sessions, self.kw = job, replica, sessions, kw
        self.warm = "unset"

    def build(self, warm_s=None):
        self.warm = warm_s
        return self


def _spec(max_batch=32, wait=0.005):
    return dict(job="j", servable=dict(factory=None, max_batch_size=max_batch, batch_wait_timeout_s=wait))


def test_model_deployment_defaults_are_the_benchmarked_replica():
    d = serve.model_deployment(factories.bert_base(), "bert", max_batch_size=32, ray_actor_options={"num_gpus": 1})
    e = d.config.engine
    assert (e.compute_streams, e.pipeline_depth, e.batch_policy, e.tile_table, e.numa_pin) == (3, 6, "timeout",
                                                                                              "auto", True)
    assert e.request_slot_bytes == 128 * 4
    # bench.py's configuration (3 x 6) resolves to the same shipped table; the round-5 2 x 4 one stays
    p = shipped_tile_table(_FakeBert(), 32, 3, 6)
    assert p == os.path.join(TUNED_DIR, "mi355x_bert_L12_S128_B32_cs3_d6.json") and os.path.exists(p)
    assert shipped_tile_table(_FakeBert(), 32, 2, 4).endswith("mi355x_bert_L12_S128_B32_cs2_d4.json")
    # a single-stream replica replays the single-stream table whatever its depth
    assert shipped_tile_table(_FakeBert(), 32, 1, 2).endswith("mi355x_bert_L12_S128_B32_cs1_d2.json")
    assert shipped_tile_table(_FakeBert(), 32, 1, 4).endswith("mi355x_bert_L12_S128_B32_cs1_d2.json")


def test_replica_engine_receives_configured_streams_and_table():
    cfg = DeploymentConfig(name="bert", engine=dict(compute_streams=2, pipeline_depth=4, batch_policy="idle",
                                                    stagger_us=150, warm_s=0.5, tile_table="auto"))
    r = build_engine_runner(_spec(), cfg, 3, _FakeBert(), runner_cls=_FakeRunner)
    assert r.replica == 3 and r.sessions[0].queue == 3 and r.sessions[0].max_batch == 32
    assert r.kw["compute_streams"] == 2 and r.kw["pipeline_depth"] == 4
    assert r.kw["batch_policy"] == "idle" and r.kw["stagger_us"] == 150 and r.warm == 0.5
    assert r.kw["tile_table"].endswith("mi355x_bert_L12_S128_B32_cs2_d4.json")
    # a configuration with no shipped table tunes at start-up; "none" forces it; a path is replayed as is
    cfg = DeploymentConfig(name="bert", engine=dict(compute_streams=4, pipeline_depth=8))
    assert build_engine_runner(_spec(), cfg, 0, _FakeBert(), runner_cls=_FakeRunner).kw["tile_table"] == ""
    assert resolve_tile_table("none", _FakeBert(), 32, 2, 4) == ""
    assert resolve_tile_table("/x/t.json", _FakeBert(), 32, 2, 4) == "/x/t.json"
    assert shipped_tile_table(object(), 32, 2, 4) == ""          # no signature: no table


def test_engine_config_validation():
    with pytest.raises(ValueError):
        EngineConfig(compute_streams=3, pipeline_depth=2)
    with pytest.raises(ValueError):
        EngineConfig(batch_policy="eager")
    with pytest.raises(ValueError):
        EngineConfig(stagger_us=-1)
    # shallow explicit pipeline: model_deployment keeps streams <= depth
    d = serve.model_deployment(factories.mlp(), "m", pipeline_depth=1)
    assert d.config.engine.compute_streams == 1 and d.config.engine.pipeline_depth == 1


def test_yaml_round_trips_engine_fields(tmp_path, monkeypatch):
    mod = tmp_path / "eng_app.py"
    mod.write_text("from ray_dynamic_batching_amd import serve\n"
                   "from ray_dynamic_batching_amd.models import factories\n"
                   "app = serve.model_deployment(factories.bert_base(), 'bert', max_batch_size=32,\n"
                   "                             ray_actor_options={'num_gpus': 1}).bind()\n")
    monkeypatch.syspath_prepend(str(tmp_path))
    doc = yaml.safe_load("""
import_path: eng_app:app
deployments:
  - name: bert
    engine: {compute_streams: 1, pipeline_depth: 2, batch_policy: idle, stagger_us: 80, tile_table: none,
             numa_pin: false}
""")
    app = build_application(ServeApplicationSchema(**doc))
    e = app.deployment.config.engine
    assert (e.compute_streams, e.pipeline_depth, e.batch_policy, e.stagger_us, e.tile_table, e.numa_pin) == \
        (1, 2, "idle", 80, "none", False)
    assert e.request_slot_bytes == 128 * 4           # a partial override keeps the other engine fields
    dumped = yaml.safe_dump(app.deployment.config.model_dump(mode="json"))
    back = DeploymentConfig(**yaml.safe_load(dumped))
    assert back.engine == e


def test_gpu_placement_plans_disjoint_cpu_sets(tmp_path):
    """Two GPUs on one NUMA node get disjoint halves of its CPUs (the split
    bench.py's ranks use); a GPU's placement is planned over the whole node,
    not the replica's HIP_VISIBLE_DEVICES view."""
    from ray_dynamic_batching_amd.runtime import numa

    for bdf in ("0000:11:00.0", "0000:22:00.0"):
        d = tmp_path / "bus" / "pci" / "devices" / bdf
        d.mkdir(parents=True)
        (d / "numa_node").write_text("0\n")
        (d / "local_cpulist").write_text("0-7\n")
    pci = ["0000:11:00.0", "0000:22:00.0"]
    allowed = set(os.sched_getaffinity(0))
    if not set(range(8)) <= allowed:
        pytest.skip("needs CPUs 0-7 in this process's affinity mask")
    a = numa.gpu_placement(0, sysfs=str(tmp_path), pci=pci)
    b = numa.gpu_placement(1, sysfs=str(tmp_path), pci=pci)
    assert a["numa_node"] == 0 and b["numa_node"] == 0
    assert a["cpus"] == [0, 1, 2, 3] and b["cpus"] == [4, 5, 6, 7]


def test_node_agent_starts_process_pinned(tmp_path):
    """The agent applies the CPU set at spawn: the child is born with it."""
    import sys
    import time

    from ray_dynamic_batching_amd.runtime import agent as ragent

    allowed = sorted(os.sched_getaffinity(0))
    want = allowed[:1]
    out = tmp_path / "aff.txt"
    a = ragent.NodeAgent(0, 0.0, "")
    try:
        code = f"import os; open({str(out)!r}, 'w').write(','.join(map(str, sorted(os.sched_getaffinity(0)))))"
        pid = a.spawn("pin", [sys.executable, "-c", code], {}, "", "", -1, [], 0.0, 0, 0.5, 1.0, want)
        t_end = time.time() + 30
        while time.time() < t_end and not (out.exists() and out.read_text()):
            time.sleep(0.05)
        assert out.read_text() == ",".join(map(str, want))
        # the agent's own thread got its mask back
        assert sorted(os.sched_getaffinity(0)) == allowed
        del pid
    finally:
        a.shutdown(2.0)


def test_hw_queues_follow_compute_streams(monkeypatch):
    """Every engine stream gets its own HIP hardware queue (runtime/queues.py):
    bench.py and Serve replicas raise GPU_MAX_HW_QUEUES before HIP starts."""
    from ray_dynamic_batching_amd.runtime.queues import ensure_hw_queues, hw_queues_needed

    assert hw_queues_needed(1) == 4 and hw_queues_needed(2) == 4 and hw_queues_needed(3) == 5
    assert hw_queues_needed(64) == 32
    env = {}
    assert ensure_hw_queues(3, env) == 5 and env["GPU_MAX_HW_QUEUES"] == "5"
    env = {"GPU_MAX_HW_QUEUES": "8"}
    assert ensure_hw_queues(3, env) == 8 and env["GPU_MAX_HW_QUEUES"] == "8"     # never lowered
    # the controller puts it in a servable replica's environment
    from ray_dynamic_batching_amd.serve.controller import ServeController

    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)

    class St:
        app_name, name = "a", "bert"
        deployment = serve.model_deployment(factories.bert_base(), "bert", engine=dict(compute_streams=3,
                                                                                        pipeline_depth=6))
        config = deployment.config

    class Rep:
        slot = 0

    class Job:
        def info(self):
            return {"name": "j"}

    ctrl = ServeController.__new__(ServeController)
    ctrl._routes_path, ctrl.agent_socket = "/x", ""
    env = ctrl._replica_env(St, Rep, Job())
    assert env["GPU_MAX_HW_QUEUES"] == "5"
