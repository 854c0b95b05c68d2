"""A tensor-parallel Llama replica deployed through ``serve.run`` on the GPU.

World 8 rehearsal on ONE MI355X: eight rank processes gang-spawned by the node
agent, each holding 1/8 of the GPU (fractional placement bundles), rendezvous
through the agent KV, xGMI IPC all-reduce between the ranks (gloo carries the
broadcasts and the line-up barriers, since RCCL refuses two ranks on one
device).  The next token of every prompt must equal the TP=1 model's.
On an 8-GPU node the same deployment with ``[{"GPU": 1}] * 8`` bundles and the
default RCCL backend gives each rank its own GPU."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from ray_dynamic_batching_amd import serve  # noqa: E402
from ray_dynamic_batching_amd.models import factories  # noqa: E402

OVR = dict(heads=8, kv_heads=8, head_dim=64, hidden=512, intermediate=1024, vocab_size=1024, layers=2)
SEQ = 32


@pytest.fixture
def tp_env(monkeypatch):
    monkeypatch.setenv("RDB_TP_XGMI", "1")
    monkeypatch.setenv("RDB_TP_GRAPHS", "0")
    monkeypatch.setenv("RDB_TP_LINE_UP", "1")
    yield
    serve.shutdown()


def test_llama_tp8_through_serve_matches_tp1(tp_env):
    fac = factories.llama3("tiny", seq_len=SEQ, **OVR)
    ref = fac(device="cuda")                          # TP = 1, same weights (full-matrix init)
    rng = np.random.default_rng(0)
    prompts = [rng.integers(0, OVR["vocab_size"], SEQ, dtype=np.int32) for _ in range(6)]
    with torch.no_grad():
        want = ref(torch.tensor(np.stack(prompts), device="cuda")).cpu().numpy()
    del ref
    torch.cuda.empty_cache()
    app = serve.model_deployment(fac, "llama", max_batch_size=4, batch_wait_timeout_s=0.01,
                                 tensor_parallel_size=8, tp_backend="gloo",
                                 placement_group_bundles=[{"GPU": 0.125}] * 8, health_check_timeout_s=120)
    h = serve.run(app.bind(), mode="process")
    got = np.stack([h.remote(p).result(timeout_s=120) for p in prompts])
    assert (got[:, 0] == want[:, 0]).all(), (got[:, 0], want[:, 0])
    from ray_dynamic_batching_amd.serve.controller import get_controller

    c = get_controller()
    rep = c.apps["default"]["llama"].proc_replicas[0]
    info = c.agent.group_info(rep.group_id)
    assert len(info["members"]) == 8 and info["restarts"] == 0


@pytest.mark.parametrize("world", [2, 8])
def test_llama_tp_through_serve_graphs_one_gpu(world, monkeypatch):
    """The deployable TP path with hipGraphs ON, rehearsed on ONE GPU: native
    leader / follower engines (runtime/tp_replica.py NativeTP) replay bucket
    graphs with the xGMI all-reduces captured inside -- no host line-up barrier.
    The all-reduce grid is capped (RDB_XGMI_MAX_GRID) so ranks spinning in it
    never hold every CU a peer's GEMM needs; next tokens equal TP = 1's."""
    monkeypatch.setenv("RDB_TP_XGMI", "1")
    monkeypatch.setenv("RDB_TP_GRAPHS", "1")
    monkeypatch.setenv("RDB_TP_LINE_UP", "0")
    monkeypatch.setenv("RDB_XGMI_MAX_GRID", "8")
    fac = factories.llama3("tiny", seq_len=SEQ, **OVR)
    ref = fac(device="cuda")
    rng = np.random.default_rng(world)
    prompts = [rng.integers(0, OVR["vocab_size"], SEQ, dtype=np.int32) for _ in range(12)]
    with torch.no_grad():
        want = ref(torch.tensor(np.stack(prompts), device="cuda")).cpu().numpy()
    del ref
    torch.cuda.empty_cache()
    try:
        app = serve.model_deployment(fac, "llama", max_batch_size=4, batch_wait_timeout_s=0.005,
                                     tensor_parallel_size=world, tp_backend="gloo",
                                     placement_group_bundles=[{"GPU": 1.0 / world}] * world,
                                     health_check_timeout_s=120)
        h = serve.run(app.bind(), mode="process")
        got = np.stack([o.result(timeout_s=90) for o in [h.remote(p) for p in prompts]])
        assert (got[:, 0] == want[:, 0]).all(), (got[:, 0], want[:, 0])
        from ray_dynamic_batching_amd.serve.controller import get_controller

        c = get_controller()
        rep = c.apps["default"]["llama"].proc_replicas[0]
        info = c.agent.group_info(rep.group_id)
        assert len(info["members"]) == world and info["restarts"] == 0
    finally:
        serve.shutdown()
