"""ResNet-50 / ViT / Llama on the HIP kernels vs their eager PyTorch baselines,
and GPU serving through serve.model_deployment (process mode + native engine)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_resnet50_hip_matches_torch():
    from ray_dynamic_batching_amd.models.resnet import ResNet50

    m = ResNet50(device="cuda", backend="hip")
    x = m.example_input(4, seed=1)
    lg = m.logits(x)
    m.backend = "torch"
    ref = m.logits(x)
    assert lg.shape == (4, 1000)
    assert torch.allclose(lg, ref, atol=3e-2, rtol=5e-2), (lg - ref).abs().max()
    m.backend = "hip"
    out = m(x)
    assert out.shape == (4, 10) and torch.all(out[:, :5] > 0)


def test_vit_hip_matches_torch():
    from ray_dynamic_batching_amd.models.vit import ViT, ViTConfig

    m = ViT(ViTConfig(layers=4), device="cuda", backend="hip")
    x = m.example_input(3, seed=2)
    lg = m._logits_hip(x)
    ref = m._logits_torch(x)
    assert torch.allclose(lg, ref, atol=3e-2, rtol=5e-2), (lg - ref).abs().max()


def test_llama_tp1_hip_matches_torch():
    from ray_dynamic_batching_amd.models.llama import LlamaConfig, LlamaTP

    m = LlamaTP(LlamaConfig.tiny(seq_len=128), device="cuda", backend="hip", init="full")
    ids = m.example_input(4, seed=3)
    xh = m.hidden_states(ids)
    m.backend = "torch"
    xr = m.hidden_states(ids)
    assert torch.allclose(xh.float(), xr.float(), atol=5e-2, rtol=5e-2), (xh.float() - xr.float()).abs().max()
    m.backend = "hip"
    out = m(ids)
    assert out.shape == (4, 2) and out.dtype == torch.int32


def test_serve_model_deployment_bert_on_gpu():
    from ray_dynamic_batching_amd import serve
    from ray_dynamic_batching_amd.models import factories

    fac = factories.bert_base(layers=2)
    d = serve.model_deployment(fac, "bert", max_batch_size=16, batch_wait_timeout_s=0.002,
                               ray_actor_options={"num_gpus": 1}, max_ongoing_requests=64)
    try:
        h = serve.run(d.bind(), mode="process")
        model = fac(device="cuda")
        ids = model.example_input(40, seed=4).cpu()
        outs = [h.remote(ids[i].numpy()) for i in range(40)]
        got = np.stack([o.result(timeout_s=60) for o in outs])
        ref = model(ids.cuda()).cpu().numpy()
        assert np.allclose(got, ref, atol=2e-2, rtol=2e-2)
        st = serve.status()["applications"]["default"]["deployments"]["bert"]
        assert st["replicas"][0]["batches"] >= 3
    finally:
        serve.shutdown()
