"""Model-level parity of the HIP kernels against an fp32 anchor: every model of
the zoo on its HIP path vs the SAME weights (upcast exactly) on the PyTorch
path in fp32 (models/reference.py, ``create(name, backend="torch32")``).
Bound: ||y - ref||_inf / ||ref||_inf <= 2e-2 on inputs whose logits are
well away from zero (the check is relative, so a logit-level bug of a few
percent fails it regardless of the logits' scale)."""
import pytest
import torch

from ray_dynamic_batching_amd.models.reference import eager_reference, fp32_reference, parity_bound, rel_err

pytestmark = pytest.mark.gpu

BOUND = 2e-2


def _nontrivial(ref):
    assert ref.abs().max() > 1e-2 and ref.std() > 1e-3, "reference output too small to anchor a relative check"


def test_bert_hip_vs_fp32():
    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification

    m = BertForSequenceClassification(BertConfig(layers=6), device="cuda", backend="hip", seed=1)
    ids = m.example_input(16, seed=3)
    ids[3, 90:] = 0          # padding exercises the key-length mask
    y = m(ids)
    ref = fp32_reference(m)(ids)
    _nontrivial(ref)
    bound = parity_bound(rel_err(eager_reference(m)(ids), ref))
    assert rel_err(y, ref) <= bound, (rel_err(y, ref), bound)


def test_bert_base_full_depth_hip_vs_fp32():
    """12 layers (the served model), fused QKV+attention, CLS-only last layer."""
    from ray_dynamic_batching_amd import models

    m = models.create("bert-base", device="cuda", seq_len=128)
    ids = m.example_input(32, seed=5)
    y = m(ids)
    ref = fp32_reference(m)(ids)
    _nontrivial(ref)
    bound = parity_bound(rel_err(eager_reference(m)(ids), ref))
    assert rel_err(y, ref) <= bound, (rel_err(y, ref), bound)


def test_resnet50_hip_vs_fp32():
    from ray_dynamic_batching_amd.models.resnet import ResNet50

    m = ResNet50(device="cuda", backend="hip")
    x = m.example_input(4, seed=1)
    y = m.logits(x)
    ref = fp32_reference(m).logits(x)
    _nontrivial(ref)
    assert rel_err(y, ref) <= BOUND, rel_err(y, ref)


def test_vit_hip_vs_fp32():
    from ray_dynamic_batching_amd.models.vit import ViT, ViTConfig

    m = ViT(ViTConfig(layers=6), device="cuda", backend="hip")
    x = m.example_input(3, seed=2)
    y = m._logits_hip(x)
    ref = fp32_reference(m)._logits_torch(x)
    _nontrivial(ref)
    assert rel_err(y, ref) <= BOUND, rel_err(y, ref)


def test_shufflenet_hip_vs_fp32():
    from ray_dynamic_batching_amd.models.shufflenet import ShuffleNetV2

    m = ShuffleNetV2(device="cuda", backend="hip")
    x = m.example_input(4, seed=4)
    y = m.logits(x)
    ref = fp32_reference(m).logits(x)
    _nontrivial(ref)
    assert rel_err(y, ref) <= BOUND, rel_err(y, ref)


def test_efficientnet_hip_vs_fp32():
    from ray_dynamic_batching_amd.models.efficientnet import EfficientNetV2S

    m = EfficientNetV2S(device="cuda", backend="hip")
    x = m.example_input(2, seed=6)
    y = m.logits(x)
    ref = fp32_reference(m).logits(x)
    _nontrivial(ref)
    assert rel_err(y, ref) <= BOUND, rel_err(y, ref)


def test_llama_hip_vs_fp32():
    from ray_dynamic_batching_amd.models.llama import LlamaConfig, LlamaTP

    m = LlamaTP(LlamaConfig.tiny(seq_len=128), device="cuda", backend="hip", init="full")
    ids = m.example_input(4, seed=3)
    y = m.hidden_states(ids)
    ref = fp32_reference(m).hidden_states(ids)
    _nontrivial(ref)
    assert rel_err(y, ref) <= BOUND, rel_err(y, ref)


def test_create_torch32_backend():
    from ray_dynamic_batching_amd import models

    r = models.create("bert-base", device="cuda", backend="torch32", layers=2)
    assert r.backend == "torch" and r.dtype == torch.float32
    assert all(t.dtype == torch.float32 for t in r.layers[0].values() if t.is_floating_point())
