"""fp32_reference (models/reference.py) on CPU: the same weights upcast, the
PyTorch path in fp32; cached kernel-layout weights dropped; the original
model untouched."""
import pytest
import torch

from ray_dynamic_batching_amd.models.reference import fp32_reference, rel_err


def test_fp32_reference_bert_cpu():
    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification

    m = BertForSequenceClassification(BertConfig.tiny(seq_len=32), device="cpu", backend="torch", seed=2)
    ids = m.example_input(4, seed=1)
    r = fp32_reference(m)
    assert r.dtype == torch.float32 and r.backend == "torch"
    assert m.dtype == torch.bfloat16 and m.layers[0]["w_qkv"].dtype == torch.bfloat16      # original untouched
    assert r.layers[0]["w_qkv"].dtype == torch.float32
    assert torch.equal(r.layers[0]["w_qkv"], m.layers[0]["w_qkv"].float())                # exact upcast
    y, ref = m(ids), r(ids)
    assert rel_err(y, ref) < 5e-2
    assert rel_err(ref, ref) == 0.0


def test_fp32_reference_llama_cpu():
    from ray_dynamic_batching_amd.models.llama import LlamaConfig, LlamaTP

    m = LlamaTP(LlamaConfig.tiny(seq_len=16, layers=1), device="cpu", backend="torch", init="full")
    ids = m.example_input(2, seed=0)
    r = fp32_reference(m)
    h = r.hidden_states(ids)
    assert h.dtype == torch.float32
    assert rel_err(m.hidden_states(ids), h) < 5e-2


def test_eager_reference_and_parity_bound_cpu():
    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification
    from ray_dynamic_batching_amd.models.reference import eager_reference, parity_bound

    m = BertForSequenceClassification(BertConfig.tiny(seq_len=32), device="cpu", backend="torch", seed=2)
    m._packed = "kernel-layout cache"
    e = eager_reference(m)
    assert e.backend == "torch" and e.dtype == torch.bfloat16 and e._packed is None and m._packed is not None
    ids = m.example_input(4, seed=1)
    assert torch.equal(e(ids), m(ids))                    # same dtype, same path: bit-identical
    assert parity_bound(0.001) == 2e-2 and parity_bound(0.02) == pytest.approx(0.035)
