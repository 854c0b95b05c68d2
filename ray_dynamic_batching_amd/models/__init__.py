"""Model zoo of the serving stack (random init by default; ``create(name, checkpoint=path)``
loads real weights through :mod:`.weights`).

Every model follows the *servable* contract used by the replica engine:
``input_shape``, ``input_dtype``, ``output_shape``, ``output_dtype`` per request
and ``forward(x[B, *input_shape]) -> y[B, *output_shape]``.

| name            | reference use                                    | module        |
|-----------------|--------------------------------------------------|---------------|
| mlp             | BASELINE config 1 (CPU plumbing)                 | mlp.py        |
| bert-base       | north-star metric (seq128, bf16)                 | bert.py       |
| resnet50        | fork registry / profiles, BASELINE config 2      | resnet.py     |
| vit-b16         | fork registry (scheduler.py:41)                  | vit.py        |
| shufflenet-v2   | fork registry (scheduler.py:42)                  | shufflenet.py |
| efficientnet-v2s| fork profile (efficientnetv2_* csv)              | efficientnet.py |
| llama3-8b (TP)  | BASELINE config 4                                | llama.py      |
"""
from __future__ import annotations

from typing import Callable, Dict

REGISTRY: Dict[str, Callable] = {}


def register(name: str):
    def deco(fn):
        REGISTRY[name] = fn
        return fn
    return deco


def create(name: str, **kw):
    """``backend="torch32"``: the PyTorch path in fp32 on the same (upcast)
    weights -- the numerics anchor of the HIP kernels (models/reference.py)."""
    _load_all()
    if name not in REGISTRY:
        raise KeyError(f"unknown model {name!r}; known: {sorted(REGISTRY)}")
    if kw.get("backend") == "torch32":
        from .reference import fp32_reference

        kw["backend"] = "torch"
        return fp32_reference(REGISTRY[name](**kw))
    return REGISTRY[name](**kw)


def _load_all():
    from . import bert, mlp  # noqa: F401
    for mod in ("resnet", "vit", "shufflenet", "efficientnet", "llama"):
        try:
            __import__(f"{__name__}.{mod}")
        except ImportError:  # pragma: no cover
            pass


@register("mlp")
def _mlp(**kw):
    from .mlp import MLP

    return MLP(**kw)


@register("bert-base")
def _bert(device="cuda", backend="hip", seq_len=128, layers=12, checkpoint=None, **kw):
    from .bert import BertConfig, BertForSequenceClassification

    if checkpoint:
        from .weights import bert_from_hf

        return bert_from_hf(checkpoint, seq_len=seq_len, device=device, backend=backend, **kw)
    return BertForSequenceClassification(BertConfig(seq_len=seq_len, layers=layers), device=device, backend=backend, **kw)


@register("resnet50")
def _resnet(device="cuda", backend="hip", checkpoint=None, **kw):
    from .resnet import ResNet50

    m = ResNet50(device=device, backend=backend, **kw)
    if checkpoint:
        from .weights import load_resnet50

        load_resnet50(m, checkpoint)
    return m


@register("llama3-8b")
def _llama(device="cuda", backend="hip", tp_rank=0, tp_size=1, group_name=None, seq_len=512, layers=32,
           checkpoint=None, **kw):
    from .llama import LlamaConfig, LlamaTP

    if checkpoint:
        from .weights import llama_from_hf

        return llama_from_hf(checkpoint, seq_len=seq_len, tp_rank=tp_rank, tp_size=tp_size, group_name=group_name,
                             device=device, backend=backend, **kw)
    return LlamaTP(LlamaConfig(seq_len=seq_len, layers=layers), tp_rank, tp_size, group_name, device=device,
                   backend=backend, **kw)


@register("vit-b16")
def _vit(device="cuda", backend="hip", checkpoint=None, **kw):
    from .vit import ViT, ViTConfig

    if checkpoint:
        from .weights import load_state_dict, vit_from_hf

        if "conv_proj.weight" in load_state_dict(checkpoint):     # torchvision vit_b_16
            from .weights import load_vit

            return load_vit(ViT(ViTConfig.b16(), device=device, backend=backend, **kw), checkpoint)
        return vit_from_hf(checkpoint, device=device, backend=backend, **kw)
    return ViT(ViTConfig.b16(), device=device, backend=backend, **kw)


@register("shufflenet-v2")
def _shufflenet(device="cuda", backend="hip", checkpoint=None, **kw):
    from .shufflenet import ShuffleNetV2

    if checkpoint:
        from .weights import shufflenet_v2_from_torchvision

        return shufflenet_v2_from_torchvision(checkpoint, device=device, backend=backend, **kw)
    return ShuffleNetV2(device=device, backend=backend, **kw)


@register("efficientnet-v2s")
def _efficientnet(device="cuda", backend="hip", checkpoint=None, **kw):
    from .efficientnet import EfficientNetV2S

    if checkpoint:
        from .weights import efficientnet_v2s_from_torchvision

        return efficientnet_v2s_from_torchvision(checkpoint, device=device, backend=backend, **kw)
    return EfficientNetV2S(device=device, backend=backend, **kw)


@register("vit-g16")
def _vit_g16(device="cuda", backend="hip", **kw):
    from .vit import ViT, ViTConfig

    return ViT(ViTConfig.g16(), device=device, backend=backend, **kw)
