"""Picklable model factories for servable deployments (shipped to replica
processes), each with the per-request I/O spec the router's codec needs."""
from __future__ import annotations

import functools

import torch


class Factory:
    """Callable factory with an ``io_spec`` (input_shape, input_dtype, output_shape, output_dtype)."""

    def __init__(self, fn, io_spec, **kw):
        self.fn = fn
        self.kw = kw
        self.io_spec = io_spec

    def __call__(self, device="cuda"):
        return self.fn(device=device, **self.kw)


def _bert(device, layers=12, seq_len=128, backend="hip", checkpoint=None):
    from .bert import BertConfig, BertForSequenceClassification

    if checkpoint:
        from .weights import bert_from_hf

        return bert_from_hf(checkpoint, seq_len=seq_len, device=device, backend=backend)
    return BertForSequenceClassification(BertConfig(layers=layers, seq_len=seq_len), device=device, backend=backend)


def _resnet(device, backend="hip", checkpoint=None):
    from .resnet import ResNet50

    m = ResNet50(device=device, backend=backend)
    if checkpoint:
        from .weights import load_resnet50

        load_resnet50(m, checkpoint)
    return m


def _vit(device, backend="hip"):
    from .vit import ViT, ViTConfig

    return ViT(ViTConfig.b16(), device=device, backend=backend)


def _mlp(device, **kw):
    from .mlp import MLP

    return MLP(device=device, **kw)


def bert_base(layers: int = 12, seq_len: int = 128, backend: str = "hip", checkpoint: str = None) -> Factory:
    """``checkpoint``: a Hugging Face BERT sequence-classification directory or
    file (models/weights.py); its config sets the shape and the label count."""
    labels = 2
    if checkpoint:
        from .weights import _bert_config, read_config

        labels = _bert_config(read_config(checkpoint), seq_len).num_labels
    return Factory(_bert, ((seq_len,), torch.int32, (labels,), torch.float32), layers=layers, seq_len=seq_len,
                   backend=backend, checkpoint=checkpoint)


def resnet50(backend: str = "hip", checkpoint: str = None) -> Factory:
    """``checkpoint``: torchvision resnet50 weights (safetensors / .pth, BN folded at load)."""
    return Factory(_resnet, ((224, 224, 3), torch.uint8, (10,), torch.float32), backend=backend,
                   checkpoint=checkpoint)


def vit_b16(backend: str = "hip") -> Factory:
    return Factory(_vit, ((224, 224, 3), torch.uint8, (10,), torch.float32), backend=backend)


def mlp(d_in: int = 32, d_out: int = 8) -> Factory:
    return Factory(_mlp, ((d_in,), torch.float32, (d_out,), torch.float32), d_in=d_in, d_out=d_out)


def _shufflenet(device, backend="hip"):
    from .shufflenet import ShuffleNetV2

    return ShuffleNetV2(device=device, backend=backend)


def _efficientnet(device, backend="hip"):
    from .efficientnet import EfficientNetV2S

    return EfficientNetV2S(device=device, backend=backend)


def shufflenet_v2(backend: str = "hip") -> Factory:
    return Factory(_shufflenet, ((224, 224, 3), torch.uint8, (10,), torch.float32), backend=backend)


def efficientnet_v2s(backend: str = "hip") -> Factory:
    return Factory(_efficientnet, ((384, 384, 3), torch.uint8, (10,), torch.float32), backend=backend)


class TPFactory(Factory):
    """Factory of a tensor-parallel servable: Serve's TP replicas call it on
    every rank with the rank's shard coordinates."""

    def __call__(self, device="cuda", tp_rank: int = 0, tp_size: int = 1, group_name=None):
        return self.fn(device=device, tp_rank=tp_rank, tp_size=tp_size, group_name=group_name, **self.kw)


def _tp_echo(device, tp_rank, tp_size, group_name, d, d_out):
    from .tp_echo import TPEcho

    return TPEcho(d, d_out, tp_rank, tp_size, group_name, device=device)


def tp_echo(d: int = 16, d_out: int = 8) -> TPFactory:
    """Row-parallel linear + all-reduce (CPU / gloo or GPU / RCCL): Serve TP plumbing."""
    return TPFactory(_tp_echo, ((d,), torch.float32, (d_out + 1,), torch.float32), d=d, d_out=d_out)


def _llama(device, tp_rank, tp_size, group_name, config, backend, seq_len, overrides):
    from .llama import LlamaConfig, LlamaTP

    kw = dict(overrides or {}, seq_len=seq_len)
    cfg = LlamaConfig.llama3_8b(**kw) if config == "8b" else LlamaConfig.tiny(**kw)
    return LlamaTP(cfg, tp_rank=tp_rank, tp_size=tp_size, group_name=group_name, device=device, backend=backend,
                   init="full" if config != "8b" else "shard")


def llama3(config: str = "8b", seq_len: int = 128, backend: str = "hip", **overrides) -> TPFactory:
    """Llama-3 prefill servable (next-token id per prompt of ``seq_len`` tokens),
    sharded over the TP group (BASELINE config 4).  ``config``: "8b" (random
    shards) or "tiny" (full-matrix init, identical for every TP size);
    ``overrides``: LlamaConfig fields (layers, heads, ...)."""
    return TPFactory(_llama, ((seq_len,), torch.int32, (2,), torch.int32), config=config, backend=backend,
                     seq_len=seq_len, overrides=dict(overrides))
