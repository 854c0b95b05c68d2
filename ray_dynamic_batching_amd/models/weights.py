"""Checkpoint loading: serve real weights, not only random init.

The reference's registry loads pretrained torchvision weights at import
(``293-project/src/scheduler.py:37-44``, ``ResNet50_Weights.DEFAULT`` at
``profiling/run_profiler.py``).  This module reads checkpoints in the formats
such models ship in and maps them onto this framework's kernel-layout models:

* files: ``*.safetensors`` (``safetensors.torch.load_file``), ``*.bin`` /
  ``*.pt`` / ``*.pth`` (``torch.load(weights_only=True)`` -- nothing in the file
  is executed), a Hugging Face model directory (``model.safetensors`` /
  ``pytorch_model.bin`` or their sharded ``*.index.json``) with ``config.json``,
  or an in-memory ``state_dict``;
* BERT: Hugging Face ``BertForSequenceClassification`` keys (also the
  ``gamma``/``beta`` LayerNorm names of old checkpoints) -> ``BertForSequenceClassification``
  (q/k/v fused into one [3D, D] projection, the layout ``ops.qkv_attention``
  packs per head);
* Llama: Hugging Face ``LlamaForCausalLM`` keys -> ``LlamaTP`` for ANY tensor-
  parallel rank (each rank slices its q/k/v heads, its gate/up rows -- stored
  interleaved for the SwiGLU epilogue --, its o/down columns and its vocab
  slice of the LM head); ``tie_word_embeddings`` and the ``llama3`` RoPE
  frequency scaling of Llama-3.x configs are honoured;
* ViT: Hugging Face ``ViTForImageClassification`` keys or torchvision
  ``vit_b_16`` keys -> ``models.vit.ViT``; a checkpoint trained on another
  input normalisation (HF ViT: mean = std = 0.5) is re-expressed in this
  model's ImageNet-normalised input space by folding the difference into the
  patch-embedding weights and bias (exact: the patch conv has no padding);
* EfficientNetV2-S: torchvision ``efficientnet_v2_s`` keys (SE 1x1 convs as
  FCs, BatchNorm eps 1e-3);
* ShuffleNetV2 x1.0: torchvision ``shufflenet_v2_x1_0`` keys, BN folded and
  channel-padded by ``cnn_common.CheckpointFolder`` in the constructor;
* ResNet-50: torchvision ``resnet50`` keys -> ``models.resnet.ResNet50`` with
  every BatchNorm folded into its convolution at load (see ``load_resnet50``).

Loading copies into the model's existing tensors in place, so derived caches
(packed QKV heads, folded LayerNorm weights) see the new version counters and
rebuild; a replica engine built afterwards captures graphs over the loaded
weights.
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, Mapping, Optional, Union

import torch

StateDict = Dict[str, torch.Tensor]
Source = Union[str, os.PathLike, Mapping[str, torch.Tensor]]

__all__ = ["load_state_dict", "read_config", "load_bert_hf", "bert_from_hf", "load_llama_hf", "llama_from_hf",
           "llama_rope_tables", "load_resnet50", "load_vit", "vit_from_hf", "shufflenet_v2_from_torchvision",
           "efficientnet_v2s_from_torchvision"]


# ---------------------------------------------------------------------------
# files
# ---------------------------------------------------------------------------
def _load_file(path: str) -> StateDict:
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file

        return load_file(path, device="cpu")
    if path.endswith((".bin", ".pt", ".pth")):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
            sd = sd["state_dict"]
        return sd
    raise ValueError(f"unsupported checkpoint file {path!r} (safetensors / .bin / .pt / .pth)")


def load_state_dict(src: Source) -> StateDict:
    """A state dict from a file, a Hugging Face model directory (single or
    sharded), or a mapping (returned as a dict)."""
    if isinstance(src, Mapping):
        return dict(src)
    path = os.fspath(src)
    if os.path.isdir(path):
        for index in ("model.safetensors.index.json", "pytorch_model.bin.index.json"):
            ip = os.path.join(path, index)
            if os.path.exists(ip):
                with open(ip) as f:
                    shards = sorted(set(json.load(f)["weight_map"].values()))
                sd: StateDict = {}
                for s in shards:
                    sd.update(_load_file(os.path.join(path, s)))
                return sd
        for name in ("model.safetensors", "pytorch_model.bin", "model.pt", "model.pth"):
            p = os.path.join(path, name)
            if os.path.exists(p):
                return _load_file(p)
        raise FileNotFoundError(f"no checkpoint file in {path!r}")
    return _load_file(path)


def read_config(src: Source, config: Optional[dict] = None) -> dict:
    if config is not None:
        return dict(config)
    if isinstance(src, Mapping):
        return {}
    p = os.fspath(src)
    cp = os.path.join(p if os.path.isdir(p) else os.path.dirname(p), "config.json")
    if os.path.exists(cp):
        with open(cp) as f:
            return json.load(f)
    return {}


def _strip(sd: StateDict, prefixes) -> StateDict:
    out = {}
    for k, v in sd.items():
        for p in prefixes:
            if k.startswith(p):
                k = k[len(p):]
                break
        out[k] = v
    return out


def _copy(dst: torch.Tensor, src: torch.Tensor, name: str) -> None:
    if tuple(dst.shape) != tuple(src.shape):
        raise ValueError(f"{name}: checkpoint shape {tuple(src.shape)} != model shape {tuple(dst.shape)}")
    with torch.no_grad():
        dst.copy_(src.to(device=dst.device, dtype=dst.dtype))


class _Keys:
    """Key lookup with alternative names and a record of what was consumed."""

    def __init__(self, sd: StateDict):
        self.sd, self.used = sd, set()

    def get(self, *names) -> torch.Tensor:
        for n in names:
            if n in self.sd:
                self.used.add(n)
                return self.sd[n]
        raise KeyError(f"checkpoint has none of {names}")

    def unused(self, ignore=()) -> list:
        return sorted(k for k in self.sd if k not in self.used and not any(i in k for i in ignore))


# ---------------------------------------------------------------------------
# BERT
# ---------------------------------------------------------------------------
def _bert_config(hf: dict, seq_len: int):
    from .bert import BertConfig

    if hf.get("hidden_act", "gelu") not in ("gelu", "gelu_python"):
        raise ValueError(f"BERT hidden_act {hf['hidden_act']!r}: the kernels implement erf GELU")
    n_labels = hf.get("num_labels") or len(hf.get("id2label", {})) or 2
    return BertConfig(vocab_size=hf.get("vocab_size", 30522), hidden=hf.get("hidden_size", 768),
                      layers=hf.get("num_hidden_layers", 12), heads=hf.get("num_attention_heads", 12),
                      intermediate=hf.get("intermediate_size", 3072),
                      max_position=hf.get("max_position_embeddings", 512), type_vocab=hf.get("type_vocab_size", 2),
                      eps=hf.get("layer_norm_eps", 1e-12), num_labels=n_labels, seq_len=seq_len,
                      pad_token_id=hf.get("pad_token_id", 0) or 0)


def load_bert_hf(model, src: Source, strict: bool = True):
    """Copy a Hugging Face BERT sequence-classification checkpoint into
    ``model`` (a ``BertForSequenceClassification`` of matching config)."""
    sd = _strip(load_state_dict(src), ("bert.",))
    k = _Keys(sd)

    def ln(prefix):
        return (k.get(prefix + ".weight", prefix + ".gamma"), k.get(prefix + ".bias", prefix + ".beta"))

    _copy(model.word, k.get("embeddings.word_embeddings.weight"), "word_embeddings")
    _copy(model.pos, k.get("embeddings.position_embeddings.weight"), "position_embeddings")
    _copy(model.typ, k.get("embeddings.token_type_embeddings.weight"), "token_type_embeddings")
    g, b = ln("embeddings.LayerNorm")
    _copy(model.emb_g, g, "embeddings.LayerNorm")
    _copy(model.emb_b, b, "embeddings.LayerNorm")
    for i, L in enumerate(model.layers):
        p = f"encoder.layer.{i}."
        wq = torch.cat([k.get(p + f"attention.self.{n}.weight") for n in ("query", "key", "value")])
        bq = torch.cat([k.get(p + f"attention.self.{n}.bias") for n in ("query", "key", "value")])
        _copy(L["w_qkv"], wq, p + "qkv")
        _copy(L["b_qkv"], bq, p + "qkv")
        _copy(L["w_o"], k.get(p + "attention.output.dense.weight"), p + "attention.output.dense")
        _copy(L["b_o"], k.get(p + "attention.output.dense.bias"), p + "attention.output.dense")
        g, b = ln(p + "attention.output.LayerNorm")
        _copy(L["ln1_g"], g, p + "ln1")
        _copy(L["ln1_b"], b, p + "ln1")
        _copy(L["w_i"], k.get(p + "intermediate.dense.weight"), p + "intermediate.dense")
        _copy(L["b_i"], k.get(p + "intermediate.dense.bias"), p + "intermediate.dense")
        _copy(L["w_out"], k.get(p + "output.dense.weight"), p + "output.dense")
        _copy(L["b_out"], k.get(p + "output.dense.bias"), p + "output.dense")
        g, b = ln(p + "output.LayerNorm")
        _copy(L["ln2_g"], g, p + "ln2")
        _copy(L["ln2_b"], b, p + "ln2")
    _copy(model.w_pool, k.get("pooler.dense.weight"), "pooler")
    _copy(model.b_pool, k.get("pooler.dense.bias"), "pooler")
    _copy(model.w_cls, k.get("classifier.weight"), "classifier")
    _copy(model.b_cls, k.get("classifier.bias"), "classifier")
    left = k.unused(ignore=("position_ids",))
    if strict and left:
        raise ValueError(f"unused checkpoint keys: {left[:8]}{' ...' if len(left) > 8 else ''}")
    if hasattr(model, "refresh_folded_weights"):
        model.refresh_folded_weights()
    return model


def bert_from_hf(src: Source, config: Optional[dict] = None, *, seq_len: int = 128, device="cuda",
                 dtype=torch.bfloat16, backend: str = "hip", strict: bool = True):
    from .bert import BertForSequenceClassification

    cfg = _bert_config(read_config(src, config), seq_len)
    m = BertForSequenceClassification(cfg, device=device, dtype=dtype, backend=backend)
    return load_bert_hf(m, src, strict=strict)


# ---------------------------------------------------------------------------
# Llama
# ---------------------------------------------------------------------------
def _rope_params(hf: dict):
    """(theta, scaling) from a config.json: top-level ``rope_theta`` /
    ``rope_scaling`` (transformers 4.x files) or ``rope_parameters`` (5.x)."""
    rp = hf.get("rope_parameters") or {}
    theta = float(rp.get("rope_theta", hf.get("rope_theta", 500000.0)))
    scaling = hf.get("rope_scaling") or (rp if rp.get("rope_type", "default") != "default" else None)
    return theta, scaling


def _llama_config(hf: dict, seq_len: int):
    from .llama import LlamaConfig

    heads = hf.get("num_attention_heads", 32)
    D = hf.get("hidden_size", 4096)
    return LlamaConfig(vocab_size=hf.get("vocab_size", 128256), hidden=D, layers=hf.get("num_hidden_layers", 32),
                       heads=heads, kv_heads=hf.get("num_key_value_heads", heads),
                       head_dim=hf.get("head_dim") or D // heads, intermediate=hf.get("intermediate_size", 14336),
                       rope_theta=_rope_params(hf)[0], eps=hf.get("rms_norm_eps", 1e-5),
                       max_position=hf.get("max_position_embeddings", 8192), seq_len=seq_len)


def llama_rope_tables(cfg, rope_scaling: Optional[dict], device=None):
    """cos / sin tables [max_position, head_dim/2]; ``rope_type == "llama3"``
    applies Llama-3.1's frequency-dependent scaling of the inverse
    frequencies (low frequencies / factor, high kept, smooth in between)."""
    D = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    rs = rope_scaling or {}
    kind = rs.get("rope_type", rs.get("type"))
    if kind == "llama3":
        factor, lo, hi = float(rs["factor"]), float(rs.get("low_freq_factor", 1.0)), float(rs.get("high_freq_factor", 4.0))
        old = float(rs.get("original_max_position_embeddings", 8192))
        wavelen = 2 * math.pi / inv
        scaled = torch.where(wavelen > old / lo, inv / factor, inv)
        smooth = (old / wavelen - lo) / (hi - lo)
        mid = (wavelen <= old / lo) & (wavelen >= old / hi)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    elif kind not in (None, "default"):
        raise ValueError(f"rope_scaling type {kind!r} is not supported")
    f = torch.outer(torch.arange(cfg.max_position, dtype=torch.float64), inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def load_llama_hf(model, src: Source, config: Optional[dict] = None, strict: bool = True):
    """Copy this rank's shard of a Hugging Face Llama checkpoint into ``model``
    (a ``LlamaTP``; any ``tp_rank`` / ``tp_size``)."""
    hf = read_config(src, config)
    sd = _strip(load_state_dict(src), ("model.",))
    k = _Keys(sd)
    c, r = model.cfg, model.rank
    Dh, Hl, Hkvl, Fl, Vl = c.head_dim, model.Hl, model.Hkvl, model.Fl, model.Vl
    _copy(model.embed, k.get("embed_tokens.weight"), "embed_tokens")
    for i, L in enumerate(model.layers):
        p = f"layers.{i}."
        q = k.get(p + "self_attn.q_proj.weight")[r * Hl * Dh:(r + 1) * Hl * Dh]
        kk = k.get(p + "self_attn.k_proj.weight")[r * Hkvl * Dh:(r + 1) * Hkvl * Dh]
        v = k.get(p + "self_attn.v_proj.weight")[r * Hkvl * Dh:(r + 1) * Hkvl * Dh]
        _copy(L["w_qkv"], torch.cat([q, kk, v]), p + "qkv")
        _copy(L["w_o"], k.get(p + "self_attn.o_proj.weight")[:, r * Hl * Dh:(r + 1) * Hl * Dh], p + "o_proj")
        g = k.get(p + "mlp.gate_proj.weight")[r * Fl:(r + 1) * Fl]
        u = k.get(p + "mlp.up_proj.weight")[r * Fl:(r + 1) * Fl]
        _copy(L["w_gu"], torch.stack([g, u], dim=1).reshape(2 * Fl, -1), p + "gate_up")
        _copy(L["w_down"], k.get(p + "mlp.down_proj.weight")[:, r * Fl:(r + 1) * Fl], p + "down_proj")
        _copy(L["attn_norm"], k.get(p + "input_layernorm.weight"), p + "input_layernorm")
        _copy(L["mlp_norm"], k.get(p + "post_attention_layernorm.weight"), p + "post_attention_layernorm")
    _copy(model.final_norm, k.get("norm.weight"), "norm")
    head = sd.get("lm_head.weight")
    if head is not None:
        k.used.add("lm_head.weight")
    elif hf.get("tie_word_embeddings", False) or "lm_head.weight" not in sd:
        head = k.get("embed_tokens.weight")
    _copy(model.lm_head, head[r * Vl:(r + 1) * Vl], "lm_head")
    if hf:
        theta, scaling = _rope_params(hf)
        if scaling or theta != c.rope_theta:
            if theta != c.rope_theta:
                raise ValueError(f"checkpoint rope_theta {theta} != model rope_theta {c.rope_theta}")
            model.cos, model.sin = llama_rope_tables(c, scaling, device=model.device)
    left = k.unused(ignore=("rotary_emb.inv_freq",))
    if strict and left:
        raise ValueError(f"unused checkpoint keys: {left[:8]}{' ...' if len(left) > 8 else ''}")
    return model


def llama_from_hf(src: Source, config: Optional[dict] = None, *, seq_len: int = 512, tp_rank: int = 0,
                  tp_size: int = 1, group_name: Optional[str] = None, device="cuda", dtype=torch.bfloat16,
                  backend: str = "hip", strict: bool = True):
    from .llama import LlamaTP

    hf = read_config(src, config)
    cfg = _llama_config(hf, seq_len)
    m = LlamaTP(cfg, tp_rank=tp_rank, tp_size=tp_size, group_name=group_name, device=device, dtype=dtype,
                backend=backend)
    return load_llama_hf(m, src, config=hf, strict=strict)


# ---------------------------------------------------------------------------
# ResNet-50 (torchvision keys)
# ---------------------------------------------------------------------------
def load_resnet50(model, src: Source, strict: bool = True):
    """torchvision ``resnet50`` state dict -> ``ResNet50``: each conv's
    BatchNorm (eval statistics) is folded into the conv weight and a bias."""
    return model.load_torchvision_state_dict(load_state_dict(src), strict=strict)


# ---------------------------------------------------------------------------
# ViT (Hugging Face or torchvision keys)
# ---------------------------------------------------------------------------
_IMAGENET_MEAN = (0.485, 0.456, 0.406)
_IMAGENET_STD = (0.229, 0.224, 0.225)


def _vit_config(hf: dict):
    from .vit import ViTConfig

    n = hf.get("num_labels") or len(hf.get("id2label", {})) or 1000
    return ViTConfig(image=hf.get("image_size", 224), patch=hf.get("patch_size", 16), hidden=hf.get("hidden_size", 768),
                     layers=hf.get("num_hidden_layers", 12), heads=hf.get("num_attention_heads", 12),
                     mlp=hf.get("intermediate_size", 3072), classes=n, eps=hf.get("layer_norm_eps", 1e-12))


def load_vit(model, src: Source, image_mean=None, image_std=None, strict: bool = True):
    """HF ``ViTForImageClassification`` (default normalisation 0.5 / 0.5) or
    torchvision ``vit_b_16`` (ImageNet normalisation) weights -> ``ViT``."""
    sd = load_state_dict(src)
    tv = "conv_proj.weight" in sd
    if image_mean is None:
        image_mean = _IMAGENET_MEAN if tv else (0.5, 0.5, 0.5)
    if image_std is None:
        image_std = _IMAGENET_STD if tv else (0.5, 0.5, 0.5)
    k = _Keys(_strip(sd, ("vit.",)))
    c = model.cfg
    if tv:
        pw, pb = k.get("conv_proj.weight"), k.get("conv_proj.bias")
        cls, pos = k.get("class_token"), k.get("encoder.pos_embedding")
    else:
        pw, pb = k.get("embeddings.patch_embeddings.projection.weight"), k.get("embeddings.patch_embeddings.projection.bias")
        cls, pos = k.get("embeddings.cls_token"), k.get("embeddings.position_embeddings")
    # the model sees x_ours = (u - m_in) / s_in; the checkpoint expects
    # x_ck = (u - m_ck) / s_ck = x_ours * s_in / s_ck + (m_in - m_ck) / s_ck
    m_in, s_in = torch.tensor(_IMAGENET_MEAN), torch.tensor(_IMAGENET_STD)
    m_ck, s_ck = torch.tensor(image_mean, dtype=torch.float32), torch.tensor(image_std, dtype=torch.float32)
    pw = pw.float()
    w_eff = pw * (s_in / s_ck)[None, :, None, None]
    b_eff = pb.float() + (pw * ((m_in - m_ck) / s_ck)[None, :, None, None]).sum(dim=(1, 2, 3))
    with torch.no_grad():
        model.patch_w.zero_()
    _copy(model.patch_w[..., :3], w_eff.permute(0, 2, 3, 1), "patch_embed")
    _copy(model.patch_b, b_eff, "patch_embed")
    _copy(model.cls, cls, "cls_token")
    _copy(model.pos, pos, "position_embeddings")
    for i, L in enumerate(model.layers):
        if tv:
            p = f"encoder.layers.encoder_layer_{i}."
            names = dict(ln1=p + "ln_1", qkv_w=[p + "self_attention.in_proj_weight"],
                         qkv_b=[p + "self_attention.in_proj_bias"], o=p + "self_attention.out_proj", ln2=p + "ln_2",
                         fc1=p + "mlp.0", fc2=p + "mlp.3")
        elif f"layers.{i}.attention.q_proj.weight" in k.sd:      # transformers 5 in-memory names
            p = f"layers.{i}."
            names = dict(ln1=p + "layernorm_before",
                         qkv_w=[p + f"attention.{n}_proj.weight" for n in "qkv"],
                         qkv_b=[p + f"attention.{n}_proj.bias" for n in "qkv"],
                         o=p + "attention.o_proj", ln2=p + "layernorm_after", fc1=p + "mlp.fc1", fc2=p + "mlp.fc2")
        else:                                                     # checkpoint-file names
            p = f"encoder.layer.{i}."
            names = dict(ln1=p + "layernorm_before",
                         qkv_w=[p + f"attention.attention.{n}.weight" for n in ("query", "key", "value")],
                         qkv_b=[p + f"attention.attention.{n}.bias" for n in ("query", "key", "value")],
                         o=p + "attention.output.dense", ln2=p + "layernorm_after", fc1=p + "intermediate.dense",
                         fc2=p + "output.dense")
        _copy(L["ln1_g"], k.get(names["ln1"] + ".weight"), p + "ln1")
        _copy(L["ln1_b"], k.get(names["ln1"] + ".bias"), p + "ln1")
        _copy(L["w_qkv"], torch.cat([k.get(n) for n in names["qkv_w"]]), p + "qkv")
        _copy(L["b_qkv"], torch.cat([k.get(n) for n in names["qkv_b"]]), p + "qkv")
        _copy(L["w_o"], k.get(names["o"] + ".weight"), p + "o")
        _copy(L["b_o"], k.get(names["o"] + ".bias"), p + "o")
        _copy(L["ln2_g"], k.get(names["ln2"] + ".weight"), p + "ln2")
        _copy(L["ln2_b"], k.get(names["ln2"] + ".bias"), p + "ln2")
        _copy(L["w1"], k.get(names["fc1"] + ".weight"), p + "fc1")
        _copy(L["b1"], k.get(names["fc1"] + ".bias"), p + "fc1")
        _copy(L["w2"], k.get(names["fc2"] + ".weight"), p + "fc2")
        _copy(L["b2"], k.get(names["fc2"] + ".bias"), p + "fc2")
    ln, head = ("encoder.ln", "heads.head") if tv else ("layernorm", "classifier")
    _copy(model.ln_g, k.get(ln + ".weight"), "final_ln")
    _copy(model.ln_b, k.get(ln + ".bias"), "final_ln")
    _copy(model.head_w, k.get(head + ".weight"), "head")
    _copy(model.head_b, k.get(head + ".bias"), "head")
    left = k.unused(ignore=("pooler",))
    if strict and left:
        raise ValueError(f"unused checkpoint keys: {left[:8]}{' ...' if len(left) > 8 else ''}")
    return model


def vit_from_hf(src: Source, config: Optional[dict] = None, *, device="cuda", dtype=torch.float16,
                backend: str = "hip", image_mean=None, image_std=None, strict: bool = True):
    from .vit import ViT

    m = ViT(_vit_config(read_config(src, config)), device=device, dtype=dtype, backend=backend)
    return load_vit(m, src, image_mean=image_mean, image_std=image_std, strict=strict)


def shufflenet_v2_from_torchvision(src: Source, *, device="cuda", dtype=torch.float16, backend: str = "hip",
                                   strict: bool = True, **kw):
    from .shufflenet import ShuffleNetV2

    sd = load_state_dict(src)
    classes = sd["fc.weight"].shape[0] if "fc.weight" in sd else 1000
    return ShuffleNetV2(device=device, dtype=dtype, backend=backend, num_classes=classes, state_dict=sd,
                        strict=strict, **kw)


def efficientnet_v2s_from_torchvision(src: Source, *, device="cuda", dtype=torch.float16, backend: str = "hip",
                                      strict: bool = True, **kw):
    from .efficientnet import EfficientNetV2S

    sd = load_state_dict(src)
    classes = sd["classifier.1.weight"].shape[0] if "classifier.1.weight" in sd else 1000
    return EfficientNetV2S(device=device, dtype=dtype, backend=backend, num_classes=classes, state_dict=sd,
                           strict=strict, **kw)
