"""Checkpoint loading (models/weights.py): Hugging Face BERT and Llama
checkpoints (built from a config with random init by ``transformers`` -- no
download) and torchvision-format ResNet-50 weights (a torchvision-compatible
nn reference defined here, since torchvision is not installed) load into this
framework's models, whose outputs then match the independent implementations.
CPU tests run the eager backends in fp32; the GPU tests run the HIP kernels."""
import math

import pytest
import torch
import torch.nn as nn

from ray_dynamic_batching_amd.models import weights as W

transformers = pytest.importorskip("transformers")


# ---------------------------------------------------------------------------
# fixtures: reference models
# ---------------------------------------------------------------------------
def _hf_bert(tmp_path, num_labels=3, hidden=128):
    cfg = transformers.BertConfig(vocab_size=1000, hidden_size=hidden, num_hidden_layers=2,
                                  num_attention_heads=hidden // 64 if hidden >= 256 else 4,
                                  intermediate_size=2 * hidden, max_position_embeddings=64, num_labels=num_labels)
    torch.manual_seed(0)
    m = transformers.BertForSequenceClassification(cfg).eval()
    with torch.no_grad():                      # non-trivial LayerNorm affine params
        for n, p in m.named_parameters():
            if "LayerNorm" in n:
                p.add_(torch.randn_like(p) * 0.1)
    m.save_pretrained(tmp_path / "bert")
    return m


def _bert_ids(n=5, S=32, vocab=1000):
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1, vocab, (n, S), generator=g)
    ids[:, 0] = 101
    ids[1, 20:] = 0                            # padded sequences
    ids[3, 5:] = 0
    return ids


def _hf_llama(tmp_path, tied=False, scaling=True):
    cfg = transformers.LlamaConfig(
        vocab_size=512, hidden_size=256, num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
        head_dim=64, intermediate_size=512, max_position_embeddings=128, rope_theta=10000.0, rms_norm_eps=1e-5,
        tie_word_embeddings=tied,
        rope_scaling=({"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                       "original_max_position_embeddings": 32} if scaling else None))
    torch.manual_seed(2)
    m = transformers.LlamaForCausalLM(cfg).eval()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.add_(torch.randn_like(p) * 0.1)
    m.save_pretrained(tmp_path / "llama")
    return m


class _Bottleneck(nn.Module):
    def __init__(self, cin, width, stride, down):
        super().__init__()
        self.conv1, self.bn1 = nn.Conv2d(cin, width, 1, bias=False), nn.BatchNorm2d(width)
        self.conv2, self.bn2 = nn.Conv2d(width, width, 3, stride, 1, bias=False), nn.BatchNorm2d(width)
        self.conv3, self.bn3 = nn.Conv2d(width, width * 4, 1, bias=False), nn.BatchNorm2d(width * 4)
        self.downsample = nn.Sequential(nn.Conv2d(cin, width * 4, 1, stride, bias=False),
                                        nn.BatchNorm2d(width * 4)) if down else None

    def forward(self, x):
        h = torch.relu(self.bn1(self.conv1(x)))
        h = torch.relu(self.bn2(self.conv2(h)))
        h = self.bn3(self.conv3(h))
        return torch.relu(h + (self.downsample(x) if self.downsample is not None else x))


class _TVResNet50(nn.Module):
    """torchvision.models.resnet50's module names and structure (v1.5: stride on the 3x3)."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.conv1, self.bn1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64)
        cin = 64
        for si, (width, n, stride) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]):
            blocks = []
            for i in range(n):
                s = stride if i == 0 else 1
                blocks.append(_Bottleneck(cin, width, s, s != 1 or cin != width * 4))
                cin = width * 4
            setattr(self, f"layer{si + 1}", nn.Sequential(*blocks))
        self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = nn.functional.max_pool2d(torch.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        for i in range(1, 5):
            x = getattr(self, f"layer{i}")(x)
        return self.fc(x.mean(dim=(2, 3)))


def _tv_resnet():
    torch.manual_seed(3)
    m = _TVResNet50()
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, nn.BatchNorm2d):
                mod.running_mean.normal_(0, 0.05)
                mod.running_var.uniform_(0.8, 1.2)
                mod.weight.uniform_(0.3, 0.7)
                mod.bias.normal_(0, 0.05)
    return m.eval()


def _normalize(img):
    mean = torch.tensor([0.485, 0.456, 0.406])
    std = torch.tensor([0.229, 0.224, 0.225])
    return ((img.float() / 255.0 - mean) / std).permute(0, 3, 1, 2)


# ---------------------------------------------------------------------------
# CPU: eager backends, fp32
# ---------------------------------------------------------------------------
def test_bert_hf_checkpoint_matches_transformers(tmp_path):
    ref = _hf_bert(tmp_path)
    ids = _bert_ids()
    with torch.no_grad():
        want = ref(input_ids=ids, attention_mask=(ids != 0).long()).logits
    m = W.bert_from_hf(tmp_path / "bert", seq_len=32, device="cpu", dtype=torch.float32, backend="torch")
    assert m.cfg.num_labels == 3 and m.cfg.hidden == 128
    got = m(ids.to(torch.int32))
    assert torch.allclose(got, want, atol=1e-4, rtol=1e-4), (got - want).abs().max()
    # a state dict in memory, old gamma/beta LayerNorm names, strictness
    sd = {k.replace("LayerNorm.weight", "LayerNorm.gamma").replace("LayerNorm.bias", "LayerNorm.beta"): v
          for k, v in ref.state_dict().items()}
    m2 = W.load_bert_hf(type(m)(m.cfg, device="cpu", dtype=torch.float32, backend="torch"), sd)
    assert torch.allclose(m2(ids.to(torch.int32)), want, atol=1e-4, rtol=1e-4)
    with pytest.raises(ValueError, match="unused"):
        W.load_bert_hf(m2, dict(sd, extra_head=torch.zeros(1)))
    with pytest.raises(ValueError, match="shape"):
        W.bert_from_hf(tmp_path / "bert", config=dict(ref.config.to_dict(), hidden_size=64, intermediate_size=128),
                       seq_len=32, device="cpu", dtype=torch.float32, backend="torch")


@pytest.mark.parametrize("tied,scaling", [(False, True), (True, False)])
def test_llama_hf_checkpoint_matches_transformers(tmp_path, tied, scaling):
    ref = _hf_llama(tmp_path, tied=tied, scaling=scaling)
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(1, 512, (3, 48), generator=g)
    with torch.no_grad():
        logits = ref(input_ids=ids).logits[:, -1].float()
    m = W.llama_from_hf(tmp_path / "llama", seq_len=48, device="cpu", dtype=torch.float32, backend="torch")
    out = m(ids.to(torch.int32))
    assert torch.equal(out[:, 0].long(), logits.argmax(-1))
    assert torch.allclose(out[:, 1].contiguous().view(torch.float32), logits.max(-1).values, atol=1e-4, rtol=1e-4)


def test_llama_hf_tp_shards_tile_the_full_model(tmp_path):
    _hf_llama(tmp_path)
    full = W.llama_from_hf(tmp_path / "llama", seq_len=16, device="cpu", dtype=torch.float32, backend="torch")
    ranks = [W.llama_from_hf(tmp_path / "llama", seq_len=16, tp_rank=r, tp_size=2, device="cpu",
                             dtype=torch.float32, backend="torch") for r in range(2)]
    Dh, Hl, Hkvl = 64, 2, 1
    for i, L in enumerate(full.layers):
        q = torch.cat([r.layers[i]["w_qkv"][:Hl * Dh] for r in ranks])
        k = torch.cat([r.layers[i]["w_qkv"][Hl * Dh:(Hl + Hkvl) * Dh] for r in ranks])
        assert torch.equal(q, L["w_qkv"][:2 * Hl * Dh]) and torch.equal(k, L["w_qkv"][4 * Dh:6 * Dh])
        assert torch.equal(torch.cat([r.layers[i]["w_o"] for r in ranks], 1), L["w_o"])
        assert torch.equal(torch.cat([r.layers[i]["w_down"] for r in ranks], 1), L["w_down"])
    assert torch.equal(torch.cat([r.lm_head for r in ranks]), full.lm_head)


def test_llama3_rope_scaling_matches_transformers():
    from ray_dynamic_batching_amd.models.llama import LlamaConfig

    rs = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
          "original_max_position_embeddings": 32}
    hf_cfg = transformers.LlamaConfig(hidden_size=256, num_attention_heads=4, head_dim=64, rope_theta=10000.0,
                                      max_position_embeddings=128, rope_scaling=rs)
    from transformers.modeling_rope_utils import ROPE_INIT_FUNCTIONS

    inv, _ = ROPE_INIT_FUNCTIONS["llama3"](hf_cfg, "cpu")
    cos, _ = W.llama_rope_tables(LlamaConfig(head_dim=64, rope_theta=10000.0, max_position=128), rs)
    want = torch.outer(torch.arange(128, dtype=torch.float64), inv.double()).cos().float()
    assert torch.allclose(cos, want, atol=1e-5)


def test_resnet50_torchvision_weights_fold_bn():
    from ray_dynamic_batching_amd.models.resnet import ResNet50

    ref = _tv_resnet()
    img = torch.randint(0, 256, (2, 64, 64, 3), dtype=torch.uint8)
    with torch.no_grad():
        want = ref(_normalize(img))
    m = ResNet50(device="cpu", backend="torch", image_size=64)
    W.load_resnet50(m, ref.state_dict())
    got = m.logits(img)
    assert torch.allclose(got, want, atol=2e-3 * want.abs().max().item(), rtol=1e-3), (got - want).abs().max()
    with pytest.raises(KeyError):
        W.load_resnet50(m, {k: v for k, v in ref.state_dict().items() if k != "fc.bias"})


def test_checkpoint_files(tmp_path):
    from safetensors.torch import save_file

    sd = {"a": torch.arange(4.0), "b": torch.ones(2, 2)}
    save_file(sd, str(tmp_path / "m.safetensors"))
    torch.save(sd, tmp_path / "m.pt")
    for p in ("m.safetensors", "m.pt"):
        got = W.load_state_dict(tmp_path / p)
        assert set(got) == {"a", "b"} and torch.equal(got["a"], sd["a"])
    (tmp_path / "shards").mkdir()
    save_file({"a": sd["a"]}, str(tmp_path / "shards" / "s1.safetensors"))
    save_file({"b": sd["b"]}, str(tmp_path / "shards" / "s2.safetensors"))
    import json

    (tmp_path / "shards" / "model.safetensors.index.json").write_text(
        json.dumps({"weight_map": {"a": "s1.safetensors", "b": "s2.safetensors"}}))
    assert set(W.load_state_dict(tmp_path / "shards")) == {"a", "b"}
    with pytest.raises(ValueError):
        W.load_state_dict(tmp_path / "m.pkl")


# ---------------------------------------------------------------------------
# GPU: the HIP kernels on loaded weights
# ---------------------------------------------------------------------------
@pytest.mark.gpu
def test_bert_hf_checkpoint_on_hip_kernels(tmp_path):
    ref = _hf_bert(tmp_path, hidden=256)           # the kernels take hidden = 256 k, head dim 64
    ids = _bert_ids()
    with torch.no_grad():
        want = ref(input_ids=ids, attention_mask=(ids != 0).long()).logits
    m = W.bert_from_hf(tmp_path / "bert", seq_len=32, device="cuda", backend="hip")
    got = m(ids.to(torch.int32).cuda()).cpu()
    assert torch.allclose(got, want, atol=5e-2, rtol=5e-2), (got - want).abs().max()


@pytest.mark.gpu
def test_llama_hf_checkpoint_on_hip_kernels(tmp_path):
    ref = _hf_llama(tmp_path)
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(1, 512, (3, 64), generator=g)
    with torch.no_grad():
        logits = ref(input_ids=ids).logits[:, -1].float()
    m = W.llama_from_hf(tmp_path / "llama", seq_len=64, device="cuda", backend="hip")
    out = m(ids.to(torch.int32).cuda()).cpu()
    top = logits.max(-1).values
    assert torch.allclose(out[:, 1].contiguous().view(torch.float32), top, atol=5e-2, rtol=5e-2)
    picked = logits[torch.arange(3), out[:, 0].long()]
    assert torch.all(top - picked < 5e-2)          # the chosen token is a (near-)argmax in fp32


@pytest.mark.gpu
def test_resnet50_torchvision_weights_on_hip_kernels():
    from ray_dynamic_batching_amd.models.resnet import ResNet50

    ref = _tv_resnet()
    img = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8)
    with torch.no_grad():
        want = ref(_normalize(img))
    m = ResNet50(device="cuda", backend="hip")
    W.load_resnet50(m, ref.state_dict())
    got = m.logits(img.cuda()).cpu()
    scale = want.abs().max().item()
    assert (got - want).abs().max().item() < 3e-2 * scale + 1e-2


def test_factories_take_checkpoints(tmp_path):
    from ray_dynamic_batching_amd.models import factories

    ref = _hf_bert(tmp_path, num_labels=5)
    f = factories.bert_base(seq_len=32, backend="torch", checkpoint=str(tmp_path / "bert"))
    assert f.io_spec[2] == (5,)
    m = f(device="cpu")
    ids = _bert_ids()
    with torch.no_grad():
        want = ref(input_ids=ids, attention_mask=(ids != 0).long()).logits
    assert torch.allclose(m(ids.to(torch.int32)).float(), want, atol=3e-2, rtol=3e-2)   # bf16 weights
    tv = _tv_resnet()
    torch.save(tv.state_dict(), tmp_path / "rn50.pth")
    r = factories.resnet50(backend="torch", checkpoint=str(tmp_path / "rn50.pth"))(device="cpu")
    assert torch.equal(r.fc_b.float(), tv.fc.bias.detach().to(r.fc_b.dtype).float())


def _hf_vit(tmp_path, hidden=256):
    cfg = transformers.ViTConfig(image_size=64, patch_size=16, hidden_size=hidden, num_hidden_layers=2,
                                 num_attention_heads=hidden // 64, intermediate_size=2 * hidden, num_labels=10,
                                 layer_norm_eps=1e-12)
    torch.manual_seed(5)
    m = transformers.ViTForImageClassification(cfg).eval()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "layernorm" in n or "embeddings" in n:
                p.add_(torch.randn_like(p) * 0.1)
    m.save_pretrained(tmp_path / "vit")
    return m


def _hf_vit_input(img):
    return ((img.float() / 255.0 - 0.5) / 0.5).permute(0, 3, 1, 2)    # HF ViT image processor


def test_vit_hf_checkpoint_matches_transformers(tmp_path):
    ref = _hf_vit(tmp_path)
    img = torch.randint(0, 256, (3, 64, 64, 3), dtype=torch.uint8)
    with torch.no_grad():
        want = ref(pixel_values=_hf_vit_input(img)).logits
    m = W.vit_from_hf(tmp_path / "vit", device="cpu", dtype=torch.float32, backend="torch")
    got = m.logits(img)
    assert torch.allclose(got, want, atol=1e-3, rtol=1e-3), (got - want).abs().max()
    # in-memory (transformers 5 module names) state dict
    m1 = W.load_vit(type(m)(m.cfg, device="cpu", dtype=torch.float32, backend="torch"), ref.state_dict())
    assert torch.allclose(m1.logits(img), want, atol=1e-3, rtol=1e-3)
    # the same weights under torchvision's vit_b_16 key names and ImageNet normalisation
    sd = W.load_state_dict(tmp_path / "vit")                  # checkpoint-file names
    tv = {"conv_proj.weight": sd["vit.embeddings.patch_embeddings.projection.weight"],
          "conv_proj.bias": sd["vit.embeddings.patch_embeddings.projection.bias"],
          "class_token": sd["vit.embeddings.cls_token"], "encoder.pos_embedding": sd["vit.embeddings.position_embeddings"],
          "encoder.ln.weight": sd["vit.layernorm.weight"], "encoder.ln.bias": sd["vit.layernorm.bias"],
          "heads.head.weight": sd["classifier.weight"], "heads.head.bias": sd["classifier.bias"]}
    for i in range(2):
        p, q = f"vit.encoder.layer.{i}.", f"encoder.layers.encoder_layer_{i}."
        for a, b in (("layernorm_before", "ln_1"), ("layernorm_after", "ln_2"), ("attention.output.dense",
                     "self_attention.out_proj"), ("intermediate.dense", "mlp.0"), ("output.dense", "mlp.3")):
            for t in ("weight", "bias"):
                tv[f"{q}{b}.{t}"] = sd[f"{p}{a}.{t}"]
        for t in ("weight", "bias"):
            tv[f"{q}self_attention.in_proj_{t}"] = torch.cat(
                [sd[f"{p}attention.attention.{n}.{t}"] for n in ("query", "key", "value")])
    m2 = W.load_vit(type(m)(m.cfg, device="cpu", dtype=torch.float32, backend="torch"), tv)
    # torchvision checkpoints expect ImageNet normalisation = this model's input space
    with torch.no_grad():
        mean = torch.tensor([0.485, 0.456, 0.406])
        std = torch.tensor([0.229, 0.224, 0.225])
        want_tv = ref(pixel_values=((img.float() / 255.0 - mean) / std).permute(0, 3, 1, 2)).logits
    assert torch.allclose(m2.logits(img), want_tv, atol=1e-3, rtol=1e-3)


@pytest.mark.gpu
def test_vit_hf_checkpoint_on_hip_kernels(tmp_path):
    ref = _hf_vit(tmp_path)
    img = torch.randint(0, 256, (3, 64, 64, 3), dtype=torch.uint8)
    with torch.no_grad():
        want = ref(pixel_values=_hf_vit_input(img)).logits
    m = W.vit_from_hf(tmp_path / "vit", device="cuda", backend="hip")
    got = m.logits(img.cuda()).cpu()
    assert (got - want).abs().max().item() < 3e-2 * want.abs().max().item() + 1e-2


class _TVInvertedResidual(nn.Module):
    """torchvision.models.shufflenetv2.InvertedResidual (module names and math)."""

    def __init__(self, inp, oup, stride):
        super().__init__()
        self.stride = stride
        bf = oup // 2
        if stride > 1:
            self.branch1 = nn.Sequential(nn.Conv2d(inp, inp, 3, stride, 1, groups=inp, bias=False), nn.BatchNorm2d(inp),
                                         nn.Conv2d(inp, bf, 1, bias=False), nn.BatchNorm2d(bf), nn.ReLU())
        else:
            self.branch1 = nn.Sequential()
        self.branch2 = nn.Sequential(
            nn.Conv2d(inp if stride > 1 else bf, bf, 1, bias=False), nn.BatchNorm2d(bf), nn.ReLU(),
            nn.Conv2d(bf, bf, 3, stride, 1, groups=bf, bias=False), nn.BatchNorm2d(bf),
            nn.Conv2d(bf, bf, 1, bias=False), nn.BatchNorm2d(bf), nn.ReLU())

    def forward(self, x):
        if self.stride == 1:
            x1, x2 = x.chunk(2, dim=1)
            out = torch.cat((x1, self.branch2(x2)), dim=1)
        else:
            out = torch.cat((self.branch1(x), self.branch2(x)), dim=1)
        b, c, h, w = out.shape
        return out.view(b, 2, c // 2, h, w).transpose(1, 2).reshape(b, c, h, w)


class _TVShuffleNetV2(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.conv1 = nn.Sequential(nn.Conv2d(3, 24, 3, 2, 1, bias=False), nn.BatchNorm2d(24), nn.ReLU())
        cin = 24
        for s, (rep, cout) in enumerate(zip([4, 8, 4], [116, 232, 464])):
            units = [_TVInvertedResidual(cin, cout, 2)] + [_TVInvertedResidual(cout, cout, 1) for _ in range(rep - 1)]
            setattr(self, f"stage{s + 2}", nn.Sequential(*units))
            cin = cout
        self.conv5 = nn.Sequential(nn.Conv2d(cin, 1024, 1, bias=False), nn.BatchNorm2d(1024), nn.ReLU())
        self.fc = nn.Linear(1024, num_classes)

    def forward(self, x):
        x = nn.functional.max_pool2d(self.conv1(x), 3, 2, 1)
        x = self.conv5(self.stage4(self.stage3(self.stage2(x))))
        return self.fc(x.mean([2, 3]))


def _tv_shufflenet():
    torch.manual_seed(6)
    m = _TVShuffleNetV2()
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, nn.BatchNorm2d):
                mod.running_mean.normal_(0, 0.05)
                mod.running_var.uniform_(0.8, 1.2)
                mod.weight.uniform_(0.5, 1.0)
                mod.bias.normal_(0, 0.05)
    return m.eval()


def test_shufflenet_torchvision_weights():
    ref = _tv_shufflenet()
    img = torch.randint(0, 256, (2, 64, 64, 3), dtype=torch.uint8)
    with torch.no_grad():
        want = ref(_normalize(img))
    m = W.shufflenet_v2_from_torchvision(ref.state_dict(), device="cpu", backend="torch", image_size=64)
    got = m.logits(img)
    assert torch.allclose(got, want, atol=2e-3 * want.abs().max().item(), rtol=1e-3), (got - want).abs().max()
    bad = dict(ref.state_dict(), extra=torch.zeros(1))
    with pytest.raises(ValueError):
        W.shufflenet_v2_from_torchvision(bad, device="cpu", backend="torch")


@pytest.mark.gpu
def test_shufflenet_torchvision_weights_on_hip_kernels():
    ref = _tv_shufflenet()
    img = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8)
    with torch.no_grad():
        want = ref(_normalize(img))
    m = W.shufflenet_v2_from_torchvision(ref.state_dict(), device="cuda", backend="hip")
    got = m.logits(img.cuda()).cpu()
    assert (got - want).abs().max().item() < 3e-2 * want.abs().max().item() + 1e-2


def _cna(cin, cout, k, s=1, groups=1, act=True):
    layers = [nn.Conv2d(cin, cout, k, s, (k - 1) // 2, groups=groups, bias=False), nn.BatchNorm2d(cout, eps=1e-3)]
    return nn.Sequential(*(layers + ([nn.SiLU()] if act else [])))


class _TVSE(nn.Module):
    def __init__(self, hid, sq):
        super().__init__()
        self.fc1, self.fc2 = nn.Conv2d(hid, sq, 1), nn.Conv2d(sq, hid, 1)

    def forward(self, x):
        z = torch.sigmoid(self.fc2(nn.functional.silu(self.fc1(x.mean((2, 3), keepdim=True)))))
        return x * z


class _TVEffBlock(nn.Module):
    """torchvision FusedMBConv / MBConv (module names; stochastic depth = identity in eval)."""

    def __init__(self, kind, e, s, ci, co):
        super().__init__()
        hid = ci * e
        self.res = s == 1 and ci == co
        if kind == "fused":
            blocks = [_cna(ci, co, 3, s)] if e == 1 else [_cna(ci, hid, 3, s), _cna(hid, co, 1, act=False)]
        else:
            blocks = [_cna(ci, hid, 1), _cna(hid, hid, 3, s, groups=hid), _TVSE(hid, max(1, ci // 4)),
                      _cna(hid, co, 1, act=False)]
        self.block = nn.Sequential(*blocks)

    def forward(self, x):
        y = self.block(x)
        return y + x if self.res else y


class _TVEfficientNetV2S(nn.Module):
    def __init__(self, config, num_classes=1000):
        super().__init__()
        feats = [_cna(3, 24, 3, 2)]
        for kind, e, s, ci, co, n in config:
            feats.append(nn.Sequential(*[_TVEffBlock(kind, e, s if i == 0 else 1, ci if i == 0 else co, co)
                                         for i in range(n)]))
        feats.append(_cna(256, 1280, 1))
        self.features = nn.Sequential(*feats)
        self.classifier = nn.Sequential(nn.Dropout(0.2), nn.Linear(1280, num_classes))

    def forward(self, x):
        return self.classifier(self.features(x).mean((2, 3)))


_EFF_SMALL = [("fused", 1, 1, 24, 24, 2), ("fused", 4, 2, 24, 48, 1), ("fused", 4, 2, 48, 64, 1),
              ("mb", 4, 2, 64, 128, 2), ("mb", 6, 1, 128, 160, 1), ("mb", 6, 2, 160, 256, 2)]


def _tv_effnet(config):
    torch.manual_seed(7)
    m = _TVEfficientNetV2S(config)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, nn.BatchNorm2d):
                mod.running_mean.normal_(0, 0.05)
                mod.running_var.uniform_(0.8, 1.2)
                mod.weight.uniform_(0.5, 1.0)
                mod.bias.normal_(0, 0.05)
    return m.eval()


def test_efficientnet_v2s_torchvision_weights():
    ref = _tv_effnet(_EFF_SMALL)
    img = torch.randint(0, 256, (2, 64, 64, 3), dtype=torch.uint8)
    with torch.no_grad():
        want = ref(_normalize(img))
    m = W.efficientnet_v2s_from_torchvision(ref.state_dict(), device="cpu", backend="torch", image_size=64,
                                            config=_EFF_SMALL)
    got = m.logits(img)
    assert torch.allclose(got, want, atol=2e-3 * want.abs().max().item(), rtol=1e-3), (got - want).abs().max()


@pytest.mark.gpu
def test_efficientnet_v2s_torchvision_weights_on_hip_kernels():
    from ray_dynamic_batching_amd.models.efficientnet import CONFIG

    ref = _tv_effnet(CONFIG)
    img = torch.randint(0, 256, (2, 384, 384, 3), dtype=torch.uint8)
    with torch.no_grad():
        want = ref(_normalize(img))
    m = W.efficientnet_v2s_from_torchvision(ref.state_dict(), device="cuda", backend="hip")
    got = m.logits(img.cuda()).cpu()
    assert (got - want).abs().max().item() < 5e-2 * want.abs().max().item() + 1e-2


def test_registry_create_with_checkpoint(tmp_path):
    from ray_dynamic_batching_amd import models

    _hf_llama(tmp_path, scaling=False)
    m = models.create("llama3-8b", checkpoint=str(tmp_path / "llama"), seq_len=16, device="cpu",
                      dtype=torch.float32, backend="torch")
    assert m.cfg.hidden == 256 and m.cfg.layers == 2
    ref = _tv_shufflenet()
    torch.save(ref.state_dict(), tmp_path / "sn.pth")
    sn = models.create("shufflenet-v2", checkpoint=str(tmp_path / "sn.pth"), device="cpu", backend="torch",
                       image_size=64)
    img = torch.randint(0, 256, (1, 64, 64, 3), dtype=torch.uint8)
    with torch.no_grad():
        assert torch.allclose(sn.logits(img), ref(_normalize(img)), atol=1e-2, rtol=1e-2)
