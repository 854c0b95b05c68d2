"""Vision Transformer (ViT-B/16 by default, random init) on the gfx950 kernels.

The fork's registry serves torchvision vit_b_16 (scheduler.py:41); its profile
was measured on ViT-G/16 (1.85B params) -- both shapes are available here
(``ViTConfig.b16()`` / ``ViTConfig.g14_like()``).

Pre-LN encoder, f16: patch embedding = 16x16/16 conv on the implicit-GEMM conv
kernel (no im2col copy), CLS + position embedding, 12 x [LN -> QKV GEMM ->
fused attention (S = 197, masked tail) -> out GEMM (+bias +residual) -> LN ->
FC1 (+GELU) -> FC2 (+residual)] -> LN -> head GEMM -> softmax_topk.
Input: uint8 RGB [224, 224, 3]; output: top-5 (prob, class) as 10 f32.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from .. import ops


@dataclass
class ViTConfig:
    image: int = 224
    patch: int = 16
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    mlp: int = 3072
    classes: int = 1000
    eps: float = 1e-6

    @staticmethod
    def b16(**kw):
        return ViTConfig(**kw)

    @staticmethod
    def g14_like(**kw):  # ViT-G/14-class width (head dim 128 on our attention kernel)
        d = dict(patch=14, hidden=1664, layers=48, heads=13, mlp=8192)
        d.update(kw)
        return ViTConfig(**d)

    @staticmethod
    def g16(**kw):  # the fork's profiled "vit_g16" class (~1.85B params, vit_g16_*_report.txt:289-291)
        d = dict(patch=16, hidden=1664, layers=48, heads=13, mlp=8192)
        d.update(kw)
        return ViTConfig(**d)

    @staticmethod
    def tiny(**kw):
        d = dict(image=64, patch=16, hidden=256, layers=2, heads=4, mlp=512, classes=100)
        d.update(kw)
        return ViTConfig(**d)


class ViT:
    def __init__(self, cfg: ViTConfig = None, device="cuda", dtype=torch.float16, backend: str = "hip", seed: int = 0,
                 topk: int = 5):
        self.cfg = c = cfg or ViTConfig()
        if c.hidden % c.heads or (c.hidden // c.heads) not in (64, 128):
            raise ValueError("head dim must be 64 or 128")
        self.device, self.dtype, self.backend, self.topk = torch.device(device), dtype, backend, topk
        g = torch.Generator(device="cpu").manual_seed(seed)
        D = c.hidden

        def w(*s, std=0.02):
            return (torch.randn(*s, generator=g) * std).to(self.device, dtype).contiguous()

        pw = torch.zeros(D, c.patch, c.patch, 8)
        pw[..., :3] = torch.randn(D, c.patch, c.patch, 3, generator=g) * (1.0 / math.sqrt(3 * c.patch * c.patch))
        self.patch_w = pw.to(self.device, dtype).contiguous()
        self.patch_b = w(D)
        self.cls = w(1, 1, D)
        self.npatch = (c.image // c.patch) ** 2
        self.pos = w(1, self.npatch + 1, D)
        one = lambda: torch.ones(D, device=self.device, dtype=dtype)
        zero = lambda: torch.zeros(D, device=self.device, dtype=dtype)
        self.layers = [dict(ln1_g=one(), ln1_b=zero(), w_qkv=w(3 * D, D), b_qkv=w(3 * D), w_o=w(D, D), b_o=w(D),
                            ln2_g=one(), ln2_b=zero(), w1=w(c.mlp, D), b1=w(c.mlp), w2=w(D, c.mlp), b2=w(D))
                       for _ in range(c.layers)]
        self.ln_g, self.ln_b = one(), zero()
        self.head_w, self.head_b = w(c.classes, D), w(c.classes)

    @property
    def input_shape(self):
        return (self.cfg.image, self.cfg.image, 3)

    input_dtype = torch.uint8

    @property
    def output_shape(self):
        return (2 * self.topk,)

    output_dtype = torch.float32

    def __call__(self, x):
        return self.forward(x)

    @torch.no_grad()
    def forward(self, img):
        logits = self._logits_hip(img) if self.backend == "hip" else self._logits_torch(img)
        if self.backend == "hip":
            return ops.softmax_topk_packed(logits, self.topk)
        p, i = ops.softmax_topk_ref(logits, self.topk)
        return torch.cat([p, i.float()], dim=1).contiguous()

    def logits(self, img):
        return self._logits_hip(img) if self.backend == "hip" else self._logits_torch(img)

    def _tokens(self, patches):  # patches [B, n, D]
        B = patches.shape[0]
        return (torch.cat([self.cls.expand(B, 1, -1), patches], dim=1) + self.pos).contiguous()

    def _logits_hip(self, img):
        c = self.cfg
        B = img.shape[0]
        D, H = c.hidden, c.heads
        x = ops.image_to_nhwc(img, 8)
        pe = ops.conv2d_nhwc(x, self.patch_w, self.patch_b, stride=c.patch, pad=0)   # [B, h, w, D]
        x = self._tokens(pe.view(B, self.npatch, D)).view(-1, D)
        S = self.npatch + 1
        for L in self.layers:
            h = ops.layer_norm(x, L["ln1_g"], L["ln1_b"], c.eps)
            qkv = ops.linear(h, L["w_qkv"], L["b_qkv"])
            a = ops.attention(qkv, B, S, H, H, D // H)
            x = ops.linear(a, L["w_o"], L["b_o"], residual=x)
            h = ops.layer_norm(x, L["ln2_g"], L["ln2_b"], c.eps)
            m = ops.linear(h, L["w1"], L["b1"], act="gelu")
            x = ops.linear(m, L["w2"], L["b2"], residual=x)
        cls = x.view(B, S, D)[:, 0, :].contiguous()
        cls = ops.layer_norm(cls, self.ln_g, self.ln_b, c.eps)
        return ops.linear(cls, self.head_w, self.head_b, out_dtype=torch.float32)

    def _logits_torch(self, img):
        c = self.cfg
        dt = self.dtype if self.device.type == "cuda" else torch.float32
        B = img.shape[0]
        D, H = c.hidden, c.heads
        mean = torch.tensor([0.485, 0.456, 0.406], device=img.device)
        std = torch.tensor([0.229, 0.224, 0.225], device=img.device)
        x = ((img.float() / 255.0 - mean) / std).permute(0, 3, 1, 2).to(dt)
        pe = F.conv2d(x, self.patch_w[..., :3].permute(0, 3, 1, 2).to(dt), self.patch_b.to(dt), stride=c.patch)
        pe = pe.flatten(2).transpose(1, 2)
        x = (torch.cat([self.cls.to(dt).expand(B, 1, -1), pe], 1) + self.pos.to(dt))
        S = x.shape[1]
        P = lambda t: t.to(dt)
        for L in self.layers:
            h = F.layer_norm(x, (D,), P(L["ln1_g"]), P(L["ln1_b"]), c.eps)
            q, k, v = F.linear(h, P(L["w_qkv"]), P(L["b_qkv"])).view(B, S, 3, H, D // H).permute(2, 0, 3, 1, 4)
            a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, S, D)
            x = x + F.linear(a, P(L["w_o"]), P(L["b_o"]))
            h = F.layer_norm(x, (D,), P(L["ln2_g"]), P(L["ln2_b"]), c.eps)
            x = x + F.linear(F.gelu(F.linear(h, P(L["w1"]), P(L["b1"]))), P(L["w2"]), P(L["b2"]))
        cls = F.layer_norm(x[:, 0], (D,), P(self.ln_g), P(self.ln_b), c.eps)
        return F.linear(cls, P(self.head_w), P(self.head_b)).float()

    def example_input(self, batch: int, seed: int = 0, device=None):
        g = torch.Generator(device="cpu").manual_seed(seed)
        return torch.randint(0, 256, (batch,) + self.input_shape, generator=g, dtype=torch.uint8).to(
            device or self.device)
