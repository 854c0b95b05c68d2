"""Shared pieces of the image-classification servables (ResNet / ShuffleNet /
EfficientNet / ViT): the serving contract (uint8 HWC image in, top-k
(probability, class id) out), BN folding and channel padding helpers."""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .. import ops

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def round8(c: int) -> int:
    return (c + 7) // 8 * 8


class BNFolder:
    """Random-init conv + BatchNorm(running stats) folded into (W, b), kept in
    both the logical layout (torch reference) and the channel-padded NHWC layout
    the HIP kernels use (padding is zero weights / zero bias)."""

    def __init__(self, seed: int, device, dtype):
        self.g = torch.Generator(device="cpu").manual_seed(seed)
        self.device = device
        self.dtype = dtype

    def conv(self, cin: int, cout: int, k: int, gamma: float = 1.0, depthwise: bool = False, bn: bool = True):
        fan_in = k * k * (1 if depthwise else cin)
        shape = (cout, k, k) if depthwise else (cout, k, k, cin)
        w = torch.randn(*shape, generator=self.g) * math.sqrt(2.0 / fan_in)
        if bn:
            mean = torch.randn(cout, generator=self.g) * 0.01
            var = 1.0 + torch.rand(cout, generator=self.g) * 0.1
            beta = torch.randn(cout, generator=self.g) * 0.01
            scale = gamma / torch.sqrt(var + 1e-5)
            w = w * scale.view(-1, *([1] * (w.dim() - 1)))
            b = beta - mean * scale
        else:
            b = torch.randn(cout, generator=self.g) * 0.01
        return w, b

    def linear(self, cin: int, cout: int, std: Optional[float] = None):
        w = torch.randn(cout, cin, generator=self.g) * (std if std is not None else math.sqrt(1.0 / cin))
        b = torch.randn(cout, generator=self.g) * 0.01
        return w, b

    def dev(self, t: torch.Tensor, dtype=None) -> torch.Tensor:
        return t.to(self.device, dtype or self.dtype).contiguous()

    def pad_conv(self, w: torch.Tensor, b: torch.Tensor, kp: int, cp: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """[K, R, S, C] -> [kp, R, S, cp] zero-padded (physical NHWC layout)."""
        K, R, S, C = w.shape
        wp = torch.zeros(kp, R, S, cp)
        wp[:K, :, :, :C] = w
        bp = torch.zeros(kp)
        bp[:K] = b
        return self.dev(wp), self.dev(bp)

    def pad_dw(self, w: torch.Tensor, b: torch.Tensor, cp: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """depthwise [C, R, R] -> [R, R, cp] (channel-contiguous kernel layout)."""
        C, R, _ = w.shape
        wp = torch.zeros(R, R, cp)
        wp[:, :, :C] = w.permute(1, 2, 0)
        bp = torch.zeros(cp)
        bp[:C] = b
        return self.dev(wp), self.dev(bp)


class CheckpointFolder(BNFolder):
    """``BNFolder`` whose convs / linears come from a checkpoint (torchvision
    key names) instead of random init: each ``conv`` call takes the next
    (conv key, BatchNorm key) pair of ``conv_names`` -- the model constructor's
    call order -- folds the BatchNorm's eval statistics into (W, b) and lays W
    out like ``BNFolder`` ([Cout, k, k, Cin], depthwise [C, k, k]); each
    ``linear`` takes the next key of ``linear_names``.  Shapes are checked
    against what the constructor asks for; ``finish()`` rejects unused keys."""

    def __init__(self, sd, conv_names, linear_names, device, dtype, eps: float = 1e-5):
        super().__init__(0, device, dtype)
        self.sd, self.eps = sd, eps
        self.conv_names, self.linear_names = list(conv_names), list(linear_names)
        self.used = set()

    def _t(self, name):
        if name not in self.sd:
            raise KeyError(f"checkpoint has no {name!r}")
        self.used.add(name)
        return self.sd[name].float()

    def conv(self, cin: int, cout: int, k: int, gamma: float = 1.0, depthwise: bool = False, bn: bool = True):
        if not self.conv_names:
            raise ValueError("checkpoint folder: more convs requested than names given")
        cname, bname = self.conv_names.pop(0)
        w = self._t(cname + ".weight")
        want = (cout, 1 if depthwise else cin, k, k)
        if tuple(w.shape) != want:
            raise ValueError(f"{cname}: checkpoint shape {tuple(w.shape)} != model shape {want}")
        w = w[:, 0] if depthwise else w.permute(0, 2, 3, 1)
        if bname:
            scale = self._t(bname + ".weight") / torch.sqrt(self._t(bname + ".running_var") + self.eps)
            b = self._t(bname + ".bias") - self._t(bname + ".running_mean") * scale
            self.used.add(bname + ".num_batches_tracked")
            w = w * scale.view(-1, *([1] * (w.dim() - 1)))
        else:
            b = self._t(cname + ".bias") if cname + ".bias" in self.sd else torch.zeros(cout)
        return w.contiguous(), b

    def linear(self, cin: int, cout: int, std: Optional[float] = None):
        name = self.linear_names.pop(0)
        w, b = self._t(name + ".weight"), self._t(name + ".bias")
        if w.dim() == 4 and w.shape[2:] == (1, 1):          # 1x1 conv used as FC (SE blocks)
            w = w[:, :, 0, 0]
        if tuple(w.shape) != (cout, cin):
            raise ValueError(f"{name}: checkpoint shape {tuple(w.shape)} != model shape {(cout, cin)}")
        return w, b

    def finish(self, strict: bool = True) -> None:
        left = sorted(k for k in self.sd if k not in self.used)
        if strict and (left or self.conv_names or self.linear_names):
            raise ValueError(f"checkpoint / model mismatch: unused keys {left[:8]}, "
                             f"unconsumed names {(self.conv_names + self.linear_names)[:4]}")


class ImageClassifier:
    """Serving contract shared by the CNN / ViT servables."""

    image_size = 224
    topk = 5
    input_dtype = torch.uint8
    output_dtype = torch.float32

    @property
    def input_shape(self):
        return (self.image_size, self.image_size, 3)

    @property
    def output_shape(self):
        return (2 * self.topk,)

    def __call__(self, x):
        return self.forward(x)

    @torch.no_grad()
    def forward(self, img: torch.Tensor) -> torch.Tensor:
        """img uint8 [B, H, W, 3] -> [B, 2k] f32 = (top-k probs, top-k class ids)."""
        logits = self.logits(img)
        if self.backend == "hip":
            return ops.softmax_topk_packed(logits, self.topk)
        p, i = ops.softmax_topk_ref(logits, self.topk)
        return torch.cat([p, i.float()], dim=1).contiguous()

    def logits(self, img: torch.Tensor) -> torch.Tensor:
        return self._logits_hip(img) if self.backend == "hip" else self._logits_torch(img)

    def example_input(self, batch: int, seed: int = 0, device=None) -> torch.Tensor:
        g = torch.Generator(device="cpu").manual_seed(seed)
        return torch.randint(0, 256, (batch,) + self.input_shape, generator=g, dtype=torch.uint8).to(
            device or self.device)

    def _normalize_torch(self, img: torch.Tensor, dt) -> torch.Tensor:
        mean = torch.tensor(IMAGENET_MEAN, device=img.device)
        std = torch.tensor(IMAGENET_STD, device=img.device)
        return ((img.float() / 255.0 - mean) / std).permute(0, 3, 1, 2).to(dt)

    def _torch_dtype(self):
        return self.dtype if self.device.type == "cuda" else torch.float32


def conv_t(x, w, b, stride=1, pad=0, groups=1, dt=None):
    """torch reference conv from [K, R, S, C] (or depthwise [C, R, R]) weights."""
    if w.dim() == 3:   # depthwise
        wt = w.unsqueeze(1)
        groups = w.shape[0]
    else:
        wt = w.permute(0, 3, 1, 2)
    return F.conv2d(x, wt.to(dt or x.dtype), b.to(dt or x.dtype), stride=stride, padding=pad, groups=groups)
