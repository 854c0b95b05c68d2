"""ShuffleNetV2 x1.0 (random init) on the NHWC f16 kernels -- the fork's
model registry entry (scheduler.py:42, shufflenet_* profile).

MI355X design: every tensor's channel dim is padded to a multiple of 8
(16-byte rows, MFMA-aligned GEMM K) with zero weights, and the unit boundary
``concat(x1, branch) -> channel_shuffle(2) -> split`` is ONE remap kernel
(ops.shuffle_remap) that writes the next unit's two halves directly, so no
torch.cat / view / transpose / chunk copies exist on the hot path.

Unit (stride 1):  x = (x1, x2);  b = relu(1x1(x2)) -> dw3x3 -> relu(1x1)
Unit (stride 2):  b1 = dw3x3/2(x) -> relu(1x1);  b2 = relu(1x1(x)) -> dw3x3/2 -> relu(1x1)
then shuffle_remap(x1|b1, b).  Stem conv3x3/2 + maxpool, conv5 1x1 -> 1024,
global avgpool, FC (f32 logits), softmax + top-k.
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn.functional as F

from .. import ops
from .cnn_common import BNFolder, CheckpointFolder, ImageClassifier, conv_t, round8

STAGE_OUT = [116, 232, 464]
STAGE_REPEATS = [4, 8, 4]


class ShuffleNetV2(ImageClassifier):
    def __init__(self, device="cuda", dtype=torch.float16, backend: str = "hip", num_classes: int = 1000,
                 seed: int = 0, image_size: int = 224, topk: int = 5, width: List[int] = None,
                 repeats: List[int] = None, state_dict=None, strict: bool = True):
        """``state_dict``: torchvision ``shufflenet_v2_x1_0`` weights (BN folded)."""
        self.device = torch.device(device)
        self.dtype = dtype
        self.backend = backend
        self.image_size = image_size
        self.topk = topk
        self.num_classes = num_classes
        self.stage_out = list(width or STAGE_OUT)
        self.repeats = list(repeats or STAGE_REPEATS)
        if state_dict is not None:
            bf = CheckpointFolder(state_dict, *self.torchvision_names(self.repeats), self.device, dtype)
        else:
            bf = BNFolder(seed, self.device, dtype)
        w, b = bf.conv(3, 24, 3)
        self.stem = (bf.dev(w), bf.dev(b))                      # logical
        self.stem_p = bf.pad_conv(w, b, 24, 8)                  # physical (C 3 -> 8)
        self.units = []
        cin = 24
        for cout, rep in zip(self.stage_out, self.repeats):
            half = cout // 2
            for i in range(rep):
                u = dict(stride=2 if i == 0 else 1, cin=cin, half=half)
                if i == 0:
                    u["dw1"] = bf.conv(cin, cin, 3, depthwise=True)
                    u["pw1"] = bf.conv(cin, half, 1)
                    u["pw2a"] = bf.conv(cin, half, 1)
                else:
                    u["pw2a"] = bf.conv(half, half, 1)
                u["dw2"] = bf.conv(half, half, 3, depthwise=True)
                u["pw2b"] = bf.conv(half, half, 1)
                u["last"] = i == rep - 1
                self.units.append(u)
                cin = cout
        self.conv5 = bf.conv(cin, 1024, 1)
        fw, fb = bf.linear(1024, num_classes, std=0.01)
        self.fc_w, self.fc_b = bf.dev(fw), bf.dev(fb)
        # physical (padded) copies for the HIP path
        for u in self.units:
            hp = round8(u["half"])
            cinp = round8(u["cin"])
            u["half_p"], u["cin_p"] = hp, cinp
            if u["stride"] == 2:
                u["dw1_p"] = bf.pad_dw(*u["dw1"], cinp)
                u["pw1_p"] = bf.pad_conv(*u["pw1"], hp, cinp)
                u["pw2a_p"] = bf.pad_conv(*u["pw2a"], hp, cinp)
            else:
                u["pw2a_p"] = bf.pad_conv(*u["pw2a"], hp, hp)
            u["dw2_p"] = bf.pad_dw(*u["dw2"], hp)
            u["pw2b_p"] = bf.pad_conv(*u["pw2b"], hp, hp)
            for k in ("dw1", "pw1", "pw2a", "dw2", "pw2b"):
                if k in u:
                    u[k] = (bf.dev(u[k][0]), bf.dev(u[k][1]))
        self.conv5_p = bf.pad_conv(*self.conv5, 1024, round8(cin))
        self.conv5 = (bf.dev(self.conv5[0]), bf.dev(self.conv5[1]))
        if state_dict is not None:
            bf.finish(strict)

    @staticmethod
    def torchvision_names(repeats):
        """(conv, BN) key pairs in constructor call order + linear keys."""
        convs = [("conv1.0", "conv1.1")]
        for s, rep in enumerate(repeats):
            for i in range(rep):
                p = f"stage{s + 2}.{i}."
                if i == 0:
                    convs += [(p + "branch1.0", p + "branch1.1"), (p + "branch1.2", p + "branch1.3"),
                              (p + "branch2.0", p + "branch2.1")]
                else:
                    convs.append((p + "branch2.0", p + "branch2.1"))
                convs += [(p + "branch2.3", p + "branch2.4"), (p + "branch2.5", p + "branch2.6")]
        convs.append(("conv5.0", "conv5.1"))
        return convs, ["fc"]

    # -- HIP path: padded NHWC f16 -----------------------------------------
    def _logits_hip(self, img):
        ws = ops.splitk_workspace(img.device)      # split-K convolutions of this forward
        x = ops.image_to_nhwc(img, 8)
        x = ops.conv2d_nhwc(x, *self.stem_p, stride=2, pad=1, act="relu", workspace=ws)
        x = ops.maxpool_nhwc(x, 3, 2, 1)
        x1 = x2 = None
        for u in self.units:
            hp = u["half_p"]
            if u["stride"] == 2:
                a = ops.dwconv_nhwc(x, *u["dw1_p"], stride=2, pad=1)
                a = ops.conv2d_nhwc(a, *u["pw1_p"], act="relu", workspace=ws)
                bsrc = x
            else:
                a, bsrc = x1, x2
            b = ops.conv2d_nhwc(bsrc, *u["pw2a_p"], act="relu", workspace=ws)
            b = ops.dwconv_nhwc(b, *u["dw2_p"], stride=u["stride"], pad=1)
            b = ops.conv2d_nhwc(b, *u["pw2b_p"], act="relu", workspace=ws)
            if u["last"]:
                x = ops.shuffle_remap(a, b, u["half"], False, round8(2 * u["half"]))
            else:
                x1, x2 = ops.shuffle_remap(a, b, u["half"], True, hp, hp)
        x = ops.conv2d_nhwc(x, *self.conv5_p, act="relu", workspace=ws)
        pooled = ops.avgpool_nhwc(x)
        return ops.linear(pooled, self.fc_w, self.fc_b, out_dtype=torch.float32)

    # -- eager PyTorch reference (NCHW, logical channels) --------------------
    def _logits_torch(self, img):
        dt = self._torch_dtype()
        x = self._normalize_torch(img, dt)
        x = F.relu(conv_t(x, *self.stem, stride=2, pad=1, dt=dt))
        x = F.max_pool2d(x, 3, 2, 1)
        for u in self.units:
            if u["stride"] == 2:
                a = conv_t(x, *u["dw1"], stride=2, pad=1, dt=dt)
                a = F.relu(conv_t(a, *u["pw1"], dt=dt))
                bsrc = x
            else:
                a, bsrc = x.chunk(2, dim=1)
            b = F.relu(conv_t(bsrc, *u["pw2a"], dt=dt))
            b = conv_t(b, *u["dw2"], stride=u["stride"], pad=1, dt=dt)
            b = F.relu(conv_t(b, *u["pw2b"], dt=dt))
            x = torch.cat([a, b], dim=1)
            n, c, h, w = x.shape
            x = x.view(n, 2, c // 2, h, w).transpose(1, 2).reshape(n, c, h, w)
        x = F.relu(conv_t(x, *self.conv5, dt=dt))
        pooled = x.float().mean(dim=(2, 3))
        return pooled @ self.fc_w.float().t() + self.fc_b.float()

    def flops_per_image(self) -> float:
        return 2 * 146e6
