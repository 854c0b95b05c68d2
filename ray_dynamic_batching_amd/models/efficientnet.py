"""EfficientNetV2-S (random init) on the NHWC f16 kernels -- the fork's
efficientnetv2_* profile (384x384 input).

Blocks (torchvision efficientnet_v2_s layout, BN folded, stochastic depth
off at inference):
  stem conv3x3/2 3->24 SiLU
  FusedMBConv(e1, 24->24) x2 | FusedMBConv(e4, s2, 24->48) x4 |
  FusedMBConv(e4, s2, 48->64) x4 | MBConv(e4, s2, 64->128, SE) x6 |
  MBConv(e6, 128->160, SE) x9 | MBConv(e6, s2, 160->256, SE) x15
  head conv1x1 256->1280 SiLU, avgpool, FC.
FusedMBConv = conv3x3(/s) expand + SiLU -> conv1x1 project (+ residual fused
into the project GEMM epilogue).  MBConv = conv1x1 expand + SiLU -> dw3x3(/s)
+ SiLU -> SE [avgpool -> FC+SiLU -> FC+sigmoid -> se_scale] -> conv1x1
project (+ residual).  Every conv is the implicit-GEMM MFMA kernel with the
bias / activation / residual epilogue; SE FCs are the GEMM kernel.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import ops
from .cnn_common import BNFolder, CheckpointFolder, ImageClassifier, conv_t

# (block, expand, stride, cin, cout, layers)
CONFIG = [("fused", 1, 1, 24, 24, 2), ("fused", 4, 2, 24, 48, 4), ("fused", 4, 2, 48, 64, 4),
          ("mb", 4, 2, 64, 128, 6), ("mb", 6, 1, 128, 160, 9), ("mb", 6, 2, 160, 256, 15)]


class EfficientNetV2S(ImageClassifier):
    def __init__(self, device="cuda", dtype=torch.float16, backend: str = "hip", num_classes: int = 1000,
                 seed: int = 0, image_size: int = 384, topk: int = 5, config=None, state_dict=None,
                 strict: bool = True):
        """``state_dict``: torchvision ``efficientnet_v2_s`` weights (BN eps 1e-3 folded)."""
        self.device = torch.device(device)
        self.dtype = dtype
        self.backend = backend
        self.image_size = image_size
        self.topk = topk
        if state_dict is not None:
            bf = CheckpointFolder(state_dict, *self.torchvision_names(config or CONFIG), self.device, dtype, eps=1e-3)
        else:
            bf = BNFolder(seed, self.device, dtype)
        w, b = bf.conv(3, 24, 3)
        self.stem = (bf.dev(w), bf.dev(b))
        self.stem_p = bf.pad_conv(w, b, 24, 8)
        self.blocks = []
        for kind, e, s, cin, cout, n in (config or CONFIG):
            for i in range(n):
                ci = cin if i == 0 else cout
                st = s if i == 0 else 1
                blk = dict(kind=kind, stride=st, res=(st == 1 and ci == cout))
                hid = ci * e
                if kind == "fused":
                    if e == 1:
                        blk["conv"] = tuple(map(bf.dev, bf.conv(ci, cout, 3)))
                    else:
                        blk["expand"] = tuple(map(bf.dev, bf.conv(ci, hid, 3)))
                        blk["project"] = tuple(map(bf.dev, bf.conv(hid, cout, 1, gamma=0.2)))
                else:
                    sq = max(1, ci // 4)
                    blk["expand"] = tuple(map(bf.dev, bf.conv(ci, hid, 1)))
                    dw, dwb = bf.conv(hid, hid, 3, depthwise=True)
                    blk["dw"] = (bf.dev(dw), bf.dev(dwb))
                    blk["dw_p"] = bf.pad_dw(dw, dwb, hid)
                    blk["se1"] = tuple(map(bf.dev, bf.linear(hid, sq)))
                    blk["se2"] = tuple(map(bf.dev, bf.linear(sq, hid)))
                    blk["project"] = tuple(map(bf.dev, bf.conv(hid, cout, 1, gamma=0.2)))
                self.blocks.append(blk)
        self.head = tuple(map(bf.dev, bf.conv(256, 1280, 1)))
        fw, fb = bf.linear(1280, num_classes, std=0.01)
        self.fc_w, self.fc_b = bf.dev(fw), bf.dev(fb)
        if state_dict is not None:
            bf.finish(strict)

    @staticmethod
    def torchvision_names(config):
        """(conv, BN) key pairs and linear keys in constructor call order."""
        convs, lins = [("features.0.0", "features.0.1")], []
        for si, (kind, e, _s, _ci, _co, n) in enumerate(config):
            for i in range(n):
                p = f"features.{si + 1}.{i}.block."
                if kind == "fused":
                    convs.append((p + "0.0", p + "0.1"))
                    if e != 1:
                        convs.append((p + "1.0", p + "1.1"))
                else:
                    convs += [(p + "0.0", p + "0.1"), (p + "1.0", p + "1.1"), (p + "3.0", p + "3.1")]
                    lins += [p + "2.fc1", p + "2.fc2"]
        convs.append((f"features.{len(config) + 1}.0", f"features.{len(config) + 1}.1"))
        return convs, lins + ["classifier.1"]

    def _logits_hip(self, img):
        ws = ops.splitk_workspace(img.device)      # split-K convolutions of this forward
        x = ops.image_to_nhwc(img, 8)
        x = ops.conv2d_nhwc(x, *self.stem_p, stride=2, pad=1, act="silu", workspace=ws)
        for blk in self.blocks:
            res = x if blk["res"] else None
            s = blk["stride"]
            if blk["kind"] == "fused":
                if "conv" in blk:   # expand 1: conv + SiLU, residual added AFTER the activation
                    y = ops.conv2d_nhwc(x, *blk["conv"], stride=s, pad=1, act="silu", workspace=ws)
                    x = y.add_(res) if res is not None else y
                else:
                    h = ops.conv2d_nhwc(x, *blk["expand"], stride=s, pad=1, act="silu", workspace=ws)
                    x = ops.conv2d_nhwc(h, *blk["project"], residual=res, workspace=ws)
            else:
                h = ops.conv2d_nhwc(x, *blk["expand"], act="silu", workspace=ws)
                h = ops.dwconv_nhwc(h, *blk["dw_p"], stride=s, pad=1, act="silu")
                z = ops.avgpool_nhwc(h)
                z = ops.linear(z, *blk["se1"], act="silu")
                z = ops.linear(z, *blk["se2"], act="sigmoid")
                h = ops.se_scale(h, z)
                x = ops.conv2d_nhwc(h, *blk["project"], residual=res, workspace=ws)
        x = ops.conv2d_nhwc(x, *self.head, act="silu", workspace=ws)
        pooled = ops.avgpool_nhwc(x)
        return ops.linear(pooled, self.fc_w, self.fc_b, out_dtype=torch.float32)

    def _logits_torch(self, img):
        dt = self._torch_dtype()
        x = self._normalize_torch(img, dt)
        x = F.silu(conv_t(x, *self.stem, stride=2, pad=1, dt=dt))
        for blk in self.blocks:
            res = x if blk["res"] else None
            s = blk["stride"]
            if blk["kind"] == "fused":
                if "conv" in blk:
                    y = F.silu(conv_t(x, *blk["conv"], stride=s, pad=1, dt=dt))
                    y = y + res if res is not None else y
                else:
                    h = F.silu(conv_t(x, *blk["expand"], stride=s, pad=1, dt=dt))
                    y = conv_t(h, *blk["project"], dt=dt)
                    y = y + res if res is not None else y
            else:
                h = F.silu(conv_t(x, *blk["expand"], dt=dt))
                h = F.silu(conv_t(h, *blk["dw"], stride=s, pad=1, dt=dt))
                z = h.float().mean(dim=(2, 3))
                z = F.silu(z @ blk["se1"][0].float().t() + blk["se1"][1].float())
                z = torch.sigmoid(z @ blk["se2"][0].float().t() + blk["se2"][1].float())
                h = (h.float() * z[:, :, None, None]).to(dt)
                y = conv_t(h, *blk["project"], dt=dt)
                y = y + res if res is not None else y
            x = y
        x = F.silu(conv_t(x, *self.head, dt=dt))
        pooled = x.float().mean(dim=(2, 3))
        return pooled @ self.fc_w.float().t() + self.fc_b.float()

    def flops_per_image(self) -> float:
        return 2 * 8.4e9 * (self.image_size / 384) ** 2
