"""ResNet-50 (random init) on the NHWC f16 implicit-GEMM conv kernels.

The fork's main profiled model (scheduler.py:43; resnet50_* profile) and
BASELINE config 2 (ResNet-50 fp16, 1 replica, dyn-batch <= 32 / 5 ms).

Serving contract: one request = one uint8 RGB image [224, 224, 3] (what a
client actually sends; half the PCIe bytes of f16 NCHW); one response =
top-5 (probability, class id) as 10 float32 (softmax + top-k fused kernel --
the Serve ResNet workload's softmax + argmax).

Forward (all on gfx950 kernels, hipGraph-captured by the replica engine):
  image_to_s2d (normalise, 2x2 space-to-depth, C 12 -> 16) -> conv7x7/2 as a
  4x4/1 conv on that tensor (+BN folded +ReLU) ->
  maxpool3x3/2 -> 16 bottlenecks [conv1x1+ReLU, conv3x3(/s)+ReLU,
  conv1x1 + (downsample conv) residual + ReLU fused in the epilogue] ->
  global avgpool -> FC GEMM (f32 logits) -> softmax_topk(5)
BatchNorm is folded into (W, b) at load time.
"""
from __future__ import annotations

import math
import os
from typing import List

import torch
import torch.nn.functional as F

from .. import ops

STAGES = [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]   # (width, blocks, stride)


class ResNet50:
    def __init__(self, device="cuda", dtype=torch.float16, backend: str = "hip", num_classes: int = 1000, seed: int = 0,
                 image_size: int = 224, topk: int = 5):
        self.device = torch.device(device)
        self.dtype = dtype
        self.backend = backend
        # shipped MI355X tile table key (runtime.engine.shipped_tile_table): 224x224 fp16 only
        self.tile_signature = "resnet50" if backend == "hip" and image_size == 224 and dtype == torch.float16 else None
        self.num_classes = num_classes
        self.image_size = image_size
        self.topk = topk
        g = torch.Generator(device="cpu").manual_seed(seed)

        def conv(cin, cout, k, gamma=1.0):
            w = torch.randn(cout, k, k, cin, generator=g) * math.sqrt(2.0 / (k * k * cin))
            # folded BN: y = gamma * (conv - mean) / sqrt(var + eps) + beta, with
            # random running stats
            mean = torch.randn(cout, generator=g) * 0.01
            var = 1.0 + torch.rand(cout, generator=g) * 0.1
            beta = torch.randn(cout, generator=g) * 0.01
            scale = gamma / torch.sqrt(var + 1e-5)
            wf = w * scale[:, None, None, None]
            bf = beta - mean * scale
            return wf.to(self.device, dtype).contiguous(), bf.to(self.device, dtype).contiguous()

        w, b = conv(3, 64, 7)
        self.stem_w = torch.zeros(64, 7, 7, 8, device=self.device, dtype=dtype)   # C padded 3 -> 8
        self.stem_w[..., :3] = w
        self.stem_b = b
        # the stem on the space-to-depth image: 4x4 / stride-1 conv, 256 reduction
        # elements per output instead of 392 (RDB_RESNET_S2D=0: the 7x7 conv)
        self.stem_s2d = os.environ.get("RDB_RESNET_S2D", "1") != "0"
        # ... and fused with the max-pool and the image conversion: +6.3 % img/s in a same-box serving A/B
        # (profiles/resnet50_stem_fused_ab_r4.json); RDB_RESNET_STEM_FUSED=0: the three-kernel stem
        self.stem_fused = os.environ.get("RDB_RESNET_STEM_FUSED", "1") != "0"
        self.stem_w_s2d = ops.stem_weight_s2d(self.stem_w)
        self.blocks: List[dict] = []
        cin = 64
        for width, n, stride in STAGES:
            for i in range(n):
                s = stride if i == 0 else 1
                blk = dict(stride=s)
                blk["w1"], blk["b1"] = conv(cin, width, 1)
                blk["w2"], blk["b2"] = conv(width, width, 3)
                blk["w3"], blk["b3"] = conv(width, width * 4, 1, gamma=0.2)   # small last-BN gamma keeps f16 stable
                if s != 1 or cin != width * 4:
                    blk["wd"], blk["bd"] = conv(cin, width * 4, 1)
                self.blocks.append(blk)
                cin = width * 4
        self.fc_w = (torch.randn(num_classes, 2048, generator=g) * 0.01).to(self.device, dtype).contiguous()
        self.fc_b = torch.zeros(num_classes, device=self.device, dtype=dtype)

    @torch.no_grad()
    def load_torchvision_state_dict(self, sd, strict: bool = True, eps: float = 1e-5) -> "ResNet50":
        """Load torchvision ``resnet50`` weights (the reference's registry model,
        ``scheduler.py:43``): BatchNorm eval statistics are folded into each
        conv -- W' = W * g / sqrt(var + eps), b' = beta - mean * g / sqrt(var + eps)
        -- and the weights are laid out NHWC ([Cout, kh, kw, Cin]) for the
        implicit-GEMM kernels (stem Cin padded 3 -> 8)."""
        used = set()

        def t(name):
            used.add(name)
            return sd[name].float()

        def fold(conv, bn):
            w = t(conv + ".weight")
            scale = t(bn + ".weight") / torch.sqrt(t(bn + ".running_var") + eps)
            b = t(bn + ".bias") - t(bn + ".running_mean") * scale
            used.add(bn + ".num_batches_tracked")
            return (w * scale[:, None, None, None]).permute(0, 2, 3, 1), b

        def put(dst, src):
            if tuple(dst.shape) != tuple(src.shape):
                raise ValueError(f"shape {tuple(src.shape)} does not fit {tuple(dst.shape)}")
            dst.copy_(src.to(dst.device, dst.dtype))

        w, b = fold("conv1", "bn1")
        self.stem_w.zero_()
        put(self.stem_w[..., :3], w)
        put(self.stem_b, b)
        self.stem_w_s2d = ops.stem_weight_s2d(self.stem_w)
        bi = 0
        for si, (_, n, _) in enumerate(STAGES):
            for i in range(n):
                blk, p = self.blocks[bi], f"layer{si + 1}.{i}."
                for j in (1, 2, 3):
                    w, b = fold(p + f"conv{j}", p + f"bn{j}")
                    put(blk[f"w{j}"], w)
                    put(blk[f"b{j}"], b)
                if "wd" in blk:
                    w, b = fold(p + "downsample.0", p + "downsample.1")
                    put(blk["wd"], w)
                    put(blk["bd"], b)
                bi += 1
        put(self.fc_w, t("fc.weight"))
        put(self.fc_b, t("fc.bias"))
        left = sorted(k for k in sd if k not in used)
        if strict and left:
            raise ValueError(f"unused checkpoint keys: {left[:8]}")
        return self

    # -- serving contract
    @property
    def input_shape(self):
        return (self.image_size, self.image_size, 3)

    input_dtype = torch.uint8

    @property
    def output_shape(self):
        return (2 * self.topk,)

    output_dtype = torch.float32

    def __call__(self, x):
        return self.forward(x)

    @torch.no_grad()
    def forward(self, img: torch.Tensor) -> torch.Tensor:
        """img uint8 [B, H, W, 3] -> [B, 2k] f32 = (top-k probs, top-k class ids)."""
        logits = self.logits(img)
        if self.backend == "hip":
            return ops.softmax_topk_packed(logits, self.topk)   # [k probs | k ids] written by the kernel
        p, i = ops.softmax_topk_ref(logits, self.topk)
        return torch.cat([p, i.float()], dim=1).contiguous()

    def logits(self, img: torch.Tensor) -> torch.Tensor:
        if self.backend == "hip":
            return self._logits_hip(img)
        return self._logits_torch(img)

    def _logits_hip(self, img):
        # one split-K workspace per forward (its tile counters zeroed once, by the
        # first kernel; the convolutions of the forward run one after another on its stream)
        s2d = self.stem_s2d and img.shape[1] % 2 == 0 and img.shape[2] % 4 == 0
        fused = s2d and self.stem_fused and img.shape[1] % 32 == 0 and img.shape[2] % 32 == 0
        ws = ops.splitk_workspace(img.device, zeroed=not s2d)
        if fused:
            # image -> space-to-depth -> stem conv -> ReLU -> max-pool in one kernel
            # (the 112x112x64 stem activation never reaches HBM); also zeroes ws
            x = ops.stem_s2d_pool(img, self.stem_w_s2d, self.stem_b, zero=ws)
        else:
            if s2d:
                x = ops.image_to_s2d(img, zero=ws)          # also zeroes the workspace's counters
                x = ops.conv2d_nhwc(x, self.stem_w_s2d, self.stem_b, stride=1, pad=2, act="relu",
                                    out_hw=(img.shape[1] // 2, img.shape[2] // 2), workspace=ws)
            else:
                x = ops.image_to_nhwc(img, 8)
                x = ops.conv2d_nhwc(x, self.stem_w, self.stem_b, stride=2, pad=3, act="relu", workspace=ws)
            x = ops.maxpool_nhwc(x, 3, 2, 1)
        for blk in self.blocks:
            s = blk["stride"]
            h = ops.conv2d_nhwc(x, blk["w1"], blk["b1"], act="relu", workspace=ws)
            h = ops.conv2d_nhwc(h, blk["w2"], blk["b2"], stride=s, pad=1, act="relu", workspace=ws)
            sc = ops.conv2d_nhwc(x, blk["wd"], blk["bd"], stride=s, workspace=ws) if "wd" in blk else x
            x = ops.conv2d_nhwc(h, blk["w3"], blk["b3"], act="relu", residual=sc, workspace=ws)
        pooled = ops.avgpool_nhwc(x)
        return ops.linear(pooled, self.fc_w, self.fc_b, out_dtype=torch.float32)

    def _torch_params(self):
        """The torch arm's weights, converted ONCE (NCHW tensors in channels_last
        memory, i.e. the NHWC layout MIOpen's fp16 convolutions run on) -- never
        inside a forward, so a captured graph holds only the convolutions."""
        tp = getattr(self, "_tp", None)
        if tp is None:
            dt = self.dtype if self.device.type == "cuda" else torch.float32
            cl = torch.channels_last

            def w(x):
                return x.permute(0, 3, 1, 2).to(dt).contiguous(memory_format=cl)
            tp = dict(dt=dt, mean=torch.tensor([0.485, 0.456, 0.406], device=self.device).view(1, 1, 1, 3),
                      std=torch.tensor([0.229, 0.224, 0.225], device=self.device).view(1, 1, 1, 3),
                      stem=(w(self.stem_w[..., :3]), self.stem_b.to(dt)),
                      blocks=[{k: (w(blk[k]), blk["b" + k[1:]].to(dt)) for k in ("w1", "w2", "w3", "wd") if k in blk}
                              for blk in self.blocks])
            self._tp = tp
        return tp

    def _logits_torch(self, img):
        """Eager PyTorch baseline (NCHW tensors in channels_last memory = MIOpen's
        NHWC fp16 convolutions, same folded weights)."""
        tp = self._torch_params()
        dt = tp["dt"]
        x = ((img.float() / 255.0 - tp["mean"]) / tp["std"]).to(dt).permute(0, 3, 1, 2)

        def cv(x, wb, s=1, p=0):
            return F.conv2d(x, wb[0], wb[1], stride=s, padding=p)

        x = F.relu(cv(x, tp["stem"], 2, 3))
        x = F.max_pool2d(x, 3, 2, 1)
        for blk, tb in zip(self.blocks, tp["blocks"]):
            s = blk["stride"]
            h = F.relu(cv(x, tb["w1"]))
            h = F.relu(cv(h, tb["w2"], s, 1))
            sc = cv(x, tb["wd"], s) if "wd" in tb else x
            x = F.relu(cv(h, tb["w3"]) + sc)
        pooled = x.float().mean(dim=(2, 3))
        return (pooled @ self.fc_w.float().t() + self.fc_b.float()).float()

    def example_input(self, batch: int, seed: int = 0, device=None) -> torch.Tensor:
        g = torch.Generator(device="cpu").manual_seed(seed)
        return torch.randint(0, 256, (batch,) + self.input_shape, generator=g, dtype=torch.uint8).to(
            device or self.device)

    def flops_per_image(self) -> float:
        return 2 * 4.1e9  # ~4.1 GMACs at 224x224
