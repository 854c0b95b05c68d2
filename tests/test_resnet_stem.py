"""The ResNet-50 stem as a space-to-depth conv (models/resnet.py, ops.image_to_s2d
/ ops.stem_weight_s2d): a 7x7 stride-2 pad-3 conv on the image equals a 4x4
stride-1 conv (pad 2 top/left, 1 bottom/right) on the 2x2 space-to-depth image.
CPU, fp32 -- the identity the GPU stem relies on (torchvision conv1 semantics,
SURVEY §2.7 ResNet row)."""
import torch
import torch.nn.functional as F

from ray_dynamic_batching_amd import ops


def test_space_to_depth_stem_equals_7x7_stride2_conv():
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (2, 64, 48, 3), generator=g, dtype=torch.uint8)
    w = torch.randn(16, 7, 7, 3, generator=g)
    x = ops.image_to_nhwc_ref(img, 3).float()
    ref = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), stride=2, padding=3)
    xs = ops.image_to_s2d_ref(img).float()
    assert xs.shape == (2, 32, 24, 16) and xs[..., 12:].abs().max() == 0
    ws = ops.stem_weight_s2d(w)
    assert ws.shape == (16, 4, 4, 16)
    y = F.conv2d(xs.permute(0, 3, 1, 2), ws.permute(0, 3, 1, 2), stride=1, padding=2)[:, :, :32, :24]
    assert torch.allclose(y, ref, atol=1e-4, rtol=1e-4)


def test_space_to_depth_layout():
    img = torch.arange(2 * 4 * 4 * 3, dtype=torch.int64).remainder(256).to(torch.uint8).view(2, 4, 4, 3)
    xs = ops.image_to_s2d_ref(img)
    full = ops.image_to_nhwc_ref(img, 3)
    for dy in range(2):
        for dx in range(2):
            ch = (dy * 2 + dx) * 3
            assert torch.equal(xs[:, 1, 0, ch:ch + 3], full[:, 2 + dy, dx, :])
