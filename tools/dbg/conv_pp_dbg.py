"""Per-variant error of the ping-pong conv tiles on small shapes (debug)."""
import torch
from ray_dynamic_batching_amd import ops

torch.manual_seed(0)
for (N, H, C, K, R, stride, pad) in [(1, 8, 64, 64, 1, 1, 0), (1, 8, 64, 64, 3, 1, 1), (2, 16, 64, 64, 3, 1, 1),
                                     (2, 56, 64, 64, 3, 1, 1), (1, 8, 128, 128, 3, 2, 1)]:
    x = torch.randn(N, H, H, C, device="cuda", dtype=torch.float16)
    w = torch.randn(K, R, R, C, device="cuda", dtype=torch.float16) * (R * R * C) ** -0.5
    b = torch.randn(K, device="cuda", dtype=torch.float16) * 0.1
    ref = ops.conv2d_nhwc_ref(x, w, b, stride=stride, pad=pad, act="none").float()
    line = [f"N{N} H{H} C{C} K{K} R{R} s{stride}"]
    y0 = ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="none", tile_cfg=0).float()
    line.append(f"t0 {(y0 - ref).abs().max().item():.3g}")
    for v in range(5):
        if C % ops._CONV_PP_BK[v]:
            continue
        y = ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="none", tile_cfg=ops.CONV_PP | v).float()
        torch.cuda.synchronize()
        e = (y - ref).abs()
        line.append(f"v{v} {e.max().item():.3g}")
        if v == 0 and e.max().item() > 0.1:
            bad = (e > 0.1).nonzero()
            print("  v0 first bad idx", bad[:6].tolist(), "y", y.flatten()[:8].tolist(), "ref", ref.flatten()[:8].tolist())
    print(" | ".join(line), flush=True)
