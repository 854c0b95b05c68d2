"""One-hot probes of the ping-pong conv tap / channel mapping (debug)."""
import torch
from ray_dynamic_batching_amd import ops

H, C, K = 8, 64, 64
for (r, s, c) in [(0, 0, 0), (0, 1, 0), (1, 0, 0), (1, 1, 0), (2, 2, 0), (0, 0, 8), (0, 0, 63), (1, 2, 17)]:
    x = torch.zeros(1, H, H, C, device="cuda", dtype=torch.float16)
    x[0, 3, 3, c] = 1.0
    w = torch.zeros(K, 3, 3, C, device="cuda", dtype=torch.float16)
    w[5, r, s, c] = 1.0
    b = torch.zeros(K, device="cuda", dtype=torch.float16)
    out = []
    for cfg in (0, ops.CONV_PP | 0, ops.CONV_PP | 3):
        y = ops.conv2d_nhwc(x, w, b, stride=1, pad=1, act="none", tile_cfg=cfg).float()
        torch.cuda.synchronize()
        nz = (y != 0).nonzero().tolist()
        out.append(f"cfg{cfg & 0xff}{'pp' if cfg & ops.CONV_PP else ''}: {nz[:4]} sum {y.sum().item():.2f}")
    print(f"tap r{r} s{s} c{c} ->", " | ".join(out), flush=True)
# all-ones image, one tap: every interior output = 1
x = torch.ones(1, H, H, C, device="cuda", dtype=torch.float16)
for (r, s) in [(0, 0), (1, 1), (2, 2)]:
    w = torch.zeros(K, 3, 3, C, device="cuda", dtype=torch.float16)
    w[0, r, s, 0] = 1.0
    b = torch.zeros(K, device="cuda", dtype=torch.float16)
    y = ops.conv2d_nhwc(x, w, b, stride=1, pad=1, act="none", tile_cfg=ops.CONV_PP | 0).float()
    y0 = ops.conv2d_nhwc(x, w, b, stride=1, pad=1, act="none", tile_cfg=0).float()
    print(f"ones r{r} s{s}: pp ch0 map\n{y[0, :, :, 0].int().tolist()}\n ref\n{y0[0, :, :, 0].int().tolist()}", flush=True)
