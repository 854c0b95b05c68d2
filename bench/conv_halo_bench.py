"""ResNet-50 3x3 stride-1 convolutions at batch 32: the halo-tile kernel
(ops.CONV_HALO | v, conv_halo.hip) against the tile the shipped table picks
(im2col 4-wave / ping-pong conv tiles), launch by launch.

    python bench/conv_halo_bench.py [--table PATH] [--iters 50] [--json-out F]

Per shape and choice: mean us per launch alone on one stream ("alone"), and
per launch with 3 streams each running the same conv back to back ("x3":
what a replica with 3 batches in flight sees), the FLOP rate and the
fraction of the 2.5 PF dense f16 peak, and the max error vs the fp32
reference.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(32, 56, 64, 64), (32, 28, 128, 128), (32, 14, 256, 256), (32, 7, 512, 512)]
PEAK = 2.5e15


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--table", default="", help="tile table to read the current choice from (default: shipped "
                    "mi355x_resnet50_B32_cs3_d6.json)")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default="", help="comma-separated indices into SHAPES (default: all)")
    ap.add_argument("--choices", default="", help="comma-separated choice names to run (table, halo0, ...)")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)

    import torch

    from ray_dynamic_batching_amd import ops
    from ray_dynamic_batching_amd.runtime.engine import TUNED_DIR

    table = a.table or os.path.join(TUNED_DIR, "mi355x_resnet50_B32_cs3_d6.json")
    with open(table) as f:
        rows = json.load(f)
    current = {tuple(k[1:6]): c for k, c in rows if k[0] == "conv" and k[6] == 3 and k[8] == 1}
    torch.cuda.set_device(0)
    streams = [torch.cuda.Stream() for _ in range(3)]
    out = []
    shapes = [SHAPES[int(i)] for i in a.shapes.split(",")] if a.shapes else SHAPES
    for N, H, C, K in shapes:
        torch.manual_seed(H)
        x = torch.randn(N, H, H, C, device="cuda", dtype=torch.float16)
        w = torch.randn(K, 3, 3, C, device="cuda", dtype=torch.float16) * (9 * C) ** -0.5
        b = torch.randn(K, device="cuda", dtype=torch.float16) * 0.1
        ref = ops.conv2d_nhwc_ref(x, w, b, pad=1, act="relu").float()
        flop = 2.0 * N * H * H * K * 9 * C
        cur = current.get((N, H, H, C, K), -1)
        choices = [("table", cur)] + [(f"halo{c & 255}" + (f"s{ops.splits_of(c)}" if ops.splits_of(c) else ""), c)
                                      for c in ops.conv_halo_candidates(N, H, H, C, K, 3, 3, 1, 1, H, H, True)]
        if a.choices:
            choices = [ch for ch in choices if ch[0] in a.choices.split(",")]
        ws = [ops.splitk_workspace("cuda") for _ in streams]
        for name, c in choices:
            y = ops.conv2d_nhwc(x, w, b, pad=1, act="relu", tile_cfg=c, workspace=ws[0])
            err = float((y.float() - ref).abs().max())
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(5):
                ops.conv2d_nhwc(x, w, b, pad=1, act="relu", tile_cfg=c, workspace=ws[0])
            torch.cuda.synchronize()
            s0.record()
            for _ in range(a.iters):
                ops.conv2d_nhwc(x, w, b, pad=1, act="relu", tile_cfg=c, workspace=ws[0])
            s1.record()
            s1.synchronize()
            alone = s0.elapsed_time(s1) * 1e3 / a.iters
            ys = [torch.empty_like(y) for _ in streams]
            cur_s = torch.cuda.current_stream()
            for i, st in enumerate(streams):       # untimed pass: first use of the side streams / outputs
                st.wait_stream(cur_s)
                with torch.cuda.stream(st):
                    ops.conv2d_nhwc(x, w, b, pad=1, act="relu", tile_cfg=c, out=ys[i], workspace=ws[i])
            torch.cuda.synchronize()
            s0.record()
            for i, st in enumerate(streams):
                st.wait_stream(cur_s)
                with torch.cuda.stream(st):
                    for _ in range(a.iters):
                        ops.conv2d_nhwc(x, w, b, pad=1, act="relu", tile_cfg=c, out=ys[i], workspace=ws[i])
            for st in streams:
                cur_s.wait_stream(st)
            s1.record()
            s1.synchronize()
            x3 = s0.elapsed_time(s1) * 1e3 / (a.iters * len(streams))
            rec = {"shape": [N, H, H, C, K], "choice": name, "cfg": c, "alone_us": round(alone, 2),
                   "alone_pct_peak": round(100 * flop / (alone * 1e-6) / PEAK, 1), "x3_us": round(x3, 2),
                   "x3_pct_peak": round(100 * flop / (x3 * 1e-6) / PEAK, 1), "max_err": round(err, 4)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump({"table": os.path.basename(table), "iters": a.iters, "results": out}, f, indent=1)


if __name__ == "__main__":
    main()
