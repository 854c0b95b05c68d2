"""ResNet-50 3x3 stride-1 convolutions at batch 32: the halo-tile kernel
(ops.CONV_HALO | v, conv_halo.hip) against the tile the shipped table picks
(im2col 4-wave / ping-pong conv tiles), launch by launch.

    python bench/conv_halo_bench.py [--table PATH] [--iters 50] [--json-out F]

Per shape and choice: mean us per launch alone on one stream ("alone"), and
per launch with 3 streams each running the same conv back to back ("x3":
what a replica with 3 batches in flight sees), both replayed from a captured
hipGraph (eager Python launches cost ~15 us each, as much as these kernels),
the FLOP rate and the fraction of the 2.5 PF dense f16 peak, and the max
error vs the fp32 reference.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(32, 56, 64, 64), (32, 28, 128, 128), (32, 14, 256, 256), (32, 7, 512, 512)]
# --stride 2: the first 3x3 of stages 2 / 3 / 4 (input H x H, output H/2 x H/2)
SHAPES_S2 = [(32, 56, 128, 128), (32, 28, 256, 256), (32, 14, 512, 512)]
PEAK = 2.5e15


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--table", default="", help="tile table to read the current choice from (default: shipped "
                    "mi355x_resnet50_B32_cs3_d6.json)")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default="", help="comma-separated indices into SHAPES (default: all)")
    ap.add_argument("--choices", default="", help="comma-separated choice names to run (table, halo0, ...)")
    ap.add_argument("--stride", type=int, default=1, choices=[1, 2])
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)

    import torch

    from ray_dynamic_batching_amd import ops
    from ray_dynamic_batching_amd.runtime.engine import TUNED_DIR

    table = a.table or os.path.join(TUNED_DIR, "mi355x_resnet50_B32_cs3_d6.json")
    with open(table) as f:
        rows = json.load(f)
    current = {tuple(k[1:6]): c for k, c in rows if k[0] == "conv" and k[6] == 3 and k[8] == a.stride}
    torch.cuda.set_device(0)
    streams = [torch.cuda.Stream() for _ in range(3)]
    out = []
    table_shapes = SHAPES if a.stride == 1 else SHAPES_S2
    shapes = [table_shapes[int(i)] for i in a.shapes.split(",")] if a.shapes else table_shapes
    st = a.stride
    for N, H, C, K in shapes:
        torch.manual_seed(H)
        x = torch.randn(N, H, H, C, device="cuda", dtype=torch.float16)
        w = torch.randn(K, 3, 3, C, device="cuda", dtype=torch.float16) * (9 * C) ** -0.5
        b = torch.randn(K, device="cuda", dtype=torch.float16) * 0.1
        ref = ops.conv2d_nhwc_ref(x, w, b, stride=st, pad=1, act="relu").float()
        P = (H - 1) // st + 1
        flop = 2.0 * N * P * P * K * 9 * C
        cur = current.get((N, H, H, C, K), -1)
        choices = [("table", cur)] + [(f"halo{c & 255}" + (f"s{ops.splits_of(c)}" if ops.splits_of(c) else ""), c)
                                      for c in ops.conv_halo_candidates(N, H, H, C, K, 3, 3, st, 1, P, P, True)]
        if a.choices:
            choices = [ch for ch in choices if ch[0] in a.choices.split(",")]
        ws = [ops.splitk_workspace("cuda") for _ in streams]
        for name, c in choices:
            y = ops.conv2d_nhwc(x, w, b, stride=st, pad=1, act="relu", tile_cfg=c, workspace=ws[0])
            err = float((y.float() - ref).abs().max())
            ys = [torch.empty_like(y) for _ in streams]
            for i, sd in enumerate(streams):       # eager first use of every stream / output / workspace
                with torch.cuda.stream(sd):
                    ops.conv2d_nhwc(x, w, b, stride=st, pad=1, act="relu", tile_cfg=c, out=ys[i], workspace=ws[i])
            torch.cuda.synchronize()

            def graph_of(nstreams):
                # the launches replayed from a hipGraph: no Python launch cost in the timed region
                cap = streams[0]
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=cap):
                    for i in range(1, nstreams):
                        streams[i].wait_stream(cap)
                    for i in range(nstreams):
                        with torch.cuda.stream(streams[i] if i else cap):
                            for _ in range(a.iters):
                                ops.conv2d_nhwc(x, w, b, stride=st, pad=1, act="relu", tile_cfg=c, out=ys[i],
                                                workspace=ws[i])
                    for i in range(1, nstreams):
                        cap.wait_stream(streams[i])
                return g

            def time_graph(g, n):
                g.replay()
                torch.cuda.synchronize()
                best = float("inf")
                for _ in range(3):
                    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s0.record()
                    g.replay()
                    s1.record()
                    s1.synchronize()
                    best = min(best, s0.elapsed_time(s1) * 1e3 / n)
                return best

            alone = time_graph(graph_of(1), a.iters)
            x3 = time_graph(graph_of(len(streams)), a.iters * len(streams))
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
