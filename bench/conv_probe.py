"""Standalone timing of every conv tile choice on the ResNet-50 bs32 3x3 layers
(and the strided 1x1 downsamples): one stream and two streams (the serving
engine's regime), median of 5 graph replays of 20 launches each.

    python bench/conv_probe.py [--batch 32] [--json-out F]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_dynamic_batching_amd import ops  # noqa: E402

SHAPES = [  # (H, C, K, R, stride, pad): input H = W
    (56, 64, 64, 3, 1, 1), (56, 128, 128, 3, 2, 1), (28, 128, 128, 3, 1, 1), (28, 256, 256, 3, 2, 1),
    (14, 256, 256, 3, 1, 1), (14, 512, 512, 3, 2, 1), (7, 512, 512, 3, 1, 1),
]


def name(c):
    if c & ops.CONV_PP:
        return f"pp{c & 255}x{ops.splits_of(c) or 1}"
    if c & ops.CONV_LINEAR:
        return f"lin{c & 255}"
    return f"t{c & 255}x{ops.splits_of(c) or 1}{'D' if c & ops.DEEP else ''}"


def time_cfg(fn, streams, reps=20, trials=5):
    cur = torch.cuda.current_stream()
    side = [torch.cuda.Stream() for _ in range(streams - 1)]
    for sd in side:
        sd.wait_stream(cur)
    g = torch.cuda.CUDAGraph()
    ws = [ops.splitk_workspace("cuda") for _ in range(streams)]
    fn(ws[0])
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(cur)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for sd in side:
                sd.wait_stream(s)
            for _ in range(reps):
                fn(ws[0])
                for i, sd in enumerate(side):
                    with torch.cuda.stream(sd):
                        fn(ws[i + 1])
            for sd in side:
                s.wait_stream(sd)
    torch.cuda.synchronize()
    ts = []
    for _ in range(trials):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / (reps * streams))
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--top", type=int, default=6)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    out = []
    for (H, C, K, R, st, pad) in SHAPES:
        N = a.batch
        x = torch.randn(N, H, H, C, device="cuda", dtype=torch.float16)
        w = torch.randn(K, R, R, C, device="cuda", dtype=torch.float16) * (R * R * C) ** -0.5
        b = torch.randn(K, device="cuda", dtype=torch.float16) * 0.1
        P = (H + 2 * pad - R) // st + 1
        M, Kg = N * P * P, R * R * C
        y = torch.empty(N, P, P, K, device="cuda", dtype=torch.float16)
        flop = 2.0 * M * K * Kg
        cands = ops._conv_candidates(M, K, Kg, False, C, True)
        res = []
        for c in cands:
            def fn(ws, c=c):
                ops.conv2d_nhwc(x, w, b, stride=st, pad=pad, act="relu", tile_cfg=c, out=y, workspace=ws)
            try:
                t1 = time_cfg(fn, 1)
                t2 = time_cfg(fn, 2)
            except Exception as e:  # noqa: BLE001
                print("skip", name(c), e, flush=True)
                continue
            res.append(dict(cfg=c, name=name(c), us_1s=round(t1, 2), us_2s=round(t2, 2),
                            tf_1s=round(flop / t1 / 1e6, 1), tf_2s=round(flop / t2 / 1e6, 1)))
        res.sort(key=lambda r: r["us_2s"])
        best1 = min(res, key=lambda r: r["us_1s"])
        line = dict(shape=dict(N=N, H=H, C=C, K=K, R=R, stride=st, pad=pad, M=M, gflop=round(flop / 1e9, 2)),
                    best_2stream=res[:a.top], best_1stream=best1,
                    best_pp_2stream=next((r for r in res if r["cfg"] & ops.CONV_PP), None))
        out.append(line)
        print(json.dumps(dict(shape=line["shape"], top2s=[(r["name"], r["us_2s"], r["us_1s"]) for r in res[:a.top]],
                              best1=(best1["name"], best1["us_1s"]),
                              pp=(line["best_pp_2stream"] or {}).get("name"),
                              pp_us=((line["best_pp_2stream"] or {}).get("us_2s"), (line["best_pp_2stream"] or {}).get("us_1s")))),
              flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
