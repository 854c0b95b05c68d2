"""Full-row GEMM + LayerNorm (ops.linear_rowln) vs the tiled GEMM + LayerNorm
kernel pair on BERT's o-proj / FFN-down shapes: solo latency and two-stream
throughput (the replica's regime), CUDA-event timed, tile table optional.

    python bench/rowln_probe.py [--tune-file ops/tuned/....json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune-file", default="")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import torch

    from ray_dynamic_batching_amd import ops

    if a.tune_file:
        ops.load_tuning(a.tune_file)
    torch.manual_seed(0)
    dev = "cuda"
    res = {}
    for name, M, K in (("o_proj", 4096, 768), ("ffn_down", 4096, 3072)):
        N = 768
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev).to(torch.bfloat16) * 0.1
        r = torch.randn(M, N, device=dev).to(torch.bfloat16)
        g = torch.ones(N, device=dev, dtype=torch.bfloat16)
        be = torch.zeros(N, device=dev, dtype=torch.bfloat16)

        wp = ops.pack_rowln_weight(w)

        def rowln(o):
            ops.linear_rowln(x, wp, b, r, g, be, 1e-12, out=o)

        def pair(o):
            t = ops.linear(x, w, b, residual=r)
            ops.layer_norm(t, g, be, 1e-12)

        outs = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        ref = ops.linear_residual_ln_ref(x, w, b, r, g, be)
        rowln(outs[0])
        err = ((outs[0].float() - ref.float()).abs().max()).item()
        for label, fn in (("rowln", rowln), ("gemm+ln", pair)):
            for _ in range(3):
                fn(outs[0])
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                fn(outs[0])
            e.record()
            torch.cuda.synchronize()
            solo = s.elapsed_time(e) * 1e3 / a.iters
            st = [torch.cuda.Stream() for _ in range(2)]
            cur = torch.cuda.current_stream()
            torch.cuda.synchronize()
            s.record()
            for sd in st:
                sd.wait_stream(cur)
            for _ in range(a.iters):
                for i, sd in enumerate(st):
                    with torch.cuda.stream(sd):
                        fn(outs[i])
            for sd in st:
                cur.wait_stream(sd)
            e.record()
            torch.cuda.synchronize()
            two = s.elapsed_time(e) * 1e3 / a.iters / 2
            res[f"{name}/{label}"] = {"solo_us": round(solo, 2), "two_stream_us_per_call": round(two, 2)}
        res[f"{name}/rowln_max_abs_err_vs_fp32"] = round(err, 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
