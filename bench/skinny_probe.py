"""Skinny-M GEMM timing (gemm_skinny.hip): per-call time of ops.linear at
M <= 64 inside a captured graph (200 back-to-back calls per replay), for the
serving shapes -- BERT's CLS-only last layer (o-proj, FFN up / down), pooler,
classifier, a CNN FC, the Llama-3 LM head on the last token of 8 prompts.
Set RDB_OPS_SO to time an A/B build of the kernels.

    python bench/skinny_probe.py [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(32, 768, 768), (32, 3072, 768), (32, 768, 3072), (32, 2, 768), (1, 1000, 2048), (32, 1000, 2048),
          (8, 128256, 4096), (64, 4096, 4096), (16, 14336, 4096)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    ap.add_argument("--calls", type=int, default=200)
    a = ap.parse_args()
    from ray_dynamic_batching_amd import ops

    rows = []
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * K ** -0.5
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
        ops.linear(x, w, b)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(a.calls):
                y = ops.linear(x, w, b, act="gelu")
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / a.calls)
        err = (y.float() - ops.linear_ref(x, w, b, act="gelu").float()).abs().max().item()
        gbs = (N * K * 2 + M * K * 2 + M * N * 2) / best / 1e3
        rows.append(dict(M=M, N=N, K=K, us=round(best, 2), weight_GBps=round(gbs, 1), max_err=round(err, 4)))
        print(json.dumps(rows[-1]), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"ops_so": os.environ.get("RDB_OPS_SO", "default"), "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
