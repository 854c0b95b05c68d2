"""Run one GEMM shape/tile many times (for rocprofv3 --pmc / --kernel-trace).

    python bench/gemm_probe.py --m 4096 --n 2304 --k 768 --cfg 0 --iters 200 [--act gelu] [--res]
Prints the per-call time from CUDA events for every tile config when --cfg -1.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--n", type=int, default=2304)
    ap.add_argument("--k", type=int, default=768)
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--act", default="none")
    ap.add_argument("--res", action="store_true")
    ap.add_argument("--bias", action="store_true")
    a = ap.parse_args(argv)
    import torch

    from ray_dynamic_batching_amd import ops

    torch.manual_seed(0)
    x = torch.randn(a.m, a.k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(a.n, a.k, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(a.n, device="cuda", dtype=torch.bfloat16) if a.bias else None
    r = torch.randn(a.m, a.n, device="cuda", dtype=torch.bfloat16) if a.res else None
    cfgs = range(ops.NUM_TILE_CFGS) if a.cfg < 0 else [a.cfg]
    out = {}
    for c in cfgs:
        for _ in range(5):
            ops.linear(x, w, b, act=a.act, residual=r, tile_cfg=c)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            ops.linear(x, w, b, act=a.act, residual=r, tile_cfg=c)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.iters * 1e3
        out[c] = dict(us=round(us, 2), tflops=round(2 * a.m * a.n * a.k / us / 1e6, 1))
    t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        torch.nn.functional.linear(x, w, b)
    torch.cuda.synchronize()
    t[0].record()
    for _ in range(a.iters):
        torch.nn.functional.linear(x, w, b)
    t[1].record()
    torch.cuda.synchronize()
    hb = t[0].elapsed_time(t[1]) / a.iters * 1e3
    print(json.dumps(dict(shape=[a.m, a.n, a.k], ours=out, hipblaslt_us=round(hb, 2),
                          hipblaslt_tflops=round(2 * a.m * a.n * a.k / hb / 1e6, 1))))


if __name__ == "__main__":
    main()
