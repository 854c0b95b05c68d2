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
    ap.add_argument("--streamk", type=int, default=0, help="also time the stream-K kernel on this many workgroups")
    ap.add_argument("--graph", type=int, default=1, help="1: time a captured graph of --iters calls (default)")
    a = ap.parse_args(argv)
    import torch

    from ray_dynamic_batching_amd import ops

    torch.manual_seed(0)
    x = torch.randn(a.m, a.k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(a.n, a.k, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(a.n, device="cuda", dtype=torch.bfloat16) if a.bias else None
    r = torch.randn(a.m, a.n, device="cuda", dtype=torch.bfloat16) if a.res else None
    cfgs = (list(range(ops.NUM_TILE_CFGS)) + [c | ops.DEEP for c in ops._DEEP_TILES]) if a.cfg < 0 else [a.cfg]
    out = {}

    def timed(fn) -> float:
        """us per call: eager loop, or (--graph, the default) one hipGraph of
        --iters calls, so host launch cost never shows in short kernels."""
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if a.graph:
            g = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st), torch.cuda.graph(g, stream=st):
                for _ in range(a.iters):
                    fn()
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            s.record()
            g.replay()
            e.record()
        else:
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.iters * 1e3

    for c in cfgs:
        us = timed(lambda: ops.linear(x, w, b, act=a.act, residual=r, tile_cfg=c))
        out[c] = dict(us=round(us, 2), tflops=round(2 * a.m * a.n * a.k / us / 1e6, 1))
    if a.streamk:
        for tile in (0, 1):
            ws = ops.streamk_workspace(x.device, a.streamk, tile)
            us = timed(lambda: ops.linear_streamk(x, w, b, act=a.act, residual=r, workspace=ws, grid=a.streamk,
                                                  tile=tile))
            out[f"streamk_t{tile}_g{a.streamk}"] = dict(us=round(us, 2), tflops=round(2 * a.m * a.n * a.k / us / 1e6, 1))
    hb = timed(lambda: torch.nn.functional.linear(x, w, b))
    print(json.dumps(dict(shape=[a.m, a.n, a.k], ours=out, hipblaslt_us=round(hb, 2),
                          hipblaslt_tflops=round(2 * a.m * a.n * a.k / hb / 1e6, 1))))


if __name__ == "__main__":
    main()
