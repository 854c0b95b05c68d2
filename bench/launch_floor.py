"""Per-kernel fixed cost inside a replayed hipGraph.

    python bench/launch_floor.py [--n 200]

Captures graphs of N back-to-back launches of (a) a trivial kernel
(ops.seq_lens on 32 x 128 ids), (b) a LayerNorm of 4096 x 768 bf16 and
(c) alternating LayerNorms reading the previous one's output, replays each and
prints microseconds per kernel.  Run it under different HIP runtime settings
(environment) to see what the dispatch / end-of-kernel floor is.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch

    from ray_dynamic_batching_amd import ops

    dev = torch.device("cuda", 0)
    ids = torch.randint(1, 1000, (32, 128), device=dev, dtype=torch.int32)
    x = torch.randn(4096, 768, device=dev, dtype=torch.bfloat16)
    g_, b_ = torch.ones(768, device=dev, dtype=torch.bfloat16), torch.zeros(768, device=dev, dtype=torch.bfloat16)
    y = torch.empty_like(x)
    lens = torch.empty(32, device=dev, dtype=torch.int32)

    def trivial():
        for _ in range(a.n):
            ops._ops().seq_lens(ids.data_ptr(), 32, 128, 0, lens.data_ptr(), ops._stream())

    def ln(src, dst):
        ops._ops().norm_fwd(0, 0, src.data_ptr(), 0, 0, g_.data_ptr(), b_.data_ptr(), dst.data_ptr(), 4096, 768,
                            768, 1e-12, ops._stream())

    def ln_same():
        for _ in range(a.n):
            ln(x, y)

    def ln_chain():
        src, dst = x, y
        for _ in range(a.n):
            ln(src, dst)
            src, dst = dst, src

    out = {"env": {k: os.environ[k] for k in sorted(os.environ) if k.startswith(("HIP_", "DEBUG_CLR", "ROC_", "AMD_", "GPU_"))}}
    s = torch.cuda.Stream()
    for name, fn in [("trivial", trivial), ("layernorm_4096x768", ln_same), ("layernorm_chain", ln_chain)]:
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                fn()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = float("inf")
        for _ in range(a.iters):
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        out[name + "_us_per_kernel"] = round(best * 1e3 / a.n, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
