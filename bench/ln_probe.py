"""A/B of the deferred-LayerNorm GEMM epilogues (ops.linear_ln) against the
plain fused-epilogue GEMM (+ the LayerNorm kernel they replace), per BERT-base
bs32 shape and tile, CUDA-event timed in one process.

    python bench/ln_probe.py [--iters 200]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    import torch

    from ray_dynamic_batching_amd import ops

    torch.manual_seed(0)
    M, D, I = 4096, 768, 3072
    bf = torch.bfloat16

    def t(f):
        for _ in range(10):
            f()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            f()
        e.record()
        e.synchronize()
        return round(s.elapsed_time(e) / a.iters * 1e3, 2)

    x = torch.randn(M, D, device="cuda", dtype=bf)
    st = torch.stack([x.float().sum(1), (x.float() ** 2).sum(1)], 1).contiguous()
    g, be = torch.ones(D, device="cuda", dtype=bf), torch.zeros(D, device="cuda", dtype=bf)
    out = []
    for name, N, K, act, cfgs in [("qkv", 3 * D, D, "none", [8, 11, 16]), ("ffn_up", I, D, "gelu", [4, 15, 8])]:
        xx = torch.randn(M, K, device="cuda", dtype=bf)
        sx = torch.stack([xx.float().sum(1), (xx.float() ** 2).sum(1)], 1).contiguous()
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.02
        b = torch.randn(N, device="cuda", dtype=bf) * 0.02
        w2, cs, b2 = ops.fold_ln_weights(w, b, torch.ones(K, device="cuda", dtype=bf), torch.zeros(K, device="cuda", dtype=bf))
        for c in cfgs:
            out.append(dict(shape=name, cfg=c,
                            plain_us=t(lambda: ops.linear(xx, w, b, act=act, tile_cfg=c)),
                            lna_us=t(lambda: ops.linear_ln(xx, w2, act=act, lna=(sx, cs, b2, K, 1e-12), tile_cfg=c))))
    ln_us = t(lambda: ops.layer_norm(x, g, be))
    for name, N, K, cfgs in [("o_proj", D, D, [9, 12, 10, 17]), ("ffn_down", D, I, [12, 10, 9, 17, 18])]:
        xx = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.02
        b = torch.randn(N, device="cuda", dtype=bf) * 0.02
        o = torch.zeros(M, 2, device="cuda")
        for c in cfgs:
            out.append(dict(shape=name, cfg=c,
                            plain_us=t(lambda: ops.linear(xx, w, b, residual=x, tile_cfg=c)),
                            stats_us=t(lambda: ops.linear_ln(xx, w, b, residual=x, out_stats=o, tile_cfg=c)),
                            lnr_stats_us=t(lambda: ops.linear_ln(xx, w, b, residual=x, lnr=(st, g, be, D, 1e-12),
                                                                  out_stats=o, tile_cfg=c))))
    print(json.dumps({"layernorm_4096x768_us": ln_us, "rows": out}))


if __name__ == "__main__":
    main()
