"""Run the fused attention kernel on one shape many times (rocprofv3 target).

    python bench/attn_probe.py --b 32 --s 128 --h 12 --d 64 --iters 100
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=32)
    ap.add_argument("--s", type=int, default=128)
    ap.add_argument("--h", type=int, default=12)
    ap.add_argument("--hkv", type=int, default=0)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--causal", action="store_true")
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    import torch

    from ray_dynamic_batching_amd import ops

    hkv = a.hkv or a.h
    qkv = torch.randn(a.b * a.s, (a.h + 2 * hkv) * a.d, device="cuda", dtype=torch.bfloat16)
    lens = torch.full((a.b,), a.s, device="cuda", dtype=torch.int32)
    out = torch.empty(a.b * a.s, a.h * a.d, device="cuda", dtype=torch.bfloat16)
    for _ in range(5):
        ops.attention(qkv, a.b, a.s, a.h, hkv, a.d, lens=lens, causal=a.causal, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        ops.attention(qkv, a.b, a.s, a.h, hkv, a.d, lens=lens, causal=a.causal, out=out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    fl = 4 * a.b * a.h * a.s * a.s * a.d / (2 if a.causal else 1)
    print(json.dumps(dict(shape=[a.b, a.s, a.h, hkv, a.d], causal=a.causal, us=round(us, 2),
                          tflops=round(fl / us / 1e6, 1))))


if __name__ == "__main__":
    main()
