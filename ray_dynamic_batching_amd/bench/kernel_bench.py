"""Per-kernel microbenchmarks of the gfx950 kernels vs the vendor path
(torch -> hipBLASLt / MIOpen / aotriton) on the shapes of the serving models.

    python -m ray_dynamic_batching_amd.bench.kernel_bench [--only gemm|attn|conv|norm] [--json out.json]

Timing: interleaved A/B in one process (guide rule 24), random data (rule 25),
CUDA-event timing over many iterations after warmup.
"""
from __future__ import annotations

import argparse
import json

import torch
import torch.nn.functional as F


def _time(fn, iters=50, warmup=10):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def bench_gemm(rows):
    from .. import ops

    shapes = [  # (name, M, N, K, act, residual)
        ("bert.qkv bs32", 4096, 2304, 768, "none", False),
        ("bert.o bs32", 4096, 768, 768, "none", True),
        ("bert.ffn1 bs32", 4096, 3072, 768, "gelu", False),
        ("bert.ffn2 bs32", 4096, 768, 3072, "none", True),
        ("bert.qkv bs8", 1024, 2304, 768, "none", False),
        ("bert.ffn1 bs8", 1024, 3072, 768, "gelu", False),
        ("square 4096", 4096, 4096, 4096, "none", False),
        ("llama.qkv tp8 1k", 1024, 768, 4096, "none", False),
        ("llama.gateup tp8 1k", 1024, 3584, 4096, "swiglu", False),
        ("llama.down tp8 1k", 1024, 4096, 1792, "none", True),
    ]
    for name, M, N, K, act, res in shapes:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * K ** -0.5
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
        n_out = N // 2 if act == "swiglu" else N
        r = torch.randn(M, n_out, device="cuda", dtype=torch.bfloat16) if res else None

        def ours():
            ops.linear(x, w, b, act=act, residual=r)

        def vendor():
            y = F.linear(x, w, b)
            if act == "gelu":
                y = F.gelu(y)
            elif act == "swiglu":
                y = F.silu(y[:, 0::2]) * y[:, 1::2]
            if r is not None:
                y = y + r
            return y

        def vendor_gemm_only():
            return F.linear(x, w, b)

        t_o, t_v, t_g = _time(ours), _time(vendor), _time(vendor_gemm_only)
        fl = 2.0 * M * N * K
        rows.append(dict(kernel="gemm", shape=name, M=M, N=N, K=K, ours_us=round(t_o, 2), vendor_us=round(t_v, 2),
                         vendor_gemm_only_us=round(t_g, 2), ours_tflops=round(fl / t_o / 1e6, 1),
                         vendor_gemm_tflops=round(fl / t_g / 1e6, 1), speedup_vs_vendor_fused=round(t_v / t_o, 3)))


def bench_attn(rows):
    from .. import ops

    for B, S, H, D, causal in [(32, 128, 12, 64, False), (8, 128, 12, 64, False), (8, 512, 32, 128, True)]:
        Hkv = H if not causal else H // 4
        qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)

        def ours():
            ops.attention(qkv, B, S, H, Hkv, D, causal=causal)

        def vendor():
            q = qkv[:, :H * D].view(B, S, H, D).transpose(1, 2)
            k = qkv[:, H * D:(H + Hkv) * D].view(B, S, Hkv, D).transpose(1, 2)
            v = qkv[:, (H + Hkv) * D:].view(B, S, Hkv, D).transpose(1, 2)
            if Hkv != H:
                k = k.repeat_interleave(H // Hkv, 1)
                v = v.repeat_interleave(H // Hkv, 1)
            return F.scaled_dot_product_attention(q, k, v, is_causal=causal).transpose(1, 2).reshape(B * S, H * D)

        t_o, t_v = _time(ours), _time(vendor)
        fl = 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)
        rows.append(dict(kernel="attention", shape=f"B{B} S{S} H{H}/{Hkv} D{D} causal={causal}", ours_us=round(t_o, 2),
                         vendor_us=round(t_v, 2), ours_tflops=round(fl / t_o / 1e6, 1),
                         speedup_vs_vendor=round(t_v / t_o, 3)))


def bench_norm(rows):
    from .. import ops

    for T, D in [(4096, 768), (8192, 4096)]:
        x = torch.randn(T, D, device="cuda", dtype=torch.bfloat16)
        g = torch.ones(D, device="cuda", dtype=torch.bfloat16)
        b = torch.zeros(D, device="cuda", dtype=torch.bfloat16)
        t_o = _time(lambda: ops.layer_norm(x, g, b))
        t_v = _time(lambda: F.layer_norm(x, (D,), g, b))
        gbs = 2 * x.numel() * 2 / t_o / 1e3
        rows.append(dict(kernel="layernorm", shape=f"{T}x{D}", ours_us=round(t_o, 2), vendor_us=round(t_v, 2),
                         ours_GBps=round(gbs, 1), speedup_vs_vendor=round(t_v / t_o, 3)))


def bench_conv(rows):
    from .. import ops

    for N, H, C, K, R, st, pad in [(32, 56, 64, 64, 3, 1, 1), (32, 56, 64, 256, 1, 1, 0), (32, 28, 128, 128, 3, 1, 1),
                                   (32, 14, 256, 256, 3, 1, 1), (32, 7, 512, 512, 3, 1, 1), (32, 224, 8, 64, 7, 2, 3)]:
        x = torch.randn(N, H, H, C, device="cuda", dtype=torch.float16)
        w = torch.randn(K, R, R, C, device="cuda", dtype=torch.float16) * (R * R * C) ** -0.5
        b = torch.randn(K, device="cuda", dtype=torch.float16)
        xc = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        t_o = _time(lambda: ops.conv2d_nhwc(x, w, b, stride=st, pad=pad, act="relu"))
        t_v = _time(lambda: F.relu(F.conv2d(xc, wc, b, stride=st, padding=pad)))
        P = (H + 2 * pad - R) // st + 1
        fl = 2.0 * N * P * P * K * R * R * C
        rows.append(dict(kernel="conv2d", shape=f"N{N} {H}x{H}x{C}->{K} r{R} s{st}", ours_us=round(t_o, 2),
                         vendor_us=round(t_v, 2), ours_tflops=round(fl / t_o / 1e6, 1),
                         speedup_vs_vendor=round(t_v / t_o, 3)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["gemm", "attn", "conv", "norm"])
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    rows = []
    for k, f in [("gemm", bench_gemm), ("attn", bench_attn), ("norm", bench_norm), ("conv", bench_conv)]:
        if a.only in (None, k):
            f(rows)
    for r in rows:
        print(json.dumps(r))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
