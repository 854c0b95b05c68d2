"""Side-by-side GEMM probe: hipBLASLt (via torch) against this repo's MFMA GEMM
on the BERT-base bs32 shapes and 4096^3, for timing and for rocprofv3.

    python bench/gemm_vendor_probe.py --which both --iters 200 > out.json
    rocprofv3 --kernel-trace --stats -- python3 bench/gemm_vendor_probe.py --which vendor
    rocprofv3 --pmc ... -- python3 bench/gemm_vendor_probe.py --which ours --iters 20

Every arm is one hipGraph of ``--iters`` calls of the same GEMM (so no host
launch cost shows), timed with events on an idle GPU: the single-kernel
latency the verdict's done-bar quotes ("standalone").  ``ours`` uses the tile
the shipped BERT table picks for that shape (``--cfg`` overrides it); a
``--sweep`` also times every tile config.  Operands are uniform random bf16
(zero-filled operands read high on MI355X: DVFS).

Shapes (M, N, K, epilogue): QKV 4096x2304x768 (+bias), o-proj 4096x768x768
(+bias +residual), FFN-up 4096x3072x768 (+bias +GELU), FFN-down
4096x768x3072 (+bias +residual), and 4096^3 (plain).  The vendor arm runs
``F.linear`` (+bias epilogue) and, for GELU, ``torch._addmm_activation``
(hipBLASLt's fused GELU epilogue); residual adds are left out of the vendor
arm (it has no such epilogue), so the vendor number is a lower bound on a
vendor implementation of the same op.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "qkv": (4096, 2304, 768, "none", False),
    "oproj": (4096, 768, 768, "none", True),
    "ffn_up": (4096, 3072, 768, "gelu", False),
    "ffn_down": (4096, 768, 3072, "none", True),
    "sq4096": (4096, 4096, 4096, "none", False),
}
# shipped BERT bs32 table (ops/tuned/mi355x_bert_L12_S128_B32_cs2_d4.json); qkv
# runs fused with attention in the model, here its plain GEMM on tile 19
SHIPPED = {"qkv": 19, "oproj": 19, "ffn_up": 23, "ffn_down": 19, "sq4096": 22}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", choices=["vendor", "ours", "both"], default="both")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5, help="timed graph replays per arm (median reported)")
    ap.add_argument("--cfg", type=int, default=-1, help="our tile config (default: shipped per shape)")
    ap.add_argument("--sweep", action="store_true", help="also time every tile config")
    ap.add_argument("--splits", default="", help="with --sweep: also time these split-K counts (e.g. 2,3,4) on "
                    "the split-capable tiles, with a caller workspace")
    a = ap.parse_args(argv)
    import torch
    import torch.nn.functional as F

    from ray_dynamic_batching_amd import ops

    def timed(fn) -> float:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st), torch.cuda.graph(g, stream=st):
            for _ in range(a.iters):
                fn()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / a.iters * 1e3)
        ts.sort()
        return ts[len(ts) // 2]

    torch.manual_seed(0)
    out = {}
    for name in a.shapes.split(","):
        m, n, k, act, res = SHAPES[name]
        x = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(n, k, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        b = None if name == "sq4096" else (torch.rand(n, device="cuda") * 0.1).to(torch.bfloat16)
        r = (torch.rand(m, n, device="cuda") * 2 - 1).to(torch.bfloat16) if res else None
        flop = 2.0 * m * n * k
        row = dict(shape=[m, n, k], act=act, residual=res)
        if a.which in ("vendor", "both"):
            if act == "gelu":
                wt = w.t()
                fn = lambda: torch._addmm_activation(b, x, wt, use_gelu=True)
            else:
                fn = lambda: F.linear(x, w, b)
            us = timed(fn)
            row["vendor_us"] = round(us, 2)
            row["vendor_tflops"] = round(flop / us / 1e6, 1)
        if a.which in ("ours", "both"):
            cfg = a.cfg if a.cfg >= 0 else SHIPPED[name]
            us = timed(lambda: ops.linear(x, w, b, act=act, residual=r, tile_cfg=cfg))
            row["ours_cfg"] = cfg
            row["ours_us"] = round(us, 2)
            row["ours_tflops"] = round(flop / us / 1e6, 1)
            if a.sweep:
                sw = {}
                for c in range(ops.NUM_TILE_CFGS):
                    try:
                        sw[c] = round(timed(lambda: ops.linear(x, w, b, act=act, residual=r, tile_cfg=c)), 2)
                    except Exception as ex:  # tile not valid for this epilogue
                        sw[c] = str(ex)[:40]
                if a.splits:
                    # the split-K choices the tuner would consider (workspace-bounded)
                    ws = ops.splitk_workspace(x.device)
                    want = {int(v) for v in a.splits.split(",") if v}
                    for c in ops._gemm_candidates(m, n, k, splitk=True):
                        if ops.splits_of(c) in want and not c & ops.DEEP:
                            sw[f"{c & 255}|{ops.splits_of(c)}"] = round(timed(
                                lambda: ops.linear(x, w, b, act=act, residual=r, tile_cfg=c, workspace=ws)), 2)
                row["ours_sweep_us"] = sw
        out[name] = row
        print(json.dumps({name: row}), flush=True)
    print(json.dumps(dict(gemm_vendor_probe=out)))


if __name__ == "__main__":
    main()
