"""Single-stream graph replay of one CNN forward (ResNet-50 by default), for
rocprofv3 kernel traces and ``--pmc`` counter passes of the conv kernels:

    rocprofv3 --pmc SQ_INSTS_MFMA ... -- python bench/cnn_breakdown.py --model resnet50 --batch 32 --iters 5

Prints the replay time per forward and the model FLOP rate.  ``--tune-file``
loads the conv / GEMM tile table when it exists, else tunes and writes it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--tune-file", default="")
    a = ap.parse_args()
    import torch

    from ray_dynamic_batching_amd import models, ops

    m = models.create(a.model, device="cuda:0")
    x = m.example_input(a.batch, seed=0)
    if a.tune_file and os.path.exists(a.tune_file):
        ops.load_tuning(a.tune_file)
    for _ in range(3):
        m(x)
    if a.tune_file and not os.path.exists(a.tune_file):
        ops.save_tuning(a.tune_file)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m(x)
        # split-K launches share one workspace, as in the engine's graphs (ops.capture_splitk_workspace)
        with torch.cuda.graph(g, stream=s), ops.capture_splitk_workspace(ops.splitk_workspace("cuda:0")):
            m(x)
    torch.cuda.synchronize()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    fl = getattr(m, "flops_per_image", lambda: 0.0)() * a.batch
    print(json.dumps(dict(model=a.model, batch=a.batch, ms_per_forward=round(ms, 4),
                          img_per_s=round(a.batch / ms * 1e3, 1), model_tflops=round(fl / ms / 1e9, 1) if fl else None)))


if __name__ == "__main__":
    main()
