"""Single-stream per-op time of one BERT-base forward (graph replay), for
rocprofv3 kernel traces:

    rocprofv3 --kernel-trace --stats -d gpurun_out/bd -- python bench/bert_breakdown.py --batch 32 --iters 50

Prints the graph replay time per forward (CUDA events) and the model FLOP rate.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--tune-file", default="", help="load the GEMM tile table from this JSON if it exists, "
                                                    "else write the tuned table to it")
    a = ap.parse_args()
    import torch

    from ray_dynamic_batching_amd import ops

    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification

    m = BertForSequenceClassification(BertConfig(layers=a.layers), device="cuda:0", backend="hip")
    ids = m.example_input(a.batch, seed=0)
    if a.tune_file and os.path.exists(a.tune_file):
        ops.load_tuning(a.tune_file)
    for _ in range(3):
        m(ids)
    if a.tune_file and not os.path.exists(a.tune_file):
        ops.save_tuning(a.tune_file)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m(ids)
        # split-K launches share one workspace, as in the engine's graphs (ops.capture_splitk_workspace)
        with torch.cuda.graph(g, stream=s), ops.capture_splitk_workspace(ops.splitk_workspace("cuda:0")):
            m(ids)
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
    fl = m.flops_per_sequence() * a.batch
    print(json.dumps(dict(batch=a.batch, ms_per_forward=round(ms, 4), seq_per_s=round(a.batch / ms * 1e3, 1),
                          model_tflops=round(fl / ms / 1e9, 1))))


if __name__ == "__main__":
    main()
