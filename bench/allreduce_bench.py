"""All-reduce microbenchmark: custom xGMI kernel (parallel/xgmi.py) vs RCCL
(torch.distributed "nccl") on the message sizes of TP prefill / decode.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench/allreduce_bench.py

One rank per GPU.  Every size is checked for the same result on both paths
(bit-exact between the ranks of the xgmi path) before it is timed; times are
the max over ranks of CUDA-event time per call over ``--iters`` calls, both
paths captured the same way (eager, same stream).  ``--fused-norm`` times the
all-reduce + RMSNorm the TP Llama uses against RCCL all-reduce + our RMSNorm
kernel.  Rank 0 prints one JSON line.

``--same-gpu N`` (1-GPU rehearsal): N processes share GPU 0 and only the xgmi
path runs (RCCL refuses two ranks on one device); the numbers then measure the
protocol (flags, barriers, HBM traffic), not xGMI links.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4x4096,64x4096,256x4096,1024x4096,2048x4096",
                    help="comma list of TxD (bf16 rows x hidden)")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--fused-norm", action="store_true")
    ap.add_argument("--same-gpu", action="store_true", help="all ranks on GPU 0, xgmi path only")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    from ray_dynamic_batching_amd import ops
    from ray_dynamic_batching_amd.parallel import collective as col

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if a.same_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    sizes = [tuple(int(v) for v in s.split("x")) for s in a.sizes.split(",")]
    max_elems = max(t * d for t, d in sizes)
    col.init_collective_group(world, rank, "gloo" if a.same_gpu else "nccl", "ar")
    xg = col.enable_xgmi("ar", max_elems=max_elems, timeout_s=20.0)
    if xg is None:
        raise SystemExit("xgmi all-reduce unavailable on this platform")
    pg = col.get_group_handle("ar")
    hdev = "cpu" if a.same_gpu else "cuda"     # where host-side scalars go for the group's backend
    res = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        dist.barrier(group=pg)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        t = torch.tensor([e0.elapsed_time(e1) / a.iters * 1e3], dtype=torch.float64, device=hdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=pg)
        return t.item()

    for T, D in sizes:
        g = torch.Generator().manual_seed(T * 7 + rank)
        x = torch.randn(T, D, generator=g).to(torch.bfloat16).cuda()
        gamma = torch.ones(D, dtype=torch.bfloat16, device="cuda")
        row = {"T": T, "D": D, "bytes": T * D * 2}
        # correctness first: same sum on every rank, and vs RCCL
        s = xg.all_reduce(x).clone()
        torch.cuda.synchronize()
        chk = s.float().sum().reshape(1).double().to(hdev)
        allc = [torch.zeros(1, dtype=torch.float64, device=hdev) for _ in range(world)]
        dist.all_gather(allc, chk, group=pg)
        row["ranks_agree"] = all(float(c) == float(allc[0]) for c in allc)
        if not a.same_gpu:
            r = x.clone()
            dist.all_reduce(r, group=pg)
            row["max_abs_diff_vs_rccl"] = float((r.float() - s.float()).abs().max())
        if a.fused_norm:
            row["xgmi_ar_norm_us"] = round(timed(lambda: xg.all_reduce_rmsnorm(x, gamma, 1e-5)), 2)
            if not a.same_gpu:
                def rccl_norm():
                    r = x.clone()
                    dist.all_reduce(r, group=pg)
                    ops.rms_norm(r, gamma, 1e-5)
                row["rccl_ar_plus_norm_us"] = round(timed(rccl_norm), 2)
        row["xgmi_us"] = round(timed(lambda: xg.all_reduce(x)), 2)
        row["xgmi_algbw_GBps"] = round(row["bytes"] / row["xgmi_us"] / 1e3, 1)
        if not a.same_gpu:
            buf = x.clone()
            row["rccl_us"] = round(timed(lambda: dist.all_reduce(buf, group=pg)), 2)
            row["rccl_algbw_GBps"] = round(row["bytes"] / row["rccl_us"] / 1e3, 1)
        res.append(row)
    if rank == 0:
        print(json.dumps(dict(metric="bf16 all-reduce time per call (max over ranks)", world=world,
                              same_gpu=a.same_gpu, iters=a.iters, results=res)), flush=True)
    col.barrier("ar")
    col.destroy_collective_group("ar")


if __name__ == "__main__":
    main()
