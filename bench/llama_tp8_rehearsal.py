#!/usr/bin/env python3
"""Config-4 rehearsal at Llama-3-8B layer dimensions on the ONE GPU a box has:
TP ranks as separate processes (spawned; gloo rendezvous, HIP IPC between the
processes, the custom xGMI all-reduce + fused RMSNorm between the shards), a
2-layer slice of Llama-3-8B (hidden 4096, 32 q / 8 kv heads of 128, FFN
14336: at TP=8 each rank holds 4 q heads + 1 kv head and a 1,792-wide FFN
shard), random init, prefill of ``--batch`` x ``--seq`` tokens.

It reports every rank's prefill time.  All ranks share one GPU here, and
before every all-reduce they drain and line up (a rank spinning in the
all-reduce kernel would hold the CU slots a peer's GEMM needs), so the times
are a REHEARSAL of the protocol at real shapes, not a TP=8 measurement.

    python bench/llama_tp8_rehearsal.py --world 8 --json-out profiles/llama3_8b_tp8_rehearsal_r4.json

Reference: the fork's TP path is Ray's collective API on NCCL
(python/ray/util/collective/collective_group/nccl_collective_group.py:175-233);
SURVEY §2.5 config 4.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import time

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)


def llama3_8b_slice(layers: int = 2, vocab: int = 32768, seq: int = 128):
    """Llama-3-8B layer geometry; the vocabulary is cut to 32k (the LM head is
    one GEMM beside the layers; a 128k random table would only slow the init)."""
    from ray_dynamic_batching_amd.models.llama import LlamaConfig

    return LlamaConfig.llama3_8b(layers=layers, vocab_size=vocab, seq_len=seq, max_position=max(seq, 1024))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _line_up():
    import torch

    from ray_dynamic_batching_amd.parallel import collective as col

    torch.cuda.synchronize()
    col.barrier("tp")


def worker(rank, world, port, q, cfg_kw, batch, reps, anchor):
    """One TP rank: build its shard, prefill ``reps`` times, report timings and
    the hidden states (first 64 columns) -- plus, at world 1 with ``anchor``,
    the fp32 PyTorch path of the same weights and the bf16 eager path."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch

    torch.set_num_threads(2)
    from ray_dynamic_batching_amd.models.llama import LlamaTP
    from ray_dynamic_batching_amd.parallel import collective as col

    torch.cuda.set_device(0)
    import faulthandler

    faulthandler.dump_traceback_later(400, exit=True)
    try:
        cfg = llama3_8b_slice(**cfg_kw)
        if world > 1:
            col.init_collective_group(world, rank, backend="gloo", group_name="tp")
            col.enable_xgmi("tp", max_elems=batch * cfg.seq_len * cfg.hidden, timeout_s=30.0)
        t0 = time.perf_counter()
        m = LlamaTP(cfg, rank, world, group_name="tp" if world > 1 else None, device="cuda", backend="hip",
                    init="full")
        build_s = time.perf_counter() - t0
        if world > 1:
            m.pre_collective = _line_up
        ids = m.example_input(batch, seed=3)
        x = m.hidden_states(ids)          # warm-up (and the checked output)
        torch.cuda.synchronize()
        times = []
        for _ in range(reps):
            if world > 1:
                _line_up()
            t = time.perf_counter()
            m.hidden_states(ids)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t) * 1e3)
        err = m._xgmi().error() if world > 1 else 0
        out = dict(rank=rank, world=world, build_s=round(build_s, 2), prefill_ms=times,
                   sample=x[:, :64].float().cpu().tolist(), xgmi_error=err,
                   local_heads=m.Hl, local_kv_heads=m.Hkvl, local_ffn=m.Fl)
        if anchor and world == 1:
            from ray_dynamic_batching_amd.models.reference import eager_reference, fp32_reference, rel_err

            ref = fp32_reference(m).hidden_states(ids)
            eager = eager_reference(m).hidden_states(ids)
            out["ref_sample"] = ref[:, :64].float().cpu().tolist()
            out["hip_vs_fp32"] = rel_err(x, ref)
            out["eager_vs_fp32"] = rel_err(eager, ref)
        q.put((rank, out))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise
    finally:
        if world > 1:
            col.barrier("tp")
            col.destroy_collective_group("tp")


def run(world: int, batch: int = 8, reps: int = 3, anchor: bool = False, timeout_s: float = 480.0, **cfg_kw):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, world, port, q, cfg_kw, batch, reps, anchor)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        got = dict(q.get(timeout=timeout_s) for _ in range(world))
    finally:
        for p in ps:
            p.join(60)
            if p.is_alive():
                p.kill()
    return got


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    res = {}
    for w in sorted({1, a.world}):
        got = run(w, a.batch, a.reps, anchor=(w == 1), seq=a.seq)
        for r, v in got.items():
            if isinstance(v, str):
                raise SystemExit(f"world {w} rank {r}: {v}")
        res[w] = {r: {k: v for k, v in d.items() if k not in ("sample", "ref_sample")} for r, d in got.items()}
        print(json.dumps({"world": w, "median_prefill_ms": {r: statistics.median(d["prefill_ms"])
                                                            for r, d in got.items()}}), flush=True)
    cfg = llama3_8b_slice(seq=a.seq)
    line = {"what": "REHEARSAL, not a measurement: Llama-3-8B 2-layer slice, TP ranks as processes sharing ONE "
                    "MI355X (lined up before every all-reduce), xGMI all-reduce + fused RMSNorm over HIP IPC",
            "config": dict(hidden=cfg.hidden, heads=cfg.heads, kv_heads=cfg.kv_heads, head_dim=cfg.head_dim,
                           intermediate=cfg.intermediate, layers=cfg.layers, vocab=cfg.vocab_size,
                           tokens=a.batch * a.seq),
            "results": res}
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(line, f, indent=1)


if __name__ == "__main__":
    main()
