"""Config-4 readiness at production dimensions on the one GPU a box has
(VERDICT r3 "next round" item 4):

* the xGMI all-reduce and all-reduce + RMSNorm at the TP=8 prefill message of
  Llama-3-8B (1024 tokens x 4096 = 8 MiB bf16), one-shot and two-shot, eager
  and under hipGraph replay x3, at world 8 (8 processes, HIP IPC);
* a Llama-3-8B 2-layer slice at TP=8 (4 q heads + 1 kv head and a 1,792-wide
  FFN shard per rank) against the TP=1 model and the fp32 anchor of the same
  weights;
* the RCCL backend of ``parallel.collective`` at world 1 -- every collective
  op -- and the xGMI -> RCCL fallbacks (message over ``max_elems``, a shape the
  custom kernel does not take, a non-SUM op, and ``enable_xgmi`` failing).

Reference: python/ray/util/collective/collective.py:258-655,
collective_group/nccl_collective_group.py:175-233.
"""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_Q_TIMEOUT = 480


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    try:
        got = dict(q.get(timeout=_Q_TIMEOUT) for _ in range(world))
    finally:
        for p in ps:
            p.join(60)
            if p.is_alive():
                p.kill()
    return got


def _inputs(world, T, D, seed):
    g = torch.Generator().manual_seed(seed)
    xs = [torch.randn(T, D, generator=g).to(torch.bfloat16) for _ in range(world)]
    gamma = (1.0 + 0.1 * torch.randn(D, generator=g)).to(torch.bfloat16)
    return xs, gamma


def _reference(xs, gamma, eps):
    acc = torch.zeros_like(xs[0], dtype=torch.float32)
    for x in xs:
        acc = acc + x.float()
    s = acc.to(torch.bfloat16)
    sf = s.float()
    h = (sf * torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + eps) * gamma.float()).to(torch.bfloat16)
    return s, h


def _ar_worker(rank, world, port, q, shapes, max_elems, one_shot_bytes):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import hashlib

    import torch

    from ray_dynamic_batching_amd.parallel import collective as col

    def digest(t):
        return hashlib.sha1(t.contiguous().view(torch.int16).cpu().numpy().tobytes()).hexdigest()

    torch.set_num_threads(2)
    torch.cuda.set_device(0)
    col.init_collective_group(world, rank, backend="gloo", group_name="tp")
    res = []
    try:
        xg = col.enable_xgmi("tp", max_elems=max_elems, one_shot_max_bytes=one_shot_bytes, timeout_s=30.0)
        eps = 1e-5
        for T, D, two in shapes:
            xs, gamma = _inputs(world, T, D, seed=T + D)
            x, g = xs[rank].cuda(), gamma.cuda()
            col.barrier("tp")
            s, h = xg.all_reduce_rmsnorm(x, g, eps, two_shot=two)
            torch.cuda.synchronize()
            ref_s, ref_h = _reference(xs, gamma, eps)
            res.append(("eager", T, D, two, xg.error(), digest(s), torch.equal(s.cpu(), ref_s),
                        float((h.cpu().float() - ref_h.float()).abs().max())))
            graph = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                with torch.cuda.graph(graph, stream=st):
                    gs, gh = xg.all_reduce_rmsnorm(x, g, eps, two_shot=two)
                    gs = gs.clone()
            torch.cuda.synchronize()
            for it in range(3):
                xs, _ = _inputs(world, T, D, seed=1000 * T + it)
                x.copy_(xs[rank].cuda())
                torch.cuda.synchronize()
                col.barrier("tp")
                graph.replay()
                torch.cuda.synchronize()
                ref_s, ref_h = _reference(xs, gamma, eps)
                res.append(("replay", T, D, two, xg.error(), digest(gs), torch.equal(gs.cpu(), ref_s),
                            float((gh.cpu().float() - ref_h.float()).abs().max())))
            del graph
        q.put((rank, res))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise
    finally:
        col.barrier("tp")
        col.destroy_collective_group("tp")


def test_xgmi_allreduce_llama3_prefill_message_world8():
    """1024 x 4096 bf16 (8 MiB, max_elems 4M) -- Llama-3-8B TP=8 prefill of 8 x 128
    tokens -- one-shot and two-shot, plus a row count not divisible by the world,
    eager and graph replay x3: bit-identical across ranks and equal to the fp32
    sum rounded to bf16; fused RMSNorm within bf16 rounding."""
    world = 8
    shapes = [(1024, 4096, False), (1024, 4096, True), (1000, 4096, True)]
    got = _spawn(_ar_worker, world, shapes, 1 << 22, 8 << 20)
    for r in range(world):
        assert not isinstance(got[r], str), got[r]
    assert len(got[0]) == 4 * len(shapes)
    for i in range(len(got[0])):
        rows = [got[r][i] for r in range(world)]
        kind, T, D, two = rows[0][:4]
        assert all(row[4] == 0 for row in rows), f"{kind} T={T}: barrier timeout"
        assert len({row[5] for row in rows}) == 1, f"{kind} T={T} two_shot={two}: ranks differ"
        assert all(row[6] for row in rows), f"{kind} T={T} two_shot={two}: sum != fp32 sum in bf16"
        assert all(row[7] < 3e-2 for row in rows), f"{kind} T={T}: norm error {[row[7] for row in rows]}"


def test_llama3_8b_slice_tp8_matches_tp1_and_fp32_anchor():
    """Llama-3-8B layer dims, 2 layers, TP=8 as 8 processes on one GPU vs TP=1,
    both against the fp32 PyTorch path of the same weights."""
    sys.path.insert(0, os.path.join(_ROOT, "bench"))
    import llama_tp8_rehearsal as reh

    from ray_dynamic_batching_amd.models.reference import parity_bound

    one = reh.run(1, batch=8, reps=1, anchor=True)[0]
    assert not isinstance(one, str), one
    eight = reh.run(8, batch=8, reps=1)
    for r in range(8):
        assert not isinstance(eight[r], str), eight[r]
        assert (eight[r]["local_heads"], eight[r]["local_kv_heads"], eight[r]["local_ffn"]) == (4, 1, 1792)
        assert eight[r]["xgmi_error"] == 0
    h = {r: torch.tensor(eight[r]["sample"]) for r in range(8)}
    for r in range(1, 8):
        assert torch.equal(h[0], h[r]), f"rank {r} differs from rank 0"
    ref = torch.tensor(one["ref_sample"])
    bound = parity_bound(one["eager_vs_fp32"])
    assert one["hip_vs_fp32"] <= bound, (one["hip_vs_fp32"], bound)
    err8 = float((h[0] - ref).abs().max() / ref.abs().max())
    assert err8 <= bound, (err8, bound)


def _rccl_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import warnings

    import torch

    from ray_dynamic_batching_amd.parallel import collective as col
    from ray_dynamic_batching_amd.parallel import xgmi as xgmi_mod

    torch.cuda.set_device(0)
    out = {}
    try:
        col.init_collective_group(1, 0, backend="nccl", group_name="g")
        assert col.get_group_handle("g") is not None and col.get_collective_group_size("g") == 1
        x = torch.arange(12, device="cuda", dtype=torch.float32)
        out["allreduce_sum"] = col.allreduce(x.clone(), "g").tolist() == x.tolist()
        out["allreduce_max"] = col.allreduce(x.clone(), "g", col.ReduceOp.MAX).tolist() == x.tolist()
        out["reduce"] = col.reduce(x.clone(), 0, "g").tolist() == x.tolist()
        out["broadcast"] = col.broadcast(x.clone(), 0, "g").tolist() == x.tolist()
        lst = [torch.empty_like(x)]
        col.allgather(lst, x, "g")
        out["allgather"] = lst[0].tolist() == x.tolist()
        big = torch.empty(12, device="cuda")
        out["allgather_into"] = col.allgather_into(big, x, "g").tolist() == x.tolist()
        rs = torch.empty_like(x)
        out["reducescatter"] = col.reducescatter(rs, [x.clone()], "g").tolist() == x.tolist()
        col.barrier("g")
        out["barrier"] = True
        col.synchronize()
        # the custom xGMI all-reduce at world 1, then every fallback to RCCL
        xg = col.enable_xgmi("g", max_elems=1 << 12, timeout_s=10.0)
        out["xgmi_enabled"] = xg is not None
        calls0 = xg.calls
        b = torch.randn(64, 64, device="cuda").to(torch.bfloat16)
        out["xgmi_path"] = torch.equal(col.allreduce(b.clone(), "g"), b) and xg.calls == calls0 + 1
        over = torch.randn(128, 64, device="cuda").to(torch.bfloat16)          # 8192 > max_elems
        out["fallback_size"] = torch.equal(col.allreduce(over.clone(), "g"), over) and xg.calls == calls0 + 1
        odd = torch.randn(7 * 3, device="cuda").to(torch.bfloat16)             # no row split the kernel takes
        out["fallback_shape"] = torch.equal(col.allreduce(odd.clone(), "g"), odd) and xg.calls == calls0 + 1
        out["fallback_op"] = (torch.equal(col.allreduce(b.clone(), "g", col.ReduceOp.MAX), b)
                              and xg.calls == calls0 + 1)
        col.destroy_collective_group("g")
        # enable_xgmi failing (no IPC on the platform) leaves RCCL in use
        col.init_collective_group(1, 0, backend="nccl", group_name="h")
        real = xgmi_mod.XgmiCommunicator.create

        def boom(*a, **k):
            raise RuntimeError("no IPC here")

        xgmi_mod.XgmiCommunicator.create = boom
        try:
            with warnings.catch_warnings(record=True) as w:
                warnings.simplefilter("always")
                out["enable_failed_none"] = col.enable_xgmi("h") is None and any("RCCL" in str(m.message) for m in w)
        finally:
            xgmi_mod.XgmiCommunicator.create = real
        out["rccl_after_failed_enable"] = torch.equal(col.allreduce(b.clone(), "h"), b)
        col.destroy_collective_group("h")
        q.put((rank, out))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise


def test_rccl_backend_world1_every_op_and_xgmi_fallbacks():
    got = _spawn(_rccl_worker, 1)[0]
    assert not isinstance(got, str), got
    bad = [k for k, v in got.items() if not v]
    assert not bad, got
