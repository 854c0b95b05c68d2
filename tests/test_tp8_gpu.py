"""The TP=8 path at world 4 / 8 on the one GPU a box has: every rank is its own
process (spawned, HIP IPC over gloo -- the exact code of a real TP group minus
the xGMI link), so the 8-rank per-block barrier and epoch logic, the two-shot
chunking at world 8, LlamaTP sharding at TP=8 and TPReplica's rank-0 broadcast
header protocol all run before an 8-GPU node exists.

Reference collective surface: python/ray/util/collective/collective.py:258-655,
NCCL group at collective_group/nccl_collective_group.py:175-400.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

_Q_TIMEOUT = 300          # first `import torch` in 8 fresh processes can take a while on a cold box


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


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
    return s, h, acc


def _digest(t):
    import hashlib

    return hashlib.sha1(t.contiguous().view(torch.int16).cpu().numpy().tobytes()).hexdigest()


def _log(rank, msg):
    """Progress to stderr (visible with -s; keeps long multi-process GPU runs observably alive)."""
    import sys
    import time

    print(f"[tp8 rank {rank} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


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


def _allreduce_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch

    from ray_dynamic_batching_amd.parallel import collective as col

    torch.cuda.set_device(0)
    col.init_collective_group(world, rank, backend="gloo", group_name="tp")
    _log(rank, "allreduce worker ready")
    res = []
    try:
        xg = col.enable_xgmi("tp", max_elems=1 << 21, timeout_s=20.0)
        eps = 1e-5
        # (T, D, two_shot): one-shot small, two-shot with rows not divisible by world
        for T, D, two in [(8, 4096, False), (37, 2048, True), (512, 2048, True)]:
            # eager, then captured + replayed x3 with fresh inputs in the captured buffers
            xs, gamma = _inputs(world, T, D, seed=T)
            x = xs[rank].cuda()
            g = gamma.cuda()
            s, h = xg.all_reduce_rmsnorm(x, g, eps, two_shot=two)
            torch.cuda.synchronize()
            ref_s, ref_h, acc = _reference(xs, gamma, eps)
            res.append(("eager", T, D, two, xg.error(), _digest(s), torch.equal(s.cpu(), ref_s),
                        float((h.cpu().float() - ref_h.float()).abs().max()),
                        float((s.cpu().float() - acc).abs().max() / (acc.abs().max() + 1e-6))))
            graph = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                with torch.cuda.graph(graph, stream=st):
                    gs, gh = xg.all_reduce_rmsnorm(x, g, eps, two_shot=two)
                    gs = gs.clone()       # the sum is a view of the gather buffer: the next call reuses it
                    gsum = xg.all_reduce(gh, two_shot=two)      # a second call in the same graph
            torch.cuda.synchronize()
            for it in range(3):
                xs, gamma2 = _inputs(world, T, D, seed=1000 * T + it)
                x.copy_(xs[rank].cuda())
                torch.cuda.synchronize()
                col.barrier("tp")
                graph.replay()
                torch.cuda.synchronize()
                ref_s, ref_h, acc = _reference(xs, gamma, eps)
                ref_sum2 = torch.zeros_like(acc)
                for _ in range(world):
                    ref_sum2 = ref_sum2 + ref_h.float()
                res.append(("replay", T, D, two, xg.error(), _digest(gs) + _digest(gsum), torch.equal(gs.cpu(), ref_s),
                            float((gh.cpu().float() - ref_h.float()).abs().max()),
                            float((gsum.cpu().float() - ref_sum2).abs().max() / (ref_sum2.abs().max() + 1e-6))))
            del graph
        q.put((rank, res))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise
    finally:
        col.barrier("tp")
        col.destroy_collective_group("tp")


@pytest.mark.parametrize("world", [4, 8])
def test_xgmi_ipc_world_n_one_gpu(world):
    """All-reduce and all-reduce + RMSNorm at world 4 / 8: bit-exact across
    ranks, sums equal to the fp32 sum rounded to bf16 (the kernel adds in rank
    order on every rank), fused norm within bf16 tolerance; one-shot and
    two-shot; eager and under hipGraph replay x3 (epochs in device memory)."""
    got = _spawn(_allreduce_worker, world)
    for r in range(world):
        assert not isinstance(got[r], str), got[r]
    n = len(got[0])
    assert n == 3 * 4
    for i in range(n):
        rows = [got[r][i] for r in range(world)]
        kind, T, D, two = rows[0][:4]
        assert all(row[4] == 0 for row in rows), f"{kind} T={T}: barrier timeout {rows}"
        assert len({row[5] for row in rows}) == 1, f"{kind} T={T} two_shot={two}: ranks differ"
        assert all(row[6] for row in rows), f"{kind} T={T} two_shot={two}: sum != fp32 sum in bf16"
        assert all(row[7] < 3e-2 for row in rows), f"{kind} T={T}: norm error {[row[7] for row in rows]}"
        assert all(row[8] < 1e-2 for row in rows), f"{kind} T={T}: relative error {[row[8] for row in rows]}"


def _tp8_cfg():
    from ray_dynamic_batching_amd.models.llama import LlamaConfig

    return LlamaConfig.tiny(heads=8, kv_heads=8, head_dim=64, hidden=512, intermediate=1024, vocab_size=1024)


def _line_up():
    """Eight TP ranks share ONE GPU here: a rank already spinning in the xGMI
    all-reduce kernel holds wave slots / VGPRs that a peer's 8-wave GEMM needs
    to reach the same all-reduce, so before each all-reduce every rank drains
    its stream and meets the others (gloo).  On an 8-GPU node each rank has its
    own GPU and nothing is lined up."""
    import torch

    from ray_dynamic_batching_amd.parallel import collective as col

    torch.cuda.synchronize()
    col.barrier("tp")


def _llama_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch

    from ray_dynamic_batching_amd.models.llama import LlamaTP
    from ray_dynamic_batching_amd.parallel import collective as col

    torch.cuda.set_device(0)
    import faulthandler

    faulthandler.dump_traceback_later(120, exit=True)     # a stuck rank shows where, then exits
    _log(rank, "started")
    if world > 1:
        col.init_collective_group(world, rank, backend="gloo", group_name="tp")
        col.enable_xgmi("tp", max_elems=1 << 20, timeout_s=20.0)
    _log(rank, "group ready")
    try:
        m = LlamaTP(_tp8_cfg(), rank, world, group_name="tp", device="cuda", backend="hip", init="full")
        if world > 1:
            m.pre_collective = _line_up
        ids = m.example_input(2, seed=3)
        _log(rank, "model built")
        xv = m.hidden_states(ids)
        torch.cuda.synchronize()
        _log(rank, "forward done")
        x = xv.float().cpu()
        err = m._xgmi().error() if world > 1 else 0
        tok = m(ids).cpu()
        q.put((rank, (x[:, :64].tolist(), tok.tolist(), err)))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise
    finally:
        if world > 1:
            col.barrier("tp")
            col.destroy_collective_group("tp")


def test_llama_tp8_matches_tp1():
    """LlamaTP at TP=8 (heads, kv heads, MLP and vocab split 8 ways; xGMI
    all-reduces between them) computes the TP=1 model's hidden states."""
    ref = _spawn(_llama_worker, 1)[0]
    assert not isinstance(ref, str), ref
    got = _spawn(_llama_worker, 8)
    for r in range(8):
        assert not isinstance(got[r], str), got[r]
    assert all(got[r][2] == 0 for r in range(8)), [got[r][2] for r in range(8)]   # no barrier timed out
    h = {r: torch.tensor(got[r][0]) for r in range(8)}
    zero = [r for r in range(8) if not h[r].abs().sum()]
    assert not zero, f"ranks with all-zero hidden states: {zero}"
    for r in range(1, 8):
        assert torch.equal(h[0], h[r])             # every TP rank holds the same x
    href = torch.tensor(ref[0])
    err = (h[0] - href).abs().max().item()
    scale = href.abs().max().item()
    assert err <= 0.05 * scale + 0.05, (err, scale)
    assert all(got[r][1] == got[0][1] for r in range(8))


def _replica_worker(rank, world, port, q, job_name, n_prompts):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch

    from ray_dynamic_batching_amd.models.llama import LlamaTP
    from ray_dynamic_batching_amd.parallel import collective as col
    from ray_dynamic_batching_amd.runtime.tp_replica import TPReplica

    torch.cuda.set_device(0)
    import faulthandler

    faulthandler.dump_traceback_later(240, exit=True)
    _log(rank, "replica worker started")
    col.init_collective_group(world, rank, backend="gloo", group_name="tp")
    col.enable_xgmi("tp", max_elems=1 << 20, timeout_s=20.0)
    try:
        m = LlamaTP(_tp8_cfg(), rank, world, group_name="tp", device="cuda", backend="hip", init="full")
        m.pre_collective = _line_up
        _log(rank, "model built")
        # eager batches (no bucket graphs): a graph replay cannot line the ranks up
        rep = TPReplica(m, job_name if rank == 0 else None, 0, 0, [1, 2, 4, 8], group="tp",
                        use_graphs=False).capture()
        served = 0
        if rank == 0:
            while served < n_prompts:
                served += max(0, rep.step(0.05))
                _log(rank, f"served {served}")
            rep.stop_all()
        else:
            while rep.step(0.05) >= 0:
                pass
        # eager forward of the same prompts on every rank (collective), rank 0 reports it
        ids = m.example_input(n_prompts, seed=11)
        direct = m(ids).cpu().tolist()
        q.put((rank, (rep.batches, served, direct)))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise
    finally:
        col.barrier("tp")
        col.destroy_collective_group("tp")


def _prompts(cfg, n, seed):
    """LlamaTP.example_input's prompts (seeded CPU generator: any process, any rank)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randint(1, cfg.vocab_size, (n, cfg.seq_len), generator=g, dtype=torch.int32)


def test_tp_replica_world8_serves_prompts_through_rings():
    """TPReplica at world 8 over gloo on one GPU: rank 0 pops prompts from the
    shm queue, broadcasts the (bucket, n) header and the ids, all 8 ranks replay
    their shard's graph, rank 0 answers through the completion ring; the
    answers equal the TP=8 model's direct forward of the same prompts."""
    import threading
    import time

    from ray_dynamic_batching_amd.runtime import job as rjob

    n = 16
    cfg = _tp8_cfg()
    name = rjob.unique_job_name("tp8")
    j = rjob.Job(name, create=True, n_replicas=1, n_queues=1, n_clients=2, req_slot_bytes=cfg.seq_len * 4 + 64,
                 cmp_slot_bytes=64)
    j.configure_queue(0, 0, 0, 256, 0.0, True)
    try:
        ids = _prompts(cfg, n, 11)
        c = rjob.Client(j, 1)
        got = {}

        def submit_and_poll():
            rids = {}
            for i in range(n):
                rids[c.submit(0, ids[i].numpy().tobytes())] = i
                time.sleep(0.003)
            t_end = time.time() + _Q_TIMEOUT
            while len(got) < n and time.time() < t_end:
                for rid, st, qq, ts, td, tr, kind, payload in c.poll(64, 100_000_000):
                    got[rids[rid]] = (st, np.frombuffer(payload, dtype=np.int32).tolist())

        t = threading.Thread(target=submit_and_poll)
        t.start()
        out = _spawn(_replica_worker, 8, name, n)
        t.join(60)
        for r in range(8):
            assert not isinstance(out[r], str), out[r]
        batches, served, direct = out[0]
        assert served == n and batches >= 2, (served, batches)
        assert all(out[r][2] == direct for r in range(8))      # every rank computed the same answers
        assert len(got) == n and all(st == 0 for st, _ in got.values()), got
        for i in range(n):
            assert got[i][1] == direct[i], (i, got[i], direct[i])
    finally:
        j.close()
