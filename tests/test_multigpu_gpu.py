"""Multi-GPU tier: one process per GPU, gated on ``torch.cuda.device_count()``.

Every ``*_cross_device`` test runs only when the box has at least N devices
(reference: the collective suite's 2-GPU fixture and device-count skips,
python/ray/util/collective/tests/conftest.py:48-52,
single_node_gpu_tests/test_allreduce.py:11).  On a one-GPU box they skip
cleanly, and the SAME per-rank bodies run today as one-GPU rehearsals:
ranks share cuda:0 and meet over gloo (RCCL refuses two ranks on one device)
or run in one process (the native TP leader / follower engines).

What only an N-GPU node exercises: peer IPC mappings between devices,
system-scope flag barriers across the XCDs of different GPUs (the xGMI
all-reduce), RCCL at world > 1, Serve TP replicas with one GPU per rank on the
native engine with graph-captured RCCL all-reduces, and bench.py's N ranks
with distinct NUMA CPU sets.
"""
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_Q_TIMEOUT = 300


def _ndev() -> int:
    try:
        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


def _need(n: int):
    return pytest.mark.skipif(_ndev() < n, reason=f"needs {n} GPUs (this box has {_ndev()})")


def _port() -> int:
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


# --------------------------------------------------------------------------
# per-rank bodies (shared by the N-GPU tests and the one-GPU rehearsals)
# --------------------------------------------------------------------------
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
    return s, (sf * torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + eps) * gamma.float()).to(torch.bfloat16)


def _xgmi_body(rank, world, port, q, one_gpu, shapes):
    """xGMI one- / two-shot all-reduce + fused residual RMSNorm, eager and under
    graph replay: every rank's sum bit-identical (digest) and equal to the fp32
    sum rounded to bf16."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import hashlib

    from ray_dynamic_batching_amd.parallel import collective as col

    def digest(t):
        return hashlib.sha1(t.contiguous().view(torch.int16).cpu().numpy().tobytes()).hexdigest()

    torch.set_num_threads(2)
    torch.cuda.set_device(0 if one_gpu else rank)
    col.init_collective_group(world, rank, backend="gloo" if one_gpu else "nccl", group_name="tp")
    res = []
    try:
        xg = col.enable_xgmi("tp", max_elems=1 << 22, one_shot_max_bytes=8 << 20, timeout_s=30.0)
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
            for it in range(2):
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


def _check_xgmi(got, world, n_rows):
    for r in range(world):
        assert not isinstance(got[r], str), got[r]
    assert len(got[0]) == n_rows
    for i in range(n_rows):
        rows = [got[r][i] for r in range(world)]
        kind, T, D, two = rows[0][:4]
        assert all(row[4] == 0 for row in rows), f"{kind} T={T}: barrier timeout"
        assert len({row[5] for row in rows}) == 1, f"{kind} T={T} two_shot={two}: ranks differ"
        assert all(row[6] for row in rows), f"{kind} T={T} two_shot={two}: sum != fp32 sum in bf16"
        assert all(row[7] < 3e-2 for row in rows), f"{kind} T={T}: norm error"


def _collective_body(rank, world, port, q, one_gpu):
    """Every parallel.collective op at world N with rank-dependent values."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from ray_dynamic_batching_amd.parallel import collective as col

    torch.set_num_threads(2)
    dev = "cpu" if one_gpu else f"cuda:{rank}"
    if not one_gpu:
        torch.cuda.set_device(rank)
    out = {}
    try:
        col.init_collective_group(world, rank, backend="gloo" if one_gpu else "nccl", group_name="c")
        x = torch.arange(8, dtype=torch.float32, device=dev) + 100 * rank
        base = torch.arange(8, dtype=torch.float32)
        s = sum(base + 100 * r for r in range(world))
        out["allreduce_sum"] = torch.equal(col.allreduce(x.clone(), "c").cpu(), s)
        out["allreduce_max"] = torch.equal(col.allreduce(x.clone(), "c", col.ReduceOp.MAX).cpu(),
                                           base + 100 * (world - 1))
        red = col.reduce(x.clone(), 0, "c").cpu()
        out["reduce"] = torch.equal(red, s) if rank == 0 else True
        out["broadcast"] = torch.equal(col.broadcast(x.clone(), world - 1, "c").cpu(), base + 100 * (world - 1))
        lst = [torch.empty_like(x) for _ in range(world)]
        col.allgather(lst, x, "c")
        out["allgather"] = all(torch.equal(lst[r].cpu(), base + 100 * r) for r in range(world))
        big = torch.empty(8 * world, device=dev)
        out["allgather_into"] = torch.equal(col.allgather_into(big, x, "c").cpu(),
                                            torch.cat([base + 100 * r for r in range(world)]))
        parts = [torch.full((4,), float(rank + 10 * j), device=dev) for j in range(world)]
        rs = torch.empty(4, device=dev)
        col.reducescatter(rs, parts, "c")
        out["reducescatter"] = torch.equal(rs.cpu(), torch.full((4,), float(sum(range(world)) + 10 * rank * world)))
        if world >= 2:
            t = torch.full((3,), float(rank), device=dev)
            if rank == 0:
                col.send(t, 1, "c")
                out["send"] = True
            elif rank == 1:
                got = col.recv(torch.empty(3, device=dev), 0, "c")
                out["recv"] = torch.equal(got.cpu(), torch.zeros(3))
        col.barrier("c")
        out["barrier"] = True
        col.destroy_collective_group("c")
        q.put((rank, out))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise


def _check_collective(got, world):
    for r in range(world):
        assert not isinstance(got[r], str), got[r]
        bad = [k for k, v in got[r].items() if not v]
        assert not bad, (r, got[r])


# --------------------------------------------------------------------------
# N-GPU tests (skip below N devices)
# --------------------------------------------------------------------------
@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_allreduce_cross_device(world):
    if _ndev() < world:
        pytest.skip(f"needs {world} GPUs (this box has {_ndev()})")
    shapes = [(1024, 4096, False), (1024, 4096, True), (1000, 4096, True)]   # 8 MiB Llama-3-8B prefill message
    _check_xgmi(_spawn(_xgmi_body, world, False, shapes), world, 3 * len(shapes))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_every_collective_cross_device(world):
    if _ndev() < world:
        pytest.skip(f"needs {world} GPUs (this box has {_ndev()})")
    _check_collective(_spawn(_collective_body, world, False), world)


@pytest.mark.parametrize("world", [2, 8])
def test_serve_tp_native_rccl_cross_device(world):
    """tp_echo and tiny Llama at TP = N through serve.run, one GPU per rank,
    default RCCL backend, native leader / follower engines with the all-reduces
    captured in the bucket graphs; checked against TP = 1."""
    if _ndev() < world:
        pytest.skip(f"needs {world} GPUs (this box has {_ndev()})")
    from ray_dynamic_batching_amd import serve
    from ray_dynamic_batching_amd.models import factories
    from ray_dynamic_batching_amd.models.tp_echo import TPEcho
    from ray_dynamic_batching_amd.serve.controller import get_controller

    try:
        app = serve.model_deployment(factories.tp_echo(d=16), "tpecho", max_batch_size=4, batch_wait_timeout_s=0.002,
                                     tensor_parallel_size=world, placement_group_bundles=[{"GPU": 1}] * world,
                                     health_check_timeout_s=120)
        h = serve.run(app.bind(), name="echo", mode="process")
        rng = np.random.default_rng(world)
        xs = [rng.standard_normal(16).astype(np.float32) for _ in range(16)]
        w = TPEcho(16, 8).w_full.numpy()
        for x, o in zip(xs, [h.remote(x) for x in xs]):
            y = o.result(timeout_s=120)
            np.testing.assert_allclose(y[:8], x @ w.T, rtol=1e-3, atol=1e-3)
            assert y[8] == world
        c = get_controller()
        info = c.agent.group_info(c.apps["echo"]["tpecho"].proc_replicas[0].group_id)
        assert info["restarts"] == 0 and len(info["members"]) == world
        ovr = dict(heads=8, kv_heads=8, head_dim=64, hidden=512, intermediate=1024, vocab_size=1024, layers=2)
        fac = factories.llama3("tiny", seq_len=32, **ovr)
        ref = fac(device="cuda")
        prompts = [rng.integers(0, 1024, 32, dtype=np.int32) for _ in range(6)]
        with torch.no_grad():
            want = ref(torch.tensor(np.stack(prompts), device="cuda")).cpu().numpy()
        del ref
        torch.cuda.empty_cache()
        app = serve.model_deployment(fac, "llama", max_batch_size=4, batch_wait_timeout_s=0.01,
                                     tensor_parallel_size=world, placement_group_bundles=[{"GPU": 1}] * world,
                                     health_check_timeout_s=120)
        h = serve.run(app.bind(), name="llama", mode="process")
        got = np.stack([h.remote(p).result(timeout_s=120) for p in prompts])
        assert (got[:, 0] == want[:, 0]).all(), (got[:, 0], want[:, 0])
    finally:
        serve.shutdown()


@pytest.mark.parametrize("world", [2, 8])
def test_bench_py_n_gpus_cross_device(world, tmp_path):
    """bench.py --gpus N: every replica serves, every rank pinned to its own CPUs."""
    if _ndev() < world:
        pytest.skip(f"needs {world} GPUs (this box has {_ndev()})")
    out = tmp_path / "b.json"
    r = subprocess.run([sys.executable, os.path.join(_ROOT, "bench.py"), "--gpus", str(world), "--steps", "20",
                        "--warmup", "5", "--json-out", str(out)], capture_output=True, text=True, timeout=800,
                       cwd=_ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(out.read_text())
    assert line["n_gpus"] == world and line["errors"] == 0
    assert len(line["per_replica_requests"]) == world and all(n > 0 for n in line["per_replica_requests"])
    cpus = [p["cpus"] for p in line["placement"] if p.get("pinned")]
    assert len(cpus) == len(set(cpus)), cpus             # distinct CPU sets per rank


# --------------------------------------------------------------------------
# one-GPU rehearsals of the same bodies (run today)
# --------------------------------------------------------------------------
def test_xgmi_body_one_gpu_rehearsal():
    shapes = [(256, 1024, False), (250, 1024, True)]
    _check_xgmi(_spawn(_xgmi_body, 2, True, shapes), 2, 3 * len(shapes))


def test_collective_body_one_gpu_rehearsal():
    _check_collective(_spawn(_collective_body, 2, True), 2)


def test_native_tp_leader_and_follower_one_gpu():
    """The native TP engines in one process on one GPU: a leader serving the
    replica's queue and a follower fed by its broadcast ring, both with a
    collective-free model (no all-reduce to pair up), so the follower must
    replay exactly the leader's batches on exactly the leader's rows."""
    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification
    from ray_dynamic_batching_amd.runtime import job as rjob
    from ray_dynamic_batching_amd.runtime.tp_replica import NativeTP

    cfg = BertConfig.tiny(seq_len=32)
    lead_m = BertForSequenceClassification(cfg, device="cuda", backend="hip")
    foll_m = BertForSequenceClassification(cfg, device="cuda", backend="hip")
    name = rjob.unique_job_name("ntp")
    j = rjob.Job(name, create=True, n_replicas=1, n_queues=1, n_clients=2, req_slot_bytes=32 * 4, cmp_slot_bytes=64)
    j.configure_queue(0, 0, 0, 1024, 0.0, True)
    ring = f"ntp_{os.getpid()}"
    lead = NativeTP(lead_m, name, 0, [1, 2, 4, 8], 0, 2, None, ring, 8, 0.002)
    foll = NativeTP(foll_m, name, 0, [1, 2, 4, 8], 1, 2, None, ring, 8, 0.002)
    lead.unlink()
    lead.start()
    foll.start()
    try:
        c = rjob.Client(j)
        ids = lead_m.example_input(40, seed=5).cpu().numpy()
        rids = [c.submit(0, ids[i].tobytes()) for i in range(40)]
        bad = c.submit(0, b"\x01" * 7)                 # not one model row: answered with an error
        done = {}
        t_end = time.time() + 60
        while len(done) < 41 and time.time() < t_end:
            for comp in c.poll(64, 0.2):
                done[comp[0]] = (comp[1], comp[7])
        assert len(done) == 41
        assert done[bad][0] == 2
        want = lead_m(torch.tensor(ids, device="cuda")).float().cpu().numpy()
        for i, rid in enumerate(rids):
            st, payload = done[rid]
            assert st == 0
            np.testing.assert_allclose(np.frombuffer(payload, np.float32), want[i], atol=5e-2, rtol=5e-2)
        t_end = time.time() + 10
        while foll.stats()["requests"] < 40 and time.time() < t_end:
            time.sleep(0.05)
        ls, fs = lead.stats(), foll.stats()
        assert fs["requests"] == ls["requests"] == 40 and fs["batches"] == ls["batches"], (ls, fs)
        assert lead.check() == "" and foll.check() == ""
    finally:
        lead.stop()                                    # STOP record: the follower leaves its loop
        t_end = time.time() + 10
        while foll.check() == "" and time.time() < t_end:
            time.sleep(0.05)
        assert foll.check() == "stopped"
        foll.stop()
        j.close()
