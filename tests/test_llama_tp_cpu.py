"""Tensor-parallel Llama on CPU: TP=2 (gloo, 2 processes) == TP=1."""
import os
import socket

import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from ray_dynamic_batching_amd.models.llama import LlamaConfig, LlamaTP
    from ray_dynamic_batching_amd.parallel import collective as col

    if world > 1:
        col.init_collective_group(world, rank, backend="gloo", group_name="tp")
    cfg = LlamaConfig.tiny()
    m = LlamaTP(cfg, rank, world, group_name="tp", device="cpu", dtype=torch.float32, backend="torch", init="full")
    ids = m.example_input(3, seed=5)
    out = m.forward(ids)
    x = m.hidden_states(ids)
    q.put((rank, out.tolist(), x[:4, :8].tolist()))
    if world > 1:
        col.destroy_collective_group("tp")


def test_tp2_matches_tp1():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p1 = ctx.Process(target=_run, args=(0, 1, _port(), q))
    p1.start()
    _, ref, xref = q.get(timeout=300)
    p1.join(60)
    port = _port()
    ps = [ctx.Process(target=_run, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (o, x)) for r, o, x in (q.get(timeout=300) for _ in range(2)))
    for p in ps:
        p.join(60)
    for r in range(2):
        toks = [row[0] for row in res[r][0]]
        assert toks == [row[0] for row in ref]
        assert torch.allclose(torch.tensor(res[r][1]), torch.tensor(xref), atol=1e-4)
