"""ray.util.collective-style API over gloo with world_size 2 (multi-process, CPU)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from ray_dynamic_batching_amd.parallel import collective as col

    col.init_collective_group(world, rank, backend="gloo", group_name="g")
    out = {}
    t = torch.tensor([float(rank + 1)] * 4)
    col.allreduce(t, "g")
    out["allreduce"] = t.tolist()
    m = torch.tensor([float(rank)])
    col.allreduce(m, "g", col.ReduceOp.MAX)
    out["max"] = m.item()
    b = torch.tensor([rank * 10.0])
    col.broadcast(b, src_rank=1, group_name="g")
    out["bcast"] = b.item()
    lst = [torch.zeros(2) for _ in range(world)]
    col.allgather(lst, torch.tensor([rank, rank + 0.5]), "g")
    out["allgather"] = [x.tolist() for x in lst]
    rs = torch.zeros(2)
    col.reducescatter(rs, [torch.full((2,), float(rank + i)) for i in range(world)], "g")
    out["reducescatter"] = rs.tolist()
    if rank == 0:
        col.send(torch.tensor([42.0]), 1, "g")
    else:
        r = torch.zeros(1)
        col.recv(r, 0, "g")
        out["recv"] = r.item()
    r2 = torch.tensor([float(rank)])
    col.reduce(r2, 0, "g")
    out["reduce"] = r2.item()
    col.barrier("g")
    out["rank"], out["size"] = col.get_rank("g"), col.get_collective_group_size("g")
    q.put((rank, out))
    col.destroy_collective_group("g")


def test_collectives_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(60)
    assert res[0]["allreduce"] == [3.0] * 4 and res[1]["allreduce"] == [3.0] * 4
    assert res[0]["max"] == 1.0
    assert res[0]["bcast"] == 10.0 and res[1]["bcast"] == 10.0
    assert res[0]["allgather"] == [[0.0, 0.5], [1.0, 1.5]]
    assert res[0]["reducescatter"] == [1.0, 1.0] and res[1]["reducescatter"] == [3.0, 3.0]
    assert res[1]["recv"] == 42.0
    assert res[0]["reduce"] == 1.0
    assert res[0]["rank"] == 0 and res[1]["size"] == 2
