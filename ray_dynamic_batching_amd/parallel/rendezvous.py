"""Rendezvous of a tensor-parallel replica's ranks through the node agent's KV.

The node agent gang-spawns the ranks of one TP replica (``spawn_group``) with
``RDB_TP_RANK / RDB_TP_WORLD / RDB_TP_GROUP / RDB_TP_EPOCH`` and
``RDB_AGENT_SOCKET`` in their environment.  Rank 0 starts the torch.distributed
store (a TCPStore on an ephemeral 127.0.0.1 port) and publishes its address
under ``tp/<group>/<epoch>/store`` in the agent's KV; the other ranks read it
from there, so no torchrun / MASTER_PORT is involved and a restarted group (new
epoch; the agent deletes the old epoch's keys) never meets a stale address.
RCCL's unique id is then exchanged through that store by
``init_process_group``.  Reference: the NCCL unique id is published through a
detached named actor (python/ray/util/collective/collective_group/
nccl_collective_group.py:555-577).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from datetime import timedelta
from typing import Optional


@dataclass
class TPEnv:
    rank: int
    world: int
    group: str
    epoch: int
    socket: str

    @classmethod
    def from_env(cls) -> Optional["TPEnv"]:
        if "RDB_TP_RANK" not in os.environ:
            return None
        return cls(int(os.environ["RDB_TP_RANK"]), int(os.environ["RDB_TP_WORLD"]), os.environ["RDB_TP_GROUP"],
                   int(os.environ.get("RDB_TP_EPOCH", "0")), os.environ.get("RDB_AGENT_SOCKET", ""))

    @property
    def key(self) -> str:
        return f"tp/{self.group}/{self.epoch}/store"


def _kv_put(sock: str, key: str, value: str) -> None:
    from ..runtime import agent

    r = agent.request(sock, f"KV_PUT {key} {value}")
    if not r.startswith("OK"):
        raise RuntimeError(f"agent KV_PUT {key} failed: {r}")


def _kv_get(sock: str, key: str) -> Optional[str]:
    from ..runtime import agent

    r = agent.request(sock, f"KV_GET {key}")
    return r[3:] if r.startswith("OK ") else None


def agent_store(env: TPEnv, timeout_s: float = 120.0):
    """The group's torch.distributed TCPStore, located through the agent KV."""
    import torch.distributed as dist

    if not env.socket:
        raise RuntimeError("TP rendezvous needs RDB_AGENT_SOCKET (the node agent's control socket)")
    to = timedelta(seconds=timeout_s)
    if env.rank == 0:
        store = dist.TCPStore("127.0.0.1", 0, env.world, is_master=True, timeout=to, wait_for_workers=False)
        _kv_put(env.socket, env.key, f"127.0.0.1:{store.port}")
        return store
    deadline = time.monotonic() + timeout_s
    while True:
        v = _kv_get(env.socket, env.key)
        if v:
            host, port = v.rsplit(":", 1)
            return dist.TCPStore(host, int(port), env.world, is_master=False, timeout=to)
        if time.monotonic() > deadline:
            raise TimeoutError(f"rank {env.rank}: no store address under {env.key} after {timeout_s}s")
        time.sleep(0.02)


def init_tp_group(backend: str, group_name: str = "tp", env: Optional[TPEnv] = None,
                  timeout_s: float = 120.0) -> TPEnv:
    """Join this process's TP group (``parallel.collective`` group ``group_name``)."""
    from . import collective as col

    env = env or TPEnv.from_env()
    if env is None:
        raise RuntimeError("not a tensor-parallel rank (RDB_TP_RANK unset)")
    store = agent_store(env, timeout_s)
    col.init_collective_group(env.world, env.rank, backend, group_name, store=store)
    return env
