"""Python face of the native node agent (runtime/csrc/node_agent.cpp).

The agent owns the node's GPU slots (whole-first-fit / fractional best-fit
with an HBM budget), the replica processes (spawn pinned to their GPUs,
exit + heartbeat supervision, fail-pending + generation bump on death,
exponential-back-off restarts), a persistent KV store and a Unix-socket
control endpoint.  One agent per serve controller process.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Sequence

from ..utils.native import load_runtime


def NodeAgent(num_gpus: int, hbm_gb_per_gpu: float = 0.0, kv_path: str = ""):
    return load_runtime().NodeAgent(num_gpus, hbm_gb_per_gpu, kv_path)


def KvStore(path: str):
    return load_runtime().KvStore(path)


def request(sock_path: str, line: str, timeout_s: float = 5.0) -> str:
    """Send one control command (PING, STATUS, KV_GET k, KV_PUT k v, KV_KEYS p, CONFIG name)."""
    return load_runtime().agent_request(sock_path, line, timeout_s)


def status(sock_path: str) -> Dict:
    return json.loads(request(sock_path, "STATUS"))


def default_socket_path() -> str:
    return os.environ.get("RDB_AGENT_SOCKET", f"/tmp/rdb_agent_{os.getuid()}.sock")


def spawn_replica(agent, owner: str, argv: Sequence[str], env: Dict[str, Optional[str]], log_path: str,
                  job: str = "", replica: int = -1, queues: Sequence[int] = (), health_timeout_s: float = 30.0,
                  max_restarts: int = -1, backoff_initial_s: float = 0.5, backoff_max_s: float = 30.0) -> int:
    return agent.spawn(owner, list(argv), dict(env), log_path, job, replica, list(queues), health_timeout_s,
                       max_restarts, backoff_initial_s, backoff_max_s)


__all__: List[str] = ["NodeAgent", "KvStore", "request", "status", "default_socket_path", "spawn_replica"]
