"""NUMA / CPU placement of the per-GPU replica processes.

On a two-socket MI355X node four GPUs hang off each socket.  A replica rank's
hot host threads -- the engine launcher's spin, the completer, the load
generator -- and the request arena its GPU gathers payloads from belong on the
socket of that GPU; otherwise every payload crosses the socket link and the
threads share cores with another rank's.  This module:

* reads each GPU's locality from sysfs: ``/sys/bus/pci/devices/<bdf>/numa_node``
  and ``local_cpulist`` (with ``/sys/devices/system/node/node<N>/cpulist`` as
  the fallback) -- the GPU's PCI address comes from the KFD topology (no HIP
  initialisation needed, so a rank pins itself before the runtime starts any
  thread), or from the HIP device properties when that is missing;
* plans one CPU set per rank: ranks on the same NUMA node split that node's
  allowed CPUs into equal contiguous chunks, so every rank gets its own cores
  (:func:`plan_cpu_sets`, a pure function the tests drive with a fake sysfs);
* pins the calling process (:func:`pin_process`) before it starts any native
  thread, so every thread it creates inherits the mask.

The request arena is bound by the native runtime (``Job.init_req_ring(q,
numa_node)``: mbind + first touch by the pinned consumer).  Everything degrades
to "no pinning" when the sysfs entries are missing (containers, CPU hosts).
Reference: the raylet pins accelerators per worker before a task runs
(python/ray/_raylet.pyx:2093-2098); SURVEY §2.4, node_agent row.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Sequence, Tuple


def parse_cpulist(s: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in s.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def format_cpulist(cpus: Iterable[int]) -> str:
    cpus = sorted(set(cpus))
    runs, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        runs.append(f"{cpus[i]}" if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(runs)


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def pci_locality(bdf: str, sysfs: str = "/sys") -> Tuple[int, List[int]]:
    """(numa node or -1, local CPUs or []) of the PCI device ``bdf``
    ('0000:75:00.0')."""
    dev = os.path.join(sysfs, "bus", "pci", "devices", bdf)
    node_s = _read(os.path.join(dev, "numa_node"))
    node = int(node_s) if node_s not in (None, "") else -1
    cpus_s = _read(os.path.join(dev, "local_cpulist"))
    cpus = parse_cpulist(cpus_s) if cpus_s else []
    if not cpus and node >= 0:
        s = _read(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist"))
        cpus = parse_cpulist(s) if s else []
    return node, cpus


def gpu_pci_addresses() -> List[str]:
    """PCI addresses of the visible HIP devices, in device order ([] if unknown)."""
    try:
        import torch

        out = []
        for i in range(torch.cuda.device_count()):
            p = torch.cuda.get_device_properties(i)
            dom = getattr(p, "pci_domain_id", 0)
            bus = getattr(p, "pci_bus_id", None)
            dv = getattr(p, "pci_device_id", None)
            if bus is None or dv is None:
                return []
            out.append(f"{dom:04x}:{bus:02x}:{dv:02x}.0")
        return out
    except Exception:  # pragma: no cover - no HIP runtime
        return []


def kfd_gpu_pci_addresses(sysfs: str = "/sys", respect_visible: bool = True) -> List[str]:
    """PCI addresses of the GPUs in HIP device order WITHOUT initialising HIP
    (so a rank can pin itself before the runtime starts any thread): the KFD
    topology nodes that have SIMDs, in node order (the order ROCr enumerates
    agents), filtered by ROCR_VISIBLE_DEVICES then HIP_VISIBLE_DEVICES (unless
    ``respect_visible`` is False: the node agent plans over every GPU)."""
    root = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        nodes = sorted(int(n) for n in os.listdir(root) if n.isdigit())
    except OSError:
        return []
    gpus = []
    for n in nodes:
        props = _read(os.path.join(root, str(n), "properties")) or ""
        kv = dict(line.split(None, 1) for line in props.splitlines() if len(line.split(None, 1)) == 2)
        if int(kv.get("simd_count", "0")) <= 0:
            continue
        loc = int(kv.get("location_id", "0"))
        dom = int(kv.get("domain", "0"))
        gpus.append(f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7}")
    for var in (("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES") if respect_visible else ()):
        v = os.environ.get(var)
        if v:
            try:
                gpus = [gpus[int(i)] for i in v.split(",") if i.strip() != "" and int(i) < len(gpus)]
            except ValueError:   # UUID-style selectors: order unknown
                return []
    return gpus


def plan_cpu_sets(rank_gpus: Sequence[int], locality: Dict[int, Tuple[int, List[int]]],
                  allowed: Optional[Iterable[int]] = None) -> List[List[int]]:
    """One CPU set per rank.  ``rank_gpus[r]`` is rank r's GPU; ``locality[gpu]``
    = (numa node, local CPUs).  Ranks whose GPUs sit on the same node share that
    node's allowed CPUs in equal contiguous chunks (rank order), so each rank
    gets distinct cores; a rank whose GPU's locality is unknown gets [] (no
    pinning).  Chunks are never empty: with more ranks than CPUs on a node the
    node's CPUs are reused round-robin."""
    allow = set(allowed) if allowed is not None else None
    by_node: Dict[int, List[int]] = {}
    node_cpus: Dict[int, List[int]] = {}
    for r, g in enumerate(rank_gpus):
        node, cpus = locality.get(g, (-1, []))
        if allow is not None:
            cpus = [c for c in cpus if c in allow]
        if not cpus:
            continue
        key = node if node >= 0 else -(g + 2)          # unknown node: group by GPU
        by_node.setdefault(key, []).append(r)
        node_cpus[key] = cpus
    out: List[List[int]] = [[] for _ in rank_gpus]
    for key, ranks in by_node.items():
        cpus = node_cpus[key]
        k = len(ranks)
        if len(cpus) >= k:
            per, extra = divmod(len(cpus), k)
            start = 0
            for i, r in enumerate(ranks):
                n = per + (1 if i < extra else 0)
                out[r] = cpus[start:start + n]
                start += n
        else:
            for i, r in enumerate(ranks):
                out[r] = [cpus[i % len(cpus)]]
    return out


def gpu_locality_map(sysfs: str = "/sys", pci: Optional[List[str]] = None) -> Dict[int, Tuple[int, List[int]]]:
    pci = gpu_pci_addresses() if pci is None else pci
    return {i: pci_locality(a, sysfs) for i, a in enumerate(pci)}


def pin_process(cpus: Sequence[int]) -> bool:
    """Pin this process (and every thread it starts afterwards) to ``cpus``."""
    if not cpus or not hasattr(os, "sched_setaffinity"):
        return False
    try:
        os.sched_setaffinity(0, set(cpus))
        return True
    except OSError:
        return False


def place_rank(rank: int, rank_gpus: Sequence[int], sysfs: str = "/sys",
               pci: Optional[List[str]] = None) -> dict:
    """Plan every rank's CPU set, pin this rank's process to its own and return
    {numa_node, cpus (cpulist string), pinned} for logging.  Set
    RDB_NUMA_PIN=0 to skip."""
    if os.environ.get("RDB_NUMA_PIN", "1") == "0":
        return dict(numa_node=-1, cpus="", pinned=False)
    if pci is None:
        pci = kfd_gpu_pci_addresses(sysfs) or gpu_pci_addresses()
    loc = gpu_locality_map(sysfs, pci)
    allowed = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    sets = plan_cpu_sets(rank_gpus, loc, allowed)
    mine = sets[rank] if rank < len(sets) else []
    node = loc.get(rank_gpus[rank], (-1, []))[0] if rank < len(rank_gpus) else -1
    pinned = pin_process(mine)
    return dict(numa_node=node, cpus=format_cpulist(mine), pinned=pinned)


def gpu_placement(gpu: int, sysfs: str = "/sys", pci: Optional[List[str]] = None) -> dict:
    """Placement of a Serve replica on physical GPU ``gpu``, planned by the
    controller / node agent (which see every GPU of the node, not a replica's
    HIP_VISIBLE_DEVICES view): {numa_node, cpus (list), cpulist}.  The CPU sets
    are :func:`plan_cpu_sets` with one rank per GPU, so replicas of GPUs on one
    NUMA node get disjoint cores -- the same split ``bench.py``'s ranks use.  The
    agent applies the set to the replica process at spawn (inherited by every
    thread it starts) and the controller binds the replica's request ring to
    ``numa_node``.  RDB_NUMA_PIN=0 disables it (numa_node -1, no CPUs)."""
    if os.environ.get("RDB_NUMA_PIN", "1") == "0" or gpu < 0:
        return dict(numa_node=-1, cpus=[], cpulist="")
    if pci is None:
        pci = kfd_gpu_pci_addresses(sysfs, respect_visible=False)
    if gpu >= len(pci):
        return dict(numa_node=-1, cpus=[], cpulist="")
    loc = gpu_locality_map(sysfs, pci)
    allowed = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    sets = plan_cpu_sets(list(range(len(pci))), loc, allowed)
    return dict(numa_node=loc.get(gpu, (-1, []))[0], cpus=list(sets[gpu]), cpulist=format_cpulist(sets[gpu]))
