"""Chrome-trace export of the per-replica shm trace rings (the
counterpart of ``ray timeline``, _private/profiling.py:84-124).

Every replica engine records, per batch, three spans into its ring in the job
segment (runtime/csrc/shm.h TraceRing): batch formation (launcher thread),
GPU execution (hipEvent-timed graph replay, mapped onto the host clock) and
completion fan-out (completer thread).  The same phases are also emitted as
roctx ranges ("rdb:form_batch", "rdb:launch", "rdb:complete") for
``rocprofv3 --marker-trace``.

    from ray_dynamic_batching_amd.utils.tracing import export_chrome_trace
    export_chrome_trace(job, "trace.json")      # open in chrome://tracing / Perfetto
"""
from __future__ import annotations

import json
from typing import Dict, Iterable, List, Optional

KIND_NAMES = {1: "form_batch", 2: "gpu", 3: "complete", 4: "drop", 5: "py_batch"}
KIND_TID = {1: 1, 2: 2, 3: 3, 4: 1, 5: 1}
TID_NAMES = {1: "launcher", 2: "gpu", 3: "completer"}


def collect(job, replicas: Optional[Iterable[int]] = None) -> List[Dict]:
    n = job.info()["n_replicas"]
    out = []
    for r in (replicas if replicas is not None else range(n)):
        for kind, t0, t1, q, nb, bucket in job.trace_events(r):
            out.append(dict(replica=r, kind=KIND_NAMES.get(kind, str(kind)), kind_id=kind, t0_ns=t0, t1_ns=t1,
                            queue=q, n=nb, bucket=bucket))
    out.sort(key=lambda e: e["t0_ns"])
    return out


def chrome_trace(events: List[Dict]) -> Dict:
    tev = []
    t_base = min((e["t0_ns"] for e in events), default=0)
    reps = sorted({e["replica"] for e in events})
    for r in reps:
        tev.append(dict(name="process_name", ph="M", pid=r, args=dict(name=f"replica {r}")))
        for tid, nm in TID_NAMES.items():
            tev.append(dict(name="thread_name", ph="M", pid=r, tid=tid, args=dict(name=nm)))
    for e in events:
        tev.append(dict(name=f"{e['kind']} q{e['queue']} n={e['n']}", cat=e["kind"], ph="X", pid=e["replica"],
                        tid=KIND_TID.get(e["kind_id"], 1), ts=(e["t0_ns"] - t_base) / 1e3,
                        dur=max(0.0, (e["t1_ns"] - e["t0_ns"]) / 1e3),
                        args=dict(queue=e["queue"], batch=e["n"], bucket=e["bucket"])))
    return {"traceEvents": tev, "displayTimeUnit": "ms"}


def export_chrome_trace(job, path: str, replicas: Optional[Iterable[int]] = None) -> Dict:
    tr = chrome_trace(collect(job, replicas))
    with open(path, "w") as f:
        json.dump(tr, f)
    return tr


def summarize(events: List[Dict]) -> Dict[str, Dict[str, float]]:
    """Mean/max duration (us) and count per span kind."""
    agg: Dict[str, List[float]] = {}
    for e in events:
        agg.setdefault(e["kind"], []).append((e["t1_ns"] - e["t0_ns"]) / 1e3)
    return {k: dict(count=len(v), mean_us=sum(v) / len(v), max_us=max(v)) for k, v in agg.items()}
