"""Batch-profile CSV contract (reference: ModelProfiler.py:350-366 writer,
scheduler.py:88-113 BatchProfiler reader).

Columns: batch_size,status,avg_latency_ms,std_latency_ms,throughput,
throughput_efficiency,peak_memory_mb,memory_per_sample_mb,memory_utilization
(failed rows carry only batch_size,status).  The planner reads avg_latency_ms
and peak_memory_mb of the successful rows.
"""
from __future__ import annotations

import csv
import os
from typing import Dict, Iterable, List

CSV_FIELDS = ["batch_size", "status", "avg_latency_ms", "std_latency_ms", "throughput", "throughput_efficiency",
              "peak_memory_mb", "memory_per_sample_mb", "memory_utilization"]
PLANNER_FIELDS = ("avg_latency_ms", "peak_memory_mb")


def load_profile_csv(path: str, fields: Iterable[str] = PLANNER_FIELDS) -> Dict[int, Dict[str, float]]:
    out: Dict[int, Dict[str, float]] = {}
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            if row.get("status", "success") not in ("success", ""):
                continue
            try:
                out[int(row["batch_size"])] = {k: float(row[k]) for k in fields}
            except (KeyError, ValueError):
                continue
    return out


def load_profiles(mapping: Dict[str, str], base_dir: str = "") -> Dict[str, Dict[int, Dict[str, float]]]:
    return {m: load_profile_csv(os.path.join(base_dir, p)) for m, p in mapping.items()}


def write_profile_csv(path: str, results: List[dict]) -> None:
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=CSV_FIELDS)
        w.writeheader()
        for r in results:
            if r.get("status") == "success":
                w.writerow({k: r.get(k) for k in CSV_FIELDS})
            else:
                w.writerow({"batch_size": r["batch_size"], "status": r.get("status", "error")})


def synthetic_profile(base_ms: float, per_item_ms: float, mem_base_mb: float, mem_per_item_mb: float,
                      batches=(1, 2, 4, 8, 16)) -> Dict[int, Dict[str, float]]:
    """Linear latency/memory model (the fork's SAMPLE_BATCH_PROFILE style)."""
    return {b: {"avg_latency_ms": base_ms + per_item_ms * b, "peak_memory_mb": mem_base_mb + mem_per_item_mb * b}
            for b in batches}
