"""Metrics export: the fork's metrics.json file contract (scheduler.py:933-983,
read by metrics_display.py) and Prometheus text exposition with Serve-compatible
metric names (replica.py:122-154, router.py:357-377).  Counters and latency
histograms live in the shm job segment; this module only reads them."""
from __future__ import annotations

import json
import os
import threading
import time
from typing import Callable, Dict, Optional


class MetricsFileWriter:
    """Writes ``stats_fn()`` to a JSON file every ``interval`` seconds (atomic replace)."""

    def __init__(self, stats_fn: Callable[[], Dict], path: str = "metrics.json", interval: float = 1.0):
        self.stats_fn = stats_fn
        self.path = path
        self.interval = interval
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None

    def write_once(self) -> None:
        data = self.stats_fn()
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(data, f, default=float)
        os.replace(tmp, self.path)

    def start(self) -> "MetricsFileWriter":
        def loop():
            while not self._stop.is_set():
                try:
                    self.write_once()
                except Exception:  # pragma: no cover
                    pass
                self._stop.wait(self.interval)
        self._t = threading.Thread(target=loop, daemon=True, name="metrics-writer")
        self._t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._t:
            self._t.join(2)


def prometheus_text(job, deployments: Dict[int, str], queue_map: Dict[int, int]) -> str:
    """Render shm counters as Prometheus text.  deployments: model id -> name;
    queue_map: queue id -> replica index."""
    lines = []

    def metric(name, typ, help_):
        lines.append(f"# HELP {name} {help_}")
        lines.append(f"# TYPE {name} {typ}")

    metric("serve_deployment_request_counter", "counter", "Requests completed by a replica")
    metric("serve_deployment_error_counter", "counter", "Requests that failed in a replica")
    metric("serve_replica_processing_queries", "gauge", "Requests queued or executing at a replica")
    metric("serve_deployment_processing_latency_ms", "summary", "End-to-end request latency (ms)")
    metric("rdb_dropped_stale_total", "counter", "Requests dropped because their SLO deadline was unreachable")
    metric("rdb_slo_violations_total", "counter", "Requests completed after their SLO")
    for q, r in queue_map.items():
        st = job.queue_stats(q)
        dep = deployments.get(st["model"], str(st["model"]))
        lab = f'deployment="{dep}",replica="{r}",queue="{q}"'
        lines.append(f"serve_deployment_request_counter{{{lab}}} {st['completed']}")
        lines.append(f"serve_deployment_error_counter{{{lab}}} {st['errors']}")
        lines.append(f"serve_replica_processing_queries{{{lab}}} {st['depth']}")
        for p in ("p50", "p90", "p95", "p99"):
            lines.append(f'serve_deployment_processing_latency_ms{{{lab},quantile="0.{p[1:]}"}} {st["e2e"][p + "_ms"]:.4f}')
        lines.append(f"serve_deployment_processing_latency_ms_count{{{lab}}} {st['e2e']['count']}")
        lines.append(f"rdb_dropped_stale_total{{{lab}}} {st['dropped']}")
        lines.append(f"rdb_slo_violations_total{{{lab}}} {st['slo_violations']}")
    return "\n".join(lines) + "\n"


def serve_prometheus(text_fn: Callable[[], str], port: int = 9464):  # pragma: no cover - network
    """Minimal /metrics endpoint on a daemon thread."""
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    class H(BaseHTTPRequestHandler):
        def do_GET(self):
            body = text_fn().encode()
            self.send_response(200)
            self.send_header("Content-Type", "text/plain; version=0.0.4")
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = ThreadingHTTPServer(("127.0.0.1", port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv
