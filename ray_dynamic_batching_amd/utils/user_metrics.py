"""Application metrics API with the surface of ``ray.util.metrics``
(reference: python/ray/util/metrics.py:137-313 Counter / Gauge / Histogram,
exported through C++ stats -> OpenCensus -> Prometheus by the metrics agent,
_private/metrics_agent.py:483).

MI355X-native data path: every process keeps a process-local registry (plain
Python objects, no RPC per update); replica processes publish a JSON snapshot
of theirs into the node agent's KV about once a second
(``start_publisher``), and the serve controller renders its own registry, the
replicas' snapshots and the native shm counters (``utils.metrics.prometheus_text``)
as one Prometheus exposition (``serve.metrics_text()`` and the HTTP proxy's
``/-/metrics``).

    from ray_dynamic_batching_amd.utils.user_metrics import Counter, Histogram
    reqs = Counter("my_requests", description="requests seen", tag_keys=("route",))
    reqs.set_default_tags({"route": "/"})
    reqs.inc()
    lat = Histogram("my_latency_ms", boundaries=[1, 5, 10, 50])
    lat.observe(3.2)
"""
from __future__ import annotations

import bisect
import json
import re
import threading
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

_NAME_RE = re.compile(r"^[a-zA-Z_:][a-zA-Z0-9_:]*$")
_lock = threading.Lock()
_registry: Dict[str, "Metric"] = {}


class Metric:
    kind = "untyped"

    def __init__(self, name: str, description: str = "", tag_keys: Optional[Sequence[str]] = None):
        if not name or not _NAME_RE.match(name):
            raise ValueError(f"invalid metric name {name!r}")
        tag_keys = tuple(tag_keys or ())
        if not all(isinstance(k, str) for k in tag_keys):
            raise TypeError("tag_keys must be a tuple of strings")
        self.name, self.description, self.tag_keys = name, description, tag_keys
        self._default: Dict[str, str] = {}
        self._lock = threading.Lock()
        with _lock:
            old = _registry.get(name)
            if old is not None and (old.kind != self.kind or old.tag_keys != tag_keys):
                raise ValueError(f"metric {name!r} already registered with another type or tag keys")
            _registry[name] = self

    def set_default_tags(self, default_tags: Dict[str, str]) -> "Metric":
        unknown = set(default_tags) - set(self.tag_keys)
        if unknown:
            raise ValueError(f"unknown tag keys {sorted(unknown)} for {self.name}")
        self._default = {k: str(v) for k, v in default_tags.items()}
        return self

    def _key(self, tags: Optional[Dict[str, str]]) -> Tuple[str, ...]:
        merged = dict(self._default)
        if tags:
            unknown = set(tags) - set(self.tag_keys)
            if unknown:
                raise ValueError(f"unknown tag keys {sorted(unknown)} for {self.name}")
            merged.update({k: str(v) for k, v in tags.items()})
        missing = [k for k in self.tag_keys if k not in merged]
        if missing:
            raise ValueError(f"missing values for tag keys {missing} of {self.name}")
        return tuple(merged[k] for k in self.tag_keys)

    def snapshot(self) -> dict:
        raise NotImplementedError


class Counter(Metric):
    """Monotonic count (``inc(value=1.0, tags=None)``, value > 0)."""
    kind = "counter"

    def __init__(self, name, description="", tag_keys=None):
        super().__init__(name, description, tag_keys)
        self._v: Dict[Tuple[str, ...], float] = {}

    def inc(self, value: float = 1.0, tags: Optional[Dict[str, str]] = None) -> None:
        if value <= 0:
            raise ValueError("Counter.inc value must be positive")
        k = self._key(tags)
        with self._lock:
            self._v[k] = self._v.get(k, 0.0) + float(value)

    def snapshot(self) -> dict:
        with self._lock:
            return dict(kind=self.kind, help=self.description, tag_keys=list(self.tag_keys),
                        series=[[list(k), v] for k, v in self._v.items()])


class Gauge(Metric):
    """Last value (``set(value, tags=None)``)."""
    kind = "gauge"

    def __init__(self, name, description="", tag_keys=None):
        super().__init__(name, description, tag_keys)
        self._v: Dict[Tuple[str, ...], float] = {}

    def set(self, value: float, tags: Optional[Dict[str, str]] = None) -> None:
        k = self._key(tags)
        with self._lock:
            self._v[k] = float(value)

    def snapshot(self) -> dict:
        with self._lock:
            return dict(kind=self.kind, help=self.description, tag_keys=list(self.tag_keys),
                        series=[[list(k), v] for k, v in self._v.items()])


class Histogram(Metric):
    """Bucketed distribution (``observe(value, tags=None)``); ``boundaries`` are
    the upper bucket bounds, positive and strictly increasing."""
    kind = "histogram"

    def __init__(self, name, description="", boundaries: Sequence[float] = (), tag_keys=None):
        b = [float(x) for x in boundaries]
        if not b or any(x <= 0 for x in b) or any(b[i] >= b[i + 1] for i in range(len(b) - 1)):
            raise ValueError("boundaries must be positive and strictly increasing")
        super().__init__(name, description, tag_keys)
        self.boundaries = b
        self._v: Dict[Tuple[str, ...], List[float]] = {}   # bucket counts..., +Inf count, sum

    def observe(self, value: float, tags: Optional[Dict[str, str]] = None) -> None:
        k = self._key(tags)
        i = bisect.bisect_left(self.boundaries, float(value))
        with self._lock:
            v = self._v.get(k)
            if v is None:
                v = self._v[k] = [0.0] * (len(self.boundaries) + 2)
            v[i] += 1
            v[-1] += float(value)

    def snapshot(self) -> dict:
        with self._lock:
            return dict(kind=self.kind, help=self.description, tag_keys=list(self.tag_keys),
                        boundaries=list(self.boundaries), series=[[list(k), list(v)] for k, v in self._v.items()])


def registry_snapshot() -> Dict[str, dict]:
    with _lock:
        items = list(_registry.items())
    return {n: m.snapshot() for n, m in items}


def clear_registry() -> None:
    with _lock:
        _registry.clear()


def _labels(keys: Iterable[str], values: Iterable[str], extra: Dict[str, str]) -> str:
    pairs = list(zip(keys, values)) + sorted(extra.items())
    if not pairs:
        return ""
    esc = [(k, str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")) for k, v in pairs]
    return "{" + ",".join(f'{k}="{v}"' for k, v in esc) + "}"


def render_prometheus(snapshots: Sequence[Tuple[Dict[str, str], Dict[str, dict]]]) -> str:
    """Prometheus text for [(extra_labels, registry_snapshot), ...] (one per process)."""
    by_name: Dict[str, List[Tuple[Dict[str, str], dict]]] = {}
    for extra, snap in snapshots:
        for name, m in snap.items():
            by_name.setdefault(name, []).append((extra, m))
    out: List[str] = []
    for name in sorted(by_name):
        first = by_name[name][0][1]
        out.append(f"# HELP {name} {first.get('help', '')}")
        out.append(f"# TYPE {name} {first['kind']}")
        for extra, m in by_name[name]:
            keys = m["tag_keys"]
            for vals, v in m["series"]:
                if m["kind"] == "histogram":
                    acc = 0.0
                    for ub, c in zip(m["boundaries"] + [float("inf")], v[:-1]):
                        acc += c
                        le = "+Inf" if ub == float("inf") else repr(ub)
                        out.append(f"{name}_bucket{_labels(keys, vals, dict(extra, le=le))} {acc:g}")
                    out.append(f"{name}_count{_labels(keys, vals, extra)} {acc:g}")
                    out.append(f"{name}_sum{_labels(keys, vals, extra)} {v[-1]:g}")
                else:
                    out.append(f"{name}{_labels(keys, vals, extra)} {v:g}")
    return "\n".join(out) + ("\n" if out else "")


# ---- replica -> controller publication through the node agent's KV ----------
KV_PREFIX = "metrics/"


def start_publisher(agent_socket: str, key: str, interval_s: float = 1.0) -> threading.Event:
    """Publish this process's registry as JSON under ``metrics/<key>`` every
    ``interval_s`` (replica processes).  Returns the stop event."""
    from ..runtime import agent as ragent

    stop = threading.Event()

    def loop():
        last = None
        while not stop.wait(interval_s):
            snap = registry_snapshot()
            if not snap:
                continue
            blob = json.dumps(snap, separators=(",", ":"))
            if blob == last:
                continue
            try:
                ragent.request(agent_socket, f"KV_PUT {KV_PREFIX}{key} {blob}")
                last = blob
            except RuntimeError:   # agent gone: the controller is shutting down
                return

    threading.Thread(target=loop, name="rdb-metrics-publisher", daemon=True).start()
    return stop


__all__ = ["Counter", "Gauge", "Histogram", "registry_snapshot", "render_prometheus", "start_publisher"]
