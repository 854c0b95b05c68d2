"""Application metrics API (ray.util.metrics surface: Counter / Gauge / Histogram)
and its Prometheus exposition through the serve instance, incl. replica
processes publishing through the node agent's KV."""
import os
import sys
import time

import pytest

from ray_dynamic_batching_amd import serve
from ray_dynamic_batching_amd.utils import user_metrics as um

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _clean():
    um.clear_registry()
    yield
    serve.shutdown()
    um.clear_registry()


def test_metric_semantics_and_prometheus_text():
    c = um.Counter("rdb_test_requests", "requests", tag_keys=("route",)).set_default_tags({"route": "/"})
    c.inc()
    c.inc(2.5, tags={"route": "/x"})
    with pytest.raises(ValueError):
        c.inc(0)
    with pytest.raises(ValueError):
        c.inc(1, tags={"nope": "1"})
    g = um.Gauge("rdb_test_depth", "queue depth")
    g.set(7)
    h = um.Histogram("rdb_test_latency_ms", "latency", boundaries=[1, 5, 10])
    for v in (0.5, 3, 3, 20):
        h.observe(v)
    with pytest.raises(ValueError):
        um.Histogram("rdb_bad", boundaries=[5, 1])
    with pytest.raises(ValueError):
        um.Gauge("rdb_test_requests")          # same name, other type
    txt = um.render_prometheus([({"process": "p0"}, um.registry_snapshot())])
    assert '# TYPE rdb_test_requests counter' in txt
    assert 'rdb_test_requests{route="/",process="p0"} 1' in txt
    assert 'rdb_test_requests{route="/x",process="p0"} 2.5' in txt
    assert 'rdb_test_depth{process="p0"} 7' in txt
    assert 'rdb_test_latency_ms_bucket{le="1.0",process="p0"} 1' in txt
    assert 'rdb_test_latency_ms_bucket{le="5.0",process="p0"} 3' in txt
    assert 'rdb_test_latency_ms_bucket{le="+Inf",process="p0"} 4' in txt
    assert 'rdb_test_latency_ms_sum{process="p0"} 26.5' in txt


def test_replica_process_metrics_reach_the_controller():
    """A process-mode replica counts its calls with a Counter; the controller's
    exposition shows them (published through the agent KV) next to the native
    serve_* counters of the same replica."""
    sys.path.insert(0, ROOT)
    from examples.metrics_app import app

    h = serve.run(app, name="m", mode="process")
    for i in range(5):
        assert h.remote(i).result(timeout_s=60) == i + 1
    deadline = time.time() + 20
    txt = ""
    while time.time() < deadline:
        txt = serve.metrics_text()
        if 'app_calls_total{application="m",deployment="Counting",replica=' in txt:
            break
        time.sleep(0.3)
    assert 'app_calls_total{application="m",deployment="Counting",replica=' in txt, txt
    assert "serve_deployment_request_counter" in txt
