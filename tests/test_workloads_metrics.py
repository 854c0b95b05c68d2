import json
import time

from ray_dynamic_batching_amd.bench.results import ResultLogger
from ray_dynamic_batching_amd.bench.workloads import PATTERNS, Pattern, PatternDriver
from ray_dynamic_batching_amd.utils.dashboard import render
from ray_dynamic_batching_amd.utils.metrics import MetricsFileWriter, prometheus_text


def test_patterns_shapes():
    assert Pattern("ramp", base=0, slope=1, ramp_s=40).rate(10) == 10
    assert Pattern("ramp", base=0, slope=1, ramp_s=40).rate(100) == 40
    assert Pattern("step", base=5, step_at_s=3, step_to=9).rate(4) == 9
    assert Pattern("spike", base=1, spike_at_s=2, spike_len_s=1, spike_rate=50).rate(2.5) == 50
    s = Pattern("sinusoidal", base=10, amplitude=5, period_s=4)
    assert abs(s.rate(1) - 15) < 1e-9 and s.rate(3) >= 0
    r = Pattern("random", base=10, amplitude=5, period_s=1, seed=3)
    assert r.rate(0.2) == r.rate(0.7) and 5 <= r.rate(0.2) <= 15
    for k in PATTERNS:
        Pattern(k).rate(1.0)


def test_pattern_driver_rates_and_live_override():
    sent = {"a": 0, "b": 0}
    d = PatternDriver(lambda m: sent.__setitem__(m, sent[m] + 1),
                      {"a": Pattern("constant", base=200), "b": Pattern("constant", base=50)}, poisson=False)
    d.start(0.5)
    time.sleep(0.25)
    d.set_rate("b", 0)
    d.join()
    assert 70 <= sent["a"] <= 110
    assert sent["b"] <= 20


def test_metrics_file_dashboard_and_logger(tmp_path):
    stats = {"resnet": dict(total_requests=100, dropped_requests=2, slo_violations=1, queue_size=3,
                            avg_latency=10.0, p95_latency=20.0, p99_latency=30.0, request_rate=40.0)}
    w = MetricsFileWriter(lambda: stats, str(tmp_path / "metrics.json"))
    w.write_once()
    m = json.load(open(tmp_path / "metrics.json"))
    txt = render(m)
    assert "resnet" in txt and "99.00" in txt and "OK" in txt
    lg = ResultLogger(str(tmp_path / "res"))
    lg.log_metrics("t", stats)
    lg.log_changes("t", [dict(time=1, model="resnet", old_rate=1, new_rate=2)])
    assert (lg.test_dir / "t_metrics.json").exists() and (lg.test_dir / "t_changes.csv").exists()


def test_prometheus_text_from_shm():
    from ray_dynamic_batching_amd.runtime import job as rjob

    j = rjob.Job(rjob.unique_job_name("prom"), create=True, n_replicas=1, n_queues=1, n_clients=1)
    j.configure_queue(0, 0, 0, 4, 10.0, True)
    c = rjob.Client(j)
    cons = rjob.Consumer(j, [0])
    c.submit(0, b"x")
    for rid, q, cl, k, ts, dl, p in cons.pop(4, 10_000_000):
        cons.complete(cl, rid, q, 0, ts, b"y", 0)
    txt = prometheus_text(j, {0: "bert"}, {0: 0})
    assert 'serve_deployment_request_counter{deployment="bert",replica="0",queue="0"} 1' in txt
    j.close()
