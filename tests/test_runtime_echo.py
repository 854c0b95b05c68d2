"""Native fake replicas (EchoServer) driving the C++ router/load generator:
pow-2 routing by shm queue depth, batching under load, and the runtime
microbenchmark (request-path overhead without a GPU)."""
import os
import subprocess
import sys

import pytest

from ray_dynamic_batching_amd.runtime import job as rjob


def _job(nq, n_clients=2, **kw):
    j = rjob.Job(rjob.unique_job_name("echo"), create=True, n_replicas=nq, n_queues=nq, n_clients=n_clients,
                 req_capacity=1024, req_slot_bytes=256, cmp_capacity=2048, cmp_slot_bytes=64, **kw)
    for q in range(nq):
        j.configure_queue(q, q, 0, 1024, 0.0, True)
    return j


def test_echo_roundtrip_payload():
    j = _job(1)
    s = rjob.EchoServer(j, 0, [0], max_batch=8, out_bytes=16)
    s.start()
    try:
        c = rjob.Client(j, 0)
        rids = {c.submit(0, bytes([i]) * 32): i for i in range(50)}
        got = {}
        while len(got) < 50:
            for rid, st, q, ts, td, tr, kind, payload in c.poll(64, 1.0):
                assert st == 0
                got[rids[rid]] = payload
        assert all(got[i] == bytes([i]) * 16 for i in range(50))
        assert s.served() == 50
    finally:
        s.stop()
        j.close()


def test_pow2_routing_prefers_less_loaded_replica():
    j = _job(2)
    fast = rjob.EchoServer(j, 0, [0], max_batch=16, service_us=50.0)
    slow = rjob.EchoServer(j, 1, [1], max_batch=16, service_us=3000.0)
    fast.start()
    slow.start()
    try:
        c = rjob.Client(j, 0)
        lg = rjob.LoadGen(c, 0, [b"x" * 64])
        res = lg.run(4000, 64, 0.0, 0.0, True, 60.0)
        assert res["ok"] == 4000
        assert fast.served() > 3 * slow.served(), (fast.served(), slow.served())
    finally:
        fast.stop()
        slow.stop()
        j.close()


def test_loadgen_histogram_state_merges_like_merge_from():
    """hist_state()/merge_state() fold a generator's latencies across processes
    (bench.py's per-rank ingress); the result equals the in-process merge_from."""
    j = _job(2, n_clients=3)
    servers = [rjob.EchoServer(j, r, [r], max_batch=16, service_us=200.0 * (r + 1)) for r in range(2)]
    for s in servers:
        s.start()
    try:
        a = rjob.LoadGen(rjob.Client(j, 0), 0, [b"a" * 32])
        b = rjob.LoadGen(rjob.Client(j, 1), 0, [b"b" * 32])
        assert a.run(800, 32, 0.0, 0.0, True, 60.0)["ok"] == 800
        assert b.run(600, 16, 0.0, 0.0, True, 60.0)["ok"] == 600
        st = b.hist_state()
        assert len(st[0]) > 0 and st[1] == 600 and sum(st[0]) == 600
        via_state = rjob.LoadGen(rjob.Client(j, 2), 0, [b"c"])
        via_state.merge_state(*a.hist_state())
        via_state.merge_state(*st)
        a.merge_from(b)
        assert via_state.latency() == a.latency()
        assert a.latency()["count"] == 1400
        with pytest.raises(ValueError):
            via_state.merge_state([1, 2, 3], 6, 0, 0)
    finally:
        for s in servers:
            s.stop()
        j.close()


def test_batches_form_under_load():
    j = _job(1)
    s = rjob.EchoServer(j, 0, [0], max_batch=32, service_us=500.0)
    s.start()
    try:
        c = rjob.Client(j, 0)
        lg = rjob.LoadGen(c, 0, [b"y" * 64])
        res = lg.run(3000, 128, 0.0, 0.0, True, 60.0)
        assert res["ok"] == 3000
        st = j.replica_stats(0)
        assert st["batch_items"] / st["batches"] > 16
    finally:
        s.stop()
        j.close()


def test_runtime_microbench_runs():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench", "runtime_microbench.py"), "--total", "5000",
                          "--queues", "2"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "1:1 sync" in out.stdout and "serve path" in out.stdout


def test_trace_ring_and_chrome_export(tmp_path):
    import json

    from ray_dynamic_batching_amd.utils import tracing

    j = _job(2)
    s = rjob.EchoServer(j, 1, [1], max_batch=8, service_us=100.0)
    s.start()
    try:
        c = rjob.Client(j, 0)
        lg = rjob.LoadGen(c, 0, [b"z" * 32])
        lg.run(400, 32, 0.0, 0.0, False, 30.0)
        j.trace_record(0, 1, 1000, 2000, 0, 3, 4)
        # the echo replica appends a batch's trace event after posting its
        # completions: the last batch's record may land just after run() returns
        import time
        deadline = time.monotonic() + 5.0
        while True:
            ev = tracing.collect(j)
            if sum(e["n"] for e in ev if e["replica"] == 1) >= 400 or time.monotonic() > deadline:
                break
            time.sleep(0.01)
        assert any(e["replica"] == 1 and e["kind"] == "gpu" for e in ev)
        assert sum(e["n"] for e in ev if e["replica"] == 1) == 400
        tr = tracing.export_chrome_trace(j, str(tmp_path / "t.json"))
        assert json.load(open(tmp_path / "t.json"))["traceEvents"] == tr["traceEvents"]
        assert tracing.summarize(ev)["gpu"]["mean_us"] >= 100.0
    finally:
        s.stop()
        j.close()


def test_seqlock_snapshot_publish_read():
    j = _job(1)
    try:
        assert j.read_snapshot() == (0, b"")
        assert j.publish(b'{"routes": 1}') == 1
        assert j.publish(b'{"routes": 2}') == 2
        other = rjob.Job(j.info()["name"], create=False)
        assert other.read_snapshot() == (2, b'{"routes": 2}')
        other.close()
    finally:
        j.close()


def test_stalled_client_cannot_wedge_the_replica(monkeypatch):
    """A client whose completion ring fills (crashed / wedged proxy) is marked
    stalled after RDB_COMPLETION_TIMEOUT_MS and loses its completions; the
    replica keeps answering every other client and stops cleanly."""
    import time

    monkeypatch.setenv("RDB_COMPLETION_TIMEOUT_MS", "100")
    j = rjob.Job(rjob.unique_job_name("stall"), create=True, n_replicas=1, n_queues=1, n_clients=2,
                 req_capacity=1024, req_slot_bytes=128, cmp_capacity=16, cmp_slot_bytes=64)
    j.configure_queue(0, 0, 0, 0, 0.0, True)
    s = rjob.EchoServer(j, 0, [0], max_batch=4, out_bytes=8)
    s.start()
    try:
        dead, live = rjob.Client(j, 0), rjob.Client(j, 1)
        for i in range(64):                 # 4x its completion ring; never polled
            assert dead.submit(0, b"d" * 16) > 0
        rids = {live.submit(0, bytes([i]) * 16) for i in range(40)}
        got, t_end = set(), time.time() + 20
        while len(got) < len(rids) and time.time() < t_end:
            for rid, st, *_ in live.poll(64, 0.2):
                assert st == 0
                got.add(rid)
        assert got == rids
        info = j.info()
        assert info["stalled_clients"] == [0] and info["completions_dropped"] >= 64 - 16
        assert j.queue_depth(0) == 0       # dropped completions still left the queue
        dead.poll(64, 0.0)                  # polling clears the stall
        assert j.info()["stalled_clients"] == []
    finally:
        t0 = time.time()
        s.stop()
        assert time.time() - t0 < 5
        j.close()
