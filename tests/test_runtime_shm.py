"""CPU tests of the native shm data plane (rings, router, consumer, load generator)."""
import multiprocessing as mp
import os
import struct
import threading
import time

import pytest

from ray_dynamic_batching_amd.runtime import job as rjob


def _name(tag):
    return rjob.unique_job_name(tag)


def test_submit_pop_complete_roundtrip():
    j = rjob.Job(_name("rt"), create=True, n_replicas=1, n_queues=2, n_clients=2, req_slot_bytes=256, cmp_slot_bytes=128)
    j.configure_queue(0, 0, 7, 100, 0.0, True)
    j.set_replica_status(0, int(rjob.ReplicaStatus.READY))
    c = rjob.Client(j)
    cons = rjob.Consumer(j, [0])
    rids = [c.submit(0, bytes([i]) * 10) for i in range(5)]
    assert all(r > 0 for r in rids)
    assert j.queue_depth(0) == 5
    got = cons.pop(16, 10_000_000)
    assert [g[0] for g in got] == rids
    for g in got:
        rid, q, client, kind, t_sub, dl, payload = g
        assert payload == bytes([rid - rids[0]]) * 10
        cons.complete(client, rid, q, 0, t_sub, payload[::-1], 0)
    comps = c.poll(16, 0.5)
    assert sorted(x[0] for x in comps) == rids
    assert all(x[1] == 0 for x in comps)
    st = j.queue_stats(0)
    assert st["submitted"] == 5 and st["completed"] == 5 and st["depth"] == 0
    assert st["e2e"]["count"] == 5
    j.close()


def test_ring_full_backpressure_and_too_large():
    j = rjob.Job(_name("bp"), create=True, n_replicas=1, n_queues=1, n_clients=1, req_capacity=8, req_slot_bytes=64)
    c = rjob.Client(j)
    ok = [c.submit(0, b"x" * 8) for _ in range(8)]
    assert all(r > 0 for r in ok)
    assert c.submit(0, b"x") == -1          # ring full
    assert c.submit(0, b"x" * 65) == -3     # larger than a slot
    j.close()


def test_pow2_router_prefers_shorter_queue_and_respects_max_ongoing():
    j = rjob.Job(_name("p2"), create=True, n_replicas=2, n_queues=2, n_clients=1)
    j.configure_queue(0, 0, 1, 4, 0.0, True)
    j.configure_queue(1, 1, 1, 4, 0.0, True)
    j.set_replica_status(0, 2)
    j.set_replica_status(1, 2)
    c = rjob.Client(j, seed=3)
    for _ in range(3):
        c.submit(0, b"a")
    # queue 1 is empty -> always chosen
    for _ in range(20):
        assert c.choose_queue(1) == 1
    for _ in range(4):
        c.submit(1, b"b")
    # q0 has 3 (< 4), q1 has 4 (== max) -> q0
    assert c.choose_queue(1) == 0
    c.submit(0, b"a")
    assert c.choose_queue(1) == -1          # both saturated
    assert c.choose_queue(99) == -2         # unknown model
    j.set_replica_status(0, 4)              # dead replica is skipped
    j.close()


def _echo_replica(name, q, n, stop_after):
    j = rjob.Job(name, create=False)
    cons = rjob.Consumer(j, [q])
    done = 0
    while done < stop_after:
        for rid, qq, client, kind, t_sub, dl, payload in cons.pop(64, 50_000_000):
            (x,) = struct.unpack("<i", payload[:4])
            cons.complete(client, rid, qq, 0, t_sub, struct.pack("<i", x * 2), 0)
            done += 1
    j.close()


def test_cross_process_loadgen_closed_loop():
    name = _name("lg")
    j = rjob.Job(name, create=True, n_replicas=2, n_queues=2, n_clients=2, req_slot_bytes=64, cmp_slot_bytes=64)
    for q in range(2):
        j.configure_queue(q, q, 0, 64, 0.0, True)
        j.set_replica_status(q, 2)
    total = 4000
    ctx = mp.get_context("fork")
    procs = [ctx.Process(target=_echo_replica, args=(name, q, 2, 10**9)) for q in range(2)]
    for p in procs:
        p.daemon = True
        p.start()
    c = rjob.Client(j)
    lg = rjob.LoadGen(c, 0, [struct.pack("<i", i) + b"\0" * 12 for i in range(16)])
    res = lg.run(total, 32, 0.0, 0.0, True, 60.0)
    for p in procs:
        p.kill()
        p.join()
    assert res["ok"] == total and res["completed"] == total and not res["timed_out"]
    assert res["latency"]["count"] == total
    # both replicas got traffic through the pow-2 router (by queue depth: a replica
    # process the host schedules less drains slower and gets a smaller share; under a
    # loaded host -- a parallel compile -- one replica can get as little as a few %)
    assert min(res["per_queue"]) > total * 0.01
    j.close()


def test_loadgen_open_loop_poisson_rate():
    name = _name("pl")
    j = rjob.Job(name, create=True, n_replicas=1, n_queues=1, n_clients=2, req_slot_bytes=64, cmp_slot_bytes=64)
    j.configure_queue(0, 0, 0, 0, 0.0, True)
    j.set_replica_status(0, 2)
    ctx = mp.get_context("fork")
    p = ctx.Process(target=_echo_replica, args=(name, 0, 1, 10**9), daemon=True)
    p.start()
    c = rjob.Client(j)
    lg = rjob.LoadGen(c, 0, [b"\1\0\0\0" + b"\0" * 12])
    t = time.perf_counter()
    res = lg.run(500, 0, 2000.0, 0.0, True, 30.0)
    dt = time.perf_counter() - t
    p.kill()
    p.join()
    assert res["ok"] == 500
    assert 0.15 < dt < 1.0  # ~0.25 s at 2000 req/s
    j.close()


def test_fail_queue_answers_pending_requests():
    j = rjob.Job(_name("fq"), create=True, n_replicas=1, n_queues=1, n_clients=1)
    c = rjob.Client(j)
    for _ in range(3):
        c.submit(0, b"zz")
    assert j.fail_queue(0, int(rjob.Status.REPLICA_DIED)) == 3
    comps = c.poll(10, 0.2)
    assert len(comps) == 3 and all(x[1] == int(rjob.Status.REPLICA_DIED) for x in comps)
    assert j.queue_depth(0) == 0
    j.close()
