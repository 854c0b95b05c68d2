"""Native node agent: GPU slot allocator rules, persistent KV, flag registry,
process supervision (restart with back-off, heartbeat loss, fail-pending +
generation bump), and the Unix-socket control protocol."""
import os
import subprocess
import sys
import time

import pytest

from ray_dynamic_batching_amd.runtime import agent as ragent
from ray_dynamic_batching_amd.runtime import job as rjob
from ray_dynamic_batching_amd.utils import config


def test_allocator_whole_first_fit_fractional_best_fit_and_hbm():
    a = ragent.NodeAgent(4, 288.0)
    try:
        x = a.allocate("x", 2)
        assert x["gpus"] == [0, 1]
        h1 = a.allocate("h1", 0.5)
        assert h1["gpus"] == [2]
        h2 = a.allocate("h2", 0.25)        # best fit: GPU 2 has the least room that still fits
        assert h2["gpus"] == [2]
        h3 = a.allocate("h3", 0.5)         # GPU 2 has 0.25 left -> goes to GPU 3
        assert h3["gpus"] == [3]
        assert a.allocate("big", 1) is None  # no whole GPU free
        assert a.allocate("hbm", 0.1, 300.0) is None  # over the 288 GB budget
        assert a.release("x")
        assert a.allocate("big", 1)["gpus"] == [0]
        snap = a.resources()
        assert snap[2]["used"] == pytest.approx(0.75)
        with pytest.raises(ValueError):
            a.allocate("bad", 1.5)
    finally:
        a.shutdown()


def test_allocator_placement_group_bundles_gang_and_strategies():
    """Placement-group bundles are reserved all-or-nothing with the Ray
    strategies: PACK fills the group's own GPU first, SPREAD / STRICT_SPREAD use
    distinct GPUs, STRICT_PACK one GPU, and a failed gang leaves nothing held."""
    a = ragent.NodeAgent(4, 288.0)
    try:
        tp = a.allocate_bundles("tp", [(1, 0), (1, 0)], "STRICT_SPREAD")
        assert tp["gpus"] == [0, 1] and tp["bundle_gpus"] == [[0], [1]]
        pk = a.allocate_bundles("pk", [(0.25, 0), (0.25, 0), (0.25, 0)], "PACK")
        assert pk["gpus"] == [2] and pk["bundle_gpus"] == [[2], [2], [2]] and abs(pk["fraction"] - 0.75) < 1e-9
        sp = a.allocate_bundles("sp", [(0.25, 0), (0.25, 0)], "SPREAD")
        assert sorted(sp["gpus"]) == [2, 3]          # GPU 2 has 0.25 left, then the group's second bundle spreads
        # STRICT_SPREAD that cannot be met (3 distinct GPUs with 0.5 free: only GPU 3 has it) -> nothing held
        before = [g["used"] for g in a.resources()]
        assert a.allocate_bundles("bad", [(0.5, 0), (0.5, 0), (0.5, 0)], "STRICT_SPREAD") is None
        assert [g["used"] for g in a.resources()] == before
        assert a.allocate_bundles("sp2", [(0.9, 0), (0.9, 0)], "STRICT_PACK") is None
        sk = a.allocate_bundles("sk", [(0.3, 0), (0.4, 0)], "STRICT_PACK")
        assert len(sk["gpus"]) == 1
        assert a.allocate_bundles("hbm", [(0.01, 290.0)], "PACK") is None   # HBM budget per GPU
        assert a.release("tp") and a.release("pk")
        assert a.allocate_bundles("tp2", [(2, 0)], "PACK")["gpus"] == [0, 1]
        with pytest.raises(ValueError):
            a.allocate_bundles("x", [(1, 0)], "NOPE")
    finally:
        a.shutdown()


def test_placement_group_config_validation():
    from ray_dynamic_batching_amd.serve.config import DeploymentConfig

    c = DeploymentConfig(ray_actor_options={"num_gpus": 1}, placement_group_bundles=[{"GPU": 1}, {"GPU": 1}],
                         placement_group_strategy="STRICT_SPREAD", num_replicas=4, max_replicas_per_node=2)
    assert c.placement_bundles() == [(1.0, 0.0), (1.0, 0.0)]
    assert c.initial_num_replicas() == 2 and c.cap_replicas(7) == 2
    for bad in [dict(placement_group_strategy="PACK"),                                   # strategy without bundles
                dict(placement_group_bundles=[]),
                dict(placement_group_bundles=[{"GPU": 1}], placement_group_strategy="RANDOM"),
                dict(ray_actor_options={"num_gpus": 1}, placement_group_bundles=[{"CPU": 1}, {"GPU": 1}]),
                dict(max_replicas_per_node=0)]:
        with pytest.raises(ValueError):
            DeploymentConfig(**bad)


def test_kv_store_persists_atomically(tmp_path):
    p = str(tmp_path / "kv.bin")
    k = ragent.KvStore(p)
    k.put("serve/app", b'{"a": 1}')
    k.put("bin", bytes(range(256)))
    k2 = ragent.KvStore(p)
    assert k2.get("serve/app") == b'{"a": 1}'
    assert k2.get("bin") == bytes(range(256))
    assert sorted(k2.keys("serve/")) == ["serve/app"]
    assert k2.delete("bin") and ragent.KvStore(p).get("bin") is None


def test_config_registry_env_override():
    env = dict(os.environ, RDB_HEALTH_CHECK_TIMEOUT_S="7.5")
    code = ("from ray_dynamic_batching_amd.utils import config;"
            "print(config.get('health_check_timeout_s'), config.get('max_restarts'))")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.stdout.split() == ["7.5", "-1"], out.stderr
    assert config.define("unit_test_flag", "int", 4, "x") == 4
    config.set("unit_test_flag", 9)
    assert config.get("unit_test_flag") == 9
    with pytest.raises(ValueError):
        config.set("unit_test_flag", "nine")


def _wait(pred, timeout=10.0):
    t = time.time() + timeout
    while time.time() < t:
        if pred():
            return True
        time.sleep(0.02)
    return False


def test_supervisor_restarts_with_backoff_and_terminate(tmp_path):
    a = ragent.NodeAgent(0)
    try:
        log = str(tmp_path / "p.log")
        pid = ragent.spawn_replica(a, "crashy", [sys.executable, "-c", "import sys; print('hi'); sys.exit(3)"],
                                   {}, log, backoff_initial_s=0.05, backoff_max_s=0.2, max_restarts=3)
        assert _wait(lambda: a.info(pid)["state"] == "EXITED")
        info = a.info(pid)
        assert info["restarts"] == 3 and "exit code 3" in info["last_exit"]
        assert open(log).read().count("hi") == 4
        kinds = [e[1] for e in a.events()]
        assert kinds.count("died") == 3 and "exited" in kinds

        pid2 = ragent.spawn_replica(a, "sleeper", [sys.executable, "-c", "import time; time.sleep(60)"], {}, "")
        assert _wait(lambda: a.info(pid2)["state"] == "RUNNING")
        assert a.terminate(pid2, 2.0)
        assert a.info(pid2)["state"] == "STOPPED"
    finally:
        a.shutdown()


def test_supervisor_heartbeat_loss_fails_pending_and_bumps_generation(tmp_path):
    name = rjob.unique_job_name("agent")
    j = rjob.Job(name, create=True, n_replicas=1, n_queues=1, n_clients=1, req_slot_bytes=128, cmp_slot_bytes=64)
    j.configure_queue(0, 0, 0, 64, 0.0, True)
    # replica: marks itself READY, heart-beats for 0.3 s, then hangs (no heartbeats, no consumption)
    code = (f"from ray_dynamic_batching_amd.runtime import job as rjob; import time, os;"
            f"j = rjob.Job('{name}', create=False); j.set_replica_status(0, 2, -1, os.getpid());"
            f"t = time.time()\n"
            f"while time.time() - t < 0.3: j.heartbeat(0); time.sleep(0.02)\n"
            f"time.sleep(60)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    a = ragent.NodeAgent(0)
    try:
        pid = ragent.spawn_replica(a, "hb", [sys.executable, "-c", code], {"PYTHONPATH": root},
                                   str(tmp_path / "hb.log"), job=name, replica=0, queues=[0],
                                   health_timeout_s=0.5, backoff_initial_s=30.0)
        assert _wait(lambda: j.replica_status(0) == 2, 60)
        c = rjob.Client(j)
        rid = c.submit(0, b"x" * 32)
        got = []
        assert _wait(lambda: bool(got.extend(c.poll(8, 0.05)) or got), 20)
        assert got[0][0] == rid and got[0][1] == int(rjob.Status.REPLICA_DIED)
        # the agent fails the pending requests first, then bumps the generation and
        # enters back-off (node_agent.cpp on_death_locked): the completion can win the race
        assert _wait(lambda: j.replica_generation(0) == 1, 10)
        assert _wait(lambda: a.info(pid)["state"] == "BACKOFF", 10)
        assert "missed heartbeats" in a.info(pid)["last_exit"]
    finally:
        a.shutdown(1.0)
        j.close()


def test_control_socket_protocol(tmp_path):
    sock = str(tmp_path / "agent.sock")
    a = ragent.NodeAgent(2, 288.0, str(tmp_path / "kv.bin"))
    try:
        a.serve(sock)
        assert ragent.request(sock, "PING") == "PONG"
        assert ragent.request(sock, "KV_PUT plan {\"gpus\": 2}") == "OK"
        assert a.kv_get("plan") == b'{"gpus": 2}'
        assert ragent.request(sock, "KV_GET plan") == 'OK {"gpus": 2}'
        assert ragent.request(sock, "KV_GET nope") == "NOTFOUND"
        assert ragent.request(sock, "CONFIG health_check_period_s").startswith("OK ")
        a.allocate("r0", 1)
        st = ragent.status(sock)
        assert st["gpus"][0]["used"] == 1.0 and st["procs"] == []
    finally:
        a.shutdown()
