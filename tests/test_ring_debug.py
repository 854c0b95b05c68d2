"""RDB_RING_DEBUG: the shared-memory rings' sequence-check debug mode
(reference analogue: the sanitizer / _RAY_TSAN_BUILD configs,
.bazelrc:103-136).  Each case runs in a fresh process because the level is
read once per process."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(body: str, level: str = "1"):
    code = textwrap.dedent("""
        import os, uuid
        from ray_dynamic_batching_amd.runtime import job as rjob
        from ray_dynamic_batching_amd.utils.native import load_runtime
        rt = load_runtime()
        j = rjob.Job("dbg" + uuid.uuid4().hex[:8], create=True, n_replicas=1, n_queues=1, n_clients=2,
                     req_capacity=16)
        j.unlink_on_close(True)
        j.configure_queue(0, 0, 0, 64)
        cli = rjob.Client(j)
        cons = rjob.Consumer(j, [0])
    """) + textwrap.dedent(body)
    env = dict(os.environ, RDB_RING_DEBUG=level, PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True,
                          timeout=120)


def test_debug_off_by_default_and_clean_traffic_has_no_violations():
    r = _run("""
        for i in range(40):
            assert cli.submit(0, b"x%d" % i) >= 0
            got = cons.pop(8, 0)
            assert len(got) == 1
        assert rt.ring_debug_level() == 1
        assert rt.ring_violations()[0] == 0, rt.ring_violations()
        print("CLEAN")
    """)
    assert r.returncode == 0 and "CLEAN" in r.stdout, r.stderr
    r = _run("""
        assert rt.ring_debug_level() == 0
        print("OFF")
    """, level="0")
    assert "OFF" in r.stdout, r.stderr


def test_corrupted_sequence_number_is_caught_at_peek():
    r = _run("""
        for i in range(3):
            assert cli.submit(0, b"r%d" % i) >= 0
        j._test_corrupt_seq(0, 1, 5)        # request 2's slot: a sequence number of no valid lap
        got = cons.pop(8, 0)
        assert [g[6] for g in got] == [b"r0"], got   # the consumer stops before the bad slot
        n, msg = rt.ring_violations()
        assert n >= 1 and "peek" in msg, (n, msg)
        print("CAUGHT", msg)
    """)
    assert r.returncode == 0 and "CAUGHT" in r.stdout, (r.stdout, r.stderr)
    assert "[rdb ring debug]" in r.stderr


def test_stray_publish_is_caught_at_reserve_instead_of_spinning():
    r = _run("""
        j._test_corrupt_seq(0, 0, 1)        # the next free slot looks published by nobody
        rid = cli.submit(0, b"late")        # without the check: an endless reserve loop
        assert rid < 0, rid
        n, msg = rt.ring_violations()
        assert n >= 1 and "reserve" in msg, (n, msg)
        print("CAUGHT", msg)
    """)
    assert r.returncode == 0 and "CAUGHT" in r.stdout, (r.stdout, r.stderr)


def test_level_two_aborts_at_the_first_violation():
    r = _run("""
        cli.submit(0, b"a"); cli.submit(0, b"b")
        j._test_corrupt_seq(0, 0, 7)
        cons.pop(8, 0)
        print("NOT REACHED")
    """, level="2")
    assert r.returncode != 0 and "NOT REACHED" not in r.stdout
    assert "[rdb ring debug]" in r.stderr
