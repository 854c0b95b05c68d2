"""The TP batch broadcast ring (runtime/csrc/tp_bcast.h): one writer, N
readers in other processes, every record seen by every reader in publish
order, back-pressure when a reader lags, close() wakes blocked parties."""
import multiprocessing as mp
import os
import threading
import time
import uuid

import pytest

from ray_dynamic_batching_amd.utils.native import load_runtime


def _reader(name, idx, n, q):
    rt = load_runtime()
    b = rt.TPBcast(name, False, attach_timeout_s=30.0)
    got = []
    while len(got) < n:
        r = b.take(idx, 30.0)
        if r is None:
            break
        got.append((r[0], r[1], r[2], r[3], r[4], bytes(r[5])))
    q.put((idx, got))


def test_broadcast_every_reader_sees_every_record_in_order():
    rt = load_runtime()
    name = f"t{os.getpid()}_{uuid.uuid4().hex[:6]}"
    w = rt.TPBcast(name, True, n_readers=3, n_slots=4, payload_bytes=256)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    n = 200
    ps = [ctx.Process(target=_reader, args=(name, i, n, q)) for i in range(3)]
    for p in ps:
        p.start()
    try:
        for k in range(n):
            payload = bytes([k % 251]) * (k % 200)
            assert w.publish(0, k, k * 2, k % 3, k % 9, payload, 30.0)
        res = dict(q.get(timeout=60) for _ in ps)
    finally:
        for p in ps:
            p.join(30)
        w.unlink()
    want = [(0, k, k * 2, k % 3, k % 9, bytes([k % 251]) * (k % 200)) for k in range(n)]
    for i in range(3):
        assert res[i] == want, f"reader {i} diverged"


def test_backpressure_and_close():
    rt = load_runtime()
    name = f"t{os.getpid()}_{uuid.uuid4().hex[:6]}"
    w = rt.TPBcast(name, True, n_readers=1, n_slots=2, payload_bytes=16)
    r = rt.TPBcast(name, False)
    w.unlink()                                  # mappings survive the unlink
    assert w.publish(0, 1, 0, 0, 1, b"a", 1.0)
    assert w.publish(0, 2, 0, 0, 1, b"b", 1.0)
    t0 = time.time()
    assert not w.publish(0, 3, 0, 0, 1, b"c", 0.2)          # ring full: the reader lags
    assert time.time() - t0 >= 0.15
    assert r.take(0, 1.0)[1] == 1                           # frees one slot
    assert w.publish(0, 3, 0, 0, 1, b"c", 1.0)
    assert [r.take(0, 1.0)[1] for _ in range(2)] == [2, 3]
    # a reader blocked on an empty ring wakes on close() and gets None
    out = []
    th = threading.Thread(target=lambda: out.append(r.take(0, 30.0)))
    th.start()
    time.sleep(0.1)
    w.close()
    th.join(5)
    assert out == [None] and r.closed()
    with pytest.raises(ValueError):
        w.publish(0, 0, 0, 0, 0, b"x" * 4096, 0.1)          # larger than a slot
