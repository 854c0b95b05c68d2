"""@serve.batch unit tests (in spirit of python/ray/serve/tests/unit/test_batching.py)."""
import asyncio
import time

import pytest

from ray_dynamic_batching_amd import serve
from ray_dynamic_batching_amd.serve.exceptions import RayServeException


def run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


def test_decorator_validation():
    with pytest.raises(TypeError):
        @serve.batch
        def not_async(xs):
            return xs
    with pytest.raises(ValueError):
        serve.batch(max_batch_size=0)
    with pytest.raises(TypeError):
        serve.batch(max_batch_size=1.5)
    with pytest.raises(ValueError):
        serve.batch(batch_wait_timeout_s=-1)
    with pytest.raises(TypeError):
        serve.batch(batch_wait_timeout_s="1")

    @serve.batch
    async def ok(xs):
        return xs
    assert ok._get_max_batch_size() == 10 and ok._get_batch_wait_timeout_s() == 0.0


def test_batch_size_one_long_timeout():
    @serve.batch(max_batch_size=1, batch_wait_timeout_s=1000)
    async def f(xs):
        return [x * 2 for x in xs]

    async def main():
        t = time.perf_counter()
        r = await f(3)
        assert time.perf_counter() - t < 1.0
        return r
    assert run(main()) == 6


def test_flush_on_full_batch_before_timeout():
    sizes = []

    @serve.batch(max_batch_size=4, batch_wait_timeout_s=1000)
    async def f(xs):
        sizes.append(len(xs))
        return xs

    async def main():
        return await asyncio.gather(*[f(i) for i in range(8)])
    assert run(main()) == list(range(8))
    assert sizes == [4, 4]


def test_flush_on_timeout_since_first_item():
    sizes = []

    @serve.batch(max_batch_size=100, batch_wait_timeout_s=0.05)
    async def f(xs):
        sizes.append(len(xs))
        return xs

    async def main():
        t = time.perf_counter()
        out = await asyncio.gather(*[f(i) for i in range(5)])
        return out, time.perf_counter() - t
    out, dt = run(main())
    assert out == list(range(5)) and sizes == [5]
    assert 0.04 <= dt < 0.5


def test_zero_timeout_batches_what_is_queued():
    gate = asyncio.Event
    sizes = []

    @serve.batch(max_batch_size=10, batch_wait_timeout_s=0)
    async def f(xs):
        sizes.append(len(xs))
        await asyncio.sleep(0.02)
        return xs

    async def main():
        first = asyncio.ensure_future(f(0))
        await asyncio.sleep(0.005)   # first batch (size 1) is executing
        rest = [asyncio.ensure_future(f(i)) for i in range(1, 6)]
        return await asyncio.gather(first, *rest)
    assert run(main()) == list(range(6))
    assert sizes[0] == 1 and sum(sizes) == 6 and max(sizes[1:]) > 1


def test_method_args_kwargs_transposed():
    class C:
        def __init__(self):
            self.calls = []

        @serve.batch(max_batch_size=3, batch_wait_timeout_s=0.05)
        async def f(self, a, b, *, k):
            self.calls.append((list(a), list(b), list(k)))
            return [x + y + z for x, y, z in zip(a, b, k)]

    c = C()

    async def main():
        return await asyncio.gather(c.f(1, 10, k=100), c.f(2, 20, k=200), c.f(3, 30, k=300))
    assert run(main()) == [111, 222, 333]
    assert c.calls == [([1, 2, 3], [10, 20, 30], [100, 200, 300])]


def test_exception_fans_out_to_all_callers():
    @serve.batch(max_batch_size=3, batch_wait_timeout_s=0.05)
    async def f(xs):
        raise ValueError("boom")

    async def main():
        return await asyncio.gather(*[f(i) for i in range(3)], return_exceptions=True)
    res = run(main())
    assert all(isinstance(r, ValueError) for r in res)


def test_wrong_result_length():
    @serve.batch(max_batch_size=2, batch_wait_timeout_s=0.05)
    async def f(xs):
        return xs[:1]

    async def main():
        return await asyncio.gather(f(1), f(2), return_exceptions=True)
    res = run(main())
    assert all(isinstance(r, RayServeException) for r in res)


def test_setters_change_behaviour():
    sizes = []

    @serve.batch(max_batch_size=2, batch_wait_timeout_s=1000)
    async def f(xs):
        sizes.append(len(xs))
        return xs

    f.set_max_batch_size(3)
    f.set_batch_wait_timeout_s(0.01)
    assert f._get_max_batch_size() == 3 and f._get_batch_wait_timeout_s() == 0.01
    with pytest.raises(ValueError):
        f.set_max_batch_size(0)

    async def main():
        return await asyncio.gather(*[f(i) for i in range(4)])
    run(main())
    assert sizes == [3, 1]


def test_async_generator_streaming():
    @serve.batch(max_batch_size=3, batch_wait_timeout_s=0.05)
    async def gen(xs):
        for i in range(3):
            yield [x * 10 + i for x in xs]

    async def consume(x):
        return [v async for v in gen(x)]

    async def main():
        return await asyncio.gather(consume(1), consume(2))
    assert run(main()) == [[10, 11, 12], [20, 21, 22]]


def test_cancelled_caller_is_skipped():
    seen = []

    @serve.batch(max_batch_size=4, batch_wait_timeout_s=0.05)
    async def f(xs):
        seen.extend(xs)
        return xs

    async def main():
        a = asyncio.ensure_future(f("a"))
        b = asyncio.ensure_future(f("b"))
        await asyncio.sleep(0)
        b.cancel()
        return await a
    assert run(main()) == "a"
    assert "b" not in seen


def test_idle_queue_leaves_no_pending_task_and_dead_loops_are_pruned():
    """The batching task exists only while requests are queued, and queues of
    closed event loops are dropped (reference: _BatchQueue.__del__ cancels its
    task, python/ray/serve/batching.py:323-333)."""
    @serve.batch(max_batch_size=4, batch_wait_timeout_s=0.01)
    async def f(xs):
        return xs

    lazy = f._rdb_batch_queue
    for _ in range(3):
        loop = asyncio.new_event_loop()
        async def main():
            return await asyncio.gather(*[f(i) for i in range(6)])
        assert f._is_batching_task_alive()        # idle is not dead
        assert loop.run_until_complete(main()) == list(range(6))
        assert f._is_batching_task_alive()        # idle again: still alive (reference semantics)
        assert f._get_handling_task_stack() is None
        assert not [t for t in asyncio.all_tasks(loop) if not t.done()]
        loop.close()
    loop = asyncio.new_event_loop()
    assert loop.run_until_complete(f(7)) == 7
    assert len(lazy._queues) == 1
    loop.close()


def test_batching_task_alive_reports_a_crashed_loop():
    """``_is_batching_task_alive`` is True before the first request and while
    idle, False once the batching loop itself died (reference
    tests/test_batching.py:190-206 and batching.py:400-410)."""
    @serve.batch(max_batch_size=4, batch_wait_timeout_s=0.01)
    async def f(xs):
        return xs

    loop = asyncio.new_event_loop()
    try:
        assert f._is_batching_task_alive()
        assert loop.run_until_complete(f(1)) == 1
        assert f._is_batching_task_alive()
        q = next(iter(f._rdb_batch_queue._queues.values()))

        async def boom():
            raise RuntimeError("loop died")
        q.wait_for_batch = boom
        with pytest.raises(RuntimeError, match="loop died"):
            loop.run_until_complete(f(2))
        assert not f._is_batching_task_alive()
    finally:
        loop.close()
