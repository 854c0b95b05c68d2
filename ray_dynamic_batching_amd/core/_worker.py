"""Actor host process of :mod:`ray_dynamic_batching_amd.core`.

One process per actor (reference: a Ray actor is one worker process leased by
the raylet, ``core_worker.cc:2242 CreateActor`` / ``:3488 HandlePushTask``).
The process builds the actor instance, then serves method calls on a Unix
socket: every connection (one per caller process) gets a reader thread that
queues its calls, in arrival order, on the actor's executor -- one thread by
default, so calls from one caller run in submission order (Ray's ordered
actor queue, ``actor_scheduling_queue.cc``); ``max_concurrency`` > 1 runs
that many at once (threaded actors).
"""
from __future__ import annotations

import os
import sys
import threading
import traceback
from concurrent.futures import ThreadPoolExecutor
from multiprocessing.connection import Listener

TERMINATE = "__rdb_terminate__"
PING = "__rdb_ping__"
DAG_EXEC = "__rdb_dag_exec__"       # start a compiled-DAG execution loop (core/channel.py)
DAG_SETUP = "__rdb_dag_setup__"     # allocate a compiled DAG's inbound tensor rings (core/channel.py)


def _reply(conn, lock, msg) -> None:
    import cloudpickle

    data = cloudpickle.dumps(msg)
    with lock:
        conn.send_bytes(data)


def serve_calls(instance, listener: Listener, max_concurrency: int, stop: threading.Event) -> None:
    import cloudpickle

    pool = ThreadPoolExecutor(max(1, max_concurrency), thread_name_prefix="rdb-actor")

    def run(conn, lock, call_id, method, args, kwargs):
        try:
            fn = getattr(instance, method)
            res = fn(*args, **kwargs)
            if hasattr(res, "__await__"):          # async def methods
                import asyncio

                res = asyncio.run(_await(res))
            _reply(conn, lock, (call_id, True, res))
        except BaseException as e:  # noqa: BLE001 - shipped to the caller
            tb = traceback.format_exc()
            try:
                _reply(conn, lock, (call_id, False, (e, tb)))
            except Exception:       # unpicklable exception: ship its text
                _reply(conn, lock, (call_id, False, (RuntimeError(f"{type(e).__name__}: {e}"), tb)))

    def reader(conn):
        lock = threading.Lock()
        try:
            while not stop.is_set():
                try:
                    msg = cloudpickle.loads(conn.recv_bytes())
                except (EOFError, OSError):
                    return
                call_id, method, args, kwargs = msg
                if method == TERMINATE:
                    _reply(conn, lock, (call_id, True, None))
                    stop.set()
                    os._exit(0)
                if method == PING:
                    _reply(conn, lock, (call_id, True, os.getpid()))
                    continue
                if method == DAG_SETUP:
                    from .channel import create_rings

                    try:
                        _reply(conn, lock, (call_id, True, create_rings(*args)))
                    except BaseException as e:  # noqa: BLE001
                        _reply(conn, lock, (call_id, False, (RuntimeError(str(e)), traceback.format_exc())))
                    continue
                if method == DAG_EXEC:
                    from .channel import start_exec_loop

                    try:
                        start_exec_loop(instance, args[0])
                        _reply(conn, lock, (call_id, True, os.getpid()))
                    except BaseException as e:  # noqa: BLE001
                        _reply(conn, lock, (call_id, False, (RuntimeError(str(e)), traceback.format_exc())))
                    continue
                pool.submit(run, conn, lock, call_id, method, args, kwargs)
        finally:
            try:
                conn.close()
            except OSError:
                pass

    while not stop.is_set():
        try:
            conn = listener.accept()
        except (OSError, EOFError):
            if stop.is_set():
                return
            continue
        threading.Thread(target=reader, args=(conn,), daemon=True).start()


async def _await(aw):
    return await aw


def actor_main(payload: bytes, sys_path: list, address: str, authkey: bytes, env: dict, max_concurrency: int,
               ready) -> None:
    """Entry point of a spawned actor process."""
    os.environ.update(env)
    for p in reversed(sys_path):          # the driver's import path, before unpickling its classes
        if p not in sys.path:
            sys.path.insert(0, p)
    import cloudpickle

    try:
        cls, args, kwargs = cloudpickle.loads(payload)
        from . import _set_worker_context

        _set_worker_context(env)
        instance = cls(*args, **kwargs)
        listener = Listener(address, family="AF_UNIX", authkey=authkey)
    except BaseException as e:  # noqa: BLE001
        ready.send(("error", f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))
        return
    ready.send(("ok", os.getpid()))
    ready.close()
    serve_calls(instance, listener, max_concurrency, threading.Event())
