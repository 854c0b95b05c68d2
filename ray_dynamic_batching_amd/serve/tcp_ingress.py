"""TCP ingress for request streams (the fork's ZMQ RequestHandle,
milind-code/scheduler.py:20-130, which bound tcp://*:5555 and promised -- but
never implemented -- results on :5556).

Protocol: newline-delimited JSON over one TCP connection per client.
  request : {"model": "resnet", "id": 7, "input": [...]?, "deadline_ms": 30?}
  response: {"id": 7, "model": "resnet", "status": "ok"|"dropped"|"error"|..., "latency_ms": 3.2,
             "output": [...]?}        (output only when the request asked "want_output": true)
A request without "input" gets a synthetic tensor of the model's input shape
(as the fork's RequestHandle did with torch.rand).

Targets: an ``SLOScheduler`` (per-model queues + planner; rates are tracked
per submit) or a mapping ``{model: DeploymentHandle}``.
"""
from __future__ import annotations

import asyncio
import json
import threading
import time
from typing import Any, Dict, Optional

import numpy as np

STATUS = {0: "ok", 1: "dropped", 2: "error", 3: "rejected", 4: "too_large", 5: "shutdown", 6: "replica_died"}


class TCPIngress:
    def __init__(self, target: Any, host: str = "127.0.0.1", port: int = 0):
        self.target = target
        self.host = host
        self.port = port
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.thread: Optional[threading.Thread] = None
        self._server = None
        self._pending: Dict[int, tuple] = {}     # scheduler rid -> (writer, client id, model, t0, want_output)
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._poller: Optional[threading.Thread] = None
        self.received = 0
        self.answered = 0
        self._rng = np.random.default_rng(0)

    # -- lifecycle
    def start(self, timeout_s: float = 10.0) -> "TCPIngress":
        ready = threading.Event()

        def run():
            self.loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self.loop)
            self._server = self.loop.run_until_complete(asyncio.start_server(self._on_client, self.host, self.port))
            self.port = self._server.sockets[0].getsockname()[1]
            ready.set()
            self.loop.run_forever()
            self._server.close()
            self.loop.run_until_complete(self._server.wait_closed())
            self.loop.close()

        self.thread = threading.Thread(target=run, name="rdb-tcp-ingress", daemon=True)
        self.thread.start()
        if not ready.wait(timeout_s):
            raise RuntimeError("TCP ingress failed to start")
        if hasattr(self.target, "poll"):
            self._poller = threading.Thread(target=self._poll_loop, name="rdb-tcp-poll", daemon=True)
            self._poller.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._poller is not None:
            self._poller.join(2)
        if self.loop is not None:
            self.loop.call_soon_threadsafe(self.loop.stop)
        if self.thread is not None:
            self.thread.join(5)

    # -- request path
    def _input_for(self, model: str, msg: dict):
        codec = self.target.codecs[model] if hasattr(self.target, "codecs") else None
        if "input" in msg:
            return np.asarray(msg["input"], dtype=codec.in_np if codec is not None else None)
        if codec is None:
            raise ValueError("request has no input and the target has no codec for it")
        if np.issubdtype(codec.in_np, np.integer):
            return self._rng.integers(0, 100, size=codec.input_shape).astype(codec.in_np)
        return self._rng.random(codec.input_shape, dtype=np.float32).astype(codec.in_np)

    async def _on_client(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        try:
            while True:
                line = await reader.readline()
                if not line:
                    break
                self.received += 1
                try:
                    msg = json.loads(line)
                    model = msg["model"]
                    x = self._input_for(model, msg)
                except Exception as e:  # malformed request
                    await self._send(writer, {"id": None, "status": "error", "error": str(e)})
                    continue
                t0 = time.perf_counter()
                want = bool(msg.get("want_output", False))
                if hasattr(self.target, "submit"):
                    rid = self.target.submit(model, x, float(msg.get("deadline_ms", 0)) / 1e3)
                    if rid < 0:
                        await self._send(writer, {"id": msg.get("id"), "model": model, "status": "rejected"})
                        continue
                    with self._lock:
                        self._pending[rid] = (writer, msg.get("id"), model, t0, want)
                else:
                    asyncio.ensure_future(self._via_handle(writer, msg.get("id"), model, x, t0, want))
        finally:
            writer.close()

    async def _via_handle(self, writer, cid, model, x, t0, want):
        try:
            out = await self.target[model].remote(x)
            resp = {"id": cid, "model": model, "status": "ok", "latency_ms": (time.perf_counter() - t0) * 1e3}
            if want:
                resp["output"] = np.asarray(out).tolist()
        except Exception as e:
            resp = {"id": cid, "model": model, "status": "error", "error": f"{type(e).__name__}: {e}"}
        await self._send(writer, resp)

    async def _send(self, writer, obj) -> None:
        try:
            writer.write((json.dumps(obj) + "\n").encode())
            await writer.drain()
            self.answered += 1
        except (ConnectionError, RuntimeError):
            pass

    def _poll_loop(self) -> None:
        while not self._stop.is_set():
            try:
                comps = self.target.poll(1024, 0.05)
            except Exception:
                break
            for rid, st, q, ts, td, tr, kind, payload in comps:
                with self._lock:
                    ent = self._pending.pop(rid, None)
                if ent is None:
                    continue
                writer, cid, model, t0, want = ent
                resp = {"id": cid, "model": model, "status": STATUS.get(st, str(st)),
                        "latency_ms": (time.perf_counter() - t0) * 1e3}
                if want and st == 0 and payload:
                    codec = self.target.codecs[model]
                    resp["output"] = codec.decode(payload).tolist()
                asyncio.run_coroutine_threadsafe(self._send(writer, resp), self.loop)
