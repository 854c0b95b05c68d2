"""Request simulator with live per-model rate changes (the fork's
milind-code/request_simulator.py: one sender thread per model at 1/rate
spacing, rate changeable at runtime, rate 0 stops the model's stream) talking
to serve.tcp_ingress.TCPIngress.

    python bench/request_simulator.py --port 5555            # then type: resnet 50 / vit 0 / stats / quit
"""
from __future__ import annotations

import argparse
import json
import socket
import sys
import threading
import time
from typing import Dict


class RequestSimulator:
    def __init__(self, host: str = "127.0.0.1", port: int = 5555):
        self.sock = socket.create_connection((host, port))
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._wlock = threading.Lock()
        self.rates: Dict[str, float] = {}
        self._threads: Dict[str, threading.Thread] = {}
        self._next_id = 0
        self._id_lock = threading.Lock()
        self.sent: Dict[str, int] = {}
        self.responses: Dict[str, Dict[str, int]] = {}
        self.latencies_ms: Dict[str, list] = {}
        self._closed = False
        self._reader = threading.Thread(target=self._read_loop, daemon=True)
        self._reader.start()

    def set_rate(self, model: str, rate: float) -> None:
        """Change a model's request rate (req/s) at runtime; 0 stops it."""
        self.rates[model] = float(rate)
        if rate > 0 and (model not in self._threads or not self._threads[model].is_alive()):
            t = threading.Thread(target=self._send_loop, args=(model,), daemon=True)
            self._threads[model] = t
            t.start()

    def _send_loop(self, model: str) -> None:
        nxt = time.perf_counter()
        while not self._closed:
            r = self.rates.get(model, 0.0)
            if r <= 0:
                return
            with self._id_lock:
                self._next_id += 1
                rid = self._next_id
            line = (json.dumps({"model": model, "id": rid}) + "\n").encode()
            with self._wlock:
                self.sock.sendall(line)
            self.sent[model] = self.sent.get(model, 0) + 1
            nxt += 1.0 / r
            d = nxt - time.perf_counter()
            if d > 0:
                time.sleep(d)
            elif d < -1.0:      # fell far behind (rate raised): resynchronise
                nxt = time.perf_counter()

    def _read_loop(self) -> None:
        buf = b""
        while not self._closed:
            try:
                chunk = self.sock.recv(65536)
            except OSError:
                return
            if not chunk:
                return
            buf += chunk
            while b"\n" in buf:
                line, buf = buf.split(b"\n", 1)
                msg = json.loads(line)
                m = msg.get("model", "?")
                self.responses.setdefault(m, {}).setdefault(msg["status"], 0)
                self.responses[m][msg["status"]] += 1
                if "latency_ms" in msg:
                    self.latencies_ms.setdefault(m, []).append(msg["latency_ms"])

    def stats(self) -> Dict[str, dict]:
        out = {}
        for m in set(self.sent) | set(self.responses):
            lat = sorted(self.latencies_ms.get(m, []))
            out[m] = dict(rate=self.rates.get(m, 0.0), sent=self.sent.get(m, 0), responses=self.responses.get(m, {}),
                          p50_ms=lat[len(lat) // 2] if lat else None,
                          p99_ms=lat[min(len(lat) - 1, int(0.99 * len(lat)))] if lat else None)
        return out

    def close(self) -> None:
        self._closed = True
        for m in list(self.rates):
            self.rates[m] = 0.0
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=5555)
    a = ap.parse_args(argv)
    sim = RequestSimulator(a.host, a.port)
    print("commands: '<model> <rate>', 'stats', 'quit'", flush=True)
    for line in sys.stdin:
        parts = line.split()
        if not parts:
            continue
        if parts[0] == "quit":
            break
        if parts[0] == "stats":
            print(json.dumps(sim.stats(), indent=1), flush=True)
        elif len(parts) == 2:
            sim.set_rate(parts[0], float(parts[1]))
    sim.close()


if __name__ == "__main__":
    main()
