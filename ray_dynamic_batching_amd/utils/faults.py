"""Fault injection knobs (reference: RAY_testing_rpc_failure,
src/ray/rpc/rpc_chaos.cc:35-80, and the killer actors of
python/ray/_private/test_utils.py:1433-1600).

All knobs are flags of the native registry (utils/config.py), so they are set
with environment variables and inherited by replica processes:

  RDB_FAULT_DROP_EVERY=N        replica fails every Nth request with
                                REPLICA_DIED (router re-dispatches it)
  RDB_FAULT_DELAY_BATCH_US=U    replica sleeps U us before each batch
  RDB_FAULT_KILL_AFTER_BATCHES=N replica process exits (code 137) after N
                                batches -- the agent must restart it
  RDB_FAULT_REJECT_EVERY=N      router treats every Nth submit as rejected
                                (back-pressure / retry path)

The GPU replica engine (ops/csrc/engine.cpp) reads the same variables.
"""
from __future__ import annotations

import os
import threading
import time


def _knob(name: str) -> int:
    try:
        from . import config

        return int(config.get(name))
    except Exception:  # runtime extension unavailable: fall back to the env var
        return int(os.environ.get("RDB_" + name.upper(), "0") or 0)


class FaultInjector:
    def __init__(self):
        self.drop_every = _knob("fault_drop_every")
        self.delay_batch_us = _knob("fault_delay_batch_us")
        self.kill_after_batches = _knob("fault_kill_after_batches")
        self.reject_every = _knob("fault_reject_every")
        self._n_req = 0
        self._n_batch = 0
        self._n_submit = 0
        self._lock = threading.Lock()

    @property
    def active(self) -> bool:
        return bool(self.drop_every or self.delay_batch_us or self.kill_after_batches or self.reject_every)

    def drop_request(self) -> bool:
        if not self.drop_every:
            return False
        with self._lock:
            self._n_req += 1
            return self._n_req % self.drop_every == 0

    def before_batch(self) -> None:
        if self.delay_batch_us:
            time.sleep(self.delay_batch_us / 1e6)
        if self.kill_after_batches:
            with self._lock:
                self._n_batch += 1
                n = self._n_batch
            if n > self.kill_after_batches:
                os._exit(137)   # simulated crash: no cleanup, no completions

    def reject_submit(self) -> bool:
        if not self.reject_every:
            return False
        with self._lock:
            self._n_submit += 1
            return self._n_submit % self.reject_every == 0


_GLOBAL = None


def injector() -> FaultInjector:
    global _GLOBAL
    if _GLOBAL is None:
        _GLOBAL = FaultInjector()
    return _GLOBAL


def reset() -> FaultInjector:
    """Re-read the knobs (tests change the environment between cases)."""
    global _GLOBAL
    from . import config

    for name in ("fault_drop_every", "fault_delay_batch_us", "fault_kill_after_batches", "fault_reject_every"):
        try:
            config.set(name, os.environ.get("RDB_" + name.upper(), "0") or "0")
        except Exception:
            pass
    _GLOBAL = FaultInjector()
    return _GLOBAL
