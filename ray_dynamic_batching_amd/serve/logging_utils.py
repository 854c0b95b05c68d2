"""Serve logging: per-replica component logs and the per-request access log.

Reference: ``python/ray/serve/_private/logging_utils.py`` (component loggers,
JSON / TEXT encodings, ``configure_component_logger`` at :274) and the access
log line every replica writes per request (``serve/_private/replica.py``
:430-437: method, route / status, latency), configured by
``LoggingConfig(encoding, log_level, logs_dir, enable_access_log)`` on a
deployment or for a whole application via ``serve.run(logging_config=...)``.

Here every replica (local-mode thread or replica process) gets a logger
``ray.serve.replica.<app>.<deployment>.<index>`` writing to
``<logs_dir>/replica_<app>_<deployment>_<index>.log``; its records carry the
component attributes (deployment, replica id) and, for access-log records,
request id, method, status and latency.  In a replica PROCESS the user's own
``logging.getLogger("ray.serve")`` records go to the same file.  Servable
models on the native engine have no per-request Python step: their
per-request latency lives in the shm histograms (``serve.status()``,
Prometheus), and their replica log carries the engine's lifecycle messages.
"""
from __future__ import annotations

import json
import logging
import os
import tempfile
import time
from typing import Any, Dict, List, Optional, Union

from pydantic import BaseModel, field_validator

__all__ = ["LoggingConfig", "configure_replica_logger", "default_logs_dir", "AccessLog"]

_LEVELS = {"CRITICAL", "ERROR", "WARNING", "INFO", "DEBUG", "NOTSET"}
_ACCESS_FIELDS = ("request_id", "method", "route", "status", "latency_ms", "multiplexed_model_id")


class LoggingConfig(BaseModel):
    """Field names of Ray Serve's ``LoggingConfig``."""
    encoding: str = "TEXT"
    log_level: Union[int, str] = "INFO"
    logs_dir: Optional[str] = None
    enable_access_log: bool = True
    additional_log_standard_attrs: List[str] = []

    @field_validator("encoding")
    @classmethod
    def _enc(cls, v):
        v = str(v).upper()
        if v not in ("TEXT", "JSON"):
            raise ValueError(f"logging encoding must be 'TEXT' or 'JSON', got {v!r}")
        return v

    @field_validator("log_level")
    @classmethod
    def _lvl(cls, v):
        if isinstance(v, int):
            return v
        v = str(v).upper()
        if v not in _LEVELS:
            raise ValueError(f"invalid log_level {v!r}; one of {sorted(_LEVELS)}")
        return v

    def level(self) -> int:
        return self.log_level if isinstance(self.log_level, int) else logging.getLevelName(self.log_level)


def default_logs_dir() -> str:
    return os.environ.get("RDB_SERVE_LOGS_DIR", os.path.join(tempfile.gettempdir(), f"rdb_serve_logs_{os.getuid()}"))


def as_logging_config(v: Any) -> Optional[LoggingConfig]:
    if v is None or isinstance(v, LoggingConfig):
        return v
    if isinstance(v, dict):
        return LoggingConfig(**v)
    raise TypeError(f"logging_config must be a dict or LoggingConfig, got {type(v).__name__}")


class _TextFormatter(logging.Formatter):
    def __init__(self, component: Dict[str, str], extra_attrs: List[str]):
        super().__init__()
        self.component = component
        self.extra_attrs = extra_attrs

    def format(self, r: logging.LogRecord) -> str:
        t = time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(r.created)) + f",{int(r.msecs):03d}"
        head = f"{r.levelname} {t} {self.component['deployment']} {self.component['replica']}"
        rid = getattr(r, "request_id", None)
        if rid is not None:
            head += f" {rid}"
        msg = r.getMessage()
        extra = " ".join(f"{a}={getattr(r, a)}" for a in self.extra_attrs if hasattr(r, a))
        out = f"{head} -- {msg}" + (f" {extra}" if extra else "")
        if r.exc_info:
            out += "\n" + self.formatException(r.exc_info)
        return out


class _JsonFormatter(logging.Formatter):
    def __init__(self, component: Dict[str, str], extra_attrs: List[str]):
        super().__init__()
        self.component = component
        self.extra_attrs = extra_attrs

    def format(self, r: logging.LogRecord) -> str:
        d = dict(levelname=r.levelname, asctime=time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(r.created)),
                 created=r.created, logger=r.name, message=r.getMessage(), component_type="replica",
                 deployment=self.component["deployment"], replica=self.component["replica"],
                 application=self.component["application"])
        for a in _ACCESS_FIELDS + tuple(self.extra_attrs):
            if hasattr(r, a):
                d[a] = getattr(r, a)
        if r.exc_info:
            d["exc_text"] = self.formatException(r.exc_info)
        return json.dumps(d, default=str)


def configure_replica_logger(app: str, deployment: str, index: int, replica_id: str,
                             cfg: Optional[LoggingConfig], capture_user_logs: bool = False) -> logging.Logger:
    """The replica's component logger (handler + formatter per ``cfg``); with
    ``capture_user_logs`` (replica processes) the ``ray.serve`` logger the
    user's code logs to writes to the same file."""
    cfg = cfg or LoggingConfig()
    name = f"ray.serve.replica.{app}.{deployment}.{index}"
    lg = logging.getLogger(name)
    lg.setLevel(cfg.level())
    lg.propagate = False
    for h in list(lg.handlers):
        lg.removeHandler(h)
        h.close()
    d = cfg.logs_dir or default_logs_dir()
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"replica_{app}_{deployment}_{index}.log")
    h = logging.FileHandler(path)
    comp = dict(application=app, deployment=deployment, replica=replica_id)
    fmt = _JsonFormatter if cfg.encoding == "JSON" else _TextFormatter
    h.setFormatter(fmt(comp, list(cfg.additional_log_standard_attrs)))
    lg.addHandler(h)
    lg.log_path = path
    if capture_user_logs:
        user = logging.getLogger("ray.serve")
        user.setLevel(cfg.level())
        user.addHandler(h)
    return lg


class AccessLog:
    """One line per request (reference replica.py:430-437), if enabled."""

    def __init__(self, logger: Optional[logging.Logger], enabled: bool):
        self.logger = logger
        self.enabled = bool(enabled and logger is not None)

    def record(self, meta, status: str, latency_s: float, route: str = "") -> None:
        if not self.enabled:
            return
        ms = latency_s * 1e3
        self.logger.info("%s %s %s %.1fms", "CALL" if not route else "HTTP", meta.method_name if not route else route,
                         status, ms,
                         extra=dict(request_id=meta.request_id, method=meta.method_name, route=route,
                                    status=status, latency_ms=round(ms, 3),
                                    multiplexed_model_id=meta.multiplexed_model_id or ""))
