"""Typed flag registry (native, runtime/csrc/node_agent.cpp Config) with
``RDB_<NAME>`` environment override -- the counterpart of Ray's RAY_CONFIG
registry (src/ray/common/ray_config.h:72-77, ray_config_def.h).

    from ray_dynamic_batching_amd.utils import config
    config.get("health_check_timeout_s")   -> 30.0   (or $RDB_HEALTH_CHECK_TIMEOUT_S)
    config.define("my_flag", "int", 4, "help")
"""
from __future__ import annotations

from typing import Any, Dict

from .native import load_runtime

_CAST = {"int": int, "float": float, "bool": lambda v: v in ("1", "true"), "str": str}


def _typed(name: str, raw: str) -> Any:
    t = load_runtime().config_all()[name]["type"]
    return _CAST.get(t, str)(raw)


def get(name: str) -> Any:
    return _typed(name, load_runtime().config_get(name))


def set(name: str, value: Any) -> None:  # noqa: A001 - mirrors RayConfig API naming
    if isinstance(value, bool):
        value = "1" if value else "0"
    load_runtime().config_set(name, str(value))


def define(name: str, type_: str, default: Any, help_: str = "") -> Any:
    if isinstance(default, bool):
        default = "1" if default else "0"
    return _typed(name, load_runtime().config_define(name, type_, str(default), help_))


def all_flags() -> Dict[str, Dict[str, Any]]:
    return dict(load_runtime().config_all())
