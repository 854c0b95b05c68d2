"""``ray.state.actors()`` (reference: ``python/ray/_private/state.py``; used by the
fork's ``slo_viewer.py:184`` to find its SLO tracker actors by name)."""
from __future__ import annotations

import json
import os
from typing import Dict


def actors() -> Dict[str, dict]:
    from . import _pid_alive, _require_ctx

    ctx = _require_ctx()
    out = {}
    d = os.path.join(ctx.registry, "_actors")
    for fn in sorted(os.listdir(d)) if os.path.isdir(d) else []:
        try:
            with open(os.path.join(d, fn)) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        alive = rec.get("local") or _pid_alive(int(rec["pid"]))
        out[rec["actor_id"]] = {"ActorID": rec["actor_id"], "Name": rec.get("name") or "",
                                "ActorClassName": rec["class_name"], "State": "ALIVE" if alive else "DEAD",
                                "Pid": rec["pid"], "GPUs": rec.get("gpus", []),
                                "Detached": rec.get("detached", False)}
    return out
