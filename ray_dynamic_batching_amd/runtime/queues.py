"""One HIP hardware queue per replica-engine stream.

HIP maps streams onto a per-process pool of hardware queues, ``GPU_MAX_HW_QUEUES``
of them (default 4); once a process has more streams than queues, streams share
a queue and their kernels run in one FIFO.  A replica engine with C compute
streams also drives a copy stream (the H2D gather) and PyTorch's current
stream, so C + 2 queues keep every stream independent: with C = 3 on the
default 4 queues two streams collided and the three-stream BERT engine ran
28.0k req/s; with 8 queues the same engine ran 37.2-37.4k
(``profiles/hw_queues_compute_streams_r6.json``).  The value must be in the
environment before the HIP runtime initialises (bench.py sets it before it
imports torch, the Serve controller puts it in each replica's environment).
"""
from __future__ import annotations

import os
import warnings

HIP_DEFAULT_HW_QUEUES = 4
MAX_HW_QUEUES = 32          # never more (the cap this pool's launcher enforces as well)


def hw_queues_needed(compute_streams: int) -> int:
    """Queues for ``compute_streams`` compute streams + the copy stream + the
    current (null) stream, at least HIP's default."""
    return max(HIP_DEFAULT_HW_QUEUES, min(MAX_HW_QUEUES, int(compute_streams) + 2))


def ensure_hw_queues(compute_streams: int, env=None) -> int:
    """Raise GPU_MAX_HW_QUEUES in ``env`` (default: this process's environment)
    to what ``compute_streams`` needs; never lowers a larger setting.  Call it
    before anything initialises HIP.  Returns the value in effect."""
    env = os.environ if env is None else env
    need = hw_queues_needed(compute_streams)
    try:
        cur = int(env.get("GPU_MAX_HW_QUEUES", HIP_DEFAULT_HW_QUEUES))
    except ValueError:
        cur = HIP_DEFAULT_HW_QUEUES
    if cur < need:
        env["GPU_MAX_HW_QUEUES"] = str(need)
        return need
    return cur


def check_hw_queues(compute_streams: int) -> bool:
    """Warn when this (already initialised) process has fewer hardware queues
    than its engine's streams: they would share queues and serialise."""
    try:
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", HIP_DEFAULT_HW_QUEUES))
    except ValueError:
        cur = HIP_DEFAULT_HW_QUEUES
    need = hw_queues_needed(compute_streams)
    if cur < need:
        warnings.warn(f"{compute_streams} compute streams + copy + current stream need {need} HIP hardware queues; "
                      f"GPU_MAX_HW_QUEUES={cur}: streams share queues and serialise (set it before HIP starts, "
                      f"runtime/queues.py ensure_hw_queues)")
        return False
    return True
