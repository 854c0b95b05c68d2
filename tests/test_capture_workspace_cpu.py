"""ops.capture_splitk_workspace (the engine's per-compute-stream split-K
workspace for its graph captures): installed for the block only, nests, and is
thread-local -- a live capture on another thread never sees it.  Outside a
capture _private_splitk_ws ignores it (CPU: nothing is ever capturing)."""
import threading

import torch

from ray_dynamic_batching_amd import ops


def test_capture_workspace_scoping_and_threads():
    a, b = torch.zeros(16, dtype=torch.uint8), torch.zeros(16, dtype=torch.uint8)
    assert getattr(ops._cap_ws_local, "ws", None) is None
    seen = {}
    with ops.capture_splitk_workspace(a) as w:
        assert w is a and ops._cap_ws_local.ws is a
        with ops.capture_splitk_workspace(b):
            assert ops._cap_ws_local.ws is b
            t = threading.Thread(target=lambda: seen.update(other=getattr(ops._cap_ws_local, "ws", None)))
            t.start()
            t.join()
        assert ops._cap_ws_local.ws is a
    assert ops._cap_ws_local.ws is None
    assert seen["other"] is None
    try:
        with ops.capture_splitk_workspace(a):
            raise RuntimeError("capture failed")
    except RuntimeError:
        pass
    assert ops._cap_ws_local.ws is None            # restored on error
