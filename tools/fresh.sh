# Refuse to start a GPU job whose native extensions are stale: load_ops() would
# otherwise rebuild them on the GPU box (minutes, and once per spawned process).
python3 - <<'PY' || { echo "STALE native build: run python -m ray_dynamic_batching_amd._build before gpurun" >&2; exit 9; }
import sys
from ray_dynamic_batching_amd import _build as b
stale = b._stale(b.ops_target(), b._deps(b._ops_sources(), [b.OPS_SRC, b.RT_SRC])) or \
        b._stale(b.runtime_target(), b._deps([b.RT_SRC / "runtime.cpp", b.RT_SRC / "node_agent.cpp"], [b.RT_SRC]))
sys.exit(1 if stale else 0)
PY
