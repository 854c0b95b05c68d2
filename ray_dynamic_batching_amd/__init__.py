"""ray_dynamic_batching_amd -- an MI355X-native dynamic-batching model server.

Capabilities of milind7777/ray-dynamic-batching (Ray Serve ``@serve.batch`` /
``DeploymentHandle`` API + the fork's Nexus-style SLO-aware multi-model
planner), re-designed for AMD Instinct MI355X (gfx950):

* ``serve``     -- Serve-compatible API: ``@serve.deployment``, ``@serve.batch``,
                   ``serve.run`` -> ``DeploymentHandle.remote()``.
* ``runtime``   -- shared-memory data plane (C++): rings, router, node agent.
* ``ops``       -- hand-written HIP/CDNA4 kernels (MFMA GEMM/conv, norms, attention).
* ``models``    -- BERT, ResNet-50, ViT, ShuffleNetV2, EfficientNetV2, Llama-3, MLP.
* ``parallel``  -- RCCL/xGMI collectives, tensor-parallel layers.
* ``planner``   -- squishy bin packing, rate tracking, re-planning.
* ``profiler``  -- batch-size sweep profiler (CSV contract of the fork).
* ``bench``     -- workload generators and result logging.
"""
# torch must be imported before the native extensions: it loads the HIP runtime
# (libamdhip64.so.7) that _rdb_ops then shares.
import torch  # noqa: F401

__version__ = "0.1.0"

from .utils.native import load_ops, load_runtime, native_available  # noqa: E402,F401
