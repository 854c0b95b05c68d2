"""Compiled-DAG tensor transport on the GPU (core/channel.py TensorRing): GPU
tensors of a ``with_tensor_transport()`` node go HBM -> HBM into the reader's
device ring (exported with HIP IPC to the writer's process) and only
descriptors travel through the shm ring.  Two actors share the one GPU of the
test box (num_gpus=0.5 each)."""
import sys
import uuid

import cloudpickle
import pytest
import torch

import ray_dynamic_batching_amd.core as ray
from ray_dynamic_batching_amd.core.dag import InputNode

pytestmark = pytest.mark.gpu
cloudpickle.register_pickle_by_value(sys.modules[__name__])


class GpuStage:
    def make(self, n):
        import torch

        x = torch.arange(n, dtype=torch.float32, device="cuda").view(-1, 64)
        return {"x": x, "h": torch.full((5,), 2.0)}          # one GPU tensor, one host tensor

    def consume(self, d):
        assert d["x"].is_cuda and not d["h"].is_cuda
        return d["x"].double().sum(dim=1) * d["h"][0]        # stays on the GPU


@pytest.fixture(params=["process", "local"])
def rt(request):
    ray.init(num_gpus=1, local_mode=request.param == "local", namespace="g" + uuid.uuid4().hex[:8])
    yield request.param
    ray.shutdown()


def test_compiled_dag_device_ring(rt):
    A = ray.remote(num_gpus=0.5)(GpuStage)
    a, b = A.remote(), A.remote()
    with InputNode() as inp:
        out = b.consume.bind(a.make.bind(inp).with_tensor_transport()).with_tensor_transport()
    cd = out.experimental_compile(_max_inflight_executions=4, _buffer_size_bytes=1 << 20)
    n = 64 * 1024                                            # 256 KB of GPU tensor per value
    refs = [cd.execute(n + 64 * i) for i in range(10)]
    for i, r in enumerate(refs):
        y = ray.get(r, timeout=120)
        assert y.is_cuda and y.shape == ((n + 64 * i) // 64,)
        ref = torch.arange(n + 64 * i, dtype=torch.float64, device="cuda").view(-1, 64).sum(dim=1) * 2.0
        assert torch.equal(y, ref)
    cd.teardown()
