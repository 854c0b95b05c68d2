"""BASELINE config 1: 2-layer MLP on CPU, 2 replicas, dyn-batch <= 4 / 10 ms.

    python -m ray_dynamic_batching_amd.serve.cli run examples.mlp_app:app --mode local --duration 5
"""
import torch

from ray_dynamic_batching_amd import serve
from ray_dynamic_batching_amd.models.mlp import MLP


@serve.deployment(num_replicas=2, max_ongoing_requests=16)
class MLPDeployment:
    def __init__(self, d_in: int = 32):
        self.model = MLP(d_in=d_in)

    @serve.batch(max_batch_size=4, batch_wait_timeout_s=0.010)
    async def __call__(self, xs):
        return list(self.model(torch.stack([torch.as_tensor(x) for x in xs])).unbind(0))


app = MLPDeployment.bind()


def build(args):
    return MLPDeployment.bind(**args)
