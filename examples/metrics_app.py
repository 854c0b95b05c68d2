"""Deployment that exports an application metric (utils.user_metrics.Counter)."""
from ray_dynamic_batching_amd import serve
from ray_dynamic_batching_amd.utils.user_metrics import Counter


@serve.deployment(num_replicas=1)
class Counting:
    def __init__(self):
        self.calls = Counter("app_calls_total", "calls handled by this replica")

    def __call__(self, x):
        self.calls.inc()
        return x + 1


app = Counting.bind()
