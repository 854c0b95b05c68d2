"""TCP ingress + live-rate request simulator driving the SLO scheduler (the
fork's ZMQ simulator -> RequestHandle path, with results actually returned)."""
import os
import sys
import time

import torch

from ray_dynamic_batching_amd.models.mlp import MLP
from ray_dynamic_batching_amd.planner import synthetic_profile
from ray_dynamic_batching_amd.planner.scheduler import SLOScheduler
from ray_dynamic_batching_amd.serve.servable import TensorCodec
from ray_dynamic_batching_amd.serve.tcp_ingress import TCPIngress

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))
from request_simulator import RequestSimulator  # noqa: E402


def test_simulator_rates_drive_scheduler_through_tcp():
    prof = {"a": synthetic_profile(2, 0.1, 50, 1, batches=range(1, 33)),
            "b": synthetic_profile(3, 0.2, 80, 2, batches=range(1, 33))}
    codecs = {m: TensorCodec((32,), torch.float32, (8,), torch.float32) for m in prof}
    s = SLOScheduler(prof, {"a": 200.0, "b": 300.0}, {"a": MLP, "b": lambda: MLP(seed=1)}, codecs, num_gpus=2,
                     monitoring_interval=0.2, rate_window_s=0.5)
    ing = TCPIngress(s).start()
    sim = RequestSimulator("127.0.0.1", ing.port)
    try:
        s.start_monitoring()
        sim.set_rate("a", 150)
        sim.set_rate("b", 60)
        time.sleep(1.5)
        assert {m for n in s.slots if n for m in n.models()} == {"a", "b"}
        sim.set_rate("b", 0)            # live rate change: stop model b
        time.sleep(0.5)
        sent_b = sim.sent["b"]
        time.sleep(0.5)
        assert sim.sent["b"] == sent_b
        sim.set_rate("a", 0)
        t_end = time.time() + 10
        while time.time() < t_end and sum(sum(v.values()) for v in sim.responses.values()) < sum(sim.sent.values()):
            time.sleep(0.05)
        st = sim.stats()
        # every request is answered (served, or dropped as stale under the plan's duty cycle)
        for m in ("a", "b"):
            assert sum(st[m]["responses"].values()) == st[m]["sent"], st
            assert st[m]["responses"].get("ok", 0) > 0 and set(st[m]["responses"]) <= {"ok", "dropped"}
        assert len(s.changes) >= 1
    finally:
        sim.close()
        ing.stop()
        s.shutdown()
