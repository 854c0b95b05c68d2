"""ResNet-50 / ViT / Llama on the HIP kernels vs their eager PyTorch baselines,
and GPU serving through serve.model_deployment (process mode + native engine)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stem", ["fused", "three_kernels"])
def test_resnet50_hip_matches_torch(stem):
    from ray_dynamic_batching_amd.models.resnet import ResNet50

    m = ResNet50(device="cuda", backend="hip")
    m.stem_fused = stem == "fused"
    x = m.example_input(4, seed=1)
    lg = m.logits(x)
    m.backend = "torch"
    ref = m.logits(x)
    assert lg.shape == (4, 1000)
    assert torch.allclose(lg, ref, atol=3e-2, rtol=5e-2), (lg - ref).abs().max()
    m.backend = "hip"
    out = m(x)
    assert out.shape == (4, 10) and torch.all(out[:, :5] > 0)


def test_vit_hip_matches_torch():
    from ray_dynamic_batching_amd.models.vit import ViT, ViTConfig

    m = ViT(ViTConfig(layers=4), device="cuda", backend="hip")
    x = m.example_input(3, seed=2)
    lg = m._logits_hip(x)
    ref = m._logits_torch(x)
    assert torch.allclose(lg, ref, atol=3e-2, rtol=5e-2), (lg - ref).abs().max()


def test_llama_tp1_hip_matches_torch():
    from ray_dynamic_batching_amd.models.llama import LlamaConfig, LlamaTP

    m = LlamaTP(LlamaConfig.tiny(seq_len=128), device="cuda", backend="hip", init="full")
    ids = m.example_input(4, seed=3)
    xh = m.hidden_states(ids)
    m.backend = "torch"
    xr = m.hidden_states(ids)
    assert torch.allclose(xh.float(), xr.float(), atol=5e-2, rtol=5e-2), (xh.float() - xr.float()).abs().max()
    m.backend = "hip"
    out = m(ids)
    assert out.shape == (4, 2) and out.dtype == torch.int32


def test_serve_model_deployment_bert_on_gpu():
    from ray_dynamic_batching_amd import serve
    from ray_dynamic_batching_amd.models import factories

    fac = factories.bert_base(layers=2)
    d = serve.model_deployment(fac, "bert", max_batch_size=16, batch_wait_timeout_s=0.002,
                               ray_actor_options={"num_gpus": 1}, max_ongoing_requests=64)
    try:
        h = serve.run(d.bind(), mode="process")
        model = fac(device="cuda")
        ids = model.example_input(40, seed=4).cpu()
        outs = [h.remote(ids[i].numpy()) for i in range(40)]
        got = np.stack([o.result(timeout_s=60) for o in outs])
        ref = model(ids.cuda()).cpu().numpy()
        assert np.allclose(got, ref, atol=2e-2, rtol=2e-2)
        st = serve.status()["applications"]["default"]["deployments"]["bert"]
        assert st["replicas"][0]["batches"] >= 3
    finally:
        serve.shutdown()


def test_serve_gpu_replica_killer_restart(monkeypatch):
    """Chaos on the GPU path: the engine replica exits after 5 batches; the node
    agent restarts it (graph re-capture) and the router re-dispatches."""
    from ray_dynamic_batching_amd import serve
    from ray_dynamic_batching_amd.models import factories
    from ray_dynamic_batching_amd.serve.controller import get_controller

    monkeypatch.setenv("RDB_FAULT_KILL_AFTER_BATCHES", "5")
    fac = factories.bert_base(layers=2)
    d = serve.model_deployment(fac, "bert", max_batch_size=8, batch_wait_timeout_s=0.002,
                               ray_actor_options={"num_gpus": 1}, max_ongoing_requests=16,
                               health_check_timeout_s=60, max_request_retries=20)
    try:
        h = serve.run(d.bind(), mode="process")
        ids = np.random.default_rng(0).integers(1, 30000, size=(120, 128)).astype(np.int32)
        outs = [h.remote(ids[i]) for i in range(120)]
        got = [o.result(timeout_s=300) for o in outs]
        assert all(g.shape == (2,) for g in got)
        assert sum(p["restarts"] for p in get_controller().agent.list()) >= 1
    finally:
        serve.shutdown()


def test_engine_fault_drop_knob(monkeypatch):
    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification
    from ray_dynamic_batching_amd.runtime import job as rjob
    from ray_dynamic_batching_amd.runtime.engine import EngineRunner, SessionSpec

    monkeypatch.setenv("RDB_FAULT_DROP_EVERY", "4")
    m = BertForSequenceClassification(BertConfig.tiny(seq_len=64), device="cuda", backend="hip")
    name = rjob.unique_job_name("fdrop")
    j = rjob.Job(name, create=True, n_replicas=1, n_queues=1, n_clients=1, req_slot_bytes=64 * 4, cmp_slot_bytes=64)
    j.configure_queue(0, 0, 0, 1024, 0.0, True)
    runner = EngineRunner(name, 0, [SessionSpec(model=m, queue=0, max_batch=8, max_wait_s=0.001)]).build().start()
    try:
        c = rjob.Client(j)
        ids = m.example_input(100, seed=1).cpu()
        for i in range(100):
            c.submit(0, ids[i].numpy().tobytes())
        st = []
        import time
        t_end = time.time() + 60
        while len(st) < 100 and time.time() < t_end:
            st += [x[1] for x in c.poll(128, 0.5)]
        assert len(st) == 100 and st.count(int(rjob.Status.REPLICA_DIED)) == 25
    finally:
        runner.stop()
        j.close()


def _rel_err(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


def test_shufflenet_hip_matches_torch():
    from ray_dynamic_batching_amd.models.shufflenet import ShuffleNetV2

    m = ShuffleNetV2(device="cuda", backend="hip")
    x = m.example_input(4, seed=5)
    lg = m._logits_hip(x)
    ref = m._logits_torch(x)
    assert lg.shape == (4, 1000)
    assert _rel_err(lg, ref) < 3e-2, _rel_err(lg, ref)
    assert m(x).shape == (4, 10)


def test_efficientnet_v2s_hip_matches_torch():
    from ray_dynamic_batching_amd.models.efficientnet import EfficientNetV2S

    m = EfficientNetV2S(device="cuda", backend="hip")
    x = m.example_input(2, seed=6)
    lg = m._logits_hip(x)
    ref = m._logits_torch(x)
    assert lg.shape == (2, 1000)
    assert _rel_err(lg, ref) < 5e-2, _rel_err(lg, ref)


def test_slo_scheduler_engine_executor_colocates_two_models():
    """Config 5 in miniature through the planner: two models on one GPU, the
    native engine executes the Nexus plan (duty cycle, shares, batch sizes)."""
    import time

    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification
    from ray_dynamic_batching_amd.planner import synthetic_profile
    from ray_dynamic_batching_amd.planner.scheduler import SLOScheduler
    from ray_dynamic_batching_amd.serve.servable import TensorCodec

    def fac(seed):
        return lambda device: BertForSequenceClassification(BertConfig.tiny(seq_len=64), device=device,
                                                             backend="hip", seed=seed)
    m0 = fac(0)("cuda")
    codec = TensorCodec.for_model(m0)
    prof = {"a": synthetic_profile(0.3, 0.01, 50, 1, batches=(1, 2, 4, 8, 16, 32)),
            "b": synthetic_profile(0.3, 0.02, 50, 1, batches=(1, 2, 4, 8, 16, 32))}
    s = SLOScheduler(prof, {"a": 50.0, "b": 80.0}, {"a": fac(0), "b": fac(1)}, {"a": codec, "b": codec},
                     num_gpus=1, executor="engine", devices=[0], max_batch={"a": 32, "b": 32})
    try:
        # planned rates above the ~600 + 300 req/s the loop below offers
        s.check_and_update({"a": 900.0, "b": 450.0})
        node = s.slots[0]
        assert node is not None and set(node.models()) == {"a", "b"}
        ids = m0.example_input(8, seed=2).cpu()
        rids = {}
        for i in range(300):
            name = "a" if i % 3 else "b"
            rids[s.submit(name, ids[i % 8].numpy())] = (name, i % 8)
            time.sleep(0.001)
        got = {}
        t_end = time.time() + 60
        while len(got) < len(rids) and time.time() < t_end:
            for c in s.poll(512, 0.2):
                got[c[0]] = c
        assert len(got) == len(rids)
        ok = [c for c in got.values() if c[1] == 0]
        assert len(ok) >= 0.95 * len(rids)
        ref = m0(ids.cuda()).cpu().numpy()
        for rid, c in got.items():
            name, k = rids[rid]
            if c[1] == 0 and name == "a":
                assert np.allclose(np.frombuffer(c[7], dtype=np.float32), ref[k], atol=2e-2)
        st = s.get_stats()
        assert st["a"]["completed"] > 0 and st["b"]["completed"] > 0
    finally:
        s.shutdown()


def test_tp_replica_serves_llama_tp1_through_rings():
    import threading

    from ray_dynamic_batching_amd.models.llama import LlamaConfig, LlamaTP
    from ray_dynamic_batching_amd.runtime import job as rjob
    from ray_dynamic_batching_amd.runtime.tp_replica import TPReplica

    m = LlamaTP(LlamaConfig.tiny(seq_len=64), device="cuda", backend="hip", init="full")
    name = rjob.unique_job_name("tp")
    j = rjob.Job(name, create=True, n_replicas=1, n_queues=1, n_clients=2, req_slot_bytes=64 * 4, cmp_slot_bytes=64)
    j.configure_queue(0, 0, 0, 256, 0.0, True)
    try:
        rep = TPReplica(m, name, 0, 0, [1, 2, 4, 8]).capture()
        ids = m.example_input(20, seed=9).cpu()
        c = rjob.Client(j, 1)
        rids = {c.submit(0, ids[i].numpy().tobytes()): i for i in range(20)}
        got = {}
        while len(got) < 20:
            rep.step(0.01)
            for rid, st, q, ts, td, tr, kind, payload in c.poll(64, 0.0):
                assert st == 0
                got[rids[rid]] = np.frombuffer(payload, dtype=np.int32)
        ref = m(ids.cuda()).cpu().numpy()
        assert all(got[i][0] == ref[i][0] for i in range(20))
        assert rep.batches >= 3
    finally:
        j.close()


def test_engine_executor_moves_bert_between_gpus_under_load():
    """Planner load/unload on the native engine (reference: GPUWorker
    _check_for_updates, 293-project/src/scheduler.py:483-523): BERT moves
    slot 0 -> 1 -> 0 (two engines on this one GPU) while requests arrive.
    Arriving copies are captured beside the serving sessions, leaving copies
    drain, retire at a batch boundary and free their HBM; every request
    completes OK with the right logits; capture time and footprint are recorded."""
    import threading
    import time

    import torch

    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification
    from ray_dynamic_batching_amd.planner import synthetic_profile
    from ray_dynamic_batching_amd.planner.scheduler import SLOScheduler
    from ray_dynamic_batching_amd.serve.servable import TensorCodec

    def fac(device):
        return BertForSequenceClassification(BertConfig.tiny(seq_len=64), device=device, backend="hip", seed=3)

    m0 = fac("cuda")
    codec = TensorCodec.for_model(m0)
    prof = {"bert": synthetic_profile(0.3, 0.01, 50, 1, batches=(1, 2, 4, 8, 16)),
            "other": synthetic_profile(0.3, 0.01, 50, 1, batches=(1, 2, 4, 8, 16))}
    s = SLOScheduler(prof, {"bert": 500.0, "other": 500.0}, {"bert": fac, "other": fac},
                     {"bert": codec, "other": codec}, num_gpus=2, executor="engine", devices=[0, 0],
                     max_batch={"bert": 16, "other": 16})

    def plan(gpu):
        st = s.plan_state()
        sess = dict(model="bert", slo_ms=500.0, rate=200.0, batch=16, occupancy=0.5)
        st["slots"] = [None, None]
        st["slots"][gpu] = dict(duty_cycle=10.0, gpu_type="MI355X", gpu_mem=288.0, sessions=[sess])
        st["sessions"] = {"bert": dict(model="bert", slo_ms=500.0, rate=200.0, batch=16)}
        return st

    try:
        assert s.restore_plan(plan(0))
        ex = s.executors
        assert "bert" in ex[0].index and ex[0].capture_s["bert"] > 0 and ex[0].footprint["bert"] > 0
        ids = m0.example_input(8, seed=2).cpu()
        ref = m0(ids.cuda()).float().cpu().numpy()
        rids, stop = {}, threading.Event()

        def load():
            i = 0
            while not stop.is_set():
                rids[s.submit("bert", ids[i % 8].numpy())] = i % 8
                i += 1
                time.sleep(0.002)

        t = threading.Thread(target=load)
        t.start()
        mem = []
        try:
            for gpu in (1, 0):
                time.sleep(0.5)
                assert s.restore_plan(plan(gpu))
                torch.cuda.synchronize()
                mem.append(torch.cuda.memory_allocated())
            time.sleep(0.5)
        finally:
            stop.set()
            t.join()
        got = {}
        t_end = time.time() + 60
        while len(got) < len(rids) and time.time() < t_end:
            for c in s.poll(512, 0.2):
                got[c[0]] = c
        assert len(got) == len(rids) and len(rids) > 200
        assert all(c[1] == 0 for c in got.values()), sorted({c[1] for c in got.values()})
        for rid, c in got.items():
            assert np.allclose(np.frombuffer(c[7], dtype=np.float32), ref[rids[rid]], atol=2e-2)
        assert ex[0].unloads == 1 and ex[1].unloads == 1 and ex[0].loads == 2 and ex[1].loads == 1
        assert "bert" in ex[0].index and "bert" not in ex[1].index
        # one copy resident at the end: memory after the second move is not above
        # the first (the copy on slot 1 was freed, slot 0's re-captured)
        assert mem[1] <= mem[0] + 16 * 2**20, mem
        assert ex[1].resident_bytes() == 0 and ex[0].resident_bytes() > 0
    finally:
        s.shutdown()
