"""core.data: Ray Data's offline batch-inference surface (SURVEY.md §2.3,
``python/ray/data/dataset.py:391`` map_batches, ``_internal/compute.py:53``
ActorPoolStrategy) -- sources, lazy transforms, batch formats, re-batching,
callable-class UDFs on GPU-pinned actor pools (process and local mode), order
preservation, pool growth and error propagation."""
import os
import sys
import uuid

import cloudpickle
import numpy as np
import pytest

import ray_dynamic_batching_amd.core as ray
from ray_dynamic_batching_amd.core import data as rd

cloudpickle.register_pickle_by_value(sys.modules[__name__])


@pytest.fixture(params=["process", "local"])
def rt(request):
    ray.init(num_gpus=2, local_mode=request.param == "local", namespace="d" + uuid.uuid4().hex[:8])
    yield request.param
    ray.shutdown()


class Scale:
    """Stand-in for a model: constructed once per pool actor, records where it runs."""

    def __init__(self, k):
        import ray_dynamic_batching_amd.core as r

        self.k = k
        self.pid = os.getpid()
        self.gpus = ",".join(str(g) for g in r.get_gpu_ids())

    def __call__(self, batch):
        return {"id": batch["id"], "y": batch["id"] * self.k, "n": np.full(len(batch["id"]), len(batch["id"])),
                "gpu": np.asarray([self.gpus] * len(batch["id"]))}


class Boom:
    def __call__(self, batch):
        raise ValueError("bad batch")


def test_sources_transforms_and_formats():
    ds = rd.range(10)
    assert ds.count() == 10 and ds.take(3) == [{"id": 0}, {"id": 1}, {"id": 2}]
    out = (ds.map(lambda r: {"id": r["id"], "sq": r["id"] ** 2})
             .filter(lambda r: r["id"] % 2 == 0)
             .flat_map(lambda r: [r, r]))
    assert [r["sq"] for r in out.take_all()] == [0, 0, 4, 4, 16, 16, 36, 36, 64, 64]
    assert rd.from_items([1, 2, 3]).take_all() == [{"item": 1}, {"item": 2}, {"item": 3}]
    # function UDF, numpy batches of exactly batch_size (last short)
    sizes = []

    def f(b):
        sizes.append(len(b["id"]))
        return {"id": b["id"], "z": b["id"] + 1}

    assert [r["z"] for r in rd.range(10).map_batches(f, batch_size=4).take_all()] == list(range(1, 11))
    assert sizes == [4, 4, 2]
    # pandas format in and out, generator UDF
    pdf = rd.range(6).map_batches(lambda df: df.assign(w=df["id"] * 3), batch_format="pandas").to_pandas()
    assert list(pdf["w"]) == [0, 3, 6, 9, 12, 15]

    def gen(b):
        for i in b["id"]:
            yield {"id": np.asarray([i, i])}

    assert rd.range(3).map_batches(gen, batch_size=None).count() == 6
    batches = list(rd.range(7).iter_batches(batch_size=3))
    assert [len(b["id"]) for b in batches] == [3, 3, 1]
    assert len(list(rd.range(7).iter_batches(batch_size=3, drop_last=True))) == 2
    assert rd.range(100).limit(5).count() == 5 and rd.range(10).repartition(3).num_blocks() == 3
    assert rd.from_numpy(np.ones((4, 2)), column="x").take_batch(4)["x"].shape == (4, 2)
    assert set(rd.range(2).map(lambda r: {"a": 1.5, "b": "s"}).schema()) == {"a", "b"}
    with pytest.raises(ValueError):
        rd.range(3).map_batches(lambda b: {"id": b["id"], "bad": np.ones(2)}, batch_size=3).take_all()
    with pytest.raises(ValueError):
        rd.range(3).map_batches(Scale, fn_constructor_args=(2,))        # class UDF without a pool


def test_actor_pool_map_batches_on_gpus(rt):
    ds = rd.range(64).map_batches(Scale, batch_size=8, num_gpus=1, fn_constructor_args=(3,),
                                  compute=rd.ActorPoolStrategy(size=2))
    rows = ds.take_all()
    assert [r["id"] for r in rows] == list(range(64))                   # input order kept
    assert all(r["y"] == 3 * r["id"] and r["n"] == 8 for r in rows)
    assert sorted({str(r["gpu"]) for r in rows}) == ["0", "1"]          # one pool actor per GPU
    assert ray.available_resources().get("GPU", 0) == 2                 # the pool released its GPUs
    # pool growth from 1 to 2 actors under a full in-flight window; concurrency= tuple form
    grow = rd.range(40).map_batches(Scale, batch_size=4, num_gpus=1, fn_constructor_args=(1,),
                                    concurrency=(1, 2))
    assert [r["y"] for r in grow.take_all()] == list(range(40))
    # UDF errors surface in the consumer
    with pytest.raises(ray.RayTaskError):
        rd.range(8).map_batches(Boom, batch_size=4, compute=rd.ActorPoolStrategy(size=1)).take_all()


class BertPredictor:
    """A GPU pool actor: random-init BERT (seeded) on the HIP kernels, loaded once."""

    def __init__(self, layers):
        import torch

        from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification

        self.torch = torch
        self.m = BertForSequenceClassification(BertConfig(layers=layers), device="cuda:0", backend="hip", seed=7)

    def __call__(self, batch):
        torch = self.torch
        ids = torch.as_tensor(np.stack(batch["ids"]), dtype=torch.int32, device="cuda:0")
        with torch.no_grad():
            logits = self.m(ids).float().cpu().numpy()
        return {"row": batch["row"], "logits": logits}


@pytest.mark.gpu
def test_map_batches_bert_on_gpu_actor_pool():
    """Offline batch inference of BERT (HIP kernels) through a GPU-pinned pool
    actor process == the same seeded model run in this process."""
    import torch

    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification

    m = BertForSequenceClassification(BertConfig(layers=2), device="cuda:0", backend="hip", seed=7)
    ids = m.example_input(40, seed=3).cpu().numpy()
    ray.init(num_gpus=1, namespace="dg" + uuid.uuid4().hex[:8])
    try:
        ds = rd.from_items([{"row": i, "ids": ids[i]} for i in range(40)])
        out = ds.map_batches(BertPredictor, batch_size=16, num_gpus=1, fn_constructor_args=(2,),
                             compute=rd.ActorPoolStrategy(size=1)).take_all()
    finally:
        ray.shutdown()
    assert [r["row"] for r in out] == list(range(40))
    got = np.stack([r["logits"] for r in out])
    with torch.no_grad():
        ref = torch.cat([m(torch.as_tensor(ids[i:i + 16], device="cuda:0")).float().cpu()
                         for i in range(0, 40, 16)]).numpy()
    assert np.abs(got - ref).max() < 2e-2
