"""TorchEstimator on Spark data (port of the reference's tests/test_torch.py and
tests/test_torch_sequential.py). CPU path: gloo workers spawned by the trainer."""
import os
import shutil

import pytest
import torch

import raydp  # noqa: F401
import pyspark.pandas as ps
from raydp.torch import TorchEstimator
from raydp.utils import random_split


@pytest.mark.parametrize("use_fs_directory", [True, False])
def test_torch_estimator(spark_on_ray_small, use_fs_directory, tmp_path):
    _ = spark_on_ray_small
    df = ps.range(0, 100000)
    df["x"] = df["id"] + 100
    df["y"] = df["id"] + 1000
    df["z"] = df["x"] * 3 + df["y"] * 4 + 5
    df = df.astype("float")
    train_df, test_df = random_split(df, [0.7, 0.3])

    class LinearModel(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.linear = torch.nn.Linear(2, 1)

        def forward(self, x):
            return self.linear(x)

    model = LinearModel()
    optimizer = torch.optim.Adam(model.parameters())
    loss = torch.nn.MSELoss()

    def lr_scheduler_creator(optimizer, config):
        return torch.optim.lr_scheduler.MultiStepLR(optimizer, milestones=[150, 250, 350], gamma=0.1)

    estimator = TorchEstimator(num_workers=2, model=model, optimizer=optimizer, loss=loss,
                               lr_scheduler_creator=lr_scheduler_creator, feature_columns=["x", "y"],
                               feature_types=torch.float, label_column="z", label_type=torch.float,
                               batch_size=1000, num_epochs=2, use_gpu=False)
    if use_fs_directory:
        d = str(tmp_path / "test_torch")
        estimator.fit_on_spark(train_df, test_df, fs_directory="file://" + d)
    else:
        estimator.fit_on_spark(train_df, test_df)
    model = estimator.get_model()
    result = model(torch.Tensor([[0, 0], [1, 1]]))
    assert result.shape == (2, 1)
    hist = estimator.results.metrics_history
    assert any("train_loss" in h for h in hist)


def test_torch_estimator_sequential(spark_on_ray_small):
    customers = [(1, "James", 21, 6), (2, "Liz", 25, 8), (3, "John", 31, 6), (4, "Jennifer", 45, 7),
                 (5, "Robert", 41, 5), (6, "Sandra", 45, 8)]
    df = spark_on_ray_small.createDataFrame(customers, ["cID", "name", "age", "grade"])
    model = torch.nn.Sequential(torch.nn.Linear(1, 2), torch.nn.Linear(2, 1))
    optimizer = torch.optim.Adam(model.parameters())
    loss = torch.nn.MSELoss()
    estimator = TorchEstimator(model=model, optimizer=optimizer, loss=loss, num_workers=3, num_epochs=5,
                               feature_columns=["age"], feature_types=torch.float, label_column="grade",
                               label_type=torch.float, batch_size=1)
    estimator.fit_on_spark(df)
    assert estimator.get_model()(torch.tensor([[30.0]])).shape == (1, 1)


_ = (os, shutil)


def test_fused_trainer_rejects_mismatched_operands_on_host():
    """The fused kernels index rows without bounds checks: shape errors must stop on the host."""
    import torch.nn as nn
    from raydp_amd.models.mlp_spec import extract_mlp_spec
    from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
    m = nn.Sequential(nn.Linear(4, 8), nn.ReLU(), nn.Linear(8, 1))
    tr = FusedMLPTrainer(extract_mlp_spec(m), optimizer_config(torch.optim.Adam(m.parameters())),
                         loss_code(nn.MSELoss()), 16, "cpu", layout_only=True)
    feats = torch.zeros(32, tr.feat_k, dtype=torch.bfloat16)
    labels = torch.zeros(32, 1)
    tr._check_operands(feats, labels, 32)
    with pytest.raises(ValueError):
        tr._check_operands(feats, labels, 64)          # more rows than the matrix holds
    with pytest.raises(ValueError):
        tr._check_operands(feats.float(), labels, 32)  # wrong dtype
    with pytest.raises(ValueError):
        tr._check_operands(feats, labels, 32, perm=torch.arange(16, dtype=torch.int32))


def _tiny_df(spark, n=512):
    import numpy as np
    rng = np.random.default_rng(0)
    x = rng.normal(size=(n, 2))
    rows = [(float(a), float(b), float(3 * a - 2 * b + 1)) for a, b in x]
    return spark.createDataFrame(rows, ["x", "y", "z"])


def _fit_linear(df, **kw):
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(2, 8), torch.nn.ReLU(), torch.nn.Linear(8, 1))
    est = TorchEstimator(num_workers=1, model=model, optimizer=torch.optim.Adam(model.parameters(), lr=1e-2),
                         loss=torch.nn.MSELoss(), feature_columns=["x", "y"], feature_types=torch.float,
                         label_column="z", label_type=torch.float, batch_size=64, num_epochs=2,
                         use_gpu=False, shuffle_seed=7, **kw)
    est.fit_on_spark(df)
    return est


def test_overlapped_conversion_matches_sequential(spark_on_ray_small, monkeypatch):
    """fit_on_spark builds the engine while the conversion stage runs (Dataset.deferred); the
    trained model is the same as with the conversion finished first."""
    from raydp_amd.torch.estimator import LAST_TIMINGS
    df = _tiny_df(spark_on_ray_small)
    monkeypatch.setenv("RAYDP_OVERLAP_CONVERSION", "0")
    a = _fit_linear(df)
    assert "conversion_wait" not in LAST_TIMINGS
    monkeypatch.setenv("RAYDP_OVERLAP_CONVERSION", "1")
    b = _fit_linear(df)
    assert "conversion_wait" in LAST_TIMINGS and "etl_and_conversion_concurrent" in LAST_TIMINGS
    sa, sb = a.get_model().state_dict(), b.get_model().state_dict()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    ha = [h["train_loss"] for h in a.results.metrics_history if "train_loss" in h]
    hb = [h["train_loss"] for h in b.results.metrics_history if "train_loss" in h]
    assert ha == hb


def test_deferred_conversion_failure_is_raised_once(spark_on_ray_small, monkeypatch):
    """A conversion that fails surfaces as its own error from fit_on_spark, without the
    trainer's worker-group restarts (max_retries) rerunning the workers."""
    from pyspark.sql.functions import col, udf
    from raydp_amd.data.dataset import Dataset, DeferredDatasetError
    from raydp_amd.train.trainer import TrainingFailedError
    monkeypatch.setenv("RAYDP_OVERLAP_CONVERSION", "1")

    @udf("double")
    def boom(v):
        raise ValueError("bad row")
    df = _tiny_df(spark_on_ray_small, 64).withColumn("x", boom(col("x")))
    calls = []

    def model_creator(config):
        calls.append(1)
        return torch.nn.Linear(2, 1)
    est = TorchEstimator(num_workers=1, model=model_creator,
                         optimizer=lambda m, c: torch.optim.SGD(m.parameters(), lr=0.1),
                         loss=torch.nn.MSELoss(), feature_columns=["x", "y"], feature_types=torch.float,
                         label_column="z", label_type=torch.float, batch_size=16, num_epochs=1,
                         use_gpu=False)
    with pytest.raises(Exception) as ei:
        est.fit_on_spark(df, max_retries=3)
    assert not isinstance(ei.value, (TrainingFailedError, DeferredDatasetError))
    assert len(calls) == 1
    # a deferred dataset reports the same failure on every access
    import concurrent.futures as cf
    f = cf.Future()
    f.set_exception(KeyError("k"))
    ds = Dataset.deferred(f)
    for _ in range(2):
        with pytest.raises(DeferredDatasetError) as e2:
            ds.count()
        assert isinstance(e2.value.original, KeyError)


def test_spawned_workers_build_their_engines_before_their_shards_exist(spark_on_ray_small, monkeypatch):
    """num_workers=2 (spawned ranks, gloo): with the conversion overlapped, every rank starts its
    loop at once and receives its shard when the stage is done (deliver_shards) -- same model as
    the conversion finished first."""
    from raydp_amd.train import trainer as T
    seen = []
    orig = T.DataParallelTrainer._deferred_datasets

    def spy(self, world):
        v = orig(self, world)
        seen.append(v)
        return v
    monkeypatch.setattr(T.DataParallelTrainer, "_deferred_datasets", spy)
    # the overlapped fit sends every rank its fit BEFORE the conversion stage starts (the started
    # hook fires, then the stage runs), and never waits out the hook's 30 s backstop
    import time as _t
    events = []
    fire = T._fire_started

    def fire_spy():
        events.append(("fired", _t.perf_counter()))
        fire()
    monkeypatch.setattr(T, "_fire_started", fire_spy)
    conv = TorchEstimator._convert_via_store

    def conv_spy(self, *a, **k):
        events.append(("stage", _t.perf_counter()))
        return conv(self, *a, **k)
    monkeypatch.setattr(TorchEstimator, "_convert_via_store", conv_spy)
    df = _tiny_df(spark_on_ray_small)
    outs, walls = [], []
    for ov in ("0", "1"):
        monkeypatch.setenv("RAYDP_OVERLAP_CONVERSION", ov)
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(2, 8), torch.nn.ReLU(), torch.nn.Linear(8, 1))
        est = TorchEstimator(num_workers=2, model=model, optimizer=torch.optim.Adam(model.parameters(), lr=1e-2),
                             loss=torch.nn.MSELoss(), feature_columns=["x", "y"], feature_types=torch.float,
                             label_column="z", label_type=torch.float, batch_size=32, num_epochs=2,
                             use_gpu=False, shuffle_seed=7, drop_last=True)
        del events[:]
        t0 = _t.perf_counter()
        est.fit_on_spark(df)
        walls.append(_t.perf_counter() - t0)
        outs.append(est)
    assert seen == [False, True], seen
    kinds = [k for k, _ in events]          # (the overlapped, warm-group fit)
    assert "fired" in kinds and "stage" in kinds and kinds.index("fired") < kinds.index("stage"), events
    assert walls[1] < 20.0, walls
    sa, sb = outs[0].get_model().state_dict(), outs[1].get_model().state_dict()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def test_spawned_deferred_conversion_failure_is_raised_once(spark_on_ray_small, monkeypatch):
    """The deferred-shard path at num_workers=2: a failing conversion reaches the caller as its
    own error, not as a worker-group failure with restarts."""
    from pyspark.sql.functions import col, udf
    from raydp_amd.data.dataset import DeferredDatasetError
    from raydp_amd.train.trainer import TrainingFailedError
    monkeypatch.setenv("RAYDP_OVERLAP_CONVERSION", "1")

    @udf("double")
    def boom(v):
        raise ValueError("bad row")
    df = _tiny_df(spark_on_ray_small, 64).withColumn("x", boom(col("x")))
    est = TorchEstimator(num_workers=2, model=lambda c: torch.nn.Linear(2, 1),
                         optimizer=lambda m, c: torch.optim.SGD(m.parameters(), lr=0.1),
                         loss=torch.nn.MSELoss(), feature_columns=["x", "y"], feature_types=torch.float,
                         label_column="z", label_type=torch.float, batch_size=16, num_epochs=1,
                         use_gpu=False)
    with pytest.raises(Exception) as ei:
        est.fit_on_spark(df, max_retries=3)
    assert not isinstance(ei.value, (TrainingFailedError, DeferredDatasetError)), repr(ei.value)
    assert "bad row" in str(ei.value)


def test_one_worker_through_a_spawned_actor(spark_on_ray_small, monkeypatch):
    """``spark.ray.mi355x.train_inprocess`` off: a one-worker fit runs in a spawned worker actor
    (Ray Train's topology, the hop every N > 1 fit pays) and trains like the in-process loop."""
    from raydp_amd.train import session
    monkeypatch.setenv("RAYDP_TRAIN_INPROCESS", "0")
    df = spark_on_ray_small.createDataFrame([(float(i), 2.0 * i + 1.0) for i in range(64)], ["x", "y"])
    pids = []

    def fn(config):
        session.report({"pid": os.getpid(), "world": session.get_world_size()})
    from raydp_amd.train.trainer import TorchTrainer
    from raydp_amd.train.config import ScalingConfig
    res = TorchTrainer(fn, scaling_config=ScalingConfig(num_workers=1, use_gpu=False)).fit()
    pids.append(res.metrics["pid"])
    assert res.metrics["world"] == 1 and pids[0] != os.getpid()
    model = torch.nn.Linear(1, 1)
    est = TorchEstimator(num_workers=1, model=model, optimizer=torch.optim.Adam(model.parameters(), lr=0.1),
                         loss=torch.nn.MSELoss(), feature_columns=["x"], feature_types=torch.float,
                         label_column="y", label_type=torch.float, batch_size=16, num_epochs=2, use_gpu=False)
    est.fit_on_spark(df)
    assert any("train_loss" in h for h in est.results.metrics_history)


def test_persist_stage_reports_every_block_as_it_lands(spark_on_ray_2_executors):
    """The block hook of a persist stage (what the fused engine's streamed ingest consumes) sees
    every partition once, with the object the final dataset references."""
    from raydp_amd.spark import cluster as C
    from raydp_amd.spark.dataset import spark_dataframe_to_ray_dataset
    df = _tiny_df(spark_on_ray_2_executors, n=2000).repartition(6)
    seen = []
    C.set_block_hook(lambda i, oid, node_id, rows, ex: seen.append((i, oid, rows)))
    try:
        ds = spark_dataframe_to_ray_dataset(df)
    finally:
        C.set_block_hook(None)
    assert sorted(i for i, _, _ in seen) == list(range(ds.num_blocks()))
    by_i = {i: (oid, rows) for i, oid, rows in seen}
    assert [by_i[i][0] for i in range(ds.num_blocks())] == [b.id for b in ds._blocks]
    assert sum(r for _, r in by_i.values()) == 2000
