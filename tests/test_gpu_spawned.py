"""The reference topology on the GPU: ONE driver, ``TorchEstimator(num_workers=2)`` whose two
worker processes are spawned by the worker-group trainer (``_run_spawned``; reference
``python/raydp/torch/estimator.py:331-355`` -> Ray Train ``TorchTrainer``), each binding the
GPU, ingesting its equal shard into HBM and training on the fused HIP engine with the gradient
all-reduced over the one-shot xGMI path.

gpurun gives one MI355X, so both workers share it (``resources_per_worker={"GPU": 0.5}``) and
their process group bootstraps over gloo (two ranks on one device cannot form an RCCL ring);
the xGMI peer mapping between the two processes is the same code that runs across 8 GPUs.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(20, 64), nn.ReLU(), nn.BatchNorm1d(64), nn.Linear(64, 16), nn.ReLU(),
                         nn.Linear(16, 1))


def _fit(tmp_path, tag):
    import pandas as pd
    from raydp_amd.data import from_pandas
    from raydp_amd.torch import TorchEstimator
    rng = np.random.default_rng(0)
    x = rng.standard_normal((64 * 16, 20)).astype(np.float32)
    df = pd.DataFrame({f"f{i}": x[:, i] for i in range(20)})
    df["y"] = x[:, :4].sum(1) * 0.5 + 1.0
    model = _model()
    est = TorchEstimator(num_workers=2, resources_per_worker={"CPU": 1, "GPU": 0.5}, model=model,
                         optimizer=torch.optim.SGD(model.parameters(), lr=0.02, momentum=0.9), loss=nn.MSELoss(),
                         feature_columns=[f"f{i}" for i in range(20)], label_column="y", batch_size=64,
                         num_epochs=3, fused="on", shuffle_seed=5, storage_path=str(tmp_path / tag),
                         metrics_name=["MeanAbsoluteError"])
    res = est.fit(from_pandas(df))
    return est, res


def test_spawned_workers_train_fused_over_xgmi_and_stay_warm(runtime_local, tmp_path, monkeypatch):
    from raydp_amd.train import trainer as T
    monkeypatch.setenv("RAYDP_TRAIN_BACKEND", "gloo")
    est, res = _fit(tmp_path, "a")
    hist = [m for m in res.metrics_history if "train_loss" in m]
    assert [m["epoch"] for m in hist] == [0, 1, 2]
    assert hist[0]["engine"] == "fused_mlp_hip", hist[0]
    # batch 64: the persistent epoch with the per-tile gradient exchange inside the launch
    assert hist[0]["allreduce"] == "xgmi_tiles_in_launch", hist[0]
    assert hist[-1]["train_loss"] < hist[0]["train_loss"]
    assert len(T._GROUPS) == 1, "a group that finished cleanly is kept warm"
    group = next(iter(T._GROUPS._groups.values()))
    # the second fit of the same shape reuses the warm workers (no process start, no HIP init)
    est2, res2 = _fit(tmp_path, "b")
    assert next(iter(T._GROUPS._groups.values())) is group
    a = est.get_model().state_dict()
    b = est2.get_model().state_dict()
    for k in a:        # same data, same seeds, same reduction order: the same model
        torch.testing.assert_close(a[k].float(), b[k].float(), atol=0, rtol=0)
    # the same fit with the gradient on the process group (gloo) instead of xGMI
    monkeypatch.setenv("RAYDP_ALLREDUCE", "rccl")
    est3, res3 = _fit(tmp_path, "c")
    h3 = [m for m in res3.metrics_history if "train_loss" in m]
    assert h3[0]["allreduce"] == "torch.distributed:gloo", h3[0]
    # a different environment is a different group; the card's GPU share was held by the warm
    # group of the first shape, which was released to place this one
    assert len(T._GROUPS) == 1 and next(iter(T._GROUPS._groups.values())) is not group
    c = est3.get_model().state_dict()
    for k in a:
        if not a[k].dtype.is_floating_point:
            continue
        # the in-launch exchange and the process-group path differ in fp32 summation order only
        rel = float((a[k].float() - c[k].float()).abs().max()) / max(1e-6, float(c[k].float().abs().max()))
        assert rel < 1e-4, (k, rel)
    T.release_worker_groups()
    assert len(T._GROUPS) == 0


def test_warm_workers_survive_consecutive_graph_captured_fits(runtime_local, tmp_path, monkeypatch):
    """The torch-loop engine at world 2 captures its DDP step (xGMI buckets) into HIP graphs. A
    warm worker group runs the next fit in the same processes: the previous fit's graphs must be
    gone before the new capture (a graph destroyed mid-capture aborts the worker)."""
    import pandas as pd
    from raydp_amd.data import from_pandas
    from raydp_amd.torch import TorchEstimator
    from raydp_amd.train import trainer as T
    monkeypatch.setenv("RAYDP_TRAIN_BACKEND", "gloo")
    rng = np.random.default_rng(1)
    x = rng.standard_normal((64 * 12, 8)).astype(np.float32)
    df = pd.DataFrame({f"f{i}": x[:, i] for i in range(8)})
    df["y"] = np.tanh(x[:, :3].sum(1))
    groups, engines = [], []
    for tag, hidden in (("a", 16), ("b", 24)):        # a different model each fit
        torch.manual_seed(0)
        model = nn.Sequential(nn.Linear(8, hidden), nn.Tanh(), nn.Linear(hidden, 1))
        est = TorchEstimator(num_workers=2, resources_per_worker={"CPU": 1, "GPU": 0.5}, model=model,
                             optimizer=torch.optim.SGD(model.parameters(), lr=0.05), loss=nn.MSELoss(),
                             feature_columns=[f"f{i}" for i in range(8)], label_column="y", batch_size=64,
                             num_epochs=2, fused="off", shuffle_seed=3, storage_path=str(tmp_path / tag))
        res = est.fit(from_pandas(df))
        hist = [m for m in res.metrics_history if "train_loss" in m]
        engines.append(hist[0]["engine"])
        groups.append(next(iter(T._GROUPS._groups.values())))
        assert hist[-1]["train_loss"] < hist[0]["train_loss"]
    assert engines == ["torch_loop_hipgraph"] * 2, engines
    assert groups[0] is groups[1], "the second fit must run on the same warm workers (no restart)"
    T.release_worker_groups()


def test_streamed_ingest_trains_like_ingest_after_conversion(spark_on_ray_2_executors, tmp_path, monkeypatch):
    """fit_on_spark with one in-process worker DMAs each training block into HBM as its conversion
    task lands (engine stream_ingest); the model trains bit for bit as with the whole conversion
    ingested afterwards (blocks assembled in partition order)."""
    import pandas as pd
    from raydp_amd.torch import TorchEstimator
    from raydp_amd.torch.estimator import LAST_TIMINGS, STREAM_STATS
    rng = np.random.default_rng(1)
    x = rng.standard_normal((64 * 40, 20)).astype(np.float32)
    pdf = pd.DataFrame({f"f{i}": x[:, i] for i in range(20)})
    pdf["y"] = x[:, :4].sum(1) * 0.5 + 1.0
    states = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("RAYDP_STREAM_INGEST", mode)
        # a fresh DataFrame per fit (an already persisted one is handed out without a stage)
        df = spark_on_ray_2_executors.createDataFrame(pdf).repartition(8)
        model = _model()
        est = TorchEstimator(num_workers=1, model=model, optimizer=torch.optim.Adam(model.parameters(), lr=1e-3),
                             loss=nn.MSELoss(), feature_columns=[f"f{i}" for i in range(20)], label_column="y",
                             batch_size=64, num_epochs=2, fused="on", shuffle_seed=5,
                             storage_path=str(tmp_path / mode))
        est.fit_on_spark(df)
        states[mode] = {k: v.detach().cpu().clone() for k, v in est.get_model().state_dict().items()}
        assert "ingest" in LAST_TIMINGS
        assert (STREAM_STATS.get("blocks", 0) > 0) == (mode == "1"), dict(STREAM_STATS)
    for k in states["0"]:
        assert torch.equal(states["0"][k], states["1"][k]), k
