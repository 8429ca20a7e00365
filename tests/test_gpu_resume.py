"""Fused HIP engine: a fit that fails mid-way resumes from the newest per-epoch checkpoint
(fp32 master weights, Adam moments + step restored into the device trainer) and ends with the
same model as an uninterrupted fit."""
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

from test_fault_tolerance import KillingScheduler

pytestmark = pytest.mark.gpu


def _sched(optimizer, config):
    return KillingScheduler(optimizer, os.environ.get("RAYDP_TEST_KILL_FLAG"))


def _fit(path, creator, retries):
    import pandas as pd
    from raydp_amd.data import from_pandas
    from raydp_amd.torch import TorchEstimator
    rng = np.random.default_rng(0)
    x = rng.standard_normal((64 * 4, 20)).astype(np.float32)
    df = pd.DataFrame({f"f{i}": x[:, i] for i in range(20)})
    df["y"] = x[:, :3].sum(1) + 0.5
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(20, 64), nn.ReLU(), nn.BatchNorm1d(64), nn.Linear(64, 32), nn.ReLU(),
                          nn.Linear(32, 1))
    est = TorchEstimator(num_workers=1, model=model, optimizer=torch.optim.Adam(model.parameters(), lr=3e-3),
                         loss=nn.MSELoss(), feature_columns=[f"f{i}" for i in range(20)], label_column="y",
                         batch_size=64, num_epochs=6, storage_path=str(path), lr_scheduler_creator=creator,
                         checkpoint_frequency=1, fused="on", shuffle_seed=3)
    return est, est.fit(from_pandas(df), max_retries=retries)


def test_fused_engine_resumes_from_epoch_checkpoint(runtime_local, tmp_path, monkeypatch):
    flag = str(tmp_path / "flag")
    monkeypatch.setenv("RAYDP_TEST_KILL_FLAG", flag)
    monkeypatch.setenv("RAYDP_TEST_KILL_MODE", "raise")
    monkeypatch.setenv("RAYDP_TEST_KILL_RANK", "0")
    est, res = _fit(tmp_path / "a", _sched, 2)
    assert os.path.exists(flag) and res.restored_from
    hist = [m for m in res.metrics_history if "train_loss" in m]
    assert hist[0]["engine"] == "fused_mlp_hip"
    assert [m["epoch"] for m in hist] == [3, 4, 5]
    monkeypatch.delenv("RAYDP_TEST_KILL_FLAG")
    est2, res2 = _fit(tmp_path / "b", _sched, 0)
    for a, b in zip(est.get_model().state_dict().values(), est2.get_model().state_dict().values()):
        torch.testing.assert_close(a.float(), b.float(), atol=0, rtol=0)
