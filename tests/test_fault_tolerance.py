"""Trainer fault tolerance: a rank dies mid-fit, the worker group restarts from the newest
per-epoch checkpoint (model.pt + optim.pt + sched.pt) and finishes with the same model an
uninterrupted run produces (reference: FailureConfig(max_failures) at
python/raydp/torch/estimator.py:331-334). Also: TorchConfig / use_ccl select the backend."""
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

STEPS_PER_EPOCH = 4      # 400 rows, 2 ranks, batch 50


class KillingScheduler(torch.optim.lr_scheduler.LambdaLR):
    """Per-batch scheduler (decaying LR, so its state matters) that kills rank 1's process
    once, in the middle of epoch 3, unless the flag file exists."""

    def __init__(self, optimizer, flag):
        self.flag = None               # the base constructor already takes one step
        super().__init__(optimizer, lambda s: 0.97 ** s)
        self.flag = flag

    def state_dict(self):
        return {k: v for k, v in super().state_dict().items() if k != "flag"}

    def step(self, *a, **k):
        super().step(*a, **k)
        if not self.flag:
            return
        from raydp_amd.train import session
        rank = int(os.environ.get("RAYDP_TEST_KILL_RANK", "1"))
        if session.get_world_rank() == rank and self.last_epoch == 3 * STEPS_PER_EPOCH + 2 \
                and not os.path.exists(self.flag):
            open(self.flag, "w").close()
            if os.environ.get("RAYDP_TEST_KILL_MODE") == "raise":
                raise RuntimeError("injected failure")      # in-process worker (one GPU)
            os._exit(1)        # the process dies: no exception, no cleanup


def _sched_killing(optimizer, config):
    return KillingScheduler(optimizer, os.environ.get("RAYDP_TEST_KILL_FLAG"))


def _sched_plain(optimizer, config):
    return KillingScheduler(optimizer, None)


def _fit(tmp_path, creator, max_retries):
    import pandas as pd
    from raydp_amd.data import from_pandas
    from raydp_amd.torch import TorchEstimator
    rng = np.random.default_rng(0)
    x = rng.standard_normal((400, 3)).astype(np.float32)
    df = pd.DataFrame({"a": x[:, 0], "b": x[:, 1], "c": x[:, 2], "y": x @ np.array([1.0, -2.0, 0.5]) + 0.3})
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(3, 16), nn.ReLU(), nn.Linear(16, 1))
    est = TorchEstimator(num_workers=2, model=model, optimizer=torch.optim.Adam(model.parameters(), lr=0.02),
                         loss=nn.MSELoss(), feature_columns=["a", "b", "c"], label_column="y",
                         batch_size=50, num_epochs=6, use_gpu=False, storage_path=str(tmp_path),
                         lr_scheduler_creator=creator, checkpoint_frequency=1, fused="off", shuffle_seed=7)
    return est, est.fit(from_pandas(df), max_retries=max_retries)


def test_rank_killed_mid_fit_resumes_from_last_epoch_checkpoint(runtime_local, tmp_path, monkeypatch):
    flag = str(tmp_path / "killed")
    monkeypatch.setenv("RAYDP_TEST_KILL_FLAG", flag)     # spawned ranks inherit the environment
    est, res = _fit(tmp_path / "a", _sched_killing, max_retries=2)
    assert os.path.exists(flag), "the injected failure did not happen"
    assert res.restored_from, "the group did not restart from a checkpoint"
    epochs = [m["epoch"] for m in res.metrics_history if "train_loss" in m]
    # the failure hit epoch 3; the checkpoint after epoch 2 is the newest: resume at 3, not 0
    assert epochs == [3, 4, 5], epochs
    assert sorted(os.listdir(res.restored_from[-1])) == ["meta.json", "model.pt", "optim.pt", "sched.pt"]
    resumed = est.get_model()
    # the same fit without a failure
    est2, res2 = _fit(tmp_path / "b", _sched_plain, max_retries=0)
    assert not res2.restored_from
    assert [m["epoch"] for m in res2.metrics_history if "train_loss" in m] == list(range(6))
    clean = est2.get_model()
    for a, b in zip(resumed.parameters(), clean.parameters()):
        torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-5)
    last = [m for m in res.metrics_history if "train_loss" in m][-1]["train_loss"]
    last2 = [m for m in res2.metrics_history if "train_loss" in m][-1]["train_loss"]
    assert abs(last - last2) <= 1e-6 * max(1.0, abs(last2))


def test_torch_config_backend_selection():
    from raydp_amd.torch.config import TorchConfig
    from raydp_amd.train.trainer import _backend
    assert _backend(None, True) == "nccl" and _backend(None, False) == "gloo"
    assert _backend(TorchConfig(backend="ccl"), True) == "nccl"        # use_ccl -> RCCL on GPU
    assert _backend(TorchConfig(backend="ccl"), False) == "gloo"
    assert _backend(TorchConfig(backend="gloo"), True) == "gloo"


def test_use_ccl_reaches_the_trainer(runtime_local, tmp_path, monkeypatch):
    import pandas as pd
    from raydp_amd.data import from_pandas
    from raydp_amd.torch import TorchEstimator
    from raydp_amd.torch import estimator as E
    seen = {}
    real = E.TorchTrainer

    class T(real):
        def __init__(self, *a, torch_config=None, **kw):
            seen["cfg"] = torch_config
            super().__init__(*a, torch_config=torch_config, **kw)
    monkeypatch.setattr(E, "TorchTrainer", T)
    df = pd.DataFrame({"a": np.arange(20.0), "y": np.arange(20.0) * 2})
    model = nn.Linear(1, 1)
    est = TorchEstimator(num_workers=1, model=model, optimizer=torch.optim.SGD(model.parameters(), lr=1e-3),
                         loss=nn.MSELoss(), feature_columns=["a"], label_column="y", batch_size=5,
                         num_epochs=1, use_ccl=True, use_gpu=False, storage_path=str(tmp_path))
    est.fit(from_pandas(df))
    assert seen["cfg"] is not None and seen["cfg"].resolve(False) == "gloo"


_ = pytest


def _loop_dies_after_final_report(config):
    """Per-epoch checkpoints with meta.json, then rank 0's final model-only checkpoint, then
    rank 1 dies once -- after every report of the attempt."""
    import json
    from raydp_amd.train import Checkpoint, session
    rank = session.get_world_rank()
    start = 0
    ck = session.get_checkpoint()
    if ck is not None:
        with open(os.path.join(ck.path, "meta.json")) as f:
            start = json.load(f)["epoch"] + 1
    for epoch in range(start, 3):
        ckpt = None
        if rank == 0:
            d = session.staging_dir()
            with open(os.path.join(d, "meta.json"), "w") as f:
                json.dump({"epoch": epoch}, f)
            ckpt = Checkpoint(d, movable=True)
        session.report({"epoch": epoch, "start": start}, checkpoint=ckpt)
    if rank == 0:
        d = session.staging_dir()
        with open(os.path.join(d, "model.pt"), "wb") as f:
            f.write(b"final")
        session.report({"final": True, "start": start}, checkpoint=Checkpoint(d, movable=True))
    else:
        session.report({"final": True, "start": start})
    flag = config["flag"]
    if rank == 1 and not os.path.exists(flag):
        open(flag, "w").close()
        os._exit(1)


def test_rank_dying_after_the_final_report_resumes_from_the_last_epoch_checkpoint(runtime_local, tmp_path):
    from raydp_amd.train import FailureConfig, RunConfig, ScalingConfig, TorchTrainer
    flag = str(tmp_path / "died")
    tr = TorchTrainer(_loop_dies_after_final_report, train_loop_config={"flag": flag},
                      scaling_config=ScalingConfig(num_workers=2, use_gpu=False),
                      run_config=RunConfig(storage_path=str(tmp_path / "runs"),
                                           failure_config=FailureConfig(max_failures=1)))
    res = tr.fit()
    assert os.path.exists(flag)
    assert len(res.restored_from) == 1
    # the final model.pt of the failed attempt carries no meta.json: the retry resumes after
    # epoch 2 (nothing re-trained), not from the trained final model at epoch 0
    assert os.path.exists(os.path.join(res.restored_from[0], "meta.json"))
    finals = [m for m in res.metrics_history if m.get("final")]
    assert finals and finals[-1]["start"] == 3, res.metrics_history
