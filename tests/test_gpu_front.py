"""Embedding-front fused trainer (csrc/hip/mlp_core.h load_front / front_backward): the stroke
tutorial's NET_Model (per-column nn.Embedding lookups + dense columns -> BN-MLP; reference
tutorials/pytorch_example.ipynb cell 32) trained by the fused HIP kernels, against plain
PyTorch fp32 and a bf16-operand emulation of the same step."""
import copy
import os
import sys

import pytest
import torch
import torch.nn as nn

from tests.test_gpu_kernels import _norm_ratio, _relerr, emulate

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tutorials"))
from stroke import NET_Model  # noqa: E402

CARD = {0: 2, 2: 2, 3: 2, 4: 2, 5: 5, 6: 2, 9: 4, 10: 5}   # raw column -> num_embeddings


def _data(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, 11, generator=g) * 1.5
    for c, k in CARD.items():
        X[:, c] = torch.randint(0, k, (n,), generator=g).float()
    Y = (torch.rand(n, 1, generator=g) < 0.3).float()
    return X, Y


def _trainer(model, loss, batch, acc_thr=0.5):
    from raydp_amd.models.mlp_spec import extract_mlp_spec
    from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    spec = extract_mlp_spec(model)
    assert spec is not None and spec.front is not None and spec.raw_features == 11
    return FusedMLPTrainer(spec, optimizer_config(opt), loss_code(loss), batch, torch.device("cuda"),
                           acc_thr=acc_thr)


def _feats(tr, X):
    f = torch.zeros(X.shape[0], tr.feat_k, dtype=torch.bfloat16)
    f[:, :11] = X.to(torch.bfloat16)
    return f.cuda()


@pytest.mark.parametrize("nvalid", [64, 45])
@pytest.mark.parametrize("loss", [nn.SmoothL1Loss(), nn.MSELoss()])
def test_front_one_step_matches_torch(nvalid, loss):
    torch.manual_seed(0)
    model = NET_Model(11)
    ref = copy.deepcopy(model).cuda().train()
    emu = copy.deepcopy(model).cuda().train()
    tr = _trainer(model, loss, 64)
    X, Y = _data(nvalid)
    g = tr.forward_backward(_feats(tr, X), Y.cuda(), nvalid).clone()
    m = tr._read_metrics()
    xin = X.to(torch.bfloat16).float().cuda()
    out = ref(xin)
    loss(out, Y.cuda()).backward()
    out_e = emulate(emu, xin)
    le = loss(out_e, Y.cuda())
    le.backward()
    assert abs(m["loss"] - le.item()) / max(abs(le.item()), 1e-6) < 2e-3, (m, le.item())
    # accuracy: (pred > 0.5) == label; predictions within rounding of the threshold may differ
    acc_e = float(((out_e.detach() > 0.5).long() == Y.cuda().long()).float().mean())
    assert abs(m["acc"] - acc_e) <= 1.5 / nvalid, (m["acc"], acc_e)
    gmap = tr.unflatten(g)
    rmods, emods = dict(ref.named_modules()), dict(emu.named_modules())
    seen_emb = 0
    for name, mod in model.named_modules():
        for attr in ("weight", "bias"):
            key = (id(mod), attr)
            if key not in gmap:
                continue
            e_emu = _relerr(gmap[key], getattr(emods[name], attr).grad)
            e_fp32 = _relerr(gmap[key], getattr(rmods[name], attr).grad)
            assert e_emu < 2e-2, (name, attr, e_emu)
            # against fp32: at most the bf16-operand cost itself (emulation vs fp32 on the same
            # inputs; large for embedding rows, whose gradient sums dX over the 2-5 rows sharing an
            # id with heavy cancellation) plus the emulation tolerance (triangle inequality)
            bf16_cost = _relerr(getattr(emods[name], attr).grad, getattr(rmods[name], attr).grad)
            tol = 2e-2 * _norm_ratio(getattr(emods[name], attr).grad, getattr(rmods[name], attr).grad)
            assert e_fp32 <= bf16_cost + tol + 1e-6, (name, attr, e_fp32, bf16_cost)
            seen_emb += isinstance(mod, nn.Embedding)
    assert seen_emb == 8


def test_front_training_tracks_torch_and_is_deterministic():
    """Several epochs of fused steps (launch-per-step loop: optimizer kernel between steps updates
    the tables the next step gathers) end close to torch's fp32 run; two runs are identical."""
    from raydp_amd.ops.fused_mlp import FusedMLPTrainer  # noqa: F401
    torch.manual_seed(1)
    model = NET_Model(11)
    ref = copy.deepcopy(model).cuda().train()
    X, Y = _data(640, seed=3)
    runs = []
    for _ in range(2):
        tr = _trainer(copy.deepcopy(model), nn.SmoothL1Loss(), 64)
        f = _feats(tr, X)
        for _ in range(5):
            m = tr.train_epoch(f, Y.cuda(), 640, None)
        runs.append((tr.params.clone(), m))
    assert torch.equal(runs[0][0], runs[1][0])
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    for _ in range(5):
        for b in range(10):
            xb, yb = X[b * 64:(b + 1) * 64].cuda(), Y[b * 64:(b + 1) * 64].cuda()
            opt.zero_grad()
            l = nn.SmoothL1Loss()(ref(xb.to(torch.bfloat16).float()), yb)
            l.backward()
            opt.step()
    assert abs(runs[0][1]["loss"] - l.item()) < 0.25 * max(l.item(), 1e-3) + 0.02, (runs[0][1], l.item())
    emb = dict(ref.named_modules())["embs.4"].weight.detach()
    tr_emb = tr.unflatten(tr.params)[(id(tr.spec.front[7].emb), "weight")]
    assert tr_emb.shape == emb.shape
    assert not torch.equal(tr_emb.cpu(), model.embs[4].weight.detach()), "embedding table never updated"


def test_front_out_of_range_id_raises():
    model = NET_Model(11)
    tr = _trainer(model, nn.SmoothL1Loss(), 64)
    X, Y = _data(64)
    X[5, 5] = 7.0                      # column 5 has 5 rows
    with pytest.raises(IndexError):
        tr.train_epoch(_feats(tr, X), Y.cuda(), 64, None)


def test_estimator_uses_fused_front_engine():
    """TorchEstimator picks the fused engine for NET_Model + SmoothL1 + Accuracy and reports
    the Accuracy metric per epoch, like the torch loop does."""
    import numpy as np
    import pandas as pd

    import raydp_amd
    from raydp_amd import runtime
    from raydp_amd.torch import TorchEstimator
    runtime.shutdown()
    runtime.init(num_cpus=4, num_gpus=1)
    try:
        spark = raydp_amd.init_spark("gpu-front", 1, 2, "500M")
        X, Y = _data(3000, seed=5)
        cols = [f"c{i}" for i in range(11)]
        pdf = pd.DataFrame(X.numpy(), columns=cols)
        pdf["label"] = Y[:, 0].numpy()
        df = spark.createDataFrame(pdf)
        res = {}
        for fused in (True, False):
            torch.manual_seed(0)
            model = NET_Model(11)
            est = TorchEstimator(num_workers=1, model=model, optimizer=torch.optim.Adam(model.parameters(), lr=1e-3),
                                 loss=nn.SmoothL1Loss(), feature_columns=cols, feature_types=[torch.float] * 11,
                                 label_column="label", label_type=torch.float, batch_size=64, num_epochs=3,
                                 metrics_name=["Accuracy"], metrics_config={"Accuracy": {"task": "binary"}},
                                 fused=fused, shuffle=False)
            est.fit_on_spark(df, df)
            hist = est.results.metrics_history
            tr_hist = [h for h in hist if "train_loss" in h]
            res[fused] = tr_hist[-1]
        assert res[True]["engine"] == "fused_mlp_hip"
        assert res[False]["engine"] != "fused_mlp_hip"
        assert "Accuracy" in str(res[True]), res[True]
        assert abs(res[True]["train_loss"] - res[False]["train_loss"]) < 0.1 * res[False]["train_loss"] + 0.01
        assert np.isfinite(res[True]["train_loss"])
    finally:
        raydp_amd.stop_spark()
        runtime.shutdown()
