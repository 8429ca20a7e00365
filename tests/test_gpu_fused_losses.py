"""Classification losses in the fused MLP epilogue (csrc/hip/mlp_core.h): BCE-with-logits and
class-weighted cross entropy (+ argmax accuracy), against PyTorch references of the same ops
on the kernel's bf16 GEMM-operand numerics (BfLin emulation, tight) and plain fp32 (loose)."""
import copy

import pytest
import torch
import torch.nn as nn

from test_gpu_kernels import _relerr, emulate

pytestmark = pytest.mark.gpu


def _mlp(out_f):
    return nn.Sequential(nn.Linear(12, 64), nn.ReLU(), nn.BatchNorm1d(64), nn.Linear(64, 32), nn.ReLU(),
                         nn.Linear(32, out_f))


def _trainer(model, loss, batch):
    from raydp_amd.models.mlp_spec import extract_mlp_spec
    from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    return FusedMLPTrainer(extract_mlp_spec(model), optimizer_config(opt), loss_code(loss), batch,
                           torch.device("cuda"))


@pytest.mark.parametrize("nvalid", [64, 41])
@pytest.mark.parametrize("kind", ["bce", "ce", "ce_weighted", "ce_ignore"])
def test_fused_classification_loss_one_step(kind, nvalid):
    from raydp_amd.ops.fused_mlp import fused_labels
    torch.manual_seed(0)
    classes = 1 if kind == "bce" else 3
    model = _mlp(classes)
    if kind == "bce":
        loss = nn.BCEWithLogitsLoss()
    elif kind == "ce":
        loss = nn.CrossEntropyLoss()
    elif kind == "ce_weighted":
        loss = nn.CrossEntropyLoss(weight=torch.tensor([0.35, 0.65, 1.5]))
    else:
        loss = nn.CrossEntropyLoss(weight=torch.tensor([1.0, 2.0, 0.5]))
    dev = torch.device("cuda")
    ref = copy.deepcopy(model).to(dev).train()
    emu = copy.deepcopy(model).to(dev).train()
    tr = _trainer(model, loss, 64)
    g = torch.Generator().manual_seed(1)
    X = torch.randn(nvalid, 12, generator=g) * 2.0
    if kind == "bce":
        Y = torch.randint(0, 2, (nvalid, 1), generator=g).float()
    else:
        Y = torch.randint(0, classes, (nvalid, 1), generator=g).float()
        if kind == "ce_ignore":
            Y[::7] = -100.0                      # torch's default ignore_index
    feats = torch.zeros(nvalid, tr.feat_k, dtype=torch.bfloat16)
    feats[:, :12] = X.to(torch.bfloat16)
    labels = fused_labels(loss, Y.to(dev), tr.desc.out_dim)
    grads = tr.forward_backward(feats.to(dev), labels, nvalid).clone()
    m = tr._read_metrics()
    xin = X.to(torch.bfloat16).float().to(dev)
    lref = loss.to(dev)
    tgt = Y.to(dev) if kind == "bce" else Y.view(-1).long().to(dev)
    out_ref = ref(xin)
    l32 = lref(out_ref, tgt)
    l32.backward()
    out_emu = emulate(emu, xin)
    le = lref(out_emu, tgt)
    le.backward()
    assert abs(m["loss"] - le.item()) <= 2e-3 * max(1.0, abs(le.item())), (m["loss"], le.item())
    assert abs(m["loss"] - l32.item()) <= 5e-2 * max(1.0, abs(l32.item())), (m["loss"], l32.item())
    if kind != "bce":
        # argmax accuracy over the rows (ignored rows never match), counted by the kernel
        want = (out_emu.argmax(1) == tgt).float().sum().item() / nvalid
        assert abs(m["acc"] - want) <= 1.0 / nvalid + 1e-6, (m["acc"], want)
        assert m["count"] == nvalid
    gmap = tr.unflatten(grads)
    emods, rmods = dict(emu.named_modules()), dict(ref.named_modules())
    for name, mod in model.named_modules():
        for attr in ("weight", "bias"):
            key = (id(mod), attr)
            if key in gmap:
                e = _relerr(gmap[key], getattr(emods[name], attr).grad)
                assert e < 2e-2, (kind, name, attr, e)


def test_fused_engine_takes_weighted_cross_entropy(runtime_local, tmp_path):
    """TorchEstimator with CrossEntropyLoss(weight=...) + Accuracy (the Ray Train stroke
    tutorial's loss, cells 30-40) runs on the fused HIP engine and learns a separable rule."""
    import numpy as np
    import pandas as pd
    from raydp_amd.data import from_pandas
    from raydp_amd.torch import TorchEstimator
    rng = np.random.default_rng(0)
    x = rng.normal(size=(64 * 20, 12)).astype(np.float32)
    y = (x[:, 0] + 0.5 * x[:, 1] > 0).astype(np.int64)
    df = pd.DataFrame({f"f{i}": x[:, i] for i in range(12)})
    df["y"] = y
    torch.manual_seed(0)
    model = _mlp(2)
    est = TorchEstimator(num_workers=1, model=model, optimizer=torch.optim.Adam(model.parameters(), lr=3e-3),
                         loss=nn.CrossEntropyLoss(weight=torch.tensor([0.35, 0.65])),
                         feature_columns=[f"f{i}" for i in range(12)], label_column="y", label_type=torch.long,
                         batch_size=64, num_epochs=8, metrics_name=["Accuracy"], storage_path=str(tmp_path),
                         fused="on")
    res = est.fit(from_pandas(df))
    hist = [h for h in res.metrics_history if "train_loss" in h]
    assert hist[0]["engine"] == "fused_mlp_hip"
    assert hist[-1]["train_loss"] < 0.5 * hist[0]["train_loss"]
    assert hist[-1]["train_res"]["Accuracy"] > 0.9
