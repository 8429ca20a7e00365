"""HIP-graph replay of TorchLoopEngine steps must train exactly like the eager loop."""
import os

import pytest
import torch
import torch.nn as nn

from raydp_amd.torch import graphs
from raydp_amd.torch.engine import TorchLoopEngine
from raydp_amd.torch.metrics import TorchMetric
from raydp_amd.train import session


from raydp_amd.torch.engine import _ShardTensors


class _Shard(_ShardTensors):
    def __init__(self, feats, labels, multi):
        self.feats, self.labels, self.n, self.multi = feats, labels, labels.shape[0], multi


class _Net(nn.Module):
    """Stroke-tutorial shaped: an embedding per categorical + BN'd MLP."""

    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(5, 3)
        self.fc1, self.bn1 = nn.Linear(7, 32), nn.BatchNorm1d(32)
        self.fc2 = nn.Linear(32, 1)

    def forward(self, cat, num):
        # list indexing as in the reference tutorial (x[:, [1, 7, 8]]): must stay capturable
        x = torch.cat([self.emb(cat.reshape(-1)), num[:, [3, 0, 1, 2]]], dim=1)
        return torch.sigmoid(self.fc2(torch.relu(self.bn1(self.fc1(x))))).reshape(-1)


def _engine(device, opt_name, sched, monkeypatch, graphed):
    monkeypatch.setenv("RAYDP_TORCH_GRAPHS", "1" if graphed else "0")
    torch.manual_seed(0)
    model = _Net()
    # the eager reference uses the same capturable Adam math (device-side bias correction, tensor
    # LR under a scheduler) as the graphed run: otherwise fp32-vs-fp64 rounding of the step size
    # is amplified by Adam on parameters whose true gradient is ~0 (the bias feeding BatchNorm).
    cap = device.type == "cuda"
    lr = torch.tensor(1e-2, device=device) if (sched and cap) else 1e-2
    opt = (torch.optim.Adam(model.parameters(), lr=lr, capturable=cap) if opt_name == "adam"
           else torch.optim.SGD(model.parameters(), lr=5e-2, momentum=0.9))
    sch = torch.optim.lr_scheduler.StepLR(opt, step_size=3, gamma=0.5) if sched else None
    cfg = {"batch_size": 32, "shuffle": True, "drop_last": False}
    e = TorchLoopEngine(model, opt, nn.MSELoss(), TorchMetric(["MeanAbsoluteError", "Accuracy"]), device, cfg, sch)
    g = torch.Generator().manual_seed(1)
    n = 32 * 21 + 9   # 21 full batches + a partial one
    cat = torch.randint(0, 5, (n, 1), generator=g).to(device)
    num = torch.randn(n, 4, generator=g).to(device)
    lab = (torch.rand(n, generator=g) > 0.5).float().to(device)
    e.train = _Shard([cat, num], lab, True)
    e.eval = _Shard([cat, num], lab, True)
    return e


def _run(device, opt_name, sched, monkeypatch, graphed, epochs=3):
    session._set_session(session._Session(session.TrainContext(), {}, lambda *a: None, "/tmp"))
    try:
        e = _engine(device, opt_name, sched, monkeypatch, graphed)
        hist = [e.train_epoch() for _ in range(epochs)]
        ev = e.evaluate_epoch()
        return e, hist, ev, {k: v.detach().float().cpu() for k, v in e.state_dict().items()}
    finally:
        session._set_session(None)


def test_graphs_not_used_on_cpu(monkeypatch):
    e, hist, _, _ = _run(torch.device("cpu"), "adam", False, monkeypatch, True, epochs=1)
    assert e.graphed is None and e.graph_status == "not on a GPU"
    assert set(hist[0][0]) == {"MeanAbsoluteError", "Accuracy"}


def test_metric_zero_in_place():
    m = TorchMetric(["MeanSquaredError"])
    m.update(torch.ones(4), torch.zeros(4))
    st = m._metrics["MeanSquaredError"].total
    m.zero_()
    assert m._metrics["MeanSquaredError"].total is st and float(st) == 0.0
    assert m.graph_safe()


def test_capture_safe_list_indexing():
    cache = {}
    x = torch.randn(5, 10, requires_grad=True)
    with graphs._CaptureSafeIndexing(cache):
        y = x[:, [1, 7, 8]]
        z = x[[0, 2]]
        w = x[:, 3]
        m = x[[True, False, True, False, True]]   # bool lists keep their mask meaning
    assert torch.equal(y, x.detach()[:, [1, 7, 8]]) and z.shape == (2, 10) and w.shape == (5,)
    assert m.shape == (3, 10)
    assert set(k[0] for k in cache) == {(1, 7, 8), (0, 2)}
    y.sum().backward()
    assert float(x.grad.sum()) == 15.0


@pytest.mark.gpu
@pytest.mark.parametrize("opt_name,sched", [("adam", False), ("sgd", False), ("adam", True)])
def test_graphed_matches_eager(monkeypatch, opt_name, sched):
    dev = torch.device("cuda:0")
    eg, hg, evg, sg = _run(dev, opt_name, sched, monkeypatch, True)
    ee, he, eve, se = _run(dev, opt_name, sched, monkeypatch, False)
    assert eg.graphed is not None and eg.graphed.failed is None, eg.graph_status
    assert ee.graphed is None
    assert eg.graphed.graphs, "no graph was captured"
    ee2, he2, _, se2 = _run(dev, opt_name, sched, monkeypatch, False)
    diffs = {k: (float((sg[k] - se[k]).abs().max()), float((se2[k] - se[k]).abs().max())) for k in se}
    assert all(d[1] == 0.0 for d in diffs.values()), f"eager loop is not deterministic: {diffs}"
    for k in se:
        torch.testing.assert_close(sg[k], se[k], rtol=2e-4, atol=2e-5, msg=f"{k}: {diffs}")
    for (rg, lg), (re_, le) in zip(hg, he):
        assert abs(lg - le) < 1e-4 * max(1.0, abs(le))
        for k in re_:
            assert abs(rg[k] - re_[k]) < 1e-4 * max(1.0, abs(re_[k])), (k, rg[k], re_[k])
    assert abs(evg[1] - eve[1]) < 1e-4
    _ = os
