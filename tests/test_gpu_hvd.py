"""Horovod API on the GPU (BASELINE config 4: Horovod-on-Ray NYCTaxi; reference
``examples/horovod_nyctaxi.py:119-162``): ``hvd.DistributedOptimizer(op=Average)`` over the
NYC_Model on cuda, at world 1 and as a 2-rank rehearsal on the one GPU, where the fused
gradient bucket rides the one-shot xGMI kernel with the 1/size average folded into its sum.
Both must match one process training on the full batch."""
import os
import sys

import pytest
import torch
import torch.nn as nn

import raydp  # noqa: F401 - installs the ray / horovod facades

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _data(n=128, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 20, generator=g)
    y = x[:, :5].sum(1, keepdim=True) + 0.1 * torch.randn(n, 1, generator=g)
    return x, y


def _model():
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    from nyc_model import NYC_Model
    torch.manual_seed(0)
    return NYC_Model(20)


def _worker(config):
    import horovod.torch as hvd
    from raydp_amd.train import session
    hvd.init()
    r, w = hvd.rank(), hvd.size()
    dev = session.get_device()
    model = _model().to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    hvd.broadcast_optimizer_state(opt, root_rank=0)
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(), op=hvd.Average)
    kind = None
    if opt._fusion is not None:
        kind = "xgmi" if opt._fusion._sum is not None and opt._fusion._sum.xg is not None else "process_group"
    x, y = _data()
    per = x.shape[0] // w
    xs, ys = x[r * per:(r + 1) * per].to(dev), y[r * per:(r + 1) * per].to(dev)
    model.eval()      # BN in eval: the per-rank half batches then average to the full-batch gradient
    for _ in range(6):
        opt.zero_grad()
        loss = nn.functional.smooth_l1_loss(model(xs), ys)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
    session.report({"flat": flat.tolist(), "kind": kind, "device": str(dev)})


def _reference():
    model = _model().cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    x, y = _data()
    x, y = x.cuda(), y.cuda()
    model.eval()
    for _ in range(6):
        opt.zero_grad()
        nn.functional.smooth_l1_loss(model(x), y).backward()
        opt.step()
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()


@pytest.mark.parametrize("world", [1, 2])
def test_hvd_nyc_on_gpu_matches_full_batch(runtime_local, monkeypatch, world):
    from ray.train.horovod import HorovodTrainer
    from raydp_amd.train import ScalingConfig
    if world > 1:
        monkeypatch.setenv("RAYDP_TRAIN_BACKEND", "gloo")    # two ranks share the one card
    sc = ScalingConfig(num_workers=world, use_gpu=True, resources_per_worker={"CPU": 1, "GPU": 1.0 / world})
    res = HorovodTrainer(_worker, scaling_config=sc).fit()
    m = res.metrics
    assert m["device"].startswith("cuda"), m["device"]
    if world > 1:
        assert m["kind"] == "xgmi", m["kind"]
    ref = _reference()
    got = torch.tensor(m["flat"])
    # smooth-L1 of the mean over 128 rows == mean of the two 64-row means: fp32 order only
    assert torch.allclose(got, ref, atol=2e-5, rtol=1e-4), float((got - ref).abs().max())
