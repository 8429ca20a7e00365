"""Horovod-compatible API (raydp_amd.hvd / horovod.torch facade) on gloo, world size 2."""
import copy

import torch
import torch.nn as nn

import raydp  # noqa: F401


def _data(n=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 6, generator=g)
    y = x @ torch.arange(1.0, 7.0).unsqueeze(1) + 0.1 * torch.randn(n, 1, generator=g)
    return x, y


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(6, 16), nn.ReLU(), nn.Linear(16, 1))


def _worker(config):
    import horovod.torch as hvd
    from raydp_amd.train import session
    hvd.init()
    r, w = hvd.rank(), hvd.size()
    assert w == 2
    model = _model()
    if r == 1:   # different init on rank 1: broadcast_parameters must fix it
        with torch.no_grad():
            for p in model.parameters():
                p.add_(1.0)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    hvd.broadcast_optimizer_state(opt, root_rank=0)
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(), op=hvd.Average)
    x, y = _data()
    xs, ys = x[r * 32:(r + 1) * 32], y[r * 32:(r + 1) * 32]
    for _ in range(5):
        opt.zero_grad()
        loss = nn.functional.mse_loss(model(xs), ys)
        loss.backward()
        opt.step()
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    gathered = hvd.allgather(flat.unsqueeze(0))
    s = hvd.allreduce(torch.tensor([float(r + 1)]), op=hvd.Sum)
    obj = hvd.broadcast_object({"from": r}, root_rank=1)
    a2a = hvd.alltoall(torch.arange(4.0) + 10 * r)
    session.report({"flat": flat.tolist(), "same": bool(torch.allclose(gathered[0], gathered[1])),
                    "sum": float(s), "obj": obj["from"], "a2a": a2a.tolist()})


def test_hvd_distributed_optimizer_matches_full_batch(runtime_local):
    from ray.train.horovod import HorovodTrainer
    from raydp_amd.train import ScalingConfig
    res = HorovodTrainer(_worker, scaling_config=ScalingConfig(num_workers=2, use_gpu=False)).fit()
    m = res.metrics
    assert m["same"] and m["sum"] == 3.0 and m["obj"] == 1
    assert m["a2a"] == [0.0, 1.0, 10.0, 11.0]
    # reference: one process, full batch (mean loss) == average of the two half-batch gradients
    model = _model()
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    x, y = _data()
    for _ in range(5):
        opt.zero_grad()
        nn.functional.mse_loss(model(x), y).backward()
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    assert torch.allclose(torch.tensor(m["flat"]), ref, atol=1e-5)


_ = copy
