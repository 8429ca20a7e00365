"""Worker backend policies (raydp_amd/train/gpu_policy.py) and the to_torch device default, on
the CPU: the BatchNorm patch is scoped (restored on exit, CPU inputs untouched) and leaves the
numerics of a CPU BatchNorm exactly as they were."""
import torch
import torch.nn as nn

from raydp_amd.train.gpu_policy import native_batchnorm, worker_policies


def test_native_batchnorm_is_scoped_and_restores_forward():
    from torch.nn.modules.batchnorm import _BatchNorm
    orig = _BatchNorm.forward
    bn = nn.BatchNorm1d(8)
    x = torch.randn(16, 8)
    want = bn(x)
    with native_batchnorm(True):
        assert _BatchNorm.forward is not orig
        assert torch.backends.cudnn.enabled        # untouched outside a BatchNorm call
        got = bn(x)
    assert _BatchNorm.forward is orig
    assert torch.equal(got, want)
    with native_batchnorm(False):
        assert _BatchNorm.forward is orig


def test_worker_policies_off_on_cpu_workers():
    from torch.nn.modules.batchnorm import _BatchNorm
    orig = _BatchNorm.forward
    with worker_policies(False):
        assert _BatchNorm.forward is orig


def test_to_torch_default_device_outside_a_worker_is_cpu():
    import pyarrow as pa
    from raydp_amd.data.dataset import Dataset
    t = pa.table({"a": [1.0, 2.0, 3.0, 4.0], "y": [0.0, 1.0, 0.0, 1.0]})
    ds = Dataset([t], t.schema)
    feats, label = next(iter(ds.to_torch(feature_columns=["a"], label_column="y", batch_size=2)))
    assert feats.device.type == "cpu" and label.device.type == "cpu"


def test_hvd_optimizer_on_cpu_keeps_torch_step():
    """CPU parameters: the fused step declines once and torch's step runs (same result)."""
    import copy
    import raydp_amd.hvd as hvd
    torch.manual_seed(0)
    net = nn.Linear(4, 2)
    ref = copy.deepcopy(net)
    hvd.init()
    try:
        opt = hvd.DistributedOptimizer(torch.optim.Adam(net.parameters(), lr=0.1))
        ropt = torch.optim.Adam(ref.parameters(), lr=0.1)
        x = torch.randn(8, 4)
        for m, o in ((net, opt), (ref, ropt)):
            for _ in range(3):
                o.zero_grad()
                m(x).square().mean().backward()
                o.step()
    finally:
        hvd.shutdown()
    for a, b in zip(net.parameters(), ref.parameters()):
        assert torch.equal(a, b)
