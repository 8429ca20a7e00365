"""The runtime pickler (raydp_amd/runtime/serialization.py): CPU tensors travel as raw storage
bytes (one copy per storage, however many tensors view it) instead of one ``torch.save`` per
storage, with torch's semantics intact -- values, dtypes, views sharing storage, Parameters,
requires_grad, optimizer state bound to the unpickled parameters."""
import cloudpickle
import torch
import torch.nn as nn

from raydp_amd.runtime import serialization as S


def _roundtrip(obj):
    return cloudpickle.loads(S.dumps(obj, transfer=False))


def test_model_and_optimizer_roundtrip():
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(6, 8), nn.BatchNorm1d(8), nn.ReLU(), nn.Linear(8, 2))
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    m(torch.randn(16, 6)).sum().backward()
    opt.step()
    m2, opt2 = _roundtrip((m, opt))
    for (k, a), (k2, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k == k2 and a.dtype == b.dtype and torch.equal(a, b), k
    assert all(isinstance(p, nn.Parameter) and p.requires_grad for p in m2.parameters())
    assert opt2.param_groups[0]["params"][0] is next(m2.parameters())
    s0, s1 = opt.state_dict()["state"], opt2.state_dict()["state"]
    for k in s0:
        for kk in s0[k]:
            assert torch.equal(torch.as_tensor(s0[k][kk]), torch.as_tensor(s1[k][kk]))


def test_views_keep_sharing_and_dtypes_survive():
    base = torch.arange(12.0).view(3, 4)
    col = base[:, 1]                       # strided view into the same storage
    bf = torch.randn(5).to(torch.bfloat16)
    empty = torch.empty(0, 3)
    tied = nn.Parameter(torch.ones(4))
    out = _roundtrip({"base": base, "col": col, "bf": bf, "empty": empty, "a": tied, "b": tied})
    assert torch.equal(out["base"], base) and torch.equal(out["col"], col)
    out["col"][0] = -1.0
    assert out["base"][0, 1] == -1.0, "a view must keep sharing its storage"
    assert out["bf"].dtype == torch.bfloat16 and torch.equal(out["bf"], bf)
    assert out["empty"].shape == (0, 3)
    assert out["a"] is out["b"], "tied parameters stay one object"


def test_tensor_payload_is_no_larger_than_torch_default():
    m = nn.Sequential(*[nn.Linear(32, 32) for _ in range(12)])
    a = S.dumps(m, transfer=False)
    b = cloudpickle.dumps(m)
    assert len(a) <= len(b)
    m2 = cloudpickle.loads(a)
    for x, y in zip(m.parameters(), m2.parameters()):
        assert torch.equal(x, y)
