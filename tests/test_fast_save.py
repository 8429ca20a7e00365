"""Cached-pickle checkpoint writer (raydp_amd/train/fast_save.py): files equal torch.save's."""
import math
import os
from collections import OrderedDict

import torch

from raydp_amd.train import fast_save as F


def _flat_state(seed=0, width=32):
    """A state dict shaped like the fused engine's export: parameters as views of one flat
    buffer, running stats as views of another, int64 counters."""
    torch.manual_seed(seed)
    m = torch.nn.Sequential(torch.nn.Linear(5, width), torch.nn.BatchNorm1d(width), torch.nn.Linear(width, 1))
    sd = m.state_dict()
    p = torch.randn(sum(v.numel() for k, v in sd.items() if "running" not in k and v.is_floating_point()))
    rs = torch.rand(2 * width)
    out, off, ro = OrderedDict(), 0, 0
    for k, v in sd.items():
        if "running" in k:
            out[k] = rs[ro:ro + v.numel()]
            ro += v.numel()
        elif v.is_floating_point():
            out[k] = p[off:off + v.numel()].view_as(v)
            off += v.numel()
        else:
            out[k] = v + 7
    out._metadata = sd._metadata
    return m, out


def _load(path):
    return torch.load(path, map_location="cpu", weights_only=True)


def _equal(a, b):
    assert list(a) == list(b)
    for k in a:
        assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, k
        assert torch.equal(F._bytes(a[k]), F._bytes(b[k])), k


def test_fast_path_matches_torch_save(tmp_path):
    m, sd = _flat_state()
    F.save_state_dict(sd, str(tmp_path / "first.pt"))
    assert F.save_state_dict(sd, str(tmp_path / "fst.pt"))      # same layout: cached pickle
    torch.save(sd, str(tmp_path / "ref.pt"))
    a, b = _load(str(tmp_path / "fst.pt")), _load(str(tmp_path / "ref.pt"))
    _equal(a, b)
    m.load_state_dict(a)
    assert os.path.getsize(tmp_path / "fst.pt") == os.path.getsize(tmp_path / "ref.pt")


def test_new_values_same_layout_are_written(tmp_path):
    _, sd = _flat_state(0)
    F.save_state_dict(sd, str(tmp_path / "a.pt"))
    for k, v in sd.items():       # same storages, new contents (the next epoch's weights)
        if v.is_floating_point():
            v.mul_(-3.0).add_(1.0)
    sd["0.weight"][0, 0] = math.nan
    assert F.save_state_dict(sd, str(tmp_path / "b.pt"))
    _equal(_load(str(tmp_path / "b.pt")), sd)


def test_layout_change_and_unsupported_fall_back(tmp_path):
    _, a = _flat_state(width=16)
    _, b = _flat_state(width=24)
    F.save_state_dict(a, str(tmp_path / "a.pt"))
    F.save_state_dict(b, str(tmp_path / "b.pt"))
    _equal(_load(str(tmp_path / "a.pt")), a)
    _equal(_load(str(tmp_path / "b.pt")), b)
    nested = {"model": {"w": torch.ones(2)}, "epoch": 3}
    assert not F.save_state_dict(nested, str(tmp_path / "n.pt"))
    got = _load(str(tmp_path / "n.pt"))
    assert got["epoch"] == 3 and torch.equal(got["model"]["w"], torch.ones(2))
